// host_fill.cpp -- host-side background fill for updateAndRender's sky bins (render_api.cpp).
//
// render.cpp:282 fills the whole frame with RGB(30,30,30) before drawing.  In the host-fill delivery
// the GPU writes only the fragment bins some triangle meets; the bins none meets ("sky") are filled
// here, by the library's fill threads, straight into the caller's buffer while the GPU works.  Plain
// C++ (g++, not the HIP compiler): streaming (non-temporal) AVX2 stores where the CPU has them, so
// the fill does not read the destination lines into the cache first.
#include <immintrin.h>
#include <stddef.h>
#include <stdint.h>

namespace s3r_host {

namespace {

__attribute__((target("avx2"))) void fill_avx2(uint32_t *p, size_t n, uint32_t v) {
    while (n && ((uintptr_t)p & 31u)) { *p++ = v; n--; }
    const __m256i x = _mm256_set1_epi32((int)v);
    for (; n >= 16; n -= 16, p += 16) {
        _mm256_stream_si256(reinterpret_cast<__m256i *>(p), x);
        _mm256_stream_si256(reinterpret_cast<__m256i *>(p + 8), x);
    }
    for (; n >= 8; n -= 8, p += 8) _mm256_stream_si256(reinterpret_cast<__m256i *>(p), x);
    while (n--) *p++ = v;
}

void fill_sse2(uint32_t *p, size_t n, uint32_t v) {
    while (n && ((uintptr_t)p & 15u)) { *p++ = v; n--; }
    const __m128i x = _mm_set1_epi32((int)v);
    for (; n >= 4; n -= 4, p += 4) _mm_stream_si128(reinterpret_cast<__m128i *>(p), x);
    while (n--) *p++ = v;
}

// 3-byte pixels (b, g, r of 0x00RRGGBB, little-endian) -> 4-byte words, 8 pixels per step: two
// 12-byte groups shuffled into place, the top byte 0
// (the 16-byte loads of a step read 4 bytes past the 24 it uses: src must have 4 readable bytes past
// its 3 n; dst 16-B aligned, as pixel rows of a malloc'd frame are, gets two 16-B streaming stores a
// step, any other alignment plain stores)
__attribute__((target("avx2"))) void widen_avx2(const uint8_t *src, uint32_t *dst, size_t n) {
    const __m256i idx = _mm256_setr_epi8(0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1,
                                         0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1);
    size_t i = 0;
    const bool a16 = ((uintptr_t)dst & 15u) == 0;
    for (; i + 8 <= n; i += 8) {
        const __m128i lo = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 3 * i));
        const __m128i hi = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 3 * i + 12));
        const __m256i v = _mm256_shuffle_epi8(_mm256_set_m128i(hi, lo), idx);
        if (a16) {
            _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i), _mm256_castsi256_si128(v));
            _mm_stream_si128(reinterpret_cast<__m128i *>(dst + i + 4), _mm256_extracti128_si256(v, 1));
        } else {
            _mm256_storeu_si256(reinterpret_cast<__m256i *>(dst + i), v);
        }
    }
    for (; i < n; i++) dst[i] = src[3 * i] | src[3 * i + 1] << 8 | src[3 * i + 2] << 16;
}

void widen_scalar(const uint8_t *src, uint32_t *dst, size_t n) {
    for (size_t i = 0; i < n; i++) dst[i] = src[3 * i] | src[3 * i + 1] << 8 | src[3 * i + 2] << 16;
}

const bool kAvx2 = __builtin_cpu_supports("avx2");

}  // namespace

// n pixels packed at 3 bytes each (the fragment kernel's staged chunks, render_api.cpp) widened to
// 0x00RRGGBB words at dst, streaming stores (store_fence() as for fill_words)
void widen_pixels(const uint8_t *src, uint32_t *dst, size_t n) {
    if (kAvx2) widen_avx2(src, dst, n);
    else widen_scalar(src, dst, n);
}

// n words of value v from p (any 4-B alignment), streaming stores; call store_fence() before the
// words must be visible to another thread.
void fill_words(uint32_t *p, size_t n, uint32_t v) {
    if (kAvx2) fill_avx2(p, n, v);
    else fill_sse2(p, n, v);
}

void store_fence() { _mm_sfence(); }

}  // namespace s3r_host
