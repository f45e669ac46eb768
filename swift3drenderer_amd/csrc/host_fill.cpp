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

const bool kAvx2 = __builtin_cpu_supports("avx2");

}  // namespace

// n words of value v from p (any 4-B alignment), streaming stores; call store_fence() before the
// words must be visible to another thread.
void fill_words(uint32_t *p, size_t n, uint32_t v) {
    if (kAvx2) fill_avx2(p, n, v);
    else fill_sse2(p, n, v);
}

void store_fence() { _mm_sfence(); }

}  // namespace s3r_host
