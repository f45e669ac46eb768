// Packed-delivery host side in isolation: a kernel writes a 4K frame's worth of staged 3-byte pixels
// (10.3 MB, system-scope stores, as k_fragment) into registered host memory; after it completes, 4
// CCD-placed threads widen them (host_fill.cpp's loop) into a malloc'd frame.  Against the same
// widening of staging data the CPU wrote itself.  Tells whether freshly DMA-written lines are slow
// to read, or the overlap with the device's writes is.
// Build: hipcc --offload-arch=gfx950 -O3 -mavx2 tools/micro/stage_read.hip -o tools/micro/stage_read -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

__global__ void k_stage(unsigned *dst, size_t ndw, unsigned v) {
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < ndw; i += (size_t)gridDim.x * blockDim.x)
        __hip_atomic_store(dst + i, v + (unsigned)i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__attribute__((target("avx2"))) static void widen(const uint8_t *src, uint32_t *dst, size_t n) {
    const __m256i idx = _mm256_setr_epi8(0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1,
                                         0, 1, 2, -1, 3, 4, 5, -1, 6, 7, 8, -1, 9, 10, 11, -1);
    for (size_t i = 0; i + 8 <= n; i += 8) {
        const __m128i lo = _mm_loadu_si128((const __m128i *)(src + 3 * i));
        const __m128i hi = _mm_loadu_si128((const __m128i *)(src + 3 * i + 12));
        const __m256i v = _mm256_shuffle_epi8(_mm256_set_m128i(hi, lo), idx);
        _mm_stream_si128((__m128i *)(dst + i), _mm256_castsi256_si128(v));
        _mm_stream_si128((__m128i *)(dst + i + 4), _mm256_extracti128_si256(v, 1));
    }
}

static std::vector<std::vector<int>> domains() {
    std::vector<std::vector<int>> out;
    std::vector<int> seen(1024, 0);
    for (int c = 0; c < 1024; c++) {
        if (seen[c]) continue;
        FILE *f = fopen(("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list").c_str(), "r");
        if (!f) continue;
        char buf[256] = {0};
        if (!fgets(buf, sizeof buf, f)) { fclose(f); continue; }
        fclose(f);
        std::vector<int> d;
        for (char *p = buf; *p;) {
            char *e; long a = strtol(p, &e, 10); if (e == p) break; long b = a; p = e;
            if (*p == '-') { b = strtol(p + 1, &e, 10); p = e; }
            for (long x = a; x <= b && x < 1024; x++) { d.push_back((int)x); seen[x] = 1; }
            while (*p == ',' || *p == '\n') p++;
        }
        out.push_back(d);
    }
    return out;
}

int main() {
    const size_t npx = 3400000, W = 3840;
    const size_t sbytes = (npx * 3 + 64 + 4095) & ~(size_t)4095;
    uint8_t *stage = (uint8_t *)aligned_alloc(4096, sbytes);
    memset(stage, 0, sbytes);
    CK(hipHostRegister(stage, sbytes, hipHostRegisterPortable | hipHostRegisterMapped));
    unsigned *sdev;
    CK(hipHostGetDevicePointer((void **)&sdev, stage, 0));
    uint32_t *frame = (uint32_t *)aligned_alloc(4096, (npx * 4 + 64 + 4095) & ~(size_t)4095);
    memset(frame, 0, npx * 4);
    auto doms = domains();
    int T = 4;
    size_t piece = 64;
    bool blocks = false;          // false: pieces in a hashed order; true: blocks of 8 consecutive pieces per thread
    auto run_widen = [&](const char *what) {
        auto t0 = std::chrono::steady_clock::now();
        std::vector<std::thread> th;
        for (int t = 0; t < T; t++) th.emplace_back([&, t] {
            if (!doms.empty()) {
                cpu_set_t set; CPU_ZERO(&set);
                for (int c : doms[(size_t)t % doms.size()]) CPU_SET(c, &set);
                pthread_setaffinity_np(pthread_self(), sizeof set, &set);
            }
            // pieces of `piece` pixels (a chunk, a bin's row of 6 chunks, or a whole bin staged
            // contiguously), in an order that jumps between rows like bins do -- or, with `blocks`, the
            // host fill's own order (thread t takes blocks t, t + T, ... of 8 consecutive pieces); the
            // frame 16 B into its first line, as a malloc'd buffer
            const size_t chunks = npx / piece - 1;
            if (blocks) {
                for (size_t b0 = 8 * t; b0 < chunks; b0 += 8 * T)
                    for (size_t c = b0; c < b0 + 8 && c < chunks; c++) widen(stage + 3 * piece * c, frame + 4 + piece * c, piece);
            } else {
                for (size_t k = t; k < chunks; k += T) {
                    const size_t c = (k * 2654435761ull) % chunks;
                    widen(stage + 3 * piece * c, frame + 4 + piece * c, piece);
                }
            }
            _mm_sfence();
        });
        for (auto &x : th) x.join();
        printf("%-48s T=%d %8.1f us\n", what, T, std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    };
    (void)W;
    for (int bl = 0; bl < 2; bl++) {
        blocks = bl == 1;
        for (size_t pc : {64, 384, 1536}) {
            if (blocks && pc != 1536) continue;
            piece = pc;
            for (int tt : {4, 8}) {
                T = tt;
                printf("pieces of %zu px%s\n", pc, blocks ? ", blocks of 8 in thread order" : ", hashed order");
                for (int rep = 0; rep < 2; rep++) {
                    memset(stage, rep, npx * 3);
                    run_widen("widen, staging written by the CPU");
                    hipLaunchKernelGGL(k_stage, dim3(1024), dim3(256), 0, nullptr, sdev, npx * 3 / 4, (unsigned)rep);
                    CK(hipDeviceSynchronize());
                    run_widen("widen, staging written by the GPU");
                }
            }
        }
    }
    return 0;
}
