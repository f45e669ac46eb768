// Host-side feasibility probe for a packed delivery (24-bit pixels over the link, widened to the
// caller's 32-bit pixels by the fill threads): T threads, one per L3 domain (as render_api.cpp
// places the fill threads), per "frame" (a) streaming-store 19.5 MB of background (the 4K frame's
// sky), (b) widen 3.4 M pixels from a 3-byte staging buffer into a 4-byte frame, (c) both.
// Build: g++ -O3 -mavx2 -std=c++17 tools/micro/host_expand.cpp -o tools/micro/host_expand -lpthread
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

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

static void fill(uint32_t *dst, size_t n) {
    const __m256i v = _mm256_set1_epi32(0x1E1E1E);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) _mm256_stream_si256((__m256i *)(dst + i), v);
    for (; i < n; i++) dst[i] = 0x1E1E1E;
}
static void widen(const uint8_t *src, uint32_t *dst, size_t n) {
    const __m256i idx = _mm256_setr_epi8(0,1,2,-1, 3,4,5,-1, 6,7,8,-1, 9,10,11,-1, 0,1,2,-1, 3,4,5,-1, 6,7,8,-1, 9,10,11,-1);
    size_t i = 0;
    for (; i + 8 <= n; i += 8) {
        __m128i lo = _mm_loadu_si128((const __m128i *)(src + 3 * i));
        __m128i hi = _mm_loadu_si128((const __m128i *)(src + 3 * i + 12));
        _mm256_stream_si256((__m256i *)(dst + i), _mm256_shuffle_epi8(_mm256_set_m128i(hi, lo), idx));
    }
    for (; i < n; i++) dst[i] = src[3*i] | (src[3*i+1] << 8) | (src[3*i+2] << 16);
}

int main() {
    auto doms = domains();
    printf("%zu L3 domains\n", doms.size());
    const bool pin = !doms.empty();
    const size_t sky = 19500000 / 4, cov = 3400000;
    auto up64 = [](size_t n) { return (n + 63) / 64 * 64; };
    uint32_t *frame = (uint32_t *)aligned_alloc(64, up64((sky + cov) * 4));
    uint8_t *stage = (uint8_t *)aligned_alloc(64, up64(cov * 3 + 64));
    memset(frame, 0, (sky + cov) * 4); memset(stage, 5, cov * 3);
    for (int T : {4, 6, 8}) {
        for (int mode = 0; mode < 3; mode++) {
            double best = 1e9;
            for (int rep = 0; rep < 30; rep++) {
                auto t0 = std::chrono::steady_clock::now();
                std::vector<std::thread> th;
                for (int t = 0; t < T; t++) th.emplace_back([&, t] {
                    if (pin) {
                        cpu_set_t set; CPU_ZERO(&set);
                        for (int c : doms[(size_t)t % doms.size()]) CPU_SET(c, &set);
                        pthread_setaffinity_np(pthread_self(), sizeof set, &set);
                    }
                    if (mode != 1) { size_t a = sky * t / T / 8 * 8, b = t == T - 1 ? sky : sky * (t + 1) / T / 8 * 8; fill(frame + a, b - a); }
                    if (mode != 0) { size_t a = cov * t / T / 8 * 8, b = t == T - 1 ? cov : cov * (t + 1) / T / 8 * 8;
                                     widen(stage + 3 * a, frame + sky + a, b - a); }
                    _mm_sfence();
                });
                for (auto &x : th) x.join();
                const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                if (us < best) best = us;
            }
            printf("T=%d %-12s %8.1f us (incl. thread start)\n", T, mode == 0 ? "fill" : mode == 1 ? "widen" : "fill+widen", best);
        }
    }
}
