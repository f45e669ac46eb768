// Latency of one exact_walk chain (s3r_common.h) in a single wave: 64 lanes walking row-like
// sequences (different starts, same step), timed in-kernel with s_memtime (core clock).
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -I../../include walk_latency.hip
#include <cstdio>
#include "../../swift3drenderer_amd/csrc/s3r_common.h"

__global__ void k_walk(float s0, float d, uint32_t n, float spread, float *out, unsigned long long *cyc,
                       uint32_t *iters) {
    const uint32_t lane = threadIdx.x;
    float s = s0 + spread * (float)lane;
    uint32_t it = 0;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    const float v = s3r::exact_walk(s, d, n, &it);
    out[lane] = v;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    cyc[lane] = t1 - t0;
    iters[lane] = it;
}

__global__ void k_seq(float s0, float d, uint32_t n, float spread, float *out, unsigned long long *cyc) {
    const uint32_t lane = threadIdx.x;
    float s = s0 + spread * (float)lane;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (uint32_t i = 0; i < n; i++) s = s + d;
    out[lane] = s;
    __builtin_amdgcn_s_waitcnt(0);
    cyc[lane] = __builtin_amdgcn_s_memtime() - t0;
}

int main() {
    float *out;
    unsigned long long *cyc;
    uint32_t *it;
    (void)hipMalloc(&out, 256);
    (void)hipMalloc(&cyc, 512);
    (void)hipMalloc(&it, 256);
    struct Case { float s0, d; uint32_t n; float spread; const char *name; };
    const Case cases[] = {
        {0.9f, -1.0f / 3840.0f, 3840, 1e-4f, "row crossing zero (x walk, 3840 px)"},
        {0.9f, -1.0f / 2160.0f, 2160, 1e-4f, "column crossing zero (y walk, 2160 rows)"},
        {0.1f, 1.0f / 3840.0f, 3840, 1e-4f, "row away from zero"},
        {-0.5f, 1.0f / 3840.0f, 384, 1e-4f, "384 px, no crossing"},
        {0.9f, -1.0f / 3840.0f, 0, 0.0f, "n = 0 (overhead)"},
    };
    for (const Case &c : cases) {
        for (int rep = 0; rep < 2; rep++) {
            hipLaunchKernelGGL(k_walk, dim3(1), dim3(64), 0, 0, c.s0, c.d, c.n, c.spread, out, cyc, it);
            (void)hipDeviceSynchronize();
        }
        unsigned long long h[64];
        uint32_t hi[64];
        (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        (void)hipMemcpy(hi, it, sizeof hi, hipMemcpyDeviceToHost);
        uint32_t imax = 0;
        for (int i = 0; i < 64; i++) imax = hi[i] > imax ? hi[i] : imax;
        printf("%-44s exact_walk: %6llu clk (s_memtime)  max iters/lane %3u\n", c.name, h[0], imax);
        hipLaunchKernelGGL(k_seq, dim3(1), dim3(64), 0, 0, c.s0, c.d, c.n, c.spread, out, cyc);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
        printf("%-44s sequential: %6llu clk\n", "", h[0]);
    }
    return 0;
}
