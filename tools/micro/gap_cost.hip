// Per-frame boundary cost between consecutive fragment-sized kernels on one stream: how much of the
// ~6 us gap between k_fragment launches (rocprof trace of the bench) comes from the cross-stream
// dependency on the geometry event in front of every launch?
//   V1  frag, frag, ...                                       (same stream, nothing between)
//   V2  wait(old completed event), frag, ...                  (barrier packet, dependency satisfied)
//   V3  geo on s2 (+ stop event), wait(that event) on s1, frag (the library's pattern)
//   V4  as V3, geo on a highest-priority stream
//   V5  geo on s1 itself, then frag (same stream, no event)
// Kernels busy-wait on the 100 MHz wall clock; frag = 1280 WGs x 256 threads (one round, 5 per CU).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <chrono>
#include <cstdio>

__global__ void k_busy(unsigned *out, unsigned ticks) {
    const unsigned long long t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(1);
    if (threadIdx.x == 0 && ticks == 0xFFFFFFFFu) out[blockIdx.x] = 1u;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    unsigned *out;
    (void)hipMalloc(&out, 1 << 20);
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipStream_t s1, s2, s3;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    (void)hipStreamCreateWithPriority(&s3, hipStreamNonBlocking, hi);
    hipEvent_t old, ev[4];
    (void)hipEventCreateWithFlags(&old, hipEventDisableTiming);
    for (auto &e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    (void)hipEventRecord(old, s2);
    (void)hipDeviceSynchronize();
    const int N = 1500;
    const unsigned frag_wg = 1280, geo_wg = 102;
    for (unsigned R : {15u, 60u}) {
        const unsigned rt = R * 100, gt = 15 * 100;
        for (int v = 1; v <= 5; v++) {
            (void)hipDeviceSynchronize();
            const double t0 = now_us();
            for (int i = 0; i < N; i++) {
                hipEvent_t e = ev[i & 3];
                if (v == 2) (void)hipStreamWaitEvent(s1, old, 0);
                if (v == 3 || v == 4) {
                    hipStream_t gs = v == 3 ? s2 : s3;
                    hipExtLaunchKernelGGL(k_busy, dim3(geo_wg), dim3(384), 0, gs, nullptr, e, 0, out, gt);
                    (void)hipStreamWaitEvent(s1, e, 0);
                }
                if (v == 5) hipLaunchKernelGGL(k_busy, dim3(geo_wg), dim3(384), 0, s1, out, gt);
                hipLaunchKernelGGL(k_busy, dim3(frag_wg), dim3(256), 0, s1, out, rt);
            }
            const double t1 = now_us();
            (void)hipDeviceSynchronize();
            const double t2 = now_us();
            printf("R=%2u us  V%d  host %6.2f us/frame  period %7.2f us  (overhead %6.2f)\n", R, v, (t1 - t0) / N,
                   (t2 - t0) / N, (t2 - t0) / N - R);
        }
    }
    return 0;
}
