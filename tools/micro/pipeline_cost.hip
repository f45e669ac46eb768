// Frame-pipeline shapes with realistic kernel durations (busy-wait kernels on the device's
// 100 MHz wall clock): what per-frame period does each launch/sync pattern achieve?
//   geo  = 1 WG busy for G us   (the latency-bound geometry stage)
//   frag = F WGs busy for R us  (the fragment stage)
#include <hip/hip_runtime.h>
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
    hipStream_t s1, s2, s3;
    (void)hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&s3, hipStreamNonBlocking);
    hipEvent_t gdone[3], fdone[3];
    for (int i = 0; i < 3; i++) {
        (void)hipEventCreateWithFlags(&gdone[i], hipEventDisableTiming);
        (void)hipEventCreateWithFlags(&fdone[i], hipEventDisableTiming);
    }
    const int N = 1000;
    const unsigned frag_wg = 4000;
    for (unsigned G : {10u, 20u}) {
        for (unsigned R : {10u, 70u}) {
            const unsigned gt = G * 100 / 1, rt = R * 100;   // 100 MHz: 100 ticks per us
            // A: same stream, geo then frag
            double t0 = now_us();
            for (int i = 0; i < N; i++) {
                hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s1, out, gt);
                hipLaunchKernelGGL(k_busy, dim3(frag_wg), dim3(256), 0, s1, out, rt);
            }
            double t1 = now_us();
            (void)hipDeviceSynchronize();
            double t2 = now_us();
            printf("G=%2u R=%2u  A same-stream:     host %6.2f  period %6.2f us\n", G, R, (t1 - t0) / N, (t2 - t0) / N);
            // B: geo on s2 (double-buffered), frag on s1, events
            t0 = now_us();
            for (int i = 0; i < N; i++) {
                const int p = i & 1;
                (void)hipStreamWaitEvent(s2, fdone[p], 0);
                hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, s2, out, gt);
                (void)hipEventRecord(gdone[p], s2);
                (void)hipStreamWaitEvent(s1, gdone[p], 0);
                hipLaunchKernelGGL(k_busy, dim3(frag_wg), dim3(256), 0, s1, out, rt);
                (void)hipEventRecord(fdone[p], s1);
            }
            t1 = now_us();
            (void)hipDeviceSynchronize();
            t2 = now_us();
            printf("G=%2u R=%2u  B 2-stream events: host %6.2f  period %6.2f us\n", G, R, (t1 - t0) / N, (t2 - t0) / N);
            // C: geo alternating on s2/s3 (triple-buffered), frag on s1
            t0 = now_us();
            for (int i = 0; i < N; i++) {
                const int p = i % 3;
                hipStream_t gs = (i & 1) ? s3 : s2;
                (void)hipStreamWaitEvent(gs, fdone[p], 0);
                hipLaunchKernelGGL(k_busy, dim3(1), dim3(64), 0, gs, out, gt);
                (void)hipEventRecord(gdone[p], gs);
                (void)hipStreamWaitEvent(s1, gdone[p], 0);
                hipLaunchKernelGGL(k_busy, dim3(frag_wg), dim3(256), 0, s1, out, rt);
                (void)hipEventRecord(fdone[p], s1);
            }
            t1 = now_us();
            (void)hipDeviceSynchronize();
            t2 = now_us();
            printf("G=%2u R=%2u  C 3-stream events: host %6.2f  period %6.2f us\n", G, R, (t1 - t0) / N, (t2 - t0) / N);
        }
    }
    return 0;
}
