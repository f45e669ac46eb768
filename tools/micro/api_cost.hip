// Host-side cost of the HIP calls a frame makes (launch, event record, stream wait, graph launch),
// and the device-side period of back-to-back tiny launches.  Build: hipcc --offload-arch=gfx950 -O2.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_tiny(unsigned *out, unsigned v) {
    if (threadIdx.x == 0 && v == 0xDEADBEEFu) out[blockIdx.x] = v;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    unsigned *out;
    hipMalloc(&out, 1 << 20);
    hipStream_t s1, s2;
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
    hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    const int N = 2000;
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, out, 1u);
    hipDeviceSynchronize();

    double t0 = now_us();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, out, (unsigned)i);
    double t1 = now_us();
    hipStreamSynchronize(s1);
    double t2 = now_us();
    printf("launch (1 WG):        host %6.2f us/call, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);

    t0 = now_us();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_tiny, dim3(5400), dim3(256), 0, s1, out, (unsigned)i);
    t1 = now_us();
    hipStreamSynchronize(s1);
    t2 = now_us();
    printf("launch (5400 WG):     host %6.2f us/call, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);

    t0 = now_us();
    for (int i = 0; i < N; i++) hipEventRecord(ev, s1);
    t1 = now_us();
    printf("eventRecord:          host %6.2f us/call\n", (t1 - t0) / N);

    t0 = now_us();
    for (int i = 0; i < N; i++) hipStreamWaitEvent(s2, ev, 0);
    t1 = now_us();
    printf("streamWaitEvent:      host %6.2f us/call\n", (t1 - t0) / N);
    hipDeviceSynchronize();

    // ping-pong two streams like the frame pipeline: launch s2, record, wait on s1, launch s1, record
    hipEvent_t e2;
    hipEventCreateWithFlags(&e2, hipEventDisableTiming);
    t0 = now_us();
    for (int i = 0; i < N; i++) {
        hipStreamWaitEvent(s2, ev, 0);
        for (int k = 0; k < 4; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s2, out, (unsigned)i);
        hipEventRecord(e2, s2);
        hipStreamWaitEvent(s1, e2, 0);
        hipLaunchKernelGGL(k_tiny, dim3(5400), dim3(256), 0, s1, out, (unsigned)i);
        hipEventRecord(ev, s1);
    }
    t1 = now_us();
    hipDeviceSynchronize();
    t2 = now_us();
    printf("frame-like 2-stream:  host %6.2f us/frame, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);

    t0 = now_us();
    for (int i = 0; i < N; i++) {
        for (int k = 0; k < 4; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, out, (unsigned)i);
        hipLaunchKernelGGL(k_tiny, dim3(5400), dim3(256), 0, s1, out, (unsigned)i);
    }
    t1 = now_us();
    hipDeviceSynchronize();
    t2 = now_us();
    printf("frame-like 1-stream:  host %6.2f us/frame, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);

    // graph of the 1-stream frame
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s1, hipStreamCaptureModeThreadLocal);
    for (int k = 0; k < 4; k++) hipLaunchKernelGGL(k_tiny, dim3(1), dim3(64), 0, s1, out, 1u);
    hipLaunchKernelGGL(k_tiny, dim3(5400), dim3(256), 0, s1, out, 1u);
    hipStreamEndCapture(s1, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s1);
    hipDeviceSynchronize();
    t0 = now_us();
    for (int i = 0; i < N; i++) hipGraphLaunch(ge, s1);
    t1 = now_us();
    hipDeviceSynchronize();
    t2 = now_us();
    printf("graph (5 kernels):    host %6.2f us/launch, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);

    hipMemcpyAsync(out, out + 1024, 48, hipMemcpyDeviceToDevice, s1);
    unsigned *hpin;
    hipHostMalloc(&hpin, 4096);
    t0 = now_us();
    for (int i = 0; i < N; i++) hipMemcpyAsync(out, hpin, 48, hipMemcpyHostToDevice, s1);
    t1 = now_us();
    hipDeviceSynchronize();
    t2 = now_us();
    printf("memcpyAsync H2D 48B:  host %6.2f us/call, device period %6.2f us\n", (t1 - t0) / N, (t2 - t0) / N);
    return 0;
}
