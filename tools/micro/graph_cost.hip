// Host cost of issuing one frame's kernels: the row path's frame is three
// launches on one stream (k_geometry, k_sky_flags, k_fragment; ~120-200 B of arguments each, the
// camera matrix among them).  Eager launches against a hipGraph of the same three kernel nodes,
// instantiated once and re-launched per frame with the geometry node's arguments updated
// (hipGraphExecKernelNodeSetParams: the camera changes every frame), and without the update.
// Reports host microseconds per frame (issue only, then the device-drained period).
// Build: hipcc --offload-arch=gfx950 -O2 tools/micro/graph_cost.hip -o tools/micro/graph_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

struct Cam { float m[12]; float factor; unsigned w, h, band, nparts, part, rows; };
struct Big { const void *p[12]; unsigned u[16]; };     // ~160 B of pointers and sizes, like k_fragment's

__global__ void k_a(Cam c, Big b, unsigned *out) { if (threadIdx.x == 0 && c.w == 0xDEAD) out[blockIdx.x] = b.u[0]; }
__global__ void k_b(const unsigned *in, unsigned n, unsigned *flags, unsigned tag, unsigned *probe, unsigned g) {
    if (threadIdx.x == 0 && n == 0xDEAD) flags[blockIdx.x] = tag + g + (probe ? 1 : 0) + in[0];
}
__global__ void k_c(Big b, unsigned *out, unsigned tag) { if (threadIdx.x == 0 && tag == 0xDEAD) out[blockIdx.x] = b.u[1]; }

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    unsigned *buf;
    CK(hipMalloc(&buf, 1 << 22));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    Cam cam{};
    Big big{};
    for (int i = 0; i < 12; i++) big.p[i] = buf;
    const int N = 2000;
    // realistic grids: geometry 102 slots x 17 row blocks, flags 22 blocks, fragment 5400 workgroups
    const dim3 ga(102, 17), gb(22), gc(5400);
    auto eager = [&](int k) {
        cam.m[0] = (float)k;
        hipLaunchKernelGGL(k_a, ga, dim3(384), 0, s, cam, big, buf);
        hipLaunchKernelGGL(k_b, gb, dim3(256), 0, s, buf, 5400u, buf, (unsigned)k, buf, 0u);
        hipLaunchKernelGGL(k_c, gc, dim3(256), 0, s, big, buf, (unsigned)k);
    };
    for (int k = 0; k < 200; k++) eager(k);
    CK(hipStreamSynchronize(s));
    double t0 = now_us();
    for (int k = 0; k < N; k++) eager(k);
    double t1 = now_us();
    CK(hipStreamSynchronize(s));
    double t2 = now_us();
    printf("eager 3 launches       issue %6.2f us/frame   drained %6.2f us/frame\n", (t1 - t0) / N, (t2 - t0) / N);

    // the same frame as a graph (stream capture), instantiated once
    hipGraph_t graph;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
    eager(0);
    CK(hipStreamEndCapture(s, &graph));
    hipGraphExec_t exec;
    CK(hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0));
    size_t nn = 0;
    CK(hipGraphGetNodes(graph, nullptr, &nn));
    hipGraphNode_t nodes[8];
    CK(hipGraphGetNodes(graph, nodes, &nn));
    hipKernelNodeParams kp{};
    CK(hipGraphKernelNodeGetParams(nodes[0], &kp));
    for (int k = 0; k < 200; k++) CK(hipGraphLaunch(exec, s));
    CK(hipStreamSynchronize(s));
    t0 = now_us();
    for (int k = 0; k < N; k++) CK(hipGraphLaunch(exec, s));
    t1 = now_us();
    CK(hipStreamSynchronize(s));
    t2 = now_us();
    printf("graph launch           issue %6.2f us/frame   drained %6.2f us/frame\n", (t1 - t0) / N, (t2 - t0) / N);

    void *args[3] = {&cam, &big, &buf};
    kp.kernelParams = args;
    t0 = now_us();
    for (int k = 0; k < N; k++) {
        cam.m[0] = (float)k;
        CK(hipGraphExecKernelNodeSetParams(exec, nodes[0], &kp));
        CK(hipGraphLaunch(exec, s));
    }
    t1 = now_us();
    CK(hipStreamSynchronize(s));
    t2 = now_us();
    printf("graph + 1 node update  issue %6.2f us/frame   drained %6.2f us/frame\n", (t1 - t0) / N, (t2 - t0) / N);

    // synchronous frames (the updateAndRender path): issue + wait per frame
    t0 = now_us();
    for (int k = 0; k < 500; k++) { eager(k); CK(hipStreamSynchronize(s)); }
    t1 = now_us();
    printf("eager + sync per frame          %6.2f us/frame\n", (t1 - t0) / 500);
    t0 = now_us();
    for (int k = 0; k < 500; k++) {
        cam.m[0] = (float)k;
        CK(hipGraphExecKernelNodeSetParams(exec, nodes[0], &kp));
        CK(hipGraphLaunch(exec, s));
        CK(hipStreamSynchronize(s));
    }
    t1 = now_us();
    printf("graph + update + sync per frame %6.2f us/frame\n", (t1 - t0) / 500);
    return 0;
}
