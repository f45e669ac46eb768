// Fixed cost of a grid shaped like k_fragment: empty-ish kernels, timed with hipEvents.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int LDS_BYTES, int ITERS>
__global__ void __launch_bounds__(256, 5) k_empty(unsigned *out, unsigned n) {
    __shared__ unsigned char lds[LDS_BYTES > 0 ? LDS_BYTES : 1];
    unsigned v = blockIdx.x;
    for (int i = 0; i < ITERS; i++) v = v * 1664525u + 1013904223u;
    if (LDS_BYTES > 0) { lds[threadIdx.x] = (unsigned char)v; __syncthreads(); v += lds[(threadIdx.x + 1) & 255]; }
    if (v == 0xDEADBEEFu) out[threadIdx.x] = v;   // never true: keep the work alive
}

// persistent: each block loops over `items` work items
__global__ void __launch_bounds__(256, 5) k_persist(unsigned *out, unsigned items) {
    __shared__ unsigned char lds[26624];
    unsigned v = 0;
    for (unsigned it = blockIdx.x; it < items; it += gridDim.x) {
        v = v * 1664525u + it;
        lds[threadIdx.x] = (unsigned char)v; __syncthreads(); v += lds[(threadIdx.x + 1) & 255]; __syncthreads();
    }
    if (v == 0xDEADBEEFu) out[threadIdx.x] = v;
}

__global__ void __launch_bounds__(256, 5) k_store(unsigned *out, unsigned W, unsigned segs) {
    // k_fragment's store pattern: block = 4 rows x 384 px, each wave 6 x 64 dwords of one row
    const unsigned lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const unsigned blk = blockIdx.x / segs, seg = blockIdx.x % segs;
    unsigned *row = out + (size_t)(blk * 4 + wave) * W;
    for (unsigned q = 0; q < 6; q++) { unsigned x = seg * 384 + q * 64 + lane; if (x < W) row[x] = 0x1E1E1E; }
}

template <class F> float timeit(F f, int reps) {
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    f(); hipDeviceSynchronize();
    hipEventRecord(a); for (int i = 0; i < reps; i++) f(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); return ms * 1000.0f / reps;
}

int main() {
    unsigned *out; hipMalloc(&out, 3840u * 2160u * 4u);
    const unsigned G = 540 * 10;   // 4K: 540 row blocks x 10 segments
    printf("empty, no LDS, 8100 WG x256:      %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k_empty<0, 1>), dim3(8100), dim3(256), 0, 0, out, 0u); }, 200));
    printf("empty, 26 KB LDS, 8100 WG:         %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k_empty<26624, 1>), dim3(8100), dim3(256), 0, 0, out, 0u); }, 200));
    printf("empty, 26 KB LDS, 5400 WG:         %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k_empty<26624, 1>), dim3(G), dim3(256), 0, 0, out, 0u); }, 200));
    printf("empty, no LDS, 1280 WG:            %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k_empty<0, 1>), dim3(1280), dim3(256), 0, 0, out, 0u); }, 200));
    printf("persistent 1280 WG, 8100 items:    %7.2f us\n", timeit([&] { hipLaunchKernelGGL(k_persist, dim3(1280), dim3(256), 0, 0, out, 8100u); }, 200));
    printf("store pattern 4K (33 MB), 5400 WG: %7.2f us\n", timeit([&] { hipLaunchKernelGGL(k_store, dim3(G), dim3(256), 0, 0, out, 3840u, 10u); }, 200));
    printf("hipMemsetD32 4K (33 MB):           %7.2f us\n", timeit([&] { hipMemsetD32((hipDeviceptr_t)out, 0x1E1E1E, 3840u * 2160u); }, 200));
    return 0;
}
