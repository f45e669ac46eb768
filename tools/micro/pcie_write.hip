// GPU -> host delivery rates for the host-fill design (render_api.cpp): the fragment kernel's direct
// stores into the caller's registered host buffer against the DMA engine's copy of the same bytes.
// Variants: store width per lane (4 B / 16 B), plain vs non-temporal stores, contiguous vs the
// frame's bin pattern (384-px x 4-row bins of a 3840-wide frame, 1536-B row segments 15360 B apart),
// 64-B aligned vs the malloc'd +16-B base, registered malloc memory vs hipHostMalloc.
// Build: hipcc --offload-arch=gfx950 -O3 tools/micro/pcie_write.hip -o tools/micro/pcie_write
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); exit(1); } } while (0)

constexpr unsigned W = 3840, H = 2160, BIN_W = 384, BIN_H = 4;
constexpr unsigned SEGS = W / BIN_W, BINS = (H / BIN_H) * SEGS;

// one workgroup (4 waves, one per row) per covered bin: the k_fragment store pattern
template <int VEC, bool NT>
__global__ void __launch_bounds__(256) k_bins(unsigned *frame, const unsigned *list, unsigned v) {
    const unsigned b = list[blockIdx.x];
    const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned y = (b / SEGS) * BIN_H + wave, xs = (b % SEGS) * BIN_W;
    unsigned *row = frame + (size_t)y * W + xs;
    if (VEC == 1) {
        for (unsigned x = lane; x < BIN_W; x += 64) {
            if (NT) __builtin_nontemporal_store(v + x, row + x);
            else row[x] = v + x;
        }
    } else {
        typedef unsigned u4 __attribute__((ext_vector_type(4)));
        u4 *r4 = reinterpret_cast<u4 *>(row);
        for (unsigned x = lane; x < BIN_W / 4; x += 64) {
            const u4 q = {v, v + 1, v + 2, v + 3};
            if (NT) __builtin_nontemporal_store(q, r4 + x);
            else r4[x] = q;
        }
    }
}

// the fragment kernel's store pattern: per covered bin, each wave (row) stores its six 64-px chunks
// one 256-B wave store at a time, ~20 % of the chunks skipped (all background: the host fills them);
// ROT: each store shifted to the 64-B line grid (the wave stores pixels [cx0 - r, cx0 - r + 64), r =
// the chunk start's pixel offset inside its line: the previous chunk's last r pixels carried over in
// lanes < r by a lane rotation), so every store covers whole lines
template <bool ROT>
__global__ void __launch_bounds__(256) k_chunks(unsigned *frame, const unsigned *list, unsigned v) {
    const unsigned b = list[blockIdx.x];
    const unsigned wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const unsigned y = (b / SEGS) * BIN_H + wave, xs = (b % SEGS) * BIN_W;
    unsigned *row = frame + (size_t)y * W;
    const unsigned r = ROT ? (unsigned)(((uintptr_t)(row + xs) >> 2) & 15u) : 0u;
    unsigned carry = 0xFFFFFFFFu;
    for (unsigned q = 0; q < BIN_W / 64; q++) {
        const bool covered = ((b * 7u + q * 13u + wave) * 2654435761u >> 20) % 10u >= 2u;
        const unsigned cx0 = xs + 64u * q;
        const unsigned px = covered ? (v + cx0 + lane) & 0xFFFFFFu : 0xFFFFFFFFu;
        if (!ROT) {
            if (covered) row[cx0 + lane] = px;
            continue;
        }
        const unsigned rot = (unsigned)__shfl((int)px, (int)((lane - r) & 63u));
        const unsigned val = lane >= r ? rot : carry;
        if (val != 0xFFFFFFFFu) row[cx0 - r + lane] = val;
        carry = rot;
    }
    if (ROT && lane < r && carry != 0xFFFFFFFFu) row[xs + BIN_W - r + lane] = carry;
}

// contiguous: one workgroup per 6 KiB (a bin's bytes), 4 B per lane
__global__ void __launch_bounds__(256) k_flat(unsigned *dst, unsigned n, unsigned v) {
    const size_t base = (size_t)blockIdx.x * 1536;
    for (unsigned i = threadIdx.x; i < 1536 && base + i < n; i += 256) dst[base + i] = v + i;
}

static float time_it(hipStream_t s, hipEvent_t a, hipEvent_t b, void (*fn)(hipStream_t, void *), void *ctx, int reps) {
    fn(s, ctx);
    CK(hipStreamSynchronize(s));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < reps; i++) fn(s, ctx);
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms / reps;
}

struct Ctx { unsigned *host_dev, *list, *dev_src, *host; unsigned nbins; size_t bytes; };

int main() {
    // covered bins: every other bin of the top half-ish, 45 % of the frame, like 4K P_over
    unsigned *hlist = (unsigned *)malloc(BINS * 4), nb = 0;
    for (unsigned b = 0; b < BINS; b++)
        if ((b * 2654435761u >> 16) % 100 < 45) hlist[nb++] = b;
    const size_t covered = (size_t)nb * BIN_W * BIN_H * 4;
    printf("bins %u covered %u (%.1f MB)\n", BINS, nb, covered / 1e6);
    Ctx c;
    c.nbins = nb;
    c.bytes = covered;
    CK(hipMalloc(&c.list, BINS * 4));
    CK(hipMemcpy(c.list, hlist, nb * 4, hipMemcpyHostToDevice));
    CK(hipMalloc(&c.dev_src, (size_t)W * H * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const size_t fb = (size_t)W * H * 4;

    for (int mode = 0; mode < 5; mode++) {
        // 0: malloc + register, base +16 B (glibc's large malloc); 1: same, 64-B aligned; 2: hipHostMalloc;
        // 3: as 0, registered uncached (extended fine-grained); 4: as 0, registered coarse-grained
        void *raw = nullptr;
        unsigned *host = nullptr;
        if (mode != 2) {
            raw = malloc(fb + 4096);
            host = (unsigned *)(((uintptr_t)raw + 4095) & ~(uintptr_t)4095) + (mode == 1 ? 0 : 4);
            const unsigned extra = mode == 3 ? hipExtHostRegisterUncached : (mode == 4 ? hipExtHostRegisterCoarseGrained : 0u);
            CK(hipHostRegister(host, fb, hipHostRegisterPortable | hipHostRegisterMapped | extra));
        } else {
            CK(hipHostMalloc((void **)&host, fb, hipHostMallocMapped));
        }
        memset(host, 0, fb);
        c.host = host;
        CK(hipHostGetDevicePointer((void **)&c.host_dev, host, 0));
        const char *name[] = {"malloc+register +16B", "malloc+register aligned", "hipHostMalloc",
                              "malloc+register +16B uncached", "malloc+register +16B coarse-grained"};
        printf("== %s\n", name[mode]);
        auto report = [&](const char *what, float ms, size_t bytes) {
            printf("  %-34s %8.1f us  %6.1f GB/s\n", what, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
        };
        report("DMA D2H contiguous (covered bytes)", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; CK(hipMemcpyAsync(q.host, q.dev_src, q.bytes, hipMemcpyDeviceToHost, st)); }, &c, 20), covered);
        report("DMA D2H whole frame", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; CK(hipMemcpyAsync(q.host, q.dev_src, (size_t)W * H * 4, hipMemcpyDeviceToHost, st)); }, &c, 20), fb);
        report("kernel contiguous 4B/lane", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; hipLaunchKernelGGL(k_flat, dim3((unsigned)(q.bytes / 6144)), dim3(256), 0, st, q.host_dev,
                                                    (unsigned)(q.bytes / 4), 7u); }, &c, 20), covered);
        report("kernel bins 4B/lane", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_bins<1, false>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered);
        report("kernel bins 4B/lane nontemporal", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_bins<1, true>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered);
        report("kernel chunks (fragment pattern)", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_chunks<false>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered * 8 / 10);
        report("kernel chunks line-aligned (rotated)", time_it(s, e0, e1, [](hipStream_t st, void *p) {
            Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_chunks<true>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered * 8 / 10);
        for (int rot = 0; rot < 2; rot++) {      // both chunk kernels write exactly the covered chunks
            memset(host, 0, fb);
            if (rot) hipLaunchKernelGGL((k_chunks<true>), dim3(c.nbins), dim3(256), 0, s, c.host_dev, c.list, 7u);
            else hipLaunchKernelGGL((k_chunks<false>), dim3(c.nbins), dim3(256), 0, s, c.host_dev, c.list, 7u);
            CK(hipStreamSynchronize(s));
            size_t bad = 0;
            for (unsigned i = 0; i < nb; i++) {
                const unsigned b = hlist[i];
                for (unsigned wv = 0; wv < BIN_H; wv++)
                    for (unsigned q = 0; q < BIN_W / 64; q++) {
                        const bool cov = ((b * 7u + q * 13u + wv) * 2654435761u >> 20) % 10u >= 2u;
                        const unsigned y = (b / SEGS) * BIN_H + wv;
                        for (unsigned l = 0; l < 64; l++) {
                            const unsigned x = (b % SEGS) * BIN_W + 64 * q + l;
                            bad += host[(size_t)y * W + x] != (cov ? ((7u + x) & 0xFFFFFFu) : 0u);
                        }
                    }
            }
            printf("  chunks %s: %zu wrong pixels\n", rot ? "rotated" : "plain", bad);
        }
        {   // (row segments are 16-B aligned in every mode)
            report("kernel bins 16B/lane", time_it(s, e0, e1, [](hipStream_t st, void *p) {
                Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_bins<4, false>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered);
            report("kernel bins 16B/lane nontemporal", time_it(s, e0, e1, [](hipStream_t st, void *p) {
                Ctx &q = *(Ctx *)p; hipLaunchKernelGGL((k_bins<4, true>), dim3(q.nbins), dim3(256), 0, st, q.host_dev, q.list, 7u); }, &c, 20), covered);
        }
        if (mode != 2) { CK(hipHostUnregister(host)); free(raw); }
        else CK(hipHostFree(host));
    }
    return 0;
}
