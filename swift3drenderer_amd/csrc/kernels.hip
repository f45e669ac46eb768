// kernels.hip -- the gfx950 HIP kernels of the rasterizer.
//
//   k_geometry  render.cpp:284-359, :374-379  per (slot, row block): vertex + normal transform of the
//                                   slot's corners, reject, near-plane clip (:212-262), cull, raster
//                                   setup (slot t, or slot T+t for a clip split); the fragment
//                                   workgroups' pair records; exact row and segment starts.
//   k_fragment  render.cpp:360-382  one wave per (row, 64*NCH-pixel segment).  Triangles are taken
//                                   in slot order, 64 at a time: lanes first act as TRIANGLES and
//                                   walk each triangle's exact barycentric sequence to this row
//                                   and to each 64-pixel chunk (exact_walk), publishing per-chunk
//                                   (start, step) records in LDS; then lanes act as PIXELS and run
//                                   the edge test and the strict-'>' 1/z depth test in registers
//                                   (the depth buffer never touches HBM).  The final winner is
//                                   shaded once (deferred): half-vector shading, colour or ripmap
//                                   texel, packed 0x00RRGGBB store.
//
// No MFMA: nothing here is a dense contraction.  Compiled with -ffp-contract=off (no FMA), IEEE
// division/sqrt -- results are bit-identical to the CPU restatement of render.cpp.
#include "s3r_common.h"
#include "s3r_kernels.h"

#include <hip/hip_ext.h>

#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <rocprim/device/device_scan.hpp>

namespace s3r {

// ------------------------------------------------------------------ transforms
// simd_mul(simd_float4x3, simd_float4) = ((c0*x + c1*y) + c2*z) + c3*w
__device__ __forceinline__ F3 mat_mul(const Mat34 &m, float4 v) {
    return mk3(((m.m[0][0] * v.x + m.m[0][1] * v.y) + m.m[0][2] * v.z) + m.m[0][3] * v.w,
               ((m.m[1][0] * v.x + m.m[1][1] * v.y) + m.m[1][2] * v.z) + m.m[1][3] * v.w,
               ((m.m[2][0] * v.x + m.m[2][1] * v.y) + m.m[2][2] * v.z) + m.m[2][3] * v.w);
}

// ------------------------------------------------------------------ K2: gather / clip / cull / setup
struct Vert {
    F3 cv, rv, n;
    float4 pay;   // colour rgb | texture (index bits, -, u, v)
};

__device__ __forceinline__ F3 lerp3(F3 a, F3 b, float one_minus_a, float a_) {
    return mk3(a.x * one_minus_a + b.x * a_, a.y * one_minus_a + b.y * a_, a.z * one_minus_a + b.z * a_);
}

// render.cpp:212-262 -- near-plane split.  `d` is edited in place; a second triangle, if any, is
// returned in `app` (what the reference appends to the scene arrays and reaches later, :249-257).
__device__ bool clip_tri(Vert d[3], Vert app[3], uint32_t *app_first, bool textured, float factor, float half_w,
                         float half_h) {
    Vert nw[3];
    uint32_t cur = 0, nxt = 0, pre = 0;
    bool new_triangle = false;
#pragma unroll
    for (uint32_t i = 0; i < 3; i++) {
        const uint32_t in = (i + 1) % 3;
        if ((d[i].rv.z > kNear) == (d[in].rv.z > kNear)) {
            cur = i; nxt = in; pre = (i + 2) % 3;
            new_triangle = d[i].rv.z > kNear;
        } else {
            const float a = (kNear - d[i].rv.z) / (d[in].rv.z - d[i].rv.z);
            const float oma = 1 - a;
            const F3 cv = lerp3(d[i].cv, d[in].cv, oma, a);
            const F3 rv = mk3((cv.x * factor) / kNear + half_w, ((-cv.y) * factor) / kNear + half_h,
                              (0.0f * factor) / kNear + kNear);
            float4 pay;
            if (!textured) {
                pay = make_float4(d[i].pay.x * oma + d[in].pay.x * a, d[i].pay.y * oma + d[in].pay.y * a,
                                  d[i].pay.z * oma + d[in].pay.z * a, 0.0f);
            } else {
                pay = make_float4(d[i].pay.x, 0.0f, d[i].pay.z * oma + d[in].pay.z * a,
                                  d[i].pay.w * oma + d[in].pay.w * a);
            }
            nw[i].cv = cv; nw[i].rv = rv; nw[i].pay = pay;
            nw[i].n = lerp3(d[i].n, d[in].n, oma, a);
        }
    }
    // Runtime-indexed selects (small, unrolled) keep the arrays in registers.
    Vert vcur = d[0], v_nxt = nw[0], v_pre = nw[0];
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
        if (k == cur) vcur = d[k];
        if (k == nxt) v_nxt = nw[k];
        if (k == pre) v_pre = nw[k];
    }
    if (new_triangle) {
#pragma unroll
        for (uint32_t k = 0; k < 3; k++) if (k == pre) d[k] = v_nxt;
        app[0] = vcur; app[1] = v_nxt; app[2] = v_pre;
        *app_first = cur;
        return true;
    }
    Vert v_prec = nw[0];
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) if (k == pre) v_prec = nw[k];
#pragma unroll
    for (uint32_t k = 0; k < 3; k++) {
        if (k == cur) d[k] = v_prec;
        if (k == nxt) d[k] = v_nxt;
    }
    return false;
}

__device__ __forceinline__ float edge_fn(F3 a, F3 b, float cx, float cy) {
    return (cx - a.x) * (a.y - b.y) + (cy - a.y) * (b.x - a.x);     // EDGE_FUNCTION, render.cpp:9
}

// render.cpp:319-336: wstart at the bbox's first pixel centre and the per-pixel / per-row steps from the
// three raster corners (x, y).  Shared by the setup and by the tile raster, which recomputes them from
// the corners in its 48-B records (the same operations on the same operands: the same floats).
__device__ __forceinline__ void raster_steps(F3 a, F3 b, F3 c, uint32_t xmin, uint32_t ymin, float *ws, float *dx,
                                             float *dy) {
    const float area = edge_fn(a, b, c.x, c.y);
    const float ooa = 1 / area;
    const float px = (float)xmin + 0.5f, py = (float)ymin + 0.5f;
    ws[0] = edge_fn(b, c, px, py) * ooa;
    ws[1] = edge_fn(c, a, px, py) * ooa;
    ws[2] = edge_fn(a, b, px, py) * ooa;
    dx[0] = (b.y - c.y) * ooa;
    dx[1] = (c.y - a.y) * ooa;
    dx[2] = (a.y - b.y) * ooa;
    dy[0] = (c.x - b.x) * ooa;
    dy[1] = (a.x - c.x) * ooa;
    dy[2] = (b.x - a.x) * ooa;
}

// render.cpp:311-336, the position-only part of the setup: reject / cull (:312, :314, :317), bbox,
// wstart, per-pixel and per-row steps, 1/z per corner.  False = no pixel of the frame.
__device__ __forceinline__ bool raster_part(const Vert d[3], float sw, float sh, TriSetup &t) {
    const float rmx = fmaxf(fmaxf(d[0].rv.x, d[1].rv.x), d[2].rv.x);
    const float rmy = fmaxf(fmaxf(d[0].rv.y, d[1].rv.y), d[2].rv.y);
    const float rnx = fminf(fminf(d[0].rv.x, d[1].rv.x), d[2].rv.x);
    const float rny = fminf(fminf(d[0].rv.y, d[1].rv.y), d[2].rv.y);
    const float area = edge_fn(d[0].rv, d[1].rv, d[2].rv.x, d[2].rv.y);
    if (rmx < 0 || rmy < 0 || rnx >= sw || rny >= sh || area < 10) return false;   // :312, :314, :317
    t.xmin = u32_of_float(fmaxf(0, rnx));
    t.xmax = u32_of_float(fminf(sw - 1, rmx));
    t.ymin = u32_of_float(fmaxf(0, rny));
    t.ymax = u32_of_float(fminf(sh - 1, rmy));
    raster_steps(d[0].rv, d[1].rv, d[2].rv, t.xmin, t.ymin, t.ws, t.dx, t.dy);
    t.ws[3] = t.dx[3] = t.dy[3] = t.rvz[3] = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; k++) t.rvz[k] = 1 / d[k].rv.z;
    return true;
}

// render.cpp:337-352, the shading constants, from the raster part's 1/z per corner and steps
// (t.rvz, t.dx, t.dy).
__device__ __forceinline__ void shading_part(const Vert d[3], bool textured, TriSetup &t) {
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float r = t.rvz[k];
        t.cvr[4 * k + 0] = d[k].cv.x * r; t.cvr[4 * k + 1] = d[k].cv.y * r; t.cvr[4 * k + 2] = d[k].cv.z * r;
        t.nr[4 * k + 0] = d[k].n.x * r; t.nr[4 * k + 1] = d[k].n.y * r; t.nr[4 * k + 2] = d[k].n.z * r;
        t.cvr[4 * k + 3] = t.nr[4 * k + 3] = 0.0f;
    }
    if (!textured) {
        t.kind = kColour;
        t.tex_base = 0;
#pragma unroll
        for (int k = 0; k < 3; k++) {
            t.col[4 * k + 0] = d[k].pay.x * t.rvz[k];
            t.col[4 * k + 1] = d[k].pay.y * t.rvz[k];
            t.col[4 * k + 2] = d[k].pay.z * t.rvz[k];
            t.col[4 * k + 3] = 0.0f;
        }
    } else {
        t.kind = kTexture;
        t.tex_base = (uint32_t)((int32_t)f2u(d[0].pay.x) << 18);          // render.cpp:347
        const float u0 = d[0].pay.z * t.rvz[0], v0 = d[0].pay.w * t.rvz[0];
        const float u1 = d[1].pay.z * t.rvz[1], v1 = d[1].pay.w * t.rvz[1];
        const float u2 = d[2].pay.z * t.rvz[2], v2 = d[2].pay.w * t.rvz[2];
        const float dzx = (t.rvz[0] * t.dx[0] + t.rvz[1] * t.dx[1]) + t.rvz[2] * t.dx[2];
        const float dzy = (t.rvz[0] * t.dy[0] + t.rvz[1] * t.dy[1]) + t.rvz[2] * t.dy[2];
        const float tx = (u0 * t.dx[0] + u1 * t.dx[1]) + u2 * t.dx[2];
        const float ty = (v0 * t.dy[0] + v1 * t.dy[1]) + v2 * t.dy[2];
        t.col[0] = u0; t.col[1] = v0; t.col[2] = u1; t.col[3] = v1;
        t.col[4] = u2; t.col[5] = v2; t.col[6] = dzx; t.col[7] = dzy;
        t.col[8] = tx; t.col[9] = ty; t.col[10] = t.col[11] = 0.0f;
    }
}

// render.cpp:311-359 for one (possibly clipped) triangle.
__device__ __forceinline__ void setup_tri(const Vert d[3], bool textured, float sw, float sh, TriSetup *out) {
    TriSetup t;
    t.kind = kDead;
    t.pad0 = t.pad1 = 0;
    if (!raster_part(d, sw, sh, t)) {
        out->kind = kDead;
        return;
    }
    shading_part(d, textured, t);
    *out = t;
}

// Slot s of the frame's triangle list, set up exactly as the reference's loop meets it
// (render.cpp:285-359): slot t < T is original triangle t after the :306 reject and the near-plane
// clip (:308, which may edit it), slot T + t the triangle clip() appended while processing t
// (:239-257; dead when none).  The vertex and normal transforms of the three corners (:285-292) are
// done in place, so the frame needs no camera-space vertex arrays.
__device__ void geo_slot_setup(uint32_t s, uint32_t ntri, const float4 *__restrict__ vtx,
                               const float4 *__restrict__ nrm, const float4 *__restrict__ pay,
                               const uint8_t *__restrict__ disc, const uint32_t *__restrict__ vidx,
                               const uint32_t *__restrict__ aidx, const Mat34 &m, float factor, float sw, float sh,
                               TriSetup &out) {
    const uint32_t t = s < ntri ? s : s - ntri;
    const float half_w = sw / 2, half_h = sh / 2;
    out.kind = kDead;
    Vert d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t vi = vidx[3 * t + k], ai = aidx[3 * t + k];
        const F3 c = mat_mul(m, vtx[vi]);                                  // :286
        const float nz = -c.z;
        d[k].cv = c;
        // (cv.x, -cv.y, 0) * factor / -cv.z + (W/2, H/2, -cv.z)            // :288
        d[k].rv = mk3((c.x * factor) / nz + half_w, ((-c.y) * factor) / nz + half_h, (0.0f * factor) / nz + nz);
        d[k].n = mat_mul(m, nrm[ai]);                                       // :291
        d[k].pay = pay[ai];
    }
    const bool textured = disc[aidx[3 * t]] != 0;                        // data[0].ca.disc, :340
    if (fmaxf(fmaxf(d[0].rv.z, d[1].rv.z), d[2].rv.z) <= kNear) return;  // :306
    Vert app[3];
    uint32_t app_first = 0;
    bool appended = false;
    if (fminf(fminf(d[0].rv.z, d[1].rv.z), d[2].rv.z) < kNear)            // :308
        appended = clip_tri(d, app, &app_first, textured, factor, half_w, half_h);
    if (s < ntri) {
        setup_tri(d, textured, sw, sh, &out);
    } else if (appended) {
        // The appended triangle is (vi[cur], new, new) with z = (z_cur > near, near, near): neither
        // the :306 reject nor another clip can trigger when the reference loop reaches it.  Its
        // data[0] is the original attribute ai[cur], whose disc picks its colour path.
        setup_tri(app, disc[aidx[3 * t + app_first]] != 0, sw, sh, &out);
    }
}

#ifdef S3R_STATS
__device__ unsigned long long g_stats[16];
__device__ unsigned long long g_tstats[8];   // k_geometry wall-clock (100 MHz) profile, stats build

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
    for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}
#define S3R_IT(p) , (p)
#else
#define S3R_IT(p)
#endif

// Timing build (-DS3R_WGTIME, tools/wg_timeline.py): per-workgroup phase timestamps of k_fragment.
#ifdef S3R_WGTIME
constexpr uint32_t kWgTimesMax = 65536;
// slots 0-3: wave 0's 100 MHz wall clock at start, list loaded, walk state loaded, end; 4-6: wave 0's
// shader-clock cycles summed over its chunks in batch 0, later batches, shading + stores; 7: list length;
// 8-10: wave 0's chunks whose batch 0 took the slow (walk + linear_run) path, had a non-linear
// component, and the live triangles its pixel phases tested
constexpr uint32_t kWgSlots = 12;
__device__ unsigned long long g_wgt[kWgTimesMax * kWgSlots];
#define S3R_WGT(k) do { if (threadIdx.x == 0 && blockIdx.x < kWgTimesMax) g_wgt[blockIdx.x * kWgSlots + (k)] = wall_clock64(); } while (0)
#define S3R_WGC_DECL unsigned long long wgc_t = 0, wgc[3] = {0, 0, 0}; uint32_t wgn[3] = {0, 0, 0}
#define S3R_WGN(k, v) (wgn[k] += (v))
#define S3R_WGC_MARK() (wgc_t = clock64())
#define S3R_WGC_ADD(k) (wgc[k] += clock64() - wgc_t)
#define S3R_WGC_STORE(n) do { if (threadIdx.x == 0 && blockIdx.x < kWgTimesMax) { \
    for (int i_ = 0; i_ < 3; i_++) g_wgt[blockIdx.x * kWgSlots + 4 + i_] = wgc[i_]; \
    g_wgt[blockIdx.x * kWgSlots + 7] = (n); \
    for (int i_ = 0; i_ < 3; i_++) g_wgt[blockIdx.x * kWgSlots + 8 + i_] = wgn[i_]; } } while (0)
// k_geometry workgroups (slot * 64 + row block): 0 start, 1 slot set up, 2 bins set, 3 last wave done
constexpr uint32_t kGeoTimesMax = 16384;
__device__ unsigned long long g_gwt[kGeoTimesMax * 4];
#define S3R_GWT(k) do { const uint32_t g_ = slot * 64u + rb; \
    if (threadIdx.x == 0 && g_ < kGeoTimesMax) g_gwt[g_ * 4 + (k)] = wall_clock64(); } while (0)
#define S3R_GWT_END() do { const uint32_t g_ = slot * 64u + rb; \
    if ((threadIdx.x & 63u) == 0 && g_ < kGeoTimesMax) atomicMax(&g_gwt[g_ * 4 + 3], wall_clock64()); } while (0)
#else
#define S3R_GWT(k) do { } while (0)
#define S3R_GWT_END() do { } while (0)
#define S3R_WGT(k) do { } while (0)
#define S3R_WGC_DECL do { } while (0)
#define S3R_WGC_MARK() do { } while (0)
#define S3R_WGC_ADD(k) do { } while (0)
#define S3R_WGC_STORE(n) do { } while (0)
#define S3R_WGN(k, v) do { } while (0)
#endif

// ------------------------------------------------------------------ ripmap sample
// getTextureColor's texel offset inside one 512 x 512 ripmap (render.cpp:124-132)
__device__ __forceinline__ uint32_t texel_offset(float u, float v, float lvx, float lvy) {
    const uint32_t ix = (uint32_t)(int32_t)fmaxf(fminf(lvx, 256.f), 1.f);
    const uint32_t iy = (uint32_t)(int32_t)fmaxf(fminf(lvy, 256.f), 1.f);
    const uint32_t lx = ix > 1u ? 1u << (32u - (uint32_t)__builtin_clz(ix - 1u)) : 1u;
    const uint32_t ly = iy > 1u ? 1u << (32u - (uint32_t)__builtin_clz(iy - 1u)) : 1u;
    const uint32_t x = u32_of_float(frac1(u) * (float)lx) + (511u & ~(2u * lx - 1u));
    const uint32_t y = u32_of_float(frac1(v) * (float)ly) + (511u & ~(2u * ly - 1u));
    return (x + (y << 9)) & (kTexTexels - 1u);
}

__device__ __forceinline__ uint32_t texel(const uint32_t *__restrict__ tex, uint32_t ntex, uint32_t base,
                                          float u, float v, float lvx, float lvy) {
    // getTextureColor, render.cpp:124-132
    // levels clamped to [1, 256] (fminf(NaN, 256) = 256): the truncation needs no range guard and
    // nextPowerOfTwo of i in [1, 256] is 1 << (32 - clz(i - 1)) for i > 1
    const uint32_t off = texel_offset(u, v, lvx, lvy);
    // Out-of-range texture index is UB in the reference; defined here (and in the oracle) as 0.
#if defined(S3R_ABLATE) && (S3R_ABLATE & 256)
    return off * 0x010101u + base;                 // ablation: no texel load
#endif
    return (base < ntex && ntex - base >= kTexTexels) ? tex[base + off] : 0u;
}

// ------------------------------------------------------------------ K4: fragment
constexpr uint32_t kTPB = 21;          // triangles per batch: lane = 3 * t + component (63 lanes)
#ifndef S3R_WAVES
#define S3R_WAVES 4
#endif
constexpr uint32_t kWaves = S3R_WAVES; // one wave per row: a workgroup is kWaves consecutive local rows
static_assert(kWaves == 4, "pair records carry the walk state of 4 rows (s3r_kernels.h)");
static_assert(kWaves * 6 <= 32, "host fill: a bin's chunk mask (rows x chunks) fits 32 bits");
// triangles listed per workgroup (rows x segment) by the in-kernel list rounds of bins met by more than
// kPairMax triangles: five batches.  (128 until round 5; with the padded tables, kTabStride, a workgroup's
// LDS must stay within 26 KiB -- 6 workgroups per CU at the LDS's allocation granularity: at 27 248 B the
// launch ran 5 per CU and the 4K kernel took 52.0 instead of 48.7 us, profiles/r06_tabpad_ab.txt.)
constexpr uint32_t kListMax = 5 * kTPB;
#ifndef S3R_STATE_BATCHES
#define S3R_STATE_BATCHES 4
#endif
#ifndef S3R_TABLES
#define S3R_TABLES 12
#endif
#ifndef S3R_OCC
#define S3R_OCC 5                      // target waves per SIMD (5: no spills at <= 96 VGPRs)
#endif
#ifndef S3R_PX
#define S3R_PX 1
#endif
#ifndef S3R_WORK_SKY
#define S3R_WORK_SKY 8                 // a sky bin's work units (its fill of the background)
#endif
#ifndef S3R_LINE_STORES
#define S3R_LINE_STORES 1              // HOSTW: wave stores on the caller buffer's 64-B line grid
#endif
constexpr uint32_t kNoPixel = 0xFFFFFFFFu;   // no store (pixels are 0x00RRGGBB)
constexpr uint32_t kPX = S3R_PX;       // pixels per lane: a chunk is 64 * kPX consecutive pixels of a row
constexpr uint32_t kChunk = 64u * kPX;
constexpr uint32_t kStateBatches = S3R_STATE_BATCHES;  // batches whose walk state persists in LDS
constexpr uint32_t kTables = S3R_TABLES;  // per wave: 64-entry exact-value tables, non-linear chunks
#ifndef S3R_TAB_PAD
#define S3R_TAB_PAD 4                  // floats of padding per table row (see kTabStride)
#endif
// A table row is kChunk floats plus S3R_TAB_PAD: the fill's ds_write_b128 of up to kTables lanes at
// the same column lands, in each 8-lane group, on eight different 4-bank groups (row stride 68 words
// = 4 banks mod 32) instead of the same four banks (stride 64 words: an 8-way conflict, 35 % of the
// launch's LDS cycles in round 5).  The pixel reads stay lane-contiguous.
constexpr uint32_t kTabStride = kChunk + S3R_TAB_PAD;
static_assert(kTabStride % 4u == 0u, "16-B aligned table rows");

struct alignas(16) Entry {              // 48 B per listed triangle (LDS, shared by the 4 waves)
    uint32_t slot, xmin, xmax, ymin;
    uint32_t ymax;
    float dx[3];
    float rvz[3];
    uint32_t pad;
};

struct FragShared {
    Entry ent[kListMax];
    float st_c[kWaves][kStateBatches * 64];
    uint32_t st_k[kWaves][kStateBatches * 64];
    float4 tab4[kWaves][kTables][kTabStride / 4];  // exact S(c, d, k), k < kChunk, filled by sequential adds
    uint32_t cnt, next;
    uint32_t bgm[kWaves];                // host fill: per wave (row), its chunks left to the host
    uint32_t wwork[kWaves];              // per wave: its work units (the bin's cost, order_bins)
};
static_assert(offsetof(FragShared, tab4) % 16 == 0, "16-B table rows");
static_assert(sizeof(FragShared) <= 26u * 1024u, "k_fragment: 6 workgroups per CU (see kListMax)");
// k_fragment stages a bin's pair records in tab4 before the chunk loop (s3r_kernels.h kPairMax x
// kPairWords uint4): a tuning build with fewer tables must still leave room for them.
static_assert(sizeof(((FragShared *)nullptr)->tab4) >= 64u * 8u * sizeof(uint4),
              "pair staging (kPairMax * kPairWords uint4) must fit in tab4");

__device__ __forceinline__ uint32_t lane_prefix(uint64_t mask, uint32_t lane) {
    return (uint32_t)__builtin_popcountll(mask & ((1ull << lane) - 1ull));
}

__device__ __forceinline__ float rdl(float v, uint32_t l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), (int)l));
}
__device__ __forceinline__ uint32_t rdl(uint32_t v, uint32_t l) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l);
}

// LDS hand-off between lanes of ONE wave: LDS operations of a wave execute in order, so only the
// compiler must be kept from reordering across this point.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Walker and shader inlined (default): no call frame, no scratch stack (measured 72.6 vs 75.1 us per
// 4K P_over launch against the out-of-line build, S3R_INLINE=0).
#ifndef S3R_INLINE
#define S3R_INLINE 1
#endif
#if S3R_INLINE
#define S3R_CALLEE __device__ __forceinline__
#else
#define S3R_CALLEE __device__ __noinline__
#endif
S3R_CALLEE float walk(float s, float d, uint32_t n
#ifdef S3R_STATS
                                   , uint32_t *iters
#endif
) {
#ifdef S3R_STATS
    return exact_walk(s, d, n, iters);
#else
    return exact_walk(s, d, n);
#endif
}


// All waves copy the raster constants of the listed slots (sh.ent[i].slot, i < cnt) into LDS.
__device__ __forceinline__ void load_entries(const TriSetup *__restrict__ tris, FragShared &sh, uint32_t cnt,
                                             uint32_t wave, uint32_t lane) {
    for (uint32_t i = wave * 64 + lane; i < cnt; i += kWaves * 64) {
        const TriSetup *t = tris + sh.ent[i].slot;
        const uint4 h0 = reinterpret_cast<const uint4 *>(t)[0];
        const uint4 h1 = reinterpret_cast<const uint4 *>(t)[1];
        const float4 dx = reinterpret_cast<const float4 *>(t)[3];
        const float4 rz = reinterpret_cast<const float4 *>(t)[5];
        Entry &e = sh.ent[i];
        e.xmin = h0.y; e.xmax = h0.z; e.ymin = h0.w; e.ymax = h1.x;
        e.dx[0] = dx.x; e.dx[1] = dx.y; e.dx[2] = dx.z;
        e.rvz[0] = rz.x; e.rvz[1] = rz.y; e.rvz[2] = rz.z;
    }
    __syncthreads();
}

// Wave 0 lists, in slot order, the live triangles whose bbox meets rows [y0, y1] and columns
// [x0, x1], starting at slot `cursor`, at most kListMax; then all waves copy each listed triangle's
// raster constants into LDS.  Must be reached by every wave of the workgroup.
__device__ void build_list(const TriSetup *__restrict__ tris, uint32_t nslots, uint32_t y0, uint32_t y1,
                           uint32_t x0, uint32_t x1, uint32_t cursor, FragShared &sh, uint32_t wave,
                           uint32_t lane) {
    __syncthreads();
    if (wave == 0) {
        uint32_t cnt = 0;
        while (cursor < nslots) {
            const uint32_t s = cursor + lane;
            bool act = false;
            if (s < nslots) {
                const uint4 h0 = reinterpret_cast<const uint4 *>(tris + s)[0];    // kind xmin xmax ymin
                const uint32_t ymax = reinterpret_cast<const uint4 *>(tris + s)[1].x;
                act = h0.x != kDead && h0.w <= y1 && ymax >= y0 && h0.y <= x1 && h0.z >= x0;
            }
            uint64_t mask = __ballot(act);
            const uint32_t room = kListMax - cnt;
            uint32_t pc = (uint32_t)__builtin_popcountll(mask);
            uint32_t adv = 64;
            if (pc > room) {
                uint64_t rest = mask;
                for (uint32_t i = 0; i < room; i++) rest &= rest - 1;
                adv = (uint32_t)__builtin_ctzll(rest);          // first slot that does not fit
                mask ^= rest;
                pc = room;
            }
            if (act && ((mask >> lane) & 1ull)) sh.ent[cnt + lane_prefix(mask, lane)].slot = s;
            cnt += pc;
            cursor += adv;
            if (cnt == kListMax) break;
        }
        if (lane == 0) { sh.cnt = cnt; sh.next = cursor < nslots ? cursor : nslots; }
    }
    __syncthreads();
    load_entries(tris, sh, sh.cnt, wave, lane);
}

// rowtab: exact walk values of a row at x = xmin (j = 0) and at every start-table boundary
// x = j' * kStartPx inside (xmin, xmax] (j = 1 + j').  The start point of a walk to pixel xs >= xmin:
// the last tabulated point at or before xs.  Fragment segments narrower than kStartPx walk the
// remaining < kStartPx pixels themselves (a few exact_walk iterations), so the geometry's serial
// chain does not grow with the number of fragment segments.
constexpr uint32_t kStartPx = 384;
// row_starts: the launch's geometry tabulated the row starts only (delivered frames, below): every
// walk starts at x = xmin.
__device__ __forceinline__ uint32_t start_index(uint32_t xmin, uint32_t xs, uint32_t *k, bool row_starts = false) {
    const uint32_t jb = xs / kStartPx;
    if (row_starts || xs <= xmin || jb * kStartPx <= xmin) { *k = xmin; return 0u; }
    *k = jb * kStartPx;
    return 1u + jb;
}
S3R_HD uint32_t start_entries_of(uint32_t W) { return (W + kStartPx - 1) / kStartPx + 1u; }
uint32_t start_entries(uint32_t W) { return start_entries_of(W); }

// Longest-first order of the fragment bins (workgroups): a fragment launch is several rounds of
// resident workgroups whose costs differ ~8x (textured floor rows vs sky), and the launch order
// (top-down) can leave the costliest rows for the last round.  One workgroup counting-sorts the bins
// by their cost when the buffer set was last used (k_fragment's order[n + bin], work units; stale
// values from another frame size are only hints; no fragment launch of the set runs meanwhile, so
// both passes read the same values) into kOrderBuckets quarter-octave buckets,
// costliest first; perm is always a permutation of [0, n).
#ifndef S3R_ORDER_STEPS
#define S3R_ORDER_STEPS 8              // buckets per octave of cost (4: 50.9 vs 50.5 us at 4K, profiles/r05_order_ab.txt)
#endif
constexpr uint32_t kOrderSteps = S3R_ORDER_STEPS, kOrderBuckets = 8u * kOrderSteps;
// bucket of a cost: 1 / kOrderSteps octave each over 8 octaves from 2^6 units (a sky bin: kWorkSky) --
// no max pass over the costs
__device__ __forceinline__ uint32_t order_bucket(uint32_t c) {
    const float l = __log2f((float)max(c, 64u)) * (float)kOrderSteps - 6.0f * (float)kOrderSteps;
    return min((uint32_t)l, kOrderBuckets - 1u);
}
// the two passes read kOrderUnroll costs per thread before using them (independent loads in flight)
constexpr uint32_t kOrderUnroll = 8;
__device__ void order_bins(const uint32_t *__restrict__ cost, uint32_t n, uint32_t *__restrict__ perm) {
    __shared__ uint32_t hist[kOrderBuckets];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (tid < kOrderBuckets) hist[tid] = 0;
    __syncthreads();
    for (uint32_t base = 0; base < n; base += kOrderUnroll * nt) {
        uint32_t b[kOrderUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kOrderUnroll; u++) {
            const uint32_t i = base + u * nt + tid;
            b[u] = i < n ? order_bucket(cost[i]) : kOrderBuckets;
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrderUnroll; u++)
            if (b[u] < kOrderBuckets) atomicAdd(&hist[b[u]], 1u);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t run = 0;
        for (int b = (int)kOrderBuckets - 1; b >= 0; b--) { const uint32_t c = hist[b]; hist[b] = run; run += c; }
    }
    __syncthreads();
    for (uint32_t base = 0; base < n; base += kOrderUnroll * nt) {
        uint32_t b[kOrderUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kOrderUnroll; u++) {
            const uint32_t i = base + u * nt + tid;
            b[u] = i < n ? order_bucket(cost[i]) : kOrderBuckets;
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrderUnroll; u++)
            if (b[u] < kOrderBuckets) perm[atomicAdd(&hist[b[u]], 1u)] = base + u * nt + tid;
    }
}

// Host fill: the bins' sky flags, published from inside k_geometry, one extra workgroup per row block
// of kGeoRows local rows (dispatched before the geometry workgroups): every geometry workgroup counts
// itself, once its bin phase is over (or at once for a dead slot), in its row block's counter
// (geo_cnt[rb * kGeoCntStride], own cache line); the row block's publisher spins until its 2T
// arrivals are in, reads the final counts of the row block's bins with device-scope (L2-bypassing)
// loads -- every bincnt atomicAdd of a workgroup returned before its barrier and its arrival was
// issued after it -- and stores flags[b] = tag, | kSkyBit for a bin no slot meets (the host fills
// it), | kGpuBit instead for sky bins with b % 8 < gpu_eighths (the fragment kernel writes their
// background).  probe: pixel 0 of the caller's buffer, set to kMapProbe through the mapping before
// flags[0] is published (the host's stale-mapping check).  Each publisher then resets its counter
// for the buffer set's next frame (no arrival is left: its row block had all of its 2T).
constexpr uint32_t kGeoCntStride = 16;           // uint32 words: one 64-B line per row block
constexpr uint32_t kGeoCntMax = 256;             // row blocks with a counter (more: k_sky_flags)
static_assert(kGeoCntMax * kGeoCntStride == kGeoCounterWords, "geometry counters: s3r_kernels.h's size");
// The publisher's spin is bounded: past spin_ticks of the device clock (100 MHz) it stores
// {kDiagPublisherTimeout, rb, arrivals seen, arrivals} into err (host-coherent) and returns without
// publishing; the host's fill threads report it and end the process (render_api.cpp fill_worker).
struct SkyFlags {
    uint32_t *flags;                  // null: no host fill
    uint32_t *probe;
    uint32_t *geo_cnt;
    uint32_t tag, gpu_eighths;
    uint32_t *err;
    uint32_t arrivals;                // geometry workgroups per row block (the host's launch count)
    uint32_t spin_ticks;
};

// the row block rb's bins: [rb * rb_bins, (rb + 1) * rb_bins), rb_bins = its fragment row blocks x segs
__device__ void publish_sky_flags(const SkyFlags &sf, const uint32_t *__restrict__ bincnt, uint32_t nbins,
                                  uint32_t rb_bins, uint32_t rb) {
    uint32_t *cnt = sf.geo_cnt + rb * kGeoCntStride;
    __shared__ uint32_t timed_out;
    if (threadIdx.x == 0) {
        timed_out = 0u;
        const uint64_t t0 = wall_clock64();
        uint32_t seen;
        while ((seen = __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) < sf.arrivals) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > sf.spin_ticks) {
                timed_out = 1u;
                if (sf.err) {
                    __hip_atomic_store(sf.err + 1, rb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(sf.err + 2, seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(sf.err + 3, sf.arrivals, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(sf.err, kDiagPublisherTimeout, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
                break;
            }
        }
    }
    __syncthreads();
    if (timed_out) return;
    const uint32_t b0 = rb * rb_bins, b1 = min(nbins, b0 + rb_bins);
    // kPubUnroll counts per thread in flight at once (the loads go to memory: one round trip each)
    constexpr uint32_t kPubUnroll = 4;
    for (uint32_t base = b0; base < b1; base += kPubUnroll * blockDim.x) {
        uint32_t cs[kPubUnroll];
#pragma unroll
        for (uint32_t u = 0; u < kPubUnroll; u++) {
            const uint32_t b = base + u * blockDim.x + threadIdx.x;
            cs[u] = b < b1 ? __hip_atomic_load(bincnt + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0u;
        }
#pragma unroll
        for (uint32_t u = 0; u < kPubUnroll; u++) {
            const uint32_t b = base + u * blockDim.x + threadIdx.x;
            if (b >= b1) break;
            const uint32_t f = cs[u] != 0u ? sf.tag : ((b & 7u) < sf.gpu_eighths ? (sf.tag | kGpuBit) : (sf.tag | kSkyBit));
            if (b == 0 && sf.probe) {
                // the probe reaches the caller's page before flag 0 does: both are stores over the link
                // from this thread, the second issued once the first completed (rather than a
                // system-scope release, which would first write back the whole L2)
                __hip_atomic_store(sf.probe, kMapProbe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __builtin_amdgcn_s_waitcnt(0);
                __hip_atomic_store(sf.flags, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            } else {
                __hip_atomic_store(sf.flags + b, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// the k-th set bit of the host's slot mask (wave-uniform: scalar loads of the kernel argument)
__device__ __forceinline__ uint32_t live_slot(const SlotMask &m, uint32_t k) {
    uint32_t w = 0;
    for (; w + 1 < kLiveMaskSlots / 64; w++) {
        const uint32_t c = (uint32_t)__popcll(m.bits[w]);
        if (k < c) break;
        k -= c;
    }
    uint64_t b = m.bits[w];
    for (; k; k--) b &= b - 1ull;
    return w * 64u + (uint32_t)__builtin_ctzll(b);
}

__device__ __forceinline__ void geo_arrive(const SkyFlags &sf, uint32_t rb) {
    if (sf.flags && threadIdx.x == 0) atomicAdd(sf.geo_cnt + rb * kGeoCntStride, 1u);
}

// ------------------------------------------------------------------ K1: geometry, one launch
// Per frame, on the geometry stream (overlapping the previous frame's fragment kernel): one
// workgroup per (slot, block of kGeoRows local rows) x 3 components.
//   * thread 0 sets the slot up (geo_slot_setup: transform, reject, clip, cull, raster setup,
//     render.cpp:285-359); the row-block-0 workgroup stores the slot's TriSetup record;
//   * bins: the slot reserves a pair record (atomicAdd on the bin's count) in every fragment
//     workgroup's bin (kWaves local rows x one segment) its bbox meets and writes its raster
//     constants and walk state there -- the fragment workgroup ranks its pairs by slot (the
//     reference's processing order) and resets the count for the buffer set's next frame;
//   * starts: lane (row, component) walks the reference's sequence exactly (exact_walk): wy += dy
//     down to its row (render.cpp:378), then w += dx along the row through every fragment-segment
//     boundary inside the bbox (:374), storing the row start and each segment start.
// rowtab[((slot * rows_local + lr) * nst + j) * 4 + c], nst = start_entries(W): j = 0 at x = xmin,
// j = 1 + j' at x = j' * kStartPx (only boundaries in (xmin, xmax] are written).
#ifndef S3R_GEO_ROWS
#define S3R_GEO_ROWS 128
#endif
constexpr uint32_t kGeoRows = S3R_GEO_ROWS;
static_assert(kGeoRows % kWaves == 0, "geometry row blocks hold whole fragment row blocks");

#ifndef S3R_GEO_OCC
#define S3R_GEO_OCC 5                  // min waves per SIMD of k_geometry: 96 VGPRs (115 uncapped), see DESIGN
#endif
__global__ void __launch_bounds__(3 * kGeoRows, S3R_GEO_OCC) k_geometry(
    const float4 *__restrict__ vtx, const float4 *__restrict__ nrm, const float4 *__restrict__ pay,
    const uint8_t *__restrict__ disc, const uint32_t *__restrict__ vidx, const uint32_t *__restrict__ aidx,
    uint32_t ntri, Mat34 m, float factor, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
    uint32_t rows_local, uint32_t segs, uint32_t segw, TriSetup *__restrict__ tris,
    float *__restrict__ rowtab, uint32_t *__restrict__ bincnt, uint4 *__restrict__ pairs,
    uint32_t nbins, uint32_t *__restrict__ order, uint32_t nrb, SkyFlags sky, uint32_t row_starts,
    uint32_t nslots, SlotMask live) {
    __shared__ TriSetup sts;
    extern __shared__ uint8_t posmap[];        // per bin of this workgroup: its pair index, 0xFF = none
    // slot-major 1-D grid: workgroup 0 (with `order`) computes this frame's fragment order, then the
    // row blocks of slot 0, of slot 1, ...  The dispatcher starts workgroups in index order, so a
    // slot's row blocks start together and the appended clip slots (2T > slot >= T, dead unless
    // the near plane cut their triangle) come last: a large triangle's long walks start within the
    // first microsecond instead of after every slot's earlier row blocks.
    const uint32_t g0 = blockIdx.x;
    if (order && g0 == 0) {
        order_bins(order + nbins, nbins, order);
        return;
    }
    // publishers, the dead-slot marker (host cull), geometry
    const uint32_t pub0 = order ? 1u : 0u, mark0 = pub0 + (sky.flags ? nrb : 0u), first = mark0 + live.on;
    if (sky.flags && g0 < mark0) {
        publish_sky_flags(sky, bincnt, nbins, (kGeoRows / kWaves) * segs, g0 - pub0);
        return;
    }
    if (live.on && g0 == mark0) {
        // the slots the host culled, and every clip slot (none launched with the mask): dead
        for (uint32_t s = threadIdx.x; s < ntri; s += blockDim.x)
            if (!((live.bits[s >> 6] >> (s & 63u)) & 1ull)) tris[s].kind = tris[ntri + s].kind = kDead;
        return;
    }
    const uint32_t tid = threadIdx.x, gs = g0 - first, gk = gs / nrb, rb = gs - gk * nrb;
    const uint32_t slot = live.on ? live_slot(live, gk) : gk;
#ifdef S3R_STATS
    const unsigned long long t_start = wall_clock64();
    if (tid == 0) atomicMin(&g_tstats[2], t_start);
#endif
    S3R_GWT(0);
    if (tid == 0) {
        TriSetup t;
        geo_slot_setup(slot, ntri, vtx, nrm, pay, disc, vidx, aidx, m, factor, (float)W, (float)H, t);
        sts = t;
        if (rb == 0) tris[slot] = t;
        if (rb == 0 && nslots == ntri) tris[ntri + slot].kind = kDead;   // (clip slots left out: dead)
#ifdef S3R_STATS
        atomicMax(&g_tstats[0], wall_clock64() - t_start);
#endif
    }
    __syncthreads();
    S3R_GWT(1);
    if (sts.kind == kDead) {
        geo_arrive(sky, rb);
        S3R_GWT_END();
        return;
    }
    const uint32_t xmin = sts.xmin, xmax = sts.xmax, ymin = sts.ymin, ymax = sts.ymax;
    auto row_of = [&](uint32_t lr) { return ((lr / band) * nparts + part) * band + lr % band; };

    // bins of this workgroup's rows: (kGeoRows / kWaves) fragment row blocks x segs segments.  The
    // slot takes the next pair of every bin its bbox meets (the count is reset by the bin's fragment
    // workgroup, the last reader of this buffer set) and writes its raster constants there; the walks
    // below add the exact walk state of the bin's rows.  Four bins per thread per step, so their
    // atomics are in flight together.
    const uint32_t nbr = kGeoRows / kWaves, nq = nbr * segs;
    constexpr uint32_t kQ = 4;
    for (uint32_t q0 = 0; q0 < nq; q0 += kQ * 3 * kGeoRows) {
        uint32_t pos[kQ];
#pragma unroll
        for (uint32_t u = 0; u < kQ; u++) {
            const uint32_t q = q0 + u * 3 * kGeoRows + tid;
            pos[u] = kPairMax;
            if (q >= nq) continue;
            const uint32_t blk = rb * nbr + q / segs, sg = q % segs;
            const uint32_t lr0 = blk * kWaves;
            if (lr0 >= rows_local) continue;
            uint32_t y0 = 0xFFFFFFFFu, y1 = 0;
            for (uint32_t k = 0; k < kWaves && lr0 + k < rows_local; k++) {
                const uint32_t yy = row_of(lr0 + k);
                y0 = min(y0, yy); y1 = max(y1, yy);
            }
            const uint32_t x0 = sg * segw, x1 = min(W, x0 + segw) - 1u;
            if (ymin <= y1 && ymax >= y0 && xmin <= x1 && xmax >= x0)
                pos[u] = atomicAdd(&bincnt[(size_t)blk * segs + sg], 1u);
        }
#pragma unroll
        for (uint32_t u = 0; u < kQ; u++) {
            const uint32_t q = q0 + u * 3 * kGeoRows + tid;
            if (q >= nq) continue;
            posmap[q] = pos[u] < kPairMax ? (uint8_t)pos[u] : (uint8_t)0xFF;
            if (pos[u] < kPairMax) {
                const size_t bin = (size_t)(rb * nbr + q / segs) * segs + q % segs;
                uint4 *pr = pairs + (bin * kPairMax + pos[u]) * kPairWords;
                pr[0] = make_uint4(slot, xmin, xmax, ymin);
                pr[1] = make_uint4(ymax, 0u, 0u, 0u);
                pr[2] = make_uint4(f2u(sts.dx[0]), f2u(sts.dx[1]), f2u(sts.dx[2]), 0u);
                pr[3] = make_uint4(f2u(sts.rvz[0]), f2u(sts.rvz[1]), f2u(sts.rvz[2]), 0u);
            }
        }
    }
    __syncthreads();
    geo_arrive(sky, rb);
    S3R_GWT(2);

    // exact row and start-table points: lane (row, component) walks the reference's sequence exactly
    // (exact_walk): wy += dy down to its row (render.cpp:378), then w += dx along the row through every
    // kStartPx boundary inside the bbox (:374); each value goes to the start table and to the pairs of
    // the fragment segments whose walks start there (start_index)
    const uint32_t c = tid / kGeoRows, lr = rb * kGeoRows + tid % kGeoRows;
    const uint32_t y = row_of(lr);
    if (lr >= rows_local || y < ymin || y > ymax || y >= H) { S3R_GWT_END(); return; }
#if defined(S3R_GEO_ABLATE)                  // 2 = no walks at all
    if (S3R_GEO_ABLATE & 2) return;
#endif
    const uint32_t nst = start_entries_of(W);
    float *row = rowtab + ((size_t)slot * rows_local + lr) * nst * 4 + c;
    const uint8_t *pm = posmap + (lr / kWaves - rb * nbr) * segs;
    float *pst = reinterpret_cast<float *>(pairs) + 16u + (lr % kWaves) * 3u + c;   // state float in pair 0
    const size_t bin0 = (size_t)(lr / kWaves) * segs;
    // the fragment segments [sg, sg_end) take their walk state from value v
    auto to_pairs = [&](uint32_t sg, uint32_t sg_end, float v) {
        for (; sg < sg_end && sg < segs; sg++) {
            const uint32_t pq = pm[sg];
            if (pq != 0xFFu) pst[((bin0 + sg) * kPairMax + pq) * (kPairWords * 4u)] = v;
        }
    };
    const float d = sts.dx[c];
#ifdef S3R_STATS
    uint32_t it_row = 0, it_seg = 0;
    float v = exact_walk(sts.ws[c], sts.dy[c], y - ymin, &it_row);
#else
    float v = exact_walk(sts.ws[c], sts.dy[c], y - ymin);
#endif
    row[0] = v;
    // segments starting at or before the first start-table boundary past xmin walk from the row start
    // -- with row_starts, every segment of the bbox does: the fragment workgroups walk along the row
    // themselves, off this kernel's critical path (delivered frames: the fragment kernel is bound by
    // the host link, so its workgroups have the time; the serial boundary walks here were ~15 us of
    // the launch's ~24)
    const uint32_t sg_xmin = xmin / segw, b1 = (xmin / kStartPx + 1u) * kStartPx;
    if (row_starts) {
        to_pairs(sg_xmin, (xmax / segw) + 1u, v);
        S3R_GWT_END();
        return;
    }
    to_pairs(sg_xmin, min((xmax / segw) + 1u, b1 / segw), v);
#if defined(S3R_GEO_ABLATE)                  // timing-only variants: 1 = no segment starts
    if (S3R_GEO_ABLATE & 1) return;
#endif
    uint32_t xp = xmin;
    for (uint32_t sb = xmin / kStartPx + 1u; sb + 1u < nst; sb++) {
        const uint32_t xb = sb * kStartPx;
        if (xb > xmax) break;
#ifdef S3R_STATS
        v = exact_walk(v, d, xb - xp, &it_seg);
#else
        v = exact_walk(v, d, xb - xp);
#endif
        xp = xb;
        row[(1 + sb) * 4] = v;
        to_pairs(xb / segw, min((xmax / segw) + 1u, (xb + kStartPx) / segw), v);
    }
#ifdef S3R_STATS
    const unsigned long long t_end = wall_clock64();
    atomicMax(&g_tstats[1], t_end - t_start);
    atomicMax(&g_tstats[3], t_end);
    atomicAdd(&g_stats[12], (unsigned long long)it_row);
    atomicMax(&g_stats[13], (unsigned long long)it_row);
    atomicAdd(&g_stats[14], (unsigned long long)it_seg);
    atomicMax(&g_stats[15], (unsigned long long)it_seg);
#endif
    S3R_GWT_END();
}

#ifndef S3R_FASTDIV
#define S3R_FASTDIV 1                  // shading: trimmed exact division / sqrt sequences in range
#endif

// Deferred shading of the winning triangle (render.cpp:366-371) from its constants: cvr (c0-c2),
// nr (n0-n2), col (k0-k2), kind and texture base.
template <bool kFast = (S3R_FASTDIV != 0)>
S3R_CALLEE uint32_t shade_core(float4 c0, float4 c1, float4 c2, float4 n0, float4 n1, float4 n2, float4 k0, float4 k1,
                               float4 k2, uint32_t kind, uint32_t tex_base, float w0, float w1, float w2, float ooz,
                               const uint32_t *__restrict__ tex, uint32_t ntex) {
    // w / (1/z), three quotients by one divisor: the refined reciprocal is shared (s3r_common.h)
    float a, b, c;
    if (kFast && (div_in_range(w0, ooz) & div_in_range(w1, ooz) & div_in_range(w2, ooz))) {
        const float r = div_recip(ooz);
        a = div_with_recip(w0, ooz, r); b = div_with_recip(w1, ooz, r); c = div_with_recip(w2, ooz, r);
    } else {
        a = w0 / ooz; b = w1 / ooz; c = w2 / ooz;
    }
    const F3 P = mk3((c0.x * a + c1.x * b) + c2.x * c, (c0.y * a + c1.y * b) + c2.y * c,
                     (c0.z * a + c1.z * b) + c2.z * c);
    auto norm = [](F3 v) { return kFast ? fast_normalize3_dev(v) : fast_normalize3(v); };
    const F3 pn = norm(P);
    const F3 point = mk3(-pn.x, -pn.y, -pn.z);
    const F3 N = mk3((n0.x * a + n1.x * b) + n2.x * c, (n0.y * a + n1.y * b) + n2.y * c,
                     (n0.z * a + n1.z * b) + n2.z * c);
    const F3 normal = norm(N);
    const F3 halfway = norm(add3(point, normal));
    const float s = dot3(halfway, normal);
    F3 col;
    if (kind == kColour) {
        col = mk3((k0.x * a + k1.x * b) + k2.x * c, (k0.y * a + k1.y * b) + k2.y * c,
                  (k0.z * a + k1.z * b) + k2.z * c);
    } else {
        // uv0=(k0.x,k0.y) uv1=(k0.z,k0.w) uv2=(k1.x,k1.y) dz=(k1.z,k1.w) tpp=(k2.x,k2.y)
        const float mu = (k0.x * a + k0.z * b) + k1.x * c;
        const float mv = (k0.y * a + k0.w * b) + k1.y * c;
        const float dvx = fabsf(k2.x - mu * k1.z), dvy = fabsf(k2.y - mv * k1.w);
        float lvx, lvy;
        if (kFast && (div_in_range(ooz, dvx) & div_in_range(ooz, dvy))) {
            lvx = div_with_recip(ooz, dvx, div_recip(dvx));
            lvy = div_with_recip(ooz, dvy, div_recip(dvy));
        } else {
            lvx = ooz / dvx;
            lvy = ooz / dvy;
        }
        const uint32_t rgb = texel(tex, ntex, tex_base, mu, mv, lvx, lvy);
        col = mk3((float)(rgb >> 16), (float)((rgb >> 8) & 255u), (float)(rgb & 255u));
    }
    return rgb_pack(s * col.x, s * col.y, s * col.z);
}

#ifndef S3R_SHADE_FLAT
#define S3R_SHADE_FLAT 1
#endif
// shade_core as one straight-line block: every correctly rounded division and sqrt takes its trimmed
// sequence unconditionally while the range conditions are collected in `ok`; a lane with any operand
// out of range is shaded again by shade_core (same bits either way).  Without the per-operation
// branches the scheduler interleaves the independent chains.  The texel is loaded unconditionally as
// soon as its coordinates exist (an index clamped to 0 where the reference's lookup would be out of
// range or the triangle is coloured: the value is then discarded) and consumed only after the
// normalisations, so its latency runs under them.
S3R_CALLEE uint32_t shade_core_flat(float4 c0, float4 c1, float4 c2, float4 n0, float4 n1, float4 n2, float4 k0,
                                    float4 k1, float4 k2, uint32_t kind, uint32_t tex_base, float w0, float w1,
                                    float w2, float ooz, const uint32_t *__restrict__ tex, uint32_t ntex) {
    // operand ranges: w, 1/z and the texture derivatives in [2^-40, 2^20) -- biased exponents in
    // [87, 146], so every quotient below meets div_in_range (NaN fails the compares)
    auto inr = [](float x) { return (fabsf(x) >= 0x1p-40f) & (fabsf(x) < 0x1p20f); };
    bool ok = inr(w0) & inr(w1) & inr(w2) & inr(ooz);
    const float r = div_recip(ooz);
    const float a = div_with_recip(w0, ooz, r), b = div_with_recip(w1, ooz, r), c = div_with_recip(w2, ooz, r);
    // texture coordinates first: the texel load overlaps the normalisations
    const float mu = (k0.x * a + k0.z * b) + k1.x * c;
    const float mv = (k0.y * a + k0.w * b) + k1.y * c;
    const float dvx = fabsf(k2.x - mu * k1.z), dvy = fabsf(k2.y - mv * k1.w);
    const bool texd = kind != kColour;
    ok &= !texd | (inr(dvx) & inr(dvy));
    const float lvx = div_with_recip(ooz, dvx, div_recip(dvx));
    const float lvy = div_with_recip(ooz, dvy, div_recip(dvy));
    // out-of-range texture index: UB in the reference, 0 here and in the oracle (texel())
    const bool tex_ok = texd & (tex_base < ntex) & (ntex - tex_base >= kTexTexels);
#if defined(S3R_ABLATE) && (S3R_ABLATE & 256)
    uint32_t rgb = (tex_ok ? tex_base + texel_offset(mu, mv, lvx, lvy) : 0u) * 0x010101u;   // ablation: no load
#else
    uint32_t rgb = tex[tex_ok ? tex_base + texel_offset(mu, mv, lvx, lvy) : 0u];
#endif
    auto norm = [&ok](F3 v) {
        const float d = dot3(v, v);
        ok &= sqrt_in_range_ok(d);
        const float sq = sqrt_in_range(d);
        const float inv = div_with_recip(1.0f, sq, div_recip(sq));
        return mk3(v.x * inv, v.y * inv, v.z * inv);
    };
    const F3 P = mk3((c0.x * a + c1.x * b) + c2.x * c, (c0.y * a + c1.y * b) + c2.y * c,
                     (c0.z * a + c1.z * b) + c2.z * c);
    const F3 N = mk3((n0.x * a + n1.x * b) + n2.x * c, (n0.y * a + n1.y * b) + n2.y * c,
                     (n0.z * a + n1.z * b) + n2.z * c);
    const F3 pn = norm(P);
    const F3 normal = norm(N);
    const F3 point = mk3(-pn.x, -pn.y, -pn.z);
    const F3 halfway = norm(add3(point, normal));
    float s = dot3(halfway, normal);
    // the texel is consumed from here on: keeps the compiler from waiting for it before the
    // normalisations above
    asm volatile("" : "+v"(rgb), "+v"(s));
    rgb = tex_ok ? rgb : 0u;
    const F3 col = texd ? mk3((float)(rgb >> 16), (float)((rgb >> 8) & 255u), (float)(rgb & 255u))
                        : mk3((k0.x * a + k1.x * b) + k2.x * c, (k0.y * a + k1.y * b) + k2.y * c,
                              (k0.z * a + k1.z * b) + k2.z * c);
    uint32_t res = rgb_pack(s * col.x, s * col.y, s * col.z);
    if (!ok) {
        // opaque copies: keeps the compiler from speculating the fallback's divisions into the fast path
        asm volatile("" : "+v"(w0), "+v"(w1), "+v"(w2), "+v"(ooz));
        res = shade_core<false>(c0, c1, c2, n0, n1, n2, k0, k1, k2, kind, tex_base, w0, w1, w2, ooz, tex, ntex);
    }
    return res;
}

// The same from a TriSetup record (tile path: a register-resident record).
S3R_CALLEE uint32_t shade(const TriSetup *__restrict__ tp, float w0, float w1, float w2, float ooz,
                          const uint32_t *__restrict__ tex, uint32_t ntex) {
    const float4 *q = reinterpret_cast<const float4 *>(tp);
#if S3R_SHADE_FLAT
    return shade_core_flat(q[6], q[7], q[8], q[9], q[10], q[11], q[12], q[13], q[14], tp->kind, tp->tex_base, w0, w1,
                           w2, ooz, tex, ntex);
#else
    return shade_core(q[6], q[7], q[8], q[9], q[10], q[11], q[12], q[13], q[14], tp->kind, tp->tex_base, w0, w1, w2,
                      ooz, tex, ntex);
#endif
}

// Per-lane values of one batch: lane 3t+c holds component c of the batch's t-th triangle; c is the
// exact value at pixel k0 of the component's walk (render.cpp:374), m the triangle's pixels in the chunk.
struct BatchLanes {
    bool ov = false;
    float c = 0.0f, d = 0.0f, rz = 0.0f;
    uint32_t k0 = 0, m = 0, xmax = 0, slot = 0;
};

// Work units (~8 VALU instructions each) a wave counts for the longest-first order of the next
// frames (order_bins): a table group's fill, one live triangle's pixel test, one shading round of a
// textured / coloured winner (a non-waterfall chunk with any winner: kWorkShade), a chunk.  Round 5:
// the wall time of a bin, used before, depends on its co-resident workgroups -- a bin that ran in
// the launch's sparse tail measures short and stays in the tail -- so the order did not converge
// to the heaviest bins first (4K P_over, per-workgroup timeline: span 54.8 us with the wall-time
// order, 55.6 in launch order; list scheduling of the measured durations costliest first: 44.0).
constexpr uint32_t kWorkFill = 12, kWorkTest = 4, kWorkTexture = 32, kWorkColour = 20, kWorkShade = 24,
                   kWorkChunk = 2, kWorkSky = S3R_WORK_SKY;

// One chunk of one batch.  Every (triangle, component) that overlaps the chunk gets the chunk's 64
// exact values by the reference's own sequential adds (render.cpp:374, w += dx) in an LDS table --
// every lane of the wave the same instruction stream: no per-lane linear-run classification, no
// exact_walk inside a row (round 5; the linear-run design it replaces classified each chunk per lane,
// jumped inside binades and filled tables only for irregular chunks: 56.8 -> 52.0 us per 4K launch,
// 31.0 -> 26.6 M VALU and 16.3 -> 12.3 M SALU wave-instructions, profiles/r05_fragment_ab.txt).  Then
// lanes act as pixels: edge test, 1/z and the strict '>' depth test in registers, reading the tables.
// v.c is the exact value at pixel v.k0; `last` returns the value at v.k0 + v.m - 1, the walk state
// of the next chunk.  Tables hold kTables components = kTables / 3 triangles: a chunk met by more runs
// in groups, in list (slot) order -- the reference's order, which decides depth ties.
static_assert(kPX == 1u && kTables % 3u == 0u, "one pixel per lane, whole triangles per table group");
__device__ __forceinline__ void alltab_chunk(const BatchLanes &v, uint32_t lane, float (*tab)[kTabStride], uint32_t xl,
                                             float (&depth)[kPX], int (&win)[kPX], float (&bw0)[kPX],
                                             float (&bw1)[kPX], float (&bw2)[kPX], float &last, uint32_t &wk) {
    last = v.c;
    const uint64_t ovl = __ballot(v.ov);
    if (ovl == 0) return;
    const uint32_t r = lane_prefix(ovl, lane), nov = (uint32_t)__builtin_popcountll(ovl);
    for (uint32_t g0 = 0; g0 < nov; g0 += kTables) {                    // wave-uniform
        wk += kWorkFill;
        const bool mine = v.ov && r >= g0 && r < g0 + kTables;
        const uint32_t ti = r - g0;
        bool neg = false;
        if (mine) {
            float w = v.c;
            float4 *tb4 = reinterpret_cast<float4 *>(tab[ti]);
#pragma unroll 4                                   // (fully unrolled, the kernel spills 68 VGPRs)
            for (uint32_t k4 = 0; k4 < kChunk / 4u; k4++) {
                const float a1 = w + v.d, a2 = a1 + v.d, a3 = a2 + v.d;
                tb4[k4] = make_float4(w, a1, a2, a3);
                w = a3 + v.d;
                __builtin_amdgcn_sched_barrier(0);   // store as it goes: the chain's values must not pile up in VGPRs
            }
        }
        wave_sync();
        if (mine) {
            last = tab[ti][v.m - 1u];
            neg = v.c < 0.0f && last < 0.0f;                               // monotone walk: all < 0
        }
        const uint64_t negm = __ballot(neg);
        const uint64_t gm = __ballot(mine);
        uint64_t live = gm & ~(negm | (negm >> 1) | (negm >> 2)) & 0x9249249249249249ull;
        wk += kWorkTest * (uint32_t)__builtin_popcountll(live);
        while (live) {
            const uint32_t l0 = (uint32_t)__builtin_ctzll(live);
            live &= live - 1;
            const uint32_t tk0 = rdl(v.k0, l0), txmax = rdl(v.xmax, l0), t0 = rdl(ti, l0);
            const float r0 = rdl(v.rz, l0), r1 = rdl(v.rz, l0 + 1u), r2 = rdl(v.rz, l0 + 2u);
            const int tslot = (int)rdl(v.slot, l0);
            // branch-free: every lane reads its table entry (a lane left of the triangle's first pixel
            // reads entry 63, one right of its last a value past it -- both discarded by `hit`), so
            // the wave runs no exec-mask save / restore per triangle (round 6: against the branching
            // test 47.8 -> 47.6 us, SALU 12.9 -> 12.6 M; profiles/r06_pix_select_ab.txt)
            const uint32_t off = min(xl - tk0, kChunk - 1u);
            const float a0 = tab[t0][off], a1 = tab[t0 + 1u][off], a2 = tab[t0 + 2u][off];
            const float ooz = (r0 * a0 + r1 * a1) + r2 * a2;                     // :363
            const bool hit = (xl >= tk0) & (xl <= txmax) & (a0 >= 0) & (a1 >= 0) & (a2 >= 0)   // :362
                             & (ooz > depth[0]);                                 // :364 (& not &&: no branches)
            depth[0] = hit ? ooz : depth[0];
            win[0] = hit ? tslot : win[0];
            bw0[0] = hit ? a0 : bw0[0];
            bw1[0] = hit ? a1 : bw1[0];
            bw2[0] = hit ? a2 : bw2[0];
        }
        wave_sync();                                                        // before the next group's fill
    }
}

// A workgroup = 4 waves = 4 consecutive local rows x one segment of SEGCH 64-pixel chunks.  The
// triangles meeting that block are listed once in LDS (slot order).  For each chunk, each wave takes
// them kTPB at a time: its lanes first act as (triangle, barycentric component) pairs and advance
// that component's exact walk (render.cpp:374) to the chunk, publishing (value, step) in LDS; then
// its lanes act as pixels: edge test, 1/z, strict '>' depth test in registers; the winner is shaded.
#ifndef S3R_WATERFALL_BINS
#define S3R_WATERFALL_BINS 4000        // launches of >= this many 384-px bins shade by the waterfall
#endif
#ifndef S3R_OCC_WIDE
#define S3R_OCC_WIDE 6                 // waterfall-shading instances: <= 80 VGPRs (79 used, no spills);
#endif                                 // 7 (72 VGPRs, 8 tables for the LDS) spills and is 5 % slower
// WF: shading by the waterfall over the wave's distinct winners, each winner's constants by scalar
// loads (79 VGPRs: occupancy 6).  It pays where the launch is throughput-bound (4K, 8K frames: +1.5 %,
// +3.7 %); launches of one or two rounds of workgroups are bound by their heaviest bins' latency,
// which the extra waterfall rounds lengthen (a 4K frame half: -4 %, 1080p: -4 %).
// HOSTW: `out` is the whole frame in the caller's mapped host buffer (direct / host-fill delivery,
// render_api.cpp): rows at their frame rows, stores crossing the PCIe link -- its own instance, so
// profiles tell the delivered launches from the HBM ones.
template <uint32_t SEGCH, bool WF, bool HOSTW>
__global__ void __launch_bounds__(64 * kWaves, WF ? S3R_OCC_WIDE : S3R_OCC) k_fragment(const TriSetup *__restrict__ tris, uint32_t nslots,
                                                  const float *__restrict__ rowtab, const uint32_t *__restrict__ tex,
                                                  uint32_t ntex, uint32_t *__restrict__ out, uint32_t W, uint32_t H,
                                                  uint32_t band, uint32_t nparts, uint32_t part, uint32_t segs,
                                                  uint32_t rows_local,
                                                  uint32_t *__restrict__ bincnt,
                                                  const uint4 *__restrict__ pairs, uint32_t *done_flag,
                                                  uint32_t prev_tag, uint32_t *__restrict__ order,
                                                  uint32_t host_fill, unsigned long long *chunk_flags,
                                                  uint32_t fill_tag, uint32_t row_starts) {
    __shared__ FragShared sh;
    S3R_WGT(0);
    // Completion for the host (buffer-set reuse without events, render_api.cpp wait_set_free): this
    // launch runs only once the previous fragment launch on its stream has completed, so its first
    // workgroup publishes that launch's tag in host-coherent memory.
    if (done_flag && blockIdx.x == 0 && threadIdx.x == 0)
        __hip_atomic_store(done_flag, prev_tag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
    // longest-first workgroup order (order = [perm | cost] of this buffer set, order_bins in
    // k_geometry) or the launch order; either way a permutation of the bins, so the pixels do not
    // depend on it
    const uint32_t bid = order ? order[blockIdx.x] : blockIdx.x;
    const uint32_t blk = bid / segs, seg = bid - blk * segs;
    const uint32_t nst = start_entries_of(W);
    auto row_of = [&](uint32_t lr) { return ((lr / band) * nparts + part) * band + lr % band; };
    const uint32_t lr0 = blk * kWaves;
    const uint32_t lr = lr0 + wave;
    const uint32_t y = row_of(lr);
    const bool row_ok = lr < rows_local && y < H;
    uint32_t y0 = 0xFFFFFFFFu, y1 = 0;
    for (uint32_t k = 0; k < kWaves && lr0 + k < rows_local; k++) {
        const uint32_t yy = row_of(lr0 + k);
        y0 = min(y0, yy); y1 = max(y1, yy);
    }
    const uint32_t xs = seg * kChunk * SEGCH;
    const uint32_t xe = min(W, xs + kChunk * SEGCH) - 1u;
    const uint32_t tl = lane / 3u, comp = lane - 3u * tl;                  // (triangle, component) role
    float *st_c = sh.st_c[wave];
    uint32_t *st_k = sh.st_k[wave];
#ifdef S3R_STATS
    uint32_t st_row = 0, st_chunk = 0, st_pix = 0, st_irr = 0, st_tests = 0, st_batches = 0;
    uint32_t *p_chunk = &st_chunk, *p_pix = &st_pix;
#endif

    // this workgroup's triangle list: its bin's pairs (k_geometry), put in slot order -- or, beyond
    // kPairMax triangles, the first round of an in-kernel slot scan.  Wave 0 fetches the first
    // 64 / kPairWords pairs speculatively with the header (one round trip for most bins); the staging
    // area is the exact-table space, unused until the chunk loop.
    bool overflow = false;
    uint4 *stage = reinterpret_cast<uint4 *>(&sh.tab4[0][0][0]);
    const uint4 *pp = pairs + (size_t)bid * kPairMax * kPairWords;
    if (wave == 0) {
        stage[lane] = pp[lane];
    } else if (wave == 1 && lane == 0) {
        // this frame's pair count; reset for the buffer set's next geometry (this launch is the set's
        // last reader: the host issues that geometry only once this launch has completed)
        sh.cnt = bincnt[bid];
        bincnt[bid] = 0u;
    }
    __syncthreads();
    const uint32_t npairs = sh.cnt;
    // output row: local row lr of a compact part buffer, or (HOSTW) frame row y of a whole frame
    const size_t orow = (size_t)(HOSTW ? y : lr) * W;
    if (npairs == 0) {
        // no triangle meets this block (sky): background only (render.cpp:282), 16 B per lane where
        // the row segment is 16-B aligned -- unless the host fills this sky bin (host_fill = 1 +
        // gpu_eighths: the frame is the caller's host buffer; k_sky_flags gave the sky bins with
        // bid % 8 >= gpu_eighths to the host and kept the others for the GPU)
        if (row_ok && (!host_fill || (bid & 7u) < host_fill - 1u)) {
            uint32_t *seg = out + orow + xs;
            const uint32_t n = xe - xs + 1u;
            if ((orow + xs) % 4u == 0u) {
                const uint4 bg4 = make_uint4(kBackground, kBackground, kBackground, kBackground);
                for (uint32_t i = lane; i < n / 4u; i += 64u) reinterpret_cast<uint4 *>(seg)[i] = bg4;
                for (uint32_t i = (n & ~3u) + lane; i < n; i += 64u) seg[i] = kBackground;
            } else {
                for (uint32_t i = lane; i < n; i += 64u) seg[i] = kBackground;
            }
        }
        S3R_WGT(3);
        if (order && threadIdx.x == 0)
            order[gridDim.x + bid] = kWorkSky;
        return;
    }
    if (npairs > kPairMax) {
        // > kPairMax triangles meet this workgroup: stateless rounds of in-kernel slot scans
        build_list(tris, nslots, y0, y1, xs, xe, 0, sh, wave, lane);
        overflow = true;
    } else {
        for (uint32_t i = 64u + threadIdx.x; i < npairs * kPairWords; i += 64u * kWaves) stage[i] = pp[i];
        if (npairs * kPairWords > 64u) __syncthreads();
        // pair i goes to list position rank(i) = the number of listed slots below its slot (the
        // reference's processing order); its walk state to the batch lanes of that position
        if (threadIdx.x < npairs) {
            const uint4 *me = stage + threadIdx.x * kPairWords;
            const uint4 h0 = me[0], h1 = me[1], dxw = me[2], rzw = me[3];
            uint32_t rank = 0;
            for (uint32_t j = 0; j < npairs; j++) rank += stage[j * kPairWords].x < h0.x ? 1u : 0u;
            Entry &e = sh.ent[rank];
            e.slot = h0.x; e.xmin = h0.y; e.xmax = h0.z; e.ymin = h0.w; e.ymax = h1.x;
            e.dx[0] = u2f(dxw.x); e.dx[1] = u2f(dxw.y); e.dx[2] = u2f(dxw.z);
            e.rvz[0] = u2f(rzw.x); e.rvz[1] = u2f(rzw.y); e.rvz[2] = u2f(rzw.z);
            const uint32_t b = rank / kTPB, lb = 3u * (rank - b * kTPB);
            if (b < kStateBatches) {
                uint32_t k;
                (void)start_index(h0.y, xs, &k, row_starts != 0u);
                const uint4 s0 = me[4], s1 = me[5], s2 = me[6];
                const float stv[kWaves * 3] = {u2f(s0.x), u2f(s0.y), u2f(s0.z), u2f(s0.w), u2f(s1.x), u2f(s1.y),
                                               u2f(s1.z), u2f(s1.w), u2f(s2.x), u2f(s2.y), u2f(s2.z), u2f(s2.w)};
#pragma unroll
                for (uint32_t w = 0; w < kWaves; w++)
#pragma unroll
                    for (uint32_t c = 0; c < 3; c++) {
                        sh.st_c[w][b * 64 + lb + c] = stv[w * 3 + c];
                        sh.st_k[w][b * 64 + lb + c] = k;
                    }
            }
        }
        __syncthreads();
    }
    const uint32_t n0 = sh.cnt;
    S3R_WGT(1);
    S3R_WGT(2);

    // ---- batch 0 (the first kTPB listed triangles: nearly every row has no more) keeps its
    // constants and walk state in registers
    const bool reg0 = !overflow && row_ok && n0 > 0;
    bool r0_in = false;
    float r0_d = 0.0f, r0_rz = 0.0f, r0_sc = 0.0f;
    uint32_t r0_xmin = 1u, r0_xmax = 0u, r0_slot = 0u, r0_sk = 0u;
    if (reg0 && lane < 63 && tl < n0) {
        const Entry &e = sh.ent[tl];
        r0_in = y >= e.ymin && y <= e.ymax;
        r0_d = e.dx[comp];
        r0_rz = e.rvz[comp];
        r0_xmin = e.xmin;
        r0_xmax = e.xmax;
        r0_slot = e.slot;
        r0_sc = st_c[lane];
        r0_sk = st_k[lane];
    }

    uint32_t *row = out + orow;
    uint32_t bgm = 0;                    // host fill: this row's chunks no triangle covers (bit q)
    // HOSTW: the wave's stores on the 64-B line grid of the caller's buffer.  A buffer from glibc's
    // malloc starts 16 B into a line, so a 64-pixel chunk store would touch five lines, two of them
    // partly; instead the wave stores the 64 pixels [cx0 - rsh, cx0 - rsh + 64), rsh = the pixel
    // offset of the row segment's start inside its line: lanes >= rsh this chunk's first 64 - rsh
    // pixels (a lane rotation), lanes < rsh the previous chunk's last rsh (carried), and after the
    // last chunk the carried pixels alone.  Every pixel is stored once, by its own workgroup; a
    // lane with nothing to store (outside the frame, a chunk left to the host fill) holds kNoPixel.
    // Over an uncached registration (render_api.cpp host_pinned) the link then carries whole lines:
    // 54.0 instead of 49.1 GB/s for this pattern (tools/micro/pcie_write.hip).
    const uint32_t rsh = (HOSTW && S3R_LINE_STORES) ? (uint32_t)(((uintptr_t)(row + xs) >> 2) & 15u) : 0u;
    uint32_t carry = kNoPixel, cx_next = xs;
    auto put = [&](uint32_t c0x, uint32_t v) {      // the lane's pixel c0x + lane, or kNoPixel
        if (rsh == 0u) {
            if (v != kNoPixel) row[c0x + lane] = v;
            return;
        }
        const uint32_t rot = (uint32_t)__shfl((int)v, (int)((lane - rsh) & 63u));
        const uint32_t o = lane >= rsh ? rot : carry;
        if (o != kNoPixel) row[c0x - rsh + lane] = o;
        carry = rot;
    };
    S3R_WGC_DECL;
    uint32_t wk = 0;                     // this wave's work units (kWorkFill ...), wave-uniform
    for (uint32_t q = 0; q < SEGCH; q++) {
        const uint32_t cx0 = xs + kChunk * q;
        if (cx0 > xe) break;
        cx_next = cx0 + kChunk;
        wk += kWorkChunk;
        const uint32_t cx1 = min(cx0 + kChunk - 1u, xe);
        const uint32_t x = cx0 + lane;                     // this lane's pixels: x + 64 p, p < kPX
        float depth[kPX], bw0[kPX], bw1[kPX], bw2[kPX];
        int win[kPX];
#pragma unroll
        for (uint32_t p = 0; p < kPX; p++) { depth[p] = 0.0f; bw0[p] = bw1[p] = bw2[p] = 0.0f; win[p] = -1; }

        S3R_WGC_MARK();
        if (reg0) {
            BatchLanes v;
            if (r0_in && r0_xmin <= cx1 && r0_xmax >= cx0) {
                v.ov = true;
                v.d = r0_d; v.rz = r0_rz; v.xmax = r0_xmax; v.slot = r0_slot;
                v.k0 = max(cx0, r0_xmin);
                v.m = min(cx1, r0_xmax) - v.k0 + 1u;
                // the state is the exact value at pixel r0_sk <= k0: the chunk before's last pixel (one
                // add), or for a triangle's first chunk the bin's start point (a jump)
                v.c = v.k0 == r0_sk ? r0_sc
                                    : (v.k0 == r0_sk + 1u ? r0_sc + v.d : walk(r0_sc, v.d, v.k0 - r0_sk S3R_IT(p_chunk)));
            }
            float last;
            alltab_chunk(v, lane, reinterpret_cast<float (*)[kTabStride]>(sh.tab4[wave]), x, depth, win, bw0, bw1, bw2, last, wk);
            if (v.ov) { r0_sc = last; r0_sk = v.k0 + v.m - 1u; }
#ifdef S3R_STATS
            st_batches += __ballot(v.ov) != 0ull ? 1u : 0u;
#endif
        }

        S3R_WGC_ADD(0);
        S3R_WGC_MARK();
        uint32_t cursor = 0, cnt = n0;
        for (;;) {
            if (overflow) {
                build_list(tris, nslots, y0, y1, cx0, cx1, cursor, sh, wave, lane);
                cnt = sh.cnt;
                cursor = sh.next;
            }
            for (uint32_t b = reg0 ? 1u : 0u; row_ok && b * kTPB < cnt; b++) {
                const bool stateful = !overflow && b < kStateBatches;
                // ---- lanes as (triangle, component): advance the exact walk to this chunk
                const uint32_t idx = b * kTPB + tl;
                BatchLanes v;
                if (lane < 63 && idx < cnt) {
                    const Entry &e = sh.ent[idx];
                    v.ov = y >= e.ymin && y <= e.ymax && e.xmin <= cx1 && e.xmax >= cx0;
                    if (v.ov) {
                        v.d = e.dx[comp];
                        v.rz = e.rvz[comp];
                        v.xmax = e.xmax;
                        v.slot = e.slot;
                        v.k0 = max(cx0, e.xmin);
                        v.m = min(cx1, e.xmax) - v.k0 + 1u;
                        if (stateful) {
                            const uint32_t kp = st_k[b * 64 + lane];
                            const float cp = st_c[b * 64 + lane];
                            v.c = v.k0 == kp ? cp : (v.k0 == kp + 1u ? cp + v.d : walk(cp, v.d, v.k0 - kp S3R_IT(p_chunk)));
                        } else {
                            uint32_t k;
                            const uint32_t j = start_index(e.xmin, xs, &k, row_starts != 0u);
                            const float c0v = rowtab[(((size_t)e.slot * rows_local + lr) * nst + j) * 4 + comp];
                            v.c = walk(c0v, v.d, v.k0 - k S3R_IT(p_chunk));
                        }
                    }
                }
                float last;
                alltab_chunk(v, lane, reinterpret_cast<float (*)[kTabStride]>(sh.tab4[wave]), x, depth, win, bw0, bw1, bw2, last, wk);
                if (v.ov && stateful) { st_c[b * 64 + lane] = last; st_k[b * 64 + lane] = v.k0 + v.m - 1u; }
#ifdef S3R_STATS
                st_batches += __ballot(v.ov) != 0ull ? 1u : 0u;
#endif
            }
            if (!overflow || cursor >= nslots) break;
        }
        S3R_WGC_ADD(1);
        S3R_WGC_MARK();
        if (HOSTW && host_fill) {
            // a chunk of this row without a winner is all background: the host writes it (bit q of
            // this bin's chunk flag), so the link does not carry it
            bool any = false;
#pragma unroll
            for (uint32_t p = 0; p < kPX; p++) any |= row_ok && x + 64u * p <= xe && win[p] >= 0;
            if (__ballot(any) == 0) {
                if (row_ok) bgm |= 1u << q;
#pragma unroll
                for (uint32_t p = 0; p < kPX; p++) put(cx0 + 64u * p, kNoPixel);
                continue;
            }
        }
#pragma unroll
        for (uint32_t p = 0; p < kPX; p++) {
            const uint32_t xp = x + 64u * p;
#if defined(S3R_ABLATE) && (S3R_ABLATE & 128)
            if (row_ok && xp <= xe && win[p] == 12345) row[xp] = 0;    // ablation: no stores
#elif defined(S3R_ABLATE) && (S3R_ABLATE & 1)
            if (row_ok && xp <= xe)
                row[xp] = win[p] < 0 ? kBackground : (uint32_t)win[p] ^ __float_as_uint(bw0[p] + bw1[p] + bw2[p] + depth[p]);
#else
#if defined(S3R_ABLATE) && (S3R_ABLATE & 512)
            if (row_ok && xp <= xe)
#endif
#if defined(S3R_ABLATE) && (S3R_ABLATE & 512)     // ablation: every shade reads one record
                row[xp] = win[p] < 0 ? kBackground : shade(tris + 40, bw0[p], bw1[p], bw2[p], depth[p], tex, ntex);
#else
            if (!WF) {
                const bool act = row_ok && xp <= xe;
                if (order && __ballot(act && win[p] >= 0)) wk += kWorkShade;
                uint32_t px = kNoPixel;
                if (act) px = win[p] < 0 ? kBackground : shade(tris + win[p], bw0[p], bw1[p], bw2[p], depth[p], tex, ntex);
                if (HOSTW) {
                    put(cx0 + 64u * p, px);
                } else if (act) {
                    row[xp] = px;
                }
            } else {
                // waterfall over the wave's distinct winners (usually one: a chunk inside one
                // triangle): each round shades the lanes of one winner, whose record address is
                // wave-uniform, so its constants arrive by scalar loads into SGPRs -- no per-lane
                // gather, and ~36 VGPRs fewer live at the shading's peak
                const int wp = win[p];
                const bool act = row_ok && xp <= xe;
                uint32_t px = kBackground;
                uint64_t todo = __ballot(act && wp >= 0);
                while (todo) {
                    const int wu = __builtin_amdgcn_readlane(wp, (int)__builtin_ctzll(todo));
                    // loaded in wave-uniform control flow: scalar loads
                    const TriSetup *tp = tris + wu;
                    const float4 *q = reinterpret_cast<const float4 *>(tp);
                    const float4 c0 = q[6], c1 = q[7], c2 = q[8], n0 = q[9], n1 = q[10], n2 = q[11];
                    const float4 k0 = q[12], k1 = q[13], k2 = q[14];
                    const uint32_t kind = tp->kind, tex_base = tp->tex_base;
                    wk += kind == kTexture ? kWorkTexture : kWorkColour;
                    const bool mine = act && wp == wu;
                    todo &= ~__ballot(mine);
                    if (mine)
                        px = shade_core_flat(c0, c1, c2, n0, n1, n2, k0, k1, k2, kind, tex_base, bw0[p], bw1[p], bw2[p],
                                             depth[p], tex, ntex);
                }
                if (HOSTW) {
                    put(cx0 + 64u * p, act ? px : kNoPixel);
                } else if (act) {
                    row[xp] = px;
                }
            }
#endif
#endif
        }
        S3R_WGC_ADD(2);
    }
    if (HOSTW && rsh != 0u && lane < rsh && carry != kNoPixel) row[cx_next - rsh + lane] = carry;
    if (HOSTW && host_fill) {
        // this bin's background chunks for the host: (tag << 32) | bit (wave * SEGCH + q)
        if (lane == 0) sh.bgm[wave] = bgm;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t m = 0;
#pragma unroll
            for (uint32_t w = 0; w < kWaves; w++) m |= sh.bgm[w] << (w * SEGCH);
            __hip_atomic_store(chunk_flags + bid, ((unsigned long long)fill_tag << 32) | m, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    S3R_WGT(3);
    // this bin's cost for the buffer set's next order_bins: its waves' work units (the bins' measured
    // wall times, rounds 3-4, were retired in round 6: see kWorkFill)
    if (order) {
        if (lane == 0) sh.wwork[wave] = wk;
        __syncthreads();
        if (threadIdx.x == 0) {
            uint32_t c = 0;
#pragma unroll
            for (uint32_t w = 0; w < kWaves; w++) c += sh.wwork[w];
            order[gridDim.x + bid] = c;
        }
    }
    S3R_WGC_STORE(n0);
#ifdef S3R_STATS
    {
        const uint32_t vals[6] = {st_row, st_chunk, st_pix, st_irr, st_tests, st_batches};
        for (int k = 0; k < 6; k++) {
            uint32_t v = vals[k], m = wave_max(v);
            for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
            if (lane == 0) { atomicAdd(&g_stats[2 * k], (unsigned long long)v); atomicAdd(&g_stats[2 * k + 1], (unsigned long long)m); }
        }
    }
#endif

}

// ------------------------------------------------------------------ tile path (many triangles)
// For scenes whose slot count makes the per-(slot, row) start table too large (the icosahedron
// stress scene, BASELINE config 5: 20 M triangles), the fragment stage is order-independent:
//   k_tile_setup   one thread per triangle, POSITIONS ONLY (vertex transform, reject, near clip,
//                  cull, raster setup; render.cpp:285-336): a 64-B RasterRec per live slot, a packed
//                  bbox word per triangle, and the per-tile counts (wave-aggregated atomics);
//   (scan)         rocprim exclusive scan of the (tile, depth bucket) counts; k_tile_fill scatters slot
//                  ids into the tile lists, each tile's depth buckets nearest first;
//   k_tile_raster  one workgroup per tile of 16 local rows x 64 px: lanes take (triangle, row)
//                  items and walk the row with the reference's own sequential adds (render.cpp:374,
//                  :378; row start by exact_walk), keeping per pixel the max of
//                  key = (bits(1/z) << 32) | ~slot in LDS (ds_max_u64).  Strict '>' on 1/z from 0.0
//                  (:364) keeps the first of the deepest fragments in slot order, i.e. the largest
//                  1/z with ties to the smallest slot = the max key (1/z > 0 orders as its bits).
//                  Each pixel's winner is then re-walked exactly and shaded; its shading constants
//                  (normals, colours / uvs: the attribute stream) are recomputed from the scene by the
//                  same setup code, so attributes are read only for visible triangles.
#ifndef S3R_TSTAGE
#define S3R_TSTAGE 128
#endif
#ifndef S3R_TSTAGE_LINK
#define S3R_TSTAGE_LINK 256
#endif
constexpr uint32_t kTileW = 64, kTileH = 16, kTileThreads = 256, kTileStage = S3R_TSTAGE;
constexpr uint32_t kTileStageLink = S3R_TSTAGE_LINK;     // the fused raster of delivered frames
static_assert(kTileStage <= kTileThreads, "one staged triangle per thread at most");
constexpr uint32_t kKeyStride = kTileW + 1;        // padded LDS row: rows of one column hit different banks
constexpr uint32_t kDeadBox = 0xFFFFFFFFu;

// Depth buckets of a tile's list (nearest first).  A listed triangle's bucket is the eighth-octave of
// its 1/z bound (ooz_bound) below 1/near = 10, the largest 1/z any pixel can have: bucket
// b = (bits(10) >> 20) - (bits(bound) >> 20), clamped to [0, kDepthBuckets): 16 octaves, z up to
// ~6 500.  Every bound in bucket b >= 1 is below bucket_ceiling(b); k_tile_raster walks a tile's
// buckets in order and stops as soon as every pixel of the tile holds a winner at least that near.
// 128 buckets (round 6; 32 before: half-octaves): the early-out stops sooner and a record-free entry's
// row-cull bound (its bucket's ceiling) is tighter -- stress scene, one MI355X, kernels serialised
// (profiles/r06_depth_buckets_ab.txt): k_tile_raster<128u> 492 -> 475 (64) -> 457 us, device-resident
// frames 1 160 -> 1 185 -> 1 204 fps, part 0 of 8's fragment stage 128 -> 120 us.  The bins hold
// 256 entries per (tile, bucket) at first either way (4.2 GB for the four buffer sets at 4K).
#ifndef S3R_DEPTH_BUCKETS
#define S3R_DEPTH_BUCKETS 128
#endif
constexpr uint32_t kDepthBuckets = S3R_DEPTH_BUCKETS;
static_assert(kDepthBuckets == 32 || kDepthBuckets == 64 || kDepthBuckets == 128, "16 octaves in 2, 4 or 8 buckets each");
constexpr uint32_t kBucketShift = kDepthBuckets == 32 ? 22u : kDepthBuckets == 64 ? 21u : 20u;   // bits below the bucket
constexpr uint32_t kBucketTop = 0x41200000u >> kBucketShift;       // bits(10.0f) >> shift
__device__ __forceinline__ uint32_t depth_bucket(uint32_t zb_bits) {
    const int b = (int)kBucketTop - (int)(zb_bits >> kBucketShift);
    return (uint32_t)min(max(b, 0), (int)kDepthBuckets - 1);
}
// bits of an upper bound (exclusive) of every bound in bucket b (b = 0: none)
__device__ __forceinline__ uint32_t bucket_ceiling(uint32_t b) {
    return b == 0 ? 0xFFFFFFFFu : (kBucketTop - b + 1u) << kBucketShift;
}

// 48 B per live slot: the box, the depth bound, 1/z per corner and the three raster corners (x, y);
// the raster and the resolve recompute wstart and the steps from the corners (raster_steps).
struct alignas(16) RasterRec {
    uint32_t bx, by, zb;                           // bx = xmin | xmax << 16, by = ymin | ymax << 16,
    float rz0;                                     // zb = bits of ooz_bound() (hierarchical depth cull)
    float rz1, rz2, x0, y0;
    float x1, y1, x2, y2;
};
static_assert(sizeof(RasterRec) == 48, "RasterRec layout");

// A bin / list entry is a slot, | kNoRecBit when the slot has no raster record.  k_tile_setup writes
// no record for a slot the raster can set up again from the scene -- an original triangle wholly past
// the near plane -- and marks its entry; the raster (k_tile_raster, resolve_pixel<DEFER, true>)
// rebuilds its box, bound, 1/z and steps from its corners (the same operations on the same operands:
// the same floats).  The clip's slots (k_tile_clip) keep their records.
constexpr uint32_t kNoRecBit = 0x80000000u;

// The corner's camera-space and raster position (render.cpp:286, :288).  The two projections share
// one refined reciprocal of -cv.z where the trimmed division is exact (div_in_range, s3r_common.h);
// z = (0 * factor) / nz + nz is nz itself unless nz == 0 (0 / 0: the reference's NaN).
__device__ __forceinline__ void project_corner(float4 v, const Mat34 &m, float factor, float half_w, float half_h,
                                               Vert &d) {
    const F3 c = mat_mul(m, v);                                           // :286
    const float nz = -c.z;
    d.cv = c;
    const float px = c.x * factor, py = (-c.y) * factor;
    float qx, qy;
#ifndef S3R_TRIM_PROJ
#define S3R_TRIM_PROJ 1
#endif
    if (S3R_TRIM_PROJ && (div_in_range(px, nz) & div_in_range(py, nz))) {
        const float r = div_recip(nz);
        qx = div_with_recip(px, nz, r);
        qy = div_with_recip(py, nz, r);
    } else {
        qx = px / nz;
        qy = py / nz;
    }
    float rz = nz;                                                          // (+-0) + nz == nz
    if (nz == 0.0f) rz = (0.0f * factor) / nz + nz;
    d.rv = mk3(qx + half_w, qy + half_h, rz);                               // :288
}
__device__ __forceinline__ void load_corner(const float4 *__restrict__ vtx, uint32_t vi, const Mat34 &m, float factor,
                                            float half_w, float half_h, Vert &d) {
    project_corner(vtx[vi], m, factor, half_w, half_h, d);
}

// Exact a / b for small operands by one float multiply (the integer division by a run-time divisor
// is ~20 instructions): inv = rcp(b) (1 + 2^-21) lies in [(1/b)(1 + 2^-22), (1/b)(1 + 2^-20)]
// (v_rcp_f32 is within 1 ulp), so fl(a inv) is >= a / b and, when a / b = k + r / b with r >= 1,
// below k + 1 as long as b (k + 1) < 2^19 -- true for a + b < 2^19 (rows, bands, tiles of frames
// up to 65 535 px a side).  Truncation then gives k.
__device__ __forceinline__ float udiv_inv(uint32_t b) { return __builtin_amdgcn_rcpf((float)b) * (1.0f + 0x1p-21f); }
__device__ __forceinline__ uint32_t udiv_small(uint32_t a, float inv) { return (uint32_t)((float)a * inv); }

// Local rows [lo, hi] of this rank that fall in frame rows [ymin, ymax] (interleaved bands: local
// row order is frame row order, so the owned rows of any frame-row interval are one local range).
__device__ __forceinline__ bool local_row_range(uint32_t ymin, uint32_t ymax, uint32_t band, uint32_t nparts,
                                                uint32_t part, uint32_t &lo, uint32_t &hi) {
    if (nparts == 1u) { lo = ymin; hi = ymax; return ymin <= ymax; }
    const float ib = udiv_inv(band), ip = udiv_inv(nparts);
    const uint32_t g0 = udiv_small(ymin, ib), g1 = udiv_small(ymax, ib);
    const uint32_t m0 = g0 - udiv_small(g0, ip) * nparts, m1 = g1 - udiv_small(g1, ip) * nparts;
    uint32_t fg = g0, fy = ymin;
    if (m0 != part) { fg = g0 + (part > m0 ? part - m0 : part + nparts - m0); fy = fg * band; }
    uint32_t lg = g1, ly = ymax;
    if (m1 != part) {
        const uint32_t d = m1 > part ? m1 - part : m1 + nparts - part;
        if (g1 < d) return false;
        lg = g1 - d; ly = lg * band + band - 1u;
    }
    if (fg > lg || fy > ly) return false;
    lo = udiv_small(fg, ip) * band + (fy - fg * band);
    hi = udiv_small(lg, ip) * band + (ly - lg * band);
    return true;
}

struct TileSpan { uint32_t tx0, ntx, ty0, n, bucket; };   // tiles tx0 .. tx0+ntx-1 x ty0 .., n in all

// The tiles of a box given in tile columns: bt = tx0 | tx1 << 12 | bucket << 24 (kDeadBox: none),
// by = ymin | ymax << 16 in frame rows.
__device__ __forceinline__ TileSpan box_tiles(uint32_t bt, uint32_t by, uint32_t band, uint32_t nparts, uint32_t part) {
    TileSpan sp{0, 1, 0, 0, 0};
    uint32_t lo, hi;
    if (bt == kDeadBox || !local_row_range(by & 0xFFFFu, by >> 16, band, nparts, part, lo, hi)) return sp;
    sp.tx0 = bt & 0xFFFu;
    sp.ntx = ((bt >> 12) & 0xFFFu) - sp.tx0 + 1u;
    sp.ty0 = lo / kTileH;
    sp.n = sp.ntx * (hi / kTileH - sp.ty0 + 1u);
    sp.bucket = bt >> 24;
    return sp;
}
// The packed tile box of a raster record's pixel bbox bx = xmin | xmax << 16 and bound bits zb, on a
// tile grid shifted left by xoff pixels (tile column c covers x in [64 c - xoff, 64 c - xoff + 64);
// k_tile_raster, tile_grid_x).
__device__ __forceinline__ uint32_t tile_box(uint32_t bx, uint32_t zb, uint32_t xoff) {
    return (((bx & 0xFFFFu) + xoff) / kTileW) | ((((bx >> 16) + xoff) / kTileW) << 12) | (depth_bucket(zb) << 24);
}
static_assert(kDepthBuckets <= 128, "bucket field of a packed tile box (never the dead box's 255)");

// Every lane adds 1 to counter[key] for each tile of its span (or nothing); lanes of the wave with
// the same key share one atomic.  With `list`, the returned positions place `slot` in the lists.
// Per step the groups are found first (ballots only), then every group leader issues its atomic in
// ONE vector instruction, so a step waits for one atomic round trip, not one per distinct tile.
// With `stride` (bins mode), counter[key] counts key's entries and entry i of key goes to
// list[key * stride + i] directly (no scan, no fill pass); an entry past stride is dropped and
// *ovf raised to the count key needs (the frame is then binned again, render_api.cpp).
__device__ __forceinline__ void tile_visit(const TileSpan &sp, uint32_t tiles_x, uint32_t *__restrict__ ctr,
                                           uint32_t *__restrict__ list, uint32_t slot, uint32_t cap = 0xFFFFFFFFu,
                                           uint32_t stride = 0, uint32_t *__restrict__ ovf = nullptr) {
    const uint32_t lane = threadIdx.x & 63u;
    uint32_t rounds = sp.n;
    for (int o = 32; o > 0; o >>= 1) rounds = max(rounds, (uint32_t)__shfl_xor((int)rounds, o));
#ifndef S3R_TV_STEPS
#define S3R_TV_STEPS 2
#endif
    // steps whose atomics are in flight together: a wave's lanes rarely span more than 1-2 tiles, so
    // wider steps mostly run empty ballot rounds (stress scene, bins: 4 -> 2 steps, whole-frame setup
    // 620-627 -> 595 us, part 0 of 8 148 -> 128 us; 8 steps 657, 1 step 606 / 131;
    // profiles/r04_setup_ab.txt)
    constexpr uint32_t kSteps = S3R_TV_STEPS;
    for (uint32_t k0 = 0; k0 < rounds; k0 += kSteps) {
        uint32_t key[kSteps], leader_of[kSteps], rank[kSteps], base[kSteps];
#pragma unroll
        for (uint32_t q = 0; q < kSteps; q++) {
            const uint32_t k = k0 + q;
            const bool act = k < sp.n;
            uint32_t ky = udiv_small(k, udiv_inv(sp.ntx));
            if (sp.n >= (1u << 18)) ky = k / sp.ntx;          // (beyond udiv_small's range: huge boxes)
            key[q] = act ? ((sp.ty0 + ky) * tiles_x + sp.tx0 + k - ky * sp.ntx) * kDepthBuckets + sp.bucket
                         : 0xFFFFFFFFu;
            uint32_t my_leader = 0, my_rank = 0, cnt = 0;
            // groups = runs of adjacent lanes with one key (consecutive triangles of a mesh share
            // tiles): a constant number of instructions per step, where a loop over the distinct keys
            // took one ballot round each; equal keys in separate runs take separate atomics (stress
            // setup: 259 -> 218 M VALU, 79 -> 59 M SALU wave-instructions, time equal, part 0 of 8
            // +2 %; profiles/r05_tvruns_ab.txt)
            const uint32_t prevk = (uint32_t)__shfl_up((int)key[q], 1);
            const bool head = act && (lane == 0u || prevk != key[q]);
            const uint64_t heads = __ballot(head);
            const uint64_t stops = heads | ~__ballot(act);             // a run ends at a head or an idle lane
            const uint64_t upto = (2ull << lane) - 1ull;                // lanes <= this one (lane 63: all)
            if (act) {
                my_leader = 63u - (uint32_t)__builtin_clzll(heads & upto);
                my_rank = lane - my_leader;
            }
            if (head) {
                const uint64_t after = stops & ~upto;
                cnt = (after ? (uint32_t)__builtin_ctzll(after) : 64u) - lane;
            }
            leader_of[q] = my_leader;
            rank[q] = my_rank;
            base[q] = 0;
            if (act && lane == my_leader) {
                if (list) base[q] = atomicAdd(&ctr[key[q]], cnt);
                else atomicAdd(&ctr[key[q]], cnt);
            }
        }
        if (list) {
#pragma unroll
            for (uint32_t q = 0; q < kSteps; q++) {
                const uint32_t b = (uint32_t)__shfl((int)base[q], (int)leader_of[q]);
                if (stride) {
                    if (k0 + q < sp.n) {
                        if (b + rank[q] < stride) list[(size_t)key[q] * stride + b + rank[q]] = slot;
                        else atomicMax(ovf, b + rank[q] + 1u);
                    }
                } else if (k0 + q < sp.n && b + rank[q] < cap) {
                    list[b + rank[q]] = slot;                                  // (past cap: overflow)
                }
            }
        }
    }
}

// A strict upper bound of every 1/z the triangle can produce at a pixel it covers, i.e. of
// ooz = (r0*a0 + r1*a1) + r2*a2 (render.cpp:363) over walked values a_i >= 0 (:362).  The walked
// a_i of pixel (x, y) come from <= nx + ny float adds (:374, :378) through values inside the bbox,
// where the exact affine w*_i(kx, ky) = ws_i + ky*dy_i + kx*dx_i is bounded by its corners: with
// A_i = |ws_i| + ny |dy_i| + nx |dx_i| >= every |w*_i| and S the largest corner sum of w*_0 + w*_1 +
// w*_2, each add rounds by <= 2^-24 (A + 1), so a0 + a1 + a2 <= S + 3 (nx + ny + 1) 2^-24 (A + 1);
// the three products and two sums add <= 2^-22 relative (r_i = 1/z_i > 0 past the near plane).
// Evaluated in float: the corner sums' own rounding is below 2^-21 sum A_i (covered by 2^-20 sum
// A_i), the sum's by 2^-20 (|S| + slack), the product's by the final 2^-18.  A pixel whose current
// winner has a larger 1/z cannot be won by this triangle (strict '>' at :364), so k_tile_raster may
// skip it.
S3R_HD float ooz_bound(const TriSetup &t) {
    const float nx = (float)(t.xmax - t.xmin), ny = (float)(t.ymax - t.ymin);   // (exact: < 2^16)
    float S = -__builtin_inff(), sumA = 0.0f, Amax = 0.0f;
#pragma unroll
    for (int i = 0; i < 3; i++) {
        const float A = (fabsf(t.ws[i]) + ny * fabsf(t.dy[i])) + nx * fabsf(t.dx[i]);
        sumA += A;
        Amax = fmaxf(Amax, A);
    }
#pragma unroll
    for (int cx = 0; cx < 2; cx++) {
#pragma unroll
        for (int cy = 0; cy < 2; cy++) {
            float sum = 0.0f;
#pragma unroll
            for (int i = 0; i < 3; i++) sum += (t.ws[i] + (cy ? ny * t.dy[i] : 0.0f)) + (cx ? nx * t.dx[i] : 0.0f);
            S = fmaxf(S, sum);
        }
    }
    const float slack = 3.0f * (nx + ny + 1.0f) * (Amax + 1.0f) * 0x1p-24f + 0x1p-20f * sumA;
    const float asum = (S + slack) + 0x1p-20f * (fabsf(S) + slack);
    const float rmax = fmaxf(fmaxf(t.rvz[0], t.rvz[1]), t.rvz[2]);
    const float b = rmax * asum * (1.0f + 0x1p-18f) + 0x1p-126f;
    return is_finite(b) && rmax > 0.0f && asum > 0.0f ? b : __builtin_inff();
}

// The live slot's raster record (emit_slot) is stored non-temporal: the records (~10 M on the stress
// scene) stream out past the setup's index / vertex loads instead of occupying L2 until the raster
// reads them.  Stress scene, one MI355X, same box (profiles/r05_ntrec_ab.txt, 64-B records then): setup
// 608-610 -> 577 us serialised, part 0 of 8 5 829-5 932 -> 6 283 fps, whole frame 979-993 -> 1 007 fps;
// the bin entries stored the same way measured slower (624 us: the raster reads them back soon).
// 48-B records (the corners instead of wstart and the steps, recomputed by raster_steps where read):
// setup 580 -> 539-545 us, raster 430 -> 420 us, whole frame pipelined 1 050 -> 1 107-1 113 fps
// (profiles/r05_rec48_ab.txt).
typedef float nt_f4 __attribute__((ext_vector_type(4)));

// Vertex stage (render.cpp:285-289 as a pass over the vertex stream, north_star's "vertex-stage
// kernel"; S3R_VERTEX_STAGE=1): every vertex transformed and projected once, coalesced, into
// rv[i] = (raster x, y, z, 0); k_tile_setup<true> then gathers three of those per triangle instead of
// transforming its three corners (an icosahedron vertex is a corner of five triangles).
__global__ void __launch_bounds__(256) k_tile_vertex(const float4 *__restrict__ vtx, uint32_t nv, Mat34 m, float factor,
                                                     float half_w, float half_h, float4 *__restrict__ rv) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= nv) return;
    Vert d;
    load_corner(vtx, i, m, factor, half_w, half_h, d);
    rv[i] = make_float4(d.rv.x, d.rv.y, d.rv.z, 0.0f);
}

// Sharded streams.  The cluster cull, the setup and the fill work on per-shard lists: a workgroup b
// serves shard b % kTileShards, so appends are wave-aggregated atomics on kTileShards separate
// counters (one cache line apart) -- device-scope atomics on ONE address serialise at ~8-11 ns each
// (measured: one shared counter made the 20 M-triangle setup 2.4 ms), distinct addresses proceed in
// parallel.  Shard s owns the positions [base(s), base(s + 1)) (with clusters: the triangles of its
// clusters, a static table, cmap holding the kept ones; without: an even split of the slots), the
// live entries [2 base(s), 2 base(s + 1)) (a slot and its clip-appended slot) and the clip queue
// [base(s), base(s + 1)).  Counters: 0 positions kept, 1 live entries, 2 clip queue.
__device__ __forceinline__ uint32_t *shard_ctr(uint32_t *ctr, uint32_t which, uint32_t s) {
    return ctr + kTileCounterWords * 16u + (which * kTileShards + s) * kTileShardStride;
}
__device__ __forceinline__ uint32_t shard_base(const uint32_t *tab, uint32_t ntri, uint32_t s) {
    return tab ? tab[s] : (uint32_t)((uint64_t)s * ntri / kTileShards);
}

// Wave-aggregated append of one entry per lane with `want` to list (counter *n): one atomic per wave.
__device__ __forceinline__ void wave_append(bool want, uint4 e, uint4 *__restrict__ list, uint32_t *__restrict__ n) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const uint32_t lane = threadIdx.x & 63u, leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(n, (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__shfl((int)base, (int)leader);
    if (want) list[base + lane_prefix(m, lane)] = e;
}

// Cluster cull (clusters.cpp): can any triangle of the cluster in sphere s (world centre, radius)
// give this part a raster record?  No when every vertex lies behind the near plane (render.cpp:306
// rejects each triangle), when the sphere's screen box lies off one side of the frame (:312-314), or
// when its rows miss the part's interleaved bands.  Conservative: the camera-space centre carries a
// float error far below E, and the screen box is widened by a pixel; a sphere reaching the near
// plane is kept (clipped triangles, :308).
__device__ __forceinline__ bool cluster_meets(float4 s, const Mat34 &m, float factor, float sw, float sh, uint32_t band,
                                              uint32_t nparts, uint32_t part) {
    if (!(s.w < __builtin_inff())) return true;
    const F3 c = mat_mul(m, make_float4(s.x, s.y, s.z, 1.0f));
    const float E = 1e-5f * (fabsf(s.x) + fabsf(s.y) + fabsf(s.z) + fabsf(m.m[0][3]) + fabsf(m.m[1][3]) +
                             fabsf(m.m[2][3]) + s.w);
    const float r = s.w + E, nz = -c.z;
    if (nz + r < kNear) return false;                           // every vertex behind the near plane
    const float z0 = nz - r, z1 = nz + r;
    if (!(z0 > 2.0f * kNear)) return true;                      // reaches the near plane: no bound
    // screen x = cv.x f / nz + W/2, y = -cv.y f / nz + H/2 (render.cpp:288) over the sphere
    // (reciprocals within 1 ulp: far inside the pixel-plus-1e-5 margin below)
    const float ax = c.x - r, bx = c.x + r, ay = -c.y - r, by = -c.y + r;
    const float i0 = __builtin_amdgcn_rcpf(z0), i1 = __builtin_amdgcn_rcpf(z1);
    const float xlo = (ax < 0 ? ax * i0 : ax * i1) * factor + sw / 2, xhi = (bx > 0 ? bx * i0 : bx * i1) * factor + sw / 2;
    const float ylo = (ay < 0 ? ay * i0 : ay * i1) * factor + sh / 2, yhi = (by > 0 ? by * i0 : by * i1) * factor + sh / 2;
    const float mx = 1.0f + 1e-5f * (fabsf(xlo) + fabsf(xhi)), my = 1.0f + 1e-5f * (fabsf(ylo) + fabsf(yhi));
    if (xhi + mx < 0 || yhi + my < 0 || xlo - mx >= sw || ylo - my >= sh) return false;   // off screen
    if (nparts == 1u) return true;
    const uint32_t y0 = u32_of_float(fmaxf(0.0f, ylo - my)), y1 = u32_of_float(fminf(sh - 1, yhi + my));
    uint32_t lo, hi;
    return local_row_range(y0, y1, band, nparts, part, lo, hi);
}

// One thread per cluster (workgroup b: clusters 256 b ..., shard b % kTileShards): the surviving
// clusters' triangle positions, appended to their shard's part of cmap (coalesced).  (Writing
// {vertex indices, slot} records here instead, to spare the setup a dependent load, measured
// worse: cull 21 -> 45 us, setup 133 -> 117 us at part 0 of 8.)
__global__ void __launch_bounds__(256) k_cluster_cull(const float4 *__restrict__ sphere, const uint32_t *__restrict__ first,
                                                      uint32_t ncl, const uint32_t *__restrict__ shard_tab,
                                                      Mat34 m, float factor, float sw, float sh, uint32_t band,
                                                      uint32_t nparts, uint32_t part, uint32_t *__restrict__ cmap,
                                                      uint32_t *__restrict__ ctr) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x, lane = threadIdx.x & 63u, sh_id = blockIdx.x % kTileShards;
    uint32_t n = 0, f0 = 0;
    if (i < ncl) {
        const float4 sp = sphere[i];
        const uint32_t a = first[i], e = first[i + 1];
        if (cluster_meets(sp, m, factor, sw, sh, band, nparts, part)) {
            f0 = a;
            n = e - a;
        }
    }
    uint32_t inc = n;                                           // wave prefix sum of the sizes
    for (uint32_t o = 1; o < 64u; o <<= 1) {
        const uint32_t v = (uint32_t)__shfl_up((int)inc, o);
        if (lane >= o) inc += v;
    }
    const uint32_t tot = (uint32_t)__shfl((int)inc, 63);
    if (tot == 0) return;
    uint32_t base = 0;
    if (lane == 63u) base = atomicAdd(shard_ctr(ctr, 0, sh_id), tot);
    base = (uint32_t)__shfl((int)base, 63) + shard_tab[sh_id];
    // the wave's kept positions, written coalesced: output o comes from the first lane whose
    // inclusive prefix exceeds o (binary search over the prefixes by lane shuffles)
    for (uint32_t o0 = 0; o0 < tot; o0 += 64u) {
        const uint32_t o = o0 + lane;
        uint32_t L = 0;
#pragma unroll
        for (uint32_t step = 32; step >= 1u; step >>= 1)
            if ((uint32_t)__shfl((int)inc, (int)(L + step - 1u)) <= o) L += step;
        L = min(L, 63u);
        const uint32_t fL = (uint32_t)__shfl((int)f0, (int)L), exL = (uint32_t)__shfl((int)(inc - n), (int)L);
        if (o < tot) cmap[base + o] = fL + (o - exL);
    }
}

// u32 flavour of wave_append (the clip queue)
__device__ __forceinline__ void wave_append_u32(bool want, uint32_t v, uint32_t *__restrict__ list, uint32_t *__restrict__ n) {
    const uint64_t m = __ballot(want);
    if (m == 0) return;
    const uint32_t lane = threadIdx.x & 63u, leader = (uint32_t)__builtin_ctzll(m);
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(n, (uint32_t)__builtin_popcountll(m));
    base = (uint32_t)__shfl((int)base, (int)leader);
    if (want) list[base + lane_prefix(m, lane)] = v;
}

// A live slot's raster record, live entry and (tile, bucket) counts -- or nothing when its box misses
// this part's rows (row-band split: the slot is dead here).  Every lane of the wave calls it (the
// entry append and the counting are wave-aggregated).
// Bins mode (tbin non-null, kernels.hip "bins"): the slot goes straight into the fixed-capacity
// bins of its (tile, bucket)s -- no live entry, no fill pass.
__device__ __forceinline__ void emit_slot(bool live, const TriSetup &ts, const Vert *dv, uint32_t slot, uint32_t band,
                                          uint32_t nparts, uint32_t part, uint32_t tiles_x, uint32_t xoff,
                                          RasterRec *__restrict__ recs, uint4 *__restrict__ lv, uint32_t *__restrict__ nlive,
                                          uint32_t *__restrict__ counts, uint32_t *__restrict__ tbin = nullptr,
                                          uint32_t bin_cap = 0, uint32_t *__restrict__ ovf = nullptr, bool rec = true) {
    uint32_t bx = kDeadBox, by = 0;
    const bool keep = rec;                              // (only the clip's slots keep records)
    TileSpan sp{0, 1, 0, 0, 0};
    if (live) {
        // the span first (it does not depend on the depth bucket) and the corners stored before the
        // depth bound is computed: they are dead by then (fewer registers at ooz_bound's peak)
        sp = box_tiles(tile_box(ts.xmin | (ts.xmax << 16), 0u, xoff), ts.ymin | (ts.ymax << 16), band, nparts, part);
        if (sp.n) {
            nt_f4 *q = reinterpret_cast<nt_f4 *>(recs + slot);
            if (keep) {
                __builtin_nontemporal_store((nt_f4){ts.rvz[1], ts.rvz[2], dv[0].rv.x, dv[0].rv.y}, q + 1);
                __builtin_nontemporal_store((nt_f4){dv[1].rv.x, dv[1].rv.y, dv[2].rv.x, dv[2].rv.y}, q + 2);
            }
            const uint32_t zb = f2u(ooz_bound(ts));
            bx = tile_box(ts.xmin | (ts.xmax << 16), zb, xoff);
            by = ts.ymin | (ts.ymax << 16);
            sp.bucket = bx >> 24;
            if (keep) __builtin_nontemporal_store((nt_f4){u2f(ts.xmin | (ts.xmax << 16)), u2f(by), u2f(zb), ts.rvz[0]}, q);
        }
    }
    if (tbin) {
#if defined(S3R_TABLATE) && (S3R_TABLATE & 16)
        if (bx == 12345u)                               // ablation: no binning
#endif
        tile_visit(sp, tiles_x, counts, tbin, rec ? slot : slot | kNoRecBit, 0xFFFFFFFFu, bin_cap, ovf);
        return;
    }
    wave_append(bx != kDeadBox, make_uint4(bx, by, rec ? slot : slot | kNoRecBit, 0), lv, nlive);
#if defined(S3R_TABLATE) && (S3R_TABLATE & 1)
    if (bx == 12345u)                                   // ablation: no tile counting
#endif
    tile_visit(sp, tiles_x, counts, nullptr, 0);
}


// Bins mode, workgroup-aggregated (k_tile_setup): one iteration's entries of the workgroup's 256
// triangles grouped by their (tile, bucket) key in an LDS hash table -- LDS atomics count them, then
// ONE returning global atomic per distinct key reserves the key's run in its bin, and the entries are
// written as one contiguous run per key.  The per-wave form before (tile_visit: runs of equal keys among
// adjacent lanes, a returning global atomic per run) paid a global atomic -- a memory-side round trip
// (MI355X_MICROARCH.md) -- per few entries: stress scene, the binning took ~240 of the setup's 424 us
// (no-binning ablation, profiles/r06_bin_agg_ab.txt).  A key that finds the table full takes the
// per-entry path (a returning atomic of its own).
#ifndef S3R_BIN_AGG
#define S3R_BIN_AGG 1
#endif
constexpr uint32_t kAggSlots = 1024, kAggEmpty = 0xFFFFFFFFu, kAggFull = 0xFFFFFFFFu, kAggProbes = 16;
struct BinAgg {
    uint32_t key[kAggSlots];         // kAggEmpty: free
    uint32_t cnt[kAggSlots];         // entries counted, then (after the reservation) the run's cursor
    uint32_t base[kAggSlots];        // the run's first position in its bin
    uint32_t used[kAggSlots];        // the occupied slots, in insertion order
    uint32_t nused;
};
__device__ __forceinline__ uint32_t agg_hash(uint32_t k) { return (k * 0x9E3779B1u) >> 22; }   // 10 bits
__device__ __forceinline__ uint32_t agg_insert(BinAgg &a, uint32_t key) {
    uint32_t h = agg_hash(key);
    for (uint32_t i = 0; i < kAggProbes; i++, h = (h + 1u) & (kAggSlots - 1u)) {
        const uint32_t prev = atomicCAS(&a.key[h], kAggEmpty, key);
        if (prev == kAggEmpty) { a.used[atomicAdd(&a.nused, 1u)] = h; return h; }
        if (prev == key) return h;
    }
    return kAggFull;
}
__device__ __forceinline__ uint32_t agg_find(const BinAgg &a, uint32_t key) {
    uint32_t h = agg_hash(key);
    for (uint32_t i = 0; i < kAggProbes; i++, h = (h + 1u) & (kAggSlots - 1u)) {
        const uint32_t k = a.key[h];
        if (k == key) return h;
        if (k == kAggEmpty) break;
    }
    return kAggFull;
}
// the (tile, bucket) key of entry k of span sp
__device__ __forceinline__ uint32_t span_key(const TileSpan &sp, uint32_t k, uint32_t tiles_x) {
    uint32_t ky = udiv_small(k, udiv_inv(sp.ntx));
    if (sp.n >= (1u << 18)) ky = k / sp.ntx;            // (beyond udiv_small's range: huge boxes)
    return ((sp.ty0 + ky) * tiles_x + sp.tx0 + k - ky * sp.ntx) * kDepthBuckets + sp.bucket;
}
// The slot's span (its tiles in this part's rows, and its depth bucket), as emit_slot computes it.
__device__ __forceinline__ TileSpan slot_span(bool live, const TriSetup &ts, uint32_t band, uint32_t nparts,
                                              uint32_t part, uint32_t xoff) {
    TileSpan sp{0, 1, 0, 0, 0};
    if (!live) return sp;
    sp = box_tiles(tile_box(ts.xmin | (ts.xmax << 16), 0u, xoff), ts.ymin | (ts.ymax << 16), band, nparts, part);
    if (sp.n) sp.bucket = tile_box(ts.xmin | (ts.xmax << 16), f2u(ooz_bound(ts)), xoff) >> 24;
    return sp;
}
// One iteration's entries of the whole workgroup (every thread calls it, with n = 0 for none):
// entry k of lane's span holds `slot`.  Three barriers; the table is left empty.
__device__ void bin_agg(BinAgg &a, const TileSpan &sp, uint32_t slot, uint32_t tiles_x, uint32_t *__restrict__ counts,
                        uint32_t *__restrict__ tbin, uint32_t bin_cap, uint32_t *__restrict__ ovf) {
    // count
    for (uint32_t k = 0; k < sp.n; k++) {
        const uint32_t key = span_key(sp, k, tiles_x);
        const uint32_t h = agg_insert(a, key);
        if (h != kAggFull) {
            atomicAdd(&a.cnt[h], 1u);
        } else {                                         // table full: this entry on its own
            const uint32_t b = atomicAdd(&counts[key], 1u);
            if (b < bin_cap) tbin[(size_t)key * bin_cap + b] = slot;
            else atomicMax(ovf, b + 1u);
        }
    }
    __syncthreads();
    // reserve each key's run (one returning global atomic per key)
    const uint32_t nu = a.nused;
    for (uint32_t i = threadIdx.x; i < nu; i += blockDim.x) {
        const uint32_t h = a.used[i], c = a.cnt[h];
        const uint32_t b = atomicAdd(&counts[a.key[h]], c);
        if (b + c > bin_cap) atomicMax(ovf, b + c);
        a.base[h] = b;
        a.cnt[h] = 0u;
    }
    __syncthreads();
    // write the runs
    for (uint32_t k = 0; k < sp.n; k++) {
        const uint32_t key = span_key(sp, k, tiles_x);
        const uint32_t h = agg_find(a, key);
        if (h == kAggFull) continue;                     // (written above)
        const uint32_t pos = a.base[h] + atomicAdd(&a.cnt[h], 1u);
        if (pos < bin_cap) tbin[(size_t)key * bin_cap + pos] = slot;
    }
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < nu; i += blockDim.x) {
        const uint32_t h = a.used[i];
        a.key[h] = kAggEmpty;
        a.cnt[h] = 0u;
    }
    if (threadIdx.x == 0) a.nused = 0u;
    __syncthreads();
}

// Setup, one lane per triangle; workgroup b serves shard s = b % kTileShards, grid-stride over the
// shard's positions p = base(s) + j (with clusters: the cull's kept positions cmap[p], each one's slot
// cperm[cmap[p]] -- the identity when cperm is null -- loaded one iteration ahead; without: slot p).
// A triangle
// wholly past the near plane is set up here (emit_slot); one that crosses it (render.cpp:308, rare)
// is queued for k_tile_clip -- the clip keeps it out of this loop's registers (occupancy: the
// setup is memory-latency-bound).
// (occupancy caps of 7 / 8 waves per SIMD, 72 / 64 VGPRs, measured slower: 580 -> 605 / 845 us, part 0
// of 8 129 -> 171 / 218 us; profiles/r05_setup_occ_ab.txt)
// No raster record for the triangles set up here (the raster rebuilds them from the corners,
// kNoRecBit): round 5 measured the record-writing setup slower on every frame kind (stress scene,
// profiles/r05_rec0_ab.txt: setup 548-554 -> 434 us, 1.34 -> 0.84 GB per frame) and round 6 retired it.
template <bool VS, bool CL>
__global__ void __launch_bounds__(256) k_tile_setup(const float4 *__restrict__ vtx, const uint32_t *__restrict__ vidx,
                                                    uint32_t ntri, const uint32_t *__restrict__ cmap,
                                                    const uint32_t *__restrict__ cperm,
                                                    const uint32_t *__restrict__ shard_tab,
                                                    Mat34 m, float factor, float sw, float sh,
                                                    uint32_t band, uint32_t nparts, uint32_t part, uint32_t tiles_x,
                                                    uint32_t xoff, RasterRec *__restrict__ recs, uint4 *__restrict__ live,
                                                    uint32_t *__restrict__ clipq, uint32_t *__restrict__ ctr,
                                                    uint32_t *__restrict__ counts, const float4 *__restrict__ vrv,
                                                    uint32_t *__restrict__ tbin, uint32_t bin_cap) {
    const uint32_t lane = threadIdx.x & 63u, sh_id = blockIdx.x % kTileShards, rank = blockIdx.x / kTileShards;
    const uint32_t per = gridDim.x / kTileShards;              // workgroups per shard (launch: a multiple)
    const uint32_t b0 = shard_base(CL ? shard_tab : nullptr, ntri, sh_id);
    const uint32_t n = CL ? __atomic_load_n(shard_ctr(ctr, 0, sh_id), __ATOMIC_RELAXED)
                          : shard_base(nullptr, ntri, sh_id + 1) - b0;
    uint4 *const lv = live + 2ull * b0;
    uint32_t *const nlive = shard_ctr(ctr, 1, sh_id), *const nclip = shard_ctr(ctr, 2, sh_id);
    const float half_w = sw / 2, half_h = sh / 2;
    // software pipeline over the loop's iterations, two deep: this iteration's corners (vertices, or
    // the vertex stage's projected ones) were loaded during the previous iteration, the next one's
    // corners and the one after's slot and vertex indices load during this one, and (with clusters) the
    // cull's position for the iteration after that -- an iteration's loads are in flight while the
    // iteration before sets up and bins its triangles, so a wave waits on no load chain
    const uint32_t step = per * 256u, jl = rank * 256u + threadIdx.x;
    __shared__ BinAgg agg;
    // (whole frames only: frame parts, their clusters culled, set few triangles up per iteration, and
    // the table's barriers cost more there than the atomics they save -- stress part 0 of 8 -5 %)
    const bool aggregate = S3R_BIN_AGG && !CL && tbin != nullptr;
    if (aggregate) {
        for (uint32_t i = threadIdx.x; i < kAggSlots; i += blockDim.x) { agg.key[i] = kAggEmpty; agg.cnt[i] = 0u; }
        if (threadIdx.x == 0) agg.nused = 0u;
        __syncthreads();
    }
    auto slot_at = [&](uint32_t jj, uint32_t q) { return CL ? (cperm ? cperm[q] : q) : b0 + jj; };
    const float4 *__restrict__ src = VS ? vrv : vtx;
    uint32_t t_cur = 0, t_nxt = 0, vi_nxt[3] = {0, 0, 0}, q_next = 0;
    float4 c_cur[3] = {make_float4(0, 0, 0, 0), make_float4(0, 0, 0, 0), make_float4(0, 0, 0, 0)};
    if (jl < n) {
        t_cur = slot_at(jl, CL ? cmap[b0 + jl] : 0u);
#pragma unroll
        for (int k = 0; k < 3; k++) c_cur[k] = src[vidx[3 * t_cur + k]];
    }
    if (jl + step < n) {
        t_nxt = slot_at(jl + step, CL ? cmap[b0 + jl + step] : 0u);
#pragma unroll
        for (int k = 0; k < 3; k++) vi_nxt[k] = vidx[3 * t_nxt + k];
    }
    if (CL && jl + 2u * step < n) q_next = cmap[b0 + jl + 2u * step];
    // aggregated binning: a workgroup-uniform trip count (its barriers) -- every wave runs while the
    // workgroup's first position is below n; otherwise each wave stops at its own end
    const uint32_t wofs = aggregate ? 0u : (threadIdx.x & ~63u);
    for (uint32_t wb = rank * 256u; wb + wofs < n; wb += step) {
        const uint32_t j = wb + threadIdx.x;
        Vert d[3];
        TriSetup ts;
        bool live_t = false, clip = false;
        const uint32_t t = t_cur;
        const float4 c0 = c_cur[0], c1 = c_cur[1], c2 = c_cur[2];
        if (j + step < n) {                                     // the next iteration's corners
            t_cur = t_nxt;
#pragma unroll
            for (int k = 0; k < 3; k++) c_cur[k] = src[vi_nxt[k]];
        }
        if (j + 2u * step < n) {                                // the one after's slot and indices
            t_nxt = slot_at(j + 2u * step, q_next);
#pragma unroll
            for (int k = 0; k < 3; k++) vi_nxt[k] = vidx[3 * t_nxt + k];
        }
        if (CL && j + 3u * step < n) q_next = cmap[b0 + j + 3u * step];
        if (j < n) {
            const float4 cc[3] = {c0, c1, c2};
#pragma unroll
            for (int k = 0; k < 3; k++) {
                if (VS) d[k].rv = mk3(cc[k].x, cc[k].y, cc[k].z);                 // the vertex stage's rv
                else project_corner(cc[k], m, factor, half_w, half_h, d[k]);
            }
            if (fmaxf(fmaxf(d[0].rv.z, d[1].rv.z), d[2].rv.z) > kNear) {                  // :306
                clip = fminf(fminf(d[0].rv.z, d[1].rv.z), d[2].rv.z) < kNear;             // :308, rare
                if (!clip) live_t = raster_part(d, sw, sh, ts);
            }
        }
        wave_append_u32(clip, b0 + j, clipq + b0, nclip);
#ifdef S3R_STATS
        {   // triangles set up live (whole frames: the aggregated binning), and the waves' lane slots
            const uint64_t lm = __ballot(live_t), am = __ballot(j < n);
            if ((threadIdx.x & 63u) == 0u && am) {
                atomicAdd(&g_stats[8], (unsigned long long)__builtin_popcountll(lm));
                atomicAdd(&g_stats[9], (unsigned long long)__builtin_popcountll(am));
            }
        }
#endif
        if (aggregate)
            bin_agg(agg, slot_span(live_t, ts, band, nparts, part, xoff), t | kNoRecBit, tiles_x, counts, tbin, bin_cap,
                    ctr + 4);
        else
            emit_slot(live_t, ts, d, t, band, nparts, part, tiles_x, xoff, recs, lv, nlive, counts, tbin, bin_cap, ctr + 4,
                      false);
    }
}

// The queued triangles that cross the near plane (render.cpp:308-310): clip, then set up the
// clip-appended slot T + t (if any) and the clipped slot t -- positions only (clip's `textured`
// affects only the payload).  Workgroup b serves shard b % kTileShards.
template <bool CL>
__global__ void __launch_bounds__(256) k_tile_clip(const float4 *__restrict__ vtx, const uint32_t *__restrict__ vidx,
                                                   uint32_t ntri, const uint32_t *__restrict__ cmap,
                                                   const uint32_t *__restrict__ cperm,
                                                   const uint32_t *__restrict__ shard_tab,
                                                   Mat34 m, float factor, float sw, float sh,
                                                   uint32_t band, uint32_t nparts, uint32_t part, uint32_t tiles_x,
                                                   uint32_t xoff, RasterRec *__restrict__ recs, uint4 *__restrict__ live,
                                                   const uint32_t *__restrict__ clipq, uint32_t *__restrict__ ctr,
                                                   uint32_t *__restrict__ counts, uint32_t *__restrict__ tbin,
                                                   uint32_t bin_cap) {
    const uint32_t lane = threadIdx.x & 63u, sh_id = blockIdx.x % kTileShards, rank = blockIdx.x / kTileShards;
    const uint32_t per = gridDim.x / kTileShards;
    const uint32_t b0 = shard_base(CL ? shard_tab : nullptr, ntri, sh_id);
    const uint32_t n = *shard_ctr(ctr, 2, sh_id);
    uint4 *const lv = live + 2ull * b0;
    uint32_t *const nlive = shard_ctr(ctr, 1, sh_id);
    const float half_w = sw / 2, half_h = sh / 2;
    for (uint32_t j0 = rank * 256u + (threadIdx.x & ~63u); j0 < n; j0 += per * 256u) {   // wave-uniform
        const uint32_t j = j0 + lane;
        Vert d[3], app[3];
        TriSetup ts, ta;
        bool live_t = false, live_a = false;
        uint32_t t = 0;
        if (j < n) {
            t = clipq[b0 + j];
            if (CL) {
                t = cmap[t];
                if (cperm) t = cperm[t];
            }
#pragma unroll
            for (int k = 0; k < 3; k++) {
                load_corner(vtx, vidx[3 * t + k], m, factor, half_w, half_h, d[k]);
                d[k].n = mk3(0, 0, 0);
                d[k].pay = make_float4(0, 0, 0, 0);
            }
            uint32_t app_first = 0;
            if (clip_tri(d, app, &app_first, false, factor, half_w, half_h)) live_a = raster_part(app, sw, sh, ta);
            live_t = raster_part(d, sw, sh, ts);
        }
        emit_slot(live_a, ta, app, ntri + t, band, nparts, part, tiles_x, xoff, recs, lv, nlive, counts, tbin, bin_cap, ctr + 4);
        emit_slot(live_t, ts, d, t, band, nparts, part, tiles_x, xoff, recs, lv, nlive, counts, tbin, bin_cap, ctr + 4);
    }
}

// After the exclusive scan of the (tile, bucket) counts (rocprim, launch_tile_setup): the fill's
// scatter cursors start at the offsets.  first (the frame's own launch, not a redo after an
// overflow): workgroup 0 also writes the summary -- ctr[0] the live entries (summed over the
// shards), ctr[1] the list length, ctr[2] the positions the cluster cull kept -- and, when sum_host
// (host-coherent, 4 words) is given, the same three words then the frame's tag into it (system
// scope, tag last: the host spins on it instead of a stream synchronisation); and every count, and
// the shards' cull and clip counters, is reset to 0 for the set's next frame (k_tile_raster reads
// the offsets only and resets the live counters once the fill has read them; all start zeroed).
__global__ void __launch_bounds__(256) k_tile_cursor(uint32_t *__restrict__ counts, const uint32_t *__restrict__ offs,
                                                     uint32_t n, uint32_t *__restrict__ cursor, uint32_t *__restrict__ ctr,
                                                     uint32_t first, uint32_t *__restrict__ sum_host, uint32_t tag) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (first && blockIdx.x == 0 && threadIdx.x < 64u) {
        static_assert(kTileShards == 64, "one lane per shard");
        uint32_t kept = *shard_ctr(ctr, 0, threadIdx.x), lv = *shard_ctr(ctr, 1, threadIdx.x);
        *shard_ctr(ctr, 0, threadIdx.x) = 0u;                 // (read by the cull / setup / clip only)
        *shard_ctr(ctr, 2, threadIdx.x) = 0u;
        for (int o = 32; o > 0; o >>= 1) {
            kept += (uint32_t)__shfl_xor((int)kept, o);
            lv += (uint32_t)__shfl_xor((int)lv, o);
        }
        if (threadIdx.x == 0) {
            const uint32_t total = offs[n - 1u] + counts[n - 1u];
            if (n - 1u >= 256u) counts[n - 1u] = 0u;       // (its own workgroup leaves it to this one)
            ctr[0] = lv; ctr[1] = total; ctr[2] = kept; ctr[3] = 0u;
            if (sum_host) {
                __hip_atomic_store(sum_host + 1, lv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(sum_host + 2, total, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(sum_host + 3, kept, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                __hip_atomic_store(sum_host, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
        }
    }
    if (first && blockIdx.x == 0) __syncthreads();              // (thread 0 has read counts[n - 1])
    if (i >= n) return;
    cursor[i] = offs[i];
    if (first && (i != n - 1u || blockIdx.x == 0)) counts[i] = 0u;
}

// Bins mode's end of binning (in place of the scan, the cursors and the fill): the summary -- ctr[2]
// the positions the cluster cull kept, ctr[5] = the count an overflowing (tile, bucket) needs (0: none,
// k_tile_raster renders nothing then) from the setup's ctr[4], which it resets -- to ctr and, when
// sum_host is given, {tag, 0, 0, kept, needed} to the host (tag last); the shards' cull and clip
// counters reset for the set's next frame.
__global__ void __launch_bounds__(64) k_tile_bins_done(uint32_t *__restrict__ ctr, uint32_t *__restrict__ sum_host,
                                                       uint32_t tag) {
    static_assert(kTileShards == 64, "one lane per shard");
    const uint32_t t = threadIdx.x;
    uint32_t kept = *shard_ctr(ctr, 0, t);
    *shard_ctr(ctr, 0, t) = 0u;
    *shard_ctr(ctr, 2, t) = 0u;
    for (int o = 32; o > 0; o >>= 1) kept += (uint32_t)__shfl_xor((int)kept, o);
    if (t == 0) {
        const uint32_t need = ctr[4];
        ctr[4] = 0u;
        ctr[0] = 0u; ctr[1] = 0u; ctr[2] = kept; ctr[3] = 0u; ctr[5] = need;
        if (sum_host) {
            __hip_atomic_store(sum_host + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(sum_host + 3, kept, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(sum_host + 4, need, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(sum_host, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
}

// Scatter: workgroup b serves shard b % kTileShards, grid-stride over its live entries (original and
// clip-appended slots): each entry's slot into the lists of its tiles.  The list holds cap entries: a
// frame whose list needs more (sized from an earlier frame, no read-back) writes only those, and the
// host renders it again with a larger list (render_api.cpp render_tiles).
__global__ void __launch_bounds__(256) k_tile_fill(const uint4 *__restrict__ live, uint32_t *__restrict__ ctr,
                                                   const uint32_t *__restrict__ shard_tab, uint32_t ntri,
                                                   uint32_t band, uint32_t nparts, uint32_t part, uint32_t tiles_x,
                                                   uint32_t *__restrict__ cursor, uint32_t *__restrict__ list, uint32_t cap) {
    const uint32_t lane = threadIdx.x & 63u, sh_id = blockIdx.x % kTileShards, rank = blockIdx.x / kTileShards;
    const uint32_t per = gridDim.x / kTileShards;
    const uint32_t n = *shard_ctr(ctr, 1, sh_id);
    const uint4 *const lv = live + 2ull * shard_base(shard_tab, ntri, sh_id);
    for (uint32_t j0 = rank * 256u + (threadIdx.x & ~63u); j0 < n; j0 += per * 256u) {   // wave-uniform
        const uint32_t j = j0 + lane;
        uint4 e = make_uint4(kDeadBox, 0, 0, 0);
        if (j < n) e = lv[j];
        tile_visit(box_tiles(e.x, e.y, band, nparts, part), tiles_x, cursor, list, e.z, cap);
    }
}

template <uint32_t STAGE>
struct TileShared {
    unsigned long long key[kTileH * kKeyStride];
    float ws[3][STAGE], dx[3][STAGE], dy[3][STAGE], rz[3][STAGE];
    uint32_t slot[STAGE], xmin[STAGE], xmax[STAGE], ymin[STAGE], r0[STAGE];
    uint32_t pre[STAGE + 1];
    uint16_t item[STAGE * kTileH];            // item -> staged triangle
    uint32_t wsum[kTileThreads / 64];
    uint32_t bstart[kDepthBuckets];                // the tile's list position where each depth bucket starts
    uint32_t zwave[kTileThreads / 64];             // per wave: min over its pixels of the winner's 1/z bits
    uint32_t zmin[kTileH][kTileW / 16];            // per tile row and 16-px group: min over its pixels of
                                                   // bits(1/z) of the current winner (0: a pixel has none)
};

// Shading constants of slot s recomputed from the scene exactly as k_setup computes them.
__device__ __forceinline__ void slot_setup(uint32_t s, uint32_t ntri, const float4 *__restrict__ vtx,
                                           const float4 *__restrict__ nrm, const float4 *__restrict__ pay,
                                           const uint8_t *__restrict__ disc, const uint32_t *__restrict__ vidx,
                                           const uint32_t *__restrict__ aidx, const Mat34 &m, float factor, float sw,
                                           float sh, TriSetup &out) {
    const uint32_t t = s < ntri ? s : s - ntri;
    const float half_w = sw / 2, half_h = sh / 2;
    Vert d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t ai = aidx[3 * t + k];
        load_corner(vtx, vidx[3 * t + k], m, factor, half_w, half_h, d[k]);
        d[k].n = mat_mul(m, nrm[ai]);                                       // :291
        d[k].pay = pay[ai];
    }
    bool textured = disc[aidx[3 * t]] != 0;                                  // :340
    if (fminf(fminf(d[0].rv.z, d[1].rv.z), d[2].rv.z) < kNear) {
        Vert app[3];
        uint32_t app_first = 0;
        const bool appended = clip_tri(d, app, &app_first, textured, factor, half_w, half_h);
        if (s >= ntri && appended) {
#pragma unroll
            for (int k = 0; k < 3; k++) d[k] = app[k];
            textured = disc[aidx[3 * t + app_first]] != 0;
        }
    }
    setup_tri(d, textured, sw, sh, &out);
}

// The scene and camera a tile-path pixel is shaded from (k_tile_resolve, the fused raster).
struct ShadeScene {
    const RasterRec *recs;
    const float4 *vtx, *nrm, *pay;
    const uint8_t *disc;
    const uint32_t *vidx, *aidx, *tex;
    uint32_t ntri, ntex;
    Mat34 m;
    float factor, sw, sh;
};
constexpr uint32_t kDeferPixel = 0xFFFFFFFFu;           // (never a pixel: 0x00RRGGBB)

// The pixel (x, frame row y) of winner key k (render.cpp:360-373 for the winner; background where no
// fragment): the winner re-walked exactly from its raster record and shaded with constants
// recomputed from the scene.  An unclipped winner takes its 1/z and steps from its record (the
// values k_tile_setup computed); a clip-appended or near-plane-crossing winner needs its full setup
// (slot_setup, the clip) -- with DEFER the pixel returns kDeferPixel for k_tile_resolve_deferred
// instead (rare, and the clip's registers stay out of the caller).
// vi (RC): the winner's three vertex indices staged in LDS by the caller, or null (read from the scene).
template <bool DEFER, bool RC = false>
__device__ __forceinline__ uint32_t resolve_pixel(const ShadeScene &sc, unsigned long long k, uint32_t x, uint32_t y,
                                                  const uint32_t *vi = nullptr) {
    if (!k) return kBackground;
    const uint32_t s = 0xFFFFFFFFu - (uint32_t)k;
    const float ooz = u2f((uint32_t)(k >> 32));
    if (DEFER && s >= sc.ntri) return kDeferPixel;
    if (RC) {
        // no record read: the winner set up again from the scene -- its positions first (raster part,
        // the walk to the pixel), then its shading constants -- or its full setup (clip)
        const uint32_t t = s < sc.ntri ? s : s - sc.ntri;
        TriSetup ts;
        float w0, w1, w2;
        bool near_cut = false;
        {
            Vert d[3];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                project_corner(sc.vtx[vi ? vi[c] : sc.vidx[3 * t + c]], sc.m, sc.factor, sc.sw / 2, sc.sh / 2, d[c]);
                near_cut = near_cut || d[c].rv.z < kNear;
            }
            if (s >= sc.ntri || near_cut) {
                if (DEFER) return kDeferPixel;
                slot_setup(s, sc.ntri, sc.vtx, sc.nrm, sc.pay, sc.disc, sc.vidx, sc.aidx, sc.m, sc.factor, sc.sw, sc.sh, ts);
            } else {
                raster_part(d, sc.sw, sc.sh, ts);
            }
            w0 = short_walk(short_walk(ts.ws[0], ts.dy[0], y - ts.ymin), ts.dx[0], x - ts.xmin);
            w1 = short_walk(short_walk(ts.ws[1], ts.dy[1], y - ts.ymin), ts.dx[1], x - ts.xmin);
            w2 = short_walk(short_walk(ts.ws[2], ts.dy[2], y - ts.ymin), ts.dx[2], x - ts.xmin);
        }
        if (s < sc.ntri && !near_cut) {
            Vert d[3];
#pragma unroll
            for (int c = 0; c < 3; c++) {
                const uint32_t ai = sc.aidx[3 * t + c];
                d[c].cv = mat_mul(sc.m, sc.vtx[vi ? vi[c] : sc.vidx[3 * t + c]]);   // (as project_corner: :286)
                d[c].n = mat_mul(sc.m, sc.nrm[ai]);
                d[c].pay = sc.pay[ai];
            }
            shading_part(d, sc.disc[sc.aidx[3 * t]] != 0, ts);
        }
        return shade(&ts, w0, w1, w2, ooz, sc.tex, sc.ntex);
    }
    const float4 *q = reinterpret_cast<const float4 *>(sc.recs + s);
    const uint32_t xmin = f2u(q[0].x) & 0xFFFFu, ymin = f2u(q[0].y) & 0xFFFFu;
    float rws[3], rdx[3], rdy[3], rrz[3];
    {
        const float4 q0 = q[0], q1 = q[1], q2 = q[2];
        raster_steps(mk3(q1.z, q1.w, 0.0f), mk3(q2.x, q2.y, 0.0f), mk3(q2.z, q2.w, 0.0f), xmin, ymin, rws, rdx, rdy);
        rrz[0] = q0.w; rrz[1] = q1.x; rrz[2] = q1.y;
    }
    const float w0 = short_walk(short_walk(rws[0], rdy[0], y - ymin), rdx[0], x - xmin);
    const float w1 = short_walk(short_walk(rws[1], rdy[1], y - ymin), rdx[1], x - xmin);
    const float w2 = short_walk(short_walk(rws[2], rdy[2], y - ymin), rdx[2], x - xmin);
    TriSetup ts;
    const uint32_t t = s < sc.ntri ? s : s - sc.ntri;
    Vert d[3];
    bool near_cut = false;
#pragma unroll
    for (int c = 0; c < 3; c++) {
        const uint32_t ai = sc.aidx[3 * t + c];
        const F3 cv = mat_mul(sc.m, sc.vtx[sc.vidx[3 * t + c]]);
        const float nz = -cv.z;
        d[c].cv = cv;
        d[c].rv = mk3(0.0f, 0.0f, (0.0f * sc.factor) / nz + nz);               // :288 (z only)
        d[c].n = mat_mul(sc.m, sc.nrm[ai]);
        d[c].pay = sc.pay[ai];
        near_cut = near_cut || d[c].rv.z < kNear;
    }
    if (s >= sc.ntri || near_cut) {
        if (DEFER) return kDeferPixel;
        slot_setup(s, sc.ntri, sc.vtx, sc.nrm, sc.pay, sc.disc, sc.vidx, sc.aidx, sc.m, sc.factor, sc.sw, sc.sh, ts);
    } else {
        ts.kind = kDead;
#pragma unroll
        for (int c = 0; c < 3; c++) { ts.rvz[c] = rrz[c]; ts.dx[c] = rdx[c]; ts.dy[c] = rdy[c]; }
        shading_part(d, sc.disc[sc.aidx[3 * t]] != 0, ts);
    }
    return shade(&ts, w0, w1, w2, ooz, sc.tex, sc.ntex);
}

// The tile's winners are shaded here, straight from LDS, and stored to out (its local row, or with
// frame_rows its frame row) -- no per-pixel key round trip through HBM and, for frames written into
// the caller's buffer, each tile's stores cross the link while other tiles rasterize; pixels whose
// winner needs a full setup go to the deferred queue (k_tile_resolve_deferred).  (Round 4 measured
// the split form -- keys through HBM, a per-pixel resolve launch -- slower everywhere: stress scene
// whole frame 800 -> 854 fps fused, delivered 583 -> 614, part 0 of 8 4 491 -> 4 672; it is gone.)
template <uint32_t STAGE = kTileStage>
#ifndef S3R_TOCC
#define S3R_TOCC 6                     // min waves per SIMD of the fused raster: 80 VGPRs (92 uncapped, occupancy 5);
#endif                                 // the 256-stage instance stays at 4 (its LDS).  Stress scene, one box
                                       // (profiles/r05_raster_occ_ab.txt): raster 462 -> 430 us serialised, whole
                                       // frame pipelined 1 030-1 036 -> 1 068-1 083 fps; 7 (72 VGPRs, 12 spilled):
                                       // the same raster time, part 0 of 8 -2.5 %
__global__ void __launch_bounds__(kTileThreads, STAGE <= 128u ? S3R_TOCC : 1) k_tile_raster(
    const RasterRec *__restrict__ recs, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
    uint32_t tiles_x, const uint32_t *__restrict__ offs, uint32_t *__restrict__ ctr,
    const uint32_t *__restrict__ list, uint32_t cap,
    ShadeScene sc, uint32_t *__restrict__ out, uint32_t frame_rows, uint4 *__restrict__ deferred,
    uint32_t *__restrict__ counts, uint32_t bin_cap, uint32_t xoff) {
    static_assert(STAGE <= kTileThreads, "one staged triangle per thread at most");
    __shared__ TileShared<STAGE> ls;
    const uint32_t *const total = ctr + 1;
    // the fill (complete before this launch) was the live counters' last reader: reset them for the
    // set's next frame -- unless the list overflowed (the frame's fill runs again, render_api.cpp)
    if (!bin_cap && blockIdx.x == 0u && threadIdx.x < kTileShards && *total <= cap)
        *shard_ctr(ctr, 1, threadIdx.x) = 0u;
    const uint32_t tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
    const uint32_t tile = blockIdx.x, ty = tile / tiles_x, tx = tile - ty * tiles_x;
    // the tile's pixel columns: [64 tx - xoff, 64 tx - xoff + 64) inside the frame (tile_box)
    const uint32_t lx0 = max(tx * kTileW, xoff) - xoff, lx1 = min(W, tx * kTileW + kTileW - xoff) - 1u;
    const uint32_t tr0 = ty * kTileH, tr1 = min(rows_local, tr0 + kTileH) - 1u;
    const float ib = udiv_inv(band);
    auto row_of = [&](uint32_t lr) {
        const uint32_t g = udiv_small(lr, ib);
        return nparts == 1u ? lr : (g * nparts + part) * band + (lr - g * band);
    };
    for (uint32_t i = tid; i < kTileH * kKeyStride; i += kTileThreads) ls.key[i] = 0ull;
    // the tile's list: its depth buckets, nearest first, one after another
    const uint32_t s0 = tile * kDepthBuckets;
    uint32_t base = 0, n = 0;
    if (bin_cap) {
        // bins mode: bucket b's entries at list[(s0 + b) * bin_cap ...], counts[s0 + b] of them; the
        // counts reset for the set's next frame once read.  An overflowed frame (ctr[5]) renders
        // nothing: it is binned again with larger bins (render_api.cpp)
        if (tid < 64u) {
            constexpr uint32_t kPB = kDepthBuckets > 64u ? kDepthBuckets / 64u : 1u;   // buckets per lane
            uint32_t c[kPB], sum = 0;
#pragma unroll
            for (uint32_t e = 0; e < kPB; e++) {
                const uint32_t b = tid * kPB + e;
                c[e] = b < kDepthBuckets ? counts[s0 + b] : 0u;
                if (b < kDepthBuckets) counts[s0 + b] = 0u;
                sum += c[e];
            }
            uint32_t inc = sum;
            for (uint32_t o = 1; o < 64u; o <<= 1) {
                const uint32_t v = (uint32_t)__shfl_up((int)inc, o);
                if (tid >= o) inc += v;
            }
            uint32_t st = inc - sum;
#pragma unroll
            for (uint32_t e = 0; e < kPB; e++) {
                const uint32_t b = tid * kPB + e;
                if (b < kDepthBuckets) ls.bstart[b] = st;
                st += c[e];
            }
            if (tid == 63u) ls.zwave[0] = ctr[5] ? 0u : inc;       // (zwave: free until the first stage)
        }
        __syncthreads();
        n = ls.zwave[0];
        // the frame's binned entries, for the statistics (bins mode has no list length): summed per
        // shard in the live counters, which bins mode leaves unused; k_tile_resolve_deferred totals them
        if (tid == 0u && n) atomicAdd(shard_ctr(ctr, 1, tile % kTileShards), n);
    } else {
        // a list longer than its buffer (overflow, see k_tile_fill) is incomplete: the frame is redone
        const uint32_t ntiles = tiles_x * ((rows_local + kTileH - 1u) / kTileH);
        const uint32_t end = tile + 1u < ntiles ? offs[s0 + kDepthBuckets] : *total;
        base = offs[s0];
        n = *total > cap ? 0u : end - base;
        if (tid < kDepthBuckets) ls.bstart[tid] = offs[s0 + tid] - base;
    }
    // software pipeline: stage c0 + STAGE's list entries and records are loaded into registers
    // while stage c0's items run
    uint32_t s_nx = 0, b_nx = 0;                 // (b_nx: the entry's depth bucket)
    float4 q0n = make_float4(0, 0, 0, 0), q1n = q0n, q2n = q0n;
    auto fetch = [&](uint32_t c) {
        if (tid < STAGE && c + tid < n) {
            {                                            // the entry's depth bucket (its bound's ceiling)
                uint32_t bb = 0;
#pragma unroll
                for (uint32_t step = kDepthBuckets / 2u; step >= 1u; step >>= 1)
                    if (ls.bstart[bb + step] <= c + tid) bb += step;
                b_nx = bb;
            }
            if (bin_cap) {
                const uint32_t v = c + tid;
                uint32_t b = 0;                                  // the bucket holding entry v
#pragma unroll
                for (uint32_t step = kDepthBuckets / 2u; step >= 1u; step >>= 1)
                    if (ls.bstart[b + step] <= v) b += step;
                s_nx = list[(size_t)(s0 + b) * bin_cap + (v - ls.bstart[b])];
#ifdef S3R_BOUNDS
                if (v - ls.bstart[b] >= bin_cap) {
                    printf("S3R_BOUNDS raster: tile %u entry %u bucket %u start %u cap %u n %u\n", tile, v, b, ls.bstart[b], bin_cap, n);
                    s_nx = 0;
                }
#endif
            } else {
                s_nx = list[base + c + tid];
            }
#ifdef S3R_BOUNDS
            if (sc.ntri && (s_nx & ~kNoRecBit) >= 2u * sc.ntri) {
                printf("S3R_BOUNDS raster: tile %u slot %u >= %u (bins %u)\n", tile, s_nx, 2u * sc.ntri, bin_cap);
                s_nx = 0;
            }
#endif
            if (s_nx & kNoRecBit) {                 // no record: the corners (set up at staging)
                const uint32_t *vi = sc.vidx + 3ull * (s_nx & ~kNoRecBit);
                const uint32_t v0 = vi[0], v1 = vi[1], v2 = vi[2];
                q0n = sc.vtx[v0]; q1n = sc.vtx[v1]; q2n = sc.vtx[v2];
            } else {
                const float4 *q = reinterpret_cast<const float4 *>(recs + s_nx);
                q0n = q[0]; q1n = q[1]; q2n = q[2];
            }
        }
    };
    fetch(0);
#ifdef S3R_STATS
    uint32_t st_staged = 0, st_culled = 0;
#endif
    for (uint32_t c0 = 0; c0 < n; c0 += STAGE) {
        __syncthreads();                                 // previous stage fully consumed
#if !(defined(S3R_TNOHIZ) && S3R_TNOHIZ)
        // hierarchical depth: each tile row's farthest current winner (0 while a pixel has none)
        if (c0 > 0) {
            const uint32_t rr = tid >> 4, cc = (tid & 15u) * 4u;
            const unsigned long long *kr = ls.key + rr * kKeyStride + cc;
            uint32_t kz[4];
#pragma unroll
            for (int k = 0; k < 4; k++) kz[k] = (uint32_t)(kr[k] >> 32);
            uint32_t m = min(min(kz[0], kz[1]), min(kz[2], kz[3]));
            // over the tile's pixels inside the frame part only (a partial tile's outside keys stay 0)
            uint32_t mt = 0xFFFFFFFFu;
#pragma unroll
            for (int k = 0; k < 4; k++)
                if (tr0 + rr <= tr1 && lx0 + cc + k <= lx1) mt = min(mt, kz[k]);
            for (int o = 2; o > 0; o >>= 1) m = min(m, (uint32_t)__shfl_xor((int)m, o));
            for (int o = 32; o > 0; o >>= 1) mt = min(mt, (uint32_t)__shfl_xor((int)mt, o));
            if ((tid & 3u) == 0u) ls.zmin[rr][(tid & 15u) >> 2] = m;
            if (lane == 0u) ls.zwave[wave] = mt;
        }
        __syncthreads();
        if (c0 > 0) {
            // the rest of the list starts in the depth bucket of position c0 (buckets run nearest
            // first): if every pixel of the tile already holds a winner at least as near as that
            // bucket's ceiling, no listed triangle from here on can win a pixel (strict '>', render.cpp:364)
            uint32_t b = 0;
#pragma unroll
            for (uint32_t step = kDepthBuckets / 2u; step >= 1u; step >>= 1)
                if (ls.bstart[b + step] <= c0) b += step;
            uint32_t zt = ls.zwave[0];
            for (uint32_t w = 1; w < kTileThreads / 64u; w++) zt = min(zt, ls.zwave[w]);
#if !(defined(S3R_TNOSKIP) && S3R_TNOSKIP)
            if (zt >= bucket_ceiling(b)) break;
#endif
        }
#endif
        const uint32_t j = c0 + tid;
        uint32_t nr = 0;
        if (tid < STAGE && j < n) {
            const uint32_t s = s_nx & ~kNoRecBit;
            float4 q0 = q0n, q1 = q1n, q2 = q2n;
            if (s_nx & kNoRecBit) {
                // the record k_tile_setup would have written, from the corners: box, bound, 1/z, corners
                Vert d[3];
                const float4 cc[3] = {q0, q1, q2};
#pragma unroll
                for (int k = 0; k < 3; k++) project_corner(cc[k], sc.m, sc.factor, sc.sw / 2, sc.sh / 2, d[k]);
                TriSetup ts;
                raster_part(d, sc.sw, sc.sh, ts);            // (true: the setup binned it)
                // the setup's bound (ooz_bound) lies below its depth bucket's ceiling: that ceiling serves as
                // the row cull's bound (coarser, never below the true one; bucket 0: none, never culled) --
                // ooz_bound here cost 80-VGPR spills (36 -> 8 B/lane): stress raster 510 -> 498 us
                const uint32_t zb = bucket_ceiling(b_nx) - 1u;
                q0 = make_float4(u2f(ts.xmin | (ts.xmax << 16)), u2f(ts.ymin | (ts.ymax << 16)), u2f(zb), ts.rvz[0]);
                q1 = make_float4(ts.rvz[1], ts.rvz[2], d[0].rv.x, d[0].rv.y);
                q2 = make_float4(d[1].rv.x, d[1].rv.y, d[2].rv.x, d[2].rv.y);
            }
            const uint32_t bx = f2u(q0.x), by = f2u(q0.y);
            const uint32_t zbits = f2u(q0.z);
            uint32_t lo = 1u, hi = 0u;
            local_row_range(by & 0xFFFFu, by >> 16, band, nparts, part, lo, hi);
            const uint32_t a = max(lo, tr0), b = min(hi, tr1);
            nr = (lo <= hi && a <= b) ? b - a + 1u : 0u;
#if !(defined(S3R_TNOHIZ) && S3R_TNOHIZ)
            // every pixel of rows [a, b] already holds a 1/z above anything this triangle can
            // produce (ooz_bound): it wins none of them (strict '>', render.cpp:364)
#ifdef S3R_STATS
            st_staged += nr ? 1u : 0u;
#endif
            if (nr && c0 > 0) {
                const uint32_t g0 = (max(bx & 0xFFFFu, lx0) - lx0) >> 4, g1 = (min(bx >> 16, lx1) - lx0) >> 4;
                const uint32_t zb = zbits;
                bool cull = true;
                for (uint32_t r = a; r <= b && cull; r++)
                    for (uint32_t g = g0; g <= g1; g++) cull = cull && zb < ls.zmin[r - tr0][g];
                if (cull) nr = 0;
#ifdef S3R_STATS
                st_culled += cull ? 1u : 0u;
#endif
            }
#endif
            ls.slot[tid] = s; ls.xmin[tid] = bx & 0xFFFFu; ls.xmax[tid] = bx >> 16; ls.ymin[tid] = by & 0xFFFFu;
            ls.r0[tid] = a;
            if (nr) {                                    // (the steps only for a triangle with rows here)
                float ws[3], dx[3], dy[3];
                raster_steps(mk3(q1.z, q1.w, 0.0f), mk3(q2.x, q2.y, 0.0f), mk3(q2.z, q2.w, 0.0f), bx & 0xFFFFu,
                             by & 0xFFFFu, ws, dx, dy);
#pragma unroll
                for (int c = 0; c < 3; c++) { ls.ws[c][tid] = ws[c]; ls.dx[c][tid] = dx[c]; ls.dy[c][tid] = dy[c]; }
            }
            ls.rz[0][tid] = q0.w; ls.rz[1][tid] = q1.x; ls.rz[2][tid] = q1.y;
        }
        fetch(c0 + STAGE);
        // exclusive scan of the row counts over the stage (wave shuffles + wave totals)
        uint32_t inc = nr;
        for (uint32_t o = 1; o < 64u; o <<= 1) {
            const uint32_t v = (uint32_t)__shfl_up((int)inc, o);
            if (lane >= o) inc += v;
        }
        if (lane == 63u) ls.wsum[wave] = inc;
        __syncthreads();
        uint32_t wbase = 0;
        for (uint32_t w = 0; w < wave; w++) wbase += ls.wsum[w];
        if (tid < STAGE) ls.pre[tid] = wbase + inc - nr;
        uint32_t items = 0;
        for (uint32_t w = 0; w < kTileThreads / 64u; w++) items += ls.wsum[w];
#if !(defined(S3R_TITEM) && S3R_TITEM)
        if (tid < STAGE)
            for (uint32_t i = 0; i < nr; i++) ls.item[ls.pre[tid] + i] = (uint16_t)tid;
        __syncthreads();
#endif
#if defined(S3R_TITEM) && S3R_TITEM
        // one lane per staged triangle: all its rows in this tile, wy += dy between rows (:378)
        if (nr) {                                        // nr == 0 beyond the stage
            const uint32_t k = tid;
            const uint32_t xmin = ls.xmin[k];
            const uint32_t x0 = max(xmin, lx0), x1 = min(ls.xmax[k], lx1);
            float wy[3], d[3], dyv[3], r[3];
            uint32_t yprev = ls.ymin[k];
#pragma unroll
            for (uint32_t c = 0; c < 3; c++) {
                d[c] = ls.dx[c][k]; dyv[c] = ls.dy[c][k]; r[c] = ls.rz[c][k]; wy[c] = ls.ws[c][k];
            }
            const unsigned long long low = 0xFFFFFFFFull - ls.slot[k];
            for (uint32_t lr = ls.r0[k], lend = lr + nr; lr < lend; lr++) {
                const uint32_t y = row_of(lr);
                float w[3];
#pragma unroll
                for (uint32_t c = 0; c < 3; c++) {
                    wy[c] = short_walk(wy[c], dyv[c], y - yprev);
                    w[c] = short_walk(wy[c], d[c], x0 - xmin);
                }
                yprev = y;
                unsigned long long *krow = ls.key + (lr - tr0) * kKeyStride - lx0;
                for (uint32_t x = x0; x <= x1; x++) {
                    if (w[0] >= 0 && w[1] >= 0 && w[2] >= 0) {                        // :362
                        const float ooz = (r[0] * w[0] + r[1] * w[1]) + r[2] * w[2];  // :363
                        if (ooz > 0.0f) atomicMax(krow + x, ((unsigned long long)f2u(ooz) << 32) | low);
                    }
                    w[0] = w[0] + d[0]; w[1] = w[1] + d[1]; w[2] = w[2] + d[2];    // :374
                }
            }
        }
        if (items == 0xFFFFFFFFu)
#endif
        for (uint32_t it = tid; it < items; it += kTileThreads) {
            const uint32_t k = ls.item[it];
            const uint32_t lr = ls.r0[k] + (it - ls.pre[k]);
            const uint32_t y = row_of(lr);
            const uint32_t xmin = ls.xmin[k];
            const uint32_t x0 = max(xmin, lx0), x1 = min(ls.xmax[k], lx1);
            float w[3], d[3], r[3];
#pragma unroll
            for (uint32_t c = 0; c < 3; c++) {
                d[c] = ls.dx[c][k];
                r[c] = ls.rz[c][k];
                w[c] = short_walk(short_walk(ls.ws[c][k], ls.dy[c][k], y - ls.ymin[k]), d[c], x0 - xmin);
            }
            const unsigned long long low = 0xFFFFFFFFull - ls.slot[k];
            unsigned long long *krow = ls.key + (lr - tr0) * kKeyStride - lx0;
#if defined(S3R_TABLATE) && (S3R_TABLATE & 4)
            if (x1 == 0xFFFFFFFFu)                      // ablation: no pixel loop
#endif
            for (uint32_t x = x0; x <= x1; x++) {
                if (w[0] >= 0 && w[1] >= 0 && w[2] >= 0) {                        // :362
                    const float ooz = (r[0] * w[0] + r[1] * w[1]) + r[2] * w[2];  // :363
#if defined(S3R_TABLATE) && (S3R_TABLATE & 2)
                    if (ooz == 1234.5f) krow[x] = low;          // ablation: no LDS atomic
#elif defined(S3R_TPRECHECK) && S3R_TPRECHECK
                    const unsigned long long kv = ((unsigned long long)f2u(ooz) << 32) | low;
                    if (ooz > 0.0f && kv > krow[x]) atomicMax(krow + x, kv);   // plain read first
#else
                    if (ooz > 0.0f) atomicMax(krow + x, ((unsigned long long)f2u(ooz) << 32) | low);
#endif
                }
                w[0] = w[0] + d[0]; w[1] = w[1] + d[1]; w[2] = w[2] + d[2];    // :374
            }
        }
    }
#ifdef S3R_STATS
    {
        uint32_t v[2] = {st_staged, st_culled};
        for (int k = 0; k < 2; k++) {
            for (int o = 32; o > 0; o >>= 1) v[k] += (uint32_t)__shfl_xor((int)v[k], o);
            if (lane == 0) atomicAdd(&g_stats[k], (unsigned long long)v[k]);
        }
    }
#endif
    __syncthreads();
#ifdef S3R_STATS
    {
        // the resolve's winners: foreground pixels, runs of one winner along a row (lane = column),
        // and per wave (its 4 rows) ceil(runs / 64) -- the setup rounds a run-shared resolve would take
        uint32_t fg = 0, runs = 0;
        for (uint32_t i = tid; i < kTileH * kTileW; i += kTileThreads) {
            const uint32_t rr = i / kTileW, cc = i % kTileW;
            const bool in = tr0 + rr <= tr1 && lx0 + cc <= lx1;
            const unsigned long long k = in ? ls.key[rr * kKeyStride + cc] : 0ull;
            const uint32_t sl = k ? (uint32_t)k : 0u;
            const uint32_t left = (uint32_t)__shfl_up((int)sl, 1);
            fg += sl ? 1u : 0u;
            runs += (sl && (lane == 0u || left != sl)) ? 1u : 0u;
        }
        uint32_t v[2] = {fg, runs};
        for (int k = 0; k < 2; k++)
            for (int o = 32; o > 0; o >>= 1) v[k] += (uint32_t)__shfl_xor((int)v[k], o);
        if (lane == 0) {
            atomicAdd(&g_stats[2], (unsigned long long)v[0]);
            atomicAdd(&g_stats[3], (unsigned long long)v[1]);
            atomicAdd(&g_stats[4], (unsigned long long)((v[1] + 63u) / 64u));
            atomicAdd(&g_stats[5], 1ull);
            atomicMax(&g_stats[6], (unsigned long long)v[1]);
        }
    }
#endif
    {
#ifndef S3R_RESOLVE_VIX
#define S3R_RESOLVE_VIX 1
#endif
        // the winners' vertex indices of all the tile's pixels loaded at once into LDS (the staging
        // arrays, free now): each pixel's chain of dependent loads then starts at its corners
        // (stages of 128 triangles and more: the staging arrays hold the tile's 1 024 x 3 indices)
        constexpr bool kVix = S3R_RESOLVE_VIX &&
            offsetof(TileShared<STAGE>, wsum) - offsetof(TileShared<STAGE>, ws) >= kTileH * kTileW * 3u * 4u;
        uint32_t *const vix = reinterpret_cast<uint32_t *>(&ls.ws[0][0]);
        if (kVix) {
#pragma unroll
            for (uint32_t q = 0; q < kTileH * kTileW / kTileThreads; q++) {
                const uint32_t i = tid + q * kTileThreads, rr = i / kTileW, cc = i % kTileW;
                const unsigned long long k = tr0 + rr <= tr1 && lx0 + cc <= lx1 ? ls.key[rr * kKeyStride + cc] : 0ull;
                const uint32_t s = 0xFFFFFFFFu - (uint32_t)k;
                uint32_t v0 = 0, v1 = 0, v2 = 0;
                if (k && s < sc.ntri) { v0 = sc.vidx[3 * s]; v1 = sc.vidx[3 * s + 1]; v2 = sc.vidx[3 * s + 2]; }
                vix[3 * i] = v0; vix[3 * i + 1] = v1; vix[3 * i + 2] = v2;
            }
            __syncthreads();
        }
        for (uint32_t i = tid; i < kTileH * kTileW; i += kTileThreads) {   // (wave-uniform trip count)
            const uint32_t rr = i / kTileW, cc = i % kTileW;
            const uint32_t lr = tr0 + rr, x = lx0 + cc;
            const bool in = lr <= tr1 && x <= lx1;
            const unsigned long long k = in ? ls.key[rr * kKeyStride + cc] : 0ull;
            const uint32_t y = row_of(lr);
            uint32_t v = kBackground;
#if defined(S3R_TABLATE) && (S3R_TABLATE & 8)
            if (in) v = (uint32_t)k & 0xFFFFFFu;                // ablation: no resolve (timing only)
#else
            if (in) v = resolve_pixel<true, true>(sc, k, x, y, kVix ? vix + 3 * i : nullptr);
#endif
            const size_t idx = frame_rows ? (size_t)y * W + x : (size_t)lr * W + x;
#ifdef S3R_BOUNDS
            if (in && idx >= (size_t)W * (frame_rows ? (uint32_t)sc.sh : rows_local)) {
                printf("S3R_BOUNDS fused store: tile %u x %u y %u lr %u idx %lu W %u rows %u\n", tile, x, y, lr,
                       (unsigned long)idx, W, frame_rows ? (uint32_t)sc.sh : rows_local);
                continue;
            }
#endif
            wave_append(in && v == kDeferPixel, make_uint4((uint32_t)idx, (uint32_t)k, (uint32_t)(k >> 32), (x & 0xFFFFu) | (y << 16)),
                        deferred, ctr + 3);
            if (in && v != kDeferPixel) out[idx] = v;
        }
    }
}

// The fused raster's deferred pixels (ctr[3] entries {out index, key, x | y << 16}): shaded with the
// winner's full setup.  Grid-stride (the queue is short: pixels of near-plane and clip-appended
// winners).
// Bins mode (bins != 0): workgroup 0 also totals the frame's binned entries from the raster's per-shard
// sums (resetting them) into ctr[1] and, when given, word 2 of the host summary (system scope; the
// host reads it once the frame is done).
__global__ void __launch_bounds__(256) k_tile_resolve_deferred(ShadeScene sc, const uint4 *__restrict__ deferred,
                                                               uint32_t *__restrict__ ctr, uint32_t *__restrict__ out,
                                                               uint32_t bins, uint32_t *__restrict__ sum_host) {
    if (bins && blockIdx.x == 0 && threadIdx.x < 64u) {
        static_assert(kTileShards == 64, "one lane per shard");
        uint32_t v = *shard_ctr(ctr, 1, threadIdx.x);
        *shard_ctr(ctr, 1, threadIdx.x) = 0u;
        for (int o = 32; o > 0; o >>= 1) v += (uint32_t)__shfl_xor((int)v, o);
        if (threadIdx.x == 0) {
            ctr[1] = v;
            if (sum_host) __hip_atomic_store(sum_host + 2, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
    }
    const uint32_t n = ctr[3];
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < n; i += gridDim.x * 256u) {
        const uint4 e = deferred[i];
        const unsigned long long k = (unsigned long long)e.y | ((unsigned long long)e.z << 32);
#ifdef S3R_BOUNDS
        if (e.x >= (uint32_t)sc.sw * (uint32_t)sc.sh || (uint32_t)(0xFFFFFFFFu - (uint32_t)k) >= 2u * sc.ntri) {
            printf("S3R_BOUNDS deferred: %u of %u idx %u slot %u\n", i, n, e.x, 0xFFFFFFFFu - (uint32_t)k);
            continue;
        }
#endif
        out[e.x] = resolve_pixel<false>(sc, k, e.w & 0xFFFFu, e.w >> 16);
    }
}

// ------------------------------------------------------------------ self-test kernel
// Batch evaluation of exact_walk / chunk_linear on the device, for tests/test_exact_walk.py.
__global__ void __launch_bounds__(256) k_walk_test(const float *s, const float *d, const uint32_t *n, float *out,
                                                   uint32_t *lin, float *del, uint32_t count) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= count) return;
    out[i] = exact_walk(s[i], d[i], n[i]);
    float dl;
    lin[i] = chunk_linear(s[i], d[i], n[i], &dl) ? 1u : 0u;
    del[i] = dl;
}

void launch_walk_test(const float *s, const float *d, const uint32_t *n, float *out, uint32_t *lin, float *del,
                      uint32_t count, hipStream_t st) {
    if (count == 0) return;
    hipLaunchKernelGGL(k_walk_test, dim3((count + 255) / 256), dim3(256), 0, st, s, d, n, out, lin, del, count);
}

// Self-test of the trimmed division / sqrt sequences (s3r_common.h) against the compiler's IEEE
// operators: mode 0 every x in [2^-96, 2^127) for sqrt, mode 1 every s in [2^-48, 2^64) for 1/s (the
// normalize reciprocal), mode 2 `count` hashed quotient pairs inside div_in_range (all-zero and
// all-one significands included), mode 3 `count` hashed vectors for the whole normalize.
// res[0] += mismatches, res[1] = min mismatching index (res[1] initialised to ~0 by the caller).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__device__ __forceinline__ float hashed_float(uint64_t h, uint32_t e) {
    uint32_t m = (uint32_t)h & 0x7FFFFFu;
    const uint32_t sel = (uint32_t)(h >> 40) & 15u;
    if (sel == 0u) m = 0u;
    if (sel == 1u) m = 0x7FFFFFu;
    return u2f(((uint32_t)(h >> 63) << 31) | (e << 23) | m);
}
__global__ void __launch_bounds__(256) k_fastmath_test(uint32_t mode, uint64_t count, unsigned long long *res) {
#if S3R_FASTDIV
    uint64_t bad = 0, first = ~0ull;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (uint64_t)gridDim.x * blockDim.x) {
        bool ok = true;
        if (mode == 0u) {
            const float x = u2f(0x0F800000u + (uint32_t)i);
            ok = f2u(sqrt_in_range(x)) == f2u(sqrtf(x));
        } else if (mode == 1u) {
            const float x = u2f((79u << 23) + (uint32_t)i);
            ok = f2u(div_with_recip(1.0f, x, div_recip(x))) == f2u(1.0f / x);
        } else if (mode == 2u) {
            const uint64_t h1 = mix64(2 * i + 1), h2 = mix64(2 * i + 2);
            const uint32_t ea = 32u + (uint32_t)(h1 % 191u);
            const int eb0 = (int)ea + (int)(h2 % 129u) - 64;
            const uint32_t eb = (uint32_t)min(max(eb0, 32), 222);
            const float a = hashed_float(h1, ea), b = hashed_float(h2, eb);
            if (div_in_range(a, b)) ok = f2u(div_with_recip(a, b, div_recip(b))) == f2u(a / b);
        } else {
            const uint64_t h1 = mix64(3 * i + 1), h2 = mix64(3 * i + 2), h3 = mix64(3 * i + 3);
            const uint32_t e0 = 60u + (uint32_t)(h1 % 130u);
            const F3 v = mk3(hashed_float(h1, e0), hashed_float(h2, e0 - (uint32_t)(h2 % 30u)),
                             hashed_float(h3, e0 - (uint32_t)(h3 % 30u)));
            const F3 p = fast_normalize3_dev(v), q = fast_normalize3(v);
            ok = f2u(p.x) == f2u(q.x) && f2u(p.y) == f2u(q.y) && f2u(p.z) == f2u(q.z);
        }
        if (!ok) { bad++; first = min(first, i); }
    }
    if (bad) { atomicAdd(&res[0], (unsigned long long)bad); atomicMin(&res[1], (unsigned long long)first); }
#else
    (void)mode; (void)count;
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(&res[0], 1ull);   // not built: report failure
#endif
}

int fastmath_test(uint32_t mode, uint64_t count, uint64_t out[2]) {
    if (mode == 0u) count = 0x7F000000ull - 0x0F800000ull;
    if (mode == 1u) count = (uint64_t)(191u - 79u) << 23;
    unsigned long long *res = nullptr;
    if (hipMalloc((void **)&res, 16) != hipSuccess) return -1;
    const unsigned long long init[2] = {0ull, ~0ull};
    (void)hipMemcpy(res, init, 16, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_fastmath_test, dim3(8192), dim3(256), 0, nullptr, mode, count, res);
    const hipError_t e = hipMemcpy(out, res, 16, hipMemcpyDeviceToHost);
    (void)hipFree(res);
    return e == hipSuccess ? 0 : -1;
}

uint32_t geo_times_read(unsigned long long *out, uint32_t max_wg) {
#ifdef S3R_WGTIME
    (void)hipDeviceSynchronize();
    const uint32_t n = max_wg < kGeoTimesMax ? max_wg : kGeoTimesMax;
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_gwt), sizeof(unsigned long long) * 4 * n, 0, hipMemcpyDeviceToHost);
    unsigned long long *z = (unsigned long long *)calloc(4 * n, sizeof(unsigned long long));
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_gwt), z, sizeof(unsigned long long) * 4 * n, 0, hipMemcpyHostToDevice);
    free(z);
    return n;
#else
    (void)out; (void)max_wg;
    return 0;
#endif
}

uint32_t wg_times_read(unsigned long long *out, uint32_t max_wg) {
#ifdef S3R_WGTIME
    (void)hipDeviceSynchronize();
    const uint32_t n = max_wg < kWgTimesMax ? max_wg : kWgTimesMax;
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wgt), sizeof(unsigned long long) * kWgSlots * n, 0, hipMemcpyDeviceToHost);
    return n;
#else
    (void)out; (void)max_wg;
    return 0;
#endif
}

void stats_read(unsigned long long out[24], bool reset) {
#ifdef S3R_STATS
    (void)hipDeviceSynchronize();
    (void)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stats), sizeof(unsigned long long) * 16, 0, hipMemcpyDeviceToHost);
    (void)hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_tstats), sizeof(unsigned long long) * 8, 0, hipMemcpyDeviceToHost);
    if (reset) {
        unsigned long long z[16] = {};
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_stats), z, sizeof z, 0, hipMemcpyHostToDevice);
        z[2] = ~0ull;
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_tstats), z, sizeof(unsigned long long) * 8, 0, hipMemcpyHostToDevice);
    }
#else
    (void)reset;
    for (int i = 0; i < 24; i++) out[i] = 0;
#endif
}

// ------------------------------------------------------------------ bounded-wait test hook
// One wave that spins `ticks` of the 100 MHz device clock and exits: a stage that is late but always
// finishes (S3R_TEST_HOLD_MS, render_api.cpp; tests/test_stall.py).
__global__ void __launch_bounds__(64) k_test_hold(uint64_t ticks) {
    const uint64_t t0 = wall_clock64();
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
}

void launch_test_hold(uint32_t ms, hipStream_t st) {
    hipLaunchKernelGGL(k_test_hold, dim3(1), dim3(64), 0, st, (uint64_t)ms * 100000ull);
}

uint32_t device_spin_ticks() {
    static const uint32_t ticks = [] {
        const char *e = getenv("S3R_SPIN_MS");
        const long ms = e ? atol(e) : 0;
        return (uint32_t)(ms > 0 && ms < 40000 ? ms : 2000) * 100000u;
    }();
    return ticks;
}

// ------------------------------------------------------------------ launchers
// S3R_CHECK=1: each launch synchronised and checked (s3r_kernels.h).  The context is per host
// thread: with several devices behind updateAndRender each device's worker launches its own part.
static thread_local int t_check_dev = -1;
static thread_local uint32_t t_check_frame = 0;
static thread_local const char *t_check_stage = "";

bool check_launches() {
    static const bool on = getenv("S3R_CHECK") && atoi(getenv("S3R_CHECK")) != 0;
    return on;
}

void check_context(int device, uint32_t frame, const char *stage) {
    t_check_dev = device;
    t_check_frame = frame;
    t_check_stage = stage;
}

void after_launch(const char *kernel, hipStream_t st) {
    if (!check_launches()) return;
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) {
        sync_stream_bounded(st, t_check_stage, kernel, t_check_dev, t_check_frame);
        e = hipGetLastError();
    }
    if (e != hipSuccess) {
        fprintf(stderr, "s3r: S3R_CHECK: %s after %s (device %d, frame %u, %s)\n", hipGetErrorName(e), kernel,
                t_check_dev, t_check_frame, t_check_stage);
        abort();
    }
}

#ifndef S3R_SEG_PIXELS
#define S3R_SEG_PIXELS 384
#endif
constexpr uint32_t kSegChunks = S3R_SEG_PIXELS / kChunk;   // widest fragment segment, in chunks
static_assert(kSegChunks * kChunk == S3R_SEG_PIXELS, "segment = whole chunks");
static_assert(kSegChunks == 6, "k_fragment instantiations below: 6, 3, 2, 1 chunks");
// k_geometry's to_pairs maps start-table points (multiples of kStartPx) to the segments they start:
// every segment width the build can choose must divide kStartPx.
static_assert(kStartPx % (kChunk * 6u) == 0 && kStartPx % (kChunk * 3u) == 0 && kStartPx % (kChunk * 2u) == 0 &&
              kStartPx % kChunk == 0, "fragment segment widths must divide the start-table spacing");

// Segment width of this frame's row path: the widest of 6, 3, 2, 1 chunks that still launches at
// least kMinFragBlocks workgroups (~8 per CU), so small frames fill the chip (a 1080p frame at
// 6 chunks is 1350 workgroups; each runs a latency-bound chain, so too few leave CUs idle).
// Widths tried: 6, 2, 1 chunks.  Round-2 sweep (tools/knob_sweep.sh, tools/part_knobs.sh): where
// 3-chunk segments were chosen (1080p: 2 700 workgroups; 1/4 of 4K: 2 700) 2-chunk ones (4 050) were
// faster (1080p flat 31.6k -> 34.3k fps, 4K part 1/4 38.7k -> 40.8k); elsewhere the choice is unchanged.
constexpr uint64_t kMinFragBlocks = 2000;   // measured best or near-best for 4K at 1, 2, 4, 8 row-band parts and 1080p
// per host thread: with several devices behind updateAndRender each device's worker thread configures
// and launches its own frame part (render_api.cpp), and parts may differ in rows
static thread_local uint32_t g_segch = kSegChunks;

static uint32_t segment_chunks(uint32_t W, uint32_t rows_local) {
    const char *mb_env = getenv("S3R_MIN_BLOCKS");                                  // tuning / test override
    const uint64_t min_blocks = mb_env ? strtoull(mb_env, nullptr, 10) : kMinFragBlocks;
    const bool try3 = getenv("S3R_SEG3") != nullptr;                                // tuning override
    for (uint32_t c : {6u, 3u, 2u}) {
        if (c == 3u && !try3) continue;
        const uint64_t blocks = (uint64_t)((rows_local + kWaves - 1) / kWaves) * ((W + kChunk * c - 1) / (kChunk * c));
        if (blocks >= min_blocks) return c;
    }
    return 1u;
}

void fragment_configure(uint32_t W, uint32_t rows_local) { g_segch = segment_chunks(W, rows_local); }

FragLayout fragment_layout(uint32_t W, uint32_t rows_local) {
    FragLayout l;
    l.seg_px = kChunk * segment_chunks(W, rows_local);
    l.segs = (W + l.seg_px - 1) / l.seg_px;
    l.rows_per_bin = kWaves;
    l.chunk_px = kChunk;
    l.bins = (uint64_t)((rows_local + kWaves - 1) / kWaves) * l.segs;
    return l;
}

uint32_t fragment_segment_pixels() { return kChunk * g_segch; }

uint32_t fragment_segments(uint32_t W) { return (W + kChunk * g_segch - 1) / (kChunk * g_segch); }

uint64_t fragment_bins(uint32_t W, uint32_t rows_local) {
    return (uint64_t)((rows_local + kWaves - 1) / kWaves) * fragment_segments(W);
}

void launch_geometry(const float4 *vtx, const float4 *nrm, const float4 *pay, const uint8_t *disc,
                     const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri, const Mat34 &m, float factor,
                     uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                     TriSetup *tris, float *rowtab, uint32_t *bincnt, uint4 *pairs, hipStream_t st, hipEvent_t done,
                     uint32_t *order, const GeoSkyFlags *gsf, bool row_starts, bool clip_slots,
                     const SlotMask *live) {
    const bool masked = live && live->on && !clip_slots && ntri <= kLiveMaskSlots;
    const uint32_t nslots = clip_slots ? 2u * ntri : ntri;
    SlotMask lm{};
    if (masked) lm = *live;
    const uint32_t nrb = (rows_local + kGeoRows - 1) / kGeoRows;
    const uint32_t nwg = (masked ? lm.nlive : nslots) * nrb + (masked ? 1u : 0u);   // + the dead-slot marker
    if (ntri == 0 || rows_local == 0 || (gsf && nrb > kGeoCntMax)) {
        // nothing to set up (every bin is sky), or more row blocks than counters: k_sky_flags publishes
        if (ntri && rows_local) {
            const uint32_t segs = fragment_segments(W), posmap_bytes = (kGeoRows / kWaves * segs + 3u) & ~3u;
            { hipExtLaunchKernelGGL(k_geometry, dim3(nwg + (order ? 1u : 0u)), dim3(3 * kGeoRows), posmap_bytes,
                                  st, nullptr, nullptr, 0, vtx, nrm, pay, disc, vidx, aidx, ntri, m, factor, W, H, band,
                                  nparts, part, rows_local, segs, kChunk * g_segch, tris, rowtab, bincnt, pairs,
                                  (uint32_t)fragment_bins(W, rows_local), order, nrb,
                                  SkyFlags{}, row_starts ? 1u : 0u, nslots, lm); after_launch("k_geometry", st); }
        }
        if (gsf)
            launch_sky_flags(bincnt, fragment_bins(W, rows_local), gsf->flags, gsf->tag, gsf->probe, gsf->gpu_eighths,
                             st, done);
        else if (done)
            (void)hipEventRecord(done, st);
        return;
    }
    // the publishers wait for one arrival per geometry workgroup of their row block: per row block,
    // one workgroup per launched slot -- the count the grid below is built from
    const uint32_t per_rb = masked ? lm.nlive : nslots;
    if (masked) {
        uint32_t bits = 0;
        for (uint64_t w : lm.bits) bits += (uint32_t)__builtin_popcountll(w);
        if (bits != lm.nlive) {
            fprintf(stderr, "s3r: k_geometry: slot mask has %u bits but counts %u live slots\n", bits, lm.nlive);
            abort();
        }
    }
    const SkyFlags sky = gsf ? SkyFlags{gsf->flags, gsf->probe, gsf->geo_cnt, gsf->tag, gsf->gpu_eighths, gsf->err,
                                        per_rb + gsf->extra_arrivals, device_spin_ticks()}
                             : SkyFlags{};
    // the completion event is recorded by the launch itself (one host call instead of two)
    // dynamic LDS: one pair index per bin of a workgroup's rows (posmap)
    const uint32_t segs = fragment_segments(W), posmap_bytes = (kGeoRows / kWaves * segs + 3u) & ~3u;
    { hipExtLaunchKernelGGL(k_geometry, dim3(nwg + (order ? 1u : 0u) + (gsf ? nrb : 0u)),
                          dim3(3 * kGeoRows), posmap_bytes, st, nullptr, done, 0, vtx, nrm, pay, disc, vidx, aidx, ntri,
                          m, factor, W, H, band, nparts, part, rows_local, segs, kChunk * g_segch, tris, rowtab, bincnt,
                          pairs, (uint32_t)fragment_bins(W, rows_local), order, nrb, sky, row_starts ? 1u : 0u, nslots, lm); after_launch("k_geometry", st); }
}

void launch_fragment(const TriSetup *tris, uint32_t nslots, const float *rowtab, const uint32_t *tex, uint32_t ntex,
                     uint32_t *out, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
                     uint32_t rows_local, uint32_t *bincnt, const uint4 *pairs,
                     hipStream_t st, hipEvent_t done, uint32_t *done_flag, uint32_t prev_tag, uint32_t *order,
                     bool frame_rows, uint32_t host_fill, unsigned long long *chunk_flags, uint32_t fill_tag,
                     bool row_starts) {
    const uint32_t segs = fragment_segments(W);
    const uint64_t blocks = fragment_bins(W, rows_local);
    if (blocks == 0) {                                   // (render_core never asks for an empty frame part)
        if (done) (void)hipEventRecord(done, st);
        return;
    }
    const char *wf_env = getenv("S3R_WATERFALL_BINS");                             // tuning / test override
    const uint64_t wf_bins = wf_env ? strtoull(wf_env, nullptr, 10) : S3R_WATERFALL_BINS;
    auto pick = [&](auto hostw) {
        constexpr bool HW = decltype(hostw)::value;
        return g_segch == 6 ? (blocks >= wf_bins ? k_fragment<6, true, HW> : k_fragment<6, false, HW>)
             : g_segch == 3 ? k_fragment<3, false, HW> : g_segch == 2 ? k_fragment<2, false, HW> : k_fragment<1, false, HW>;
    };
    auto kern = frame_rows ? pick(std::true_type{}) : pick(std::false_type{});
    if (done)
        { hipExtLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(64 * kWaves), 0, st, nullptr, done, 0, tris, nslots,
                              rowtab, tex, ntex, out, W, H, band, nparts, part, segs, rows_local, bincnt, pairs,
                              done_flag, prev_tag, order, host_fill, chunk_flags, fill_tag, row_starts ? 1u : 0u); after_launch("k_fragment", st); }
    else
        { hipLaunchKernelGGL(kern, dim3((uint32_t)blocks), dim3(64 * kWaves), 0, st, tris, nslots, rowtab, tex, ntex, out,
                           W, H, band, nparts, part, segs, rows_local, bincnt, pairs, done_flag, prev_tag, order,
                           host_fill, chunk_flags, fill_tag, row_starts ? 1u : 0u); after_launch("k_fragment", st); }
}

// Host fill (render_api.cpp): once k_geometry's pair counts are final, one flag per fragment bin in
// host-coherent memory -- tag, with kSkyBit when no triangle meets the bin -- so the host writes the
// background of sky bins while k_fragment writes only the covered bins into the caller's buffer.
// probe (may be null): the device address of the caller's pixel 0; the magic written there before
// bin 0's flag (release) lets the host check that the mapping reaches the caller's pages.
// gpu_eighths: sky bins with b % 8 below it are written by the fragment kernel (kGpuBit), the rest by
// the host (kSkyBit) -- the host / link balance of render_api.cpp's adaptive host fill.
__global__ void __launch_bounds__(256) k_sky_flags(const uint32_t *__restrict__ bincnt, uint32_t nbins, uint32_t *flags,
                                                   uint32_t tag, uint32_t *probe, uint32_t gpu_eighths) {
    const uint32_t b = blockIdx.x * 256u + threadIdx.x;
    if (b >= nbins) return;
    const uint32_t f = bincnt[b] != 0u ? tag : ((b & 7u) < gpu_eighths ? (tag | kGpuBit) : (tag | kSkyBit));
    if (b == 0 && probe) {
        __hip_atomic_store(probe, kMapProbe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(flags, f, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
        __hip_atomic_store(flags + b, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

void launch_sky_flags(const uint32_t *bincnt, uint64_t nbins, uint32_t *flags, uint32_t tag, uint32_t *probe,
                      uint32_t gpu_eighths, hipStream_t st, hipEvent_t done) {
    const uint32_t blocks = (uint32_t)((nbins + 255) / 256);
    if (blocks == 0) {
        if (done) (void)hipEventRecord(done, st);
        return;
    }
    { hipExtLaunchKernelGGL(k_sky_flags, dim3(blocks), dim3(256), 0, st, nullptr, done, 0, bincnt, (uint32_t)nbins, flags,
                          tag, probe, gpu_eighths); after_launch("k_sky_flags", st); }
}

// ------------------------------------------------------------------ band de-interleave
// The gathered parts (part p's compact rows at gathered + p * part_stride_rows * W, as one RCCL gather
// leaves them on GPU 0) -> the W x H frame in row order (frame row y belongs to part
// (y / band) % nparts, local row (y / band / nparts) * band + y % band).  One thread per 4 pixels
// (16-B loads and stores when W % 4 == 0 and both buffers are 16-B aligned); grid (x blocks, H).
template <bool V4>
__global__ void __launch_bounds__(256) k_deinterleave_bands(const uint32_t *__restrict__ gathered, uint32_t part_stride_rows,
                                                            uint32_t W, uint32_t band, uint32_t nparts,
                                                            uint32_t *__restrict__ frame) {
    const uint32_t y = blockIdx.y, g = y / band, part = g % nparts, lr = (g / nparts) * band + y % band;
    const uint32_t *src = gathered + ((size_t)part * part_stride_rows + lr) * W;
    uint32_t *dst = frame + (size_t)y * W;
    const uint32_t x = (blockIdx.x * 256u + threadIdx.x) * 4u;
    if (V4) {
        if (x < W) *reinterpret_cast<uint4 *>(dst + x) = *reinterpret_cast<const uint4 *>(src + x);
    } else {
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
            if (x + k < W) dst[x + k] = src[x + k];
    }
}

void launch_deinterleave_bands(const uint32_t *gathered, uint32_t part_stride_rows, uint32_t W, uint32_t H,
                               uint32_t band, uint32_t nparts, uint32_t *frame, hipStream_t st) {
    if (!W || !H) return;
    const dim3 grid((W + 1023u) / 1024u, H);
    const bool v4 = W % 4 == 0 && ((uintptr_t)gathered & 15u) == 0 && ((uintptr_t)frame & 15u) == 0;
    if (v4)
        { hipLaunchKernelGGL(k_deinterleave_bands<true>, grid, dim3(256), 0, st, gathered, part_stride_rows, W, band, nparts,
                           frame); after_launch("k_deinterleave_bands", st); }
    else
        { hipLaunchKernelGGL(k_deinterleave_bands<false>, grid, dim3(256), 0, st, gathered, part_stride_rows, W, band,
                           nparts, frame); after_launch("k_deinterleave_bands", st); }
}

// Test hook (include/render.h s3r_ooz_bound): the tile path's 1/z bound of a raster setup, computed
// on the host by the same code the kernels run.
float ooz_bound_host(const float ws[3], const float dx[3], const float dy[3], const float rvz[3], uint32_t xmin,
                     uint32_t xmax, uint32_t ymin, uint32_t ymax) {
    TriSetup t{};
    for (int i = 0; i < 3; i++) { t.ws[i] = ws[i]; t.dx[i] = dx[i]; t.dy[i] = dy[i]; t.rvz[i] = rvz[i]; }
    t.xmin = xmin; t.xmax = xmax; t.ymin = ymin; t.ymax = ymax;
    return ooz_bound(t);
}

uint32_t tile_grid_x(uint32_t W, uint32_t xoff = 0) { return (W + xoff + kTileW - 1) / kTileW; }
uint32_t tile_height() { return kTileH; }
static_assert(kTileH % 4u == 0, "tile rows = whole 4-row resolve blocks (slabbed fragment stage)");
uint32_t tile_count(uint32_t W, uint32_t rows_local, uint32_t xoff) {
    return tile_grid_x(W, xoff) * ((rows_local + kTileH - 1) / kTileH);
}
uint64_t tile_slots(uint32_t W, uint32_t rows_local, uint32_t xoff) {
    return (uint64_t)tile_count(W, rows_local, xoff) * kDepthBuckets;
}

size_t tile_scan_temp_bytes(uint64_t nslots) {
    size_t bytes = 0;
    (void)rocprim::exclusive_scan(nullptr, bytes, (const uint32_t *)nullptr, (uint32_t *)nullptr, 0u, (size_t)nslots,
                                  rocprim::plus<uint32_t>(), nullptr);
    return bytes;
}
size_t raster_rec_bytes() { return sizeof(RasterRec); }

std::vector<uint32_t> cluster_shard_table(const std::vector<uint32_t> &first) {
    std::vector<uint32_t> tab(kTileShards + 1, 0u);
    const uint32_t ncl = first.empty() ? 0u : (uint32_t)first.size() - 1;
    for (uint32_t c = 0; c < ncl; c++) tab[(c / 256u) % kTileShards + 1] += first[c + 1] - first[c];
    for (uint32_t s = 0; s < kTileShards; s++) tab[s + 1] += tab[s];
    return tab;
}

// Grid of a sharded grid-stride kernel: kTileShards x (up to what the whole chip holds resident at
// once, so every workgroup runs from the start and the shards' loops end together -- a grid larger
// than that leaves its late workgroups to run all their iterations after the others have finished),
// fewer when there is less work.
// Workgroups per shard: S3R_TILE_GRID = k (k > 0) or 0 (what the device keeps resident); default
// `dflt` (measured on the stress scene: 256 for the cluster-culled frame parts' setup, 1024 -- about
// one workgroup per 256 slots, no loop -- for whole frames).
uint32_t shard_grid(const void *kernel, uint64_t work, uint32_t dflt = 256) {
    static const int knob = getenv("S3R_TILE_GRID") ? atoi(getenv("S3R_TILE_GRID")) : -1;
    uint64_t cap = knob > 0 ? (uint64_t)knob : knob < 0 ? dflt : 0;
    if (!cap) {
        static std::mutex mu;                      // (device worker threads launch concurrently)
        static std::map<const void *, uint32_t> resident;   // workgroups of 256 the device keeps resident
        std::lock_guard<std::mutex> lk(mu);
        uint32_t &r = resident[kernel];
        if (!r) {
            int dev = 0, cus = 0, per_cu = 0;
            (void)hipGetDevice(&dev);
            (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
            (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0);
            r = std::max(kTileShards, (uint32_t)(std::max(cus, 1) * std::max(per_cu, 1)));
        }
        cap = std::max<uint64_t>(1, r / kTileShards);
    }
    const uint64_t per = std::min<uint64_t>(cap, std::max<uint64_t>(1, (work / kTileShards + 255) / 256));
    return (uint32_t)(per * kTileShards);
}
template <class K> uint32_t shard_grid(K *kernel, uint64_t work, uint32_t dflt = 256) {
    return shard_grid(reinterpret_cast<const void *>(kernel), work, dflt);
}

template <bool VS, bool CL>
void setup_launch(const float4 *vtx, const uint32_t *vidx, uint32_t ntri, const TileClusters *cl, const Mat34 &m,
                  float factor, float sw, float sh, uint32_t band, uint32_t nparts, uint32_t part, uint32_t tx, uint32_t xoff,
                  void *recs, uint4 *live, uint32_t *clipq, uint32_t *ctr, uint32_t *counts, const float4 *vrv,
                  hipStream_t st, uint32_t *tbin, uint32_t bin_cap) {
    const uint32_t *cmap = CL ? cl->cmap : nullptr, *perm = CL ? cl->perm : nullptr, *tab = CL ? cl->shard : nullptr;
    { hipLaunchKernelGGL((k_tile_setup<VS, CL>), dim3(shard_grid(k_tile_setup<VS, CL>, ntri, CL ? 256 : 1024)), dim3(256),
                       0, st, vtx, vidx, ntri, cmap, perm, tab, m, factor, sw, sh, band, nparts, part, tx, xoff,
                       (RasterRec *)recs, live, clipq, ctr, counts, vrv, tbin, bin_cap); after_launch("k_tile_setup", st); }
    // the clip queue is short (triangles crossing the near plane): one workgroup per shard
    { hipLaunchKernelGGL((k_tile_clip<CL>), dim3(kTileShards), dim3(256), 0, st, vtx, vidx, ntri, cmap, perm, tab, m,
                       factor, sw, sh, band, nparts, part, tx, xoff, (RasterRec *)recs, live, clipq, ctr, counts, tbin,
                       bin_cap); after_launch("k_tile_clip", st); }
}

void launch_tile_setup(const float4 *vtx, const uint32_t *vidx, uint32_t ntri, const Mat34 &m, float factor, float sw,
                       float sh, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                       void *recs, uint4 *live, uint32_t *clipq, uint32_t *ctr, uint32_t *counts, uint32_t *offs,
                       uint32_t *cursor, void *scan_temp, size_t scan_temp_bytes, hipStream_t st, float4 *vrv,
                       uint32_t nv, const TileClusters *cl, uint32_t *sum_host, uint32_t tag, uint32_t *tbin,
                       uint32_t bin_cap, uint32_t xoff) {
    const uint64_t ns = tile_slots(W, rows_local, xoff);  // (counts and ctr's shard counters: left zeroed)
    const bool clustered = cl && cl->ncl;
    if (vrv && nv && !clustered)
        { hipLaunchKernelGGL(k_tile_vertex, dim3((nv + 255) / 256), dim3(256), 0, st, vtx, nv, m, factor, sw / 2, sh / 2, vrv); after_launch("k_tile_vertex", st); }
    if (ntri) {
        const uint32_t tx = tile_grid_x(W, xoff);
        if (clustered) {
            { hipLaunchKernelGGL(k_cluster_cull, dim3((cl->ncl + 255) / 256), dim3(256), 0, st, cl->sphere, cl->first,
                               cl->ncl, cl->shard, m, factor, sw, sh, band, nparts, part, cl->cmap, ctr); after_launch("k_cluster_cull", st); }
            setup_launch<false, true>(vtx, vidx, ntri, cl, m, factor, sw, sh, band, nparts, part, tx, xoff, recs, live, clipq,
                                      ctr, counts, nullptr, st, tbin, bin_cap);
        } else if (vrv) {
            setup_launch<true, false>(vtx, vidx, ntri, cl, m, factor, sw, sh, band, nparts, part, tx, xoff, recs, live, clipq,
                                      ctr, counts, vrv, st, tbin, bin_cap);
        } else {
            setup_launch<false, false>(vtx, vidx, ntri, cl, m, factor, sw, sh, band, nparts, part, tx, xoff, recs, live,
                                       clipq, ctr, counts, nullptr, st, tbin, bin_cap);
        }
    }
    if (bin_cap) {                                       // bins mode: binned already
        { hipLaunchKernelGGL(k_tile_bins_done, dim3(1), dim3(64), 0, st, ctr, sum_host, tag); after_launch("k_tile_bins_done", st); }
        return;
    }
    size_t bytes = scan_temp_bytes;
    (void)rocprim::exclusive_scan(scan_temp, bytes, (const uint32_t *)counts, offs, 0u, (size_t)ns,
                                  rocprim::plus<uint32_t>(), st);
    after_launch("rocprim_exclusive_scan", st);
    { hipLaunchKernelGGL(k_tile_cursor, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, st, counts, offs, (uint32_t)ns,
                       cursor, ctr, 1u, sum_host, tag); after_launch("k_tile_cursor", st); }
}

void launch_tile_cursor(const uint32_t *counts, const uint32_t *offs, uint32_t W, uint32_t rows_local, uint32_t *cursor,
                        uint32_t *ctr, hipStream_t st, uint32_t xoff) {
    const uint64_t ns = tile_slots(W, rows_local, xoff);
    if (ns == 0) return;
    { hipLaunchKernelGGL(k_tile_cursor, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, st, (uint32_t *)counts, offs,
                       (uint32_t)ns, cursor, ctr, 0u, (uint32_t *)nullptr, 0u); after_launch("k_tile_cursor", st); }
}

void launch_tile_fill(const uint4 *live, uint32_t *ctr, const TileClusters *cl, uint32_t ntri, uint32_t W,
                      uint32_t band, uint32_t nparts, uint32_t part, uint32_t *cursor, uint32_t *list, uint64_t cap,
                      hipStream_t st, uint32_t xoff) {
    if (ntri == 0) return;
    { hipLaunchKernelGGL(k_tile_fill, dim3(shard_grid(k_tile_fill, ntri)), dim3(256), 0, st, live, ctr,
                       cl && cl->ncl ? cl->shard : nullptr, ntri, band, nparts, part, tile_grid_x(W, xoff), cursor, list,
                       (uint32_t)(cap < 0xFFFFFFFFull ? cap : 0xFFFFFFFFull)); after_launch("k_tile_fill", st); }
}

void launch_tile_raster_resolve(const void *recs, const float4 *vtx, const float4 *nrm, const float4 *pay,
                                const uint8_t *disc, const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri,
                                const Mat34 &m, float factor, float sw, float sh, const uint32_t *tex, uint32_t ntex,
                                uint32_t *out, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part,
                                uint32_t rows_local, const uint32_t *offs, uint32_t *ctr, const uint32_t *list,
                                uint64_t cap, uint4 *deferred, hipStream_t st, bool frame_rows, uint32_t *counts,
                                uint32_t bin_cap, uint32_t xoff, uint32_t *sum_host) {
    const uint32_t tx = tile_grid_x(W, xoff), ty = (rows_local + kTileH - 1) / kTileH;
    if (tx == 0 || ty == 0) return;
    const ShadeScene sc{(const RasterRec *)recs, vtx, nrm, pay, disc, vidx, aidx, tex, ntri, ntex, m, factor, sw, sh};
    // frames written into the caller's buffer stage 256 triangles at a time, frames into HBM 128: on
    // the stress scene (one MI355X, profiles/r04_tstage_ab.txt) the wider stage delivers 772 / 726 ->
    // 802 / 803 fps (the raster waits on the link anyway, and half the stage rounds and barriers
    // remain), but costs the HBM frame 975 -> 952 fps (its LDS lowers the occupancy).  Both rebuild the
    // records the setup leaves out at staging (kNoRecBit).
    const uint32_t capw = (uint32_t)(cap < 0xFFFFFFFFull ? cap : 0xFFFFFFFFull);
    if (frame_rows)
        { hipLaunchKernelGGL((k_tile_raster<kTileStageLink>), dim3(tx * ty), dim3(kTileThreads), 0, st,
                           (const RasterRec *)recs, W, band, nparts, part, rows_local, tx, offs, ctr, list,
                           capw, sc, out, 1u, deferred, counts, bin_cap, xoff); after_launch("k_tile_raster", st); }
    else
        { hipLaunchKernelGGL((k_tile_raster<kTileStage>), dim3(tx * ty), dim3(kTileThreads), 0, st,
                           (const RasterRec *)recs, W, band, nparts, part, rows_local, tx, offs, ctr, list, capw, sc,
                           out, 0u, deferred, counts, bin_cap, xoff); after_launch("k_tile_raster", st); }
    { hipLaunchKernelGGL(k_tile_resolve_deferred, dim3(64), dim3(256), 0, st, sc, (const uint4 *)deferred, ctr, out,
                       bin_cap ? 1u : 0u, sum_host); after_launch("k_tile_resolve_deferred", st); }
}

void launch_tile_resolve_deferred(const void *recs, const float4 *vtx, const float4 *nrm, const float4 *pay,
                                  const uint8_t *disc, const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri,
                                  const Mat34 &m, float factor, float sw, float sh, const uint32_t *tex, uint32_t ntex,
                                  uint32_t *out, const uint4 *deferred, uint32_t *ctr, hipStream_t st, bool bins,
                                  uint32_t *sum_host) {
    const ShadeScene sc{(const RasterRec *)recs, vtx, nrm, pay, disc, vidx, aidx, tex, ntri, ntex, m, factor, sw, sh};
    { hipLaunchKernelGGL(k_tile_resolve_deferred, dim3(64), dim3(256), 0, st, sc, deferred, ctr, out, bins ? 1u : 0u,
                       sum_host); after_launch("k_tile_resolve_deferred", st); }
}

}  // namespace s3r
