// kernels.hip -- the gfx950 HIP kernels of the rasterizer.
//
//   k_vertex    render.cpp:284-292  camera-space + raster transform of the vertex stream and the
//                                   normal transform of the attribute stream (coalesced float4).
//   k_setup     render.cpp:297-359  per triangle: gather, reject, near-plane clip (:212-262), cull,
//                                   raster setup.  Writes slot t and, for a clip split, slot T+t.
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

namespace s3r {

// ------------------------------------------------------------------ K1: vertex + normal transform
// simd_mul(simd_float4x3, simd_float4) = ((c0*x + c1*y) + c2*z) + c3*w
__device__ __forceinline__ F3 mat_mul(const Mat34 &m, float4 v) {
    return mk3(((m.m[0][0] * v.x + m.m[0][1] * v.y) + m.m[0][2] * v.z) + m.m[0][3] * v.w,
               ((m.m[1][0] * v.x + m.m[1][1] * v.y) + m.m[1][2] * v.z) + m.m[1][3] * v.w,
               ((m.m[2][0] * v.x + m.m[2][1] * v.y) + m.m[2][2] * v.z) + m.m[2][3] * v.w);
}

__global__ void __launch_bounds__(256) k_vertex(const float4 *__restrict__ vtx, uint32_t nv,
                                                const float4 *__restrict__ nrm, uint32_t na, Mat34 m,
                                                float factor, float half_w, float half_h,
                                                float4 *__restrict__ cv, float4 *__restrict__ rv,
                                                float4 *__restrict__ ncam) {
    const uint32_t n = nv > na ? nv : na;
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        if (i < nv) {
            const F3 c = mat_mul(m, vtx[i]);
            const float nz = -c.z;
            cv[i] = make_float4(c.x, c.y, c.z, 0.0f);
            // (cv.x, -cv.y, 0) * factor / -cv.z + (W/2, H/2, -cv.z)   (render.cpp:288)
            rv[i] = make_float4((c.x * factor) / nz + half_w, ((-c.y) * factor) / nz + half_h,
                                (0.0f * factor) / nz + nz, 0.0f);
        }
        if (i < na) {
            const F3 r = mat_mul(m, nrm[i]);                       // render.cpp:291
            ncam[i] = make_float4(r.x, r.y, r.z, 0.0f);
        }
    }
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

// render.cpp:311-359 for one (possibly clipped) triangle.
__device__ void setup_tri(const Vert d[3], bool textured, float sw, float sh, TriSetup *out) {
    TriSetup t;
    t.kind = kDead;
    t.pad0 = t.pad1 = 0;
    const float rmx = fmaxf(fmaxf(d[0].rv.x, d[1].rv.x), d[2].rv.x);
    const float rmy = fmaxf(fmaxf(d[0].rv.y, d[1].rv.y), d[2].rv.y);
    const float rnx = fminf(fminf(d[0].rv.x, d[1].rv.x), d[2].rv.x);
    const float rny = fminf(fminf(d[0].rv.y, d[1].rv.y), d[2].rv.y);
    const float area = edge_fn(d[0].rv, d[1].rv, d[2].rv.x, d[2].rv.y);
    if (rmx < 0 || rmy < 0 || rnx >= sw || rny >= sh || area < 10) {   // :312, :314, :317
        out->kind = kDead;
        return;
    }
    const float ooa = 1 / area;
    t.xmin = u32_of_float(fmaxf(0, rnx));
    t.xmax = u32_of_float(fminf(sw - 1, rmx));
    t.ymin = u32_of_float(fmaxf(0, rny));
    t.ymax = u32_of_float(fminf(sh - 1, rmy));
    const float px = (float)t.xmin + 0.5f, py = (float)t.ymin + 0.5f;
    t.ws[0] = edge_fn(d[1].rv, d[2].rv, px, py) * ooa;
    t.ws[1] = edge_fn(d[2].rv, d[0].rv, px, py) * ooa;
    t.ws[2] = edge_fn(d[0].rv, d[1].rv, px, py) * ooa;
    t.dx[0] = (d[1].rv.y - d[2].rv.y) * ooa;
    t.dx[1] = (d[2].rv.y - d[0].rv.y) * ooa;
    t.dx[2] = (d[0].rv.y - d[1].rv.y) * ooa;
    t.dy[0] = (d[2].rv.x - d[1].rv.x) * ooa;
    t.dy[1] = (d[0].rv.x - d[2].rv.x) * ooa;
    t.dy[2] = (d[1].rv.x - d[0].rv.x) * ooa;
    t.ws[3] = t.dx[3] = t.dy[3] = t.rvz[3] = 0.0f;
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const float r = 1 / d[k].rv.z;
        t.rvz[k] = r;
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
    *out = t;
}

__global__ void __launch_bounds__(256) k_setup(const float4 *__restrict__ cvb, const float4 *__restrict__ rvb,
                                               const float4 *__restrict__ ncam, const float4 *__restrict__ pay,
                                               const uint8_t *__restrict__ disc, const uint32_t *__restrict__ vidx,
                                               const uint32_t *__restrict__ aidx, uint32_t ntri, float factor,
                                               float sw, float sh, TriSetup *__restrict__ tris) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= ntri) return;
    Vert d[3];
#pragma unroll
    for (int k = 0; k < 3; k++) {
        const uint32_t vi = vidx[3 * t + k], ai = aidx[3 * t + k];
        const float4 c = cvb[vi], r = rvb[vi], n = ncam[ai];
        d[k].cv = mk3(c.x, c.y, c.z);
        d[k].rv = mk3(r.x, r.y, r.z);
        d[k].n = mk3(n.x, n.y, n.z);
        d[k].pay = pay[ai];
    }
    const bool textured = disc[aidx[3 * t]] != 0;                        // data[0].ca.disc, :340
    tris[ntri + t].kind = kDead;
    if (fmaxf(fmaxf(d[0].rv.z, d[1].rv.z), d[2].rv.z) <= kNear) {         // :306
        tris[t].kind = kDead;
        return;
    }
    Vert app[3];
    uint32_t app_first = 0;
    bool appended = false;
    const float half_w = sw / 2, half_h = sh / 2;
    if (fminf(fminf(d[0].rv.z, d[1].rv.z), d[2].rv.z) < kNear)            // :308
        appended = clip_tri(d, app, &app_first, textured, factor, half_w, half_h);
    setup_tri(d, textured, sw, sh, &tris[t]);
    if (appended) {
        // The appended triangle is (vi[cur], new, new) with z = (z_cur > near, near, near): neither
        // the :306 reject nor another clip can trigger when the reference loop reaches it.  Its
        // data[0] is the original attribute ai[cur], whose disc picks its colour path.
        setup_tri(app, disc[aidx[3 * t + app_first]] != 0, sw, sh, &tris[ntri + t]);
    }
}

// ------------------------------------------------------------------ K4: fragment
struct ChunkRec {           // 32 B, one per (triangle lane, chunk)
    uint32_t k0;            // first pixel x of the triangle in this chunk, kInvalidK if none
    uint32_t lin;           // bit c: component c is c + k*delta across the chunk
    float c[3];             // exact barycentric value at x = k0
    float del[3];
};
struct TriInfo {            // 32 B, one per triangle lane of the batch
    float rvz[3];
    uint32_t xmax;
    float dx[3];
    uint32_t slot;
};

__device__ __forceinline__ uint32_t texel(const uint32_t *__restrict__ tex, uint32_t ntex, uint32_t base,
                                          float u, float v, float lvx, float lvy) {
    // getTextureColor, render.cpp:124-132
    const uint32_t lx = next_power_of_two(u32_of_float(fmaxf(fminf(lvx, 256.f), 1.f)));
    const uint32_t ly = next_power_of_two(u32_of_float(fmaxf(fminf(lvy, 256.f), 1.f)));
    const uint32_t x = u32_of_float(frac1(u) * (float)lx) + (511u & ~(2u * lx - 1u));
    const uint32_t y = u32_of_float(frac1(v) * (float)ly) + (511u & ~(2u * ly - 1u));
    const uint32_t off = (x + (y << 9)) & (kTexTexels - 1u);
    // Out-of-range texture index is UB in the reference; defined here (and in the oracle) as 0.
    return (base < ntex && ntex - base >= kTexTexels) ? tex[base + off] : 0u;
}

// Deferred shading of the winning triangle (render.cpp:366-371).
__device__ uint32_t shade(const TriSetup *__restrict__ tp, float w0, float w1, float w2, float ooz,
                          const uint32_t *__restrict__ tex, uint32_t ntex) {
    const float4 *q = reinterpret_cast<const float4 *>(tp);
    const uint4 hdr = reinterpret_cast<const uint4 *>(tp)[0];
    const uint4 hdr2 = reinterpret_cast<const uint4 *>(tp)[1];
    const uint32_t kind = hdr.x, tex_base = hdr2.y;
    const float4 c0 = q[6], c1 = q[7], c2 = q[8];      // cvr
    const float4 n0 = q[9], n1 = q[10], n2 = q[11];    // nr
    const float4 k0 = q[12], k1 = q[13], k2 = q[14];   // col
    const float a = w0 / ooz, b = w1 / ooz, c = w2 / ooz;
    const F3 P = mk3((c0.x * a + c1.x * b) + c2.x * c, (c0.y * a + c1.y * b) + c2.y * c,
                     (c0.z * a + c1.z * b) + c2.z * c);
    const F3 pn = fast_normalize3(P);
    const F3 point = mk3(-pn.x, -pn.y, -pn.z);
    const F3 N = mk3((n0.x * a + n1.x * b) + n2.x * c, (n0.y * a + n1.y * b) + n2.y * c,
                     (n0.z * a + n1.z * b) + n2.z * c);
    const F3 normal = fast_normalize3(N);
    const F3 halfway = fast_normalize3(add3(point, normal));
    const float s = dot3(halfway, normal);
    F3 col;
    if (kind == kColour) {
        col = mk3((k0.x * a + k1.x * b) + k2.x * c, (k0.y * a + k1.y * b) + k2.y * c,
                  (k0.z * a + k1.z * b) + k2.z * c);
    } else {
        // uv0=(k0.x,k0.y) uv1=(k0.z,k0.w) uv2=(k1.x,k1.y) dz=(k1.z,k1.w) tpp=(k2.x,k2.y)
        const float mu = (k0.x * a + k0.z * b) + k1.x * c;
        const float mv = (k0.y * a + k0.w * b) + k1.y * c;
        const float lvx = ooz / fabsf(k2.x - mu * k1.z);
        const float lvy = ooz / fabsf(k2.y - mv * k1.w);
        const uint32_t rgb = texel(tex, ntex, tex_base, mu, mv, lvx, lvy);
        col = mk3((float)(rgb >> 16), (float)((rgb >> 8) & 255u), (float)(rgb & 255u));
    }
    return rgb_pack(s * col.x, s * col.y, s * col.z);
}

template <int NCH>
__global__ void __launch_bounds__(64) k_fragment(const TriSetup *__restrict__ tris, uint32_t nslots,
                                                 const uint32_t *__restrict__ tex, uint32_t ntex,
                                                 uint32_t *__restrict__ out, uint32_t W, uint32_t H,
                                                 uint32_t band, uint32_t nparts, uint32_t part,
                                                 uint32_t segs) {
    __shared__ ChunkRec rec[64];
    __shared__ TriInfo info[64];
    const uint32_t lane = threadIdx.x;
    const uint32_t lr = blockIdx.x / segs, seg = blockIdx.x - lr * segs;
    const uint32_t y = ((lr / band) * nparts + part) * band + lr % band;   // interleaved row bands
    if (y >= H) return;
    const uint32_t xs = seg * 64u * NCH;
    const uint32_t xe = min(W, xs + 64u * NCH) - 1u;

    float depth[NCH], bw0[NCH], bw1[NCH], bw2[NCH];
    int win[NCH];
#pragma unroll
    for (int q = 0; q < NCH; q++) { depth[q] = 0.0f; win[q] = -1; bw0[q] = bw1[q] = bw2[q] = 0.0f; }

    for (uint32_t base = 0; base < nslots; base += 64u) {
        // ---- lanes as triangles
        const uint32_t s = base + lane;
        bool act = false;
        uint4 h0 = make_uint4(0, 0, 0, 0);
        uint32_t ymax = 0;
        if (s < nslots) {
            h0 = reinterpret_cast<const uint4 *>(tris + s)[0];
            ymax = reinterpret_cast<const uint4 *>(tris + s)[1].x;
            act = h0.x != kDead && y >= h0.w && y <= ymax && h0.y <= xe && h0.z >= xs;
        }
        const uint64_t mask = __ballot(act);
        if (mask == 0) continue;
        float c0 = 0, c1 = 0, c2 = 0, dx0 = 0, dx1 = 0, dx2 = 0;
        uint32_t kpos = 0;
        if (act) {
            const float4 *q = reinterpret_cast<const float4 *>(tris + s);
            const float4 ws = q[2], dx = q[3], dy = q[4], rz = q[5];
            const uint32_t j = y - h0.w;
            c0 = exact_walk(ws.x, dy.x, j);          // row start wy after j steps (render.cpp:378)
            c1 = exact_walk(ws.y, dy.y, j);
            c2 = exact_walk(ws.z, dy.z, j);
            dx0 = dx.x; dx1 = dx.y; dx2 = dx.z;
            kpos = h0.y;
            TriInfo ti;
            ti.rvz[0] = rz.x; ti.rvz[1] = rz.y; ti.rvz[2] = rz.z; ti.xmax = h0.z;
            ti.dx[0] = dx.x; ti.dx[1] = dx.y; ti.dx[2] = dx.z; ti.slot = s;
            info[lane] = ti;
        }
#pragma unroll
        for (int q = 0; q < NCH; q++) {
            const uint32_t cx0 = xs + 64u * q;
            if (cx0 > xe) break;
            const uint32_t cx1 = min(cx0 + 63u, xe);
            if (act) {
                ChunkRec r;
                r.k0 = kInvalidK;
                r.lin = 0;
                r.c[0] = r.c[1] = r.c[2] = 0.0f;
                r.del[0] = r.del[1] = r.del[2] = 0.0f;
                if (h0.y <= cx1 && h0.z >= cx0) {
                    const uint32_t k0 = max(cx0, h0.y);
                    const uint32_t m = min(cx1, h0.z) - k0 + 1u;
                    c0 = exact_walk(c0, dx0, k0 - kpos);    // pixel walk (render.cpp:374)
                    c1 = exact_walk(c1, dx1, k0 - kpos);
                    c2 = exact_walk(c2, dx2, k0 - kpos);
                    kpos = k0;
                    r.k0 = k0;
                    r.c[0] = c0; r.c[1] = c1; r.c[2] = c2;
                    r.lin = (chunk_linear(c0, dx0, m, &r.del[0]) ? 1u : 0u) |
                            (chunk_linear(c1, dx1, m, &r.del[1]) ? 2u : 0u) |
                            (chunk_linear(c2, dx2, m, &r.del[2]) ? 4u : 0u);
                }
                rec[lane] = r;
            }
            __syncthreads();
            // ---- lanes as pixels
            const uint32_t x = cx0 + lane;
            uint64_t mm = mask;
            while (mm) {
                const uint32_t t = (uint32_t)__builtin_ctzll(mm);
                mm &= mm - 1;
                const ChunkRec r = rec[t];
                if (r.k0 == kInvalidK) continue;
                const TriInfo ti = info[t];
                if (x >= r.k0 && x <= ti.xmax) {
                    const uint32_t off = x - r.k0;
                    const float fo = (float)off;
                    const float a0 = (r.lin & 1u) ? r.c[0] + fo * r.del[0] : exact_walk(r.c[0], ti.dx[0], off);
                    const float a1 = (r.lin & 2u) ? r.c[1] + fo * r.del[1] : exact_walk(r.c[1], ti.dx[1], off);
                    const float a2 = (r.lin & 4u) ? r.c[2] + fo * r.del[2] : exact_walk(r.c[2], ti.dx[2], off);
                    if (a0 >= 0 && a1 >= 0 && a2 >= 0) {                         // :362
                        const float ooz = (ti.rvz[0] * a0 + ti.rvz[1] * a1) + ti.rvz[2] * a2;   // :363
                        if (ooz > depth[q]) {                                        // :364
                            depth[q] = ooz; win[q] = (int)ti.slot;
                            bw0[q] = a0; bw1[q] = a1; bw2[q] = a2;
                        }
                    }
                }
            }
            __syncthreads();
        }
    }
    uint32_t *row = out + (size_t)lr * W;
#pragma unroll
    for (int q = 0; q < NCH; q++) {
        const uint32_t x = xs + 64u * q + lane;
        if (x <= xe) {
            row[x] = win[q] < 0 ? kBackground : shade(tris + win[q], bw0[q], bw1[q], bw2[q], depth[q], tex, ntex);
        }
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

// ------------------------------------------------------------------ launchers
constexpr int kNCH = 8;

void launch_vertex(const float4 *vtx, uint32_t nv, const float4 *nrm, uint32_t na, const Mat34 &m,
                   float factor, float sw, float sh, float4 *cv, float4 *rv, float4 *ncam, hipStream_t st) {
    const uint32_t n = nv > na ? nv : na;
    if (n == 0) return;
    uint32_t blocks = (n + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_vertex, dim3(blocks), dim3(256), 0, st, vtx, nv, nrm, na, m, factor, sw / 2,
                       sh / 2, cv, rv, ncam);
}

void launch_setup(const float4 *cv, const float4 *rv, const float4 *ncam, const float4 *pay,
                  const uint8_t *disc, const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri,
                  float factor, float sw, float sh, TriSetup *tris, hipStream_t st) {
    if (ntri == 0) return;
    hipLaunchKernelGGL(k_setup, dim3((ntri + 255) / 256), dim3(256), 0, st, cv, rv, ncam, pay, disc, vidx,
                       aidx, ntri, factor, sw, sh, tris);
}

uint32_t fragment_segment_pixels() { return 64u * kNCH; }

void launch_fragment(const TriSetup *tris, uint32_t nslots, const uint32_t *tex, uint32_t ntex, uint32_t *out,
                     uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                     hipStream_t st) {
    const uint32_t segs = (W + 64u * kNCH - 1) / (64u * kNCH);
    const uint64_t blocks = (uint64_t)rows_local * segs;
    if (blocks == 0) return;
    hipLaunchKernelGGL(k_fragment<kNCH>, dim3((uint32_t)blocks), dim3(64), 0, st, tris, nslots, tex, ntex, out,
                       W, H, band, nparts, part, segs);
}

}  // namespace s3r
