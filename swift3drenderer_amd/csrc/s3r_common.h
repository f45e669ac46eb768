// s3r_common.h -- types and exact float32 arithmetic shared by the host shim and the gfx950 kernels.
//
// Reference: /root/reference/render-cpp/render.cpp (sarastro-nl/Swift3DRenderer).  Every float
// operation here is ONE IEEE binary32 op in the order render.cpp evaluates it; the library is built
// with -ffp-contract=off and without fast-math so hipcc emits no FMA and keeps IEEE div/sqrt.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define S3R_HD __host__ __device__ __forceinline__

namespace s3r {

constexpr float kNear = 0.1f;                                  // render.cpp:90
constexpr float kSpeed = 0.1f;                                 // render.cpp:94
constexpr float kRotationSpeed = 0.3f;                         // render.cpp:95
constexpr uint32_t kBackground = (30u << 16) | (30u << 8) | 30u;  // RGB(30,30,30), render.cpp:96
constexpr uint32_t kTexTexels = 1u << 18;                      // 512 x 512 per texture, render.cpp:347
constexpr uint32_t kInvalidK = 0xFFFFFFFFu;

enum : uint32_t { kDead = 0, kColour = 1, kTexture = 2 };

// One triangle after gather / clip / cull / raster setup (render.cpp:297-359).  The frame's
// triangle list has 2T slots: slot t = original triangle t, slot T+t = the triangle clip() appended
// while processing t (render.cpp:239-257).  Slot order == the reference's processing order, which
// decides depth ties (strict '>' at render.cpp:364).
struct alignas(16) TriSetup {
    uint32_t kind, xmin, xmax, ymin;
    uint32_t ymax, tex_base, pad0, pad1;
    float ws[4];     // wstart (render.cpp:324)
    float dx[4];     // per-pixel step (render.cpp:327)
    float dy[4];     // per-row step (render.cpp:328)
    float rvz[4];    // 1/z per vertex (render.cpp:336)
    float cvr[12];   // cv_i * rvz_i, 3 x float4 (render.cpp:337)
    float nr[12];    // n_i * rvz_i (render.cpp:338)
    float col[12];   // colour: cc_i (render.cpp:342);  texture: uv0 uv1 | uv2 dz | tpp (render.cpp:348-352)
};
static_assert(sizeof(TriSetup) == 240, "TriSetup layout");

// Camera matrix as rows (simd_matrix_from_rows, render.cpp:152-154).
struct Mat34 { float m[3][4]; };

S3R_HD uint32_t f2u(float x) { return __builtin_bit_cast(uint32_t, x); }
S3R_HD float u2f(uint32_t x) { return __builtin_bit_cast(float, x); }
S3R_HD uint32_t fexp(float x) { return (f2u(x) >> 23) & 0xFFu; }
S3R_HD float pow2_biased(uint32_t e) { return u2f(e << 23); }   // 2^(e-127), e in [1, 254]
S3R_HD bool is_finite(float x) { return fexp(x) != 0xFFu; }

S3R_HD float quot_approx(float num, float den) {
#if defined(__HIP_DEVICE_COMPILE__)
    return num * __builtin_amdgcn_rcpf(den);   // ~1 ulp; every use below is re-checked exactly
#else
    return num / den;
#endif
}

// Regular steps available from s inside its binade [2^(e-127), 2^(e-126)) with steady step delta:
// the number of j >= 0 whose input s_j = s + j*delta still rounds on this binade's grid u, i.e.
// |s_j| + |d| < 2^(e-126) moving away from zero, |s_j| - |d| >= 2^(e-127) moving towards it.  In
// units of u every quantity is an integer below 2^24 (|d| need not be), so floats hold them exactly:
// with A = |delta|/u, D = |d|/u, the bound on j*A is N = T - floor(D) - 1 (away; T = edge distance)
// or N = L - ceil(D) (towards; L = distance to the lower edge); the count is floor(N/A) + 1.
S3R_HD float regular_steps(float s, float d, float delta, uint32_t e) {
    const float inv_u = pow2_biased(277u - e);          // 1/u = 2^(150 - e): biased exponent 277 - e
    const float as = fabsf(s);
    const float A = fabsf(delta) * inv_u;
    const float D = fabsf(d) * inv_u;
    const bool away = (s > 0.0f) == (delta > 0.0f);
    const float n_away = (pow2_biased(e + 1u) - as) * inv_u - floorf(D) - 1.0f;
    const float n_towards = (as - pow2_biased(e)) * inv_u - ceilf(D);
    const float N = away ? n_away : n_towards;
    float q = floorf(quot_approx(N, A));                  // ~1 ulp; corrected exactly below
    q = q * A > N ? q - 1.0f : q;
    q = q * A > N ? q - 1.0f : q;
    q = (q + 1.0f) * A <= N ? q + 1.0f : q;
    return N >= 0.0f ? q + 1.0f : 0.0f;                  // (NaN for out-of-range e: never selected)
}

// exact_walk(s, d, n) == the float32 value after n sequential steps s = fl(s + d)
// (render.cpp:374 `weight.w += weight.dx`, :378 `weight.wy += weight.dy`), in O(binades) work.
//
// Inside one binade every sum s + d rounds onto the grid u, and the step fl(s + d) - s is the same
// for every s there (for a d exactly half-way between grid points the tie-to-even parity settles
// after at most one step).  Once two consecutive steps are equal and in the binade, all
// regular_steps() steps up to the binade edge are s + j*delta (exact); one ordinary add then
// crosses the edge -- one loop iteration per binade.  Near zero (|s| < 8|d|, where binades hold
// too few steps to jump) the walk takes the reference's own single adds in a tight inner loop; a
// monotone walk passes that zone at most once.  Validated against the sequential loop on host and
// device (tests/test_exact_walk.py).
S3R_HD float exact_walk(float s, float d, uint32_t n, uint32_t *iters = nullptr) {
    if (n == 0) return s;
    const float ad = fabsf(d);
    if (ad == 0.0f || !is_finite(s) || !is_finite(d)) return s + d;   // one add is a fixed point
    const float ad8 = 8.0f * ad;
    for (;;) {
        while ((n != 0u) & (fabsf(s) < ad8)) {   // near zero: single steps
            if (iters) ++*iters;
            s = s + d;
            n--;
        }
        if (n == 0u) break;
        if (iters) ++*iters;
        const uint32_t e = fexp(s);
        const float s1 = s + d;
        const float s2 = s1 + d;
        const float delta = s1 - s;           // exact whenever `steady`
        // non-short-circuit '&' keeps hipcc from turning the test into nested branches
        const bool steady = (e >= 32u) & (e < 254u) & (fexp(s1) == e) & (fexp(s2) == e) & (delta == s2 - s1);
        if (steady & (delta == 0.0f)) break;  // fl(s + d) == s: stagnated for good
        // steady: j regular steps (exact: lands on the grid, at most on the edge), then one add
        // across the edge; otherwise (a tie-to-even step, a non-finite value) one single add
        const float j = steady ? fminf(regular_steps(s, d, delta, e), (float)n) : 0.0f;
        s = steady ? s + j * delta : s;
        n -= (uint32_t)j;
        if (n != 0u) {
            s = s + d;
            n--;
        }
    }
    return s;
}

// exact_walk for walks that are usually short (small triangles): up to kSeqWalk steps are the
// reference's own sequential adds (one add per step; exact_walk would single-step them anyway near
// zero and across binades, at ~40 instructions a step), longer walks jump.
constexpr uint32_t kSeqWalk = 48;
S3R_HD float short_walk(float s, float d, uint32_t n) {
    if (n > kSeqWalk) return exact_walk(s, d, n);
    for (uint32_t i = 0; i < n; i++) s = s + d;
    return s;
}

// Length of the linear run starting at c: the largest j such that S(c, d, k) == c + k*delta for
// every k <= j (0: not even one regular step; +inf: the walk has stagnated, delta == 0).
S3R_HD float linear_run(float c, float d, float *delta) {
    *delta = 0.0f;
    const float ad = fabsf(d);
    if (!is_finite(c) || !is_finite(d)) return 0.0f;
    if (ad == 0.0f) return c != 0.0f ? __builtin_inff() : 0.0f;   // c + 0 == c unless c is -0
    const float ac = fabsf(c);
    const bool towards_zero = (c < 0.0f) != (d < 0.0f);
    const float s1 = c + d, s2 = s1 + d;
    const uint32_t e = fexp(c);
    const float del = s1 - c;
    const bool steady = (ac >= 4.0f * ad) & !(towards_zero & (ac < 8.0f * ad)) & (e >= 32u) & (e < 254u) &
                        (fexp(s1) == e) & (fexp(s2) == e) & (del == s2 - s1);
    *delta = steady ? del : 0.0f;
    const float j = del == 0.0f ? __builtin_inff() : regular_steps(c, d, del, e);
    return steady ? j : 0.0f;
}

// True when the m values S(c, d, k), k = 0..m-1, are exactly c + k*delta (one binade, constant
// step); *delta receives the step.  This is exact_walk's jump test applied to a chunk of m pixels.
S3R_HD bool chunk_linear(float c, float d, uint32_t m, float *delta) {
    *delta = 0.0f;
    if (m <= 1u) return true;
    const float ad = fabsf(d);
    if (!is_finite(c) || !is_finite(d)) return false;
    if (ad == 0.0f) return c != 0.0f;                     // c + 0 == c unless c is -0
    const float ac = fabsf(c);
    const bool towards_zero = (c < 0.0f) != (d < 0.0f);
    const float s1 = c + d, s2 = s1 + d;
    const uint32_t e = fexp(c);
    const float del = s1 - c;
    const bool steady = (ac >= 4.0f * ad) & !(towards_zero & (ac < 8.0f * ad)) & (e >= 32u) & (e < 254u) &
                        (fexp(s1) == e) & (fexp(s2) == e) & (del == s2 - s1);
    *delta = steady ? del : 0.0f;
    // m-1 regular steps reach the chunk end (or the walk has stagnated: del == 0)
    return steady & ((del == 0.0f) | (regular_steps(c, d, del, e) >= (float)(m - 1u)));
}

// ---- float3 helpers in the reference's evaluation order ----
struct F3 { float x, y, z; };
S3R_HD F3 mk3(float x, float y, float z) { return F3{x, y, z}; }
S3R_HD F3 add3(F3 a, F3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
S3R_HD F3 muls3(F3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
S3R_HD float dot3(F3 a, F3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }   // simd_dot
S3R_HD F3 fast_normalize3(F3 a) { return muls3(a, 1.0f / sqrtf(dot3(a, a))); }  // simd_fast_normalize

// ---- correctly rounded division and sqrt without the range-scaling steps (device) ----
// hipcc expands IEEE a / b on gfx950 as v_div_scale (x2), v_rcp, one Newton step for 1/b, q = a*r,
// two fma residual corrections, v_div_fmas, v_div_fixup; and sqrtf(x) as a range scale, v_sqrt, the
// +-1 ulp candidates tested by fma residuals, an unscale and a special-value select.  Inside the
// ranges below every scaling step is the identity (v_div_scale returns its operand with VCC = 0,
// v_div_fmas is a plain fma, v_div_fixup passes a finite normal quotient through; x >= 2^-96 skips the
// sqrt scale), so the trimmed sequences return the same bits as the full ones: correctly rounded.
// Callers test the range and take the ordinary operator outside it.  Checked exhaustively (sqrt,
// reciprocal) and on random pairs (quotients) against the compiler's operators on the device
// (tests/test_exact_walk.py::test_fast_div_sqrt_device).  (The host compilation pass sees plain
// operators in place of the gfx950 builtins; these are never run on the host.)
#if defined(__HIP_DEVICE_COMPILE__)
#define S3R_RCP(x) __builtin_amdgcn_rcpf(x)
#define S3R_SQRT(x) __builtin_amdgcn_sqrtf(x)
#else
#define S3R_RCP(x) (1.0f / (x))
#define S3R_SQRT(x) sqrtf(x)
#endif
// biased exponents of a and b in [32, 222], |ea - eb| <= 64: no scaling anywhere (a = +-0 is out of
// range: the residual corrections would lose the sign of a -0 quotient)
__device__ __forceinline__ bool div_in_range(float a, float b) {
    const int ea = (int)fexp(a), eb = (int)fexp(b);
    return ((unsigned)(ea - 32) <= 190u) & ((unsigned)(eb - 32) <= 190u) & ((unsigned)(ea - eb + 64) <= 128u);
}
// refined reciprocal of the v_rcp + Newton step (the r the division sequence uses)
__device__ __forceinline__ float div_recip(float b) {
    const float r = S3R_RCP(b);
    const float e = __builtin_fmaf(-b, r, 1.0f);
    return __builtin_fmaf(e, r, r);
}
// a / b from the refined reciprocal r of b (div_in_range(a, b))
__device__ __forceinline__ float div_with_recip(float a, float b, float r) {
    const float q0 = a * r;
    const float q1 = __builtin_fmaf(__builtin_fmaf(-b, q0, a), r, q0);
    return __builtin_fmaf(__builtin_fmaf(-b, q1, a), r, q1);
}
// sqrtf(x) for x in [2^-96, 2^127): the v_sqrt result corrected by its fma residuals
__device__ __forceinline__ float sqrt_in_range(float x) {
    const float s = S3R_SQRT(x);
    const float sm = u2f(f2u(s) - 1u), sp = u2f(f2u(s) + 1u);
    const float rm = __builtin_fmaf(-sm, s, x), rp = __builtin_fmaf(-sp, s, x);
    const float t = rm <= 0.0f ? sm : s;
    return rp > 0.0f ? sp : t;
}
__device__ __forceinline__ bool sqrt_in_range_ok(float x) { return x >= 0x1p-96f && x < 0x1p127f; }

// simd_fast_normalize(a) = a * (1 / sqrtf(dot(a, a))), exactly, with the trimmed sequences
__device__ __forceinline__ F3 fast_normalize3_dev(F3 a) {
    const float d = dot3(a, a);
    float inv;
    if (sqrt_in_range_ok(d)) {                   // sqrt in [2^-48, 2^63.5): 1/s in range as well
        const float s = sqrt_in_range(d);
        inv = div_with_recip(1.0f, s, div_recip(s));
    } else {
        inv = 1.0f / sqrtf(d);
    }
    return mk3(a.x * inv, a.y * inv, a.z * inv);
}

// (uint8_t)(float) as x86 computes it: cvttss2si to int32 (0x80000000 when out of range or NaN),
// then the low byte (render.cpp:8 RGB macro).
S3R_HD uint32_t u8_of_float(float f) {
    const int32_t i = (fabsf(f) < 2147483648.0f) ? (int32_t)f : (int32_t)0x80000000;
    return (uint32_t)i & 0xFFu;
}
S3R_HD uint32_t rgb_pack(float r, float g, float b) {
    return (u8_of_float(r) << 16) + (u8_of_float(g) << 8) + u8_of_float(b);
}
// (uint32_t)(float) for |f| < 2^31 (render.cpp:126-129, :319-322): truncation, low 32 bits.
S3R_HD uint32_t u32_of_float(float f) {
    return (fabsf(f) < 2147483648.0f) ? (uint32_t)(int32_t)f : 0u;
}
// render.cpp:115-122
S3R_HD uint32_t next_power_of_two(uint32_t i) {
    i--; i |= i >> 1; i |= i >> 2; i |= i >> 4; return i + 1;
}
// fmodf(x, 1) for the ripmap (render.cpp:128-129): x - trunc(x) is exact for every finite x.
S3R_HD float frac1(float x) { return x - truncf(x); }

}  // namespace s3r
