/*
 * render_oracle.c -- CPU ORACLE (test infrastructure only; never shipped, never on the product path).
 *
 * A literal, single-threaded C restatement of the reference rasterizer
 *   /root/reference/render-cpp/render.cpp   (sarastro-nl/Swift3DRenderer)
 * Every function cites the reference line range it follows. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this file's shared object.
 *
 * PARITY UNPINNED.  The reference ships no tests, fixtures or golden vectors, and
 * it cannot be built here: it needs Apple's <simd/simd.h> and Apple libc's memset_pattern4, which
 * this image does not have (no stand-in headers are written for it, by rule).  This restatement
 * therefore *defines* parity: render.cpp's operation order, with the Apple simd functions restated
 * as below and every float operation a single IEEE-754 binary32 operation (round to nearest even,
 * no FMA contraction, no fast-math, denormals kept) -- i.e. the semantics of an x86-64
 * `clang++ -O2` build of render.cpp.
 *
 * Third-party arithmetic restated (Apple simd, Apple SDK header-only library, not vendored, no
 * version pinned by the reference; call sites render.cpp:142-154, :286, :291, :349, :363-370):
 *   simd_dot(a,b)            = (a.x*b.x + a.y*b.y) + a.z*b.z
 *   simd_fast_normalize(a)   = a * (1.0f / sqrtf(simd_dot(a,a)))      (correctly rounded sqrt, div)
 *   simd_mul(M4x3, v4)       = ((c0*v.x + c1*v.y) + c2*v.z) + c3*v.w   (c_j = column j)
 *   simd_matrix_from_rows    = column j = (r0[j], r1[j], r2[j])
 *   simd_cross(a,b)          = (a.y*b.z - a.z*b.y, a.z*b.x - a.x*b.z, a.x*b.y - a.y*b.x)
 *   simd_quaternion(f,t)     = reduced form (dot(f,t) >= 0 always holds in update_camera):
 *                              h = normalize(f+t); q = (cross(f,h), dot(f,h))
 *   simd_act(q,v)            = t = 2*cross(q.im, v); v + q.re*t + cross(q.im, t)
 *   simd_abs/min/max         = lane-wise fabsf/fminf/fmaxf
 *   memset_pattern4          = 4-byte pattern fill
 * x86 conversions mirrored: (uint8_t)(float) = low byte of cvttss2si (int32 truncation);
 * (uint32_t)(float) = low 32 bits of a 64-bit truncation.
 *
 * Build: gcc -O2 -std=c11 -ffp-contract=off -fno-fast-math -fPIC -shared (oracle/Makefile).
 */
#define _GNU_SOURCE
#include <math.h>
#if ORACLE_RSQRT
#include <immintrin.h>
#endif
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ---- ABI structs: render-cpp/render.hpp:7-21 (PixelData 24 B, Input 24 B, mouse at +16) ---- */
typedef struct { uint32_t *buffer; uint32_t width, height, bytesPerPixel, bufferSize; } PixelData;
typedef struct { float x, y; } f2;
typedef struct { float up, down, left, right; f2 mouse; } Input;

typedef struct { float x, y, z; } f3;
typedef struct { float x, y, z, w; } f4;

/* ---- vector helpers: every line is one binary32 op per lane, in the order the C++ evaluates ---- */
static inline f3 v3(float x, float y, float z) { f3 r = {x, y, z}; return r; }
static inline f3 add3(f3 a, f3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline f3 sub3(f3 a, f3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline f3 mul3(f3 a, f3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline f3 muls3(f3 a, float s) { return v3(a.x * s, a.y * s, a.z * s); }
static inline f3 smul3(float s, f3 a) { return v3(s * a.x, s * a.y, s * a.z); }
static inline f3 divs3(f3 a, float s) { return v3(a.x / s, a.y / s, a.z / s); }
static inline f3 neg3(f3 a) { return v3(-a.x, -a.y, -a.z); }
static inline float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
static inline f3 cross3(f3 a, f3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
/* Sensitivity variants (tools/parity_sensitivity.py; never the parity oracle): ORACLE_RSQRT = 1
 * takes simd_fast_normalize's 1/sqrt from the hardware estimate (x86 rsqrtss, relative error
 * <= 1.5 * 2^-12), 2 adds one Newton-Raphson step -- the kind of approximation Apple's "fast"
 * variant is allowed to make (render.cpp:142-147, :367-369). */
static inline float inv_sqrt(float x) {
#if ORACLE_RSQRT
    float y = _mm_cvtss_f32(_mm_rsqrt_ss(_mm_set_ss(x)));
#if ORACLE_RSQRT == 2
    y = y * (1.5f - 0.5f * x * y * y);
#endif
    return y;
#else
    return 1.0f / sqrtf(x);
#endif
}
static inline f3 fast_normalize3(f3 a) { return muls3(a, inv_sqrt(dot3(a, a))); }
static inline f3 max3(f3 a, f3 b) { return v3(fmaxf(a.x, b.x), fmaxf(a.y, b.y), fmaxf(a.z, b.z)); }
static inline f3 min3(f3 a, f3 b) { return v3(fminf(a.x, b.x), fminf(a.y, b.y), fminf(a.z, b.z)); }
static inline f2 v2(float x, float y) { f2 r = {x, y}; return r; }
static inline f2 add2(f2 a, f2 b) { return v2(a.x + b.x, a.y + b.y); }
static inline f2 sub2(f2 a, f2 b) { return v2(a.x - b.x, a.y - b.y); }
static inline f2 mul2(f2 a, f2 b) { return v2(a.x * b.x, a.y * b.y); }
static inline f2 muls2(f2 a, float s) { return v2(a.x * s, a.y * s); }

static inline uint8_t u8_of_float(float f) { return (uint8_t)(int32_t)f; }        /* cvttss2si */
static inline uint32_t u32_of_float(float f) { return (uint32_t)(int64_t)f; }     /* cvttss2si r64 */
/* RGB macro, render.cpp:8 */
static inline uint32_t rgb_pack(float r, float g, float b) {
    return (uint32_t)((((uint32_t)u8_of_float(r) << 8) + u8_of_float(g)) << 8) + u8_of_float(b);
}
/* EDGE_FUNCTION, render.cpp:9 */
static inline float edge_fn(f3 a, f3 b, float cx, float cy) {
    return (cx - a.x) * (a.y - b.y) + (cy - a.y) * (b.x - a.x);
}

/* ---- types: render.cpp:11-36 ---- */
typedef struct { uint32_t index; uint32_t pad; f2 uv; } texture_t;  /* uv at +8 */
enum { DISC_COLOR = 0, DISC_TEXTURE = 1 };
typedef struct {
    union { float color[4]; texture_t texture; } u;                   /* 16 B */
    uint32_t disc;                                                    /* +16 */
    uint32_t pad[3];                                                  /* 32 B */
} color_attribute_t;
typedef struct { f4 normal; color_attribute_t ca; } vertex_attribute_t; /* 48 B */
typedef struct { f3 cv; f3 rv; color_attribute_t ca; f3 n; } data_t;

/* ---- static state: render.cpp:51-113 ---- */
static struct {
    f3 pos, ax, ay, az;
    float m[3][4];          /* rows */
    f2 mouse;
} state;
static float *depth_buffer;
static uint32_t depth_buffer_size;
static uint32_t *texture_buffer;
static uint64_t texel_count;
static const float cfg_near = 0.1f;
static float cfg_scale;      /* near * tan(fov/2), fov = (float)M_PI/5 */
static float cfg_factor = 1;
static const float cfg_speed = 0.1f;
static const float cfg_rotation_speed = 0.3f;
static const uint32_t cfg_background = (30u << 16) | (30u << 8) | 30u;   /* RGB(30,30,30), :96 */
static int initialized;
static char data_path[4096];

static struct {
    f4 *vertices; uint64_t vertex_count;
    uint64_t *vertex_indices; uint64_t vertex_indices_count;
    vertex_attribute_t *attributes; uint64_t attributes_count;
    uint64_t *attribute_indices; uint64_t attribute_indices_count;
    f3 *camera_vertices, *raster_vertices;
    color_attribute_t *color_attributes;
    f3 *normals;
} scene;

static void reset_state(void) {
    state.pos = v3(0, 0, 0);
    state.ax = v3(1, 0, 0); state.ay = v3(0, 1, 0); state.az = v3(0, 0, 1);
    memset(state.m, 0, sizeof state.m);
    state.m[0][0] = state.m[1][1] = state.m[2][2] = 1;
    state.mouse = v2(0, 0);
    cfg_factor = 1;
    {
        const float fov = (float)M_PI / 5.f;
#if ORACLE_TAN_DOUBLE
        /* sensitivity variant: near * tan evaluated in double, then rounded to float */
        cfg_scale = (float)((double)cfg_near * tan((double)(fov / 2)));
#else
        cfg_scale = cfg_near * tanf(fov / 2);                             /* :92 */
#endif
    }
}

/* render.cpp:115-122 */
static uint32_t next_power_of_two(uint32_t i) {
    i--; i |= i >> 1; i |= i >> 2; i |= i >> 4; return i + 1;
}

/* render.cpp:124-132 */
static f3 get_texture_color(uint64_t base, f2 uv, f2 level) {
    uint32_t lx = next_power_of_two(u32_of_float(fmaxf(fminf(level.x, 256.f), 1.f)));
    uint32_t ly = next_power_of_two(u32_of_float(fmaxf(fminf(level.y, 256.f), 1.f)));
    uint32_t x = u32_of_float(fmodf(uv.x, 1) * (float)lx) + (511u & ~(2u * lx - 1u));
    uint32_t y = u32_of_float(fmodf(uv.y, 1) * (float)ly) + (511u & ~(2u * ly - 1u));
    /* An out-of-range texel (negative uv or texture index, UB in the reference) is defined as 0
     * here and in the GPU library; with uv >= 0 and a valid index the mask is a no-op. */
    const uint32_t off = (x + (y << 9)) & ((1u << 18) - 1);
    uint32_t rgb = (base + (1u << 18) <= texel_count) ? texture_buffer[base + off] : 0;
    return v3((float)(rgb >> 16), (float)((rgb >> 8) & 255), (float)(rgb & 255));
}

/* simd_act (reduced quaternion) -- see header */
static f3 quat_act(f3 im, float re, f3 v) {
    f3 t = smul3(2.0f, cross3(im, v));
    return add3(add3(v, smul3(re, t)), cross3(im, t));
}

/* render.cpp:134-156 */
static void update_camera(const Input *in, int force) {
    int changed = 0;
    if (in->left > 0 || in->right > 0 || in->up > 0 || in->down > 0) {
        changed = 1;
        f3 mv = add3(smul3(in->right - in->left, state.ax), smul3(in->down - in->up, state.az));
        state.pos = add3(state.pos, smul3(cfg_speed, mv));
    }
    if (in->mouse.x != state.mouse.x || in->mouse.y != state.mouse.y) {
        changed = 1;
        f3 d = add3(add3(smul3(state.mouse.x - in->mouse.x, state.ax),
                         smul3(state.mouse.y - in->mouse.y, state.ay)),
                    smul3(100 / cfg_rotation_speed, state.az));
        f3 z = fast_normalize3(d);
        /* simd_quaternion(from = az, to = z), reduced form */
        f3 h = fast_normalize3(add3(state.az, z));
        f3 im = cross3(state.az, h);
        float re = dot3(state.az, h);
        state.ax = fast_normalize3(quat_act(im, re, state.ax));
        state.ay = fast_normalize3(quat_act(im, re, state.ay));
        state.az = z;
        state.mouse = in->mouse;
    }
    if (changed || force) {
        f3 r[3] = {state.ax, state.ay, state.az};
        for (int i = 0; i < 3; i++) {
            state.m[i][0] = r[i].x; state.m[i][1] = r[i].y; state.m[i][2] = r[i].z;
            state.m[i][3] = -dot3(r[i], state.pos);
        }
    }
}

/* simd_mul(simd_float4x3, simd_float4): ((c0*x + c1*y) + c2*z) + c3*w */
static f3 mat_mul(const float m[3][4], f4 v) {
    f3 r;
    r.x = ((m[0][0] * v.x + m[0][1] * v.y) + m[0][2] * v.z) + m[0][3] * v.w;
    r.y = ((m[1][0] * v.x + m[1][1] * v.y) + m[1][2] * v.z) + m[1][3] * v.w;
    r.z = ((m[2][0] * v.x + m[2][1] * v.y) + m[2][2] * v.z) + m[2][3] * v.w;
    return r;
}

static int read_exact(void *dst, size_t sz, size_t n, FILE *fp) {
    return fread(dst, sz, n, fp) == n;
}

/* render.cpp:160-210 (path search replaced by an explicit path; see oracle_set_data_path) */
static int initialize(void) {
    FILE *fp = fopen(data_path, "rb");
    if (!fp) return -1;
    uint64_t count[2];
    if (!read_exact(count, 8, 2, fp)) goto bad;
    scene.vertex_count = count[0];
    scene.vertices = malloc(count[0] * sizeof(f4) + 16);
    if (!read_exact(scene.vertices, sizeof(f4), count[0], fp)) goto bad;
    uint64_t nv = count[0];

    if (!read_exact(count, 8, 2, fp)) goto bad;
    scene.vertex_indices_count = count[0];
    uint64_t aligned = count[0] + (count[0] % 2);
    scene.vertex_indices = malloc(2 * aligned * sizeof(uint64_t) + 16);
    if (!read_exact(scene.vertex_indices, 8, aligned, fp)) goto bad;
    /* The reference sizes these scratch arrays at 2x (render.cpp:182-183, :195-196), which a scene
     * where more than V/2 triangles are split by clip() would overflow (UB there). The oracle sizes
     * them for the worst case (2 appended per triangle) so every scene is defined. */
    uint64_t tri = count[0] / 3;
    scene.camera_vertices = malloc((2 * nv + 2 * tri + 2) * sizeof(f3));
    scene.raster_vertices = malloc((2 * nv + 2 * tri + 2) * sizeof(f3));

    if (!read_exact(count, 8, 2, fp)) goto bad;
    scene.attributes_count = count[0];
    scene.attributes = malloc(count[0] * sizeof(vertex_attribute_t) + 16);
    if (!read_exact(scene.attributes, sizeof(vertex_attribute_t), count[0], fp)) goto bad;
    scene.color_attributes = malloc((2 * count[0] + 2 * tri + 2) * sizeof(color_attribute_t));
    scene.normals = malloc((2 * count[0] + 2 * tri + 2) * sizeof(f3));
    for (uint64_t i = 0; i < scene.attributes_count; i++) scene.color_attributes[i] = scene.attributes[i].ca;

    if (!read_exact(count, 8, 2, fp)) goto bad;
    scene.attribute_indices_count = count[0];
    aligned = count[0] + (count[0] % 2);
    scene.attribute_indices = malloc(2 * aligned * sizeof(uint64_t) + 16);
    if (!read_exact(scene.attribute_indices, 8, aligned, fp)) goto bad;

    if (!read_exact(count, 8, 2, fp)) goto bad;
    texel_count = count[0];
    texture_buffer = malloc(count[0] * sizeof(uint32_t) + 16);
    if (!read_exact(texture_buffer, 4, count[0], fp)) goto bad;
    fclose(fp);
    return 0;
bad:
    fclose(fp);
    return -2;
}

/* render.cpp:212-262 */
static void clip(data_t *data, uint64_t *v_count, uint64_t *a_count, uint64_t *vi_count,
                 const uint64_t *vi, const uint64_t *ai, f2 screen) {
    data_t data_new[3];
    memset(data_new, 0, sizeof data_new);
    uint64_t vi_current = 0, vi_next = 0, vi_preceding = 0;
    int new_triangle = 0;
    for (uint32_t i = 0; i < 3; i++) {
        uint32_t in = (i + 1) % 3;
        if ((data[i].rv.z > cfg_near) == (data[in].rv.z > cfg_near)) {
            vi_current = i; vi_next = in; vi_preceding = (i + 2) % 3;
            new_triangle = data[i].rv.z > cfg_near;
        } else {
            float a = (cfg_near - data[i].rv.z) / (data[in].rv.z - data[i].rv.z);
            f3 cv = add3(muls3(data[i].cv, 1 - a), muls3(data[in].cv, a));
            f3 rv = add3(divs3(muls3(v3(cv.x, -cv.y, 0), cfg_factor), cfg_near),
                         v3(screen.x / 2, screen.y / 2, cfg_near));
            color_attribute_t ca;
            memset(&ca, 0, sizeof ca);
            ca.disc = data[0].ca.disc;
            if (ca.disc == DISC_COLOR) {
                for (int k = 0; k < 3; k++)
                    ca.u.color[k] = data[i].ca.u.color[k] * (1 - a) + data[in].ca.u.color[k] * a;
            } else {
                texture_t t1 = data[i].ca.u.texture, t2 = data[in].ca.u.texture;
                ca.u.texture.index = t1.index;
                ca.u.texture.uv = add2(muls2(t1.uv, 1 - a), muls2(t2.uv, a));
            }
            f3 n = add3(muls3(data[i].n, 1 - a), muls3(data[in].n, a));
            data_new[i].cv = cv; data_new[i].rv = rv; data_new[i].ca = ca; data_new[i].n = n;
        }
    }
    if (new_triangle) {
        data[vi_preceding] = data_new[vi_next];
        scene.camera_vertices[*v_count] = data_new[vi_next].cv;
        scene.raster_vertices[*v_count] = data_new[vi_next].rv;
        scene.color_attributes[*a_count] = data_new[vi_next].ca;
        scene.normals[*a_count] = data_new[vi_next].n;
        scene.camera_vertices[*v_count + 1] = data_new[vi_preceding].cv;
        scene.raster_vertices[*v_count + 1] = data_new[vi_preceding].rv;
        scene.color_attributes[*a_count + 1] = data_new[vi_preceding].ca;
        scene.normals[*a_count + 1] = data_new[vi_preceding].n;
        scene.vertex_indices[*vi_count] = vi[vi_current];
        scene.vertex_indices[*vi_count + 1] = *v_count;
        scene.vertex_indices[*vi_count + 2] = *v_count + 1;
        scene.attribute_indices[*vi_count] = ai[vi_current];
        scene.attribute_indices[*vi_count + 1] = *a_count;
        scene.attribute_indices[*vi_count + 2] = *a_count + 1;
        *v_count += 2; *a_count += 2; *vi_count += 3;
    } else {
        data[vi_current] = data_new[vi_preceding];
        data[vi_next] = data_new[vi_next];
    }
}

/* Test extension (not in the reference): with row windows set, rows outside every window are still
 * walked -- wy += dy once per row (render.cpp:378), exactly as the loop below does -- but not
 * rasterised, so a full-size frame (the 20 M-triangle stress scene) can be checked on a few rows in
 * seconds.  A row's pixels depend only on its walk state, so the windows' rows are the reference's. */
#define ORACLE_MAX_WINDOWS 32
static uint32_t win_count = 0, win_rows[2 * ORACLE_MAX_WINDOWS];
static int row_in_windows(uint32_t y) {
    if (!win_count) return 1;
    for (uint32_t i = 0; i < win_count; i++)
        if (y >= win_rows[2 * i] && y < win_rows[2 * i + 1]) return 1;
    return 0;
}

/* render.cpp:264-384 */
static void render_frame(const PixelData *pd, const Input *in) {
    if (!initialized) {
        initialized = 1;
        if (initialize() != 0) { fprintf(stderr, "oracle: data.bin not found: %s\n", data_path); exit(666); }
        update_camera(in, 1);
    } else {
        update_camera(in, 0);
    }
    const uint32_t dbs = pd->width * pd->height * (uint32_t)sizeof(float);
    if (depth_buffer_size != dbs) {
        depth_buffer_size = dbs;
        depth_buffer = realloc(depth_buffer, dbs);
        cfg_factor = cfg_near * (float)pd->height / (2 * cfg_scale);     /* :279 */
    }
    memset(depth_buffer, 0, depth_buffer_size);
    for (uint32_t i = 0; i < pd->bufferSize / 4; i++) pd->buffer[i] = cfg_background;

    const f2 screen = v2((float)pd->width, (float)pd->height);
    for (uint32_t i = 0; i < scene.vertex_count; i++) {                  /* :285-289 */
        f3 v = mat_mul(state.m, scene.vertices[i]);
        scene.camera_vertices[i] = v;
        scene.raster_vertices[i] = add3(divs3(muls3(v3(v.x, -v.y, 0), cfg_factor), -v.z),
                                        v3(screen.x / 2, screen.y / 2, -v.z));
    }
    for (uint32_t i = 0; i < scene.attributes_count; i++)                 /* :290-292 */
        scene.normals[i] = mat_mul(state.m, scene.attributes[i].normal);

    uint64_t vic = scene.vertex_indices_count, vc = scene.vertex_count, ac = scene.attributes_count;
    for (uint32_t index = 0; index < vic; index += 3) {                  /* :297 */
        const uint64_t vi[3] = {scene.vertex_indices[index], scene.vertex_indices[index + 1],
                                scene.vertex_indices[index + 2]};
        const uint64_t ai[3] = {scene.attribute_indices[index], scene.attribute_indices[index + 1],
                                scene.attribute_indices[index + 2]};
        data_t data[3];
        for (int k = 0; k < 3; k++) {
            data[k].cv = scene.camera_vertices[vi[k]];
            data[k].rv = scene.raster_vertices[vi[k]];
            data[k].ca = scene.color_attributes[ai[k]];
            data[k].n = scene.normals[ai[k]];
        }
        if (fmaxf(fmaxf(data[0].rv.z, data[1].rv.z), data[2].rv.z) <= cfg_near) continue;   /* :306 */
        if (fminf(fminf(data[0].rv.z, data[1].rv.z), data[2].rv.z) < cfg_near)              /* :308 */
            clip(data, &vc, &ac, &vic, vi, ai, screen);
        const f3 rvmax = max3(max3(data[0].rv, data[1].rv), data[2].rv);
        if (rvmax.x < 0 || rvmax.y < 0) continue;
        const f3 rvmin = min3(min3(data[0].rv, data[1].rv), data[2].rv);
        if (rvmin.x >= screen.x || rvmin.y >= screen.y) continue;
        const float area = edge_fn(data[0].rv, data[1].rv, data[2].rv.x, data[2].rv.y);
        if (area < 10) continue;                                          /* :317 */
        const float ooa = 1 / area;
        const uint32_t xmin = u32_of_float(fmaxf(0, rvmin.x));
        const uint32_t xmax = u32_of_float(fminf(screen.x - 1, rvmax.x));
        const uint32_t ymin = u32_of_float(fmaxf(0, rvmin.y));
        const uint32_t ymax = u32_of_float(fminf(screen.y - 1, rvmax.y));
        const float px = (float)xmin + 0.5f, py = (float)ymin + 0.5f;
        f3 w = muls3(v3(edge_fn(data[1].rv, data[2].rv, px, py), edge_fn(data[2].rv, data[0].rv, px, py),
                        edge_fn(data[0].rv, data[1].rv, px, py)), ooa);
        f3 wy = w;
        const f3 dx = muls3(v3(data[1].rv.y - data[2].rv.y, data[2].rv.y - data[0].rv.y,
                               data[0].rv.y - data[1].rv.y), ooa);
        const f3 dy = muls3(v3(data[2].rv.x - data[1].rv.x, data[0].rv.x - data[2].rv.x,
                               data[1].rv.x - data[0].rv.x), ooa);
        const uint32_t start = ymin * pd->width + xmin;
        uint32_t *pb = pd->buffer + start;
        float *db = depth_buffer + start;
        const uint32_t xdelta = pd->width - xmax + xmin - 1;

        const f3 rvz = v3(1 / data[0].rv.z, 1 / data[1].rv.z, 1 / data[2].rv.z);
        const f3 cv[3] = {muls3(data[0].cv, rvz.x), muls3(data[1].cv, rvz.y), muls3(data[2].cv, rvz.z)};
        const f3 nn[3] = {muls3(data[0].n, rvz.x), muls3(data[1].n, rvz.y), muls3(data[2].n, rvz.z)};
        const int textured = data[0].ca.disc != DISC_COLOR;
        f3 cc[3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
        f2 uv[3] = {{0, 0}, {0, 0}, {0, 0}}, dz = v2(0, 0), tpp = v2(0, 0);
        uint64_t tbase = 0;
        if (!textured) {
            for (int k = 0; k < 3; k++) {
                const float r = k == 0 ? rvz.x : (k == 1 ? rvz.y : rvz.z);
                cc[k] = muls3(v3(data[k].ca.u.color[0], data[k].ca.u.color[1], data[k].ca.u.color[2]), r);
            }
        } else {
            tbase = (uint32_t)((int32_t)data[0].ca.u.texture.index << 18);                 /* :347 */
            uv[0] = muls2(data[0].ca.u.texture.uv, rvz.x);
            uv[1] = muls2(data[1].ca.u.texture.uv, rvz.y);
            uv[2] = muls2(data[2].ca.u.texture.uv, rvz.z);
            dz = v2(dot3(rvz, dx), dot3(rvz, dy));
            tpp = add2(add2(mul2(uv[0], v2(dx.x, dy.x)), mul2(uv[1], v2(dx.y, dy.y))), mul2(uv[2], v2(dx.z, dy.z)));
        }
        for (uint32_t y = ymin; y <= ymax; y++) {                          /* :360-382 */
            if (!row_in_windows(y)) {                                      /* (test extension) */
                pb += xmax - xmin + 1; db += xmax - xmin + 1;
                wy = add3(wy, dy);
                w = wy;
                pb += xdelta; db += xdelta;
                continue;
            }
            for (uint32_t x = xmin; x <= xmax; x++) {
                if (w.x >= 0 && w.y >= 0 && w.z >= 0) {
                    const float ooz = dot3(rvz, w);
                    if (ooz > *db) {
                        *db = ooz;
                        const f3 ww = divs3(w, ooz);
                        const f3 point = neg3(fast_normalize3(
                            add3(add3(muls3(cv[0], ww.x), muls3(cv[1], ww.y)), muls3(cv[2], ww.z))));
                        const f3 normal = fast_normalize3(
                            add3(add3(muls3(nn[0], ww.x), muls3(nn[1], ww.y)), muls3(nn[2], ww.z)));
                        const f3 halfway = fast_normalize3(add3(point, normal));
                        f3 col;
                        if (!textured) {
                            col = add3(add3(muls3(cc[0], ww.x), muls3(cc[1], ww.y)), muls3(cc[2], ww.z));
                        } else {
                            const f2 mapping = add2(add2(muls2(uv[0], ww.x), muls2(uv[1], ww.y)), muls2(uv[2], ww.z));
                            const f2 q = sub2(tpp, mul2(mapping, dz));
                            const f2 level = v2(ooz / fabsf(q.x), ooz / fabsf(q.y));
                            col = get_texture_color(tbase, mapping, level);
                        }
                        const f3 s = smul3(dot3(halfway, normal), col);
                        *pb = rgb_pack(s.x, s.y, s.z);
                    }
                }
                w = add3(w, dx);
                pb++; db++;
            }
            wy = add3(wy, dy);
            w = wy;
            pb += xdelta; db += xdelta;
        }
    }
}

static void free_scene(void) {
    free(scene.vertices); free(scene.vertex_indices); free(scene.attributes); free(scene.attribute_indices);
    free(scene.camera_vertices); free(scene.raster_vertices); free(scene.color_attributes); free(scene.normals);
    free(texture_buffer); free(depth_buffer);
    memset(&scene, 0, sizeof scene);
    texture_buffer = NULL; depth_buffer = NULL; depth_buffer_size = 0;
}

/* ---------------- exported oracle interface (test infrastructure) ---------------- */
void oracle_set_data_path(const char *path) {
    free_scene();
    win_count = 0;
    initialized = 0;
    reset_state();
    strncpy(data_path, path, sizeof data_path - 1);
    data_path[sizeof data_path - 1] = 0;
}

/* Same contract as the reference's updateAndRender (render.cpp:264-265). */
void oracle_updateAndRender(const PixelData *pixel_data, const Input *input) {
    if (cfg_scale == 0) reset_state();
    render_frame(pixel_data, input);
}

/* Row windows [rows[2i], rows[2i+1]), i < n (n <= 32; n = 0: every row) -- see row_in_windows. */
int oracle_set_row_windows(const uint32_t *rows, uint32_t n) {
    if (n > ORACLE_MAX_WINDOWS) return -1;
    for (uint32_t i = 0; i < 2 * n; i++) win_rows[i] = rows[i];
    win_count = n;
    return 0;
}

/* Debug view of the camera matrix (rows), for host-logic tests. */
void oracle_camera_matrix(float out[12]) { memcpy(out, state.m, sizeof state.m); }
float oracle_factor(void) { return cfg_factor; }
float oracle_scale(void) { if (cfg_scale == 0) reset_state(); return cfg_scale; }

/* Exact sequential float32 walk: s_{k+1} = fl(s_k + d), n times (render.cpp:374-379). */
float oracle_repeat_add(float s, float d, uint32_t n) {
    for (uint32_t k = 0; k < n; k++) s = s + d;
    return s;
}
