// render_api.cpp -- the C-ABI shim: what render.cpp's host side did, with the per-pixel work moved
// to the gfx950 kernels (kernels.hip).
//
//   updateAndRender   render.cpp:264-384   lazy init, camera update, resize, frame, copy-out
//   initialize        render.cpp:160-210   data.bin search next to the library (dladdr), load, upload
//   update_camera     render.cpp:134-156   host float32, same operation order as the reference
//
// State is process-global like the reference's statics (render.cpp:51-113); calls are expected from
// one thread at a time (main.swift calls from its main-thread timer only).
#include <dlfcn.h>
#include <limits.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <vector>

#include "../../include/render.h"
#include "s3r_kernels.h"

using namespace s3r;

#define HIPCHECK(x)                                                                                   \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "s3r: HIP error %s at %s:%d: %s\n", hipGetErrorName(e_), __FILE__,        \
                    __LINE__, #x);                                                                    \
            abort();                                                                                  \
        }                                                                                             \
    } while (0)

namespace {

struct TimingSlot { hipEvent_t frame0, frag0, frag1; };

// Per-frame buffer sets in flight: frame k's geometry writes set k % kSets once the fragment kernel
// of frame k - kSets (the set's last reader) is done, on geometry stream k % kGeoStreams, so the
// geometry of two consecutive frames and the previous frame's fragment kernel can all overlap.
constexpr int kSets = 4;
#ifndef S3R_GEO_STREAMS
#define S3R_GEO_STREAMS 2
#endif
constexpr int kGeoStreams = S3R_GEO_STREAMS;
constexpr uint64_t kLptMinBins = 4000;      // longest-first fragment order from this many bins (~3 rounds; see render_core)

struct Lib {
    bool initialized = false;
    std::string data_path;     // "" = reference search
    int device = -1;

    // camera state, render.cpp:51-65
    F3 pos{0, 0, 0}, ax{1, 0, 0}, ay{0, 1, 0}, az{0, 0, 1};
    Mat34 m{{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}}};
    float mouse[2] = {0, 0};
    // config, render.cpp:81-97
    float factor = 1;
    uint32_t depth_buffer_size = 0;

    // scene on the device
    uint32_t nv = 0, na = 0, ntri = 0, ntex = 0;
    uint64_t nindices = 0;
    float4 *vtx = nullptr, *nrm = nullptr, *pay = nullptr;
    uint8_t *disc = nullptr;
    uint32_t *vidx = nullptr, *aidx = nullptr, *tex = nullptr;
    // per-frame geometry, double-buffered: frame k's geometry (k_geometry on stream `geo`) overlaps
    // frame k-1's fragment kernel on the caller's stream
    TriSetup *tris[kSets] = {};
    float *rowtab[kSets] = {};     // 2T x rows x (segments + 1) x float4 exact row starts
    size_t rowtab_cap = 0;
    uint32_t *bincnt[kSets] = {};            // per fragment workgroup (bin): pair count (s3r_kernels.h)
    uint4 *pairs[kSets] = {};                // per bin: kPairMax pair records (s3r_kernels.h)
    uint64_t bins_cap = 0;
    // longest-first fragment order, per buffer set: [perm | cost] (s3r_kernels.h launch_fragment)
    uint32_t *order[kSets] = {};
    uint64_t order_cap = 0;
    // tile path (many triangles): per-tile counts, offsets, scatter cursors, slot lists
    uint32_t *tile_counts[kSets] = {}, *tile_offs[kSets] = {};
    uint32_t *tile_cursor[kSets] = {}, *tile_total[kSets] = {};
    uint32_t *tile_list[kSets] = {};
    void *recs[kSets] = {};        // 2T raster records (positions-only setup)
    uint32_t *boxes[kSets] = {};   // T packed bboxes
    uint32_t *app_list[kSets] = {}, *app_count[kSets] = {};
    uint64_t tiles_cap = 0, tile_list_cap[kSets] = {};
    unsigned long long *keys = nullptr;        // W x rows per-pixel (1/z, slot) winners
    size_t keys_cap = 0;
    uint32_t *tile_total_host = nullptr;       // pinned: (total, appended) per buffer set
    int raster_path = 0;                       // 0 auto, 1 rows (k_geometry + k_fragment), 2 tiles
    bool serial = false;                       // S3R_SERIAL: no geometry/fragment overlap (profiling)
    uint64_t last_pairs = 0;                   // tile path: (slot, tile) pairs of the last frame
    int last_path = 0;                         // 1 rows, 2 tiles: the last frame's fragment stage
    hipEvent_t geo_done[kSets] = {}, frag_done[kSets] = {};
    // row path, buffer-set reuse without events: each k_fragment launch stores the tag of the previous
    // fragment launch (complete by stream order) in *done_host (host-coherent memory;
    // done_dev is its device address); issued_tag[p] = the tag of the last fragment launch that read
    // set p (0: none); last_tag = the previous row-path fragment launch, last_stream = the stream of
    // the previous frame (either path)
    volatile uint32_t *done_host = nullptr;
    uint32_t *done_dev = nullptr;
    uint32_t issued_tag[kSets] = {}, last_tag = 0;
    // the previous frame's stream; NULL is a valid caller stream (the legacy default stream), so
    // whether a previous frame exists is its own flag
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    hipEvent_t handoff = nullptr;
    uint32_t frame_no = 0;                     // frames issued: set frame_no % kSets
    uint32_t *frame = nullptr;
    size_t frame_cap = 0;
    hipStream_t stream = nullptr, geo[kGeoStreams] = {};

    // caller buffers registered as pinned memory (double buffer: main.swift:117-118)
    struct Reg { void *p; size_t n; bool ok; };
    std::vector<Reg> regs;
    uint64_t stale_pins = 0;                   // registrations found stale and replaced (updateAndRender)

    bool timing = false;
    std::vector<TimingSlot> tslots;
    size_t tcount = 0;
};

Lib g;

// S3R_HOSTPROF=1 (diagnostics): host time per s3r_render_bands section, printed at shutdown.
struct HostProf {
    bool on = getenv("S3R_HOSTPROF") != nullptr;
    double t[6] = {};
    uint64_t frames = 0;
    std::chrono::steady_clock::time_point last;
    void start() { if (on) last = std::chrono::steady_clock::now(); }
    void lap(int i) {
        if (!on) return;
        const auto now = std::chrono::steady_clock::now();
        t[i] += std::chrono::duration<double, std::micro>(now - last).count();
        last = now;
    }
    void report() {
        if (!on || !frames) return;
        fprintf(stderr, "s3r hostprof (us/frame over %llu): begin %.2f  prep %.2f  geo-wait %.2f  geo-launch %.2f  "
                "frag-wait %.2f  frag-launch %.2f\n", (unsigned long long)frames, t[0] / frames, t[1] / frames,
                t[2] / frames, t[3] / frames, t[4] / frames, t[5] / frames);
    }
} hp;

float config_scale() {
    const float fov = (float)M_PI / 5.f;        // render.cpp:91
    return kNear * tanf(fov / 2);               // render.cpp:92
}

// ---------------------------------------------------------------- camera, render.cpp:134-156
F3 smul3(float s, F3 a) { return mk3(s * a.x, s * a.y, s * a.z); }
F3 cross3(F3 a, F3 b) { return mk3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
// simd_act(q, v) = v + re*t + cross(im, t), t = 2*cross(im, v)
F3 quat_act(F3 im, float re, F3 v) {
    const F3 t = smul3(2.0f, cross3(im, v));
    return add3(add3(v, smul3(re, t)), cross3(im, t));
}

void update_camera(const Input *in, bool force) {
    bool changed = false;
    if (in->left > 0 || in->right > 0 || in->up > 0 || in->down > 0) {
        changed = true;
        const F3 mv = add3(smul3(in->right - in->left, g.ax), smul3(in->down - in->up, g.az));
        g.pos = add3(g.pos, smul3(kSpeed, mv));
    }
    if (in->mouse.x != g.mouse[0] || in->mouse.y != g.mouse[1]) {
        changed = true;
        const F3 d = add3(add3(smul3(g.mouse[0] - in->mouse.x, g.ax), smul3(g.mouse[1] - in->mouse.y, g.ay)),
                          smul3(100 / kRotationSpeed, g.az));
        const F3 z = fast_normalize3(d);
        // simd_quaternion(az, z): dot(az, z) > 0 always here, so the reduced form applies
        const F3 h = fast_normalize3(add3(g.az, z));
        const F3 im = cross3(g.az, h);
        const float re = dot3(g.az, h);
        g.ax = fast_normalize3(quat_act(im, re, g.ax));
        g.ay = fast_normalize3(quat_act(im, re, g.ay));
        g.az = z;
        g.mouse[0] = in->mouse.x;
        g.mouse[1] = in->mouse.y;
    }
    if (changed || force) {
        const F3 r[3] = {g.ax, g.ay, g.az};
        for (int i = 0; i < 3; i++) {
            g.m.m[i][0] = r[i].x; g.m.m[i][1] = r[i].y; g.m.m[i][2] = r[i].z;
            g.m.m[i][3] = -dot3(r[i], g.pos);
        }
    }
}

// ---------------------------------------------------------------- data.bin, render.cpp:160-210
std::string find_data_path() {
    if (const char *e = getenv("S3R_DATA_PATH")) return e;
    if (!g.data_path.empty()) return g.data_path;
    Dl_info info;
    if (dladdr((const void *)updateAndRender, &info) && info.dli_fname) {
        std::string lib = info.dli_fname;
        const size_t slash = lib.rfind('/');
        const std::string dir = slash == std::string::npos ? "." : lib.substr(0, slash);
        for (const char *suffix : {"/data.bin", "/Resources/data.bin", "/../data-generator/data.bin"}) {
            const std::string p = dir + suffix;
            if (FILE *f = fopen(p.c_str(), "rb")) { fclose(f); return p; }
        }
    }
    return "";
}

template <class T> T *dalloc(size_t n) {
    T *p = nullptr;
    HIPCHECK(hipMalloc((void **)&p, (n ? n : 1) * sizeof(T)));
    return p;
}

[[noreturn]] void bad_scene(const std::string &path, const char *why) {
    fprintf(stderr, "s3r: %s: malformed data.bin (%s)\n", path.c_str(), why);
    exit(666);
}

void initialize() {
    const std::string path = find_data_path();
    FILE *fp = path.empty() ? nullptr : fopen(path.c_str(), "rb");
    if (!fp) exit(666);                                                 // render.cpp:173
    auto rd = [&](void *dst, size_t bytes) {
        if (bytes && fread(dst, 1, bytes, fp) != bytes) bad_scene(path, "truncated");
    };
    uint64_t cnt[2];
    rd(cnt, 16);
    const uint64_t nv = cnt[0];
    std::vector<float4> vtx(nv);
    rd(vtx.data(), nv * 16);
    rd(cnt, 16);
    const uint64_t ni = cnt[0];
    std::vector<int64_t> vi(ni + ni % 2);
    rd(vi.data(), vi.size() * 8);
    rd(cnt, 16);
    const uint64_t na = cnt[0];
    std::vector<uint8_t> attr(na * 48);
    rd(attr.data(), attr.size());
    rd(cnt, 16);
    const uint64_t nai = cnt[0];
    std::vector<int64_t> ai(nai + nai % 2);
    rd(ai.data(), ai.size() * 8);
    rd(cnt, 16);
    const uint64_t nt = cnt[0];
    std::vector<uint32_t> tex(nt);
    rd(tex.data(), nt * 4);
    fclose(fp);

    // The reference trusts the file; the GPU must not read out of bounds, so check it here.
    if (nv >= (1ull << 32) || na >= (1ull << 32) || nt >= (1ull << 32)) bad_scene(path, "too large");
    if (nai < ni) bad_scene(path, "fewer attribute indices than vertex indices");
    const uint64_t ntri = ni / 3;
    std::vector<uint32_t> vi32(3 * ntri), ai32(3 * ntri);
    for (uint64_t k = 0; k < 3 * ntri; k++) {
        if (vi[k] < 0 || (uint64_t)vi[k] >= nv) bad_scene(path, "vertex index out of range");
        if (ai[k] < 0 || (uint64_t)ai[k] >= na) bad_scene(path, "attribute index out of range");
        vi32[k] = (uint32_t)vi[k];
        ai32[k] = (uint32_t)ai[k];
    }
    std::vector<float4> nrm(na), pay(na);
    std::vector<uint8_t> disc(na);
    for (uint64_t k = 0; k < na; k++) {
        memcpy(&nrm[k], &attr[48 * k], 16);
        memcpy(&pay[k], &attr[48 * k + 16], 16);
        uint32_t d;
        memcpy(&d, &attr[48 * k + 32], 4);                              // disc_t at +32
        disc[k] = d != 0;
    }

    if (g.device < 0) {
        if (const char *e = getenv("S3R_DEVICE")) g.device = atoi(e);
        else HIPCHECK(hipGetDevice(&g.device));
    }
    HIPCHECK(hipSetDevice(g.device));
    if (!g.stream) HIPCHECK(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking));
    g.serial = getenv("S3R_SERIAL") != nullptr;
    g.nv = (uint32_t)nv; g.na = (uint32_t)na; g.ntri = (uint32_t)ntri; g.ntex = (uint32_t)nt;
    g.nindices = ni;
    g.vtx = dalloc<float4>(nv); g.nrm = dalloc<float4>(na); g.pay = dalloc<float4>(na);
    g.disc = dalloc<uint8_t>(na);
    g.vidx = dalloc<uint32_t>(3 * ntri); g.aidx = dalloc<uint32_t>(3 * ntri);
    g.tex = dalloc<uint32_t>(nt);
    for (int p = 0; p < kSets; p++) {
        g.tris[p] = dalloc<TriSetup>(2 * ntri);
        HIPCHECK(hipEventCreateWithFlags(&g.geo_done[p], hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&g.frag_done[p], hipEventDisableTiming));
    }
    {
        void *h = nullptr;
        HIPCHECK(hipHostMalloc(&h, sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
        memset(h, 0, sizeof(uint32_t));
        g.done_host = static_cast<volatile uint32_t *>(h);
        HIPCHECK(hipHostGetDevicePointer((void **)&g.done_dev, h, 0));
        HIPCHECK(hipEventCreateWithFlags(&g.handoff, hipEventDisableTiming));
    }
    // geometry streams at the highest priority: their (small, latency-bound) workgroups are
    // dispatched as soon as the previous frame's fragment workgroups free a slot
    int prio_least = 0, prio_greatest = 0;
    HIPCHECK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    for (hipStream_t &gs : g.geo)
        if (!gs) HIPCHECK(hipStreamCreateWithPriority(&gs, hipStreamNonBlocking, prio_greatest));
    HIPCHECK(hipMemcpy(g.vtx, vtx.data(), nv * 16, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.nrm, nrm.data(), na * 16, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.pay, pay.data(), na * 16, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.disc, disc.data(), na, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.vidx, vi32.data(), 12 * ntri, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.aidx, ai32.data(), 12 * ntri, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(g.tex, tex.data(), nt * 4, hipMemcpyHostToDevice));
}

void unregister_all() {
    for (auto &r : g.regs)
        if (r.ok) (void)hipHostUnregister(r.p);
    g.regs.clear();
}

void release_all() {
    if (g.initialized) {
        (void)hipSetDevice(g.device);
        if (g.stream) (void)hipStreamSynchronize(g.stream);
        for (hipStream_t gs : g.geo)
            if (gs) (void)hipStreamSynchronize(gs);
        (void)hipDeviceSynchronize();
        unregister_all();
        void *ptrs[] = {g.vtx, g.nrm, g.pay, g.disc, g.vidx, g.aidx, g.tex, g.frame, g.keys};
        for (void *p : ptrs)
            if (p) (void)hipFree(p);
        for (int q = 0; q < kSets; q++) {      // tile_total aliases app_count
            void *set[] = {g.tris[q], g.rowtab[q], g.bincnt[q], g.pairs[q], g.order[q], g.tile_counts[q], g.tile_offs[q], g.tile_cursor[q],
                           g.tile_list[q], g.recs[q], g.boxes[q], g.app_list[q], g.app_count[q]};
            for (void *p : set)
                if (p) (void)hipFree(p);
        }
        if (g.done_host) (void)hipHostFree((void *)g.done_host);
        if (g.handoff) (void)hipEventDestroy(g.handoff);
        if (g.tile_total_host) (void)hipHostFree(g.tile_total_host);
        for (int p = 0; p < kSets; p++) {
            if (g.geo_done[p]) (void)hipEventDestroy(g.geo_done[p]);
            if (g.frag_done[p]) (void)hipEventDestroy(g.frag_done[p]);
        }
        for (hipStream_t gs : g.geo)
            if (gs) (void)hipStreamDestroy(gs);
        for (auto &t : g.tslots) {
            (void)hipEventDestroy(t.frame0); (void)hipEventDestroy(t.frag0); (void)hipEventDestroy(t.frag1);
        }
        if (g.stream) (void)hipStreamDestroy(g.stream);
    }
    const std::string path = g.data_path;
    const int dev = g.device, rp = g.raster_path;
    g.~Lib();
    new (&g) Lib();
    g.data_path = path;
    g.device = dev;
    g.raster_path = rp;
}

// render.cpp:266-280: first-call init, camera, resize.
void frame_begin(const Input *input, uint32_t width, uint32_t height) {
    if (!g.initialized) {
        g.initialized = true;
        initialize();
        update_camera(input, true);
    } else {
        update_camera(input, false);
        HIPCHECK(hipSetDevice(g.device));
    }
    const uint32_t dbs = width * height * (uint32_t)sizeof(float);
    if (g.depth_buffer_size != dbs) {
        g.depth_buffer_size = dbs;
        g.factor = kNear * (float)height / (2 * config_scale());          // render.cpp:279
        unregister_all();
    }
}

TimingSlot *timing_slot() {
    if (!g.timing) return nullptr;
    if (g.tcount == g.tslots.size()) {
        TimingSlot t;
        HIPCHECK(hipEventCreate(&t.frame0)); HIPCHECK(hipEventCreate(&t.frag0)); HIPCHECK(hipEventCreate(&t.frag1));
        g.tslots.push_back(t);
    }
    return &g.tslots[g.tcount++];
}

// Frame tags are the uint32 frame number (0 = none): the slot-mask words' high halves, issued_tag,
// last_tag and the completion word.  Before the count wraps (~62 h at 19 k fps) every stream is
// drained, the slot masks are zeroed and the count restarts, so no tag is reused while a word or a
// completion flag still carries it.
constexpr uint32_t kTagLimit = 0xFFFFFF00u;

void restart_tags(uint32_t next_frame_no) {
    HIPCHECK(hipDeviceSynchronize());
    for (int p = 0; p < kSets; p++)
        if (g.bincnt[p]) HIPCHECK(hipMemset(g.bincnt[p], 0, g.bins_cap * sizeof(uint32_t)));
    HIPCHECK(hipDeviceSynchronize());
    g.frame_no = next_frame_no;
    for (uint32_t &t : g.issued_tag) t = 0;
    g.last_tag = 0;
    if (g.done_host) __atomic_store_n(g.done_host, 0u, __ATOMIC_RELEASE);
}

// The buffer set of the frame being issued; frames cycle through kSets sets.
uint32_t next_set() {
    if (g.frame_no >= kTagLimit) restart_tags(0);
    g.frame_no++;
    return g.frame_no % kSets;
}

// Row path: block until the last fragment kernel that read buffer set p has finished.  *done_host
// holds the tag of the newest fragment launch known complete: every launch's first workgroup stores
// its predecessor's tag there, and tags grow by frame.  Usually the set is free (the host runs at
// most kSets frames ahead of the GPU); otherwise the launch after it -- issued already, in order on
// the same stream -- reports it when it starts.
void wait_set_free(uint32_t p) {
    const uint32_t want = g.issued_tag[p];
    if (want == 0 || __atomic_load_n(g.done_host, __ATOMIC_ACQUIRE) >= want) return;
    if (want == g.last_tag) {
        // no row-path fragment launch after it to report it (tile-path frames followed): drain its stream
        HIPCHECK(hipStreamSynchronize(g.last_stream));
        __atomic_store_n(g.done_host, want, __ATOMIC_RELEASE);
        return;
    }
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(g.done_host, __ATOMIC_ACQUIRE) < want) {
        __builtin_ia32_pause();
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(10)) {
            HIPCHECK(hipDeviceSynchronize());      // (never expected) surfaces a device fault
            __atomic_store_n(g.done_host, g.last_tag, __ATOMIC_RELEASE);
        }
    }
}

// Frames are ordered on the caller's stream.  When a frame arrives on another stream than the
// previous one, that stream first waits for the previous frame's fragment stage (one event): the
// row path's completion chain (wait_set_free) and the tile path's shared key buffer assume it.
void follow_previous_frame(hipStream_t st) {
    // the null stream does not order our non-blocking streams (nor they it): a switch from or to
    // NULL needs the event like any other
    if (g.have_last && st != g.last_stream) {
        HIPCHECK(hipEventRecord(g.handoff, g.last_stream));
        HIPCHECK(hipStreamWaitEvent(st, g.handoff, 0));
    }
    g.last_stream = st;
    g.have_last = true;
}

// S3R_SERIAL (profiling): the geometry waits for every earlier fragment kernel -- no overlap.
void wait_all_fragments(hipStream_t geo) {
    for (int q = 0; q < kSets; q++) HIPCHECK(hipStreamWaitEvent(geo, g.frag_done[q], 0));
}

// Slots above which the row path's start table (2T x H x segments x 16 B) is not worth building:
// the order-independent tile path takes over (the icosahedron stress scene).
constexpr uint64_t kRowPathMaxSlots = 8192;

bool use_tile_path() {
    if (g.raster_path == 1) return false;
    if (g.raster_path == 2) return true;
    return 2ull * g.ntri > kRowPathMaxSlots;
}

void render_tiles(uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                  uint32_t *out, hipStream_t st, TimingSlot *ts) {
    if (W > 65535 || H > 65535) {                       // packed 16-bit bboxes
        fprintf(stderr, "s3r: tile path supports frames up to 65535 x 65535\n");
        exit(1);
    }
    const float sw = (float)W, sh = (float)H;
    const uint64_t nt = tile_count(W, rows_local);
    if (g.tiles_cap < nt) {
        HIPCHECK(hipDeviceSynchronize());
        for (int p = 0; p < kSets; p++) {
            for (uint32_t **q : {&g.tile_counts[p], &g.tile_offs[p], &g.tile_cursor[p]}) {
                if (*q) HIPCHECK(hipFree(*q));
                *q = dalloc<uint32_t>(nt);
            }
        }
        g.tiles_cap = nt;
    }
    const size_t npx = (size_t)W * rows_local;
    if (g.keys_cap < npx) {                    // per-pixel winners (fragment stage, caller's stream)
        HIPCHECK(hipDeviceSynchronize());
        if (g.keys) HIPCHECK(hipFree(g.keys));
        g.keys = dalloc<unsigned long long>(npx);
        g.keys_cap = npx;
    }
    if (!g.recs[0]) {
        for (int p = 0; p < kSets; p++) {
            g.recs[p] = dalloc<uint8_t>((size_t)2 * g.ntri * raster_rec_bytes());
            g.boxes[p] = dalloc<uint32_t>((size_t)2 * g.ntri);
            g.app_list[p] = dalloc<uint32_t>(g.ntri);
            g.app_count[p] = dalloc<uint32_t>(2);          // [0] appended count, [1] tile-pair total
            g.tile_total[p] = g.app_count[p] + 1;
        }
        HIPCHECK(hipHostMalloc((void **)&g.tile_total_host, 2 * kSets * sizeof(uint32_t)));
    }
    const uint32_t p = next_set();
    hipStream_t geo = g.geo[0];
    HIPCHECK(hipStreamWaitEvent(geo, g.frag_done[p], 0));
    if (g.serial) wait_all_fragments(geo);
    if (ts) HIPCHECK(hipEventRecord(ts->frame0, geo));
    launch_tile_setup(g.vtx, g.vidx, g.ntri, g.m, g.factor, sw, sh, W, band, nparts, part, rows_local, g.recs[p],
                      g.boxes[p], g.app_list[p], g.app_count[p], g.tile_counts[p], g.tile_offs[p], g.tile_cursor[p],
                      g.tile_total[p], geo);
    // the list size is data-dependent: read it back (the tile path's one host sync per frame)
    uint32_t *host = g.tile_total_host + 2 * p;
    HIPCHECK(hipMemcpyAsync(host, g.app_count[p], 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, geo));
    HIPCHECK(hipStreamSynchronize(geo));
    const uint32_t napp = host[0];
    const uint64_t total = host[1];
    g.last_pairs = total;
    g.last_path = 2;
    if (g.tile_list_cap[p] < total) {
        HIPCHECK(hipDeviceSynchronize());
        if (g.tile_list[p]) HIPCHECK(hipFree(g.tile_list[p]));
        const uint64_t cap = total + total / 4 + 1024;
        g.tile_list[p] = dalloc<uint32_t>(cap);
        g.tile_list_cap[p] = cap;
    }
    launch_tile_fill(g.boxes[p], g.ntri, g.recs[p], g.app_list[p], napp, W, band, nparts, part, g.tile_cursor[p],
                     g.tile_list[p], geo);
    HIPCHECK(hipEventRecord(g.geo_done[p], geo));
    follow_previous_frame(st);
    HIPCHECK(hipStreamWaitEvent(st, g.geo_done[p], 0));
    if (ts) HIPCHECK(hipEventRecord(ts->frag0, st));
    launch_tile_raster(g.recs[p], W, band, nparts, part, rows_local, g.tile_offs[p], g.tile_counts[p], g.tile_list[p],
                       g.keys, st);
    launch_tile_resolve(g.keys, g.recs[p], g.vtx, g.nrm, g.pay, g.disc, g.vidx, g.aidx, g.ntri, g.m, g.factor, sw, sh,
                        g.tex, g.ntex, out, W, band, nparts, part, rows_local, st);
    if (ts) HIPCHECK(hipEventRecord(ts->frag1, st));
    HIPCHECK(hipEventRecord(g.frag_done[p], st));
    HIPCHECK(hipGetLastError());
}

void render_core(uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                 uint32_t *out, hipStream_t st) {
    TimingSlot *ts = timing_slot();
    if (use_tile_path()) {
        render_tiles(W, H, band, nparts, part, rows_local, out, st, ts);
        return;
    }
    g.last_path = 1;
    fragment_configure(W, rows_local);
    const size_t need = (size_t)2 * g.ntri * rows_local * start_entries(W) * 4;
    if (g.rowtab_cap < need) {
        HIPCHECK(hipDeviceSynchronize());
        for (int p = 0; p < kSets; p++) {
            if (g.rowtab[p]) HIPCHECK(hipFree(g.rowtab[p]));
            g.rowtab[p] = dalloc<float>(need);
        }
        g.rowtab_cap = need;
    }
    const uint64_t nbins = fragment_bins(W, rows_local);
    if (g.bins_cap < nbins) {
        HIPCHECK(hipDeviceSynchronize());
        for (int p = 0; p < kSets; p++) {
            if (g.bincnt[p]) HIPCHECK(hipFree(g.bincnt[p]));
            if (g.pairs[p]) HIPCHECK(hipFree(g.pairs[p]));
            g.bincnt[p] = dalloc<uint32_t>(nbins);
            g.pairs[p] = dalloc<uint4>(nbins * kPairMax * kPairWords);
            HIPCHECK(hipMemset(g.bincnt[p], 0, nbins * sizeof(uint32_t)));
        }
        // hipMemset runs on the null stream, which does not order the non-blocking geometry
        // streams: finish it before the next k_geometry counts pairs in these bins
        HIPCHECK(hipDeviceSynchronize());
        g.bins_cap = nbins;
    }
    // longest-first order only where a launch is several rounds of resident workgroups (~1 280 on
    // the chip): a frame part of one round gains nothing and would pay the order column's time
    const uint64_t bins = fragment_bins(W, rows_local);
    const char *lpt_env = getenv("S3R_LPT_MIN");            // tuning / test override
    const bool lpt = g.ntri > 0 && bins >= (lpt_env ? strtoull(lpt_env, nullptr, 10) : kLptMinBins);
    if (lpt && g.order_cap < bins) {
        HIPCHECK(hipDeviceSynchronize());
        for (int q = 0; q < kSets; q++) {
            if (g.order[q]) HIPCHECK(hipFree(g.order[q]));
            g.order[q] = dalloc<uint32_t>(2 * bins);
            HIPCHECK(hipMemset(g.order[q], 0, 2 * bins * sizeof(uint32_t)));
        }
        HIPCHECK(hipDeviceSynchronize());     // (as for the slot masks: before k_geometry writes perm)
        g.order_cap = bins;
    }
    // geometry for this frame into buffer set p, once the fragment kernel that last read set p is done
    const uint32_t p = next_set();
    hipStream_t geo = g.geo[g.frame_no % kGeoStreams];
    hp.lap(1);
    // the set's last reader (frame k - kSets) has usually finished: then no cross-stream wait
    if (g.serial) {
        HIPCHECK(hipStreamWaitEvent(geo, g.frag_done[p], 0));
        wait_all_fragments(geo);
    } else {
        wait_set_free(p);
    }
    if (ts) HIPCHECK(hipEventRecord(ts->frame0, geo));
    hp.lap(2);
    const uint32_t tag = g.frame_no;              // >= 1: frame k's tag for its slot masks and completion
    launch_geometry(g.vtx, g.nrm, g.pay, g.disc, g.vidx, g.aidx, g.ntri, g.m, g.factor, W, H, band, nparts, part,
                    rows_local, g.tris[p], g.rowtab[p], g.bincnt[p], g.pairs[p], geo, g.geo_done[p],
                    lpt ? g.order[p] : nullptr);
    hp.lap(3);
    // fragment on the caller's stream, after the previous frame and this frame's geometry; its first
    // workgroup reports the previous fragment launch complete (wait_set_free); the completion event
    // only where S3R_SERIAL waits on it
    follow_previous_frame(st);
    HIPCHECK(hipStreamWaitEvent(st, g.geo_done[p], 0));
    hp.lap(4);
    if (ts) HIPCHECK(hipEventRecord(ts->frag0, st));
    launch_fragment(g.tris[p], 2 * g.ntri, g.rowtab[p], g.tex, g.ntex, out, W, H, band, nparts, part, rows_local,
                    g.bincnt[p], g.pairs[p], tag, st, g.serial ? g.frag_done[p] : nullptr, g.done_dev, g.last_tag,
                    lpt ? g.order[p] : nullptr);
    g.issued_tag[p] = tag;
    g.last_tag = tag;
    if (ts) HIPCHECK(hipEventRecord(ts->frag1, st));
    HIPCHECK(hipGetLastError());
    hp.lap(5);
    hp.frames++;
}

bool host_pinned(void *p, size_t n) {
    for (auto &r : g.regs)
        if (r.p == p && r.n == n) return r.ok;
    if (getenv("S3R_NO_PIN")) return false;
    if (g.regs.size() >= 4) unregister_all();
    const bool ok = hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess;
    if (!ok) (void)hipGetLastError();
    g.regs.push_back({p, n, ok});
    return ok;
}

void drop_registration(void *p, size_t n) {
    for (size_t i = 0; i < g.regs.size(); i++) {
        if (g.regs[i].p == p && g.regs[i].n == n) {
            if (g.regs[i].ok) (void)hipHostUnregister(p);
            g.regs.erase(g.regs.begin() + (long)i);
            return;
        }
    }
}

// A cached registration is keyed by (pointer, size).  If the caller freed its buffer and got a new
// one at the same address, a registration that still pins the old pages would take the frame.
// Pixels are 0x00RRGGBB, so a word with a set high byte is never a pixel: such a sentinel is stored
// through the caller's pointer at the buffer's ends and every 64 KiB before the copy; if one
// survives the copy, the copy did not reach the caller's pages and is redone through a new
// registration.
constexpr uint32_t kStaleProbe = 0xFF5A5A5Au;
constexpr size_t kProbeStride = 16384;        // words: 64 KiB

void stamp_probes(uint32_t *buf, size_t words) {
    for (size_t i = 0; i < words; i += kProbeStride) buf[i] = kStaleProbe;
    buf[words - 1] = kStaleProbe;
}

bool probes_overwritten(const uint32_t *buf, size_t words) {
    const volatile uint32_t *b = buf;
    for (size_t i = 0; i < words; i += kProbeStride)
        if (b[i] == kStaleProbe) return false;
    return b[words - 1] != kStaleProbe;
}

}  // namespace

extern "C" {

__attribute__((visibility("default"))) void updateAndRender(const PixelData *pixel_data, const Input *input) {
    const uint32_t W = pixel_data->width, H = pixel_data->height;
    frame_begin(input, W, H);
    const size_t npx = (size_t)W * H;
    if (g.frame_cap < npx) {
        if (g.frame) HIPCHECK(hipFree(g.frame));
        g.frame = dalloc<uint32_t>(npx);
        g.frame_cap = npx;
    }
    if (npx) render_core(W, H, H ? H : 1, 1, 0, H, g.frame, g.stream);
    // memset_pattern4 fills bufferSize bytes (render.cpp:282); the frame covers W*H pixels.
    const size_t frame_bytes = npx * 4;
    const size_t copy_bytes = pixel_data->bufferSize < frame_bytes ? pixel_data->bufferSize : frame_bytes;
    const size_t copy_words = copy_bytes / 4;
    bool pinned = false;
    if (copy_bytes) {
        pinned = host_pinned(pixel_data->buffer, pixel_data->bufferSize);
        if (pinned && copy_words) stamp_probes(pixel_data->buffer, copy_words);
        HIPCHECK(hipMemcpyAsync(pixel_data->buffer, g.frame, copy_bytes, hipMemcpyDeviceToHost, g.stream));
    }
    for (size_t i = frame_bytes / 4; i < pixel_data->bufferSize / 4; i++) pixel_data->buffer[i] = kBackground;
    HIPCHECK(hipStreamSynchronize(g.stream));
    if (pinned && copy_words && !probes_overwritten(pixel_data->buffer, copy_words)) {
        // a stale registration (buffer freed and reallocated at the same address): pin anew, copy again
        drop_registration(pixel_data->buffer, pixel_data->bufferSize);
        g.stale_pins++;
        host_pinned(pixel_data->buffer, pixel_data->bufferSize);
        HIPCHECK(hipMemcpyAsync(pixel_data->buffer, g.frame, copy_bytes, hipMemcpyDeviceToHost, g.stream));
        HIPCHECK(hipStreamSynchronize(g.stream));
    }
}

__attribute__((visibility("default"))) int s3r_configure(const char *data_path, int device) {
    release_all();
    g.data_path = data_path ? data_path : "";
    g.device = device;
    return 0;
}

__attribute__((visibility("default"))) void s3r_shutdown(void) {
    hp.report();
    release_all();
}

__attribute__((visibility("default"))) int s3r_set_raster_path(int mode) {
    if (mode < 0 || mode > 2) return -1;
    g.raster_path = mode;
    return 0;
}

__attribute__((visibility("default"))) int s3r_raster_path(void) { return use_tile_path() ? 2 : 1; }

__attribute__((visibility("default"))) uint32_t s3r_band_rows_local(uint32_t height, uint32_t band_rows,
                                                                   uint32_t n_parts, uint32_t part) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts) return 0;
    uint32_t rows = 0;
    for (uint64_t b = part; b * band_rows < height; b += n_parts) {
        const uint64_t y0 = b * band_rows;
        rows += (uint32_t)((height - y0) < band_rows ? (height - y0) : band_rows);
    }
    return rows;
}

__attribute__((visibility("default"))) int64_t s3r_render_bands(const Input *input, uint32_t width, uint32_t height,
                                                               uint32_t band_rows, uint32_t n_parts, uint32_t part,
                                                               uint32_t *dev_out, void *stream) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts || (!dev_out && width && height)) return -1;
    hp.start();
    frame_begin(input, width, height);
    hp.lap(0);
    const uint32_t rows = s3r_band_rows_local(height, band_rows, n_parts, part);
    // NULL is the legacy default (null) stream -- e.g. torch's default stream -- never our own.
    hipStream_t st = (hipStream_t)stream;
    if (rows && width) render_core(width, height, band_rows, n_parts, part, rows, dev_out, st);
    return rows;
}

// Test hook: drain the device and continue the frame count at `frame_no` (tags above every tag in use
// keep the slot masks valid), to exercise the tag restart before the uint32 count wraps.
__attribute__((visibility("default"))) void s3r_debug_set_frame_count(uint32_t frame_no) {
    if (!g.initialized) return;
    HIPCHECK(hipSetDevice(g.device));
    restart_tags(frame_no > kTagLimit ? kTagLimit : frame_no);
}

__attribute__((visibility("default"))) int64_t s3r_bands_to_host(const uint32_t *dev_rows, uint32_t width, uint32_t height,
                                                                uint32_t band_rows, uint32_t n_parts, uint32_t part,
                                                                uint32_t *host_frame, void *stream) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts || ((!dev_rows || !host_frame) && width && height)) return -1;
    const uint32_t rows = s3r_band_rows_local(height, band_rows, n_parts, part);
    if (!rows || !width) return rows;
    if (g.device >= 0) HIPCHECK(hipSetDevice(g.device));
    host_pinned(host_frame, (size_t)width * height * sizeof(uint32_t));
    hipStream_t st = (hipStream_t)stream;
    const size_t rowb = (size_t)width * sizeof(uint32_t);
    // this part's bands: b = part, part + n_parts, ...; all full except perhaps the frame's last band
    const uint32_t nbands = (height + band_rows - 1) / band_rows, last = nbands - 1u;
    const uint32_t mine = (nbands > part) ? (nbands - part + n_parts - 1u) / n_parts : 0u;
    const bool partial_last = (uint64_t)nbands * band_rows > height && last % n_parts == part;
    const uint32_t full = mine - (partial_last ? 1u : 0u);
    if (full)
        HIPCHECK(hipMemcpy2DAsync(host_frame + (size_t)part * band_rows * width, (size_t)n_parts * band_rows * rowb, dev_rows,
                                  (size_t)band_rows * rowb, (size_t)band_rows * rowb, full, hipMemcpyDeviceToHost, st));
    if (partial_last)
        HIPCHECK(hipMemcpyAsync(host_frame + (size_t)last * band_rows * width, dev_rows + (size_t)full * band_rows * width,
                                (size_t)(height - last * band_rows) * rowb, hipMemcpyDeviceToHost, st));
    return rows;
}

__attribute__((visibility("default"))) void s3r_unregister_host(void *ptr) {
    if (!ptr) return;
    for (size_t i = g.regs.size(); i-- > 0;) {
        if (g.regs[i].p != ptr) continue;
        if (g.regs[i].ok) {
            if (g.device >= 0) HIPCHECK(hipSetDevice(g.device));
            HIPCHECK(hipDeviceSynchronize());          // no copy into it may still be in flight
            (void)hipHostUnregister(ptr);
        }
        g.regs.erase(g.regs.begin() + (long)i);
    }
}

__attribute__((visibility("default"))) void s3r_timing(int enable) {
    g.timing = enable != 0;
    g.tcount = 0;
}

__attribute__((visibility("default"))) void s3r_timing_collect(double out[3]) {
    double frag = 0, frame = 0;
    for (size_t i = 0; i < g.tcount; i++) {
        float a = 0, b = 0;
        HIPCHECK(hipEventSynchronize(g.tslots[i].frag1));
        HIPCHECK(hipEventElapsedTime(&a, g.tslots[i].frag0, g.tslots[i].frag1));
        HIPCHECK(hipEventElapsedTime(&b, g.tslots[i].frame0, g.tslots[i].frag1));
        frag += a;
        frame += b;
    }
    out[0] = frag;
    out[1] = frame;
    out[2] = (double)g.tcount;
    g.tcount = 0;
}

__attribute__((visibility("default"))) void s3r_scene_counts(uint64_t out[8]) {
    out[0] = g.nv; out[1] = g.nindices; out[2] = g.na; out[3] = g.ntex; out[4] = 2ull * g.ntri;
    out[5] = g.last_pairs;                   // tile path: (slot, tile) pairs binned last frame
    out[6] = (uint64_t)g.last_path;          // fragment stage of the last frame: 1 rows, 2 tiles
    out[7] = g.stale_pins;                   // stale host registrations replaced by updateAndRender
}

__attribute__((visibility("default"))) void s3r_camera(float out_matrix[12], float *out_factor) {
    memcpy(out_matrix, g.m.m, sizeof g.m.m);
    if (out_factor) *out_factor = g.factor;
}

// Diagnostic counters (non-zero only in the S3R_STATS build, librender_stats.so): pairs of
// (sum over lanes, sum over waves of the wave maximum) for row-walk, chunk-walk and per-pixel walker
// iterations, irregular chunk components, pixel-triangle tests and triangle batches.
__attribute__((visibility("default"))) void s3r_stats(uint64_t out[16], int reset) {
    unsigned long long tmp[24];
    stats_read(tmp, reset != 0);
    for (int i = 0; i < 16; i++) out[i] = tmp[i];
}

// Timing build only (-DS3R_WGTIME): the last k_fragment launch's per-workgroup phase timestamps (100 MHz wall clock,
// wave 0): out[4 * wg + k], k = 0 start, 1 list loaded, 2 walk state loaded, 3 end.  Returns the
// number of workgroups copied (0 in the product build).
__attribute__((visibility("default"))) uint32_t s3r_stats_wg_times(uint64_t *out, uint32_t max_wg) {
    return wg_times_read(reinterpret_cast<unsigned long long *>(out), max_wg);
}

// Timing build only (-DS3R_WGTIME): per k_geometry workgroup (slot + row block * 2T) of the launches since the
// last call, 100 MHz wall clock: out[4 * wg + k], k = 0 start, 1 slot set up, 2 bins set, 3 end.  Returns
// the number of workgroup records copied (0 in the product build) and clears them.
__attribute__((visibility("default"))) uint32_t s3r_stats_geo_times(uint64_t *out, uint32_t max_wg) {
    return geo_times_read(reinterpret_cast<unsigned long long *>(out), max_wg);
}

// Stats build only: k_geometry wall-clock profile (100 MHz ticks): {max setup time of a workgroup,
// max workgroup time, first start, last end, 0...}.  Reset together with s3r_stats(.., 1).
__attribute__((visibility("default"))) void s3r_stats_geometry(uint64_t out[8]) {
    unsigned long long tmp[24];
    stats_read(tmp, false);
    for (int i = 0; i < 8; i++) out[i] = tmp[16 + i];
}

// ---- self-test hooks: the exact repeated-addition walker on the host and on the device ----
__attribute__((visibility("default"))) void s3r_selftest_walk_host(const float *s, const float *d, const uint32_t *n,
                                                                  float *out, uint32_t *lin, float *del,
                                                                  uint64_t count) {
    for (uint64_t i = 0; i < count; i++) {
        out[i] = exact_walk(s[i], d[i], n[i]);
        lin[i] = chunk_linear(s[i], d[i], n[i], &del[i]) ? 1u : 0u;
    }
}

__attribute__((visibility("default"))) int s3r_selftest_fastmath_device(uint32_t mode, uint64_t count,
                                                                       uint64_t out[2]) {
    return fastmath_test(mode, count, out);
}

__attribute__((visibility("default"))) int s3r_selftest_walk_device(const float *s, const float *d, const uint32_t *n,
                                                                   float *out, uint32_t *lin, float *del,
                                                                   uint32_t count) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return -1;
    float *ds, *dd, *dout, *ddel;
    uint32_t *dn, *dlin;
    const size_t b = (size_t)count * 4;
    HIPCHECK(hipMalloc((void **)&ds, b + 4)); HIPCHECK(hipMalloc((void **)&dd, b + 4));
    HIPCHECK(hipMalloc((void **)&dn, b + 4)); HIPCHECK(hipMalloc((void **)&dout, b + 4));
    HIPCHECK(hipMalloc((void **)&dlin, b + 4)); HIPCHECK(hipMalloc((void **)&ddel, b + 4));
    HIPCHECK(hipMemcpy(ds, s, b, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dd, d, b, hipMemcpyHostToDevice));
    HIPCHECK(hipMemcpy(dn, n, b, hipMemcpyHostToDevice));
    launch_walk_test(ds, dd, dn, dout, dlin, ddel, count, nullptr);
    HIPCHECK(hipGetLastError());
    HIPCHECK(hipMemcpy(out, dout, b, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(lin, dlin, b, hipMemcpyDeviceToHost));
    HIPCHECK(hipMemcpy(del, ddel, b, hipMemcpyDeviceToHost));
    void *ptrs[] = {ds, dd, dn, dout, dlin, ddel};
    for (void *p : ptrs) HIPCHECK(hipFree(p));
    return 0;
}

}  // extern "C"
