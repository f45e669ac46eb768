// render_api.cpp -- the C-ABI shim: what render.cpp's host side did, with the per-pixel work moved
// to the gfx950 kernels (kernels.hip).
//
//   updateAndRender   render.cpp:264-384   lazy init, camera update, resize, frame, copy-out
//   initialize        render.cpp:160-210   data.bin search next to the library (dladdr), load, upload
//   update_camera     render.cpp:134-156   host float32, same operation order as the reference
//
// State is process-global like the reference's statics (render.cpp:51-113); calls are expected from
// one thread at a time (main.swift calls from its main-thread timer only).
//
// Devices.  The camera, the scene's counts and the caller's host-buffer registrations are the
// library's (Lib); everything that lives on a GPU -- the scene replica, the per-frame buffer sets,
// streams and frame tags -- is one Dev per device.  With one device (the default) updateAndRender
// renders the whole frame on it.  With N devices (s3r_configure_devices, or S3R_DEVICES=0,1,... for a
// caller that only knows updateAndRender, like the Swift app) the frame's rows are split into
// interleaved bands (band b -> device b % N) and every device renders its bands and
// copies them straight into their rows of the caller's buffer over its own PCIe link; device 0's
// part runs on the calling thread, the others on one persistent worker thread per device, so the
// devices' HIP calls do not serialise.  The call returns when every part has landed.
#include <dlfcn.h>
#include <limits.h>
#include <pthread.h>
#include <sched.h>
#include <sys/syscall.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/render.h"
#include "s3r_kernels.h"

namespace s3r_host {   // clusters.cpp
void build_clusters(const float *vtx, uint32_t nv, const uint32_t *vidx, uint32_t ntri, uint32_t kmin, uint32_t kmax,
                    std::vector<uint32_t> &first, std::vector<float> &sphere, std::vector<uint32_t> &perm);
}
namespace s3r_host {   // host_fill.cpp
void fill_words(uint32_t *p, size_t n, uint32_t v);
void store_fence();
}

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

// ---------------------------------------------------------------- bounded waits
// A dlopen'ed library must never hang its caller (the reference's only failure is exit(666),
// render.cpp:173).  Every wait of the library on a GPU has a deadline, S3R_WAIT_MS (default 30 s,
// far above any frame: a 20 M-triangle 4K frame takes ~1 ms):
//   * the waits on host-coherent words the kernels write (buffer-set reuse, the tile summary, the
//     host fill's bin flags) spin with the clock in view and, past a short grace, poll the stream
//     they are waiting on with hipStreamQuery -- finished without the word is a protocol error,
//     unfinished at the deadline a stall;
//   * the blocking HIP calls (stream / event / device synchronisation before frees, at frame ends,
//     in the statistics getters) run with a watchdog armed for the call: a thread that wakes a few
//     times a second and ends the process when an armed call has passed its deadline;
//   * the one device-side spin (k_geometry's sky-flag publishers, kernels.hip publish_sky_flags)
//     has a clock deadline of its own and reports through the device's error words (Dev::diag_host).
// Expiry prints the stage, the kernel waited for, the device and the frame to stderr and ends the
// process with status kStallExit: no retry, no re-exec, no further HIP call (_exit: the runtime's
// exit handlers would wait for the same queue).
int wait_deadline_ms() {
    static const int ms = [] {
        const char *e = getenv("S3R_WAIT_MS");
        const long v = e ? atol(e) : 0;
        return v > 0 ? (int)std::min<long>(v, 3600000L) : 30000;
    }();
    return ms;
}

int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct WaitSite {
    const char *stage;      // what the library was doing
    const char *kernel;     // what it waited for
    int device;
    uint32_t frame;
};

[[noreturn]] void stall_exit(const WaitSite &w, const char *how, double waited_ms) {
    fprintf(stderr, "s3r: stall: %s -- waited %.0f ms for %s (%s; device %d, frame %u, S3R_WAIT_MS %d); exiting with "
            "status %d\n", w.stage, waited_ms, w.kernel, how, w.device, w.frame, wait_deadline_ms(), kStallExit);
    fflush(stderr);
    _exit(kStallExit);
}

[[noreturn]] void fault_exit(const WaitSite &w, hipError_t e) {
    fprintf(stderr, "s3r: HIP error %s while waiting for %s (%s; device %d, frame %u)\n", hipGetErrorName(e), w.kernel,
            w.stage, w.device, w.frame);
    fflush(stderr);
    abort();
}

// The watchdog: one slot per thread that makes blocking HIP calls (the caller's thread and the
// device workers), armed with a deadline and the call's site for the duration of the call.
class Watchdog {
  public:
    struct Guard {
        Guard(const WaitSite &w) : slot_(instance().arm(w)) {}
        ~Guard() { instance().disarm(slot_); }
        int slot_;
    };
    static Watchdog &instance() {
        static Watchdog *w = new Watchdog();   // never destroyed: the thread outlives static teardown
        return *w;
    }

  private:
    static constexpr int kSlots = 128;
    struct Slot {
        std::atomic<int64_t> deadline{0};      // 0: disarmed
        std::atomic<int64_t> start{0};
        WaitSite site{"", "", -1, 0};
        std::atomic<bool> used{false};
    };
    Slot slots_[kSlots];
    std::once_flag started_;

    // this thread's slot, taken on its first armed call and returned when the thread ends
    struct Owner {
        int idx = -1;
        ~Owner() { if (idx >= 0) instance().slots_[idx].used.store(false, std::memory_order_release); }
    };
    int my_slot() {
        thread_local Owner o;
        if (o.idx < 0) {
            for (int i = 0; i < kSlots && o.idx < 0; i++) {
                bool f = false;
                if (slots_[i].used.compare_exchange_strong(f, true, std::memory_order_acq_rel)) o.idx = i;
            }
            if (o.idx < 0) {
                fprintf(stderr, "s3r: watchdog: more than %d threads wait on the GPU at once\n", kSlots);
                abort();
            }
        }
        return o.idx;
    }
    int arm(const WaitSite &w) {
        std::call_once(started_, [this] { std::thread([this] { run(); }).detach(); });
        const int i = my_slot();
        Slot &s = slots_[i];
        s.site = w;
        const int64_t now = mono_ns();
        s.start.store(now, std::memory_order_relaxed);
        s.deadline.store(now + (int64_t)wait_deadline_ms() * 1000000, std::memory_order_release);
        return i;
    }
    void disarm(int i) { slots_[i].deadline.store(0, std::memory_order_release); }
    [[noreturn]] void run() {
        const int period_ms = std::max(2, std::min(250, wait_deadline_ms() / 8));
        for (;;) {
            std::this_thread::sleep_for(std::chrono::milliseconds(period_ms));
            const int64_t now = mono_ns();
            for (Slot &s : slots_) {
                const int64_t d = s.deadline.load(std::memory_order_acquire);
                if (d && now > d) {
                    const WaitSite w = s.site;    // (its thread is blocked in the call: the site is stable)
                    stall_exit(w, "a blocking HIP call did not return",
                               (double)(now - s.start.load(std::memory_order_relaxed)) / 1e6);
                }
            }
        }
    }
};

// Blocking synchronisations under the watchdog.
void sync_device(const char *stage, int device = -1, uint32_t frame = 0) {
    Watchdog::Guard guard(WaitSite{stage, "every kernel and copy of the device", device, frame});
    HIPCHECK(hipDeviceSynchronize());
}
void sync_stream(hipStream_t st, const WaitSite &w) {
    Watchdog::Guard guard(w);
    HIPCHECK(hipStreamSynchronize(st));
}
void sync_event(hipEvent_t ev, const WaitSite &w) {
    Watchdog::Guard guard(w);
    HIPCHECK(hipEventSynchronize(ev));
}

// One poll of a stream the host is spinning on: true when it has drained (a device fault ends the
// process with its name), a stall exit once `t0` is past the deadline.
bool stream_drained(hipStream_t st, const WaitSite &w, int64_t t0) {
    const hipError_t e = hipStreamQuery(st);
    if (e == hipSuccess) return true;
    if (e != hipErrorNotReady) fault_exit(w, e);
    const int64_t waited = mono_ns() - t0;
    if (waited > (int64_t)wait_deadline_ms() * 1000000) stall_exit(w, "its stream never drained", (double)waited / 1e6);
    return false;
}

// Test hooks for the deadline tests (tests/test_stall.py), read once, acting from a device's second
// frame on (the first one initialises the library): S3R_TEST_HOLD_MS puts a kernel that spins that
// long (and then exits) in front of every frame's geometry / tile setup; S3R_TEST_ARRIVALS_EXTRA
// makes the sky-flag publishers wait for that many arrivals more than the launch has.
uint32_t env_u32(const char *name) {
    const char *e = getenv(name);
    const long v = e ? atol(e) : 0;
    return v > 0 ? (uint32_t)std::min<long>(v, 60000L) : 0u;
}
uint32_t test_hold_ms() { static const uint32_t v = env_u32("S3R_TEST_HOLD_MS"); return v; }
uint32_t test_extra_arrivals() { static const uint32_t v = env_u32("S3R_TEST_ARRIVALS_EXTRA"); return v; }

struct TimingSlot { hipEvent_t frame0, geo1, frag0, frag1; };   // geo1: the frame's geometry / setup stage done

// Per-frame buffer sets in flight: frame k's geometry writes set k % kSets once the fragment kernel
// of frame k - kSets (the set's last reader) is done, on geometry stream k % kGeoStreams, so the
// geometry of two consecutive frames and the previous frame's fragment kernel can all overlap.
constexpr int kSets = 4;
#ifndef S3R_GEO_STREAMS
#define S3R_GEO_STREAMS 2
#endif
constexpr int kGeoStreams = S3R_GEO_STREAMS;
constexpr uint64_t kLptMinBins = 2000;      // longest-first fragment order from this many bins (~1.5 rounds; see render_core)
// Slots above which the row path's start table (2T x H x segments x 16 B) is not worth building:
// the order-independent tile path takes over (the icosahedron stress scene).
constexpr uint64_t kRowPathMaxSlots = 8192;
constexpr uint64_t kNearCheckMaxTri = 1024;   // the host's near-plane check: scenes up to this many triangles
constexpr uint32_t kDefaultBand = 16;       // rows per interleaved band when updateAndRender spans devices
constexpr uint32_t kSumWords = 8;           // tile path: host-coherent summary words per buffer set
constexpr int kMaxDevices = 64;

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
    void report(int device) {
        if (!on || !frames) return;
        fprintf(stderr, "s3r hostprof device %d (us/frame over %llu): begin %.2f  prep %.2f  geo-wait %.2f  "
                "geo-launch %.2f  frag-wait %.2f  frag-launch %.2f\n", device, (unsigned long long)frames,
                t[0] / frames, t[1] / frames, t[2] / frames, t[3] / frames, t[4] / frames, t[5] / frames);
    }
};

// One GPU: its replica of the scene, its per-frame buffer sets, streams and frame tags.

struct Dev {
    int device = -1;
    float4 *vtx = nullptr, *nrm = nullptr, *pay = nullptr;
    uint8_t *disc = nullptr;
    uint32_t *vidx = nullptr, *aidx = nullptr, *tex = nullptr;
    // per-frame geometry, kSets buffer sets: frame k's geometry (k_geometry on a geometry stream)
    // overlaps earlier frames' fragment kernels on the caller's stream
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
    void *scan_temp = nullptr;                 // rocprim scan of the (tile, bucket) counts
    size_t scan_temp_bytes = 0;
    float4 *vrv = nullptr;                     // tile path vertex stage (frame parts): projected vertices
    void *recs[kSets] = {};        // 2T raster records (positions-only setup)
    uint4 *live[kSets] = {};       // 2T live entries (tile box, rows, slot), per shard
    uint32_t *clipq = nullptr;     // T: positions whose triangle crosses the near plane (one: setups run on geo[0])
    uint32_t *tile_ctr[kSets] = {};  // kTileCounterWords: live count, list total, cluster-kept triangles
    // init-time clusters (clusters.cpp): spheres, position ranges, position -> slot (null: identity),
    // and the cull's per-frame position list (one: every tile-path setup runs on geo[0])
    float4 *cl_sphere = nullptr;
    uint32_t *cl_first = nullptr, *cl_perm = nullptr, *cl_shard = nullptr, *cl_map = nullptr;
    uint64_t tiles_cap = 0, tile_list_cap[kSets] = {};
    uint4 *deferred = nullptr;                 // fused raster + resolve: pixels whose winner needs a full setup
    size_t deferred_cap = 0;
    // bins (the default; S3R_TILE_BINS=0: the lists): per buffer set, bin_cap entries for every (tile, bucket) slot
    uint32_t *tbin[kSets] = {};
    uint64_t tbin_slots[kSets] = {};           // slots each set's bins were allocated for
    uint32_t bin_cap = 0;                      // entries per slot (grown when a frame overflows)
    uint64_t bin_regrows = 0;                  // frames binned again into larger bins
    bool bins_off = false;                     // bins past the memory budget: this device uses the lists
    // host-coherent, per buffer set: {tag, live entries, list length, cluster-kept positions}, written
    // by k_tile_cursor as soon as they are known (tag = the frame's number)
    uint32_t *tile_sum_host = nullptr, *tile_sum_dev = nullptr;
    // a synchronous tile-path frame awaiting its overflow check (tile_redo_if_overflowed): its set
    // and what its fragment stage needs to run again
    bool tile_pending = false, tile_pending_bins = false;
    uint32_t tile_xoff = 0;                    // the current frame's tile-grid shift (tile_xoff_for)
    uint32_t tile_pending_set = 0, tile_W = 0, tile_H = 0, tile_band = 0, tile_nparts = 1, tile_part = 0, tile_rows = 0;
    uint32_t *tile_out = nullptr;
    bool tile_frame_rows = false;
    uint64_t tile_overflows = 0, tile_readbacks = 0;
    uint64_t last_pairs = 0;                   // tile path: (slot, tile) pairs of the last frame
    int last_set = -1;                         // tile path: the last frame's buffer set (refresh_pairs)
    bool last_set_bins = false;                // ... binned (its entry total arrives at the frame's end)
    uint64_t last_live = 0, last_kept = 0;     // tile path, last read-back frame: live slots, cluster-kept triangles
    int last_path = 0;                         // 1 rows, 2 tiles: the last frame's fragment stage
    hipEvent_t geo_done[kSets] = {}, frag_done[kSets] = {};
    // row path, buffer-set reuse without events: each k_fragment launch stores the tag of the previous
    // fragment launch (complete by stream order) in *done_host (host-coherent memory; done_dev is its
    // device address); issued_tag[p] = the tag of the last fragment launch that read set p (0: none);
    // last_tag = the previous row-path fragment launch, last_stream = the stream of the previous frame
    // (either path)
    volatile uint32_t *done_host = nullptr;
    uint32_t *done_dev = nullptr;
    // kDiagWords device error words (host-coherent, in done_host's allocation): a device spin that
    // passed its deadline reports there (s3r_kernels.h GeoSkyFlags::err)
    uint32_t *diag_host = nullptr, *diag_dev = nullptr;
    uint32_t *geo_cnt = nullptr;             // host fill: per buffer set, k_geometry's bin-phase count
    uint32_t issued_tag[kSets] = {}, last_tag = 0;
    // the previous frame's stream; NULL is a valid caller stream (the legacy default stream), so
    // whether a previous frame exists is its own flag
    hipStream_t last_stream = nullptr;
    bool have_last = false;
    hipEvent_t handoff = nullptr;
    uint32_t frame_no = 0;                     // frames issued: set frame_no % kSets
    uint32_t *frame = nullptr;                 // updateAndRender: this device's rows of the frame
    size_t frame_cap = 0;
    hipStream_t stream = nullptr, geo[kGeoStreams] = {};
    std::vector<TimingSlot> tslots;
    size_t tcount = 0;
    HostProf hp;
    // host fill: one flag per fragment bin (host-coherent; k_sky_flags), this device's tag sequence,
    // and the device address of the caller-buffer registration the last host-fill frame used
    uint32_t *fill_flags = nullptr, *fill_flags_dev = nullptr;
    unsigned long long *fill_chunks = nullptr, *fill_chunks_dev = nullptr;   // per bin: (tag << 32) | chunk mask
    uint64_t fill_cap = 0;
    uint32_t fill_tag = 0;
    uintptr_t map_host = 0, map_dev = 0;
    uint64_t map_epoch = 0;
};

// The scene as read from data.bin (render.cpp:177-209), converted to the device layout once and
// uploaded to every device.
struct HostScene {
    std::vector<float4> vtx, nrm, pay;
    std::vector<uint8_t> disc;
    std::vector<uint32_t> vidx, aidx, tex;
    std::vector<uint32_t> cl_first, cl_perm;   // clusters (tile path): position ranges, position -> slot
    std::vector<uint32_t> cl_shard;            // where each shard's positions start (cluster_shard_table)
    std::vector<float> cl_sphere;              // 4 per cluster: centre, radius
};

// Persistent worker threads, one per device beyond the first: run(fn, arg, n) calls fn(arg, 0) on
// the calling thread and fn(arg, i) on worker i for 0 < i < n, and returns when all have returned.
// Workers spin briefly on the frame generation (back-to-back frames hand over in ~1 us) and then
// sleep on a condition variable (a 60 Hz caller does not keep cores busy).
class Pool {
  public:
    // cpus (optional): worker i runs on the CPUs of cpus[i - 1]
    void start(int workers, const std::vector<cpu_set_t> *cpus = nullptr) {
        stop();
        stop_.store(false);
        // each worker starts from the generation of now: a run() issued before it is scheduled is
        // still seen as new
        const uint64_t g0 = gen_.load(std::memory_order_acquire);
        for (int i = 1; i <= workers; i++) {
            cpu_set_t set;
            const bool pin = cpus && (size_t)i <= cpus->size();
            if (pin) set = (*cpus)[i - 1];
            th_.emplace_back([this, i, g0, pin, set] {
                if (pin) (void)pthread_setaffinity_np(pthread_self(), sizeof set, &set);
                loop(i, g0);
            });
        }
    }
    void stop() {
        if (th_.empty()) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_.store(true);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_work_.notify_all();
        for (auto &t : th_) t.join();
        th_.clear();
    }
    // fn(arg, i) on workers 0 < i < n, asynchronously; join() waits for them
    void launch(void (*fn)(void *, int), void *arg, int n) {
        launched_ = n > 1;
        if (!launched_) return;
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = fn;
            arg_ = arg;
            active_ = n;
            pending_.store(n - 1, std::memory_order_relaxed);
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_work_.notify_all();
    }
    void join() {
        if (!launched_) return;
        launched_ = false;
        if (!spin([&] { return pending_.load(std::memory_order_acquire) == 0; })) {
            std::unique_lock<std::mutex> lk(mu_);
            cv_done_.wait(lk, [&] { return pending_.load(std::memory_order_acquire) == 0; });
        }
    }
    void run(void (*fn)(void *, int), void *arg, int n) {
        launch(fn, arg, n);
        fn(arg, 0);
        join();
    }
    int workers() const { return (int)th_.size(); }
    ~Pool() { stop(); }

  private:
    template <class Pred> static bool spin(Pred done) {
        const auto t0 = std::chrono::steady_clock::now();
        for (uint32_t k = 1;; k++) {
            if (done()) return true;
            __builtin_ia32_pause();
            if ((k & 255u) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(2000)) return done();
        }
    }
    void loop(int idx, uint64_t seen) {
        for (;;) {
            if (!spin([&] { return gen_.load(std::memory_order_acquire) != seen; })) {
                std::unique_lock<std::mutex> lk(mu_);
                cv_work_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
            }
            seen = gen_.load(std::memory_order_acquire);
            if (stop_.load()) return;
            void (*fn)(void *, int);
            void *arg;
            int active;
            {
                std::lock_guard<std::mutex> lk(mu_);
                fn = fn_; arg = arg_; active = active_;
            }
            if (idx >= active) continue;     // (run() with fewer parts than workers: not used)
            fn(arg, idx);
            if (pending_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
                std::lock_guard<std::mutex> lk(mu_);
                cv_done_.notify_all();
            }
        }
    }
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_work_, cv_done_;
    std::atomic<uint64_t> gen_{0};
    std::atomic<int> pending_{0};
    std::atomic<bool> stop_{false};
    void (*fn_)(void *, int) = nullptr;
    void *arg_ = nullptr;
    int active_ = 0;
    bool launched_ = false;
};

struct Lib {
    bool initialized = false;
    std::string data_path;     // "" = reference search
    int device = -1;           // s3r_configure: the single device (-1: S3R_DEVICE or the current one)
    std::vector<int> device_ids;   // s3r_configure_devices: updateAndRender's devices (empty: single)
    uint32_t band_rows = 0;        // rows per interleaved band across devices (0: S3R_BAND or 16)

    // camera state, render.cpp:51-65
    F3 pos{0, 0, 0}, ax{1, 0, 0}, ay{0, 1, 0}, az{0, 0, 1};
    Mat34 m{{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1, 0}}};
    float mouse[2] = {0, 0};
    // config, render.cpp:81-97
    float factor = 1;
    uint32_t depth_buffer_size = 0;

    // scene counts (the same on every device)
    uint32_t nv = 0, na = 0, ntri = 0, ntex = 0;
    uint64_t nindices = 0;
    uint32_t ncl = 0;                          // clusters (clusters.cpp; 0: the scene has none)
    // row-path scenes up to kNearCheckMaxTri triangles: positions and vertex indices kept on the host
    // for the per-frame near-plane check (near_plane_crossing)
    std::vector<float4> near_vtx;
    std::vector<uint32_t> near_vidx;
    std::vector<uint8_t> near_side;
    bool clip_slots = true;                    // this frame: launch k_geometry's clip-appended slots
    SlotMask live{};                           // this frame: the slots k_geometry launches (cull_slots)
    // the camera state clip_slots and live were computed for (frame_begin: unchanged -> reused)
    struct CullKey { Mat34 m; float factor; uint32_t W, H; bool valid; } cull_key{};
    std::vector<double> near_rv;               // per vertex: screen x, y and their error bound (cull_slots)
    bool clusters = true;                      // tile path: cull clusters before the setup (S3R_CLUSTERS)
    bool clusters_whole = false;               // ... also for whole frames (S3R_CLUSTERS=2)
    int raster_path = 0;                       // 0 auto, 1 rows (k_geometry + k_fragment), 2 tiles
    bool tile_line_grid = true;                // tile path, direct delivery: tiles on the caller's line grid (S3R_TILE_LINE)
    bool tile_bins = true;                     // tile path: fixed-capacity bins filled by the setup (S3R_TILE_BINS)
    uint64_t tile_bin_budget = 32ull << 30;    // bytes of bins per device, all buffer sets (S3R_TILE_BIN_BUDGET_MB)
    bool serial = false;                       // S3R_SERIAL: no geometry/fragment overlap (profiling)
    bool timing = false;

    std::vector<Dev *> devs;                   // devs[0]: s3r_render_bands' device, updateAndRender's first
    uint32_t band = 0;                         // resolved band_rows (0: per frame, frame_band)
    Pool pool;

    // caller buffers registered as pinned memory (the double buffer: main.swift:117-118, :164):
    // byte ranges [a, b) whose pages do not overlap; a request whose pages overlap existing ranges is
    // merged with them into one registration, so two halves of one allocation -- which share the
    // page at the seam -- end up in one registration that covers both
    struct Reg { uintptr_t a, b; bool ok; };
    std::vector<Reg> regs;
    uint64_t stale_pins = 0;                   // registrations found stale and replaced (updateAndRender)
    uint64_t pinned_frames = 0, pageable_frames = 0, registrations = 0, merges = 0;
    uint64_t reg_epoch = 1;                    // bumped whenever a registration goes away

    // updateAndRender's delivery into the caller's buffer (see "deliveries" below): -1 unset (the
    // S3R_DELIVERY environment or auto), 0 auto, 1 copy, 2 direct, 3 host fill
    int delivery = -1;
    int fill_threads = -1;                     // host fill threads; -1: S3R_FILL_THREADS or the default
    Pool fill_pool;
    int fill_node = -2;                        // NUMA node the fill threads were placed for
    bool fill_placed = false;                  // fill threads pinned one per CPU domain (fill_placement)
    uint64_t copy_frames = 0, direct_frames = 0, fill_frames = 0;
    // adaptive host fill: eighths of the sky bins the GPUs write themselves, and the smoothed
    // (fill threads' finish - devices' finish) in microseconds that steers it
    int fill_gpu = -1;
    double fill_skew_us = 0;                   // smoothed (threads' sky-fill end - devices' end)
    double fill_eighth_us = 0;                 // smoothed F: the threads' fill time per eighth (0: none yet)
    // s3r_fill_profile: frames, sums of the devices' / fill threads' finish times (ns after the
    // frame's start), and per fill thread its last CPU, summed finish time and pixels
    uint64_t prof_frames = 0, prof_dev_ns = 0, prof_fill_ns = 0, prof_pre_ns = 0, prof_issued_ns = 0, prof_done_ns = 0;
    std::chrono::steady_clock::time_point call_t0;     // updateAndRender's entry (the profile's pre_ns)
    struct ThreadProf { int64_t cpu = -1; uint64_t end_ns = 0, px = 0, covered_ns = 0; } prof_thread[65];
    // a device could not map the registration starting at unmapped_a (in registration epoch
    // unmapped_epoch): frames into it go by copy; other registrations still try the mapping
    uintptr_t unmapped_a = 0;
    uint64_t unmapped_epoch = 0;
    // environment switches read once per library state (release_all resets them: a configure re-reads)
    // fill-thread placement: frames in a row whose buffer sat on another node than the placement's
    int fill_node_streak = 0;
    uint64_t link_bytes = 0;                   // bytes the devices sent over their links, last frame
    // s3r_device_profile: per device behind updateAndRender, frames, the sum of its part's finish
    // times (ns after the call's entry: rendered and in the caller's buffer) and its link bytes of
    // the last frame
    struct DevProf { uint64_t frames = 0, end_ns = 0, link_bytes = 0; } dev_prof[kMaxDevices];
};

Lib g;

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

HostScene read_scene() {
    const std::string path = find_data_path();
    FILE *fp = path.empty() ? nullptr : fopen(path.c_str(), "rb");
    if (!fp) exit(666);                                                 // render.cpp:173
    auto rd = [&](void *dst, size_t bytes) {
        if (bytes && fread(dst, 1, bytes, fp) != bytes) bad_scene(path, "truncated");
    };
    uint64_t cnt[2];
    rd(cnt, 16);
    const uint64_t nv = cnt[0];
    HostScene s;
    s.vtx.resize(nv);
    rd(s.vtx.data(), nv * 16);
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
    s.tex.resize(nt);
    rd(s.tex.data(), nt * 4);
    fclose(fp);

    // The reference trusts the file; the GPU must not read out of bounds, so check it here.
    if (nv >= (1ull << 32) || na >= (1ull << 32) || nt >= (1ull << 32)) bad_scene(path, "too large");
    if (nai < ni) bad_scene(path, "fewer attribute indices than vertex indices");
    const uint64_t ntri = ni / 3;
    s.vidx.resize(3 * ntri);
    s.aidx.resize(3 * ntri);
    for (uint64_t k = 0; k < 3 * ntri; k++) {
        if (vi[k] < 0 || (uint64_t)vi[k] >= nv) bad_scene(path, "vertex index out of range");
        if (ai[k] < 0 || (uint64_t)ai[k] >= na) bad_scene(path, "attribute index out of range");
        s.vidx[k] = (uint32_t)vi[k];
        s.aidx[k] = (uint32_t)ai[k];
    }
    s.nrm.resize(na);
    s.pay.resize(na);
    s.disc.resize(na);
    for (uint64_t k = 0; k < na; k++) {
        memcpy(&s.nrm[k], &attr[48 * k], 16);
        memcpy(&s.pay[k], &attr[48 * k + 16], 16);
        uint32_t d;
        memcpy(&d, &attr[48 * k + 32], 4);                              // disc_t at +32
        s.disc[k] = d != 0;
    }
    g.nv = (uint32_t)nv; g.na = (uint32_t)na; g.ntri = (uint32_t)ntri; g.ntex = (uint32_t)nt;
    g.nindices = ni;
    g.near_vtx.clear(); g.near_vidx.clear();
    g.cull_key.valid = false;
    if (ntri <= kNearCheckMaxTri && 2 * ntri <= kRowPathMaxSlots) { g.near_vtx = s.vtx; g.near_vidx = s.vidx; }
    // clusters for the tile path's per-frame cull (scenes the tile path renders by default, or any
    // scene with S3R_CLUSTERS=2): connected meshes of 8-32 triangles, larger ones cut, smaller pooled
    const char *ce = getenv("S3R_CLUSTERS");
    g.clusters = !(ce && atoi(ce) == 0);
    g.clusters_whole = ce && atoi(ce) == 2;
    if (g.clusters && (2 * ntri > kRowPathMaxSlots || (ce && atoi(ce) == 2)))
        s3r_host::build_clusters(reinterpret_cast<const float *>(s.vtx.data()), (uint32_t)nv, s.vidx.data(),
                                 (uint32_t)ntri, 8, 32, s.cl_first, s.cl_sphere, s.cl_perm);
    g.ncl = s.cl_first.empty() ? 0 : (uint32_t)s.cl_first.size() - 1;
    if (g.ncl) s.cl_shard = cluster_shard_table(s.cl_first);
    return s;
}

// The scene's upload: every array copied through one page-locked staging buffer of the library's own
// (hipHostMalloc) in 16-MiB pieces on the device's stream.  Not the runtime's pageable hipMemcpy:
// that path may take a source address for user memory a registration once covered (the tests free
// caller buffers the library had page-locked, and the heap reuses their addresses) -- round 4 and
// round 6 each saw an illegal-address error at a scene load's third upload.
struct Uploader {
    static constexpr size_t kPiece = 16u << 20;
    Dev &d;
    void *stage = nullptr;
    explicit Uploader(Dev &dev) : d(dev) { HIPCHECK(hipHostMalloc(&stage, kPiece, hipHostMallocDefault)); }
    ~Uploader() { if (stage) (void)hipHostFree(stage); }
    void put(void *dst, const void *src, size_t bytes) {
        for (size_t o = 0; o < bytes; o += kPiece) {
            const size_t n = std::min(kPiece, bytes - o);
            memcpy(stage, static_cast<const uint8_t *>(src) + o, n);
            HIPCHECK(hipMemcpyAsync(static_cast<uint8_t *>(dst) + o, stage, n, hipMemcpyHostToDevice, d.stream));
            sync_stream(d.stream, WaitSite{"scene upload", "a host-to-device copy", d.device, 0u});
        }
    }
};

void dev_init(Dev &d, const HostScene &s) {
    HIPCHECK(hipSetDevice(d.device));
    HIPCHECK(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
    const uint32_t ntri = g.ntri;
    d.vtx = dalloc<float4>(g.nv); d.nrm = dalloc<float4>(g.na); d.pay = dalloc<float4>(g.na);
    d.disc = dalloc<uint8_t>(g.na);
    d.vidx = dalloc<uint32_t>(3 * (size_t)ntri); d.aidx = dalloc<uint32_t>(3 * (size_t)ntri);
    d.tex = dalloc<uint32_t>(g.ntex);
    for (int p = 0; p < kSets; p++) {           // (the row path's TriSetup records: ensure_row_sets)
        HIPCHECK(hipEventCreateWithFlags(&d.geo_done[p], hipEventDisableTiming));
        HIPCHECK(hipEventCreateWithFlags(&d.frag_done[p], hipEventDisableTiming));
    }
    {
        void *h = nullptr;
        // word 0: the completion tag (wait_set_free); words 4 .. 4 + kDiagWords: the error words
        constexpr size_t kWords = 4 + kDiagWords;
        HIPCHECK(hipHostMalloc(&h, kWords * sizeof(uint32_t), hipHostMallocCoherent | hipHostMallocMapped));
        memset(h, 0, kWords * sizeof(uint32_t));
        d.done_host = static_cast<volatile uint32_t *>(h);
        HIPCHECK(hipHostGetDevicePointer((void **)&d.done_dev, h, 0));
        d.diag_host = static_cast<uint32_t *>(h) + 4;
        d.diag_dev = d.done_dev + 4;
        HIPCHECK(hipEventCreateWithFlags(&d.handoff, hipEventDisableTiming));
    }
    // geometry streams at the highest priority: their (small, latency-bound) workgroups are
    // dispatched as soon as the previous frame's fragment workgroups free a slot
    int prio_least = 0, prio_greatest = 0;
    HIPCHECK(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest));
    // (the default priority instead measured the same for pipelined HBM frames, profiles/r05_order_ab.txt)
    // (round 6, frame parts: the default priority measured the same, profiles/r06_part_negatives.txt)
    for (hipStream_t &gs : d.geo) HIPCHECK(hipStreamCreateWithPriority(&gs, hipStreamNonBlocking, prio_greatest));
    // (a fault pending from before -- the previous scene's release, its allocations -- is reported here
    // as such, not by the uploads below; round 4 and round 6 each saw one illegal-address error at the
    // third upload of a scene load in the tile suite)
    {
        const hipError_t e = hipDeviceSynchronize();
        if (e != hipSuccess) {
            fprintf(stderr, "s3r: HIP error %s on device %d before the scene upload (a fault pending from the "
                    "previous scene's release or this scene's allocations)\n", hipGetErrorName(e), d.device);
            fflush(stderr);
            abort();
        }
    }
    Uploader up(d);
    up.put(d.vtx, s.vtx.data(), (size_t)g.nv * 16);
    up.put(d.nrm, s.nrm.data(), (size_t)g.na * 16);
    up.put(d.pay, s.pay.data(), (size_t)g.na * 16);
    up.put(d.disc, s.disc.data(), g.na);
    up.put(d.vidx, s.vidx.data(), 12 * (size_t)ntri);
    up.put(d.aidx, s.aidx.data(), 12 * (size_t)ntri);
    up.put(d.tex, s.tex.data(), (size_t)g.ntex * 4);
    if (g.ncl) {
        d.cl_sphere = dalloc<float4>(g.ncl);
        d.cl_first = dalloc<uint32_t>((size_t)g.ncl + 1);
        d.cl_map = dalloc<uint32_t>(ntri);
        d.cl_shard = dalloc<uint32_t>(kTileShards + 1);
        up.put(d.cl_shard, s.cl_shard.data(), (kTileShards + 1) * 4);
        up.put(d.cl_sphere, s.cl_sphere.data(), (size_t)g.ncl * 16);
        up.put(d.cl_first, s.cl_first.data(), ((size_t)g.ncl + 1) * 4);
        if (!s.cl_perm.empty()) {
            d.cl_perm = dalloc<uint32_t>(ntri);
            up.put(d.cl_perm, s.cl_perm.data(), (size_t)ntri * 4);
        }
    }
}

// "0,1,2" -> {0, 1, 2}; empty on a malformed list.
std::vector<int> parse_devices(const char *s) {
    std::vector<int> ids;
    while (s && *s) {
        char *end = nullptr;
        const long v = strtol(s, &end, 10);
        if (end == s || v < 0 || v > INT_MAX) return {};
        ids.push_back((int)v);
        s = end;
        while (*s == ',' || *s == ' ') s++;
    }
    if ((int)ids.size() > kMaxDevices) return {};
    return ids;
}

void initialize() {
    const HostScene s = read_scene();
    std::vector<int> ids = g.device_ids;
    if (ids.empty()) ids = parse_devices(getenv("S3R_DEVICES"));
    if (ids.empty()) {
        int dev = g.device;
        if (dev < 0) {
            if (const char *e = getenv("S3R_DEVICE")) dev = atoi(e);
            else HIPCHECK(hipGetDevice(&dev));
        }
        ids.push_back(dev);
    }
    g.band = g.band_rows;
    if (!g.band) {
        const char *e = getenv("S3R_BAND");
        g.band = e && atoi(e) > 0 ? (uint32_t)atoi(e) : 0u;
    }
    g.serial = getenv("S3R_SERIAL") != nullptr;
    {
        const char *l = getenv("S3R_TILE_LINE");
        g.tile_line_grid = !(l && atoi(l) == 0);
        const char *tb = getenv("S3R_TILE_BINS");
        g.tile_bins = !(tb && atoi(tb) == 0);
        const char *bb = getenv("S3R_TILE_BIN_BUDGET_MB");
        if (bb && atoll(bb) > 0) g.tile_bin_budget = (uint64_t)atoll(bb) << 20;
    }
    for (int id : ids) {
        Dev *d = new Dev();
        d->device = id;
        dev_init(*d, s);
        g.devs.push_back(d);
    }
    HIPCHECK(hipSetDevice(g.devs[0]->device));
    if (g.devs.size() > 1) g.pool.start((int)g.devs.size() - 1);
}

// Wait for every device of the library (no copy into a caller buffer may still be in flight).
void drain_devices() {
    for (Dev *d : g.devs) {
        HIPCHECK(hipSetDevice(d->device));
        sync_device("drain: every device before host registrations go", d->device, d->frame_no);
    }
    if (g.devs.empty()) sync_device("drain: the device before host registrations go");
    else HIPCHECK(hipSetDevice(g.devs[0]->device));
}

// Drops every host registration.  A registration may belong to a host frame s3r_bands_to_host is
// still filling (its copies are asynchronous), so the devices are drained first.
void unregister_all() {
    bool any = false;
    for (auto &r : g.regs) any |= r.ok;
    if (any) drain_devices();
    for (auto &r : g.regs)
        if (r.ok) (void)hipHostUnregister((void *)r.a);
    g.regs.clear();
    g.reg_epoch++;
}

// Every call's status is checked (round 6: a device fault that surfaced at the third upload of the
// next scene could have been raised -- and discarded -- here); the first failure is reported with
// the call and the device, then the process aborts.
void dev_release(Dev &d) {
    hipError_t first = hipSuccess;
    const char *what = "";
    auto chk = [&](hipError_t e, const char *w) {
        if (e != hipSuccess && first == hipSuccess) { first = e; what = w; }
    };
    chk(hipSetDevice(d.device), "hipSetDevice");
    void *ptrs[] = {d.vtx, d.nrm, d.pay, d.disc, d.vidx, d.aidx, d.tex, d.frame, d.deferred, d.scan_temp, d.vrv, d.geo_cnt,
                    d.cl_sphere, d.cl_first, d.cl_perm, d.cl_map, d.cl_shard, d.clipq};
    for (void *p : ptrs)
        if (p) chk(hipFree(p), "hipFree (scene / frame buffers)");
    for (int q = 0; q < kSets; q++) {      // tile_total aliases tile_ctr
        void *set[] = {d.tris[q], d.rowtab[q], d.bincnt[q], d.pairs[q], d.order[q], d.tile_counts[q], d.tile_offs[q],
                       d.tile_cursor[q], d.tile_list[q], d.recs[q], d.live[q], d.tile_ctr[q], d.tbin[q]};
        for (void *p : set)
            if (p) chk(hipFree(p), "hipFree (buffer sets)");
    }
    if (d.done_host) chk(hipHostFree((void *)d.done_host), "hipHostFree (completion and error words)");
    if (d.handoff) chk(hipEventDestroy(d.handoff), "hipEventDestroy");
    if (d.tile_sum_host) chk(hipHostFree(d.tile_sum_host), "hipHostFree (tile summary)");
    if (d.fill_flags) chk(hipHostFree(d.fill_flags), "hipHostFree (fill flags)");
    if (d.fill_chunks) chk(hipHostFree(d.fill_chunks), "hipHostFree (fill chunk masks)");
    for (int p = 0; p < kSets; p++) {
        if (d.geo_done[p]) chk(hipEventDestroy(d.geo_done[p]), "hipEventDestroy");
        if (d.frag_done[p]) chk(hipEventDestroy(d.frag_done[p]), "hipEventDestroy");
    }
    for (hipStream_t gs : d.geo)
        if (gs) chk(hipStreamDestroy(gs), "hipStreamDestroy (geometry)");
    for (auto &t : d.tslots) {
        chk(hipEventDestroy(t.frame0), "hipEventDestroy"); chk(hipEventDestroy(t.geo1), "hipEventDestroy");
        chk(hipEventDestroy(t.frag0), "hipEventDestroy"); chk(hipEventDestroy(t.frag1), "hipEventDestroy");
    }
    if (d.stream) chk(hipStreamDestroy(d.stream), "hipStreamDestroy");
    // the frees and destructions above complete before anything else runs on the device
    if (first == hipSuccess) {
        Watchdog::Guard guard(WaitSite{"release: after freeing the device's memory", "the device", d.device, d.frame_no});
        chk(hipDeviceSynchronize(), "hipDeviceSynchronize after the frees");
    }
    if (first != hipSuccess) {
        fprintf(stderr, "s3r: HIP error %s from %s on device %d while releasing the library's memory\n",
                hipGetErrorName(first), what, d.device);
        fflush(stderr);
        abort();
    }
}

void release_all() {
    g.pool.stop();
    g.fill_pool.stop();
    if (g.initialized) {
        // a device fault of an earlier frame surfaces here at the latest: report it as such (the
        // context is unusable after it) rather than in whatever HIP call comes next
        for (Dev *d : g.devs) {
            hipError_t e = hipSetDevice(d->device);
            if (e == hipSuccess) {
                Watchdog::Guard guard(WaitSite{"release: draining the device", "every kernel of the device", d->device,
                                               d->frame_no});
                e = hipDeviceSynchronize();
            }
            if (e != hipSuccess) {
                fprintf(stderr, "s3r: HIP error %s on device %d while releasing the library: a fault of an "
                        "earlier frame's kernels (run with S3R_CHECK=1 to name the launch)\n", hipGetErrorName(e),
                        d->device);
                abort();
            }
        }
        unregister_all();
        for (Dev *d : g.devs) {
            dev_release(*d);
            delete d;
        }
        g.devs.clear();
    } else {
        unregister_all();
    }
    const std::string path = g.data_path;
    const int dev = g.device, rp = g.raster_path;
    const std::vector<int> ids = g.device_ids;
    const uint32_t band = g.band_rows;
    const int fill = g.fill_threads, delivery = g.delivery;
    g.~Lib();
    new (&g) Lib();
    g.fill_threads = fill;
    g.delivery = delivery;
    g.data_path = path;
    g.device = dev;
    g.raster_path = rp;
    g.device_ids = ids;
    g.band_rows = band;
}

bool near_plane_crossing();
void cull_slots(uint32_t W, uint32_t H);

// render.cpp:266-280: first-call init, camera, resize.
void frame_begin(const Input *input, uint32_t width, uint32_t height) {
    if (!g.initialized) {
        g.initialized = true;
        initialize();
        update_camera(input, true);
    } else {
        update_camera(input, false);
        HIPCHECK(hipSetDevice(g.devs[0]->device));
    }
    const uint32_t dbs = width * height * (uint32_t)sizeof(float);
    if (g.depth_buffer_size != dbs) {
        g.depth_buffer_size = dbs;
        g.factor = kNear * (float)height / (2 * config_scale());          // render.cpp:279
        unregister_all();
    }
    // the near-plane check and the slot cull depend on the camera matrix, factor and frame size only
    // (and the scene, whose load invalidates the key): a frame that repeats them reuses their result
    Lib::CullKey &k = g.cull_key;
    if (k.valid && k.factor == g.factor && k.W == width && k.H == height && !memcmp(&k.m, &g.m, sizeof(Mat34))) return;
    g.clip_slots = near_plane_crossing();
    g.live.on = 0;
    if (!g.clip_slots) cull_slots(width, height);
    k = Lib::CullKey{g.m, g.factor, width, height, true};
}

TimingSlot *timing_slot(Dev &d) {
    if (!g.timing) return nullptr;
    if (d.tcount == d.tslots.size()) {
        TimingSlot t;
        HIPCHECK(hipEventCreate(&t.frame0)); HIPCHECK(hipEventCreate(&t.geo1));
        HIPCHECK(hipEventCreate(&t.frag0)); HIPCHECK(hipEventCreate(&t.frag1));
        d.tslots.push_back(t);
    }
    return &d.tslots[d.tcount++];
}

// Frame tags are the uint32 frame number (0 = none): issued_tag, last_tag and the completion word
// k_fragment's first workgroup stores.  Before the count wraps (~62 h at 19 k fps) every stream is
// drained, the completion word and issued tags are reset and the count restarts, so no tag is
// reused while the completion word may still carry it.  The bins' pair counts are reset by the
// fragment workgroups that read them (the set's last reader); they are zeroed here as well, in case
// a frame was abandoned between its geometry and fragment launches.
constexpr uint32_t kTagLimit = 0xFFFFFF00u;

void restart_tags(Dev &d, uint32_t next_frame_no) {
    sync_device("frame-tag restart", d.device, d.frame_no);
    for (int p = 0; p < kSets; p++)
        if (d.bincnt[p]) HIPCHECK(hipMemset(d.bincnt[p], 0, d.bins_cap * sizeof(uint32_t)));
    sync_device("frame-tag restart: bin counts cleared", d.device, d.frame_no);
    d.frame_no = next_frame_no;
    if (d.tile_sum_host) memset(d.tile_sum_host, 0, kSumWords * kSets * sizeof(uint32_t));   // (tags restart)
    for (uint32_t &t : d.issued_tag) t = 0;
    d.last_tag = 0;
    if (d.done_host) __atomic_store_n(d.done_host, 0u, __ATOMIC_RELEASE);
}

// The buffer set of the frame being issued; frames cycle through kSets sets.
uint32_t next_set(Dev &d) {
    if (d.frame_no >= kTagLimit) restart_tags(d, 0);
    d.frame_no++;
    return d.frame_no % kSets;
}

// Row path: block until the last fragment kernel that read buffer set p has finished.  *done_host
// holds the tag of the newest fragment launch known complete: every launch's first workgroup stores
// its predecessor's tag there, and tags grow by frame.  Usually the set is free (the host runs at
// most kSets frames ahead of the GPU); otherwise the launch after it -- issued already, in order on
// the same stream -- reports it when it starts.
void wait_set_free(Dev &d, uint32_t p) {
    const uint32_t want = d.issued_tag[p];
    if (want == 0 || __atomic_load_n(d.done_host, __ATOMIC_ACQUIRE) >= want) return;
    const WaitSite w{"row path: buffer set reuse (its last reader, an earlier frame's fragment launch)", "k_fragment",
                     d.device, d.frame_no};
    const int64_t t0 = mono_ns();
    if (want == d.last_tag) {
        // no row-path fragment launch after it to report it (tile-path frames followed): drain its stream
        while (!stream_drained(d.last_stream, w, t0)) sched_yield();
        __atomic_store_n(d.done_host, want, __ATOMIC_RELEASE);
        return;
    }
    // the later launch that reports it is issued; after a grace of spinning, the previous frame's
    // stream (every earlier frame is ordered before it, follow_previous_frame) is polled as well:
    // drained means every reader is done even if the report was somehow missed
    for (uint32_t k = 1; __atomic_load_n(d.done_host, __ATOMIC_ACQUIRE) < want; k++) {
        __builtin_ia32_pause();
        if ((k & 1023u) == 0 && mono_ns() - t0 > 2000000 && stream_drained(d.last_stream, w, t0)) {
            __atomic_store_n(d.done_host, d.last_tag, __ATOMIC_RELEASE);
            return;
        }
    }
}

// Frames are ordered on the caller's stream.  When a frame arrives on another stream than the
// previous one, that stream first waits for the previous frame's fragment stage (one event): the
// row path's completion chain (wait_set_free) and the tile path's shared key buffer assume it.
void follow_previous_frame(Dev &d, hipStream_t st) {
    // the null stream does not order our non-blocking streams (nor they it): a switch from or to
    // NULL needs the event like any other
    if (d.have_last && st != d.last_stream) {
        HIPCHECK(hipEventRecord(d.handoff, d.last_stream));
        HIPCHECK(hipStreamWaitEvent(st, d.handoff, 0));
    }
    d.last_stream = st;
    d.have_last = true;
}

// S3R_SERIAL (profiling): the geometry waits for every earlier fragment kernel -- no overlap.
void wait_all_fragments(Dev &d, hipStream_t geo) {
    for (int q = 0; q < kSets; q++) HIPCHECK(hipStreamWaitEvent(geo, d.frag_done[q], 0));
}


// Can any triangle cross the near plane this frame (render.cpp:308: some corner in front of it, some
// behind)?  If not, k_geometry leaves out the clip-appended slots (launch_geometry clip_slots).  Each
// vertex's camera depth nz = -(row 2 of the camera matrix . v) (render.cpp:286) is classified against
// kNear with a margin far above float rounding (1e-4 of the summed term magnitudes): a vertex inside
// the margin, or a non-finite one, counts as crossing.  Scenes without the host copy: always true.
#ifndef S3R_NEAR_CHECK
#define S3R_NEAR_CHECK 1
#endif
bool near_plane_crossing() {
    if (!S3R_NEAR_CHECK || g.near_vidx.empty()) return true;
    const size_t nv = g.near_vtx.size();
    g.near_side.resize(nv);
    const float *r = g.m.m[2];
    for (size_t i = 0; i < nv; i++) {
        const float4 v = g.near_vtx[i];
        const float a = r[0] * v.x, b = r[1] * v.y, c = r[2] * v.z, e = r[3] * v.w;
        const float nz = -(((a + b) + c) + e);
        const float margin = 1e-4f * (fabsf(a) + fabsf(b) + fabsf(c) + fabsf(e)) + 1e-6f;
        if (!std::isfinite(nz) || !std::isfinite(margin) || fabsf(nz - kNear) <= margin) return true;
        g.near_side[i] = nz > kNear ? 1u : 2u;          // 1: in front of the near plane, 2: behind it
    }
    for (size_t t = 0; t + 2 < g.near_vidx.size(); t += 3) {
        const uint8_t m = g.near_side[g.near_vidx[t]] | g.near_side[g.near_vidx[t + 1]] | g.near_side[g.near_vidx[t + 2]];
        if (m == 3u) return true;
    }
    return false;
}

// Host slot cull, frames without clip slots (near_plane_crossing false: each triangle wholly in front
// of the near plane or wholly behind it): slot t (original triangle t) is launched unless its setup
// surely rejects it -- every corner behind the plane (render.cpp:306), or the triangle off the frame
// or of area < 10 (:312, :314, :317: back faces included).  The host projects the corners in double
// and widens each test by a bound on the device's float rounding (1e-6 of every summed term's
// magnitude, four times float's worst case, carried through the divide and the area): a triangle
// within that bound of a test stays launched, and the device decides it exactly.  k_geometry starts
// no workgroup for a culled slot; one marker workgroup stores it dead (launch_geometry live).
void cull_slots(uint32_t W, uint32_t H) {
    if (g.ntri > kLiveMaskSlots || g.near_vidx.size() != 3 * (size_t)g.ntri) return;
    const size_t nv = g.near_vtx.size();
    g.near_rv.resize(3 * nv);
    const double f = g.factor, hw = (double)((float)W / 2), hh = (double)((float)H / 2);
    for (size_t i = 0; i < nv; i++) {
        if (g.near_side[i] != 1u) continue;                  // behind the plane: no projection
        const float4 v = g.near_vtx[i];
        double c[3], sum[3];
        for (int r = 0; r < 3; r++) {
            const float *m = g.m.m[r];
            const double a = (double)m[0] * v.x, b = (double)m[1] * v.y, e = (double)m[2] * v.z, h = (double)m[3] * v.w;
            c[r] = ((a + b) + e) + h;
            sum[r] = fabs(a) + fabs(b) + fabs(e) + fabs(h);
        }
        const double nz = -c[2], dz = 1e-6 * sum[2];
        const double qx = c[0] * f / nz, qy = -c[1] * f / nz;
        const double ex = f * (1e-6 * sum[0] + fabs(c[0]) * dz / nz) / nz + 1e-6 * (fabs(qx) + hw);
        const double ey = f * (1e-6 * sum[1] + fabs(c[1]) * dz / nz) / nz + 1e-6 * (fabs(qy) + hh);
        g.near_rv[3 * i] = qx + hw;
        g.near_rv[3 * i + 1] = qy + hh;
        g.near_rv[3 * i + 2] = ex > ey ? ex : ey;
    }
    SlotMask &lm = g.live;
    memset(lm.bits, 0, sizeof(lm.bits));
    lm.nlive = 0;
    const double sw = W, sh = H;
    for (uint32_t t = 0; t < g.ntri; t++) {
        const uint32_t *vi = &g.near_vidx[3 * (size_t)t];
        const uint8_t side = g.near_side[vi[0]] | g.near_side[vi[1]] | g.near_side[vi[2]];
        if (side == 2u) continue;                            // :306
        bool live = side != 1u;
        if (!live) {
            const double *a = &g.near_rv[3 * (size_t)vi[0]], *b = &g.near_rv[3 * (size_t)vi[1]],
                         *c = &g.near_rv[3 * (size_t)vi[2]];
            const double E = std::max(std::max(a[2], b[2]), c[2]);
            const double rmx = std::max(std::max(a[0], b[0]), c[0]), rnx = std::min(std::min(a[0], b[0]), c[0]);
            const double rmy = std::max(std::max(a[1], b[1]), c[1]), rny = std::min(std::min(a[1], b[1]), c[1]);
            const double t1 = (c[0] - a[0]) * (a[1] - b[1]), t2 = (c[1] - a[1]) * (b[0] - a[0]);
            const double aerr = 2 * E * (fabs(a[1] - b[1]) + fabs(c[0] - a[0]) + fabs(c[1] - a[1]) + fabs(b[0] - a[0])) +
                                8 * E * E + 1e-6 * (fabs(t1) + fabs(t2));
            const bool off = rmx < -E || rmy < -E || rnx >= sw + E || rny >= sh + E;
            live = !off && t1 + t2 + aerr >= 10 && std::isfinite(E) && std::isfinite(t1 + t2 + aerr);
        }
        if (live) { lm.bits[t >> 6] |= 1ull << (t & 63u); lm.nlive++; }
    }
    lm.on = 1;
}

bool use_tile_path() {
    if (g.raster_path == 1) return false;
    if (g.raster_path == 2) return true;
    return 2ull * g.ntri > kRowPathMaxSlots;
}

// Rows per interleaved band of an H-row frame split over nparts devices: the configured band
// (s3r_configure_devices, S3R_BAND), else by fragment path.  Row path: 16 rows (its fragment
// workgroups are 4-row blocks of 384-px bins; the floor and sky rows spread evenly).  Tile path:
// two bands per part, ceil(H / 2N) rows -- a part's cluster cull keeps the clusters that reach its
// bands, and an icosahedron of the stress scene (17-27 rows tall) meets ~(band + 22) / (N band) of
// them: part 0 of 8 at 4K (config 5), one MI355X, 16-row bands 4 539-4 663 fps, 54: 5 322, 135:
// 5 855, 270 (one contiguous band): 6 015 (profiles/r04_band_sweep.txt).  Two bands rather than one
// keep some balance for scenes that are not uniform across the frame.
uint32_t frame_band(uint32_t H, uint32_t nparts) {
    if (g.band) return g.band;
    if (nparts <= 1) return H ? H : 1u;
    if (!use_tile_path()) return kDefaultBand;
    return std::max(kDefaultBand, (H + 2 * nparts - 1) / (2 * nparts));
}

// The device's clusters as the tile kernels take them for a frame of nparts parts (ncl 0: no cull).
// S3R_CLUSTERS: 0 never, 1 (default) for frame parts only -- a whole frame in view keeps nearly every
// cluster, and the cull's records cost more than they save there (stress scene, one MI355X: whole
// frame 96 us of cull for a 40 us shorter setup) -- 2 always.
TileClusters tile_clusters(const Dev &d, uint32_t nparts) {
    const bool on = g.clusters && g.ncl && (nparts > 1 || g.clusters_whole);
    return TileClusters{d.cl_sphere, d.cl_first, d.cl_perm, d.cl_shard, on ? g.ncl : 0u, d.cl_map};
}

bool bins_on(const Dev &d);

// The tile path's fill and fragment stage of buffer set p (its setup done): scatter into the set's
// list (capacity d.tile_list_cap[p]), raster, resolve into out, on st after the geometry stream.
// frame_rows: out is the whole W x H frame (the caller's mapped buffer; direct delivery), each local
// row stored at its frame row.
void tile_fragment_stage(Dev &d, uint32_t p, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part,
                         uint32_t rows_local, uint32_t *out, hipStream_t geo, hipStream_t st, TimingSlot *ts,
                         bool frame_rows) {
    const float sw = (float)W, sh = (float)d.tile_H;
    const TileClusters cl = tile_clusters(d, nparts);
    const bool bins = d.tbin[p] != nullptr && bins_on(d);
    if (!bins)
        launch_tile_fill(d.live[p], d.tile_ctr[p], &cl, g.ntri, W, band, nparts, part, d.tile_cursor[p],
                         d.tile_list[p], d.tile_list_cap[p], geo, d.tile_xoff);
    const uint32_t *list = bins ? d.tbin[p] : d.tile_list[p];
    uint32_t *bcounts = bins ? d.tile_counts[p] : nullptr;
    const uint32_t bcap = bins ? d.bin_cap : 0u;
    HIPCHECK(hipEventRecord(d.geo_done[p], geo));
    if (ts) HIPCHECK(hipEventRecord(ts->geo1, geo));
    follow_previous_frame(d, st);
    HIPCHECK(hipStreamWaitEvent(st, d.geo_done[p], 0));
    if (ts) HIPCHECK(hipEventRecord(ts->frag0, st));
    // raster and resolve fused (kernels.hip k_tile_raster) -- stress scene, one MI355X: whole frame 800
    // -> 854 fps in HBM, delivered 583 -> 614 (profiles/r04_tile_fused_ab.txt), part 0 of 8 4 491-4 632
    // -> 4 672-4 696 with the bins (profiles/r04_part8_ab.txt); the split launches are gone (round 5)
    const size_t npx = (size_t)W * rows_local;
    if (d.deferred_cap < npx) {                // pixels whose winner needs its full setup
        sync_device("tile path: growing the deferred-pixel buffer", d.device, d.frame_no);
        if (d.deferred) HIPCHECK(hipFree(d.deferred));
        d.deferred = dalloc<uint4>(npx);
        d.deferred_cap = npx;
    }
    launch_tile_raster_resolve(d.recs[p], d.vtx, d.nrm, d.pay, d.disc, d.vidx, d.aidx, g.ntri, g.m, g.factor, sw, sh,
                               d.tex, g.ntex, out, W, band, nparts, part, rows_local, d.tile_offs[p], d.tile_ctr[p],
                               list, d.tile_list_cap[p], d.deferred, st, frame_rows, bcounts, bcap, d.tile_xoff,
                               d.tile_sum_dev + kSumWords * p);
    if (ts) HIPCHECK(hipEventRecord(ts->frag1, st));
    HIPCHECK(hipEventRecord(d.frag_done[p], st));
    HIPCHECK(hipGetLastError());
}

void grow_tile_list(Dev &d, uint32_t p, uint64_t total) {
    if (d.tile_list_cap[p] >= total && d.tile_list_cap[p] > 0) return;
    sync_device("tile path: growing the tile lists", d.device, d.frame_no);
    if (d.tile_list[p]) HIPCHECK(hipFree(d.tile_list[p]));
    // a quarter of headroom (S3R_TILE_LIST_EXACT=1, tests: none, so the next larger frame overflows)
    const bool exact = getenv("S3R_TILE_LIST_EXACT") && atoi(getenv("S3R_TILE_LIST_EXACT")) != 0;
    const uint64_t cap = exact ? (total ? total : 1) : total + total / 4 + 1024;
    d.tile_list[p] = dalloc<uint32_t>(cap);
    d.tile_list_cap[p] = cap;
}

// After a synchronous tile-path frame (its stream drained): if its list overflowed the capacity the
// set had from earlier frames, render its fragment stage again into a list of the right size and
// return true (the caller redoes its delivery); the totals are in tile_sum_host by then.
// Spin until buffer set p's summary (k_tile_cursor / k_tile_bins_done) carries this frame's tag: a
// stream synchronisation's wake-up costs ~10-20 us a frame; after 2 ms fall back to synchronising,
// which also surfaces a device fault.
bool bins_on(const Dev &d);

void wait_tile_summary(Dev &d, uint32_t p, hipStream_t geo) {
    volatile uint32_t *sum = d.tile_sum_host + kSumWords * p;
    const WaitSite w{"tile path: the frame's setup summary (list and bin sizes)", "k_tile_setup / k_tile_cursor",
                     d.device, d.frame_no};
    const int64_t t0 = mono_ns();
    for (uint32_t k = 1; __atomic_load_n(&sum[0], __ATOMIC_ACQUIRE) != d.frame_no; k++) {
        __builtin_ia32_pause();
        if ((k & 255u) == 0 && mono_ns() - t0 > 2000000 && stream_drained(geo, w, t0) &&
            __atomic_load_n(&sum[0], __ATOMIC_ACQUIRE) != d.frame_no) {
            fprintf(stderr, "s3r: tile path: the setup of frame %u finished on device %d without its summary "
                    "(buffer set %u carries tag %u)\n", d.frame_no, d.device, p, (unsigned)sum[0]);
            fflush(stderr);
            abort();
        }
    }
    // (bins mode: word 2, the binned entries, is written by the frame's last kernel, after this
    // point -- refresh_pairs reads it once the frame is done)
    if (!bins_on(d)) d.last_pairs = sum[2];
    d.last_live = sum[1];
    d.last_kept = sum[3];
    d.tile_readbacks++;
}

// Bins mode (the default, S3R_TILE_BINS=0: the lists): every buffer set's bins for nt (tile, bucket)
// slots of d.bin_cap entries each (the first capacity S3R_TILE_BIN_CAP or 256; grow_bins doubles it
// at least when a frame overflows).  Bins are sized by the fullest (tile, bucket), so a scene piling
// many triangles into one tile could need far more memory than its lists: past the budget
// (S3R_TILE_BIN_BUDGET_MB, 32 GiB for all buffer sets) the device drops its bins and uses the lists.
bool bins_on(const Dev &d) { return g.tile_bins && !d.bins_off; }

// Per-path storage, allocated on a path's first frame (the other path's would be wasted: the row path's
// 240-B TriSetup per slot is 38 GB for the four buffer sets of the 20 M-triangle stress scene, which
// only the tile path renders; the lists' 16-B live entries are 2.6 GB that bins mode never touches).
void ensure_row_sets(Dev &d) {
    if (d.tris[0]) return;
    sync_device("row path: first frame, TriSetup records", d.device, d.frame_no);
    for (int p = 0; p < kSets; p++) d.tris[p] = dalloc<TriSetup>(2 * (size_t)g.ntri);
}
void ensure_live(Dev &d) {
    if (d.live[0]) return;
    sync_device("tile path: live-entry lists", d.device, d.frame_no);
    for (int p = 0; p < kSets; p++) d.live[p] = dalloc<uint4>((size_t)2 * g.ntri);
}

void drop_bins(Dev &d) {
    sync_device("tile path: dropping the bins", d.device, d.frame_no);
    for (int q = 0; q < kSets; q++) {
        if (d.tbin[q]) HIPCHECK(hipFree(d.tbin[q]));
        d.tbin[q] = nullptr;
        d.tbin_slots[q] = 0;
    }
    d.bins_off = true;
}

void ensure_bins(Dev &d, uint64_t nt) {
    if (!d.bin_cap) {
        const char *e = getenv("S3R_TILE_BIN_CAP");
        d.bin_cap = e && atoi(e) > 0 ? (uint32_t)atoi(e) : 256u;
    }
    if ((uint64_t)kSets * nt * d.bin_cap * sizeof(uint32_t) > g.tile_bin_budget) {
        drop_bins(d);
        return;
    }
    for (int q = 0; q < kSets; q++) {
        if (d.tbin[q] && d.tbin_slots[q] >= nt) continue;
        sync_device("tile path: allocating the bins", d.device, d.frame_no);
        if (d.tbin[q]) HIPCHECK(hipFree(d.tbin[q]));
        d.tbin[q] = dalloc<uint32_t>(nt * d.bin_cap);
        d.tbin_slots[q] = nt;
    }
}

// Larger bins for a (tile, bucket) that needs `need` entries; false (bins dropped) past the budget.
bool grow_bins(Dev &d, uint32_t need) {
    uint64_t cap = (uint64_t)d.bin_cap * 2u;
    while (cap < (uint64_t)need + need / 4u) cap *= 2u;
    uint64_t total = 0;
    for (int q = 0; q < kSets; q++) total += d.tbin_slots[q] * cap * sizeof(uint32_t);
    if (total > g.tile_bin_budget || cap > 0x80000000ull) {
        drop_bins(d);
        return false;
    }
    sync_device("tile path: growing the bins", d.device, d.frame_no);
    for (int q = 0; q < kSets; q++) {
        if (d.tbin[q]) HIPCHECK(hipFree(d.tbin[q]));
        d.tbin[q] = dalloc<uint32_t>(d.tbin_slots[q] * cap);
    }
    d.bin_cap = (uint32_t)cap;
    d.bin_regrows++;
    return true;
}

void rebin(Dev &d, uint32_t p, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
           uint32_t rows_local, hipStream_t geo);

bool tile_redo_if_overflowed(Dev &d, hipStream_t st) {
    if (!d.tile_pending) return false;
    d.tile_pending = false;
    const uint32_t p = d.tile_pending_set;
    const volatile uint32_t *sum = d.tile_sum_host + kSumWords * p;
    const uint64_t total = sum[2];
    d.last_pairs = total;
    d.last_live = sum[1];
    d.last_kept = sum[3];
    if (d.tile_pending_bins) {
        if (sum[4] == 0) return false;
        // a (tile, bucket) outgrew its bin: bin the frame again into larger bins (or, past the budget,
        // into the lists), then its fragment stage
        d.tile_overflows++;
        if (check_launches()) check_context(d.device, d.frame_no, "tile path, overflowed bins binned again");
        hipStream_t geo = d.geo[0];
        rebin(d, p, d.tile_W, d.tile_H, d.tile_band, d.tile_nparts, d.tile_part, d.tile_rows, geo);
        tile_fragment_stage(d, p, d.tile_W, d.tile_band, d.tile_nparts, d.tile_part, d.tile_rows, d.tile_out, geo, st,
                            nullptr, d.tile_frame_rows);
        sync_stream(st, WaitSite{"tile path: an overflowed frame binned and rendered again", "k_tile_raster", d.device, d.frame_no});
        return true;
    }
    if (total <= d.tile_list_cap[p]) return false;
    d.tile_overflows++;
    grow_tile_list(d, p, total);
    hipStream_t geo = d.geo[0];
    launch_tile_cursor(d.tile_counts[p], d.tile_offs[p], d.tile_W, d.tile_rows, d.tile_cursor[p], d.tile_ctr[p], geo,
                       d.tile_xoff);
    tile_fragment_stage(d, p, d.tile_W, d.tile_band, d.tile_nparts, d.tile_part, d.tile_rows, d.tile_out, geo, st,
                        nullptr, d.tile_frame_rows);
    sync_stream(st, WaitSite{"tile path: an overflowed frame listed and rendered again", "k_tile_raster", d.device, d.frame_no});
    return true;
}

// Buffer set p's frame binned again after its bins overflowed (the summary's need in sum[4]), until it
// fits: the counts zeroed (the overflowed pass left them counted -- k_tile_raster resets them only
// where a raster ran), larger bins, the setup again, waiting for its summary; past the budget the set
// is set up into the lists instead (grow_bins dropped the bins, so its fragment stage reads the lists).
void rebin(Dev &d, uint32_t p, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
           uint32_t rows_local, hipStream_t geo) {
    const TileClusters cl = tile_clusters(d, nparts);
    volatile uint32_t *sum = d.tile_sum_host + kSumWords * p;
    const uint64_t nt = tile_slots(W, rows_local, d.tile_xoff);
    while (sum[4] != 0) {
        const bool bins = grow_bins(d, sum[4]);
        if (!bins) ensure_live(d);
        HIPCHECK(hipMemsetAsync(d.tile_counts[p], 0, nt * sizeof(uint32_t), geo));
        __atomic_store_n(&d.tile_sum_host[kSumWords * p], 0u, __ATOMIC_RELEASE);   // (the earlier pass carried this tag)
        launch_tile_setup(d.vtx, d.vidx, g.ntri, g.m, g.factor, (float)W, (float)H, W, band, nparts, part, rows_local,
                          d.recs[p], d.live[p], d.clipq, d.tile_ctr[p], d.tile_counts[p], d.tile_offs[p],
                          d.tile_cursor[p], d.scan_temp, d.scan_temp_bytes, geo, d.vrv, g.nv, &cl,
                          d.tile_sum_dev + kSumWords * p, d.frame_no, bins ? d.tbin[p] : nullptr, bins ? d.bin_cap : 0u,
                          d.tile_xoff);
        wait_tile_summary(d, p, geo);
        if (!bins) {
            grow_tile_list(d, p, sum[2]);
            break;
        }
    }
}

void render_tiles(Dev &d, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                  uint32_t *out, hipStream_t st, TimingSlot *ts, bool sync, bool frame_rows) {
    if (W > 65535 || H > 65535) {                       // packed 16-bit bboxes
        fprintf(stderr, "s3r: tile path supports frames up to 65535 x 65535\n");
        exit(1);
    }
    const float sw = (float)W, sh = (float)H;
    // a frame written into the caller's buffer: tiles on its 64-B line grid -- a malloc'd buffer starts
    // 16 B into a line, so 64-px tiles at x = 64 c would store each tile row as five lines, two partly
    // written; shifted left by that offset (W a multiple of 16, so every row shares it) each tile row
    // crosses the link as four whole lines (stress frame, one MI355X: 689-710 fps at the malloc offset,
    // 741-747 into a line-aligned buffer, profiles/r04_line_offset.txt)
    d.tile_xoff = frame_rows && g.tile_line_grid && W % 16u == 0u ? (uint32_t)(((uintptr_t)out >> 2) & 15u) : 0u;
    const uint64_t nt = tile_slots(W, rows_local, d.tile_xoff);   // (tile, depth bucket) entries
    if (d.tiles_cap < nt) {
        sync_device("tile path: growing the tile counters", d.device, d.frame_no);
        for (int p = 0; p < kSets; p++) {
            for (uint32_t **q : {&d.tile_counts[p], &d.tile_offs[p], &d.tile_cursor[p]}) {
                if (*q) HIPCHECK(hipFree(*q));
                *q = dalloc<uint32_t>(nt);
            }
            // counts start zeroed (each frame's k_tile_cursor leaves them zero); the null-stream
            // memset does not order the geometry streams, hence the synchronisation
            HIPCHECK(hipMemset(d.tile_counts[p], 0, nt * sizeof(uint32_t)));
        }
        sync_device("tile path: tile counters zeroed", d.device, d.frame_no);
        if (d.scan_temp) HIPCHECK(hipFree(d.scan_temp));
        d.scan_temp_bytes = tile_scan_temp_bytes(nt);
        d.scan_temp = dalloc<uint8_t>(d.scan_temp_bytes);
        d.tiles_cap = nt;
    }
    // vertex stage (k_tile_vertex): measured on the 20 M-triangle stress scene at 4K, part 0 of 8
    // 1 996 -> 2 108 fps (setup 307 -> 235 us + 57 us for the stage), whole frame 826 -> 808 fps: on
    // for frame parts without clusters, where the per-triangle setup is replicated on every device
    if (nparts > 1 && !tile_clusters(d, nparts).ncl) {
        if (!d.vrv) d.vrv = dalloc<float4>(g.nv);
    } else if (d.vrv) {
        sync_device("tile path: dropping the vertex stage", d.device, d.frame_no);
        HIPCHECK(hipFree(d.vrv));
        d.vrv = nullptr;
    }
    if (!d.recs[0]) {
        for (int p = 0; p < kSets; p++) {
            d.recs[p] = dalloc<uint8_t>((size_t)2 * g.ntri * raster_rec_bytes());
            if (!d.clipq) d.clipq = dalloc<uint32_t>(g.ntri);
            d.tile_ctr[p] = dalloc<uint32_t>(kTileCtrWords);
            HIPCHECK(hipMemset(d.tile_ctr[p], 0, kTileCtrWords * sizeof(uint32_t)));
            d.tile_total[p] = d.tile_ctr[p] + 1;
        }
        HIPCHECK(hipHostMalloc((void **)&d.tile_sum_host, kSumWords * kSets * sizeof(uint32_t),
                               hipHostMallocCoherent | hipHostMallocMapped));
        memset(d.tile_sum_host, 0, kSumWords * kSets * sizeof(uint32_t));
        HIPCHECK(hipHostGetDevicePointer((void **)&d.tile_sum_dev, d.tile_sum_host, 0));
        sync_device("tile path: first frame, summary words", d.device, d.frame_no);          // (the null-stream memsets vs the geometry streams)
    }
    const uint32_t p = next_set(d);
    hipStream_t geo = d.geo[0];
    HIPCHECK(hipStreamWaitEvent(geo, d.frag_done[p], 0));
    if (g.serial) wait_all_fragments(d, geo);
    if (ts) HIPCHECK(hipEventRecord(ts->frame0, geo));
    const TileClusters cl = tile_clusters(d, nparts);
    if (bins_on(d)) ensure_bins(d, nt);
    const bool bins = bins_on(d);
    if (!bins) ensure_live(d);
    // no raster records for the slots the raster can set up again (kernels.hip kNoRecBit).  Stress
    // scene, one MI355X (profiles/r05_rec0_ab.txt): setup 548-554 -> 434 us, its traffic 1.34 -> 0.84 GB;
    // delivered frames 831-833 -> 915-924 fps; frames into HBM 1 151 -> 1 174 fps whole, part 0 of 8 at
    // the 135-row band 6 503-6 524 -> 6 846-6 880 (the record-writing setup was retired in round 6)
    if (test_hold_ms() && d.frame_no >= 2) launch_test_hold(test_hold_ms(), geo);
    launch_tile_setup(d.vtx, d.vidx, g.ntri, g.m, g.factor, sw, sh, W, band, nparts, part, rows_local, d.recs[p],
                      d.live[p], d.clipq, d.tile_ctr[p], d.tile_counts[p], d.tile_offs[p], d.tile_cursor[p], d.scan_temp,
                      d.scan_temp_bytes, geo, d.vrv, g.nv, &cl, d.tile_sum_dev + kSumWords * p, d.frame_no,
                      bins ? d.tbin[p] : nullptr, bins ? d.bin_cap : 0u, d.tile_xoff);
    // The list size is data-dependent.  Asynchronous frames (s3r_render_bands), and the first frame
    // of each buffer set, read it back before the fill (one host sync); synchronous frames
    // (updateAndRender) fill the set's list as sized by earlier frames, with no sync, and are
    // rendered again after the frame if it overflowed (tile_redo_if_overflowed; the fill and raster
    // kernels bound their list accesses).  S3R_TILE_READBACK=1: always read back.
    const bool readback_env = getenv("S3R_TILE_READBACK") && atoi(getenv("S3R_TILE_READBACK")) != 0;
    volatile uint32_t *sum = d.tile_sum_host + kSumWords * p;
    d.last_path = 2;
    d.last_set = (int)p;
    d.last_set_bins = bins;
    d.tile_H = H;
    if (bins) {
        // bins mode: asynchronous frames check the bins before their fragment stage (a spin on the
        // summary); synchronous ones after the frame (tile_redo_if_overflowed)
        if (!sync || readback_env) {
            wait_tile_summary(d, p, geo);
            if (sum[4] != 0) {
                d.tile_overflows++;
                rebin(d, p, W, H, band, nparts, part, rows_local, geo);
            }
        }
    } else if (!sync || d.tile_list_cap[p] == 0 || readback_env) {
        wait_tile_summary(d, p, geo);
        grow_tile_list(d, p, sum[2]);
    }
    tile_fragment_stage(d, p, W, band, nparts, part, rows_local, out, geo, st, ts, frame_rows);
    if (sync) {
        // the overflow check reads this frame's summary once the frame is done
        d.tile_pending = true;
        d.tile_pending_bins = bins && bins_on(d);
        d.tile_pending_set = p;
        d.tile_W = W; d.tile_band = band; d.tile_nparts = nparts; d.tile_part = part; d.tile_rows = rows_local;
        d.tile_out = out;
        d.tile_frame_rows = frame_rows;
    }
}

// A frame part written straight into the caller's mapped host buffer (direct / host-fill delivery):
// with flags_dev (host fill) the sky-flag kernel publishes the bins' flags with this tag, and the
// fragment kernel leaves sky bins and, in covered bins, the row chunks without a winner to the host
// (their masks in chunks_dev); without, the fragment kernel writes every pixel.
struct HostFill {
    uint32_t *flags_dev;
    uint32_t tag;
    uint32_t *probe_dev;
    unsigned long long *chunks_dev;
    uint32_t gpu_eighths;     // sky bins with bin % 8 below this stay with the GPU (adaptive split)
};

// One frame part on device d (its current device must be set): rows_local rows of an interleaved
// band split (nparts = 1, band = H: the whole frame) into `out` on `st`, asynchronously.  With hf
// `out` is the whole W x H frame in the caller's mapped host buffer: the fragment kernel writes this
// part's bins at their frame rows -- only the covered ones for host fill (row path only; the tile
// path's resolve writes every pixel of the part at its frame row, direct delivery).
//
// sync (updateAndRender's frames, waited for before the call returns): the geometry runs on `st`
// itself -- nothing could overlap it, and stream order replaces the cross-stream event (~9 us per
// frame measured); otherwise it runs on a geometry stream so later frames' geometry overlaps
// earlier frames' fragment kernels.
void render_core(Dev &d, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                 uint32_t *out, hipStream_t st, const HostFill *hf = nullptr, bool sync = false) {
    TimingSlot *ts = timing_slot(d);
    if (check_launches())
        check_context(d.device, d.frame_no + 1u, use_tile_path() ? (sync ? "tile path, synchronous frame" : "tile path")
                                                                  : (sync ? "row path, synchronous frame" : "row path"));
    if (use_tile_path()) {
        render_tiles(d, W, H, band, nparts, part, rows_local, out, st, ts, sync, hf != nullptr);
        return;
    }
    d.last_path = 1;
    ensure_row_sets(d);
    fragment_configure(W, rows_local);
    const size_t need = (size_t)2 * g.ntri * rows_local * start_entries(W) * 4;
    if (d.rowtab_cap < need) {
        sync_device("row path: growing the start table", d.device, d.frame_no);
        for (int p = 0; p < kSets; p++) {
            if (d.rowtab[p]) HIPCHECK(hipFree(d.rowtab[p]));
            d.rowtab[p] = dalloc<float>(need);
        }
        d.rowtab_cap = need;
    }
    const uint64_t nbins = fragment_bins(W, rows_local);
    if (d.bins_cap < nbins) {
        sync_device("row path: growing the bins", d.device, d.frame_no);
        for (int p = 0; p < kSets; p++) {
            if (d.bincnt[p]) HIPCHECK(hipFree(d.bincnt[p]));
            if (d.pairs[p]) HIPCHECK(hipFree(d.pairs[p]));
            d.bincnt[p] = dalloc<uint32_t>(nbins);
            d.pairs[p] = dalloc<uint4>(nbins * kPairMax * kPairWords);
            HIPCHECK(hipMemset(d.bincnt[p], 0, nbins * sizeof(uint32_t)));
        }
        // hipMemset runs on the null stream, which does not order the non-blocking geometry
        // streams: finish it before the next k_geometry counts pairs in these bins
        sync_device("row path: bin counts zeroed", d.device, d.frame_no);
        d.bins_cap = nbins;
    }
    // longest-first order only where a launch is more than one round of resident workgroups (~1 280
    // on the chip): a frame part of one round gains nothing and would pay the order column's time.
    // Round 4 (tools/lpt_sweep.sh, two repeats): 2 000 instead of 4 000 bins puts part 0 of 8 of the
    // 8K frame (2 700 bins) on it, 27 100-27 200 -> 29 400-29 500 fps; 4K part 0 of 8 (2 040 bins) and
    // 1080p (flat) move by <= 0.3 %
    const uint64_t bins = nbins;
    const char *lpt_env = getenv("S3R_LPT_MIN");            // tuning / test override
    // (delivered frames are bound by the link, not by their heaviest bins: launch order, no order
    // column; measured equal or 1 us better)
    // ... and only for the widest (6-chunk) bins: with 2-chunk bins (1080p, 4K parts of 4 and 8) the launch
    // order measured best (1080p flat, k_fragment: launch order 24.2-24.3 us, wall-time order 25.0-25.3,
    // work-unit order 27.5-28.1; profiles/r05_order_ab.txt) -- short bins leave no long tail to fix,
    // and heavy-first groups the textured floor's bins on the chip at once
    const bool lpt = g.ntri > 0 && !hf && bins >= (lpt_env ? strtoull(lpt_env, nullptr, 10) : kLptMinBins) &&
                     (lpt_env || fragment_segment_pixels() >= 384u);     // (6 chunks of 64 px)
    if (lpt && d.order_cap < bins) {
        sync_device("row path: growing the order column", d.device, d.frame_no);
        for (int q = 0; q < kSets; q++) {
            if (d.order[q]) HIPCHECK(hipFree(d.order[q]));
            d.order[q] = dalloc<uint32_t>(2 * bins);
            HIPCHECK(hipMemset(d.order[q], 0, 2 * bins * sizeof(uint32_t)));
        }
        sync_device("row path: order column zeroed", d.device, d.frame_no);     // (as for the bin counts: before k_geometry writes perm)
        d.order_cap = bins;
    }
    // geometry for this frame into buffer set p, once the fragment kernel that last read set p is done
    const uint32_t p = next_set(d);
    hipStream_t geo = sync && !g.serial ? st : d.geo[d.frame_no % kGeoStreams];
    const bool chained = geo == st;            // geometry -> fragment by stream order, no event
    if (chained) follow_previous_frame(d, st);
    d.hp.lap(1);
    // the set's last reader (frame k - kSets) has usually finished: then no cross-stream wait
    if (g.serial) {
        HIPCHECK(hipStreamWaitEvent(geo, d.frag_done[p], 0));
        wait_all_fragments(d, geo);
    } else {
        wait_set_free(d, p);
    }
    if (ts) HIPCHECK(hipEventRecord(ts->frame0, geo));
    d.hp.lap(2);
    const uint32_t tag = d.frame_no;              // >= 1: frame k's completion tag (wait_set_free)
    // host fill: the geometry launch also publishes the bins' sky flags, as soon as every workgroup's
    // pair reservations are in (one extra workgroup waits for them on per-row-block counters)
    // delivered frames: the geometry tabulates row starts only, the fragment workgroups walk along
    // their rows themselves (kernels.hip k_geometry)
    const bool row_starts = hf != nullptr;
    GeoSkyFlags gsf{};
    if (hf && hf->flags_dev) {
        if (!d.geo_cnt) {
            d.geo_cnt = dalloc<uint32_t>((size_t)kSets * kGeoCounterWords);
            HIPCHECK(hipMemset(d.geo_cnt, 0, (size_t)kSets * kGeoCounterWords * sizeof(uint32_t)));
            sync_device("row path: geometry counters zeroed", d.device, d.frame_no);      // (null-stream memset: finish before the geometry stream)
        }
        gsf = GeoSkyFlags{hf->flags_dev, hf->probe_dev, d.geo_cnt + (size_t)p * kGeoCounterWords, hf->tag,
                          hf->gpu_eighths, d.diag_dev, d.frame_no >= 2 ? test_extra_arrivals() : 0u};
    }
    if (test_hold_ms() && d.frame_no >= 2) launch_test_hold(test_hold_ms(), geo);
    launch_geometry(d.vtx, d.nrm, d.pay, d.disc, d.vidx, d.aidx, g.ntri, g.m, g.factor, W, H, band, nparts, part,
                    rows_local, d.tris[p], d.rowtab[p], d.bincnt[p], d.pairs[p], geo, chained ? nullptr : d.geo_done[p],
                    lpt ? d.order[p] : nullptr, gsf.flags ? &gsf : nullptr, row_starts, g.clip_slots, &g.live);
    d.hp.lap(3);
    if (ts) HIPCHECK(hipEventRecord(ts->geo1, geo));
    // fragment on the caller's stream, after the previous frame and this frame's geometry; its first
    // workgroup reports the previous fragment launch complete (wait_set_free); the completion event
    // only where S3R_SERIAL waits on it.  The fragment workgroups reset their bins' pair counts: the
    // launch is the set's last reader, and the set's next geometry waits for it (wait_set_free).
    if (!chained) {
        follow_previous_frame(d, st);
        HIPCHECK(hipStreamWaitEvent(st, d.geo_done[p], 0));
    }
    d.hp.lap(4);
    if (ts) HIPCHECK(hipEventRecord(ts->frag0, st));
    launch_fragment(d.tris[p], 2 * g.ntri, d.rowtab[p], d.tex, g.ntex, out, W, H, band, nparts, part, rows_local,
                    d.bincnt[p], d.pairs[p], st, g.serial ? d.frag_done[p] : nullptr, d.done_dev, d.last_tag,
                    lpt ? d.order[p] : nullptr, hf != nullptr, hf && hf->flags_dev ? 1u + hf->gpu_eighths : 0u,
                    hf ? hf->chunks_dev : nullptr, hf ? hf->tag : 0u, row_starts);
    d.issued_tag[p] = tag;
    d.last_tag = tag;
    if (ts) HIPCHECK(hipEventRecord(ts->frag1, st));
    HIPCHECK(hipGetLastError());
    d.hp.lap(5);
    d.hp.frames++;
}

// ---------------------------------------------------------------- caller host buffers
size_t page_size() {
    static const size_t p = (size_t)sysconf(_SC_PAGESIZE);
    return p;
}

// The registration covering [p, p + n), if any (ok or failed).
Lib::Reg *find_reg(const void *p, size_t n) {
    const uintptr_t a = (uintptr_t)p, b = a + n;
    for (auto &r : g.regs)
        if (r.a <= a && b <= r.b) return &r;
    return nullptr;
}

void unregister_range(Lib::Reg &r) {
    if (r.ok) (void)hipHostUnregister((void *)r.a);
    g.reg_epoch++;
}

// Page-lock [p, p + n) for DMA (cached).  Registrations whose pages the request's pages overlap --
// the other half of a double buffer shares the seam page -- are dropped (after draining the devices)
// and re-registered as one range covering the union, so each half of the reference's double buffer
// lies inside ONE registration and its copy runs at the pinned rate.
bool host_pinned(void *p, size_t n) {
    if (Lib::Reg *r = find_reg(p, n)) return r->ok;
    if (getenv("S3R_NO_PIN")) return false;
    // merged when the page ranges overlap (the driver pins whole pages), but the registered range is
    // the exact byte union of the caller's buffers: a page-rounded one would also cover bytes of a
    // neighbouring allocation, and a copy into that allocation straddling the registration's end is
    // then refused by the runtime
    const size_t pg = page_size();
    auto page_lo = [&](uintptr_t x) { return x & ~(uintptr_t)(pg - 1); };
    auto page_hi = [&](uintptr_t x) { return (x + pg - 1) & ~(uintptr_t)(pg - 1); };
    uintptr_t a = (uintptr_t)p, b = (uintptr_t)p + n;
    bool drained = false;
    for (size_t i = g.regs.size(); i-- > 0;) {
        Lib::Reg &r = g.regs[i];
        if (page_hi(r.b) <= page_lo(a) || page_hi(b) <= page_lo(r.a)) continue;
        if (r.ok && !drained) { drain_devices(); drained = true; }
        a = a < r.a ? a : r.a;
        b = b > r.b ? b : r.b;
        unregister_range(r);
        g.regs.erase(g.regs.begin() + (long)i);
        g.merges++;
    }
    if (g.regs.size() >= 4) unregister_all();
    // mapped: the host-fill delivery has the GPU write covered bins straight into these pages;
    // uncached (the extended fine-grained pool): with the fragment kernel's line-grid stores the
    // link then carries whole 64-B lines (54.0 vs 52.0 GB/s for a malloc + 16-B buffer,
    // tools/micro/pcie_write.hip).  A runtime that refuses the flag gets the plain registration.
    bool ok = hipHostRegister((void *)a, b - a, hipHostRegisterPortable | hipHostRegisterMapped |
                              hipExtHostRegisterUncached) == hipSuccess;
    if (!ok) {
        (void)hipGetLastError();
        ok = hipHostRegister((void *)a, b - a, hipHostRegisterPortable | hipHostRegisterMapped) == hipSuccess;
    }
    if (!ok) (void)hipGetLastError();
    else g.registrations++;
    g.regs.push_back({a, b, ok});
    return ok;
}

// Drop the registration covering [p, p + n) (a stale one: its pages are no longer the caller's).
void drop_registration(void *p, size_t n) {
    for (size_t i = 0; i < g.regs.size(); i++) {
        const uintptr_t a = (uintptr_t)p, b = a + n;
        if (g.regs[i].a <= a && b <= g.regs[i].b) {
            if (g.regs[i].ok) drain_devices();
            unregister_range(g.regs[i]);
            g.regs.erase(g.regs.begin() + (long)i);
            return;
        }
    }
}

// A cached registration is keyed by its address range.  If the caller freed its buffer and got a new
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

uint32_t band_rows_local(uint32_t height, uint32_t band_rows, uint32_t n_parts, uint32_t part) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts) return 0;
    uint32_t rows = 0;
    for (uint64_t b = part; b * band_rows < height; b += n_parts) {
        const uint64_t y0 = b * band_rows;
        rows += (uint32_t)((height - y0) < band_rows ? (height - y0) : band_rows);
    }
    return rows;
}

// One part's rows (compact on the device, as render_core wrote them) into their frame rows of a host
// frame, asynchronously on st: one 2-D copy for the part's full bands (band_rows x W blocks spaced
// n_parts bands apart) and one for a trailing partial band.
void copy_bands_to_host(const uint32_t *dev_rows, uint32_t W, uint32_t H, uint32_t band_rows, uint32_t n_parts,
                        uint32_t part, uint32_t *host_frame, hipStream_t st) {
    const size_t rowb = (size_t)W * sizeof(uint32_t);
    const uint32_t nbands = (H + band_rows - 1) / band_rows, last = nbands - 1u;
    const uint32_t mine = (nbands > part) ? (nbands - part + n_parts - 1u) / n_parts : 0u;
    const bool partial_last = (uint64_t)nbands * band_rows > H && last % n_parts == part;
    const uint32_t full = mine - (partial_last ? 1u : 0u);
    if (full)
        HIPCHECK(hipMemcpy2DAsync(host_frame + (size_t)part * band_rows * W, (size_t)n_parts * band_rows * rowb, dev_rows,
                                  (size_t)band_rows * rowb, (size_t)band_rows * rowb, full, hipMemcpyDeviceToHost, st));
    if (partial_last)
        HIPCHECK(hipMemcpyAsync(host_frame + (size_t)last * band_rows * W, dev_rows + (size_t)full * band_rows * W,
                                (size_t)(H - last * band_rows) * rowb, hipMemcpyDeviceToHost, st));
}

// ---------------------------------------------------------------- updateAndRender's frame delivery
// Device i's part of the frame is in the caller's buffer: its finish time and link bytes (profile).
void note_device_done(int i, uint64_t link_bytes) {
    Lib::DevProf &p = g.dev_prof[i];
    p.frames++;
    p.end_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() -
                                                                                 g.call_t0).count();
    p.link_bytes = link_bytes;
}

struct Delivery {
    uint32_t W, H, band, nparts;
    uint32_t *host;            // the caller's buffer (whole frame)
    size_t copy_bytes;         // single device: bytes of the frame copied (min(bufferSize, 4 W H))
    bool copy_only;            // redo the copies of the frame already rendered (stale registration)
};

// Part i of the frame on device i: render its rows, copy them into the caller's buffer over this
// device's link, wait for both.  Runs on the calling thread (i = 0) or device i's worker thread.
void deliver_part(void *arg, int i) {
    const Delivery &job = *static_cast<const Delivery *>(arg);
    Dev &d = *g.devs[i];
    HIPCHECK(hipSetDevice(d.device));
    const uint32_t rows = job.nparts == 1 ? job.H : band_rows_local(job.H, job.band, job.nparts, (uint32_t)i);
    if (rows && job.W) {
        const size_t npx = (size_t)job.W * rows;
        if (d.frame_cap < npx) {
            if (d.frame) HIPCHECK(hipFree(d.frame));
            d.frame = dalloc<uint32_t>(npx);
            d.frame_cap = npx;
        }
        if (!job.copy_only)
            render_core(d, job.W, job.H, job.nparts == 1 ? job.H : job.band, job.nparts, (uint32_t)i, rows, d.frame,
                        d.stream, nullptr, true);
        if (job.nparts == 1) {
            if (job.copy_bytes)
                HIPCHECK(hipMemcpyAsync(job.host, d.frame, job.copy_bytes, hipMemcpyDeviceToHost, d.stream));
        } else {
            copy_bands_to_host(d.frame, job.W, job.H, job.band, job.nparts, (uint32_t)i, job.host, d.stream);
        }
    }
    sync_stream(d.stream, WaitSite{"updateAndRender: the frame part rendered and copied to the caller", "the frame's kernels and copy", d.device, d.frame_no});
    if (rows && job.W && tile_redo_if_overflowed(d, d.stream)) {
        // the tile list was too short for this frame: rendered again, delivered again
        if (job.nparts == 1) {
            if (job.copy_bytes)
                HIPCHECK(hipMemcpyAsync(job.host, d.frame, job.copy_bytes, hipMemcpyDeviceToHost, d.stream));
        } else {
            copy_bands_to_host(d.frame, job.W, job.H, job.band, job.nparts, (uint32_t)i, job.host, d.stream);
        }
        sync_stream(d.stream, WaitSite{"updateAndRender: the frame part rendered and copied to the caller", "the frame's kernels and copy", d.device, d.frame_no});
    }
    note_device_done(i, job.nparts == 1 ? job.copy_bytes : (uint64_t)rows * job.W * 4);
}

// ---------------------------------------------------------------- deliveries
// How updateAndRender's frame reaches the caller's host buffer.  The PCIe link is the bound: a 4K
// frame is 33 MB, rendered in ~60 us but carried in ~0.6 ms.
//   copy    every device renders its rows into HBM, then the DMA engine copies them into their rows
//           of the caller's page-locked buffer (deliver_part above).
//   direct  the fragment kernel writes its pixels straight into their rows of the caller's mapped,
//           page-locked buffer (frame_rows): the link's transfer overlaps the rendering, and no DMA
//           setup is paid (kernel stores to registered host memory measured at 55.7 GB/s against
//           ~50 GB/s for the copy, tools/micro/pcie_write.hip).
//   fill    (host fill) as direct, but typically half the frame's bins are sky -- bins no triangle
//           meets, all background (render.cpp:282): each device publishes every bin's sky flag as
//           soon as its geometry has binned the triangles (k_geometry), writes only its covered bins, and the
//           library's fill threads write the sky bins' background with streaming stores meanwhile.
//           The link carries the covered bins only; the host's memory writes overlap the GPU's.
// The host fill is adaptive: with N devices the links carry N times the bytes of one while the fill
// threads' memory bandwidth stays what it is, so the flags leave g/8 of the sky bins (bin % 8 < g)
// to the GPUs, and after every frame g moves one step where that shortens the frame.  Moving an
// eighth to the GPUs adds its bytes to the links (L us) and takes its fill (F us) off the threads:
// worth it when the threads' sky fill ends more than L after the devices; moving one back is worth
// it when the devices end more than F after the sky fill (smoothed over frames).  The threads' end
// itself is no measure: the covered bins' background chunks are filled as the last fragment
// workgroups finish, so the threads never end much before the devices -- judged by it, g only ever
// climbed.  Any g gives the same pixels; g = 8 is direct delivery plus the flags.  S3R_FILL_GPU=g
// fixes it.
// Auto = host fill.  Tile-path frames and buffers that cannot be page-locked are copied.
constexpr int kDefaultFillThreads = 4;     // one device; measured: 2 CPU-bound, 8-16 add scheduling jitter (p90)
constexpr int kDefaultFillThreadsMulti = 8;
constexpr double kLinkBytesPerUs = 52000.0;  // one device's link for delivered pixels (~52 GB/s)
constexpr double kFillEighthUs0 = 30.0;       // F before the first measurement (4K, 4 threads)
enum Delivery_ { kAuto = 0, kCopy = 1, kDirect = 2, kFill = 3 };

int delivery_mode() {
    if (g.delivery < 0) {
        const char *e = getenv("S3R_DELIVERY");
        g.delivery = !e ? kAuto : !strcmp(e, "copy") ? kCopy : !strcmp(e, "direct") ? kDirect
                   : !strcmp(e, "fill") ? kFill : kAuto;
    }
    return g.delivery;
}

constexpr uint32_t kFillBlock = 8;            // bins per fill-thread work block (contiguous: whole lines)

// CPUs this process may keep busy: its affinity mask, capped by a cgroup v2 CPU quota (cpu.max,
// e.g. "1600000 100000" = 16 CPUs).  Busy threads beyond a quota get the whole process throttled.
int available_cpus() {
    static int n = -1;
    if (n >= 0) return n;
    cpu_set_t set;
    n = sched_getaffinity(0, sizeof set, &set) == 0 ? CPU_COUNT(&set) : 64;
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
        char q[32] = {0};
        long period = 0;
        if (fscanf(f, "%31s %ld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
            const long quota = atol(q);
            const int c = (int)(quota / period);
            if (c > 0 && c < n) n = c;
        }
        fclose(f);
    }
    return n;
}

// Where the fill threads run.  The fill is streaming stores into the caller's buffer, ~20 GB/s per
// core; on a chiplet CPU (EPYC: 8 cores per L3 / CCD, one link into the I/O die per CCD) the
// writes of one CCD share that link, and writes to the other socket's memory cross the socket
// link.  Unplaced, two fill threads may share a CCD or sit on the far socket, and a frame's fill
// then takes up to half again as long (measured on the MI355X host, an EPYC 9575F shared with
// other jobs).  So each fill thread gets a CCD of its own (all that CCD's CPUs: the scheduler picks
// the core), on the buffer's NUMA node first, least busy CCDs first (/proc/stat over 10 ms).
// S3R_FILL_PIN=0: no placement.
struct CpuDomain {
    std::vector<int> cpus;
    int node = -1;
    double busy = 0;
};

std::vector<int> parse_cpulist(const char *txt) {
    std::vector<int> out;
    const char *p = txt;
    while (*p) {
        char *e;
        const long a = strtol(p, &e, 10);
        if (e == p) break;
        long b = a;
        p = e;
        if (*p == '-') {
            b = strtol(p + 1, &e, 10);
            p = e;
        }
        for (long c = a; c <= b && c < CPU_SETSIZE; c++) out.push_back((int)c);
        while (*p == ',' || *p == '\n' || *p == ' ') p++;
    }
    return out;
}

bool read_text(const std::string &path, char *buf, size_t n) {
    FILE *f = fopen(path.c_str(), "r");
    if (!f) return false;
    const size_t k = fread(buf, 1, n - 1, f);
    fclose(f);
    buf[k] = 0;
    return k > 0;
}

// per-CPU busy jiffies (all fields but idle and iowait) from /proc/stat
std::vector<uint64_t> cpu_busy() {
    std::vector<uint64_t> out;
    FILE *f = fopen("/proc/stat", "r");
    if (!f) return out;
    char line[512];
    while (fgets(line, sizeof line, f)) {
        if (strncmp(line, "cpu", 3) || line[3] < '0' || line[3] > '9') continue;
        int cpu;
        unsigned long long v[8] = {};
        if (sscanf(line + 3, "%d %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, v, v + 1, v + 2, v + 3, v + 4, v + 5,
                   v + 6, v + 7) < 5 || cpu < 0 || cpu >= CPU_SETSIZE)
            continue;
        if ((size_t)cpu >= out.size()) out.resize(cpu + 1, 0);
        out[cpu] = v[0] + v[1] + v[2] + v[5] + v[6] + v[7];
    }
    fclose(f);
    return out;
}

// The process's CPUs grouped by last-level cache, each with its NUMA node (empty: no topology)
std::vector<CpuDomain> cpu_domains() {
    std::vector<CpuDomain> doms;
    cpu_set_t aff;
    if (sched_getaffinity(0, sizeof aff, &aff) != 0) return doms;
    std::vector<int> node_of(CPU_SETSIZE, -1);
    char buf[4096];
    for (int n = 0; n < 64; n++)
        if (read_text("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist", buf, sizeof buf))
            for (int c : parse_cpulist(buf)) node_of[c] = n;
    std::vector<int> seen(CPU_SETSIZE, 0);
    for (int c = 0; c < CPU_SETSIZE; c++) {
        if (!CPU_ISSET(c, &aff) || seen[c]) continue;
        if (!read_text("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/cache/index3/shared_cpu_list", buf, sizeof buf))
            return {};
        CpuDomain d;
        for (int x : parse_cpulist(buf))
            if (x < CPU_SETSIZE && CPU_ISSET(x, &aff) && !seen[x]) {
                seen[x] = 1;
                d.cpus.push_back(x);
            }
        d.node = node_of[c];
        if (!d.cpus.empty()) doms.push_back(d);
    }
    return doms;
}

// NUMA node of the page holding p (-1: unknown)
int page_node(const void *p) {
    int node = -1;
    constexpr unsigned long kMpolFNode = 1, kMpolFAddr = 2;
    if (syscall(SYS_get_mempolicy, &node, nullptr, 0UL, p, kMpolFNode | kMpolFAddr) != 0) return -1;
    return node;
}

// One CPU set per fill thread (empty: leave the threads to the scheduler)
std::vector<cpu_set_t> fill_placement(int threads, int node) {
    std::vector<cpu_set_t> out;
    const char *e = getenv("S3R_FILL_PIN");
    if (e && atoi(e) == 0) return out;
    std::vector<CpuDomain> doms = cpu_domains();
    if (doms.size() < 2) return out;
    const std::vector<uint64_t> b0 = cpu_busy();
    std::this_thread::sleep_for(std::chrono::milliseconds(10));
    const std::vector<uint64_t> b1 = cpu_busy();
    for (auto &d : doms) {
        for (int c : d.cpus)
            if ((size_t)c < b0.size() && (size_t)c < b1.size()) d.busy += (double)(b1[c] - b0[c]);
        d.busy /= (double)d.cpus.size();
    }
    std::stable_sort(doms.begin(), doms.end(), [&](const CpuDomain &a, const CpuDomain &b) {
        const bool la = a.node == node, lb = b.node == node;
        return la != lb ? la : a.busy < b.busy;
    });
    for (int t = 0; t < threads; t++) {
        const CpuDomain &d = doms[(size_t)t % doms.size()];
        cpu_set_t set;
        CPU_ZERO(&set);
        for (int c : d.cpus) CPU_SET(c, &set);
        out.push_back(set);
    }
    return out;
}

// Fill threads for a frame of nparts device parts (S3R_FILL_THREADS / s3r_set_delivery override):
// by default 4 (one device) or 8, but no more than the CPUs left beside the calling thread and the
// nparts - 1 device workers.
int fill_threads(uint32_t nparts = 1) {
    if (g.fill_threads < 0) {
        if (const char *e = getenv("S3R_FILL_THREADS")) {
            const int v = atoi(e);
            g.fill_threads = v < 1 ? 1 : (v > 64 ? 64 : v);
        }
    }
    if (g.fill_threads > 0) return g.fill_threads;
    const int want = nparts > 1 ? kDefaultFillThreadsMulti : kDefaultFillThreads;
    const int spare = available_cpus() - (int)nparts - 1;
    return want < spare ? want : (spare > 1 ? spare : 1);
}

struct FillPart {
    uint32_t *flags;                 // host view of the device's sky flags
    unsigned long long *chunks;      // host view of its covered bins' chunk masks
    uint32_t tag, seg_px, segs, rpb, chunk_px, rows_local, band, nparts, part;
    uint64_t bins;
    const uint32_t *diag;            // the device's error words (Dev::diag_host)
    int device;
};

struct FillJob {
    uint32_t *frame;                 // the caller's buffer (host address)
    uint32_t W, H;
    int nparts, threads;
    FillPart parts[kMaxDevices];
    HostFill hf[kMaxDevices];
    std::atomic<bool> stale{false};  // pixel 0 checked before its bin was filled: the mapping is stale
    std::atomic<uint64_t> sky_px{0}; // background pixels the fill threads wrote
    std::chrono::steady_clock::time_point t0;
    std::atomic<int64_t> dev_end_ns{0}, fill_end_ns{0};   // latest finish of a device part / a fill thread
    // the adaptive split's measures: the first flag any thread saw, the last sky bin a thread filled,
    // and the sky bins of the frame (the host's and the GPUs')
    std::atomic<int64_t> flags_ns{INT64_MAX}, sky_end_ns{0};
    std::atomic<uint64_t> sky_bins{0};
    std::atomic<uint64_t> part_px[kMaxDevices] = {};   // per part, as sky_px
    int64_t issued_ns = 0;                                 // part 0's launches issued
    std::atomic<int> parts_done{0};                        // device parts synchronised
    std::chrono::steady_clock::time_point dev_done_ns[kMaxDevices];   // each device part's end
    int64_t thread_end_ns[65] = {};  // per fill thread (written by that thread, read after the join)
    uint64_t thread_px[65] = {};
    int64_t thread_covered_ns[65] = {};  // time in covered bins (their background chunks)
    int thread_cpu[65] = {};
};

void note_end(const FillJob &job, std::atomic<int64_t> &end) {
    const int64_t t = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - job.t0).count();
    int64_t cur = end.load(std::memory_order_relaxed);
    while (t > cur && !end.compare_exchange_weak(cur, t, std::memory_order_relaxed)) {}
}

// Fills bin b's background -- the whole bin (sky), or the row chunks in mask (bit
// row_in_bin * chunks_per_row + chunk) of a covered bin; returns the pixels written.
uint64_t fill_bin(const FillJob &job, const FillPart &fp, uint64_t b, bool sky, uint32_t mask) {
    const uint32_t blk = (uint32_t)(b / fp.segs), seg = (uint32_t)(b % fp.segs);
    const uint32_t xs = seg * fp.seg_px, xe = xs + fp.seg_px < job.W ? xs + fp.seg_px : job.W;
    const uint32_t cpr = fp.seg_px / fp.chunk_px;
    uint64_t px = 0;
    for (uint32_t k = 0; k < fp.rpb; k++) {
        const uint32_t lr = blk * fp.rpb + k;
        if (lr >= fp.rows_local) break;
        const uint32_t y = ((lr / fp.band) * fp.nparts + fp.part) * fp.band + lr % fp.band;
        if (y >= job.H) continue;
        uint32_t *row = job.frame + (size_t)y * job.W;
        if (sky) {
            s3r_host::fill_words(row + xs, xe - xs, kBackground);
            px += xe - xs;
            continue;
        }
        for (uint32_t q = 0; q < cpr; q++) {
            const uint32_t c0 = xs + q * fp.chunk_px, c1 = c0 + fp.chunk_px < xe ? c0 + fp.chunk_px : xe;
            if (c0 < c1 && ((mask >> (k * cpr + q)) & 1u)) {
                s3r_host::fill_words(row + c0, c1 - c0, kBackground);
                px += c1 - c0;
            }
        }
    }
    return px;
}

// Fill thread idx (1..threads): the blocks of kFillBlock bins it owns in every part, each handled as
// soon as its flags carry this frame's tag: a sky bin (k_sky_flags, right after the geometry) is
// filled whole; a covered bin waits for its workgroup's chunk mask (end of the workgroup) and gets
// the row chunks without a winner filled.
constexpr uint64_t kWaitChunks = 1ull << 47;    // pending entry: sky flag seen, covered, mask awaited

// A fill thread still waiting for flags or chunk masks (bounded waits, above): a sky-flag publisher
// that timed out on its device ends the process at once, naming its row block and arrival count;
// past the deadline, a frame whose device parts have all been synchronised is a flag protocol error,
// and one whose parts are still running a stall (the parts' own waits are bounded by the watchdog).
void fill_check(const FillJob &job, size_t waiting, std::chrono::steady_clock::time_point t0) {
    for (int p = 0; p < job.nparts; p++) {
        const uint32_t *e = job.parts[p].diag;
        if (e && __atomic_load_n(e, __ATOMIC_ACQUIRE) == kDiagPublisherTimeout) {
            fprintf(stderr, "s3r: stall: host fill -- k_geometry's sky-flag publisher of row block %u timed out on device "
                    "%d (frame tag %u): %u of %u geometry workgroups arrived within S3R_SPIN_MS; exiting with status %d\n",
                    __atomic_load_n(e + 1, __ATOMIC_ACQUIRE), job.parts[p].device, job.parts[p].tag,
                    __atomic_load_n(e + 2, __ATOMIC_ACQUIRE), __atomic_load_n(e + 3, __ATOMIC_ACQUIRE), kStallExit);
            fflush(stderr);
            _exit(kStallExit);
        }
    }
    const double waited_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    if (waited_ms <= wait_deadline_ms()) return;
    const WaitSite w{"host fill: the frame's bin flags and chunk masks", "k_geometry's publishers / k_fragment",
                     job.parts[0].device, job.parts[0].tag};
    if (job.parts_done.load(std::memory_order_acquire) == job.nparts) {
        fprintf(stderr, "s3r: host fill: %zu bins never flagged although every device part finished (flag protocol "
                "broken)\n", waiting);
        stall_exit(w, "every device part finished", waited_ms);
    }
    stall_exit(w, "device parts still running", waited_ms);
}

void fill_worker(void *arg, int idx) {
    FillJob &job = *static_cast<FillJob *>(arg);
    const uint64_t t = (uint64_t)idx - 1, T = (uint64_t)job.threads;
    thread_local std::vector<uint64_t> pend;
    pend.clear();
    for (int p = 0; p < job.nparts; p++)
        for (uint64_t b = t * kFillBlock; b < job.parts[p].bins; b += T * kFillBlock)
            for (uint64_t k = b; k < b + kFillBlock && k < job.parts[p].bins; k++) pend.push_back((uint64_t)p << 48 | k);
    size_t n = pend.size();
    const auto t0 = std::chrono::steady_clock::now();
    auto since_start = [&job]() {
        return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - job.t0).count();
    };
    uint32_t idle = 0;
    uint64_t px = 0, sky_bins = 0;
    thread_local std::vector<uint64_t> ppx;                 // per part: background pixels
    ppx.assign((size_t)job.nparts, 0);
    int64_t covered_ns = 0;
    int64_t first_flag = -1, sky_end = 0;
    while (n) {
        size_t keep = 0;
        for (size_t i = 0; i < n; i++) {
            const uint64_t e = pend[i];
            const uint32_t part = (uint32_t)(e >> 48);
            const FillPart &fp = job.parts[part];
            const uint64_t b = e & (kWaitChunks - 1);
            bool sky = false;
            uint32_t mask = 0;
            if (!(e & kWaitChunks)) {
                const uint32_t f = __atomic_load_n(fp.flags + b, __ATOMIC_ACQUIRE);
                if ((f & ~(kSkyBit | kGpuBit)) != fp.tag) { pend[keep++] = e; continue; }
                if (first_flag < 0) first_flag = since_start();
                sky_bins += (f & (kSkyBit | kGpuBit)) ? 1u : 0u;
                if (f & kGpuBit) continue;                      // a sky bin the GPU writes itself
                if (!(f & kSkyBit)) { pend[keep++] = e | kWaitChunks; continue; }
                sky = true;
            } else {
                const unsigned long long c = __atomic_load_n(fp.chunks + b, __ATOMIC_ACQUIRE);
                if ((uint32_t)(c >> 32) != fp.tag) { pend[keep++] = e; continue; }
                mask = (uint32_t)c;
                if (!mask) continue;
            }
            // pixel 0 (part 0, bin 0, its first row and chunk): the flag publisher wrote kMapProbe
            // there through its mapping before publishing the bin's flag; the host writes pixel 0 when
            // the chunk is background
            if (part == 0 && b == 0 && (sky || (mask & 1u)) && __atomic_load_n(job.frame, __ATOMIC_ACQUIRE) != kMapProbe)
                job.stale.store(true, std::memory_order_relaxed);
            const uint64_t px0 = px;
            if (!sky) {
                const auto w0 = std::chrono::steady_clock::now();
                px += fill_bin(job, fp, b, sky, mask);
                covered_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - w0).count();
            } else {
                px += fill_bin(job, fp, b, sky, mask);
            }
            ppx[part] += px - px0;
            if (sky) sky_end = since_start();
        }
        if (keep == n) {
            __builtin_ia32_pause();
            if ((++idle & 4095u) == 0) fill_check(job, keep, t0);
        }
        n = keep;
    }
    s3r_host::store_fence();
    job.sky_px.fetch_add(px, std::memory_order_relaxed);
    for (int p = 0; p < job.nparts; p++)
        if (ppx[p]) job.part_px[p].fetch_add(ppx[p], std::memory_order_relaxed);
    job.sky_bins.fetch_add(sky_bins, std::memory_order_relaxed);
    if (first_flag >= 0) {
        int64_t cur = job.flags_ns.load(std::memory_order_relaxed);
        while (first_flag < cur && !job.flags_ns.compare_exchange_weak(cur, first_flag, std::memory_order_relaxed)) {}
    }
    if (sky_end) {
        int64_t cur = job.sky_end_ns.load(std::memory_order_relaxed);
        while (sky_end > cur && !job.sky_end_ns.compare_exchange_weak(cur, sky_end, std::memory_order_relaxed)) {}
    }
    job.thread_px[idx] = px;
    job.thread_covered_ns[idx] = covered_ns;
    job.thread_cpu[idx] = sched_getcpu();
    job.thread_end_ns[idx] = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - job.t0).count();
    note_end(job, job.fill_end_ns);
}

// The device address of host buffer p inside registration r on device d (cached per registration).
// Null if this device has no mapping of the registration (the frame is then delivered by copy).
uint32_t *mapped_ptr(Dev &d, const Lib::Reg &r, void *p) {
    if (d.map_epoch != g.reg_epoch || d.map_host != r.a) {
        void *dp = nullptr;
        if (hipHostGetDevicePointer(&dp, (void *)r.a, 0) != hipSuccess) {
            (void)hipGetLastError();
            dp = nullptr;
        }
        d.map_host = r.a;
        d.map_dev = (uintptr_t)dp;
        d.map_epoch = g.reg_epoch;
    }
    return d.map_dev ? (uint32_t *)(d.map_dev + ((uintptr_t)p - r.a)) : nullptr;
}

struct DirectDelivery {
    FillJob *job;
    uint32_t *frame_dev[kMaxDevices];    // each device's address of the caller's buffer
};

// Part i of a direct / host-fill frame on device i: render it into the caller's mapped buffer.
void deliver_part_direct(void *arg, int i) {
    const DirectDelivery &dd = *static_cast<const DirectDelivery *>(arg);
    FillJob &job = *dd.job;
    Dev &d = *g.devs[i];
    HIPCHECK(hipSetDevice(d.device));
    const FillPart &fp = job.parts[i];
    if (fp.rows_local && job.W) {
        uint32_t *frame_dev = dd.frame_dev[i];
        HostFill hf = job.hf[i];
        hf.probe_dev = i == 0 && hf.flags_dev ? frame_dev : nullptr;
        render_core(d, job.W, job.H, fp.band, fp.nparts, fp.part, fp.rows_local, frame_dev, d.stream, &hf, true);
    }
    if (i == 0)
        job.issued_ns = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - job.t0).count();
    sync_stream(d.stream, WaitSite{"updateAndRender: the frame part written into the caller's buffer", "the frame's kernels", d.device, d.frame_no});
    // a tile-path frame whose list overflowed is rendered again, into the same rows
    if (fp.rows_local && job.W) tile_redo_if_overflowed(d, d.stream);
    job.parts_done.fetch_add(1, std::memory_order_acq_rel);
    note_end(job, job.dev_end_ns);
    job.dev_done_ns[i] = std::chrono::steady_clock::now();
}

// One updateAndRender frame by direct delivery or host fill (fill).  kStaleMap: the caller's
// registration turned out to be stale (the frame did not reach the caller's pages); kUnmapped: a
// device has no mapping of the buffer (nothing was rendered) -- either way the caller redoes the
// frame by copy.
enum MappedResult { kMapped, kStaleMap, kUnmapped };

// One step of the adaptive split (see "deliveries" above) after a host-fill frame.
void fill_adapt(const FillJob &job, uint32_t nparts) {
    const double dev = (double)job.dev_end_ns.load() / 1e3, t_flags = (double)job.flags_ns.load() / 1e3;
    const double sky_end = job.sky_end_ns.load() ? (double)job.sky_end_ns.load() / 1e3 : t_flags;
    const int host = 8 - g.fill_gpu;
    if (host > 0 && job.sky_end_ns.load()) {
        const double f = (sky_end - t_flags) / host;
        g.fill_eighth_us = g.fill_eighth_us > 0 ? 0.75 * g.fill_eighth_us + 0.25 * f : f;
    }
    const double F = g.fill_eighth_us > 0 ? g.fill_eighth_us : kFillEighthUs0;
    const FillPart &fp = job.parts[0];
    const double L = (double)job.sky_bins.load() * fp.seg_px * fp.rpb * 4.0 / 8.0 / (kLinkBytesPerUs * nparts);
    g.fill_skew_us = 0.75 * g.fill_skew_us + 0.25 * (sky_end - dev);
    if (g.fill_skew_us > L && g.fill_gpu < 8) { g.fill_gpu++; g.fill_skew_us = 0; }
    else if (-g.fill_skew_us > F && g.fill_gpu > 0) { g.fill_gpu--; g.fill_skew_us = 0; }
}

MappedResult mapped_frame(uint32_t *buffer, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, bool fill) {
    const Lib::Reg *reg = find_reg(buffer, (size_t)W * H * 4);
    DirectDelivery dd{};
    for (uint32_t i = 0; i < nparts; i++) {
        Dev &d = *g.devs[i];
        HIPCHECK(hipSetDevice(d.device));
        dd.frame_dev[i] = reg ? mapped_ptr(d, *reg, buffer) : nullptr;
        if (!dd.frame_dev[i]) {
            HIPCHECK(hipSetDevice(g.devs[0]->device));
            return kUnmapped;
        }
    }
    FillJob job;
    job.frame = buffer;
    job.W = W;
    job.H = H;
    job.nparts = (int)nparts;
    job.threads = fill ? fill_threads(nparts) : 0;
    if (fill && g.fill_gpu < 0) {
        const char *e = getenv("S3R_FILL_GPU");
        g.fill_gpu = e ? atoi(e) : (int)(2 * (nparts - 1));
        g.fill_gpu = g.fill_gpu < 0 ? 0 : (g.fill_gpu > 8 ? 8 : g.fill_gpu);
    }
    if (fill) {
        // (re)start the fill threads, placed for this buffer's memory node, when the thread count
        // changes, or when the buffer has sat on another node for kNodeStreak frames in a row (the two
        // halves of a double buffer on different nodes must not re-place them every frame: a
        // placement samples the CPUs' load for 10 ms)
        constexpr int kNodeStreak = 16;
        const int node = page_node(buffer);
        g.fill_node_streak = node == g.fill_node ? 0 : g.fill_node_streak + 1;
        if (g.fill_pool.workers() != job.threads || g.fill_node_streak >= kNodeStreak) {
            g.fill_node_streak = 0;
            const std::vector<cpu_set_t> cpus = fill_placement(job.threads, node);
            g.fill_pool.start(job.threads, cpus.empty() ? nullptr : &cpus);
            g.fill_node = node;
            g.fill_placed = !cpus.empty();
        }
    }
    if (nparts == 1) band = H;
    for (uint32_t i = 0; i < nparts; i++) {                 // the parts' bin layouts
        FillPart &fp = job.parts[i];
        fp.rows_local = nparts == 1 ? H : band_rows_local(H, band, nparts, i);
        const FragLayout l = fragment_layout(W, fp.rows_local);
        fp.seg_px = l.seg_px; fp.segs = l.segs; fp.rpb = l.rows_per_bin; fp.chunk_px = l.chunk_px;
        fp.bins = fp.rows_local ? l.bins : 0;
        fp.band = band; fp.nparts = nparts; fp.part = i;
        fp.diag = g.devs[i]->diag_host;
        fp.device = g.devs[i]->device;
    }
    for (uint32_t i = 0; i < nparts; i++) {
        Dev &d = *g.devs[i];
        FillPart &fp = job.parts[i];
        if (!fill) {
            job.hf[i] = HostFill{nullptr, 0, nullptr, nullptr, 0};
            continue;
        }
        if (d.fill_cap < fp.bins) {
            HIPCHECK(hipSetDevice(d.device));
            if (d.fill_flags) HIPCHECK(hipHostFree(d.fill_flags));
            if (d.fill_chunks) HIPCHECK(hipHostFree(d.fill_chunks));
            const unsigned flags = hipHostMallocCoherent | hipHostMallocMapped | hipHostMallocPortable;
            HIPCHECK(hipHostMalloc((void **)&d.fill_flags, fp.bins * sizeof(uint32_t), flags));
            HIPCHECK(hipHostMalloc((void **)&d.fill_chunks, fp.bins * sizeof(unsigned long long), flags));
            memset(d.fill_flags, 0, fp.bins * sizeof(uint32_t));
            memset(d.fill_chunks, 0, fp.bins * sizeof(unsigned long long));
            HIPCHECK(hipHostGetDevicePointer((void **)&d.fill_flags_dev, d.fill_flags, 0));
            HIPCHECK(hipHostGetDevicePointer((void **)&d.fill_chunks_dev, d.fill_chunks, 0));
            d.fill_cap = fp.bins;
            d.fill_tag = 0;
        }
        if (++d.fill_tag >= kGpuBit) {                 // (after 2^30 frames) restart the tags
            memset(d.fill_flags, 0, d.fill_cap * sizeof(uint32_t));
            memset(d.fill_chunks, 0, d.fill_cap * sizeof(unsigned long long));
            d.fill_tag = 1;
        }
        fp.flags = d.fill_flags;
        fp.chunks = d.fill_chunks;
        fp.tag = d.fill_tag;
        job.hf[i] = HostFill{d.fill_flags_dev, d.fill_tag, nullptr, d.fill_chunks_dev, (uint32_t)g.fill_gpu};
    }
    HIPCHECK(hipSetDevice(g.devs[0]->device));
    buffer[0] = kStaleProbe;      // overwritten through the mapping (a pixel, or k_sky_flags' probe)
    dd.job = &job;
    job.t0 = std::chrono::steady_clock::now();
    if (fill) g.fill_pool.launch(fill_worker, &job, job.threads + 1);
    g.pool.run(deliver_part_direct, &dd, (int)nparts);
    if (fill) {
        g.fill_pool.join();
        g.prof_frames++;
        const auto now = std::chrono::steady_clock::now();
        g.prof_pre_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(job.t0 - g.call_t0).count();
        g.prof_issued_ns += (uint64_t)job.issued_ns;
        g.prof_done_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(now - job.t0).count();
        g.prof_dev_ns += (uint64_t)job.dev_end_ns.load();
        g.prof_fill_ns += (uint64_t)job.fill_end_ns.load();
        for (int t = 1; t <= job.threads && t <= 64; t++) {
            g.prof_thread[t].cpu = job.thread_cpu[t];
            g.prof_thread[t].end_ns += (uint64_t)job.thread_end_ns[t];
            g.prof_thread[t].px += job.thread_px[t];
            g.prof_thread[t].covered_ns += (uint64_t)job.thread_covered_ns[t];
        }
    }
    if (fill && !getenv("S3R_FILL_GPU") && job.flags_ns.load() != INT64_MAX) fill_adapt(job, nparts);
    // pixel 0 written by the GPU (direct, or a covered chunk under host fill) is a pixel, neither
    // probe, unless the mapping is stale; a pixel 0 the host filled was checked by its fill thread
    bool host0 = false;
    if (fill && job.parts[0].bins) {
        const uint32_t f0 = job.parts[0].flags[0];
        host0 = (f0 & kSkyBit) || (!(f0 & kGpuBit) && (job.parts[0].chunks[0] & 1ull));
    }
    const bool stale = job.stale.load() || (!host0 && (buffer[0] == kStaleProbe || buffer[0] == kMapProbe));
    if (stale) return kStaleMap;             // (redone by copy, which profiles the frame itself)
    (fill ? g.fill_frames : g.direct_frames)++;
    g.link_bytes = 4 * ((uint64_t)W * H - job.sky_px.load());
    for (uint32_t i = 0; i < nparts; i++) {
        Lib::DevProf &dp = g.dev_prof[i];
        const uint64_t px = (uint64_t)job.parts[i].rows_local * W, sky = job.part_px[i].load();
        dp.frames++;
        dp.end_ns += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(job.dev_done_ns[i] - g.call_t0).count();
        dp.link_bytes = 4 * (px - sky);
    }
    return kMapped;
}

// Bins mode: the last tile-path frame's binned-entry total (summary word 2) is written by its last
// kernel; the statistics read it once the device is drained.
void refresh_pairs(Dev &d) {
    if (d.last_path != 2 || !d.last_set_bins || d.last_set < 0 || !d.tile_sum_host) return;
    // only the last tile frame's fragment stage, and the caller's current device left as it was
    int prev = -1;
    HIPCHECK(hipGetDevice(&prev));
    HIPCHECK(hipSetDevice(d.device));
    sync_event(d.frag_done[d.last_set], WaitSite{"statistics: the last tile frame", "k_tile_raster", d.device, d.frame_no});
    d.last_pairs = __atomic_load_n(d.tile_sum_host + kSumWords * (uint32_t)d.last_set + 2, __ATOMIC_ACQUIRE);
    HIPCHECK(hipSetDevice(prev));
}

}  // namespace

namespace s3r {
void sync_stream_bounded(hipStream_t st, const char *stage, const char *kernel, int device, uint32_t frame) {
    sync_stream(st, WaitSite{stage, kernel, device, frame});
}
}  // namespace s3r

extern "C" {

__attribute__((visibility("default"))) void updateAndRender(const PixelData *pixel_data, const Input *input) {
    g.call_t0 = std::chrono::steady_clock::now();
    const uint32_t W = pixel_data->width, H = pixel_data->height;
    frame_begin(input, W, H);
    const size_t npx = (size_t)W * H;
    // memset_pattern4 fills bufferSize bytes (render.cpp:282); the frame covers W*H pixels.
    const size_t frame_bytes = npx * 4;
    const size_t copy_bytes = pixel_data->bufferSize < frame_bytes ? pixel_data->bufferSize : frame_bytes;
    const size_t copy_words = copy_bytes / 4;
    // several devices: each renders its interleaved bands and copies them into their rows (a caller
    // buffer smaller than the frame -- not the reference's usage -- takes the one-device path)
    const uint32_t ndev = (uint32_t)g.devs.size();
    const uint32_t band = frame_band(H, ndev);
    const uint32_t nparts = (ndev > 1 && copy_bytes == frame_bytes && H > band) ? ndev : 1u;
    Delivery job{W, H, band, nparts, pixel_data->buffer, copy_bytes, false};
    bool pinned = false;
    if (copy_bytes) pinned = host_pinned(pixel_data->buffer, pixel_data->bufferSize);
    const int mode = delivery_mode();
    if (pinned && npx && copy_bytes == frame_bytes && mode != kCopy) {
        // direct / host fill: the GPU(s) write straight into the buffer (host fill: covered bins only,
        // the sky bins by the host; the tile path delivers direct -- its resolve writes every pixel)
        const bool fill = (mode == kFill || mode == kAuto) && !use_tile_path();
        const Lib::Reg *reg = find_reg(pixel_data->buffer, frame_bytes);
        const bool unmapped = reg && g.unmapped_epoch == g.reg_epoch && g.unmapped_a == reg->a;
        const MappedResult mr = unmapped ? kUnmapped : mapped_frame(pixel_data->buffer, W, H, band, nparts, fill);
        if (mr == kMapped) {
            g.pinned_frames++;
            for (size_t i = frame_bytes / 4; i < pixel_data->bufferSize / 4; i++) pixel_data->buffer[i] = kBackground;
            HIPCHECK(hipSetDevice(g.devs[0]->device));
            return;
        }
        if (mr == kStaleMap) {
            // the registration no longer maps the caller's pages: pin anew, render the frame by copy
            drop_registration(pixel_data->buffer, pixel_data->bufferSize);
            g.stale_pins++;
            pinned = host_pinned(pixel_data->buffer, pixel_data->bufferSize);
        } else if (!unmapped && reg) {
            // a device cannot address this registration: its frames go by copy
            g.unmapped_a = reg->a;
            g.unmapped_epoch = g.reg_epoch;
            fprintf(stderr, "s3r: a device has no mapping of the caller's buffer; delivering it by copy\n");
        }
    }
    if (copy_bytes) {
        if (pinned && copy_words) stamp_probes(pixel_data->buffer, copy_words);
        (pinned ? g.pinned_frames : g.pageable_frames)++;
        g.copy_frames++;
    }
    if (npx) g.pool.run(deliver_part, &job, (int)nparts);
    g.link_bytes = copy_bytes;
    for (size_t i = frame_bytes / 4; i < pixel_data->bufferSize / 4; i++) pixel_data->buffer[i] = kBackground;
    if (pinned && copy_words && !probes_overwritten(pixel_data->buffer, copy_words)) {
        // a stale registration (buffer freed and reallocated at the same address): pin anew, copy again
        drop_registration(pixel_data->buffer, pixel_data->bufferSize);
        g.stale_pins++;
        host_pinned(pixel_data->buffer, pixel_data->bufferSize);
        job.copy_only = true;
        g.pool.run(deliver_part, &job, (int)nparts);
    }
    HIPCHECK(hipSetDevice(g.devs[0]->device));
}

__attribute__((visibility("default"))) int s3r_configure(const char *data_path, int device) {
    release_all();
    g.data_path = data_path ? data_path : "";
    g.device = device;
    return 0;
}

__attribute__((visibility("default"))) int s3r_configure_devices(const int *device_ids, int n_devices,
                                                                uint32_t band_rows) {
    if (n_devices < 0 || n_devices > kMaxDevices || (n_devices > 0 && !device_ids)) return -1;
    for (int i = 0; i < n_devices; i++)
        if (device_ids[i] < 0) return -1;
    release_all();
    g.device_ids.assign(device_ids, device_ids + n_devices);
    g.band_rows = band_rows;
    return 0;
}

__attribute__((visibility("default"))) uint32_t s3r_frame_band(uint32_t height, uint32_t n_parts) {
    return frame_band(height, n_parts);
}

__attribute__((visibility("default"))) int s3r_devices(int *out_ids, int max_ids) {
    std::vector<int> ids;
    if (g.initialized) {
        for (Dev *d : g.devs) ids.push_back(d->device);
    } else {
        ids = g.device_ids;
        if (ids.empty()) ids = parse_devices(getenv("S3R_DEVICES"));
        if (ids.empty()) ids.push_back(g.device);
    }
    for (int i = 0; i < max_ids && i < (int)ids.size(); i++) out_ids[i] = ids[i];
    return (int)ids.size();
}

__attribute__((visibility("default"))) void s3r_shutdown(void) {
    for (Dev *d : g.devs) d->hp.report(d->device);
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
    return band_rows_local(height, band_rows, n_parts, part);
}

__attribute__((visibility("default"))) int64_t s3r_render_bands(const Input *input, uint32_t width, uint32_t height,
                                                               uint32_t band_rows, uint32_t n_parts, uint32_t part,
                                                               uint32_t *dev_out, void *stream) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts || (!dev_out && width && height)) return -1;
    hipStream_t st = (hipStream_t)stream;   // NULL is the legacy default (null) stream -- e.g. torch's default
    if (!g.initialized) {
        frame_begin(input, width, height);
    } else {
        g.devs[0]->hp.start();
        frame_begin(input, width, height);
        g.devs[0]->hp.lap(0);
    }
    Dev &d = *g.devs[0];
    const uint32_t rows = band_rows_local(height, band_rows, n_parts, part);
    if (rows && width) render_core(d, width, height, band_rows, n_parts, part, rows, dev_out, st);
    return rows;
}

// Test hook: drain the device and continue the frame count at `frame_no` (tags above every tag in use
// keep the completion chain valid), to exercise the tag restart before the uint32 count wraps.
__attribute__((visibility("default"))) void s3r_debug_set_frame_count(uint32_t frame_no) {
    if (!g.initialized) return;
    for (Dev *d : g.devs) {
        HIPCHECK(hipSetDevice(d->device));
        restart_tags(*d, frame_no > kTagLimit ? kTagLimit : frame_no);
    }
    HIPCHECK(hipSetDevice(g.devs[0]->device));
}

__attribute__((visibility("default"))) int64_t s3r_bands_to_host(const uint32_t *dev_rows, uint32_t width, uint32_t height,
                                                                uint32_t band_rows, uint32_t n_parts, uint32_t part,
                                                                uint32_t *host_frame, void *stream) {
    if (band_rows == 0 || n_parts == 0 || part >= n_parts || ((!dev_rows || !host_frame) && width && height)) return -1;
    const uint32_t rows = band_rows_local(height, band_rows, n_parts, part);
    if (!rows || !width) return rows;
    if (g.initialized) HIPCHECK(hipSetDevice(g.devs[0]->device));
    else if (g.device >= 0) HIPCHECK(hipSetDevice(g.device));
    host_pinned(host_frame, (size_t)width * height * sizeof(uint32_t));
    copy_bands_to_host(dev_rows, width, height, band_rows, n_parts, part, host_frame, (hipStream_t)stream);
    return rows;
}

__attribute__((visibility("default"))) int s3r_deinterleave_bands(const uint32_t *gathered, uint32_t part_stride_rows,
                                                                 uint32_t width, uint32_t height, uint32_t band_rows,
                                                                 uint32_t n_parts, uint32_t *frame, void *stream) {
    if (band_rows == 0 || n_parts == 0 || ((!gathered || !frame) && width && height)) return -1;
    for (uint32_t p = 0; p < n_parts; p++)            // every part's rows must fit its stride
        if (band_rows_local(height, band_rows, n_parts, p) > part_stride_rows) return -1;
    if (g.initialized) HIPCHECK(hipSetDevice(g.devs[0]->device));
    else if (g.device >= 0) HIPCHECK(hipSetDevice(g.device));
    launch_deinterleave_bands(gathered, part_stride_rows, width, height, band_rows, n_parts, frame, (hipStream_t)stream);
    HIPCHECK(hipGetLastError());
    return 0;
}

__attribute__((visibility("default"))) void s3r_unregister_host(void *ptr) {
    if (!ptr) return;
    for (size_t i = g.regs.size(); i-- > 0;) {
        const uintptr_t a = (uintptr_t)ptr;
        if (a < g.regs[i].a || a >= g.regs[i].b) continue;
        if (g.regs[i].ok) {
            if (g.initialized) drain_devices();
            else {
                if (g.device >= 0) HIPCHECK(hipSetDevice(g.device));
                sync_device("s3r_unregister_host: before the registration goes", g.device);          // no copy into it may still be in flight
            }
        }
        unregister_range(g.regs[i]);
        g.regs.erase(g.regs.begin() + (long)i);
    }
}

__attribute__((visibility("default"))) int s3r_host_pinned(const void *ptr, uint64_t bytes) {
    const Lib::Reg *r = ptr ? find_reg(ptr, (size_t)bytes) : nullptr;
    return r && r->ok ? 1 : 0;
}

__attribute__((visibility("default"))) void s3r_host_stats(uint64_t out[12]) {
    out[0] = g.pinned_frames;
    out[1] = g.pageable_frames;
    out[2] = g.registrations;
    out[3] = g.merges;
    out[4] = g.regs.size();
    out[5] = g.stale_pins;
    out[6] = g.copy_frames;
    out[7] = g.direct_frames;
    out[8] = g.fill_frames;
    out[9] = (uint64_t)fill_threads(g.devs.size() > 1 ? (uint32_t)g.devs.size() : 1u);
    out[10] = g.link_bytes;
    out[11] = g.fill_gpu < 0 ? 0 : (uint64_t)g.fill_gpu;
}

__attribute__((visibility("default"))) uint32_t s3r_device_profile(uint64_t *out, uint32_t max_devices) {
    const uint32_t n = std::min<uint32_t>((uint32_t)g.devs.size(), max_devices);
    for (uint32_t i = 0; i < n; i++) {
        out[4 * i] = (uint64_t)g.devs[i]->device;
        out[4 * i + 1] = g.dev_prof[i].frames;
        out[4 * i + 2] = g.dev_prof[i].end_ns;
        out[4 * i + 3] = g.dev_prof[i].link_bytes;
        g.dev_prof[i] = Lib::DevProf{};
    }
    return n;
}

__attribute__((visibility("default"))) uint32_t s3r_fill_profile(uint64_t *out, uint32_t max_threads) {
    uint32_t n = 0;
    for (uint32_t t = 1; t <= 64; t++)
        if (g.prof_thread[t].cpu >= 0) n = t;
    n = n < max_threads ? n : max_threads;
    out[0] = g.prof_frames;
    out[1] = g.prof_pre_ns;
    out[2] = g.prof_issued_ns;
    out[3] = g.prof_dev_ns;
    out[4] = g.prof_fill_ns;
    out[5] = g.prof_done_ns;
    out[6] = g.fill_placed ? 1 : 0;
    out[7] = (uint64_t)(int64_t)g.fill_node;
    for (uint32_t t = 1; t <= n; t++) {
        uint64_t *o = out + 8 + 4 * (t - 1);
        o[0] = (uint64_t)g.prof_thread[t].cpu;
        o[1] = g.prof_thread[t].end_ns;
        o[2] = g.prof_thread[t].px;
        o[3] = g.prof_thread[t].covered_ns;
    }
    g.prof_frames = g.prof_dev_ns = g.prof_fill_ns = g.prof_pre_ns = g.prof_issued_ns = g.prof_done_ns = 0;
    for (auto &t : g.prof_thread) t = Lib::ThreadProf{};
    return n;
}

__attribute__((visibility("default"))) int s3r_set_delivery(int mode, int fill_threads) {
    if (mode < -1 || mode > kFill || fill_threads == 0 || fill_threads > 64) return -1;
    g.fill_pool.stop();
    g.delivery = mode;
    g.fill_threads = fill_threads < 0 ? -1 : fill_threads;
    return 0;
}

__attribute__((visibility("default"))) int s3r_delivery(void) { return delivery_mode(); }

__attribute__((visibility("default"))) void s3r_timing(int enable) {
    g.timing = enable != 0;
    for (Dev *d : g.devs) d->tcount = 0;
}

__attribute__((visibility("default"))) void s3r_timing_stages(double out[4]) {
    double frag = 0, frame = 0, geo = 0;
    size_t n = 0;
    if (!g.devs.empty()) {
        Dev &d = *g.devs[0];
        HIPCHECK(hipSetDevice(d.device));
        for (size_t i = 0; i < d.tcount; i++) {
            float a = 0, b = 0, c = 0;
            sync_event(d.tslots[i].frag1, WaitSite{"s3r_timing_stages", "a timed frame", d.device, d.frame_no});
            HIPCHECK(hipEventElapsedTime(&a, d.tslots[i].frag0, d.tslots[i].frag1));
            HIPCHECK(hipEventElapsedTime(&b, d.tslots[i].frame0, d.tslots[i].frag1));
            HIPCHECK(hipEventElapsedTime(&c, d.tslots[i].frame0, d.tslots[i].geo1));
            frag += a;
            frame += b;
            geo += c;
        }
        n = d.tcount;
        for (Dev *e : g.devs) e->tcount = 0;
    }
    out[0] = frag;
    out[1] = frame;
    out[2] = (double)n;
    out[3] = geo;
}

__attribute__((visibility("default"))) void s3r_timing_collect(double out[3]) {
    double o[4];
    s3r_timing_stages(o);
    out[0] = o[0]; out[1] = o[1]; out[2] = o[2];
}

__attribute__((visibility("default"))) void s3r_scene_counts(uint64_t out[8]) {
    if (!g.devs.empty()) refresh_pairs(*g.devs[0]);
    const Dev *d = g.devs.empty() ? nullptr : g.devs[0];
    out[0] = g.nv; out[1] = g.nindices; out[2] = g.na; out[3] = g.ntex; out[4] = 2ull * g.ntri;
    out[5] = d ? d->last_pairs : 0;          // tile path: (slot, tile) pairs binned last frame
    out[6] = d ? (uint64_t)d->last_path : 0; // fragment stage of the last frame: 1 rows, 2 tiles
    out[7] = g.stale_pins;                   // stale host registrations replaced by updateAndRender
}

__attribute__((visibility("default"))) void s3r_tile_stats(uint64_t out[4]) {
    if (!g.devs.empty()) refresh_pairs(*g.devs[0]);
    const Dev *d = g.devs.empty() ? nullptr : g.devs[0];
    out[0] = d ? d->tile_readbacks : 0;      // frames whose list size was read back before the fill
    out[1] = d ? d->tile_overflows : 0;      // synchronous frames rendered again into a larger list
    out[2] = d ? d->last_pairs : 0;
    out[3] = d ? d->last_live : 0;           // live slots (meeting this part's rows), last read-back frame
}

__attribute__((visibility("default"))) float s3r_ooz_bound(const float ws[3], const float dx[3], const float dy[3],
                                                           const float rvz[3], uint32_t xmin, uint32_t xmax,
                                                           uint32_t ymin, uint32_t ymax) {
    return ooz_bound_host(ws, dx, dy, rvz, xmin, xmax, ymin, ymax);
}

__attribute__((visibility("default"))) void s3r_cluster_stats(uint64_t out[4]) {
    const Dev *d = g.devs.empty() ? nullptr : g.devs[0];
    out[0] = g.ncl;                          // clusters built at load (0: none)
    out[1] = g.clusters && g.ncl ? 1 : 0;    // the tile path culls them (S3R_CLUSTERS)
    out[2] = d ? d->last_kept : 0;           // triangles of the clusters kept, last read-back frame
    out[3] = d && d->cl_perm ? 1 : 0;        // positions are a permutation (not the file order)
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

// Timing build only (-DS3R_WGTIME): per k_geometry workgroup (slot * 64 + row block) of the launches since the
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
