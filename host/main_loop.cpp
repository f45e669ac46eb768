// main_loop.cpp -- C++ counterpart of the reference's Swift main loop (main.swift:30-165), for
// driving the rasterizer without AppKit/Metal: dlopen the library, dlsym("updateAndRender"), and
// call it once per frame with a double-buffered caller-owned pixel buffer, timing every call and
// printing the reference's own metric -- the share of the 1/60 s frame budget -- once per second.
//
//   main.swift:96-98    dlopen(dylibPath, RTLD_NOW) + dlsym("updateAndRender")
//   main.swift:112-122  per tick: update input, pick buffer half, time the call
//   main.swift:143-153  "# loops", "%.2f%%", "average: %.2f%%" once per timeInterval
//   main.swift:156-165  resize: bufferSize = 4*W*H, buffer realloc'ed to 2*bufferSize
//
// Input comes from a script instead of a keyboard, mouse or touch sticks.  The Input struct persists
// across frames like main.swift's `input` var; each script line is one of
//   up down left right mouse_x mouse_y [frames]   raw Input tuple, held `frames` frames (default 1)
//   mac KEYS dx dy [frames]                       macOS (input.swift:78-85): KEYS = the held keys
//        among w a s d, '+' = shift held (speed 2), '-' = none; each frame the captured mouse moves
//        by (dx, dy) (GCMouse deltas accumulated, :41-45) and input.mouse = that position
//   ios lx ly rx ry [frames]                      iOS virtual sticks (input.swift:87-91):
//        left = -lx, right = lx, up = ly, down = -ly (negative values pass through), and each
//        frame input.mouse += 6 * (rx, ry)
//   resize W H                                    the window resized (main.swift:156-165) before
//        the next frame: bufferSize = 4*W*H, buffer = realloc(buffer, 2*bufferSize)
// After the script the movement keys are released and the mouse held.  No script = hold still.
// With --pace the loop sleeps to a 60 Hz cadence like the Timer (main.swift:109); without it frames
// run back to back.  --log writes each frame's (W, H, Input) as it was passed (tests).
//
// Build: g++ -O2 -std=c++17 host/main_loop.cpp -ldl -o host/main_loop   (no HIP needed: dlopen)
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../include/render.h"

using Clock = std::chrono::steady_clock;
typedef void (*UpdateAndRender)(const PixelData *, const Input *);
typedef void (*HostStats)(uint64_t *);
typedef int (*HostPinned)(const void *, uint64_t);

enum Kind { kRaw, kMac, kIos, kResize };
struct Step {
    Kind kind = kRaw;
    Input in{};                  // kRaw
    bool w = false, a = false, s = false, d = false, shift = false;   // kMac
    float v[4] = {0, 0, 0, 0};   // kMac: dx dy; kIos: lx ly rx ry
    uint32_t width = 0, height = 0;   // kResize
    int frames = 1;
};

static std::vector<Step> load_script(const char *path) {
    std::vector<Step> s;
    if (!path) return s;
    FILE *f = fopen(path, "r");
    if (!f) { fprintf(stderr, "cannot open script %s\n", path); exit(2); }
    char line[512];
    int lineno = 0;
    while (fgets(line, sizeof line, f)) {
        lineno++;
        if (line[0] == '#' || line[0] == '\n') continue;
        Step st;
        char keys[64];
        if (!strncmp(line, "mac", 3)) {
            st.kind = kMac;
            if (sscanf(line + 3, "%63s %f %f %d", keys, &st.v[0], &st.v[1], &st.frames) < 3) goto bad;
            for (const char *k = keys; *k; k++) {
                switch (*k) {
                    case 'w': st.w = true; break;
                    case 'a': st.a = true; break;
                    case 's': st.s = true; break;
                    case 'd': st.d = true; break;
                    case '+': st.shift = true; break;
                    case '-': break;
                    default: goto bad;
                }
            }
        } else if (!strncmp(line, "ios", 3)) {
            st.kind = kIos;
            if (sscanf(line + 3, "%f %f %f %f %d", &st.v[0], &st.v[1], &st.v[2], &st.v[3], &st.frames) < 4) goto bad;
        } else if (!strncmp(line, "resize", 6)) {
            st.kind = kResize;
            st.frames = 0;
            if (sscanf(line + 6, "%u %u", &st.width, &st.height) != 2) goto bad;
        } else {
            if (sscanf(line, "%f %f %f %f %f %f %d", &st.in.up, &st.in.down, &st.in.left, &st.in.right,
                       &st.in.mouse.x, &st.in.mouse.y, &st.frames) < 6) goto bad;
        }
        s.push_back(st);
        continue;
    bad:
        fprintf(stderr, "%s:%d: bad script line\n", path, lineno);
        exit(2);
    }
    fclose(f);
    return s;
}

// input.swift:75-93 for one frame of step st (mouse: the captured mouse position on macOS).
static void apply_step(const Step &st, Input &in, float mouse[2]) {
    switch (st.kind) {
        case kRaw:
            in = st.in;
            break;
        case kMac: {
            const float speed = st.shift ? 2.f : 1.f;                 // input.swift:78
            in.left = st.a ? speed : 0;                                 // :79-82
            in.right = st.d ? speed : 0;
            in.up = st.w ? speed : 0;
            in.down = st.s ? speed : 0;
            mouse[0] += st.v[0];                                        // :43-44
            mouse[1] += st.v[1];
            in.mouse.x = mouse[0];                                      // :84
            in.mouse.y = mouse[1];
            break;
        }
        case kIos:
            in.left = -st.v[0];                                         // :87-90
            in.right = st.v[0];
            in.up = st.v[1];
            in.down = -st.v[1];
            in.mouse.x += 6 * st.v[2];                                  // :91
            in.mouse.y += 6 * st.v[3];
            break;
        case kResize:
            break;
    }
}

static void write_ppm(const char *path, const uint32_t *px, uint32_t w, uint32_t h) {
    FILE *f = fopen(path, "wb");
    if (!f) return;
    fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> row(3 * (size_t)w);
    for (uint32_t y = 0; y < h; y++) {
        for (uint32_t x = 0; x < w; x++) {
            const uint32_t p = px[(size_t)y * w + x];
            row[3 * x] = (uint8_t)(p >> 16); row[3 * x + 1] = (uint8_t)(p >> 8); row[3 * x + 2] = (uint8_t)p;
        }
        fwrite(row.data(), 1, row.size(), f);
    }
    fclose(f);
}

// main.swift:156-165
static uint32_t *resize(PixelData &pd, uint32_t *memory, uint32_t w, uint32_t h) {
    pd.width = w;
    pd.height = h;
    pd.bufferSize = pd.bytesPerPixel * w * h;
    memory = (uint32_t *)realloc(memory, 2 * (size_t)pd.bufferSize);
    if (!memory && pd.bufferSize) { fprintf(stderr, "realloc failed\n"); exit(1); }
    return memory;
}

int main(int argc, char **argv) {
    const char *lib = "swift3drenderer_amd/render.dylib", *script = nullptr, *dump = nullptr, *log = nullptr;
    uint32_t w = 960, h = 540;                  // main.swift:66 window size
    int frames = 600, dump_every = 0;
    bool pace = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&]() { return i + 1 < argc ? argv[++i] : (exit(2), (char *)nullptr); };
        if (a == "--lib") lib = next();
        else if (a == "--size") { w = (uint32_t)atoi(next()); h = (uint32_t)atoi(next()); }
        else if (a == "--frames") frames = atoi(next());
        else if (a == "--script") script = next();
        else if (a == "--pace") pace = true;
        else if (a == "--dump") { dump = next(); dump_every = atoi(next()); }
        else if (a == "--log") log = next();
        else { fprintf(stderr, "usage: %s [--lib L] [--size W H] [--frames N] [--script F] [--pace] [--dump PREFIX EVERY] [--log F]\n", argv[0]); return 2; }
    }
    void *handle = dlopen(lib, RTLD_NOW);                                  // main.swift:96
    if (!handle) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 1; }
    UpdateAndRender update_and_render = (UpdateAndRender)dlsym(handle, "updateAndRender");   // :97
    if (!update_and_render) { fprintf(stderr, "dlsym: %s\n", dlerror()); return 1; }
    // extensions of this library (absent from the reference's dylib): pinning report only
    HostStats host_stats = (HostStats)dlsym(handle, "s3r_host_stats");
    HostPinned host_pinned = (HostPinned)dlsym(handle, "s3r_host_pinned");
    FILE *logf = log ? fopen(log, "w") : nullptr;

    PixelData pd{};
    pd.bytesPerPixel = 4;                                                   // main.swift:44
    uint32_t *memory = resize(pd, nullptr, w, h);                           // :12 (resize() at startup)
    const std::vector<Step> steps = load_script(script);
    size_t si = 0;
    int left_in_step = steps.empty() ? 0 : steps[0].frames;
    Input input{};
    float mouse[2] = {0, 0};
    std::vector<double> times;
    times.reserve(frames > 0 ? (size_t)frames : 0);

    const double frame_target = 1.0 / 60.0;                                 // main.swift:39
    double total = 0, total_pct = 0, all = 0;
    int loops = 0, sessions = 0, cur = 0;
    auto last = Clock::now();
    for (int f = 0; f < frames; f++) {
        const auto tick = Clock::now();
        // script steps: resizes take effect before the frame, input steps last `frames` frames
        while (si < steps.size() && (steps[si].kind == kResize || left_in_step <= 0)) {
            if (steps[si].kind == kResize) memory = resize(pd, memory, steps[si].width, steps[si].height);
            if (++si < steps.size()) left_in_step = steps[si].frames;
        }
        if (si < steps.size()) {
            apply_step(steps[si], input, mouse);                            // input.swift:75-93
            left_in_step--;
        } else if (!steps.empty()) {
            input.up = input.down = input.left = input.right = 0;           // hold the last mouse
        }
        pd.buffer = memory + (size_t)cur * pd.width * pd.height;            // main.swift:117-118
        cur = (cur + 1) % 2;
        if (logf)
            fprintf(logf, "%d %u %u %.9g %.9g %.9g %.9g %.9g %.9g\n", f, pd.width, pd.height, input.up, input.down,
                    input.left, input.right, input.mouse.x, input.mouse.y);
        const auto t0 = Clock::now();                                       // :120
        update_and_render(&pd, &input);                                     // :121
        const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
        times.push_back(dt);
        total += dt;
        all += dt;
        loops++;
        if (dump && dump_every > 0 && f % dump_every == 0) {
            char path[1024];
            snprintf(path, sizeof path, "%s_%05d.ppm", dump, f);
            write_ppm(path, pd.buffer, pd.width, pd.height);
        }
        if (std::chrono::duration<double>(Clock::now() - last).count() >= 1.0) {   // :143-153
            last = Clock::now();
            const double pct = 100.0 * total / (frame_target * loops);
            sessions++;
            total_pct += pct;
            printf("# loops: %d\n%.2f%%\naverage: %.2f%%\n", loops, pct, total_pct / sessions);
            total = 0;
            loops = 0;
        }
        if (pace) std::this_thread::sleep_until(tick + std::chrono::duration<double>(frame_target));
    }
    if (logf) fclose(logf);
    double median = 0;
    if (!times.empty()) {
        std::vector<double> t = times;
        std::nth_element(t.begin(), t.begin() + t.size() / 2, t.end());
        median = t[t.size() / 2];
    }
    printf("frames %d  mean updateAndRender %.3f ms  median %.3f ms  (%.1f fps, %ux%u)\n", frames,
           frames ? 1e3 * all / frames : 0.0, 1e3 * median, all > 0 ? frames / all : 0.0, pd.width, pd.height);
    if (host_stats) {
        uint64_t s[12];
        host_stats(s);
        printf("host_stats pinned_frames %llu pageable_frames %llu registrations %llu merges %llu held %llu stale %llu "
               "copy_frames %llu direct_frames %llu fill_frames %llu fill_threads %llu link_bytes %llu fill_gpu_eighths %llu\n",
               (unsigned long long)s[0], (unsigned long long)s[1], (unsigned long long)s[2],
               (unsigned long long)s[3], (unsigned long long)s[4], (unsigned long long)s[5],
               (unsigned long long)s[6], (unsigned long long)s[7], (unsigned long long)s[8],
               (unsigned long long)s[9], (unsigned long long)s[10], (unsigned long long)s[11]);
    }
    if (host_pinned && pd.bufferSize)
        printf("halves_pinned %d %d\n", host_pinned(memory, pd.bufferSize),
               host_pinned((const uint8_t *)memory + pd.bufferSize, pd.bufferSize));
    free(memory);
    return 0;
}
