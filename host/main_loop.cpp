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
// Input comes from a script instead of a keyboard/mouse (input.swift:75-93): each line of the
// script file is "up down left right mouse_x mouse_y [frames]" (the tuple is repeated `frames`
// times, default 1); no script = hold still.  With --pace the loop sleeps to a 60 Hz cadence like the
// Timer (main.swift:109); without it frames run back to back.
//
// Build: g++ -O2 -std=c++17 host/main_loop.cpp -ldl -o host/main_loop   (no HIP needed: dlopen)
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <string>
#include <thread>
#include <vector>

#include "../include/render.h"

using Clock = std::chrono::steady_clock;
typedef void (*UpdateAndRender)(const PixelData *, const Input *);

struct Step { Input in; int frames; };

static std::vector<Step> load_script(const char *path) {
    std::vector<Step> s;
    if (!path) return s;
    FILE *f = fopen(path, "r");
    if (!f) { fprintf(stderr, "cannot open script %s\n", path); exit(2); }
    char line[512];
    while (fgets(line, sizeof line, f)) {
        if (line[0] == '#' || line[0] == '\n') continue;
        Step st{};
        st.frames = 1;
        const int n = sscanf(line, "%f %f %f %f %f %f %d", &st.in.up, &st.in.down, &st.in.left, &st.in.right,
                             &st.in.mouse.x, &st.in.mouse.y, &st.frames);
        if (n >= 6) s.push_back(st);
    }
    fclose(f);
    return s;
}

static void write_ppm(const char *path, const uint32_t *px, uint32_t w, uint32_t h) {
    FILE *f = fopen(path, "wb");
    if (!f) return;
    fprintf(f, "P6\n%u %u\n255\n", w, h);
    std::vector<uint8_t> row(3 * w);
    for (uint32_t y = 0; y < h; y++) {
        for (uint32_t x = 0; x < w; x++) {
            const uint32_t p = px[(size_t)y * w + x];
            row[3 * x] = (uint8_t)(p >> 16); row[3 * x + 1] = (uint8_t)(p >> 8); row[3 * x + 2] = (uint8_t)p;
        }
        fwrite(row.data(), 1, row.size(), f);
    }
    fclose(f);
}

int main(int argc, char **argv) {
    const char *lib = "swift3drenderer_amd/render.dylib", *script = nullptr, *dump = nullptr;
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
        else { fprintf(stderr, "usage: %s [--lib L] [--size W H] [--frames N] [--script F] [--pace] [--dump PREFIX EVERY]\n", argv[0]); return 2; }
    }
    void *handle = dlopen(lib, RTLD_NOW);                                  // main.swift:96
    if (!handle) { fprintf(stderr, "dlopen: %s\n", dlerror()); return 1; }
    UpdateAndRender update_and_render = (UpdateAndRender)dlsym(handle, "updateAndRender");   // :97
    if (!update_and_render) { fprintf(stderr, "dlsym: %s\n", dlerror()); return 1; }

    PixelData pd{};
    pd.bytesPerPixel = 4;                                                   // main.swift:44
    pd.width = w; pd.height = h;
    pd.bufferSize = pd.bytesPerPixel * w * h;                                 // :163
    uint32_t *memory = (uint32_t *)malloc(2 * (size_t)pd.bufferSize);        // :164
    const std::vector<Step> steps = load_script(script);
    size_t si = 0;
    int left_in_step = steps.empty() ? 0 : steps[0].frames;
    Input input{};

    const double frame_target = 1.0 / 60.0;                                 // main.swift:39
    double total = 0, total_pct = 0, all = 0;
    int loops = 0, sessions = 0, cur = 0;
    auto last = Clock::now();
    for (int f = 0; f < frames; f++) {
        const auto tick = Clock::now();
        if (!steps.empty()) {                                               // input.swift:75-93
            if (si < steps.size()) {
                input = steps[si].in;
                if (--left_in_step <= 0 && ++si < steps.size()) left_in_step = steps[si].frames;
            } else {
                input.up = input.down = input.left = input.right = 0;       // hold the last mouse
            }
        }
        pd.buffer = memory + (size_t)cur * w * h;                           // main.swift:117-118
        cur = (cur + 1) % 2;
        const auto t0 = Clock::now();                                       // :120
        update_and_render(&pd, &input);                                     // :121
        const double dt = std::chrono::duration<double>(Clock::now() - t0).count();
        total += dt;
        all += dt;
        loops++;
        if (dump && dump_every > 0 && f % dump_every == 0) {
            char path[1024];
            snprintf(path, sizeof path, "%s_%05d.ppm", dump, f);
            write_ppm(path, pd.buffer, w, h);
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
    printf("frames %d  mean updateAndRender %.3f ms  (%.1f fps, %ux%u)\n", frames, 1e3 * all / frames,
           frames / all, w, h);
    free(memory);
    return 0;
}
