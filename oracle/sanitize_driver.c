/*
 * sanitize_driver.c -- TEST INFRASTRUCTURE: the CPU oracle (render_oracle.c, compiled into this one
 * translation unit) as a standalone program, for the AddressSanitizer / UndefinedBehaviorSanitizer
 * build (`make -C oracle sanitize`).  It replays a script of frames and writes the
 * last frame's pixels, so tests/test_sanitizers.py can check the sanitized oracle renders the same
 * bits as the regular one while ASan/UBSan watch the reference's UB points: the float -> uint8 and
 * float -> uint32 conversions (render.cpp:8, :128-129), the clip-appended scratch arrays
 * (render.cpp:182-196, :239-257), the depth-buffer realloc on resize (:275-280).
 *
 *   sanitize_driver DATA.bin OUT.raw SCRIPT
 * SCRIPT: one frame per line, "W H up down left right mouse_x mouse_y".  OUT.raw: the last frame,
 * W*H little-endian u32.
 */
#include "render_oracle.c"

int main(int argc, char **argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s DATA.bin OUT.raw SCRIPT\n", argv[0]);
        return 2;
    }
    FILE *sf = fopen(argv[3], "r");
    if (!sf) { fprintf(stderr, "cannot open %s\n", argv[3]); return 2; }
    oracle_set_data_path(argv[1]);
    uint32_t *buf = NULL;
    unsigned w = 0, h = 0;
    Input in;
    int frames = 0;
    while (fscanf(sf, "%u %u %f %f %f %f %f %f", &w, &h, &in.up, &in.down, &in.left, &in.right, &in.mouse.x,
                  &in.mouse.y) == 8) {
        /* exactly W*H words (no slack), so an out-of-frame write is an ASan heap overflow */
        buf = realloc(buf, (size_t)w * h * sizeof(uint32_t) + (w * h ? 0 : 4));
        PixelData pd = {buf, w, h, 4, 4 * w * h};
        oracle_updateAndRender(&pd, &in);
        frames++;
    }
    fclose(sf);
    FILE *of = fopen(argv[2], "wb");
    if (!of || !frames) { fprintf(stderr, "no frames / cannot write %s\n", argv[2]); return 2; }
    fwrite(buf, sizeof(uint32_t), (size_t)w * h, of);
    fclose(of);
    free(buf);
    free_scene();
    return 0;
}
