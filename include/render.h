/*
 * render.h -- C ABI of the MI355X rasterizer (librender.so, also installed as render.dylib).
 *
 * Drop-in for the reference's dylib boundary:
 *   struct layouts      /root/reference/render-cpp/render.hpp:7-21 (PixelData 24 B, Input 24 B)
 *   updateAndRender     /root/reference/render-cpp/render.cpp:264-265, bound by the Swift main loop
 *                       with dlopen + dlsym("updateAndRender") (main.swift:96-98) and called once per
 *                       60 Hz tick (main.swift:121).
 * Everything else (s3r_*) is an extension the reference does not have; a caller that only uses
 * updateAndRender sees the reference's behaviour: lazy init from data.bin found next to the library
 * (render.cpp:160-176, exit(666) if missing), the same camera and resize semantics, and the full
 * frame written into pixel_data->buffer before the call returns.
 */
#ifndef S3R_RENDER_H
#define S3R_RENDER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* render.hpp:7-13 */
typedef struct {
    uint32_t *buffer;       /* caller-owned host buffer, 0x00RRGGBB, row-major, stride = width */
    uint32_t width;
    uint32_t height;
    uint32_t bytesPerPixel; /* 4 */
    uint32_t bufferSize;    /* bytes; 4 * width * height (main.swift:163) */
} PixelData;

/* simd_float2: 8 bytes, 8-byte aligned */
typedef struct __attribute__((aligned(8))) { float x, y; } s3r_float2;

/* render.hpp:15-21 */
typedef struct {
    float up;
    float down;
    float left;
    float right;
    s3r_float2 mouse;
} Input;

/* Replaces render.cpp:264-384.  Renders one frame on the GPU into pixel_data->buffer. */
void updateAndRender(const PixelData *pixel_data, const Input *input);

/* ---------------- extensions (not in the reference) ---------------- */

/* Use `data_path` (NULL: the reference's dladdr search) on HIP device `device` (-1: the calling
 * thread's current device) and drop all state so the next call re-initialises like a first call.
 * Environment overrides: S3R_DATA_PATH, S3R_DEVICE.  Returns 0. */
int s3r_configure(const char *data_path, int device);

/* Several GPUs behind updateAndRender (the reference's one call per frame, main.swift:121 ->
 * render.cpp:264-265, from one thread).  With n_devices > 1, every updateAndRender splits the
 * frame's rows into interleaved bands of band_rows rows (0: S3R_BAND, else by fragment path,
 * s3r_frame_band) -- frame row y belongs to
 * device ((y / band_rows) % n_devices) -- and each device renders its bands and copies them
 * straight into their rows of pixel_data->buffer over its own PCIe link, device 0 on the calling
 * thread and the others on one library worker thread each; the call returns when every part has
 * landed.  Pixels are identical to the one-device frame.  n_devices = 0 restores one device
 * (s3r_configure's).  The same ids may repeat (parts on one GPU: tests).  For a caller that only
 * binds updateAndRender (the Swift app), S3R_DEVICES="0,1,2,..." selects the devices instead.  Drops
 * all state like s3r_configure.  Returns 0, or -1 on bad arguments (negative id, n_devices > 64). */
int s3r_configure_devices(const int *device_ids, int n_devices, uint32_t band_rows);
/* Rows per band updateAndRender uses for a frame of `height` rows over n_parts devices (after
 * s3r_configure / the first frame, which fix the fragment path): the configured band_rows, else 16 on
 * the row path and ceil(height / (2 n_parts)) on the tile path (two bands per device). */
uint32_t s3r_frame_band(uint32_t height, uint32_t n_parts);

/* The devices updateAndRender uses (after init: the ones in use); writes up to max_ids ids and
 * returns the count. */
int s3r_devices(int *out_ids, int max_ids);

/* Release every GPU resource and registered host buffer; the next call re-initialises. */
void s3r_shutdown(void);

/* Fragment-stage strategy (extension; both are bit-identical to render.cpp):
 *   1 = row path: per-(slot, row) exact start table + per-workgroup triangle lists, lanes as
 *       (triangle, component) then as pixels -- for the packaged-size scenes;
 *   2 = tile path: order-independent 16x64-pixel tiles, per-pixel (1/z, slot) max in LDS, then
 *       deferred shading -- for many triangles (the icosahedron stress scene);
 *   0 = automatic (default): tile path above 8192 triangle slots (2 x triangles).
 * Returns 0, or -1 for an unknown mode.  s3r_raster_path() reports the path the next frame takes. */
int s3r_set_raster_path(int mode);
int s3r_raster_path(void);

/* One frame for one part of an interleaved row-band split (multi-GPU).  Same camera / init /
 * resize semantics as updateAndRender.  Frame row y belongs to part ((y / band_rows) % n_parts);
 * this part's rows are written compactly, in increasing y, to the DEVICE buffer dev_out
 * (rows_local x width u32), asynchronously on `stream` (a hipStream_t; NULL = the default (null)
 * stream).  The geometry stage runs on internal streams and is ordered before this frame's
 * fragment stage by an event, so later frames' geometry overlaps earlier frames' fragment kernels.
 * Frames are ordered: a frame issued on another stream than the previous frame first waits for the
 * previous frame's fragment stage.  The call returns without waiting for the GPU unless the host is
 * 4 frames ahead (it then waits for the oldest frame's buffers).  n_parts = 1 renders the whole
 * frame.  Returns rows_local, or -1 on bad arguments. */
int64_t s3r_render_bands(const Input *input, uint32_t width, uint32_t height, uint32_t band_rows,
                         uint32_t n_parts, uint32_t part, uint32_t *dev_out, void *stream);

/* Deliver one part's rows -- compact in DEVICE memory as s3r_render_bands wrote them -- into their
 * frame rows of a caller-owned HOST frame (width x height u32, row-major), asynchronously on `stream`:
 * one rectangular copy over this GPU's own PCIe link (the part's bands are band_rows x width blocks
 * spaced n_parts bands apart) plus one for a trailing partial band.  The host frame is page-locked
 * on first use (cached per pointer and size, dropped on resize and shutdown, or by
 * s3r_unregister_host -- call it before unmapping or freeing the frame).  N GPUs -- one process
 * each, the frame in shared memory -- fill one host frame over N links in parallel.  Returns the rows
 * copied, or -1 on bad arguments. */
int64_t s3r_bands_to_host(const uint32_t *dev_rows, uint32_t width, uint32_t height, uint32_t band_rows,
                          uint32_t n_parts, uint32_t part, uint32_t *host_frame, void *stream);

/* One process per GPU, frames kept in HBM: after one RCCL gather has put the N parts'
 * compact band buffers on GPU 0 one after another (part p's rows from row p * part_stride_rows of
 * `gathered`, device memory), write the W x H frame in row order into `frame` (device memory) on
 * `stream`, asynchronously -- one kernel.  Returns 0, or -1 on bad arguments (a part with more rows
 * than part_stride_rows).  Extension: the multi-GPU reassembly; render.cpp renders the whole frame
 * (render.cpp:264-265). */
int s3r_deinterleave_bands(const uint32_t *gathered, uint32_t part_stride_rows, uint32_t width, uint32_t height,
                           uint32_t band_rows, uint32_t n_parts, uint32_t *frame, void *stream);

/* Drop the library's page-lock of a caller host buffer starting at ptr (waits for the device first);
 * a no-op for a pointer the library never registered.  For host frames about to be unmapped or freed
 * (updateAndRender buffers need not: a stale registration is detected and replaced there). */
void s3r_unregister_host(void *ptr);

/* Host buffers.  updateAndRender page-locks the caller's buffer (hipHostRegister, cached) so the
 * frame reaches it at the pinned rate.  A buffer sharing a page with an existing registration -- the
 * second half of the reference's double buffer (one 2 * bufferSize allocation, main.swift:164)
 * shares the seam page with the first -- is merged with it into one registration covering both.
 * s3r_host_pinned: 1 if [ptr, ptr + bytes) lies inside a successful registration.  s3r_host_stats:
 * {frames delivered into a pinned buffer, frames copied into a pageable one, successful
 * registrations, registrations merged into a larger one, registrations held, stale registrations
 * replaced, frames delivered by copy, by direct writes, by host fill, host fill threads, bytes the
 * devices sent over their PCIe links for the last frame, eighths of the sky bins the GPUs write
 * themselves under host fill}. */
int s3r_host_pinned(const void *ptr, uint64_t bytes);
void s3r_host_stats(uint64_t out[12]);

/* How updateAndRender delivers the frame into a page-locked caller buffer (pixels identical in
 * every mode):
 *   1 copy    render into device memory, then a DMA copy over the PCIe link;
 *   2 direct  the fragment kernel writes the pixels straight into the caller's buffer;
 *   3 fill    host fill: the GPU writes the bins and row chunks some triangle covers, library threads
 *             write the background of the rest (render.cpp:282's fill) meanwhile, so the link
 *             carries mostly covered pixels; adaptive: a share of the background bins goes back to
 *             the GPU(s) whenever the threads finish after the devices (S3R_FILL_GPU=0..8 fixes the
 *             share in eighths);
 *   0 auto    (default) host fill; -1: S3R_DELIVERY (copy|direct|fill|auto) or auto.
 * Tile-path frames take copy or direct (auto: direct; host fill is a row-path delivery); buffers
 * that cannot be page-locked are always copied.  fill_threads -1:
 * S3R_FILL_THREADS, or 4 (one device) / 8 (several).  Returns 0, or -1 on a bad mode or thread
 * count (0 or > 64).  s3r_delivery() returns the mode in effect (0-3). */
int s3r_set_delivery(int mode, int fill_threads);

/* Host fill profile since the last call (then cleared), sums over its frames in ns: out[0] frames,
 * out[1] updateAndRender's entry to the frame's start (t0), then after t0: out[2] device 0's
 * launches issued, out[3] the devices' finish (stream drained), out[4] the fill threads' finish,
 * out[5] fill threads joined; out[6] 1 if the fill threads are placed one per CPU domain, out[7]
 * the NUMA node of the buffer they were placed for (int64, -1 unknown); for fill thread t = 1..n at
 * out[8 + 4(t - 1)]: the CPU it last ran on,
 * its summed finish time, the background pixels it wrote, its summed time in covered bins (their
 * background chunks).  Returns n
 * (<= max_threads); out holds 8 + 4 * max_threads words. */
uint32_t s3r_fill_profile(uint64_t *out, uint32_t max_threads);
int s3r_delivery(void);

/* Rows of a height-row frame owned by `part`. */
uint32_t s3r_band_rows_local(uint32_t height, uint32_t band_rows, uint32_t n_parts, uint32_t part);

/* Device-side timing: with enable != 0 every frame records HIP events on its stream around the
 * fragment kernel and around the whole frame.  s3r_timing_collect synchronises, writes
 * out[0] = summed fragment-kernel ms, out[1] = summed frame ms, out[2] = frames, and resets. */
void s3r_timing(int enable);
void s3r_timing_collect(double out[3]);
/* The same plus out[3] = summed ms of the frames' geometry / setup stage (from the frame's first
 * launch to the end of k_geometry, or of the tile path's setup and binning). */
void s3r_timing_stages(double out[4]);

/* Scene counts after init: out = {vertices, indices, attributes, texels, triangle slots,
 * (slot, tile) pairs binned in the last frame (tile path), the last frame's path (1 rows, 2 tiles),
 * host-buffer registrations updateAndRender found stale and replaced}. */
void s3r_scene_counts(uint64_t out[8]);

/* Tile path (device 0): out[0] frames whose tile-list size was read back before the fill (one host
 * sync: asynchronous frames and each buffer set's first), out[1] synchronous updateAndRender frames
 * whose list, sized by earlier frames, overflowed and that were rendered again, out[2] the last
 * frame's (tile, triangle) pairs, out[3] the live slots (meeting this part's rows) of the last
 * frame whose counters were read back. */
void s3r_tile_stats(uint64_t out[4]);

/* Per device behind updateAndRender (s3r_configure_devices), for the frames since the last call:
 * out[4 i] the device id, out[4 i + 1] the frames, out[4 i + 2] the sum of the times (ns after the
 * call's entry) at which its part of each frame was in the caller's buffer, out[4 i + 3] the bytes
 * it sent over its host link in the last frame.  Returns the device count (at most max_devices)
 * and resets the sums.  Extension (a multi-GPU run's explanation; no render.cpp counterpart). */
uint32_t s3r_device_profile(uint64_t *out, uint32_t max_devices);

/* Tile path clusters (built at load for scenes the tile path renders, clusters.cpp): out[0] the
 * cluster count (0: none), out[1] 1 when the tile path culls them (S3R_CLUSTERS: 0 never, 1 frame
 * parts -- the default --, 2 whole frames too, and clusters for every scene), out[2] the
 * triangles of the clusters the last read-back frame kept, out[3] 1 when the setup order is a
 * permutation of the file order.  Extension: replaces nothing in render.cpp (render.cpp:297 visits
 * every triangle). */
void s3r_cluster_stats(uint64_t out[4]);

/* Test hook, no GPU needed: the tile path's upper bound of every 1/z a triangle with this raster
 * setup (render.cpp:319-336: ws, per-pixel steps dx, per-row steps dy, 1/z per corner, bbox) can
 * produce at a pixel it covers, as the kernels compute it (k_tile_raster skips a triangle whose bound
 * is below every current winner of the rows it meets). */
float s3r_ooz_bound(const float ws[3], const float dx[3], const float dy[3], const float rvz[3], uint32_t xmin,
                    uint32_t xmax, uint32_t ymin, uint32_t ymax);

/* Test hook, no GPU needed: the clusters the library builds for a vertex list (nv x float4) and
 * index list (3 ntri vertex indices < nv).  Returns the cluster count C; writes the first
 * min(C + 1, first_cap) position-range starts to first_out, min(C, first_cap) bounding spheres
 * (centre xyz, radius) to sphere_out and, when perm_out is not null, the ntri slots in cluster order. */
uint32_t s3r_build_clusters(const float *vtx, uint32_t nv, const uint32_t *vidx, uint32_t ntri, uint32_t *first_out,
                            float *sphere_out, uint32_t first_cap, uint32_t *perm_out);

/* Copy the current camera matrix (3 rows x 4) and raster factor. */
void s3r_camera(float out_matrix[12], float *out_factor);

/* Diagnostic counters of the S3R_STATS build (all zero in the product build). */
void s3r_stats(uint64_t out[16], int reset);
/* Stats build: the geometry kernel's wall-clock profile (100 MHz ticks): {max workgroup setup time,
 * max workgroup time, first start, last end, 0, 0, 0, 0}. */
void s3r_stats_geometry(uint64_t out[8]);
/* Timing build (-DS3R_WGTIME): the last fragment launch's per-workgroup phase timestamps (100 MHz wall clock):
 * out[4 * wg + k], k = 0 start, 1 list loaded, 2 walk state loaded, 3 end; returns workgroups copied. */
uint32_t s3r_stats_wg_times(uint64_t *out, uint32_t max_wg);
/* Timing build: per geometry workgroup (slot + row block * 2T) of the launches since the last call, 100 MHz
 * wall clock: out[4 * wg + k], k = 0 start, 1 slot set up, 2 bins set, 3 end; clears them; returns the count. */
uint32_t s3r_stats_geo_times(uint64_t *out, uint32_t max_wg);

/* Self-test hooks (tests only): out[i] = the float32 value after n[i] sequential steps
 * s = fl(s + d) (the render.cpp:374/:378 walk) computed by the library's O(binades) walker;
 * lin[i]/del[i] = whether n[i] consecutive walk values are s + k*del exactly. */
void s3r_selftest_walk_host(const float *s, const float *d, const uint32_t *n, float *out, uint32_t *lin,
                            float *del, uint64_t count);
int s3r_selftest_walk_device(const float *s, const float *d, const uint32_t *n, float *out, uint32_t *lin,
                             float *del, uint32_t count);
/* Self-test (tests only): the shading stage's range-checked exact division / sqrt sequences against
 * the IEEE operators on the device.  mode 0: every sqrt input in [2^-96, 2^127); 1: every 1/s for s in
 * [2^-48, 2^64); 2: `count` hashed in-range quotients; 3: `count` hashed vector normalisations.
 * out = {mismatches, first mismatching index or ~0}; returns 0 when the test ran. */
int s3r_selftest_fastmath_device(uint32_t mode, uint64_t count, uint64_t out[2]);
/* Test hook: drain the device and continue the frame count at frame_no (clamped below the point
 * where the library restarts its uint32 frame tags), so tests reach the restart in a few frames.
 * No effect before the first frame. */
void s3r_debug_set_frame_count(uint32_t frame_no);

#ifdef __cplusplus
}
#endif

#endif
