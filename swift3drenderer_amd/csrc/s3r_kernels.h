// s3r_kernels.h -- host-callable launchers for the gfx950 kernels (kernels.hip).
#pragma once
#include "s3r_common.h"

#include <vector>

namespace s3r {

// S3R_CHECK=1 (diagnostics): every launcher below synchronises its stream after each kernel it
// launches and checks for a device fault; a fault is reported with the kernel's name and the
// calling thread's frame context (check_context: device, frame number, stage) and the process
// aborts -- a fault then names the launch that caused it instead of surfacing in a later HIP call.
bool check_launches();
void check_context(int device, uint32_t frame, const char *stage);
void after_launch(const char *kernel, hipStream_t st);

// Bounded waits (render_api.cpp "bounded waits"): a wait past its deadline (S3R_WAIT_MS) prints
// its stage, kernel, device and frame and ends the process with this status.
constexpr int kStallExit = 86;
// hipStreamSynchronize under the library's watchdog (what after_launch uses)
void sync_stream_bounded(hipStream_t st, const char *stage, const char *kernel, int device, uint32_t frame);
// Test hook (S3R_TEST_HOLD_MS): a one-wave kernel that spins `ms` milliseconds of the device clock
// and exits -- a stage that is late but always finishes, for the deadline tests.
void launch_test_hold(uint32_t ms, hipStream_t st);
// The clock-tick budget of the device spins (S3R_SPIN_MS, default 2000 ms; 100 MHz ticks).
uint32_t device_spin_ticks();

// `done` (may be null): recorded on `st` when the launched kernel completes.
// order (may be null: launch order): 2 x fragment_bins() words, [perm | cost] -- launch_geometry's
// extra workgroup (order non-null there) writes perm, the launch's workgroup -> bin map, from the
// costs; the fragment launch reads perm and stores each bin's time into cost, for the next frame
// on the same buffer set (a hint only: any permutation renders the same pixels).
// Renders `rows_local` rows: local row lr is frame row ((lr / band) * nparts + part) * band + lr % band
// (interleaved row bands; nparts = 1, band = H renders the whole frame).  Output is compact,
// out[lr * W + x], or with frame_rows the whole frame's row, out[y * W + x] (out = a W x H frame, e.g.
// the caller's host buffer).  host_fill = 1 + g (0: off): sky bins (no triangle) with bin % 8 >= g
// write nothing -- the host fills them (launch_sky_flags) -- and neither do the row chunks of covered
// bins that end without a winner:
// each bin's workgroup stores chunk_flags[bin] = (fill_tag << 32) | mask at its end, bit
// (row_in_bin * chunks_per_row + chunk) for every such chunk, for the host to fill.
void launch_fragment(const TriSetup *tris, uint32_t nslots, const float *rowtab, const uint32_t *tex, uint32_t ntex,
                     uint32_t *out, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
                     uint32_t rows_local, uint32_t *bincnt, const uint4 *pairs,
                     hipStream_t st, hipEvent_t done, uint32_t *done_flag, uint32_t prev_tag, uint32_t *order,
                     bool frame_rows = false, uint32_t host_fill = 0, unsigned long long *chunk_flags = nullptr,
                     uint32_t fill_tag = 0, bool row_starts = false);

// Fragment workgroups (bins = blocks of 4 local rows x segments) and their triangle lists: per bin a
// pair count -- k_geometry counts up from 0, the bin's fragment workgroup reads it and resets it to 0
// (the fragment launch is the buffer set's last reader, and the set's next geometry is issued only
// once it has completed) -- and kPairMax pair records of kPairWords uint4 (128 B) in arrival order:
// {slot, xmin, xmax, ymin}, {ymax, 0, 0, 0}, {dx[3], 0}, {1/z[3], 0}, then the exact walk state of the
// bin's 4 rows x 3 components at the start-table point of the bin's first pixel (row-major, 12 floats;
// rows outside the triangle's bbox are left unwritten).  A bin met by more than kPairMax triangles
// scans the slots itself.
constexpr uint32_t kPairMax = 64;
constexpr uint32_t kPairWords = 8;
uint64_t fragment_bins(uint32_t W, uint32_t rows_local);

// The frame's geometry in one launch (k_geometry): TriSetup records for the 2T slots, the bins'
// headers and pairs, and rowtab (2T x rows_local x start_entries(W) x float4): exact barycentrics of
// every live slot's bbox rows at x = xmin and at each 384-pixel boundary inside the bbox.
uint32_t start_entries(uint32_t W);
// row_starts: rowtab and the pairs get the row starts (x = xmin) only, not the start-table boundaries;
// the fragment launch reading them must be given row_starts too (its walks then start at xmin).
// Host fill (render_api.cpp): with gsf the launch also publishes the bins' sky flags as soon as every
// workgroup's pair reservations are in (see launch_sky_flags for flags / tag / probe / gpu_eighths);
// geo_cnt: kGeoCounterWords zeroed device words (the launch leaves them 0), one set per launch in flight.
constexpr uint32_t kGeoCounterWords = 256 * 16;
// err: kDiagWords host-coherent words (Dev::diag_host) -- a publisher whose spin passes its clock
// deadline stores {kDiagPublisherTimeout, row block, arrivals seen, arrivals expected} there and
// returns without publishing (the host reports it; render_api.cpp fill_worker).  extra_arrivals: a
// test hook (S3R_TEST_ARRIVALS_EXTRA) added to the arrivals the publishers wait for.
constexpr uint32_t kDiagWords = 4, kDiagPublisherTimeout = 1;
struct GeoSkyFlags {
    uint32_t *flags, *probe, *geo_cnt;
    uint32_t tag, gpu_eighths;
    uint32_t *err;
    uint32_t extra_arrivals;
};
// clip_slots = false: no triangle can cross the near plane this frame (the host's check,
// render_api.cpp near_plane_crossing), so the launch leaves out the clip-appended slots T..2T-1 (their
// records are marked dead) -- half the workgroups, one dispatch round fewer for small scenes.
// Host slot cull (render_api.cpp cull_slots): with `live`, k_geometry starts workgroups only for the
// original slots whose bit is set (frames without clip slots, scenes up to kLiveMaskSlots triangles);
// one extra workgroup marks every other slot dead.
constexpr uint32_t kLiveMaskSlots = 1024;
struct SlotMask {
    uint64_t bits[kLiveMaskSlots / 64];
    uint32_t nlive;                    // set bits
    uint32_t on;                       // 0: every slot launched (bits unused)
};
void launch_geometry(const float4 *vtx, const float4 *nrm, const float4 *pay, const uint8_t *disc,
                     const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri, const Mat34 &m, float factor,
                     uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                     TriSetup *tris, float *rowtab, uint32_t *bincnt, uint4 *pairs, hipStream_t st, hipEvent_t done,
                     uint32_t *order, const GeoSkyFlags *gsf = nullptr, bool row_starts = false,
                     bool clip_slots = true, const SlotMask *live = nullptr);
uint32_t fragment_segments(uint32_t W);

uint32_t fragment_segment_pixels();

// The row path's fragment bins for a frame part of W x rows_local (what fragment_configure picks):
// bin b covers local rows (b / segs) * rows_per_bin ... + rows_per_bin - 1, columns
// (b % segs) * seg_px ... + seg_px - 1 (clipped to the part and the frame).
struct FragLayout { uint32_t seg_px, segs, rows_per_bin, chunk_px; uint64_t bins; };
FragLayout fragment_layout(uint32_t W, uint32_t rows_local);

// Host fill: flags[b] = tag | (kSkyBit if bin b has no pair) for the bins' counts of the geometry
// just launched on st (system-scope stores into host-coherent memory); `done` recorded on completion.
// probe (may be null): device address of the caller's pixel 0, set to kMapProbe before flags[0] is
// published (the host's check that the mapping of its buffer is not stale).  Neither value is a
// pixel (pixels are 0x00RRGGBB).
// gpu_eighths: sky bins with bin % 8 < gpu_eighths stay with the GPU (flag tag | kGpuBit: the fragment
// kernel writes their background); tags stay below kGpuBit.
constexpr uint32_t kSkyBit = 0x80000000u;
constexpr uint32_t kGpuBit = 0x40000000u;
constexpr uint32_t kMapProbe = 0xFEA5A5A5u;
void launch_sky_flags(const uint32_t *bincnt, uint64_t nbins, uint32_t *flags, uint32_t tag, uint32_t *probe,
                      uint32_t gpu_eighths, hipStream_t st, hipEvent_t done);
// Picks the row path's segment width for a frame of W x rows_local; call before the helpers above.
void fragment_configure(uint32_t W, uint32_t rows_local);

// Tile path (order-independent fragment stage for many triangles): tiles of 16 local rows x 64 px,
// each tile's list split into depth buckets (nearest first; kernels.hip depth_bucket).
// recs: 2T x raster_rec_bytes(); counts / offs / cursor: tile_slots() (tile, bucket) entries;
// scan_temp: tile_scan_temp_bytes(tile_slots()) bytes.
// xoff (every tile launch of a frame the same): the tile grid shifted left by xoff < 16 pixels, tile
// column c covering x in [64 c - xoff, 64 c - xoff + 64) -- a frame written into the caller's
// buffer puts each tile row's 64 pixels on the buffer's 64-B line grid (render_api.cpp tile_xoff).
uint32_t tile_count(uint32_t W, uint32_t rows_local, uint32_t xoff = 0);
uint32_t tile_height();                        // rows of a tile (a multiple of the resolve's 4-row blocks)
uint64_t tile_slots(uint32_t W, uint32_t rows_local, uint32_t xoff = 0);
size_t tile_scan_temp_bytes(uint64_t nslots);
size_t raster_rec_bytes();
// Init-time clusters (clusters.cpp) on the device: ncl bounding spheres (world centre, radius),
// first[ncl + 1] position ranges, perm (position -> slot; null: identity), shard[kTileShards + 1]
// (cluster_shard_table: where each shard's positions start) and cmap, a per-frame scratch of ntri
// words (the surviving clusters' positions, per shard).
struct TileClusters {
    const float4 *sphere;
    const uint32_t *first, *perm, *shard;
    uint32_t ncl;
    uint32_t *cmap;
};
// The cull, setup and fill append to kTileShards per-shard lists (kernels.hip "sharded streams");
// cluster c is culled by workgroup c / 256, which serves shard (c / 256) % kTileShards.
constexpr uint32_t kTileShards = 64, kTileShardStride = 64;
// Shard s's first position: the triangles of the clusters of shards < s (kTileShards + 1 entries).
std::vector<uint32_t> cluster_shard_table(const std::vector<uint32_t> &first);
// ctr: kTileCtrWords device words per buffer set (allocate them zeroed; the tile kernels leave the
// shard counters zero again after each frame): [0] live entries, [1] the
// tile lists' total length, [2] positions the cluster cull kept, [3] the fused raster's deferred
// pixels (the first kTileCounterWords are
// the summary the host reads back), then the shards' counters.  live: 2T entries (tile box, rows,
// slot, 0); clipq: T words (the positions whose triangle crosses the near plane).  cl (may be null
// or empty): cull clusters first and set up only their triangles; vrv (nv float4, may be null;
// unused with clusters): run the vertex stage first (k_tile_vertex) and set triangles up from its
// projected vertices.  counts must be zero on entry (allocate them zeroed): the launch leaves them
// zero again.  sum_host (host-coherent, mapped; may be null): {tag, ctr[0], ctr[1], ctr[2]} written
// by the device as soon as the summary is known, the tag last (system scope).
constexpr uint32_t kTileCounterWords = 4;
constexpr uint32_t kTileCtrWords = kTileCounterWords * 16 + 3 * kTileShards * kTileShardStride;
void launch_tile_setup(const float4 *vtx, const uint32_t *vidx, uint32_t ntri, const Mat34 &m, float factor, float sw,
                       float sh, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part, uint32_t rows_local,
                       void *recs, uint4 *live, uint32_t *clipq, uint32_t *ctr, uint32_t *counts, uint32_t *offs,
                       uint32_t *cursor, void *scan_temp, size_t scan_temp_bytes, hipStream_t st,
                       float4 *vrv = nullptr, uint32_t nv = 0, const TileClusters *cl = nullptr,
                       uint32_t *sum_host = nullptr, uint32_t tag = 0, uint32_t *tbin = nullptr, uint32_t bin_cap = 0,
                       uint32_t xoff = 0);
// No raster record is written for the slots the raster can set up again from the scene (kernels.hip
// kNoRecBit); the clip's slots keep theirs.
// tbin / bin_cap (bins mode): every (tile, bucket) slot s gets bin_cap entries at tbin + s x bin_cap
// and counts[s] of them filled by the setup itself -- no scan, no fill pass; the summary's word 4 is
// then the count the fullest slot needed when it exceeded bin_cap (0: none; the frame is rendered
// empty and must be binned again with larger bins), and offs / cursor / live are unused.
// list: cap entries -- a frame whose list (ctr[1] entries) needs more writes only cap of them, and
// k_tile_raster then renders no triangle (the caller renders the frame again with a larger list).
// The fill's scatter cursors reset to the offsets (as launch_tile_setup leaves them): a frame's fill
// again, e.g. into a larger list after an overflow.
void launch_tile_cursor(const uint32_t *counts, const uint32_t *offs, uint32_t W, uint32_t rows_local, uint32_t *cursor,
                        uint32_t *ctr, hipStream_t st, uint32_t xoff = 0);
// The same cl as the setup's (it says where the shards' live entries start).
void launch_tile_fill(const uint4 *live, uint32_t *ctr, const TileClusters *cl, uint32_t ntri, uint32_t W,
                      uint32_t band, uint32_t nparts, uint32_t part, uint32_t *cursor, uint32_t *list, uint64_t cap,
                      hipStream_t st, uint32_t xoff = 0);
// Raster and resolve in one launch (each tile shades its winners from LDS and stores them into out:
// its local rows, or with frame_rows the frame rows of a W x H frame), then the pixels whose winner
// needs a full setup (ctr[3] of them, in `deferred`: W x rows_local entries) in a second, short one.
void launch_tile_raster_resolve(const void *recs, const float4 *vtx, const float4 *nrm, const float4 *pay,
                                const uint8_t *disc, const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri,
                                const Mat34 &m, float factor, float sw, float sh, const uint32_t *tex, uint32_t ntex,
                                uint32_t *out, uint32_t W, uint32_t band, uint32_t nparts, uint32_t part,
                                uint32_t rows_local, const uint32_t *offs, uint32_t *ctr, const uint32_t *list,
                                uint64_t cap, uint4 *deferred, hipStream_t st, bool frame_rows,
                                uint32_t *counts = nullptr, uint32_t bin_cap = 0, uint32_t xoff = 0,
                                uint32_t *sum_host = nullptr);      // bins: the entries' total (launch_tile_resolve_deferred)
// Those pixels, shaded with the winner's full setup (after every resolve launch of the frame).
void launch_tile_resolve_deferred(const void *recs, const float4 *vtx, const float4 *nrm, const float4 *pay,
                                  const uint8_t *disc, const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri,
                                  const Mat34 &m, float factor, float sw, float sh, const uint32_t *tex, uint32_t ntex,
                                  uint32_t *out, const uint4 *deferred, uint32_t *ctr, hipStream_t st,
                                  bool bins = false,                   // bins mode: also total the binned entries
                                  uint32_t *sum_host = nullptr);       // (into ctr[1] and word 2 of sum_host)

// The N parts of an interleaved band split, gathered one after another (part p's compact rows from
// row p * part_stride_rows), written into the W x H frame in frame-row order (one launch).
void launch_deinterleave_bands(const uint32_t *gathered, uint32_t part_stride_rows, uint32_t W, uint32_t H,
                               uint32_t band, uint32_t nparts, uint32_t *frame, hipStream_t st);

float ooz_bound_host(const float ws[3], const float dx[3], const float dy[3], const float rvz[3], uint32_t xmin,
                     uint32_t xmax, uint32_t ymin, uint32_t ymax);
void stats_read(unsigned long long out[24], bool reset);
uint32_t wg_times_read(unsigned long long *out, uint32_t max_wg);
uint32_t geo_times_read(unsigned long long *out, uint32_t max_wg);

int fastmath_test(uint32_t mode, uint64_t count, uint64_t out[2]);
void launch_walk_test(const float *s, const float *d, const uint32_t *n, float *out, uint32_t *lin, float *del,
                      uint32_t count, hipStream_t st);

}  // namespace s3r
