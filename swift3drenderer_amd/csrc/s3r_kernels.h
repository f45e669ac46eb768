// s3r_kernels.h -- host-callable launchers for the gfx950 kernels (kernels.hip).
#pragma once
#include "s3r_common.h"

namespace s3r {

void launch_setup(const float4 *vtx, const float4 *nrm, const float4 *pay, const uint8_t *disc,
                  const uint32_t *vidx, const uint32_t *aidx, uint32_t ntri, const Mat34 &m, float factor,
                  float sw, float sh, TriSetup *tris, hipStream_t st);

// Renders `rows_local` rows: local row lr is frame row ((lr / band) * nparts + part) * band + lr % band
// (interleaved row bands; nparts = 1, band = H renders the whole frame).  Output is compact:
// out[lr * W + x].
void launch_fragment(const TriSetup *tris, uint32_t nslots, const float *rowtab, const uint32_t *tex, uint32_t ntex,
                     uint32_t *out, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts, uint32_t part,
                     uint32_t rows_local, const void *bins, const uint32_t *counts, hipStream_t st);

// Per-workgroup triangle lists (bins = row blocks x segments): fragment_bins() bins of
// bin_entry_bytes() each plus one u32 count per bin.
uint64_t fragment_bins(uint32_t W, uint32_t rows_local);
size_t bin_entry_bytes();
void launch_bin(const TriSetup *tris, uint32_t nslots, uint32_t W, uint32_t H, uint32_t band, uint32_t nparts,
                uint32_t part, uint32_t rows_local, void *bins, uint32_t *counts, hipStream_t st);

// rowtab (nslots x H x (segments + 1) x float4): exact barycentrics of every live slot's bbox rows at
// x = xmin and at each fragment-segment boundary inside the bbox.
void launch_rowstart(const TriSetup *tris, uint32_t nslots, uint32_t W, uint32_t H, float *rowtab, hipStream_t st);
uint32_t fragment_segments(uint32_t W);

uint32_t fragment_segment_pixels();

void stats_read(unsigned long long out[16], bool reset);

void launch_walk_test(const float *s, const float *d, const uint32_t *n, float *out, uint32_t *lin, float *del,
                      uint32_t count, hipStream_t st);

}  // namespace s3r
