// group_map.h -- the band partition of the multi-GPU paths, shared by the
// C-ABI group (group.hip: partition, device de-interleave kernel, host emulation) and
// restated in octreeraytracer_amd/distributed.py (rank_tile / assemble) for the
// one-process-per-GPU bench path.  16-row bands dealt round-robin: rank r renders bands
// r, r + N, r + 2N, ... (cheap sky rows balanced against geometry rows); every rank the same
// number of rows (rows past the frame render as zeros), so every message has one size.
#pragma once
#include "../../include/ort.h"

#if defined(__HIPCC__)
#define ORT_GM_FN __host__ __device__ inline
#else
#define ORT_GM_FN inline
#endif

namespace ort {

constexpr int kGroupBand = 16;

// Bands of one rank (all ranks render the same number).
ORT_GM_FN int group_bands_per_rank(int height, int world) {
    const int nbands = (height + kGroupBand - 1) / kGroupBand;
    return (nbands + world - 1) / world;
}

// Rank r's tile: every column, its bands in order (ort_tile's band_height / band_stride).
ORT_GM_FN ort_tile group_tile(int width, int height, int rank, int world) {
    ort_tile t;
    t.x0 = 0;
    t.width = width;
    if (world <= 1) {
        t.y0 = 0;
        t.rows = height;
        t.band_height = 0;
        t.band_stride = 0;
        return t;
    }
    t.y0 = rank * kGroupBand;
    t.rows = group_bands_per_rank(height, world) * kGroupBand;
    t.band_height = kGroupBand;
    t.band_stride = kGroupBand * world;
    return t;
}

// Frame row y (GL row, 0 = bottom) -> the rank that rendered it and its row in that rank's tile.
ORT_GM_FN void group_src_row(int y, int world, int& rank, int& trow) {
    if (world <= 1) {
        rank = 0;
        trow = y;
        return;
    }
    const int b = y / kGroupBand;
    rank = b % world;
    trow = (b / world) * kGroupBand + y % kGroupBand;
}

}  // namespace ort
