// ort_kernel.hip -- gfx950 primary/secondary-ray kernel and the device half of the C ABI.
//
// Replaces the reference's GL dispatch: setupBuffers' SSBO uploads
// (src/raytracer.cpp:74-152) become ort_upload_*; the per-frame uniform update +
// glDrawArrays (src/raytracer.cpp:491-499) becomes ort_render, which runs the fragment
// shader (glsl:636-664) as a wavefront pipeline, per sample and bounce:
//   ort_trace_kernel    camera ray (bounce 0) or stored ray + octree walk -> 8-byte hit
//                       record; one path per lane, a wave = 8x8 pixels, a workgroup = 16x16.
//                       Only the sign-specialised fast walk is compiled in, so it runs at
//                       8 waves/SIMD; rays it cannot take are appended to a defer list.
//   ort_trace_persistent  bounces >= 1: the sorted alive-path list, lanes refilled from a queue.
//   ort_trace_exact     the exact walk for the (rare) deferred rays, persistent grid.
//   ort_shade_kernel    BSDF / sky, path state or (1 spp, 1 bounce) the final pixel.
//   ort_finalize_kernel average + gamma for the multi-sample / multi-bounce case.
// The walk keeps one frame per tree level in LDS (columns indexed by lane: conflict-free),
// per-level child masks in registers, and the tree's split-plane table in LDS
// (3 x (2^D+1) floats, loaded once per workgroup).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <type_traits>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "camera.h"
#include "gpu_build.h"
#include "layout.h"
#include "path_key.h"
#include "ort_internal.h"
#include "render_core.h"

#pragma clang fp contract(off)

// ORT_ANALYSIS (Makefile `analysis`: octreeraytracer_amd/lib/libort_analysis.so) adds the
// test/analysis surface: the ort_debug_* entry points (host emulation of the kernel's per-pixel
// code for the CPU suite, walk statistics for tools/), ORT_OPT_DEBUG_FLAGS, and the per-wave
// timeline builds (ORT_TILE_CLOCK, ORT_PERSIST_CLOCK, ORT_PERSIST_STATS, ORT_PIXEL_CLOCK).  The product library
// libort.so is built without it and exports only include/ort.h.
#ifndef ORT_ANALYSIS
#define ORT_ANALYSIS 0
#endif
#if !ORT_ANALYSIS && ((defined(ORT_TILE_CLOCK) && ORT_TILE_CLOCK) || (defined(ORT_PERSIST_CLOCK) && ORT_PERSIST_CLOCK) || \
                      (defined(ORT_PERSIST_STATS) && ORT_PERSIST_STATS) || (defined(ORT_PIXEL_CLOCK) && ORT_PIXEL_CLOCK))
#error "per-wave timeline builds are analysis builds: add -DORT_ANALYSIS=1"
#endif

namespace {

constexpr int kBlock = 256;  // 4 waves, 16x16 pixels

struct TileMap {
    int x0, tw, y0, th, bh, bs;
};

struct PipeArgs {
    ort::PixelParams pp;
    ort::KScene S;
    TileMap tm;
    int tilesX, tilesY;  // the dispatch grid: tiles, or (pair) tile pairs across x tiles
    int pair;         // ORT_OPT_TILE_PAIRS: a camera-ray workgroup renders two tiles side by side (trace_pair_body)
    int swizzle;      // ORT_OPT_XCD_SWIZZLE (block_tile)
    int xrun_log2;    // swizzle 2: log2 of the tiles per XCD run (xcd_run_log2)
    int total;        // path slots = workgroups x 256 (tile-block order, some are holes)
    int sample;       // s of main()'s sample loop
    int last;         // this bounce is the last one (b == maxDepth - 1)
    int nobounce;     // maxDepth <= 0: radiance() returns (1,1,1) without tracing
    int exact_only;   // ORT_OPT_EXACT_TRAVERSAL: every compact ray takes the exact walk
    int refill;       // persistent trace: refill a wave when at least this many lanes idle
    int final_out;    // a path that ends in the last sample writes its final pixel (no finalize pass)
    const int* qlist;    // bounce >= 1: the alive path slots (compacted, increasing), or null = all
    const int* qcount;   // their number (device)
    int* qnext;          // shade kernels: append the paths that go on here (next bounce's list), or null
    int* qnext_count;
    uint32_t* qnext_keys;  // ... and their coherence keys beside them (ORT_OPT_SORT_PATHS 2), or null
    ort::MortonPlan mp;    // the keys' origin code (path_key.h)
    const uint32_t* key_spread;  // ... as table lookups (mortonSpread)
    int2* hit;        // per path: {entry (-1 miss), t bits}
    int* defer_list;
    int* sync;        // [0] deferred count, [1] work cursor of the persistent trace
    int* sync_next;   // ort_trace_exact zeroes these 16 ints: the next trace launch's sync (the other set)
    const uint16_t* scan_pcost;  // ort_trace_exact also lists the next frame's heavy rays (split frames)
    int scan_T;
    uint32_t* scan_bits;
    int* scan_list;
    int* scan_count;
    float4* po;       // o.xyz, importance
    float4* pd;       // d.xyz, alive (1/0)
    float4* pc;       // path throughput c.xyz
    float2* prng;     // randState
    float4* pcol;     // running sum of samples
    float* out;
    unsigned long long* counters;
    uint16_t* pcost;  // ORT_OPT_COST_ORDER: per slot, the walk steps of its last camera ray, or null
    uint16_t* bcost_w;        // ORT_OPT_HEAVY_FIRST: the persistent bounce trace records each walk's steps here
    const uint16_t* bcost_r;  // ... the kernels appending the next bounce's list read that bounce's last-frame steps
    int heavy;                // ... walks of at least this many steps are heavy: they sort first
    // ... and after a camera move (no fresh steps), the class of a path from its ray alone: the
    // root box (lo xyz, hi xyz) and the exit-distance thresholds of classes 0-2 (geo_heavy)
    int geo_heavy;
    float gbox[6];
    float gthr[3];
    int prio_steps;   // ORT_OPT_HEAVY_PRIO: a camera-ray wave holding a ray whose last walk took >= this many
                      // steps runs at raised issue priority (0: off)
    // ORT_OPT_SPLIT_HEAVY (1 sample, 1 bounce): the camera rays whose walk took >= split steps in the
    // previous frame, listed by k_heavy_scan, are walked by ort_trace_split (their walk dealt over 8
    // lanes by level-split_level subtrees) on the context's second stream; the per-tile kernel
    // passes over the slots hbits marks
    const uint32_t* hbits;
    const int* hlist;
    int* hsync;       // [0] heavy rays found (the list holds the first hcap), [1] ort_trace_split's cursor
    int* hsync_next;  // the other pair: ort_trace_split zeroes it for the next frame's scan
    int hcap;
    int split_level;
    // ort_pixel_paths with an LDS-resident scene: byte offset of nk[] in the dynamic LDS (leaf
    // spheres at lds_sph_off), their sizes in 16-byte chunks
    int lds_nk_off, lds_sph_off, lds_nk_n16, lds_sph_n16;
    // ort_pixel_paths, heavy blocks first: the 8x8 blocks in kPixelClasses cost classes (last
    // frame of this shape, read: pl_r / pl_rcnt, or null = tile order) and this frame's classes
    // for the next (pl_w / pl_wcnt; pl_cost: per block {bounces, slots done}); pl_stride blocks
    // per class segment
    const int* pl_r;
    int* pl_rcnt;
    int* pl_w;
    int* pl_wcnt;
    unsigned long long* pl_cost;
    int pl_stride;
    // whole-pixel paths, samples in parallel (ORT_OPT_PIXEL_SPECULATE): a pixel's samples in
    // sp_nch chunks of sp_chunk; per chunk c and slot k (index c * total + k) the RNG state the
    // chunk ends with -- sp_prev last frame's (chunk c+1 of this frame starts from sp_prev[c]),
    // sp_cur this frame's -- and per sample s the radiance (sp_col: three planes of ns * total
    // floats, index s * total + k).  A whole-pixel launch with sp_cur records its chunks' end
    // states; one with fx_slot runs the fixup list: pixel fx_slot[i] from sample fx_s0[i] with
    // state fx_st[i] and the colour sum of its earlier samples fx_col (three planes of total
    // floats), *fx_n entries
    const float2* sp_prev;
    float2* sp_cur;
    float* sp_col;
    int sp_chunk, sp_nch;  // samples per SPEC item (a chunk of a pixel's samples), chunks per pixel
    // sp_ctl[0] the fixup list's length, [1] the pixels the last frame found moved, [2] this
    // frame's mode (1 speculate, 0 fall back: every pixel's whole chain through the fixup list)
    // -- decided on the device by ort_sample_decide, so frames queued ahead of the host follow it
    int* sp_ctl;
    int* fx_n;
    int* fx_slot;
    int* fx_s0;
    float2* fx_st;
    float* fx_col;
#if ORT_ANALYSIS
    ulonglong4* wclock;  // analysis builds only (ORT_PERSIST_CLOCK, ort_debug_wave_clock): per wave a timeline record
    int wclock_n;
#endif
};

__host__ __device__ inline int tile_row_to_y(const TileMap& t, int j) {
    return t.bh > 0 ? t.y0 + (j / t.bh) * t.bs + (j % t.bh) : t.y0 + j;
}

__host__ __device__ inline size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

constexpr size_t kRankLutBytes = 8 * 256;  // ort::rank_lut_entry table

// The persistent bounce kernel at depth 9-10 (Masks96Lean with ORT_REV_BOUNCE): 512-thread
// workgroups over the reversed-table image (fast_rev_planes: 32.8 KB at depth 10, the rank
// LUT in its gap), 53.3 KB of LDS with 512 lanes' frames -- 3 workgroups = 6 waves/SIMD.
constexpr bool kRevBounce = ORT_REV_BOUNCE;
#ifndef ORT_PERSIST_DEEP_BLOCK
#define ORT_PERSIST_DEEP_BLOCK 512
#endif
constexpr int kPersistDeepBlock = kRevBounce ? ORT_PERSIST_DEEP_BLOCK : kBlock;

// with_tm: the exact walk also keeps a per-level tmin column; the fast walk needs none.
// rev / nb: the image layout and workgroup size (the deep persistent kernel's: true, 512).
size_t lds_bytes(int mode, int depth, bool with_tm, bool rev = false, int nb = kBlock) {
    if (mode != 0) return 0;
    const ort::LdsLayout l = ort::lds_layout(depth, rev || ort::fast_rev_planes(depth));
    const size_t levels = (size_t)std::max(depth, 1);
    return (size_t)l.frames + (with_tm ? 2 : 1) * levels * (size_t)nb * sizeof(int);
}

// LDS image of one workgroup: split planes | rank LUT | frame columns (co[, tmin]).
struct LdsView {
    const float* planes;
    const uint8_t* lut;
    ort::LdsFrames fr;
};
template <bool WITH_LUT, int NB = kBlock>
__device__ inline LdsView lds_view(unsigned char* smem, int D, bool rev = false) {
    const ort::LdsLayout l = ort::lds_layout(D, rev || ort::fast_rev_planes(D));
    LdsView v;
    v.planes = reinterpret_cast<float*>(smem);
    v.lut = WITH_LUT ? smem + l.lut : nullptr;
    v.fr.co = reinterpret_cast<int*>(smem + l.frames);
    v.fr.tm = reinterpret_cast<float*>(smem + l.frames + (size_t)(D > 0 ? D : 1) * NB * sizeof(int));
    v.fr.stride = NB;
    v.fr.lane = threadIdx.x;
    return v;
}
// The plane tables and rank LUT are the same for every workgroup of a scene: k_lds_image
// builds them once per scene (ort_ctx::lds_img; at depth 9-10 also the reversed-table image
// ort_ctx::lds_rev) and each workgroup copies the image in 16-byte pieces -- building them
// per workgroup (an integer division per plane entry, ~80 VALU per LUT byte) cost as much
// VALU as several walk steps of every wave.
__global__ void __launch_bounds__(kBlock) k_lds_image(const float* planes, int D, bool rev, unsigned char* img) {
    const int tid = threadIdx.x;
    rev = rev || ort::fast_rev_planes(D);
    ort::fill_fast_planes(planes, reinterpret_cast<float*>(img), D, rev, tid, kBlock);  // forward, then reversed
    __syncthreads();  // the LUT may sit in a gap of the tables (lds_layout)
    uint8_t* lut = img + ort::lds_layout(D, rev).lut;
    for (int i = tid; i < (int)kRankLutBytes; i += kBlock) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
}
// REV: the reversed-table image of a depth 9-10 tree (S.lds_rev), for NB-thread workgroups.
template <bool WITH_LUT, int NB = kBlock, bool REV = false>
__device__ inline LdsView setup_lds(unsigned char* smem, const ort::KScene& S) {
#if defined(__HIP_DEVICE_COMPILE__)
    // The reversed plane tables rely on absolute LDS addresses aligned to their 4T-byte
    // blocks (1 KiB at depth <= 8, up to 4 KiB in the depth 9-10 reversed image); dynamic
    // LDS follows any static LDS (append_slots' counters), so check it.  The address is a
    // link-time constant: the check folds away when it holds and traps loudly when not.
    if (reinterpret_cast<uintptr_t>(smem) & (REV ? 4095u : 1023u)) __builtin_trap();
#endif
    const int n16 = REV ? S.lds_rev_n16 : (WITH_LUT ? S.lds_img_n16 : S.lds_img_p16);
    const uint4* src = REV ? S.lds_rev : S.lds_img;
    uint4* dst = reinterpret_cast<uint4*>(smem);
    for (int i = threadIdx.x; i < n16; i += NB) dst[i] = src[i];
    __syncthreads();
    return lds_view<WITH_LUT, NB>(smem, S.depth, REV);
}

// Tile (bx, by) of 16x16 pixels rendered by workgroup blk.  The dispatcher deals workgroup b
// to XCD b % 8, each XCD with its own L2.  ORT_OPT_XCD_SWIZZLE picks the order:
//   0  raster: XCD x renders every 8th tile of a tile row -- neighbouring tiles, whose rays
//      walk the same octree nodes, are spread over all 8 L2s;
//   2  (default above kRasterAutoPixels) within every 8*run consecutive workgroups the `run` that land on one XCD
//      get `run` consecutive raster tiles (run = xcd_run_log2: 16 tiles, a 256x16-pixel run,
//      at 3840 px): c3 +2% (8-tile runs) and another +1.7% (16), c5 +2% in interleaved A/B
//      (tools/ab_stream.py);
//   1  within every 512 the 64 of one XCD get an 8x8-tile super-tile (128x128 pixels): more
//      compact but slower at c3 (-1.5% vs raster) -- the run order keeps consecutive
//      workgroups of one XCD on neighbouring tiles while they are resident together.
// Each is a bijection on any tile grid (a last partial group keeps raster order; super-tiles at
// the frame's right/bottom edge are narrower), so the pixels are the same whichever order runs.
// Swizzle 2's run length: the largest power of two <= tilesX / 15 (1..64), i.e. each XCD's
// run covers about a fifteenth of a tile row.  Measured (interleaved A/B): 8-tile runs are
// best at 1920 px (120 tiles per row; 16 is 1.9 % slower), 16-tile runs at 3840 px (+1.2 %
// over 8).
#ifndef ORT_XRUN_LOG2
#define ORT_XRUN_LOG2 -1  // A/B builds: a fixed run length (log2); -1: from the frame width
#endif
inline int xcd_run_log2(int tilesX) {
    if (ORT_XRUN_LOG2 >= 0) return ORT_XRUN_LOG2;
    int lr = 0;
    while (lr < 6 && (2 << lr) * 15 <= tilesX) ++lr;
    return lr;
}
__host__ __device__ inline void block_tile_grid(const PipeArgs& A, int blk, int& bx, int& by) {
    if (!A.swizzle) {
        bx = blk % A.tilesX;
        by = blk / A.tilesX;
        return;
    }
    int l = blk;
    if (A.swizzle == 2) {  // raster order in chunks of 8 tiles per XCD
        const int lr = A.xrun_log2, run = 1 << lr, group = 8 << lr;
        if ((blk | (group - 1)) < A.tilesX * A.tilesY)
            l = (blk & ~(group - 1)) | ((blk & 7) << lr) | ((blk >> 3) & (run - 1));
        bx = l % A.tilesX;
        by = l / A.tilesX;
        return;
    }
    if ((blk | 511) < A.tilesX * A.tilesY) l = (blk & ~511) | ((blk & 7) << 6) | ((blk >> 3) & 63);
    // logical order: super-rows of 8 tile rows; in one, super-tiles of 8 tile columns left to
    // right; in one, tiles in raster order
    const int srow = l / (A.tilesX * 8);
    const int rem = l - srow * A.tilesX * 8;
    const int rows = A.tilesY - srow * 8 < 8 ? A.tilesY - srow * 8 : 8;
    const int sc = rem / (8 * rows);
    const int r2 = rem - sc * 8 * rows;
    const int cols = A.tilesX - sc * 8 < 8 ? A.tilesX - sc * 8 : 8;
    bx = sc * 8 + r2 % cols;
    by = srow * 8 + r2 / cols;
}
// Tile pairs (ORT_OPT_TILE_PAIRS): slot blocks 2b and 2b+1 are the two tiles of pair b, which the
// swizzle places on the pair grid (x-adjacent tiles; a last odd column's second tile is a hole).
__host__ __device__ inline void block_tile(const PipeArgs& A, int blk, int& bx, int& by) {
    if (!A.pair) {
        block_tile_grid(A, blk, bx, by);
        return;
    }
    block_tile_grid(A, blk >> 1, bx, by);
    bx = 2 * bx + (blk & 1);
}

// Path slot k (tile-block order: 256 slots = one 16x16 tile, 64 = one 8x8 wave block)
// -> tile column/row.  Returns false for slots outside the tile.  UNI: every lane of the wave
// holds a slot of the same 256-slot block (the per-tile kernels), so the tile lookup -- two
// integer divisions by the tile-grid width -- runs once per wave on the scalar unit.  UNI 2:
// every lane holds a slot of the same tile PAIR (tile pairs, cost_order_pair), so the pair's
// place is looked up once per wave and each lane picks its tile of the two.
template <int UNI = 0>
__host__ __device__ inline bool slot_coords(const PipeArgs& A, int k, int& col, int& row) {
    const int tid = k & 255, wave = tid >> 6, lane = tid & 63;
    int bx, by;
#if defined(__HIP_DEVICE_COMPILE__)
    if (UNI == 2) {
        block_tile_grid(A, __builtin_amdgcn_readfirstlane(k >> 9), bx, by);
        bx = 2 * bx + ((k >> 8) & 1);
    } else {
        block_tile(A, UNI ? __builtin_amdgcn_readfirstlane(k >> 8) : k >> 8, bx, by);
    }
#else
    block_tile(A, k >> 8, bx, by);
#endif
    col = bx * 16 + (wave & 1) * 8 + (lane & 7);  // an 8x8 block per wave (16x4 and 4x16: no faster, §8)
    row = by * 16 + (wave >> 1) * 8 + (lane >> 3);
    return col < A.tm.tw && row < A.tm.th;
}

template <bool COUNT>
__device__ inline void flush_counts(const ort::Counters& c, unsigned long long* dst) {
    if (COUNT)
        for (int k = 0; k < 6; ++k)
            if (c.v[k]) atomicAdd(dst + k, c.v[k]);
}

__device__ inline ort::Ray load_ray(const PipeArgs& A, int k, bool& alive) {
    const float4 o = A.po[k], d = A.pd[k];
    ort::Ray r;
    r.o = ort::mk(o.x, o.y, o.z);
    r.d = ort::mk(d.x, d.y, d.z);
    alive = d.w != 0.0f;
    return r;
}

// Persistent trace over the compact layout: every lane keeps one ray's FastState; the
// wave owns a chunk of kChunk consecutive path slots (one atomic on the global cursor per
// chunk, MI355X_MICROARCH.md 'dequeue') and hands the next slots of its chunk to lanes
// that finished, so the wave stays full until the queue drains.  Rays the fast walk
// cannot take are appended to the defer list for ort_trace_exact.
// Waves per SIMD (minimum, amdgpu_waves_per_eu): the per-lane trace kernels run at 8 (59-64
// VGPRs, spill-free; tools/kernel_resources.py).  The persistent bounce kernel is asked for 6:
// its depth 9-10 walk over the reversed plane tables fits 79 VGPRs there without spills (the
// forward-table walk needed 87 unconstrained and spilled 5 at 6 waves), and its LDS (53.3 KB
// per 512-thread workgroup at depth 10) caps it at 6 anyway; the depth <= 8 instance 78.
#ifndef ORT_PERSISTENT_WAVES
#define ORT_PERSISTENT_WAVES 6
#endif
#ifndef ORT_TRACE_WAVES
#define ORT_TRACE_WAVES 8
#endif
// Deep (depth > 8) per-lane kernel: its LDS image (24.6 KB per 256-thread workgroup at depth 10)
// caps a CU at 6 workgroups = 6 waves/SIMD, so it may use the registers of 6 waves: 60-64
// VGPRs without spills.  (512-thread workgroups, whose LDS would allow 8 waves/SIMD at these
// 64 VGPRs, measured no faster: C5 -0.1 % at 6, -0.4 % at 8 in A/B.)
#ifndef ORT_TRACE_WAVES_DEEP
#define ORT_TRACE_WAVES_DEEP 6
#endif
// Items a wave takes from the global cursor at a time.  The resident waves then work on a
// window of about (waves x kChunk) consecutive list items -- neighbouring paths, overlapping
// node sets, one L2 working set: C5 frame 58.2 (256) -> 56.7 (128) -> 55.8 ms (64; 32: 56.0)
// in A/B.  (One queue per XCD over 8 contiguous list ranges measured no better: -0.4 %.)
#ifndef ORT_PERSIST_CLOCK
#define ORT_PERSIST_CLOCK 0
#endif
// Analysis builds only (-DORT_PERSIST_STATS=1, tools/persist_stats.py): per wave of the persistent
// kernel, how its loop iterations went -- refills, steps, and how many lanes stepped an internal
// node or a leaf (the two blocks of a step run one after the other, each with its own lanes).
#ifndef ORT_PERSIST_STATS
#define ORT_PERSIST_STATS 0
#endif
// Leaf hold in the depth 9-10 bounce walk: a lane whose next node is a leaf waits until this many
// lanes of its wave are at leaves (or none is at an internal node), so the leaf block -- run in 92 %
// of the steps for 6.5 lanes on average (tools/persist_stats.py) -- runs less often for more lanes.
// C5 +2.4 / +2.7 / +2.3 / -2.4 % at 8 / 12 / 16 / 24 (tools/ab_stream.py); the depth <= 8 bounce
// walk loses (C3 at 4 bounces: -1.7 % at 8), so it is off there.
#ifndef ORT_LEAF_HOLD
#define ORT_LEAF_HOLD 12
#endif
// ... and only while at least this many lanes are at internal nodes: in a launch's drain (few lanes
// left) a held leaf lane would wait for a lone internal walk -- C5 1/8 band at one frame in
// flight 7.2 -> 8.2 ms with 1 (full frame: 16 and 1 alike)
#ifndef ORT_LEAF_HOLD_MIN_INTERNAL
#define ORT_LEAF_HOLD_MIN_INTERNAL 16
#endif
#ifndef ORT_CHUNK
#define ORT_CHUNK 64
#endif
constexpr int kChunk = ORT_CHUNK;
// Lists of at least ORT_CHUNK_ADAPT items per resident wave take chunks of 2 x kChunk: C5
// +0.7 % (bounces 1-2 of the full frame), band tiles unchanged (tools/ab_stream.py); fixed
// 128-item chunks lost 20 % on a 1/8 band (too few chunks per wave to balance).  0: kChunk.
#ifndef ORT_CHUNK_ADAPT
#define ORT_CHUNK_ADAPT 1024
#endif

// DEEP: trees deeper than 8 levels (96-bit masks, lean state); depth <= 8 takes the
// primary-ray walk's 64-bit masks and reversed plane tables (71 VGPRs, 7 waves/SIMD).
template <bool COUNT, bool DEEP>
__global__ void __launch_bounds__(DEEP ? kPersistDeepBlock : kBlock) __attribute__((amdgpu_waves_per_eu(ORT_PERSISTENT_WAVES)))
ort_trace_persistent(PipeArgs A) {
    // plane tables at 4T-byte-aligned absolute LDS addresses (fast_rev_planes; no static LDS here)
    extern __shared__ __attribute__((aligned(4096))) unsigned char smem[];
    constexpr bool REV = DEEP && kRevBounce;
    LdsView L = setup_lds<true, DEEP ? kPersistDeepBlock : kBlock, REV>(smem, A.S);
    const uint8_t* lut = L.lut;
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    ort::Counters cnt;
    for (int q = 0; q < 6; ++q) cnt.v[q] = 0;
    // depth <= 8 without the inline leaf children: on incoherent bounce rays they cost 9 %
    // (C3 scene, 8 bounces); the plain 64-bit walk is 5 % faster than the 96-bit one there
    using Masks = typename std::conditional<DEEP, ort::Masks96Lean, ort::Masks64Plain>::type;
    ort::FastStateT<Masks> st;
    int k = -1;
    int nst = 0;             // steps of the lane's walk (ORT_OPT_HEAVY_FIRST's record)
    int next = 0, end = 0;   // wave-uniform: remaining work items [next, end) of the wave's chunk
    bool drained = false;    // wave-uniform: the global cursor passed the item count
    // items: the compacted (sorted) alive-path list of a bounce >= 1, or every slot
    const int total = A.qlist ? *A.qcount : A.total;
#if ORT_CHUNK_ADAPT
    // long lists (>= ORT_CHUNK_ADAPT items per resident wave): twice the chunk
    const int chunk = total >= (int)(gridDim.x * (blockDim.x >> 6)) * ORT_CHUNK_ADAPT ? 2 * kChunk : kChunk;
#else
    constexpr int chunk = kChunk;
#endif
#if ORT_PERSIST_CLOCK  // analysis builds only (tools/build_variant.sh): per-wave timeline
    const unsigned long long clk0 = __builtin_amdgcn_s_memrealtime();
    unsigned long long clk_drain = 0;
    int n_items = 0;
#endif
#if ORT_PERSIST_STATS
    unsigned long long ps[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // iterations, refills, steps, internal lanes,
                                                            // leaf lanes, steps with internal / leaf / both
#endif
    for (;;) {
        const unsigned long long idle = __ballot(k < 0);
        const int n_idle = __popcll(idle);
        if (n_idle == 64 && drained) break;
#if ORT_PERSIST_STATS
        ps[0] += 1;
#endif
        if (!drained && n_idle >= A.refill) {
#if ORT_PERSIST_STATS
            ps[1] += 1;
#endif
            if (next == end) {
                int base = 0;
                if (lane == 0) base = atomicAdd(A.sync + 1, chunk);
                base = __shfl(base, 0);
                if (base >= total) {
                    drained = true;
#if ORT_PERSIST_CLOCK
                    clk_drain = __builtin_amdgcn_s_memrealtime();
#endif
                    continue;
                }
#if ORT_PERSIST_CLOCK
                n_items += min(base + chunk, total) - base;
#endif
                next = base;
                end = min(base + chunk, total);
            }
            const int take = min(n_idle, end - next);
            if (k < 0) {
                const int rank = __popcll(idle & below);
                if (rank < take) {
                    const int cand = A.qlist ? A.qlist[next + rank] : next + rank;
                    bool alive;
                    const ort::Ray ray = load_ray(A, cand, alive);
                    if (alive) {
                        ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
                        if (A.exact_only || !ort::fast_prepare(A.S, ray, inv)) {
                            A.defer_list[atomicAdd(A.sync, 1)] = cand;
                        } else {
                            if (COUNT) cnt.v[5] += 1;
                            nst = 0;
                            if (ort::fast_begin(A.S, L.planes, lut, ray, inv, 0.001f, ORT_MAXFLOAT, st)) k = cand;
                            else A.hit[cand] = make_int2(-1, 0);
                        }
                    }
                }
            }
            next += take;
            continue;
        }
#if ORT_PERSIST_STATS
        {
            const bool in = k >= 0 && (st.rec.y & ORT_INTERNAL_FLAG);
            const bool lf = k >= 0 && !(st.rec.y & ORT_INTERNAL_FLAG);
            const int ni = __popcll(__ballot(in)), nl = __popcll(__ballot(lf));
            ps[2] += 1;
            ps[3] += ni;
            ps[4] += nl;
            ps[5] += ni > 0;
            ps[6] += nl > 0;
            ps[7] += (ni > 0 && nl > 0);
        }
#endif
#if ORT_LEAF_HOLD
        // leaf hold (DEEP): each lane's own walk is unchanged, only when it steps (same pixels)
        bool hold = false;
        if (DEEP) {
            const bool at_leaf = k >= 0 && !(st.rec.y & ORT_INTERNAL_FLAG);
            const unsigned long long lm = __ballot(at_leaf), im = __ballot(k >= 0 && !at_leaf);
            hold = at_leaf && __popcll(im) >= ORT_LEAF_HOLD_MIN_INTERNAL && __popcll(lm) < ORT_LEAF_HOLD;
        }
        if (k >= 0 && !hold) {
#else
        if (k >= 0) {
#endif
            ++nst;
            if (ort::fast_step<COUNT>(A.S, lut, st, L.fr, cnt)) {
                A.hit[k] = make_int2(st.hitEntry, __float_as_int(st.closest));
                if (!COUNT && A.bcost_w) A.bcost_w[k] = (uint16_t)min(nst, 65535);
                k = -1;
            }
        }
    }
#if ORT_PERSIST_CLOCK
    const int gw = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
    if (A.wclock && lane == 0 && gw < A.wclock_n) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        A.wclock[gw] = make_ulonglong4(clk0, clk_drain, __builtin_amdgcn_s_memrealtime(),
                                       (unsigned long long)(xcc & 15u) | ((unsigned long long)n_items << 8));
    }
#endif
#if ORT_PERSIST_STATS
    {
        const int gw = (int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6));
        if (A.wclock && lane == 0 && 2 * gw + 1 < A.wclock_n) {
            A.wclock[2 * gw] = make_ulonglong4(ps[0], ps[1], ps[2], ps[3]);
            A.wclock[2 * gw + 1] = make_ulonglong4(ps[4], ps[5], ps[6], ps[7]);
        }
    }
#endif
    flush_counts<COUNT>(cnt, A.counters);
}

// Bounce >= 1 with a compacted list: thread index -> alive path slot (false past the list).
__device__ inline bool list_slot(const PipeArgs& A, int& k) {
    if (!A.qlist) return true;
    if (k >= *A.qcount) return false;
    k = A.qlist[k];
    return true;
}

// Path-slot ray for the trace kernels: bounce 0 generates the sample's camera ray here
// (main() up to radiance()'s first line; the shade kernel regenerates it identically),
// later bounces read the ray the previous shade kernel stored.
template <bool PRIMARY, int UNI = 0>
__device__ inline ort::Ray slot_ray(const PipeArgs& A, int k, bool& alive, ort_rng* st_out = nullptr) {
    if constexpr (PRIMARY) {
        int col, row;
        alive = slot_coords<UNI>(A, k, col, row);
        const int y = alive ? tile_row_to_y(A.tm, row) : 0;
        alive = alive && y < A.pp.H;
        ort::Ray ray;
        ray.o = ort::mk(0.0f, 0.0f, 0.0f);
        ray.d = ray.o;
        if (!alive) return ray;
        ort_rng st;
        if (A.sample == 0) {
            ort::pixel_rng_init(A.pp, A.tm.x0 + col, y, st);
        } else {
            const float2 v = A.prng[k];
            st.x = v.x;
            st.y = v.y;
        }
        const ort::Ray r = ort::primary_ray(A.pp, A.tm.x0 + col, y, A.sample, st);
        if (st_out) *st_out = st;
        return r;
    } else {
        return load_ray(A, k, alive);
    }
}

// 1 sample, 1 bounce (the primary-ray benchmark mode): the trace kernels shade their own
// rays -- exactly ort_shade_kernel<0, true, true> -- instead of writing hit records for it.
template <int UNI = 0>
__device__ inline void shade_direct(const PipeArgs& A, int k, ort::Ray ray, ort_rng st, bool hit, int entry, float t) {
    int col, row;
    (void)slot_coords<UNI>(A, k, col, row);
    ort::V3 c = ort::mk(1.0f, 1.0f, 1.0f);
    float importance = 1.0f;
    ort::HitRec rec;
    if (hit) rec = ort::hit_record<0>(A.S, ray, t, entry);
    (void)ort::shade_bounce<true>(hit, rec, ray, c, importance, st);  // 1 sample, 1 bounce: final
    const ort::V3 v = ort::finish_pixel(ort::add(ort::mk(0.0f, 0.0f, 0.0f), c), 1);
    float* o = A.out + 3 * ((size_t)row * A.tm.tw + col);
    // plain stores (one global_store_dwordx3): non-temporal ones ran no faster and, their
    // partial 64-byte lines written out unmerged, moved 1.38x the frame's bytes (PMC WRITE_SIZE)
    o[0] = v.x;
    o[1] = v.y;
    o[2] = v.z;
}
// Tile rows past the frame (band padding) are written as zeros, as the shade kernel does.
template <int UNI = 1>
__device__ inline void shade_direct_padding(const PipeArgs& A, int k) {
    int col, row;
    if (!slot_coords<UNI>(A, k, col, row) || tile_row_to_y(A.tm, row) < A.pp.H) return;
    float* o = A.out + 3 * ((size_t)row * A.tm.tw + col);
    o[0] = 0.0f;
    o[1] = 0.0f;
    o[2] = 0.0f;
}

// The shading proper of path slot k, given its ray and RNG state and the walk's result
// (entry < 0: no hit); shared by ort_shade_kernel and the trace kernels that shade bounce 0
// themselves.  Returns true when the path goes on to the next bounce.
template <int MODE, bool FIRST, bool DIRECT>
__device__ __forceinline__ bool shade_state(const PipeArgs& A, int k, size_t p, ort::Ray ray, ort_rng st, int entry,
                                            float t) {
    ort::V3 c = ort::mk(1.0f, 1.0f, 1.0f);
    float importance = 1.0f;
    if (!FIRST) {
        const float4 cc = A.pc[k];
        c = ort::mk(cc.x, cc.y, cc.z);
        importance = A.po[k].w;
    }
    bool done = true;
    if (!A.nobounce) {
        ort::HitRec rec;
        if (entry >= 0) rec = ort::hit_record<MODE>(A.S, ray, t, entry);
        if (A.last && A.sample == A.pp.ns - 1)  // nothing reads the ray or RNG state after this bounce
            done = ort::shade_bounce<true>(entry >= 0, rec, ray, c, importance, st);
        else
            done = ort::shade_bounce(entry >= 0, rec, ray, c, importance, st);
        if (!done && (A.last || importance < 0.01f)) done = true;  // loop bound / glsl:605
    }
    if constexpr (DIRECT) {
        const ort::V3 v = ort::finish_pixel(ort::add(ort::mk(0.0f, 0.0f, 0.0f), c), 1);
        float* o = A.out + 3 * p;
        o[0] = v.x; o[1] = v.y; o[2] = v.z;
    } else {
        // the last sample of a final_out frame: a path that ends here writes its pixel and
        // nothing else -- the later kernels walk the lists of alive paths only, and no sample
        // follows to read its RNG state
        const bool fin = A.final_out && A.sample == A.pp.ns - 1;
        if (done) {
            ort::V3 acc = ort::mk(0.0f, 0.0f, 0.0f);
            if (A.sample > 0) {
                const float4 a = A.pcol[k];
                acc = ort::mk(a.x, a.y, a.z);
            }
            acc = ort::add(acc, c);
            if (fin) {  // ort_finalize_kernel's work for this pixel
                const ort::V3 v = ort::finish_pixel(acc, A.pp.ns);
                float* o = A.out + 3 * p;
                o[0] = v.x; o[1] = v.y; o[2] = v.z;
            } else {
                A.pcol[k] = make_float4(acc.x, acc.y, acc.z, 0.0f);
                A.pd[k] = make_float4(ray.d.x, ray.d.y, ray.d.z, 0.0f);
            }
        } else {
            A.po[k] = make_float4(ray.o.x, ray.o.y, ray.o.z, importance);
            A.pd[k] = make_float4(ray.d.x, ray.d.y, ray.d.z, 1.0f);
            A.pc[k] = make_float4(c.x, c.y, c.z, 0.0f);
        }
        if (!(done && fin)) A.prng[k] = make_float2(st.x, st.y);
    }
    return !DIRECT && !done;
}

// Appends slot k (where go) to list / count: one atomic per workgroup, the workgroup's slots
// kept in increasing order.  Every thread of the workgroup must call it.
__device__ inline void append_slots(bool go, int k, uint32_t key, int* list, uint32_t* keys, int* count) {
    __shared__ int wcnt[kBlock / 64];
    __shared__ int wbase;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const unsigned long long m = __ballot(go);
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int i = 0; i < kBlock / 64; ++i) t += wcnt[i];
        wbase = t ? atomicAdd(count, t) : 0;
    }
    __syncthreads();
    int off = wbase;
    for (int i = 0; i < w; ++i) off += wcnt[i];
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    if (go) {
        const int pos = off + __popcll(m & below);
        list[pos] = k;
        if (keys) keys[pos] = key;
    }
}

// Heavy first (ORT_OPT_HEAVY_FIRST): the key of a path appended to the next bounce's list gets
// a 2-bit cost class above its coherence bits, from the steps c that bounce's walk took in
// the previous frame of the same shape: 0 for c >= 4T, 1 for >= 2T, 2 for >= T, 3 below (T =
// A.heavy) -- the list sort then puts the longest walks first, each class in coherence order,
// and the persistent trace starts them early instead of in its drain tail.
#ifndef ORT_HEAVY_LEVELS
#define ORT_HEAVY_LEVELS 3  // classes above the lightest (1: one threshold)
#endif
#ifndef ORT_HEAVY_RATIO_LOG2
#define ORT_HEAVY_RATIO_LOG2 1  // class thresholds T, 2T, 4T
#endif
static_assert(ORT_HEAVY_LEVELS >= 1 && ORT_HEAVY_LEVELS <= 7, "ORT_HEAVY_LEVELS: 1..7 classes above the lightest");
constexpr int kHeavyKeyBits = ORT_HEAVY_LEVELS > 3 ? 3 : (ORT_HEAVY_LEVELS > 1 ? 2 : 1);
// the class sits above the path key's bits in a 32-bit radix key (sortListBounded's end bit)
static_assert(ort::kPathKeyBits + kHeavyKeyBits <= 32, "heavy-first class bits + path key bits exceed 32");
// Heavy first after a camera move: the class from the new ray alone -- bounce walks of rays that
// leave the root box soon run longest (the C5 slab, bounce 1: exit within 1.2x the box's
// smallest extent, half of the rays, 29 % of them >= 256 steps; beyond 6.8x, 0.5 %;
// tools/bounce_texit.py).  Classes 0-2 by the thresholds gthr, 3 beyond (as light_bit's).
__device__ __forceinline__ uint32_t geo_class_bits(const float* gb, const float* th, float4 o, float4 d) {
    float tx = 3.0e38f;
    const float oa[3] = {o.x, o.y, o.z}, da[3] = {d.x, d.y, d.z};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float inv = 1.0f / da[a];  // (+-inf for a zero component: that axis never bounds)
        const float t = fmaxf((gb[a] - oa[a]) * inv, (gb[3 + a] - oa[a]) * inv);
        tx = fminf(tx, t);
    }
    const uint32_t cls = tx <= th[0] ? 0u : (tx <= th[1] ? 1u : (tx <= th[2] ? 2u : 3u));
    return min(cls, (uint32_t)ORT_HEAVY_LEVELS) << ort::kPathKeyBits;
}
__device__ __forceinline__ uint32_t light_bit(const uint16_t* bcost_r, int heavy, int k) {
    if (!bcost_r) return 0u;
    const int c = bcost_r[k];
    uint32_t cls = ORT_HEAVY_LEVELS;
    for (int l = 0; l < ORT_HEAVY_LEVELS; ++l) cls -= c >= (heavy << (ORT_HEAVY_RATIO_LOG2 * l)) ? 1u : 0u;
    return cls << ort::kPathKeyBits;
}
// The sort key of path k (its state just stored) with its heavy-first class.
__device__ __forceinline__ uint32_t path_key_class(const PipeArgs& A, int k) {
    const float4 o = A.po[k], d = A.pd[k];
    return ort::path_key(o, d, A.mp, A.key_spread) |
           (A.geo_heavy ? geo_class_bits(A.gbox, A.gthr, o, d) : light_bit(A.bcost_r, A.heavy, k));
}

// One ray per lane over the compact layout (default): the tile-block order of the path
// slots keeps each wave on an 8x8 pixel block, whose rays walk nearly the same nodes.
// DEEP: trees deeper than 8 levels need the 96-bit level masks (ort_trace_compact_deep).
// One path slot k of the compact-layout trace (the per-lane walk); counts accumulate in cnt.
// FUSE: 0 the walk's hit record is stored (shaded by ort_shade_kernel); 1 (1 sample, 1 bounce)
// the kernel shades its ray into the final pixel; 2 (bounce 0 of a multi-bounce frame) the
// kernel shades its ray into the path state and returns whether the path goes on.
// UNI: every lane of the wave holds a slot of the same tile (slot_coords); tile pairs: of either.
template <bool COUNT, bool PRIMARY, bool DEEP, int FUSE, int UNI = 1>
__device__ __forceinline__ bool trace_slot(PipeArgs& A, LdsView& L, int k, ort::Counters& cnt) {
    bool alive;
    ort_rng rng0;  // FUSE: the camera ray's RNG state, kept for the shading after the walk
    const ort::Ray ray = slot_ray<PRIMARY, UNI>(A, k, alive, FUSE ? &rng0 : nullptr);
    if (!alive) {
        if (FUSE == 1) shade_direct_padding<UNI>(A, k);
        if (FUSE == 2) {
            A.pd[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // never alive (ort_shade_kernel's hole)
            if (A.final_out && A.sample == A.pp.ns - 1) shade_direct_padding<UNI>(A, k);  // band padding rows
        }
        return false;
    }
    ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    // camera rays (jittered: practically never a zero component) keep the plain check, which
    // costs the hot kernel less (C3 +0.7 %); bounce rays take zero components fast too
    if constexpr (PRIMARY && !COUNT && FUSE != 0) {
        if (A.hbits && ((A.hbits[k >> 5] >> (k & 31)) & 1u)) return false;  // ort_trace_split walks and shades it
    }
    if (A.exact_only || !(PRIMARY ? ort::fast_path_ok(ray, inv, 0.001f, ORT_MAXFLOAT) : ort::fast_prepare(A.S, ray, inv))) {
        A.defer_list[atomicAdd(A.sync, 1)] = k;  // ort_trace_exact walks (and, FUSE, shades) it
        if (PRIMARY && !COUNT && A.pcost) A.pcost[k] = 0;
        return false;
    }
    if (COUNT) cnt.v[5] += 1;
    float t = 0.0f;
    int entry = -1;
    using Masks = typename std::conditional<DEEP, ort::Masks96, ort::Masks64>::type;
    ort::Ray walked;
    int steps = 0;
    const bool hit = ort::traverse_fast_t<COUNT, Masks>(A.S, L.planes, L.lut, ray, inv, 0.001f, ORT_MAXFLOAT, entry, t,
                                                        L.fr, cnt, FUSE ? &walked : nullptr,
                                                        (PRIMARY && !COUNT) ? &steps : nullptr);
    if (PRIMARY && !COUNT) {  // the cost order's record for the next frame (cost_order_slot)
#if defined(__HIP_DEVICE_COMPILE__)
        typedef __attribute__((address_space(4))) const PipeArgs KernArgs;
        KernArgs* kp = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        uint16_t* pc = kp->pcost;
#else
        uint16_t* pc = A.pcost;
#endif
        if (pc) pc[k] = (uint16_t)min(steps, 65535);
    }
    if (FUSE) {
        // shade with the ray rebuilt from the walk state (bit-identical, no registers held
        // across the walk) and the RNG state kept from the camera ray (2 registers) -- 4 %
        // faster at C3 than regenerating both after the walk; the kernel arguments are re-read
        // through a laundered pointer: held across the walk they overflow the SGPRs
        int k2 = k;
        asm volatile("" : "+v"(k2));
#if defined(__HIP_DEVICE_COMPILE__)
        typedef __attribute__((address_space(4))) const PipeArgs KernArgs;  // the kernarg segment
        KernArgs* kp = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        const PipeArgs A2 = *kp;
#else
        const PipeArgs& A2 = A;
#endif
        if constexpr (FUSE == 1) {
            shade_direct<UNI>(A2, k2, walked, rng0, hit, entry, t);
        } else {
            int col, row;
            (void)slot_coords<UNI>(A2, k2, col, row);
            return shade_state<0, true, false>(A2, k2, (size_t)row * A2.tm.tw + col, walked, rng0, hit ? entry : -1, t);
        }
    } else {
        A.hit[k] = make_int2(hit ? entry : -1, __float_as_int(t));
    }
    return false;
}

// Cost order (ORT_OPT_COST_ORDER): a wave runs as long as its slowest lane, and the camera
// rays of one 8x8 block differ by up to several times in walk steps (background next to a
// sphere's silhouette).  Each workgroup deals its 256 slots to its 4 waves by the walk steps
// their rays took in the previous frame (pcost, a bucket per 4 steps, stable counting sort:
// equal buckets keep tile order), so rays of like cost share a wave.  Only which lane walks
// which slot changes -- every slot's ray, path state and pixel are the same (bit-identical
// frames).  A first frame (pcost cleared) keeps tile order.  Scratch: the first 512 ints of the
// frame columns (free before the walk; lds_bytes >= 2 levels).
#ifndef ORT_COST_SHIFT
// bucket = steps >> shift (64 buckets): 2-step buckets since tile pairs (C3 +1.3 % in A/B over
// 4-step ones, profiles/r04_c3_xr.log; with one tile per workgroup they measured alike)
#define ORT_COST_SHIFT 1
#endif
#ifndef ORT_COST_SHIFT_DEEP
#define ORT_COST_SHIFT_DEEP 2  // the depth 9-10 camera kernel's bucket width
#endif
template <int SHIFT>
__device__ __forceinline__ int cost_order_slot(const uint16_t* pcost, int* sc, int k) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t b = min((uint32_t)pcost[k] >> SHIFT, 63u);
    uint64_t m = ~0ull;  // the lanes of this wave in the same bucket
    for (int i = 0; i < 6; ++i) {
        const uint64_t bal = __ballot((b >> i) & 1u);
        m &= ((b >> i) & 1u) ? bal : ~bal;
    }
    const int below = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    int* cnt = sc;         // [wave][bucket]: lanes, then first position
    int* perm = sc + 256;  // position -> thread of the natural order
    cnt[tid] = 0;
    __syncthreads();
    if (below == 0) cnt[wave * 64 + b] = __popcll(m);
    __syncthreads();
    if (wave == 0) {  // lane = bucket: exclusive scan of the bucket totals
        const int c0 = cnt[lane], c1 = cnt[64 + lane], c2 = cnt[128 + lane], c3 = cnt[192 + lane];
        const int tot = c0 + c1 + c2 + c3;
        int incl = tot;
        for (int off = 1; off < 64; off <<= 1) {
            const int v = __shfl_up(incl, off);
            if (lane >= off) incl += v;
        }
        const int base = incl - tot;
        cnt[lane] = base;
        cnt[64 + lane] = base + c0;
        cnt[128 + lane] = base + c0 + c1;
        cnt[192 + lane] = base + c0 + c1 + c2;
    }
    __syncthreads();
    perm[cnt[wave * 64 + b] + below] = tid;
    __syncthreads();
    const int kk = (k & ~(kBlock - 1)) | perm[tid];
    __syncthreads();  // the frame columns are the walk's from here
    return kk;
#else
    (void)pcost;
    (void)sc;
    return k;
#endif
}

// Cost order over a tile pair (ORT_OPT_TILE_PAIRS): the 512 slots of workgroup b (slots 512b ..
// 512b + 511, two tiles) in eight blocks of 64 by last frame's walk steps (the stable counting
// sort of cost_order_slot, buckets of 2^SHIFT steps: 2 by default), and wave w walks block 7 - w and then block w: a
// workgroup holds its LDS until its slowest wave ends, and with one block per wave the cost
// order left 12-13 % of the waves' time idle inside the workgroups (tools/tile_clock.py); the
// longest-processing-time pairs (7,0) (6,1) (5,2) (4,3) even the waves out.  Scratch: the
// first 1024 ints of the frame columns (free before the walk; lds_bytes >= 4 levels).
template <int SHIFT>
__device__ __forceinline__ void cost_order_pair(const uint16_t* pcost, int* sc, int base, int& kk0, int& kk1) {
#if defined(__HIP_DEVICE_COMPILE__)
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const uint32_t b0 = min((uint32_t)pcost[base + tid] >> SHIFT, 63u);
    const uint32_t b1 = min((uint32_t)pcost[base + 256 + tid] >> SHIFT, 63u);
    uint64_t m0 = ~0ull, m1 = ~0ull;  // the lanes of this wave in the same bucket, per item
    for (int i = 0; i < 6; ++i) {
        const uint64_t bal0 = __ballot((b0 >> i) & 1u), bal1 = __ballot((b1 >> i) & 1u);
        m0 &= ((b0 >> i) & 1u) ? bal0 : ~bal0;
        m1 &= ((b1 >> i) & 1u) ? bal1 : ~bal1;
    }
    const int below0 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m0, 0u));
    const int below1 = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m1, 0u));
    int* cnt = sc;         // [virtual wave 0..7][bucket]: items, then first position
    int* perm = sc + 512;  // position -> item (0..511)
    cnt[tid] = 0;
    cnt[256 + tid] = 0;
    __syncthreads();
    if (below0 == 0) cnt[wave * 64 + b0] = __popcll(m0);
    if (below1 == 0) cnt[(4 + wave) * 64 + b1] = __popcll(m1);
    __syncthreads();
    if (wave == 0) {  // lane = bucket: exclusive scan of the bucket totals, then the virtual waves in order
        int c[8];
        int tot = 0;
        for (int v = 0; v < 8; ++v) {
            c[v] = cnt[v * 64 + lane];
            tot += c[v];
        }
        int incl = tot;
        for (int off = 1; off < 64; off <<= 1) {
            const int x = __shfl_up(incl, off);
            if (lane >= off) incl += x;
        }
        int pos = incl - tot;
        for (int v = 0; v < 8; ++v) {
            cnt[v * 64 + lane] = pos;
            pos += c[v];
        }
    }
    __syncthreads();
    perm[cnt[wave * 64 + b0] + below0] = tid;
    perm[cnt[(4 + wave) * 64 + b1] + below1] = 256 + tid;
    __syncthreads();
    kk0 = base + perm[64 * (7 - wave) + lane];
    kk1 = base + perm[64 * wave + lane];
    __syncthreads();  // the frame columns are the walk's from here
#else
    (void)pcost;
    (void)sc;
    kk0 = base + (int)threadIdx.x;
    kk1 = kk0 + 256;
#endif
}

// Analysis builds only (-DORT_TILE_CLOCK=1, tools/tile_clock.py): the per-tile camera-ray
// kernels record per wave {start, end, XCC id, the longest walk of its lanes} into wclock.
#ifndef ORT_TILE_CLOCK
#define ORT_TILE_CLOCK 0
#endif
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
template <bool ON>
__device__ inline void tile_clock_record(int k0, int k1, unsigned long long tclk0) {
    if (!ON) return;
    typedef __attribute__((address_space(4))) const PipeArgs KernArgs;
    KernArgs* kp = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
    int st = kp->pcost ? max((int)kp->pcost[k0], (int)kp->pcost[k1]) : 0;
    for (int o = 32; o >= 1; o >>= 1) st = max(st, __shfl_xor(st, o));
    const int gw = (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
    if (kp->wclock && (threadIdx.x & 63) == 0 && gw < kp->wclock_n) {
        const unsigned xcc = __builtin_amdgcn_s_getreg((15 << 11) | 20);  // XCC_ID
        kp->wclock[gw] = make_ulonglong4(tclk0, __builtin_amdgcn_s_memrealtime(), xcc & 15u, (unsigned long long)st);
    }
}
#endif
template <bool COUNT, bool PRIMARY, bool DEEP, int FUSE>
__device__ __forceinline__ void trace_compact_body(PipeArgs& A, unsigned char* smem) {
    if (!PRIMARY && A.qlist && (int)(blockIdx.x * kBlock) >= *A.qcount) return;  // whole block past the list
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long tclk0 = __builtin_amdgcn_s_memrealtime();
#endif
    LdsView L = setup_lds<true>(smem, A.S);
    int k = blockIdx.x * kBlock + threadIdx.x;
    if (PRIMARY && !COUNT && A.pcost) {  // (the counting pass: tile order)
        k = cost_order_slot<DEEP ? ORT_COST_SHIFT_DEEP : ORT_COST_SHIFT>(A.pcost, L.fr.co, k);
#if defined(__HIP_DEVICE_COMPILE__)
        // heavy priority: the few waves holding the frame's longest walks start with the first
        // workgroups but, sharing their SIMD with 7 others, finish long after the rest of a small
        // tile (tools/tile_clock.py); they get the SIMD's issue slots first
        if (A.prio_steps > 0 && __ballot((int)A.pcost[k] >= A.prio_steps)) __builtin_amdgcn_s_setprio(3);
#endif
    }
    if (!PRIMARY && !list_slot(A, k)) return;
    ort::Counters cnt;
    for (int q = 0; q < 6; ++q) cnt.v[q] = 0;
    const bool go = trace_slot<COUNT, PRIMARY, DEEP, FUSE>(A, L, k, cnt);
    (void)go;
    if constexpr (FUSE == 2) {  // the paths that go on join the next bounce's list
#if defined(__HIP_DEVICE_COMPILE__)
        typedef __attribute__((address_space(4))) const PipeArgs KernArgs;
        KernArgs* kp = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        uint32_t key = 0;
        if (go && kp->qnext_keys) {  // the state just stored
            const float4 o = kp->po[k], d = kp->pd[k];
            key = ort::path_key(o, d, kp->mp, kp->key_spread) |
                  (kp->geo_heavy ? geo_class_bits(kp->gbox, kp->gthr, o, d) : light_bit(kp->bcost_r, kp->heavy, k));
        }
        append_slots(go, k, key, kp->qnext, kp->qnext_keys, kp->qnext_count);
#endif
    }
    flush_counts<COUNT>(cnt, A.counters);
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    tile_clock_record<PRIMARY && !COUNT>(k, k, tclk0);
#endif
}

// Tile pairs (ORT_OPT_TILE_PAIRS): a workgroup renders the two tiles of pair blockIdx.x, each
// wave a heavy and then a light 64-slot block (cost_order_pair).  Between the blocks the kernel
// arguments are re-read through a laundered pointer (hoisted out of the loop they stay live
// across the walk and spill) and the second block's slot is kept in one VGPR.
template <bool COUNT, bool PRIMARY, bool DEEP, int FUSE>
__device__ __forceinline__ void trace_pair_body(PipeArgs& A, unsigned char* smem) {
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long tclk0 = __builtin_amdgcn_s_memrealtime();
#endif
    LdsView L0 = setup_lds<true>(smem, A.S);
    const int base = blockIdx.x * (2 * kBlock);
    int kk0 = base + threadIdx.x, kk1 = kk0 + kBlock;
    if (!COUNT && A.pcost) cost_order_pair<DEEP ? ORT_COST_SHIFT_DEEP : ORT_COST_SHIFT>(A.pcost, L0.fr.co, base, kk0, kk1);
    ort::Counters cnt;
    for (int q = 0; q < 6; ++q) cnt.v[q] = 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#if defined(__HIP_DEVICE_COMPILE__)
        typedef __attribute__((address_space(4))) const PipeArgs KernArgs;
        KernArgs* kp = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
        asm volatile("" : "+s"(kp));
        PipeArgs A1 = *kp;
#else
        PipeArgs& A1 = A;
#endif
        LdsView L = lds_view<true>(smem, A1.S.depth);
        int k = j ? kk1 : kk0;
#if defined(__HIP_DEVICE_COMPILE__)
        asm volatile("" : "+v"(k));
        if (!COUNT && A1.pcost && A1.prio_steps > 0) {  // heavy priority, per block
            if (__ballot((int)A1.pcost[k] >= A1.prio_steps)) __builtin_amdgcn_s_setprio(3);
            else __builtin_amdgcn_s_setprio(0);
        }
#endif
        const bool go = trace_slot<COUNT, PRIMARY, DEEP, FUSE, 2>(A1, L, k, cnt);
        (void)go;
        if constexpr (FUSE == 2) {  // the paths that go on join the next bounce's list
#if defined(__HIP_DEVICE_COMPILE__)
            KernArgs* kq = (KernArgs*)__builtin_amdgcn_kernarg_segment_ptr();
            uint32_t key = 0;
            if (go && kq->qnext_keys) {
                const float4 o = kq->po[k], d = kq->pd[k];
                key = ort::path_key(o, d, kq->mp, kq->key_spread) |
                      (kq->geo_heavy ? geo_class_bits(kq->gbox, kq->gthr, o, d) : light_bit(kq->bcost_r, kq->heavy, k));
            }
            append_slots(go, k, key, kq->qnext, kq->qnext_keys, kq->qnext_count);
#endif
        }
    }
    flush_counts<COUNT>(cnt, A.counters);
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    tile_clock_record<PRIMARY && !COUNT>(kk0, kk1, tclk0);
#endif
}

// FUSE: 1 sample, 1 bounce -- the kernel also shades (shade_direct), no hit records.
template <bool COUNT, bool PRIMARY, int FUSE>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ORT_TRACE_WAVES))) ort_trace_compact(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    trace_compact_body<COUNT, PRIMARY, false, FUSE>(A, smem);
}
template <bool COUNT, bool PRIMARY, int FUSE>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ORT_TRACE_WAVES_DEEP)))
ort_trace_compact_deep(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    trace_compact_body<COUNT, PRIMARY, true, FUSE>(A, smem);
}
// camera rays, tile pairs (ORT_OPT_TILE_PAIRS)
template <bool COUNT, int FUSE>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ORT_TRACE_WAVES))) ort_trace_pair(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    trace_pair_body<COUNT, true, false, FUSE>(A, smem);
}
template <bool COUNT, int FUSE>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ORT_TRACE_WAVES_DEEP)))
ort_trace_pair_deep(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    trace_pair_body<COUNT, true, true, FUSE>(A, smem);
}
// Heavy camera rays (ORT_OPT_SPLIT_HEAVY): the slots whose walk took >= T steps in the previous
// frame (pcost), listed (the first `cap` of them) and marked in a bitmap the per-tile kernel
// reads.  A wave's slots are listed in slot order after one atomic.
// One wave scans 1024 slots from `base` (a multiple of 1024; n a multiple of 256): 16 per lane,
// read as two 16-byte loads, one atomic per wave, each lane pair writing one bitmap word.
struct HeavyScan {
    const uint16_t* pcost;
    int n, T, cap;
    uint32_t* bits;
    int* list;
    int* count;
};
__device__ inline void heavy_scan_wave(const HeavyScan& H, int base) {
    const int lane = threadIdx.x & 63;
    const int s0 = base + 16 * lane;
    uint32_t m = 0;
    if (s0 < H.n) {
        const uint4 a = *(const uint4*)(H.pcost + s0), b = *(const uint4*)(H.pcost + s0 + 8);
        const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
        for (int i = 0; i < 8; ++i) {
            m |= (uint32_t)((int)(w[i] & 0xffffu) >= H.T) << (2 * i);
            m |= (uint32_t)((int)(w[i] >> 16) >= H.T) << (2 * i + 1);
        }
    }
    const int c = __popc(m);
    int incl = c;  // inclusive scan of the lanes' counts
    for (int off = 1; off < 64; off <<= 1) {
        const int v = __shfl_up(incl, off);
        if (lane >= off) incl += v;
    }
    const int total = __shfl(incl, 63);
    int at = 0;
    if (lane == 0 && total) at = atomicAdd(H.count, total);
    int pos = __shfl(at, 0) + incl - c;
    uint32_t mh = 0;  // the listed ones (past the cap the per-tile kernel walks them itself)
    for (uint32_t r = m; r; r &= r - 1, ++pos) {
        const int i = __builtin_ctz(r);
        if (pos < H.cap) {
            H.list[pos] = s0 + i;
            mh |= 1u << i;
        }
    }
    const uint32_t other = (uint32_t)__shfl_xor((int)mh, 1);
    if (s0 < H.n && !(lane & 1)) H.bits[s0 >> 5] = mh | (other << 16);
}
__global__ void __launch_bounds__(kBlock) k_heavy_scan(HeavyScan H) {
    for (int base = (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 1024; base < H.n;
         base += (int)(gridDim.x * (kBlock / 64)) * 1024)
        heavy_scan_wave(H, base);
}

// The heavy camera rays of k_heavy_scan's list, each walked by a group of 8 lanes that deal its
// walk's level-split_level subtrees round robin (traverse_split), then shaded like the per-tile
// kernel shades (FUSE 1: shade_direct).  Runs on the context's second stream beside the per-tile
// kernel and ahead of it in the GPU's dispatch, at raised issue priority: the frame's longest
// walks, run by one lane each, are what a small tile's frame waits for (tools/tile_clock.py).
constexpr int kSplitLanes = 8;
template <bool DEEP, int FUSE>
__global__ void __launch_bounds__(kBlock) ort_trace_split(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
#if defined(__HIP_DEVICE_COMPILE__)
    __builtin_amdgcn_s_setprio(3);
#endif
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    const unsigned long long sclk0 = __builtin_amdgcn_s_memrealtime();
    int sitems = 0;
#endif
    if (A.hsync_next && blockIdx.x == 0 && threadIdx.x < 2) A.hsync_next[threadIdx.x] = 0;
    const int count = min(A.hsync[0], A.hcap);
    if (count == 0) return;
    LdsView L = setup_lds<true>(smem, A.S);
    using Masks = typename std::conditional<DEEP, ort::Masks96Split, ort::Masks64Split>::type;
    const int lane = threadIdx.x & 63, g = lane / kSplitLanes, j = lane % kSplitLanes;
    constexpr int kNoHit = 0x7fffffff;
    for (;;) {
        int base = 0;
        if (lane == 0) base = atomicAdd(A.hsync + 1, 64 / kSplitLanes);
        base = __shfl(base, 0);
        if (base >= count) break;
        const int idx = base + g;
        const int k = idx < count ? A.hlist[idx] : -1;
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
        sitems += min(64 / kSplitLanes, count - base);
#endif
        int pos = kNoHit, entry = -1, steps = 0, own = 0;
        float t = 0.0f;
        bool walked = false;
        ort_rng rng0;
        ort::Ray ray;
        ray.o = ray.d = ort::mk(0.0f, 0.0f, 0.0f);
        if (k >= 0) {
            bool alive;
            ray = slot_ray<true>(A, k, alive, &rng0);
            const ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
            if (alive && !A.exact_only && ort::fast_path_ok(ray, inv, 0.001f, ORT_MAXFLOAT)) {
                walked = true;
                ort::traverse_split<Masks>(A.S, L.planes, L.lut, ray, inv, A.split_level, kSplitLanes, j, pos, entry, t,
                                           L.fr, steps, own);
            } else if (alive && j == 0) {  // (a moved camera: rare) the exact kernel walks and shades it
                A.defer_list[atomicAdd(A.sync, 1)] = k;
                if (A.pcost) A.pcost[k] = 0;
            }
        }
        // the group's result: the hit with the lowest DFS position; the walk's steps as ONE walk
        // would take them (the next frame's cost order and heavy list read them): the longest
        // stretch above the level plus every lane's own subtree steps
        steps -= own;
        for (int o = 1; o < kSplitLanes; o <<= 1) {
            const int op = __shfl_xor(pos, o, kSplitLanes);
            const int oe = __shfl_xor(entry, o, kSplitLanes);
            const float ot = __shfl_xor(t, o, kSplitLanes);
            if (op < pos) {
                pos = op;
                entry = oe;
                t = ot;
            }
            steps = max(steps, __shfl_xor(steps, o, kSplitLanes));
            own += __shfl_xor(own, o, kSplitLanes);
        }
        steps += own;
        if (walked && j == 0) {
            if (A.pcost) A.pcost[k] = (uint16_t)min(steps, 65535);
            if constexpr (FUSE == 1) {
                shade_direct(A, k, ray, rng0, pos != kNoHit, entry, t);
            } else {  // bounce 0 of a multi-bounce frame: path state, and the next bounce's list
                int col, row;
                (void)slot_coords(A, k, col, row);
                if (shade_state<0, true, false>(A, k, (size_t)row * A.tm.tw + col, ray, rng0, pos != kNoHit ? entry : -1, t)) {
                    const int q = atomicAdd(A.qnext_count, 1);
                    A.qnext[q] = k;
                    if (A.qnext_keys)
                        A.qnext_keys[q] = path_key_class(A, k);
                }
            }
        }
    }
#if ORT_TILE_CLOCK && defined(__HIP_DEVICE_COMPILE__)
    {   // analysis: per wave {start, end, 1 << 63 (a split-kernel record), rays walked}, from the records' end
        const int gw = (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
        if (A.wclock && (threadIdx.x & 63) == 0 && gw < A.wclock_n)
            A.wclock[A.wclock_n - 1 - gw] =
                make_ulonglong4(sclk0, __builtin_amdgcn_s_memrealtime(), 1ull << 63, (unsigned long long)sitems);
    }
#endif
}

// One-ray-per-lane trace for the explicit layout (MODE 1) and brute force (MODE 2).
template <int MODE, bool COUNT, bool PRIMARY>
__global__ void __launch_bounds__(kBlock) ort_trace_kernel(PipeArgs A) {
    int k = blockIdx.x * kBlock + threadIdx.x;
    if (!PRIMARY && !list_slot(A, k)) return;
    bool alive;
    const ort::Ray ray = slot_ray<PRIMARY>(A, k, alive);
    if (!alive) return;
    ort::Counters cnt;
    for (int q = 0; q < 6; ++q) cnt.v[q] = 0;
    ort::LocalFrames unused;
    float t;
    int entry;
    int st;
    if constexpr (MODE == 1) {
        int snode[ORT_MAX_STACK];
        float stmin[ORT_MAX_STACK];
        st = ort::trace_ray<MODE, COUNT>(A.S, nullptr, nullptr, ray, false, t, entry, unused, snode, stmin, cnt);
    } else {
        st = ort::trace_ray<MODE, COUNT>(A.S, nullptr, nullptr, ray, false, t, entry, unused, nullptr, nullptr, cnt);
    }
    A.hit[k] = make_int2(st == ORT_TRACE_HIT ? entry : -1, __float_as_int(t));
    flush_counts<COUNT>(cnt, A.counters);
}

// Exact compact walk (traverse_compact) for the deferred rays; grid-stride loop.
template <bool COUNT, bool PRIMARY, int FUSE>
__global__ void __launch_bounds__(kBlock) ort_trace_exact(PipeArgs A) {
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    const int n = *A.sync;
    // the next launch's counters (the other set: its last users ended before this launch began),
    // instead of a memset node per launch (a fill kernel: ~5 us of a 0.33 ms band frame)
    if (A.sync_next && blockIdx.x == 0 && threadIdx.x < 16) A.sync_next[threadIdx.x] = 0;
    if (A.scan_pcost) {  // the next frame's heavy list from this frame's final steps (split frames)
        const HeavyScan H{A.scan_pcost, (int)A.total, A.scan_T, A.hcap, A.scan_bits, A.scan_list, A.scan_count};
        for (int base = (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6)) * 1024; base < H.n;
             base += (int)(gridDim.x * (kBlock / 64)) * 1024)
            heavy_scan_wave(H, base);
    }
    if ((int)(blockIdx.x * kBlock) >= n) return;  // usually no deferred ray at all: skip the LDS image copy
    LdsView L = setup_lds<false>(smem, A.S);
    ort::Counters cnt;
    for (int q = 0; q < 6; ++q) cnt.v[q] = 0;
    for (int i = blockIdx.x * kBlock + threadIdx.x; i < n; i += gridDim.x * kBlock) {
        const int k = A.defer_list[i];
        bool alive;
        ort_rng rng;
        const ort::Ray ray = slot_ray<PRIMARY>(A, k, alive, FUSE ? &rng : nullptr);
        float t;
        int entry;
        const int st = ort::trace_ray<0, COUNT>(A.S, L.planes, nullptr, ray, false, t, entry, L.fr, nullptr, nullptr, cnt);
        if (FUSE == 1) {
            shade_direct(A, k, ray, rng, st == ORT_TRACE_HIT, entry, t);
        } else if (FUSE == 2) {  // bounce 0 shaded here; the rare deferred path joins the list alone
            int col, row;
            (void)slot_coords(A, k, col, row);
            if (shade_state<0, true, false>(A, k, (size_t)row * A.tm.tw + col, ray, rng, st == ORT_TRACE_HIT ? entry : -1, t)) {
                const int pos = atomicAdd(A.qnext_count, 1);
                A.qnext[pos] = k;
                if (A.qnext_keys)
                    A.qnext_keys[pos] = path_key_class(A, k);
            }
        } else {
            A.hit[k] = make_int2(st == ORT_TRACE_HIT ? entry : -1, __float_as_int(t));
        }
    }
    flush_counts<COUNT>(cnt, A.counters);
}

// Bounce shading (glsl:607-627) of path slot k.  FIRST: bounce 0 (c = 1, importance = 1).
// DIRECT (1 sample, 1 bounce): writes the final pixel.  Returns true when the path goes on
// to the next bounce.
template <int MODE, bool FIRST, bool DIRECT>
__device__ __forceinline__ bool shade_slot(const PipeArgs& A, int k) {
    int col, row;
    const bool in_tile = FIRST ? slot_coords<true>(A, k, col, row) : slot_coords(A, k, col, row);
    const int y = in_tile ? tile_row_to_y(A.tm, row) : 0;
    const size_t p = (size_t)row * A.tm.tw + col;
    if (!in_tile || y >= A.pp.H) {
        if (DIRECT && in_tile) {
            float* o = A.out + 3 * p;
            o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
        }
        if (FIRST && !DIRECT) A.pd[k] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);  // never alive (compaction)
        return false;
    }
    bool alive = true;
    ort::Ray ray;
    ort_rng st;
    if (FIRST) {
        if (A.sample == 0) {
            ort::pixel_rng_init(A.pp, A.tm.x0 + col, y, st);
        } else {
            const float2 v = A.prng[k];
            st.x = v.x;
            st.y = v.y;
        }
        ray = ort::primary_ray(A.pp, A.tm.x0 + col, y, A.sample, st);
    } else {
        ray = load_ray(A, k, alive);
        if (!alive) return false;
        const float2 r2 = A.prng[k];
        st.x = r2.x;
        st.y = r2.y;
    }
    int2 h = make_int2(-1, 0);
    if (!A.nobounce) h = A.hit[k];
    return shade_state<MODE, FIRST, DIRECT>(A, k, p, ray, st, h.x, __int_as_float(h.y));
}


// Shades every path slot of its workgroup (slot order); with A.qnext, the paths that go on
// are appended to the next bounce's list (the compaction, without a separate select pass).
template <int MODE, bool FIRST, bool DIRECT>
__global__ void __launch_bounds__(kBlock) ort_shade_kernel(PipeArgs A) {
    int k = blockIdx.x * kBlock + threadIdx.x;
    bool in = true;
    if (!FIRST && A.qlist) {  // the bounce's alive paths in append order (not the sorted trace list)
        const int n = *A.qcount;
        if ((int)(blockIdx.x * kBlock) >= n) return;  // whole workgroup past the list
        in = k < n;
        if (in) k = A.qlist[k];
    }
    const bool go = in && shade_slot<MODE, FIRST, DIRECT>(A, k);
    if (!DIRECT && A.qnext) {
        uint32_t key = 0;
        if (go && A.qnext_keys)  // the state just stored
            key = path_key_class(A, k);
        append_slots(go, k, key, A.qnext, A.qnext_keys, A.qnext_count);
    }
}

// col / ns, gamma (glsl:659-661) for the multi-sample / multi-bounce case.
__global__ void __launch_bounds__(kBlock) ort_finalize_kernel(PipeArgs A) {
    const int k = blockIdx.x * kBlock + threadIdx.x;
    int col, row;
    if (!slot_coords<true>(A, k, col, row)) return;
    const int y = tile_row_to_y(A.tm, row);
    float* o = A.out + 3 * ((size_t)row * A.tm.tw + col);
    if (y >= A.pp.H) {
        o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
        return;
    }
    ort::V3 acc = ort::mk(0.0f, 0.0f, 0.0f);
    if (A.pp.ns > 0) {
        const float4 a = A.pcol[k];
        acc = ort::mk(a.x, a.y, a.z);
    }
    const ort::V3 v = ort::finish_pixel(acc, A.pp.ns);
    o[0] = v.x; o[1] = v.y; o[2] = v.z;
}

// ---------------------------------------------------------------------------------------
// Whole-pixel paths (ORT_OPT_PIXEL_PATHS): main() of the fragment shader (glsl:636-664) for
// every pixel in ONE launch -- all samples, all bounces -- instead of the wavefront pipeline's
// per-sample, per-bounce launches (trace, exact walk, shade, list sort: ~10 launches per bounce).
// Samples cannot be batched across launches: the RNG state runs on from one sample to the next
// (randState, glsl:640), so a pixel's samples are a sequential chain.  Each lane therefore owns
// a pixel and steps it one bounce at a time, regenerating the path when it ends (the pixel's
// next sample starts in the same iteration: lanes stay on the walk code whatever sample or
// bounce they are at), and a lane whose pixel is done takes the next pixel of its wave's chunk
// (persistent grid, one atomic per 64-pixel chunk, pixels in the tile-block order of the path
// slots: a chunk is an 8x8 block).  Every pixel runs exactly shade_pixel's chain (render_core.h),
// so the frames are the pipeline's bit for bit.  MODE 0: compact octree (DEEP: depth 9-10, the
// camera walk's 96-bit masks over the forward tables; else the bounce walk's Masks64Plain), the
// exact walk inline for the rays the fast walk cannot take; MODE 2: brute force.
// The grid's work cursor and done count (A.sync[1], [2]) start at zero (the counter set of the
// launch) and the last workgroup to finish resets them.
template <int MODE, bool DEEP, bool LDS>
__device__ __forceinline__ bool pixel_trace(const PipeArgs& A, const ort::KScene& S, LdsView& L, const ort::Ray& r,
                                            float& t, int& entry) {
    ort::Counters cnt;  // (not counted: counting renders take the pipeline)
    entry = -1;
    t = 0.0f;
    if (MODE == 2) return ort::traverse_brute<false>(S, r, 0.001f, ORT_MAXFLOAT, entry, t, cnt);
    ort::V3 inv = ort::mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    if (!A.exact_only && ort::fast_prepare(S, r, inv)) {
        using Masks = typename std::conditional<DEEP, ort::Masks96,
                                                typename std::conditional<LDS, ort::Masks64PlainLds, ort::Masks64Plain>::type>::type;
        return ort::traverse_fast_t<false, Masks>(S, L.planes, L.lut, r, inv, 0.001f, ORT_MAXFLOAT, entry, t, L.fr, cnt);
    }
    return ort::traverse_compact<false>(S, L.planes, r, 0.001f, ORT_MAXFLOAT, entry, t, L.fr, cnt);
}

#ifndef ORT_PIXEL_LPT
#define ORT_PIXEL_LPT 1  // whole-pixel paths take last frame's heaviest 8x8 blocks first
#endif
constexpr int kPixelClasses = 32;  // cost classes of a block: mean bounces per sample in quarters
// Accounts one slot of a block (a finished pixel and the bounces it traced, or a slot that is no
// pixel): the block's last slot files the block under its cost class for the next frame and
// clears its accumulator (cost in the high word, slots in the low word).
__device__ __forceinline__ void block_account(const PipeArgs& A, int slot, int bounces) {
    unsigned long long* acc = A.pl_cost + (slot >> 6);
    const unsigned long long add = ((unsigned long long)min(bounces, 1 << 24) << 32) | 1ull;
    const unsigned long long old = atomicAdd(acc, add);
    if ((unsigned)(old & 0xffffffffu) == 63u) {
        const unsigned long long cost = (old >> 32) + (unsigned long long)min(bounces, 1 << 24);
        *acc = 0;
        const unsigned long long quarters = cost / (16ull * (unsigned long long)A.pp.ns);
        const int q = kPixelClasses - 1 - (int)min(quarters, (unsigned long long)(kPixelClasses - 1));
        const int pos = atomicAdd(A.pl_wcnt + q, 1);
        A.pl_w[(size_t)q * A.pl_stride + pos] = slot >> 6;
    }
}

#ifndef ORT_PIXEL_WAVES
#define ORT_PIXEL_WAVES 4
#endif


// LDS: small scenes (depth <= 8) walk the workgroup's copies of nk[] and leaf_sph[] in LDS
// (ds_read, ~50 cycles) instead of global memory: the kernel waits on memory for most of its
// cycles (SQ_WAIT_ANY 0.64 at config.h's default scene, profiles/r06/), and a walk is a chain
// of dependent record loads.
// SPEC: samples in parallel.  A pixel's samples form a chain only through the RNG state, and
// the state a sample ends with depends on the path only through how many draws it took -- so
// with a static or slowly moving camera it repeats from frame to frame.  SPEC launches take
// (8x8 block, sample s) items: sample s >= 1 starts from the state sample s-1 ended with LAST
// frame (sp_prev), writes its radiance and end state, and flags the pixel when its end state
// differs from last frame's -- the samples after it then started from a wrong state.
// ort_sample_resolve sums each pixel's samples in order up to the first flagged one and lists
// the pixels that need the rest; a whole-pixel launch over that list (fx_*) continues them
// from the true state.  Every pixel's samples are thus the sequential chain's, summed in the
// chain's order: the frames stay bit-identical, and a frame is no longer as long as its longest
// pixel's chain (16 samples x 8 bounces at config.h's default).
// PM: 0 whole pixels, 1 SPEC samples, 2 whole pixels that record their samples' end states or
// run the fixup list (kept apart from 0: its registers are the ones-sample frames' too)
template <int MODE, bool DEEP, bool LDS, int PM = 0>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(ORT_PIXEL_WAVES)))
ort_pixel_paths(PipeArgs A) {
    constexpr bool SPEC = PM == 1;
    // a SPEC launch in a fall-back frame, and the fixup launch's workgroups beyond what its list
    // needs, only count themselves out (before any LDS set-up)
    const bool idle_wg = (SPEC && A.sp_ctl[2] == 0) ||
                         (PM == 2 && A.fx_slot && (long long)blockIdx.x * kBlock >= (long long)*A.fx_n + kBlock);
    if (idle_wg) {
        if (threadIdx.x == 0 && atomicAdd(A.sync + 2, 1) == (int)gridDim.x - 1) {
            atomicExch(A.sync + 1, 0);
            atomicExch(A.sync + 2, 0);
            if (PM == 2 && A.fx_slot) {
                if (A.sp_ctl[2]) atomicExch(A.sp_ctl + 1, *A.fx_n);  // speculated: the list = the moved pixels
                atomicExch(A.fx_n, 0);
            }
        }
        return;
    }
    extern __shared__ __attribute__((aligned(1024))) unsigned char smem[];  // plane tables: 1 KiB-aligned
    LdsView L{};
    ort::KScene S = A.S;
    if (LDS) {  // before setup_lds's barrier
        uint4* dn = reinterpret_cast<uint4*>(smem + A.lds_nk_off);
        uint4* ds = reinterpret_cast<uint4*>(smem + A.lds_sph_off);
        const uint4* sl = reinterpret_cast<const uint4*>(A.S.leaf_sph);
        for (int i = threadIdx.x; i < A.lds_nk_n16; i += kBlock) dn[i] = A.S.nk[i];
        for (int i = threadIdx.x; i < A.lds_sph_n16; i += kBlock) ds[i] = sl[i];
        S.lds_nk = (uint32_t)(size_t)(const __attribute__((address_space(3))) unsigned char*)(smem + A.lds_nk_off);
        S.lds_sph = (uint32_t)(size_t)(const __attribute__((address_space(3))) unsigned char*)(smem + A.lds_sph_off);
    }
    if (MODE == 0) L = setup_lds<true>(smem, A.S);
    const int lane = threadIdx.x & 63;
    const unsigned long long below = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
    const int maxd = A.pp.maxDepth, ns = A.pp.ns;
    // the work items: 8x8 blocks, last frame's heaviest class first (a longest-first list
    // schedule: a frame ends with its longest pixels -- a pixel's samples run one after another --
    // and a block keeps its pixels' rays coherent), else in tile order; SPEC: (block, sample)
    // pairs, a block's samples one after another; the fixup list: 64 of its entries at a time.
    // Lane q < 32 holds the inclusive prefix of the class counts.
    const bool fixup = PM == 2 && A.fx_slot;
    const int n_blocks = A.total >> 6;
    const int n_items = SPEC ? n_blocks * A.sp_nch : (fixup ? (*A.fx_n + 63) >> 6 : n_blocks);
    int cls_end = 0;
    if (ORT_PIXEL_LPT && A.pl_r) {
        cls_end = lane < kPixelClasses ? A.pl_rcnt[lane] : 0;
        for (int d = 1; d < kPixelClasses; d <<= 1) {
            const int v = __shfl_up(cls_end, d);
            if (lane >= d) cls_end += v;
        }
    }
    const bool listed = ORT_PIXEL_LPT && !fixup && A.pl_r && __shfl(cls_end, kPixelClasses - 1) == n_blocks;
    int k = -1;              // the lane's path slot (pixel), -1 idle
    int nb = 0;              // bounces traced for the lane's pixel so far (its cost class)
    int px = 0, py = 0, s = 0, b = 0;
    ort::Ray ray;
    ray.o = ray.d = ort::mk(0.0f, 0.0f, 0.0f);
    ort::V3 c = ort::mk(1.0f, 1.0f, 1.0f), col = ort::mk(0.0f, 0.0f, 0.0f);
    float importance = 1.0f;
    ort_rng st;
    st.x = st.y = 0.0f;
    int next = 0, end = 0;   // wave-uniform: the rest of the wave's block (or fixup entries)
    int item_s = 0;          // wave-uniform, SPEC: the sample of those slots
    bool drained = false;    // wave-uniform: the cursor passed the last item
#if ORT_PIXEL_CLOCK  // analysis: per wave the cycles of the refill, the walk and the shading, and the walk's lanes
    unsigned long long ck_refill = 0, ck_trace = 0, ck_shade = 0, ck_iter = 0, ck_lanes = 0, ck_t = 0;
    const unsigned long long ck_rt0 = __builtin_amdgcn_s_memrealtime();
#define ORT_CK_MARK(acc)                                            \
    do {                                                            \
        const unsigned long long now = __builtin_amdgcn_s_memtime(); \
        acc += now - ck_t;                                          \
        ck_t = now;                                                 \
    } while (0)
#else
#define ORT_CK_MARK(acc) do { } while (0)
#endif
    for (;;) {
#if ORT_PIXEL_CLOCK
        ck_t = __builtin_amdgcn_s_memtime();
#endif
        const unsigned long long idle = __ballot(k < 0);
        if (idle && !drained) {  // refill: idle lanes take the item's next pixels
            if (next == end) {  // the next item
                int j = 0;
                if (lane == 0) j = atomicAdd(A.sync + 1, 1);
                j = __shfl(j, 0);
                if (j >= n_items) {
                    drained = true;
                } else if (fixup) {
                    next = j << 6;
                    end = min(next + 64, *A.fx_n);
                } else {  // SPEC: block j / nch (its pixels' chunk j % nch), heavy blocks first as well
                    const int jb = SPEC ? j / A.sp_nch : j;
                    int blk = jb;
                    if (listed) {  // item jb of the class lists: class q = the first with jb < its prefix end
                        const unsigned long long in = __ballot(lane < kPixelClasses && jb < cls_end);
                        const int q = __builtin_ctzll(in);
                        const int before = q ? __shfl(cls_end, q - 1) : 0;
                        blk = A.pl_r[(size_t)q * A.pl_stride + (jb - before)];
                    }
                    next = blk << 6;
                    end = next + 64;
                    if (SPEC) item_s = j - jb * A.sp_nch;
                }
            }
            if (!drained) {
                const int n_idle = __popcll(idle);
                const int take = min(n_idle, end - next);
                if (k < 0) {
                    const int rank = __popcll(idle & below);
                    if (rank < take) {
                        const int cand = fixup ? A.fx_slot[next + rank] : next + rank;
                        bool pixel = false;
                        int cx, cy;
                        if (slot_coords(A, cand, cx, cy)) {
                            const int y = tile_row_to_y(A.tm, cy);
                            if (y < A.pp.H) {  // a pixel: its first sample's camera ray
                                k = cand;
                                nb = 0;
                                px = A.tm.x0 + cx;
                                py = y;
                                b = 0;
                                c = ort::mk(1.0f, 1.0f, 1.0f);
                                importance = 1.0f;
                                if (SPEC) {  // chunk item_s from last frame's end state of chunk item_s - 1
                                    s = item_s * A.sp_chunk;
                                    if (item_s == 0) {
                                        ort::pixel_rng_init(A.pp, px, py, st);
                                    } else {
                                        const float2 v = A.sp_prev[(size_t)(item_s - 1) * A.total + k];
                                        st.x = v.x;
                                        st.y = v.y;
                                    }
                                } else if (fixup) {  // the rest of the pixel's chain from its true state
                                    const int e = next + rank;
                                    s = A.fx_s0[e];
                                    const float2 v = A.fx_st[e];
                                    st.x = v.x;
                                    st.y = v.y;
                                    col = ort::mk(A.fx_col[e], A.fx_col[(size_t)A.total + e], A.fx_col[2 * (size_t)A.total + e]);
                                } else {
                                    ort::pixel_rng_init(A.pp, px, py, st);
                                    s = 0;
                                    col = ort::mk(0.0f, 0.0f, 0.0f);
                                }
                                ray = ort::primary_ray(A.pp, px, py, s, st);
                                pixel = true;
                            } else if (!SPEC) {  // a band's padding row (past the frame): zeros, as the pipeline writes
                                float* o = A.out + 3 * ((size_t)cy * A.tm.tw + cx);
                                o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
                            }
                        }
                        if (ORT_PIXEL_LPT && !SPEC && A.pl_w && !pixel) block_account(A, cand, 0);
                    }
                }
                next += take;
            }
        }
        ORT_CK_MARK(ck_refill);
        if (!__ballot(k >= 0)) {
            if (drained) break;
            continue;
        }
#if ORT_PIXEL_CLOCK
        ck_iter += 1;
        ck_lanes += __popcll(__ballot(k >= 0));
#endif
        if (k >= 0) {  // one bounce of the lane's current path (radiance(), glsl:604-627)
            float t;
            int entry;
            const bool hit = pixel_trace<MODE, DEEP, LDS>(A, S, L, ray, t, entry);
#if ORT_PIXEL_CLOCK
            __builtin_amdgcn_wave_barrier();
#endif
            ORT_CK_MARK(ck_trace);
            ort::HitRec h;
            if (hit) h = ort::hit_record<MODE>(A.S, ray, t, entry);
            bool ended = ort::shade_bounce(hit, h, ray, c, importance, st);
            ++b;
            ++nb;
            ended = ended || b >= maxd || importance < 0.01f;
            if (ended && SPEC) {  // the sample's radiance; the chunk's next sample, or its end state
                const size_t i = (size_t)s * A.total + k;
                A.sp_col[i] = c.x;
                A.sp_col[(size_t)ns * A.total + i] = c.y;
                A.sp_col[2 * (size_t)ns * A.total + i] = c.z;
                if (++s < ns && s % A.sp_chunk != 0) {
                    b = 0;
                    c = ort::mk(1.0f, 1.0f, 1.0f);
                    importance = 1.0f;
                    ray = ort::primary_ray(A.pp, px, py, s, st);
                } else {
                    A.sp_cur[(size_t)((s - 1) / A.sp_chunk) * A.total + k] = make_float2(st.x, st.y);
                    k = -1;
                }
            } else if (ended) {  // col += radiance(r) (glsl:655); the pixel's next sample, or its final colour
                col = ort::add(col, c);
                if (PM == 2 && A.sp_cur && ((s + 1) % A.sp_chunk == 0 || s + 1 == ns))  // a chunk's end state, for SPEC
                    A.sp_cur[(size_t)(s / A.sp_chunk) * A.total + k] = make_float2(st.x, st.y);
                if (++s < ns) {
                    b = 0;
                    c = ort::mk(1.0f, 1.0f, 1.0f);
                    importance = 1.0f;
                    ray = ort::primary_ray(A.pp, px, py, s, st);
                } else {
                    int cx, cy;
                    (void)slot_coords(A, k, cx, cy);
                    const ort::V3 v = ort::finish_pixel(col, ns);
                    float* o = A.out + 3 * ((size_t)cy * A.tm.tw + cx);
                    o[0] = v.x; o[1] = v.y; o[2] = v.z;
                    if (ORT_PIXEL_LPT && A.pl_w) block_account(A, k, nb);  // its block's cost for the next frame
                    k = -1;
                }
            }
        }
        ORT_CK_MARK(ck_shade);
    }
#if ORT_PIXEL_CLOCK
    {
        const int gw = (int)(blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6));
        if (A.wclock && lane == 0 && !fixup && 2 * gw + 1 < A.wclock_n) {  // (the fixup launch keeps none)
            A.wclock[2 * gw] = make_ulonglong4(ck_refill, ck_trace, ck_shade, ck_iter);
            A.wclock[2 * gw + 1] = make_ulonglong4(ck_lanes, ck_rt0, __builtin_amdgcn_s_memrealtime(), 1ull);
        }
    }
#endif
#undef ORT_CK_MARK
    // the last workgroup out resets the cursor and the done count for the next launch (and the
    // fixup list's length, read by every wave at its start)
    __syncthreads();
    if (threadIdx.x == 0) {
        __threadfence();
        if (atomicAdd(A.sync + 2, 1) == (int)gridDim.x - 1) {
            atomicExch(A.sync + 1, 0);
            atomicExch(A.sync + 2, 0);
            if (fixup) {
                if (A.sp_ctl[2]) atomicExch(A.sp_ctl + 1, *A.fx_n);  // speculated: the list = the moved pixels
                atomicExch(A.fx_n, 0);
            }
            // the class counts read this frame become the next frame's write counts
            if (ORT_PIXEL_LPT && A.pl_rcnt && !SPEC)  // (SPEC frames read the lists, and keep them)
                for (int q = 0; q < kPixelClasses; ++q) atomicExch(A.pl_rcnt + q, 0);
        }
    }
}

// SPEC frames: per slot, the pixel's samples summed in order up to the end of the first chunk
// whose end state differs from last frame's (all of them when none does: every chunk started
// from its true state) -> the final pixel, or an entry of the fixup list (the pixel's next
// sample, its true start state, the sum so far).  Padding rows: zeros.
__global__ void __launch_bounds__(256) ort_sample_resolve(PipeArgs A) {
    const int k = (int)(blockIdx.x * 256 + threadIdx.x);
    if (k >= A.total) return;
    int cx, cy;
    if (!slot_coords(A, k, cx, cy)) return;
    float* o = A.out + 3 * ((size_t)cy * A.tm.tw + cx);
    if (tile_row_to_y(A.tm, cy) >= A.pp.H) {
        o[0] = 0.0f; o[1] = 0.0f; o[2] = 0.0f;
        return;
    }
    const int ns = A.pp.ns;
    if (A.sp_ctl[2] == 0) {  // a fall-back frame: the whole chain from sample 0
        ort_rng st;
        ort::pixel_rng_init(A.pp, A.tm.x0 + cx, tile_row_to_y(A.tm, cy), st);
        const int e = atomicAdd(A.fx_n, 1);
        A.fx_slot[e] = k;
        A.fx_s0[e] = 0;
        A.fx_st[e] = make_float2(st.x, st.y);
        A.fx_col[e] = 0.0f;
        A.fx_col[(size_t)A.total + e] = 0.0f;
        A.fx_col[2 * (size_t)A.total + e] = 0.0f;
        return;
    }
    int bad = A.sp_nch - 1;  // the first chunk whose end state moved (the last: none did)
    for (int c = 0; c < A.sp_nch - 1; ++c) {
        const size_t i = (size_t)c * A.total + k;
        const float2 u = A.sp_cur[i], v = A.sp_prev[i];
        if (__float_as_uint(u.x) != __float_as_uint(v.x) || __float_as_uint(u.y) != __float_as_uint(v.y)) {
            bad = c;
            break;
        }
    }
    const int last = min((bad + 1) * A.sp_chunk, ns) - 1;  // samples 0..last are the chain's
    const size_t plane = (size_t)ns * A.total;
    ort::V3 col = ort::mk(0.0f, 0.0f, 0.0f);
    for (int s = 0; s <= last; ++s) {
        const size_t i = (size_t)s * A.total + k;
        col = ort::add(col, ort::mk(A.sp_col[i], A.sp_col[plane + i], A.sp_col[2 * plane + i]));
    }
    if (last == ns - 1) {
        const ort::V3 v = ort::finish_pixel(col, ns);
        o[0] = v.x; o[1] = v.y; o[2] = v.z;
        return;
    }
    const int e = atomicAdd(A.fx_n, 1);
    A.fx_slot[e] = k;
    A.fx_s0[e] = last + 1;
    A.fx_st[e] = A.sp_cur[(size_t)bad * A.total + k];
    A.fx_col[e] = col.x;
    A.fx_col[(size_t)A.total + e] = col.y;
    A.fx_col[2 * (size_t)A.total + e] = col.z;
}

// The mode of a frame whose states last frame recorded: speculate while at most 1/kSpecMovedMax
// of the pixels moved last frame (sp_ctl[1]), else fall back; a fall-back frame recounts them.
__global__ void ort_sample_decide(int* ctl, long long pixels, long long moved_max) {
    if (threadIdx.x == 0) {
        const int spec = (long long)ctl[1] * moved_max <= pixels;
        ctl[2] = spec;
        if (!spec) ctl[1] = 0;
    }
}

// A frame that ran the pixels' chains whole (recording their chunk end states): the pixels whose
// chunk end states differ from last frame's -- the ones a SPEC frame would have re-traced -- into
// *count (the camera or the scene moved: the next frame then does not speculate).
__global__ void __launch_bounds__(256) ort_sample_moved(PipeArgs A, int* count) {
    if (A.sp_ctl[2] != 0) return;  // a speculating frame: its fixup list counted them
    const int k = (int)(blockIdx.x * 256 + threadIdx.x);
    bool moved = false;
    int cx, cy;
    if (k < A.total && slot_coords(A, k, cx, cy) && tile_row_to_y(A.tm, cy) < A.pp.H)
        for (int c = 0; c < A.sp_nch - 1 && !moved; ++c) {
            const size_t i = (size_t)c * A.total + k;
            const float2 u = A.sp_cur[i], v = A.sp_prev[i];
            moved = __float_as_uint(u.x) != __float_as_uint(v.x) || __float_as_uint(u.y) != __float_as_uint(v.y);
        }
    const unsigned long long m = __ballot(moved);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(count, __popcll(m));
}

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

}  // namespace

#ifndef ORT_HEAVY_STEPS
#define ORT_HEAVY_STEPS 64  // ORT_OPT_HEAVY_FIRST default: classes >= 256, >= 128, >= 64 steps
#endif
// Camera-ray defaults, measured with tools/ab_stream.py: a raised issue priority
// for waves holding a >= 150-step walk (C3 1/8 band +15 %, full frame +-0); split walks of the
// >= 200-step rays on tiles of at most 2^21 pixels (C3 1/8 band +26 %, 1/4 band +21 %, 1/2 band
// -2 %, full frame -2 %) and tile pairs on the larger ones (full frame +1.2 %, 1/2 band +0.8 %;
// 1/4 band: split +21 % > pairs +16 %; 1/8 band: pairs with split -22 %).
constexpr int kHeavyPrioSteps = 150;
constexpr int kSplitAutoSteps = 200;
constexpr long long kSplitAutoPixels = 1ll << 21;
constexpr long long kPairsAutoPixels = kSplitAutoPixels + 1;
// ORT_OPT_XCD_SWIZZLE -1 (auto): raster order (0) for the per-tile kernel on tiles of at most
// this many pixels, runs (2) otherwise.  A C3 1/8 band (1 M pixels, ~2 generations of
// workgroups) at one frame in flight: 0.307 -> 0.298 ms with raster order (its heavy region
// spread over all 8 XCDs instead of runs of 16 tiles on one); a 1/4 band 0.492 vs 0.505 and
// tile pairs (frames in flight) 0.224 vs 0.242 ms the other way (profiles/r05_band_swizzle.log)
constexpr long long kRasterAutoPixels = 3ll << 19;
struct ort_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    hipEvent_t ev0_last = nullptr;  // the last frame's start: ev0, or its first trace-timing event
    static constexpr int kRing = 64;           // trace-kernel timing of the last 64 frames
    static constexpr int kSeg = 16;            // ... of their first 16 trace launches each
    hipEvent_t tr0[kRing][kSeg] = {}, tr1[kRing][kSeg] = {};  // segment 0 created up front, others lazily
    int tseg[kRing] = {};                      // trace launches timed in each frame slot
    long long frames = 0;                      // frames whose first trace kernel was timed
    bool timed = false;
    std::string err;
    int force_layout = -1;
    int exact_only = 0;
    int pixel_paths = -1;  // ORT_OPT_PIXEL_PATHS: -1 auto (use_pixel_paths), 0 off, 1 on where it applies
    int pixel_lds_scene = 1;  // ORT_OPT_PIXEL_LDS_SCENE: small scenes in LDS for whole-pixel paths
    int pixel_heavy_first = -1;  // ORT_OPT_PIXEL_HEAVY_FIRST: -1 auto (2+ samples), 0 off, 1 on
    int refill = 16;  // ORT_OPT_REFILL: C5 (64-item chunks) 16 > 12 (-0.6 %) > 8 (-1.2 %); tools/ab_stream.py
    int persistent = 2;  // ORT_OPT_PERSISTENT: 0 off, 2 bounce >= 1 traces (default)
#if ORT_ANALYSIS
    void* wclock = nullptr;  // ort_debug_wave_clock (ORT_PERSIST_CLOCK analysis builds)
    long long wclock_n = 0;
#endif
    int xcd_swizzle = -1;  // ORT_OPT_XCD_SWIZZLE: workgroup -> tile order (block_tile); -1 auto
    int kid_skip = 1;     // ORT_OPT_KID_SKIP: rejected-sphere skip of one-sphere leaf children (2: without nk)
    // ORT_OPT_SORT_PATHS: order of the alive paths between bounces.  2 (default): the list the
    // shade kernel appended, radix-sorted by the coherence key after reading its length back --
    // C5 bounce traces 33.8 -> 31.2 ms, frame 55.5 -> 54.9 ms (A/B).  1 (every slot's key sorted,
    // dead ones last) costs as much as it saves; coarser orders lose: octant only or 12-18 key
    // bits ~ slot order, octant + direction bits and 16-bit atomic buckets slower than slot
    // order, a block-local sort of 4096-entry runs (rocprim block_radix_sort) 55.4 ms.
    int sort_paths = 2;
    // The list sort without a host wait (sortListBounded): its size is a host-side bound, the
    // list's length from the same bounce of an earlier frame (read back asynchronously into
    // pinned memory: alive_host[sample * bounces + bounce]) plus a margin; a longer list goes
    // on unsorted (same pixels).  hint_sig: the frame shape the hints belong to.  The hints live
    // in one of kHintBanks banks: a new shape takes a bank that no copy is still headed for (the
    // event after the bank's last copy has completed), so a copy of the old shape's frames
    // still in flight cannot land in the new shape's hints.
    static constexpr int kHints = 64;
    static constexpr int kHintBanks = 4;
    int* alive_host = nullptr;         // kHintBanks x kHints
    int hint_bank = 0;
    hipEvent_t hint_ev[kHintBanks] = {};
    bool hint_ev_used[kHintBanks] = {};
    unsigned long long hint_sig = 0;
    int sort_bound = 0;  // ORT_OPT_SORT_BOUND (testing): > 0 forces this bound
    // ORT_OPT_COST_ORDER (cost_order_slot): per slot the walk steps of its last camera ray,
    // cleared when the frame shape or scene changes (cost_sig)
    int cost_order = 1;
    DevBuf pcost;
    // whole-pixel paths, heavy blocks first: two {kPixelClasses segments of block lists} buffers
    // and their counts, the blocks' cost accumulators, the parity of the next frame's write
    // buffer, and the shape the read buffer's lists belong to (0: none)
    DevBuf pplist, ppcnt, ppcost;
    // samples in parallel (ORT_OPT_PIXEL_SPECULATE): the two per-chunk end-state buffers (spst,
    // which one is last frame's: sp_par), the samples' radiance, the fixup list and its length,
    // and the shape the recorded states belong to (0: none)
    DevBuf spst, spcol, spfix, spfixn;
    int sp_par = 0;
    unsigned long long sp_sig = 0;
    // (the pixels a frame found moved, and whether the next one speculates: spfixn, PipeArgs::sp_ctl)
    // ORT_OPT_PIXEL_SPECULATE auto (-1): per shape, a whole-chain frame's time (frame slot
    // sp_tslot[0]) against a speculating frame's (sp_tslot[1]) decides sp_use
    // 0 fresh, 1 first frame done, 2 first speculating frame done (warm-up of both), 3 whole-chain
    // frame measured, 4 speculating frame measured, 5 decided
    int sp_tune = 0;
    int sp_tslot[2] = {0, 0};
    long long sp_tframe = 0;  // ctx->frames when the whole-chain side was measured
    bool sp_use = true;

    int pixel_spec = -1;  // ORT_OPT_PIXEL_SPECULATE: -1 auto, 0 off, 1 on
    int pp_par = 0;
    unsigned long long pp_sig = 0;
    unsigned long long cost_sig = 0;
    // ORT_OPT_HEAVY_FIRST: threshold in walk steps (0 off); bcost holds, per bounce >= 1 of the
    // first kCostBounces of a frame, every slot's last walk steps (cleared with cost_sig)
    static constexpr int kCostBounces = 8;
    int heavy_first = ORT_HEAVY_STEPS;
    int heavy_prio = kHeavyPrioSteps;  // ORT_OPT_HEAVY_PRIO (steps; 0 off)
    ort::KCamera prio_cam{};           // the camera of this context's last frame (heavy priority: static only)
    // ORT_OPT_TILE_PAIRS: camera-ray workgroups of two tiles (cost_order_pair); -1 = auto (tiles
    // of at least kPairsAutoPixels)
    int tile_pairs = -1;
    // ORT_OPT_SPLIT_HEAVY (steps; 0 off; -1 = auto: kSplitAutoSteps on tiles of at most
    // kSplitAutoPixels) / ORT_OPT_SPLIT_LEVEL (0: auto): the heavy camera rays of a 1-sample
    // frame walked by ort_trace_split on aux_stream (k_heavy_scan lists them)
    int split_steps = -1;
    int split_level = 0;
    static constexpr int kSplitCap = 4096;  // heavy rays listed per frame at most
    hipStream_t aux_stream = nullptr;
    hipEvent_t ev_scan = nullptr, ev_split = nullptr, ev_pre = nullptr;
    // the next frame's heavy list is listed by a split frame's exact kernel (pcost final by then)
    // instead of by a scan opening the next frame: pre_ok when the list in hbits/hlist/hcnt[hpar]
    // is that of a frame of shape pre_sig and threshold pre_steps
    bool pre_ok = false;
    unsigned long long pre_sig = 0;
    int pre_steps = 0, hpar = 0;
    DevBuf hcnt;  // two {heavy count, split cursor} pairs (16 ints): ort_trace_split zeroes the other
    DevBuf hbits, hlist;
    DevBuf bcost;
    unsigned long long bcost_sig = 0;
    float root_lo[3] = {0, 0, 0}, root_hi[3] = {0, 0, 0};  // root box (coherence-sort key)
    ort::GpuTree tree;  // reference-layout tree of the last ort_build_scene(keep_tree)
    float build_ms = 0.0f;
    bool has_scene = false;
    int layout = ORT_LAYOUT_EXPLICIT;
    int depth = 0;
    bool ordered = true;  // compact layout: fast walk allowed (CompactLayout::ordered)
    int32_t n_spheres = 0, n_nodes = 0;
    int64_t n_indices = 0;
    DevBuf sph_cr, sph_ma, sph_fr;
    DevBuf node, leaf_sph, leaf_idx, planes, kid;  // compact
    DevBuf nk;                                   // ... node records and kid entries interleaved (build_nk)
    DevBuf lds_img;                              // compact: the workgroup LDS image (k_lds_image)
    DevBuf lds_rev;                              // ... depth 9-10: the reversed-table image (persistent kernel)
    DevBuf nodeA, nodeB, cnt, indices;           // explicit
    DevBuf scratch_out, counters;
    // wavefront pipeline state, sized for the largest tile rendered so far
    DevBuf hit, defer_list, defer_count, po, pd, pc, prng, pcol;
    int sync_set = 0;      // defer_count's counter set of the next trace launch (render_impl)
    int debug_flags = 0;   // ORT_OPT_DEBUG_FLAGS (A/B of the per-frame stream structure only)
    int launch_times = 1;  // ORT_OPT_LAUNCH_TIMES: per-launch trace-timing events
    bool sync_ok = false;  // both sets zero except the one the last exact kernel left to zero
    DevBuf qlist, qlist2, qcount, qtemp;  // bounce >= 1 path compaction (two lists: read one, append the other)
    DevBuf skeys, skeys2, svals;  // coherence sort
    DevBuf key_spread;            // its origin-code tables for the scene's root box (path_key.h)
    float spread_box[6] = {0, 0, 0, 0, 0, 0};  // the root box key_spread was built for
};

namespace {

int fail(ort_ctx* ctx, int code, const std::string& msg) {
    if (ctx) ctx->err = msg;
    ort::set_thread_error(msg);
    return code;
}

int hip_fail(ort_ctx* ctx, hipError_t e, const char* what) {
    return fail(ctx, e == hipErrorOutOfMemory ? ORT_ERR_OUT_OF_MEMORY : ORT_ERR_HIP,
                std::string(what) + ": " + hipGetErrorString(e));
}

#define HIPCHK(ctx, expr)                                  \
    do {                                                   \
        hipError_t _e = (expr);                            \
        if (_e != hipSuccess) return hip_fail(ctx, _e, #expr); \
    } while (0)

void free_buf(DevBuf& b) {
    if (b.p) (void)hipFree(b.p);
    b.p = nullptr;
    b.bytes = 0;
}

void free_scene(ort_ctx* c) {
    DevBuf* all[] = {&c->sph_cr, &c->sph_ma, &c->sph_fr, &c->node, &c->kid, &c->nk, &c->leaf_sph, &c->leaf_idx,
                     &c->planes, &c->lds_img, &c->lds_rev, &c->nodeA, &c->nodeB, &c->cnt, &c->indices};
    for (DevBuf* b : all) free_buf(*b);
    ort::freeGpuTree(c->tree);
    c->has_scene = false;
}

int upload(ort_ctx* ctx, DevBuf& b, const void* src, size_t bytes) {
    free_buf(b);
    if (bytes == 0) bytes = 16;  // keep a valid pointer for empty arrays
    HIPCHK(ctx, hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    if (src) HIPCHK(ctx, hipMemcpyAsync(b.p, src, bytes, hipMemcpyHostToDevice, ctx->stream));
    return ORT_OK;
}

// The compact layout's workgroup LDS image (plane tables | rank LUT) from ctx->planes.
int build_lds_image(ort_ctx* ctx) {
    for (int rev = 0; rev < 2; ++rev) {
        if (rev && !(kRevBounce && ctx->depth > 8)) break;
        DevBuf& img = rev ? ctx->lds_rev : ctx->lds_img;
        const size_t bytes = (size_t)ort::lds_layout(ctx->depth, rev || ort::fast_rev_planes(ctx->depth)).frames;
        int rc;
        if ((rc = upload(ctx, img, nullptr, bytes))) return rc;
        hipLaunchKernelGGL(k_lds_image, dim3(1), dim3(kBlock), 0, ctx->stream, (const float*)ctx->planes.p, ctx->depth,
                           rev != 0, (unsigned char*)img.p);
        HIPCHK(ctx, hipGetLastError());
    }
    return ORT_OK;
}

__global__ void __launch_bounds__(kBlock) k_interleave_nk(const uint2* node, const uint2* kid, uint4* nk, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x;
    if (i >= n) return;
    const uint2 a = node[i], b = kid[i];
    nk[i] = make_uint4(a.x, a.y, b.x, b.y);
}

// The walks that use the rejected-sphere skip load a node's record and kid entry together
// (fetch_rec): one 16-byte load, one cache line per record instead of one in each array.
// Built when both arrays are there and 16 bytes per node stay under the buffer loads' 4 GiB.
int build_nk(ort_ctx* ctx) {
    free_buf(ctx->nk);
    const int64_t n = (int64_t)(ctx->node.bytes / 8);
    if (!ORT_NODE_KID || !ctx->kid.p || ctx->kid.bytes < ctx->node.bytes || n == 0 || 16 * n >= (int64_t)UINT32_MAX)
        return ORT_OK;
    int rc;
    if ((rc = upload(ctx, ctx->nk, nullptr, 16 * (size_t)n))) return rc;
    hipLaunchKernelGGL(k_interleave_nk, dim3((unsigned)((n + kBlock - 1) / kBlock)), dim3(kBlock), 0, ctx->stream,
                       (const uint2*)ctx->node.p, (const uint2*)ctx->kid.p, (uint4*)ctx->nk.p, n);
    HIPCHK(ctx, hipGetLastError());
    return ORT_OK;
}

// Root box for the coherence-sort key: the tree's root node, or the spheres' bounds when
// there is no tree (brute force).  Only orders work; never affects pixels.
void set_root_box(ort_ctx* ctx, const float* nmin, const float* nmax, const float* cr, int32_t n) {
    for (int a = 0; a < 3; ++a) {
        ctx->root_lo[a] = 0.0f;
        ctx->root_hi[a] = 0.0f;
    }
    if (nmin && nmax) {
        for (int a = 0; a < 3; ++a) {
            ctx->root_lo[a] = nmin[a];
            ctx->root_hi[a] = nmax[a];
        }
        return;
    }
    for (int32_t i = 0; i < n && cr; ++i)
        for (int a = 0; a < 3; ++a) {
            const float lo = cr[4 * (size_t)i + a] - cr[4 * (size_t)i + 3], hi = cr[4 * (size_t)i + a] + cr[4 * (size_t)i + 3];
            if (i == 0 || lo < ctx->root_lo[a]) ctx->root_lo[a] = lo;
            if (i == 0 || hi > ctx->root_hi[a]) ctx->root_hi[a] = hi;
        }
}

// Spheres -> device (bindings 0, 1 and the .xy of binding 2).
int upload_spheres(ort_ctx* ctx, const float* cr, const float* ma, const float* fr, int32_t n) {
    std::vector<float> fr2((size_t)n * 2);
    for (int32_t i = 0; i < n; ++i) {
        fr2[2 * (size_t)i] = fr[4 * (size_t)i];
        fr2[2 * (size_t)i + 1] = fr[4 * (size_t)i + 1];
    }
    int rc;
    if ((rc = upload(ctx, ctx->sph_cr, cr, 16 * (size_t)n))) return rc;
    if ((rc = upload(ctx, ctx->sph_ma, ma, 16 * (size_t)n))) return rc;
    if ((rc = upload(ctx, ctx->sph_fr, fr2.data(), 8 * (size_t)n))) return rc;
    ctx->n_spheres = n;
    return ORT_OK;
}

// ort_build_scene: GPU octree build (gpu_build.hip) straight into the kernel layout.
int build_impl(ort_ctx* ctx, const float* cr, const float* ma, const float* fr, int32_t n, int32_t max_depth,
               int32_t max_per_node, int32_t keep_tree) {
    if (n <= 0) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_build_scene: Sphere list is empty");
    if (!cr || !ma || !fr) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_build_scene: null sphere array");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    free_scene(ctx);
    int rc;
    if ((rc = upload_spheres(ctx, cr, ma, fr, n))) return rc;
    ort::GpuTree t;
    const std::string e = ort::gpuBuildOctree((const float4*)ctx->sph_cr.p, n, max_depth, max_per_node, ctx->stream, t);
    if (!e.empty()) {
        ort::freeGpuTree(t);
        return fail(ctx, e.find("out of memory") != std::string::npos ? ORT_ERR_OUT_OF_MEMORY : ORT_ERR_INTERNAL,
                    "ort_build_scene: " + e);
    }
    ctx->n_nodes = t.n_nodes;
    ctx->n_indices = t.n_indices;
    ctx->depth = t.depth;
    ctx->ordered = t.ordered;
    {
        float lo[3], hi[3];
        if (hipMemcpy(lo, t.node_min, 12, hipMemcpyDeviceToHost) == hipSuccess &&
            hipMemcpy(hi, t.node_max, 12, hipMemcpyDeviceToHost) == hipSuccess)
            set_root_box(ctx, lo, hi, nullptr, 0);
    }
    ctx->build_ms = (float)(t.seconds * 1e3);
    std::string why;
    ort::CompactDev cd;
    const bool compact_ok = ctx->force_layout != ORT_LAYOUT_EXPLICIT &&
                            ort::gpuCompactLayout(t, (const float4*)ctx->sph_cr.p, ORT_COMPACT_MAX_DEPTH, ctx->stream, cd, why);
    if (compact_ok) {
        ctx->layout = ORT_LAYOUT_COMPACT;
        ctx->node = {cd.node, cd.node_bytes};
        ctx->kid = {cd.kid, cd.node_bytes};
        ctx->leaf_sph = {cd.leaf_sph, cd.leaf_bytes};
        ctx->leaf_idx = {cd.leaf_idx, cd.idx_bytes};
        ctx->planes = {cd.planes, cd.plane_bytes};
        if ((rc = build_lds_image(ctx)) || (rc = build_nk(ctx))) {
            ort::freeGpuTree(t);
            return rc;
        }
    } else {
        if (ctx->force_layout == ORT_LAYOUT_COMPACT) {
            ort::freeGpuTree(t);
            return fail(ctx, ORT_ERR_UNSUPPORTED, "compact layout forced but not possible: " + why);
        }
        ort::ExplicitDev ed;
        const std::string ee = ort::gpuExplicitLayout(t, ctx->stream, ed);
        ctx->nodeA = {ed.nodeA, 16 * (size_t)std::max(t.n_nodes, 1)};
        ctx->nodeB = {ed.nodeB, 16 * (size_t)std::max(t.n_nodes, 1)};
        ctx->cnt = {ed.cnt, 4 * (size_t)std::max(t.n_nodes, 1)};
        ctx->indices = {ed.indices, 4 * (size_t)std::max<int64_t>(t.n_indices, 1)};
        if (!ee.empty()) {
            ort::freeGpuTree(t);
            free_scene(ctx);
            return fail(ctx, ORT_ERR_HIP, "ort_build_scene: " + ee);
        }
        ctx->layout = ORT_LAYOUT_EXPLICIT;
    }
    if (keep_tree) ctx->tree = t;
    else ort::freeGpuTree(t);
    ctx->has_scene = true;
    return ORT_OK;
}

int upload_impl(ort_ctx* ctx, const ort::SceneInput& in) {
    const std::string bad = ort::validateScene(in);
    if (!bad.empty()) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_upload_scene: " + bad);
    HIPCHK(ctx, hipSetDevice(ctx->device));
    free_scene(ctx);
    int rc;
    if ((rc = upload_spheres(ctx, in.sph_cr, in.sph_ma, in.sph_fr, in.n_spheres))) return rc;
    ctx->n_nodes = in.n_nodes;
    ctx->n_indices = in.n_indices;
    ctx->layout = ORT_LAYOUT_EXPLICIT;
    ctx->depth = 0;
    set_root_box(ctx, in.n_nodes > 0 ? in.node_min : nullptr, in.n_nodes > 0 ? in.node_max : nullptr, in.sph_cr,
                 in.n_spheres);
    if (in.n_nodes > 0) {
        ort::CompactLayout cl;
        std::string why;
        const bool want_compact = ctx->force_layout != ORT_LAYOUT_EXPLICIT;
        const bool compact_ok = want_compact && ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why);
        if (ctx->force_layout == ORT_LAYOUT_COMPACT && !compact_ok)
            return fail(ctx, ORT_ERR_UNSUPPORTED, "compact layout forced but not possible: " + why);
        if (compact_ok) {
            ctx->layout = ORT_LAYOUT_COMPACT;
            ctx->depth = cl.depth;
            ctx->ordered = cl.ordered;
            if ((rc = upload(ctx, ctx->node, cl.node.data(), 4 * cl.node.size()))) return rc;
            if ((rc = upload(ctx, ctx->kid, cl.kid.data(), 4 * cl.kid.size()))) return rc;
            if ((rc = upload(ctx, ctx->leaf_sph, cl.leaf_sph.data(), 4 * cl.leaf_sph.size()))) return rc;
            if ((rc = upload(ctx, ctx->leaf_idx, cl.leaf_idx.data(), 4 * cl.leaf_idx.size()))) return rc;
            if ((rc = upload(ctx, ctx->planes, cl.planes.data(), 4 * cl.planes.size()))) return rc;
            if ((rc = build_lds_image(ctx))) return rc;
            if ((rc = build_nk(ctx))) return rc;
            HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        } else {
            const int d = ort::treeDepth(in);
            ctx->depth = d < 0 ? 0 : d;
            std::vector<float> A(4 * (size_t)in.n_nodes), B(4 * (size_t)in.n_nodes);
            for (int32_t i = 0; i < in.n_nodes; ++i) {
                for (int k = 0; k < 3; ++k) {
                    A[4 * (size_t)i + k] = in.node_min[3 * (size_t)i + k];
                    B[4 * (size_t)i + k] = in.node_max[3 * (size_t)i + k];
                }
                std::memcpy(&A[4 * (size_t)i + 3], &in.co[i], 4);
                std::memcpy(&B[4 * (size_t)i + 3], &in.oo[i], 4);
            }
            if ((rc = upload(ctx, ctx->nodeA, A.data(), 4 * A.size()))) return rc;
            if ((rc = upload(ctx, ctx->nodeB, B.data(), 4 * B.size()))) return rc;
            if ((rc = upload(ctx, ctx->cnt, in.cnt, 4 * (size_t)in.n_nodes))) return rc;
            if ((rc = upload(ctx, ctx->indices, in.indices, 4 * (size_t)in.n_indices))) return rc;
            HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
        }
    } else {
        HIPCHK(ctx, hipStreamSynchronize(ctx->stream));
    }
    ctx->has_scene = true;
    return ORT_OK;
}

ort::KScene device_scene(const ort_ctx* c) {
    ort::KScene S;
    std::memset(&S, 0, sizeof(S));
    S.sph_cr = (const float4*)c->sph_cr.p;
    S.sph_ma = (const float4*)c->sph_ma.p;
    S.sph_fr = (const float2*)c->sph_fr.p;
    S.n_spheres = c->n_spheres;
    S.n_nodes = c->n_nodes;
    S.node = (const uint2*)c->node.p;
    S.kid = c->kid_skip ? (const uint2*)c->kid.p : nullptr;
    S.nk = c->kid_skip == 1 ? (const uint4*)c->nk.p : nullptr;  // 2: the separate arrays (testing)
    S.nk_bytes = (uint32_t)c->nk.bytes;
    S.tail_base = (uint32_t)c->n_indices;
    S.leaf_sph = (const float4*)c->leaf_sph.p;
    S.node_bytes = (uint32_t)c->node.bytes;
    S.leaf_bytes = (uint32_t)c->leaf_sph.bytes;
    S.leaf_idx = (const int*)c->leaf_idx.p;
    S.planes = (const float*)c->planes.p;
    S.lds_img = (const uint4*)c->lds_img.p;
    S.lds_img_p16 = (int)(align16(sizeof(float) * (size_t)ort::fast_plane_floats(c->depth)) / 16);
    S.lds_img_n16 = ort::lds_layout(c->depth, ort::fast_rev_planes(c->depth)).frames / 16;
    S.lds_rev = (const uint4*)c->lds_rev.p;
    S.lds_rev_n16 = ort::lds_layout(c->depth, true).frames / 16;
    S.depth = c->depth;
    S.nodeA = (const float4*)c->nodeA.p;
    S.nodeB = (const float4*)c->nodeB.p;
    S.count = (const int*)c->cnt.p;
    S.indices = (const int*)c->indices.p;
    return S;
}

ort::KCamera to_kcamera(const ort::CameraFrame& f) {
    ort::KCamera k;
    k.origin = ort::mk(f.origin[0], f.origin[1], f.origin[2]);
    k.lowerLeft = ort::mk(f.lowerLeft[0], f.lowerLeft[1], f.lowerLeft[2]);
    k.horizontal = ort::mk(f.horizontal[0], f.horizontal[1], f.horizontal[2]);
    k.vertical = ort::mk(f.vertical[0], f.vertical[1], f.vertical[2]);
    k.u = ort::mk(f.u[0], f.u[1], f.u[2]);
    k.v = ort::mk(f.v[0], f.v[1], f.v[2]);
    k.w = ort::mk(f.w[0], f.w[1], f.w[2]);
    k.lensRadius = f.lensRadius;
    return k;
}

std::string check_params(const ort_params* p, const ort_tile* t) {
    if (!p || !t) return "null params or tile";
    if (p->width <= 0 || p->height <= 0) return "width/height must be positive";
    if (t->width < 0 || t->rows < 0) return "negative tile size";
    if (t->x0 < 0 || (int64_t)t->x0 + t->width > p->width) return "tile columns outside the frame";
    if (t->y0 < 0) return "negative y0";
    if (t->band_height > 0 && t->band_stride < t->band_height) return "band_stride < band_height";
    return "";
}

ort::PixelParams pixel_params(const ort_params* p) {
    ort::PixelParams pp;
    const ort::CameraFrame f = ort::cameraFrameFromView(p->view, p->camera_position, p->camera_zoom,
                                                        (float)p->width / (float)p->height);
    pp.cam = to_kcamera(f);
    pp.W = p->width;
    pp.H = p->height;
    pp.ns = p->num_samples;
    pp.maxDepth = p->max_depth;
    return pp;
}

int ensure(ort_ctx* ctx, DevBuf& b, size_t bytes) {
    if (b.bytes >= bytes && b.p) return ORT_OK;
    free_buf(b);
    HIPCHK(ctx, hipMalloc(&b.p, bytes));
    b.bytes = bytes;
    return ORT_OK;
}

template <bool COUNT, bool PRIMARY>
hipError_t launch_trace_p(int mode, const PipeArgs& a, int blocks, int pblocks, size_t lds, hipStream_t s, int fuse) {
    if (PRIMARY && mode == 0 && a.pair && pblocks == 0) {  // tile pairs: blocks = workgroups (one per pair)
        const dim3 g(blocks), t(kBlock);
        if (a.S.depth > 8) {
            if (fuse == 1) hipLaunchKernelGGL((ort_trace_pair_deep<COUNT, 1>), g, t, lds, s, a);
            else if (fuse == 2) hipLaunchKernelGGL((ort_trace_pair_deep<COUNT, 2>), g, t, lds, s, a);
            else hipLaunchKernelGGL((ort_trace_pair_deep<COUNT, 0>), g, t, lds, s, a);
        } else {
            if (fuse == 1) hipLaunchKernelGGL((ort_trace_pair<COUNT, 1>), g, t, lds, s, a);
            else if (fuse == 2) hipLaunchKernelGGL((ort_trace_pair<COUNT, 2>), g, t, lds, s, a);
            else hipLaunchKernelGGL((ort_trace_pair<COUNT, 0>), g, t, lds, s, a);
        }
        return hipGetLastError();
    }
    if (mode == 0 && pblocks > 0) {
        if (a.S.depth > 8)
            hipLaunchKernelGGL((ort_trace_persistent<COUNT, true>), dim3(pblocks), dim3(kPersistDeepBlock),
                               lds_bytes(0, a.S.depth, false, kRevBounce, kPersistDeepBlock), s, a);
        else hipLaunchKernelGGL((ort_trace_persistent<COUNT, false>), dim3(pblocks), dim3(kBlock), lds, s, a);
    }
    else if (mode == 0 && a.S.depth > 8)
    {
        if (fuse == 1) hipLaunchKernelGGL((ort_trace_compact_deep<COUNT, PRIMARY, 1>), dim3(blocks), dim3(kBlock), lds, s, a);
        else if (fuse == 2) hipLaunchKernelGGL((ort_trace_compact_deep<COUNT, PRIMARY, 2>), dim3(blocks), dim3(kBlock), lds, s, a);
        else hipLaunchKernelGGL((ort_trace_compact_deep<COUNT, PRIMARY, 0>), dim3(blocks), dim3(kBlock), lds, s, a);
    }
    else if (mode == 0 && fuse == 1)
        hipLaunchKernelGGL((ort_trace_compact<COUNT, PRIMARY, 1>), dim3(blocks), dim3(kBlock), lds, s, a);
    else if (mode == 0 && fuse == 2)
        hipLaunchKernelGGL((ort_trace_compact<COUNT, PRIMARY, 2>), dim3(blocks), dim3(kBlock), lds, s, a);
    else if (mode == 0) hipLaunchKernelGGL((ort_trace_compact<COUNT, PRIMARY, 0>), dim3(blocks), dim3(kBlock), lds, s, a);
    else if (mode == 1) hipLaunchKernelGGL((ort_trace_kernel<1, COUNT, PRIMARY>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((ort_trace_kernel<2, COUNT, PRIMARY>), dim3(blocks), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

template <bool COUNT>
hipError_t launch_trace(int mode, bool primary, const PipeArgs& a, int blocks, int pblocks, size_t lds, hipStream_t s,
                        int fuse) {
    return primary ? launch_trace_p<COUNT, true>(mode, a, blocks, pblocks, lds, s, fuse)
                   : launch_trace_p<COUNT, false>(mode, a, blocks, pblocks, lds, s, 0);
}

template <int MODE>
hipError_t launch_shade_mode(bool first, bool direct, const PipeArgs& a, int blocks, hipStream_t s) {
    if (direct) hipLaunchKernelGGL((ort_shade_kernel<MODE, true, true>), dim3(blocks), dim3(kBlock), 0, s, a);
    else if (first) hipLaunchKernelGGL((ort_shade_kernel<MODE, true, false>), dim3(blocks), dim3(kBlock), 0, s, a);
    else hipLaunchKernelGGL((ort_shade_kernel<MODE, false, false>), dim3(blocks), dim3(kBlock), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_shade(int mode, bool first, bool direct, const PipeArgs& a, int blocks, hipStream_t s) {
    if (mode == 0) return launch_shade_mode<0>(first, direct, a, blocks, s);
    if (mode == 1) return launch_shade_mode<1>(first, direct, a, blocks, s);
    return launch_shade_mode<2>(first, direct, a, blocks, s);
}

// Resident workgroups of the persistent trace kernel (a plain launch: extra groups just
// start when others finish; no grid-wide synchronisation depends on residency).
int persistent_blocks(int device, bool count, bool deep, int depth, size_t lds, long long needed) {
    int per_cu = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    const size_t dlds = lds_bytes(0, depth, false, kRevBounce, kPersistDeepBlock);
    if (count)
        (void)(deep ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ort_trace_persistent<true, true>, kPersistDeepBlock, dlds)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ort_trace_persistent<true, false>, kBlock, lds));
    else
        (void)(deep ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ort_trace_persistent<false, true>, kPersistDeepBlock, dlds)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ort_trace_persistent<false, false>, kBlock, lds));
    long long b = (long long)std::max(per_cu, 1) * std::max(cus, 1);
    return (int)std::max(1LL, std::min(b, needed));
}

// Whole-pixel paths (ort_pixel_paths): the frame in one launch.  Auto (ORT_OPT_PIXEL_PATHS -1):
// frames of more than one traversal per pixel on brute force, and on trees of at most
// kPixelPathsAutoNodes nodes, kPixelPathsAutoNodes5 with 5+ bounces, kPixelPathsAutoNodes8 with
// 8+ -- where the pipeline's per-bounce launches and sorts cost more than its coherence gains.
// The crossover follows the bounces: the pipeline pays a launch, a sort and a copy per bounce
// even when few paths are left, whole-pixel paths only the paths' own work (1080p grid over
// 1.5-11 M nodes x 1-4 samples x 4-16 bounces, profiles/r06/grid/).
constexpr long long kPixelPathsAutoNodes = 1ll << 19;   // any bounce depth
constexpr long long kPixelPathsAutoNodes5 = 1ll << 23;  // maxDepth 5-7
constexpr long long kPixelPathsAutoNodes8 = 1ll << 24;  // maxDepth 8+ (measured to 11 M nodes)
#ifndef ORT_PIXEL_LDS_SCENE_BYTES
#define ORT_PIXEL_LDS_SCENE_BYTES 32768
#endif
constexpr int kPixelLdsSceneBytes = ORT_PIXEL_LDS_SCENE_BYTES;  // LDS-resident scene budget (ort_pixel_paths)
// samples in parallel: device bytes of the per-sample buffers (two end states, the radiance) and
// the per-slot ones (flags, fixup list); frames above the budget run the pixels' chains whole
constexpr size_t kSpecBudget = size_t(8) << 30;
#ifndef ORT_PIXEL_SPEC_CHUNKS
#define ORT_PIXEL_SPEC_CHUNKS 4
#endif
// a pixel's samples in (about) this many chunks of at least kSpecMinChunk samples: a SPEC item
// is one chunk of a block's pixels -- shorter chains with more chunks, but each item starts with
// a load of its state and a refill (one-sample chunks: 4 x 4 on 10 spheres at 1080p 0.55 ->
// 1.69 ms; config.h's 16 x 8 in 2 / 4 / 8 chunks: 1.46 / 1.77 / 1.60x, profiles/r06/ab_spec_*)
constexpr int kSpecChunks = ORT_PIXEL_SPEC_CHUNKS;
constexpr int kSpecMinChunk = 4;
inline int spec_chunk(int ns) { return std::max(kSpecMinChunk, (ns + kSpecChunks - 1) / kSpecChunks); }
inline int spec_nch(int ns) { return (ns + spec_chunk(ns) - 1) / spec_chunk(ns); }
#ifndef ORT_PIXEL_SPEC_MOVED_MAX
#define ORT_PIXEL_SPEC_MOVED_MAX 1000
#endif
constexpr long long kSpecMovedMax = ORT_PIXEL_SPEC_MOVED_MAX;
constexpr float kSpecAutoGain = 1.0f;           // auto keeps speculating when it ran at most this x the whole-chain frame
constexpr long long kSpecAutoPixels = 1 << 20;  // ... and without timing events, on frames of at most this many pixels
inline size_t spec_bytes(size_t slots, int ns) { return slots * ((size_t)spec_nch(ns) * 16 + (size_t)ns * 12 + 28); }
bool use_pixel_paths(const ort_ctx* ctx, int mode, int ns, int maxd);

template <int MODE, bool DEEP, bool LDS, int PM>
int pixel_paths_blocks(int device, size_t lds, long long needed) {
    int per_cu = 0, cus = 0;
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, ort_pixel_paths<MODE, DEEP, LDS, PM>, kBlock, lds);
    const long long b = (long long)std::max(per_cu, 1) * std::max(cus, 1);
    return (int)std::max(1LL, std::min(b, needed));
}

// One ort_pixel_paths launch (the variant of the scene's walk) over a persistent grid sized by
// the variant's occupancy, at most `needed` workgroups.
template <int PM>
hipError_t launch_pixel_paths(const ort_ctx* ctx, int mode, bool deep, bool lds_scene, size_t lds, long long needed,
                              const PipeArgs& a, hipStream_t s) {
    if (mode == 2) {
        const int g = pixel_paths_blocks<2, false, false, PM>(ctx->device, 0, needed);
        hipLaunchKernelGGL((ort_pixel_paths<2, false, false, PM>), dim3(g), dim3(kBlock), 0, s, a);
    } else if (deep) {
        const int g = pixel_paths_blocks<0, true, false, PM>(ctx->device, lds, needed);
        hipLaunchKernelGGL((ort_pixel_paths<0, true, false, PM>), dim3(g), dim3(kBlock), lds, s, a);
    } else if (lds_scene) {
        const int g = pixel_paths_blocks<0, false, true, PM>(ctx->device, lds, needed);
        hipLaunchKernelGGL((ort_pixel_paths<0, false, true, PM>), dim3(g), dim3(kBlock), lds, s, a);
    } else {
        const int g = pixel_paths_blocks<0, false, false, PM>(ctx->device, lds, needed);
        hipLaunchKernelGGL((ort_pixel_paths<0, false, false, PM>), dim3(g), dim3(kBlock), lds, s, a);
    }
    return hipGetLastError();
}

// FNV-1a of the frame shape and scene: the previous-frame hints (list lengths, walk costs)
// belong to one of these
unsigned long long frame_sig(const ort_ctx* ctx, const ort_params* p, const ort_tile* t) {
    const long long v[] = {p->width, p->height, p->num_samples, p->max_depth, t->x0, t->width, t->y0,
                           t->rows, t->band_height, t->band_stride, ctx->n_nodes, ctx->n_spheres,
                           (long long)ctx->n_indices, ctx->xcd_swizzle, ctx->tile_pairs};
    unsigned long long sig = 1469598103934665603ull;
    for (long long x : v) sig = (sig ^ (unsigned long long)x) * 1099511628211ull;
    return sig;
}

bool use_pixel_paths(const ort_ctx* ctx, int mode, int ns, int maxd) {
    if (mode == 1 || maxd < 1 || (ns == 1 && maxd == 1) || ctx->pixel_paths == 0) return false;
    if (ctx->pixel_paths > 0) return true;
    // 1080p, whole-pixel paths over the pipeline: 8 bounces 1.02-1.50x from 1.5 to 11 M nodes
    // (1 to 4 samples), 5 bounces 1.09-1.10x to 5 M, 1.00x at 8.3 M, 0.95x at 11 M; 4 bounces
    // 0.74-1.02x from 1.5 M nodes on, 1.09x at 209 k (profiles/r06/grid/)
    const long long limit = maxd >= 8 ? kPixelPathsAutoNodes8 : (maxd >= 5 ? kPixelPathsAutoNodes5 : kPixelPathsAutoNodes);
    return mode == 2 || ctx->n_nodes <= limit;
}

// The frame as one ort_pixel_paths launch (use_pixel_paths); dout: the frame on the device.
int render_pixel_paths(ort_ctx* ctx, const ort_params* p, const ort_tile* t, int mode, float* dout, hipStream_t s) {
    const int tilesX = (t->width + 15) / 16, tilesY = (t->rows + 15) / 16;
    const long long blocks = (long long)tilesX * tilesY;
    PipeArgs a;
    std::memset(&a, 0, sizeof(a));
    a.pp = pixel_params(p);
    a.S = device_scene(ctx);
    a.tm = {t->x0, t->width, t->y0, t->rows, t->band_height, t->band_stride};
    a.tilesX = tilesX;
    a.tilesY = tilesY;
    a.total = (int)(blocks * kBlock);
    a.exact_only = ctx->exact_only || !ctx->ordered;
    a.out = dout;
    // the cursor and done count: this frame's counter set (zero; the kernel's last workgroup
    // zeroes them again, so the set stays the pipeline's next one)
    if (!ctx->sync_ok) {
        HIPCHK(ctx, hipMemsetAsync(ctx->defer_count.p, 0, 128, s));
        ctx->sync_set = 0;
        ctx->pre_ok = false;
        ctx->pp_sig = 0;  // (the class lists' counts re-zeroed below)
    }
    ctx->sync_ok = false;
    a.sync = (int*)ctx->defer_count.p + 16 * ctx->sync_set;
#if ORT_ANALYSIS
    a.wclock = (ulonglong4*)ctx->wclock;  // ORT_PIXEL_CLOCK builds (tools/pixel_clock.py)
    a.wclock_n = (int)ctx->wclock_n;
#endif
    const unsigned long long sig = frame_sig(ctx, p, t);
    // samples in parallel (ORT_OPT_PIXEL_SPECULATE, ort_pixel_paths<..., SPEC>): from the second
    // frame of a shape on, when the per-sample state buffers fit kSpecBudget; the first frame
    // runs the pixels' chains whole and records their samples' end states
    const int ns = p->num_samples;
    const size_t slots = (size_t)a.total;
    const int nch = spec_nch(ns);
    const bool timed_now = !((ctx->debug_flags & 1) || !ctx->launch_times);
    const bool spec_on = ctx->pixel_spec != 0 && nch > 1 && spec_bytes(slots, ns) <= kSpecBudget;
    if (!spec_on) ctx->sp_sig = 0;
    bool spec_frame = false;
    float2 *sp_prev = nullptr, *sp_cur = nullptr;
    if (spec_on) {
        const void* had = ctx->spst.p;
        int rc;
        if ((rc = ensure(ctx, ctx->spst, 2 * sizeof(float2) * (size_t)nch * slots)) ||
            (rc = ensure(ctx, ctx->spcol, 3 * sizeof(float) * (size_t)ns * slots)) ||
            (rc = ensure(ctx, ctx->spfix, (2 * sizeof(int) + sizeof(float2) + 3 * sizeof(float)) * slots)) ||
            (rc = ensure(ctx, ctx->spfixn, 64)))
            return rc;
        if (ctx->spst.p != had) ctx->sp_sig = 0;  // reallocated: no recorded states
        const long long pixels = (long long)t->width * t->rows;
        if (ctx->sp_sig != sig) {  // a fresh start: an empty fixup list, nothing moved
            HIPCHK(ctx, hipMemsetAsync(ctx->spfixn.p, 0, 64, s));
            ctx->sp_tune = 0;
            // untimed contexts cannot compare: speculate on frames of at most kSpecAutoPixels
            ctx->sp_use = ctx->pixel_spec > 0 || timed_now || pixels <= kSpecAutoPixels;
        }
        if (ctx->sp_tune >= 3 && ctx->sp_tune < 5 && ctx->frames - ctx->sp_tframe >= ort_ctx::kRing - 2)
            ctx->sp_tune = 2;  // the measured frames' timing slots are being reused: measure again
        if (ctx->pixel_spec < 0 && ctx->sp_tune == 4) {  // auto: a measured whole-chain frame against a measured SPEC frame
            float tw = 0.0f, tsp = 0.0f, x = 0.0f;
            bool ok = hipEventQuery(ctx->tr1[ctx->sp_tslot[1]][2]) == hipSuccess;
            for (int j = 0; ok && j < 3; ++j) {
                ok = hipEventElapsedTime(&x, ctx->tr0[ctx->sp_tslot[1]][j], ctx->tr1[ctx->sp_tslot[1]][j]) == hipSuccess;
                tsp += x;
            }
            if (ok) ok = hipEventElapsedTime(&tw, ctx->tr0[ctx->sp_tslot[0]][0], ctx->tr1[ctx->sp_tslot[0]][0]) == hipSuccess;
            if (ok) {
                ctx->sp_use = tsp < kSpecAutoGain * tw;
                ctx->sp_tune = 5;
            }
        }
        spec_frame = ctx->sp_sig == sig && ctx->sp_use &&
                     !(ctx->pixel_spec < 0 && timed_now && ctx->sp_tune == 2);  // auto: the measured whole-chain frame
        a.sp_ctl = (int*)ctx->spfixn.p;
        float2* st0 = (float2*)ctx->spst.p;
        sp_prev = ctx->sp_par ? st0 + (size_t)nch * slots : st0;
        sp_cur = ctx->sp_par ? st0 : st0 + (size_t)nch * slots;
        a.sp_chunk = spec_chunk(ns);
        a.sp_nch = nch;
    }
    // heavy blocks first (ORT_OPT_PIXEL_HEAVY_FIRST; auto: several samples -- a pixel's chain is
    // then long enough for the frame's tail to matter, while one-sample frames keep tile order's
    // locality: 1080p 1 x 4 on 10k spheres 0.89x in heavy-first order, profiles/r06/ab_blk_*);
    // not in a frame of parallel samples (nothing there is as long as a pixel's chain)
    const bool heavy_first = !spec_frame &&
                             (ctx->pixel_heavy_first > 0 || (ctx->pixel_heavy_first < 0 && p->num_samples > 1));
    if (ORT_PIXEL_LPT && !heavy_first && !spec_frame) ctx->pp_sig = 0;
    if (ORT_PIXEL_LPT && heavy_first) {  // last frame's class lists (same shape) and this frame's
        const size_t nb = (size_t)blocks * (kBlock / 64), cnt_b = 2 * kPixelClasses * sizeof(int);
        int rc;
        if ((rc = ensure(ctx, ctx->pplist, 2 * kPixelClasses * 4 * nb)) || (rc = ensure(ctx, ctx->ppcnt, cnt_b)) ||
            (rc = ensure(ctx, ctx->ppcost, 8 * nb)))
            return rc;
        if (ctx->pp_sig == 0 || ctx->pp_sig != sig) {  // no lists of this shape: zero counts and accumulators
            HIPCHK(ctx, hipMemsetAsync(ctx->ppcnt.p, 0, cnt_b, s));
            HIPCHK(ctx, hipMemsetAsync(ctx->ppcost.p, 0, 8 * nb, s));
        }
        const int w = ctx->pp_par, r = w ^ 1;
        int* lists = (int*)ctx->pplist.p;
        int* cnt = (int*)ctx->ppcnt.p;
        a.pl_stride = (int)nb;
        a.pl_w = lists + (size_t)w * kPixelClasses * nb;
        a.pl_wcnt = cnt + kPixelClasses * w;
        a.pl_rcnt = cnt + kPixelClasses * r;
        a.pl_cost = (unsigned long long*)ctx->ppcost.p;
        a.pl_r = (ctx->pp_sig == sig) ? lists + (size_t)r * kPixelClasses * nb : nullptr;
        ctx->pp_par = r;
        ctx->pp_sig = sig;
    }
    const bool deep = ctx->depth > 8;
    size_t lds = mode == 0 ? lds_bytes(0, ctx->depth, true) : 0;
    // an LDS-resident scene: node records + kid entries (16 B per node) and the leaf spheres
    // (16 B per entry: objectIndices, then the per-sphere tail), when they fit the budget
    const size_t nk_b = 16 * (size_t)ctx->n_nodes, sph_b = 16 * ((size_t)ctx->n_indices + (size_t)ctx->n_spheres);
    const bool lds_scene = mode == 0 && !deep && a.S.nk && ctx->pixel_lds_scene &&
                           nk_b + sph_b <= (size_t)kPixelLdsSceneBytes;
    if (lds_scene) {
        a.lds_nk_off = (int)align16(lds);
        a.lds_sph_off = (int)(a.lds_nk_off + nk_b);
        a.lds_nk_n16 = (int)(nk_b / 16);
        a.lds_sph_n16 = (int)(sph_b / 16);
        lds = (size_t)a.lds_sph_off + sph_b;
    }
    const int fslot = (int)(ctx->frames % ort_ctx::kRing);
    ctx->tseg[fslot] = 0;
    const bool timed = !((ctx->debug_flags & 1) || !ctx->launch_times);
    const int nseg = spec_frame ? 3 : 1;  // SPEC: the samples, the resolve, the fixup list
    for (int j = 0; timed && j < nseg; ++j)
        if (!ctx->tr0[fslot][j]) {
            HIPCHK(ctx, hipEventCreate(&ctx->tr0[fslot][j]));
            HIPCHK(ctx, hipEventCreate(&ctx->tr1[fslot][j]));
        }
    ctx->ev0_last = timed ? ctx->tr0[fslot][0] : ctx->ev0;  // the frame's start is its trace launch's
    HIPCHK(ctx, hipEventRecord(ctx->ev0_last, s));
    if (!spec_frame) {  // every pixel's whole chain (recording its samples' end states when spec_on)
        a.sp_cur = sp_cur;
        const bool rec = spec_on && ctx->sp_use;  // (auto found speculation slower on this shape: no recording)
        const hipError_t e = rec ? launch_pixel_paths<2>(ctx, mode, deep, lds_scene, lds, blocks, a, s)
                                 : launch_pixel_paths<0>(ctx, mode, deep, lds_scene, lds, blocks, a, s);
        if (e != hipSuccess) return hip_fail(ctx, e, "ort_pixel_paths launch");
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr1[fslot][0], s));
        if (rec && timed && ctx->sp_tune == 0) ctx->sp_tune = 1;  // auto: a shape's first frame (not measured)
        if (rec && timed && ctx->sp_tune == 2) {  // auto: this frame's time is the whole-chain side
            ctx->sp_tslot[0] = fslot;
            ctx->sp_tframe = ctx->frames;
            ctx->sp_tune = 3;
        }
        if (rec && ctx->sp_sig == sig) {  // how many pixels moved since last frame (mode word 0: count)
            int* cnt = (int*)ctx->spfixn.p + 1;
            a.sp_prev = sp_prev;
            HIPCHK(ctx, hipMemsetAsync(cnt, 0, 2 * sizeof(int), s));
            hipLaunchKernelGGL(ort_sample_moved, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, a, cnt);
            hipError_t e2;
            if ((e2 = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e2, "ort_sample_moved launch");
        }
    } else {
        int* fx = (int*)ctx->spfix.p;
        a.sp_prev = sp_prev;
        a.sp_cur = sp_cur;
        a.sp_col = (float*)ctx->spcol.p;
        a.fx_n = (int*)ctx->spfixn.p;
        a.fx_slot = fx;
        a.fx_s0 = fx + slots;
        a.fx_st = (float2*)(fx + 2 * slots);
        a.fx_col = (float*)(fx + 4 * slots);
        PipeArgs as = a;  // the samples: no fixup list; heavy blocks first by the lists the last
        as.fx_slot = nullptr;  // whole-chain frame of this shape wrote (read only: SPEC frames keep them)
        if (ORT_PIXEL_LPT && ctx->pp_sig == sig && ctx->pplist.p) {
            const size_t nbk = (size_t)blocks * (kBlock / 64);
            const int r = ctx->pp_par ^ 1;
            as.pl_stride = (int)nbk;
            as.pl_r = (int*)ctx->pplist.p + (size_t)r * kPixelClasses * nbk;
            as.pl_rcnt = (int*)ctx->ppcnt.p + kPixelClasses * r;
        }
        hipLaunchKernelGGL(ort_sample_decide, dim3(1), dim3(64), 0, s, a.sp_ctl, (long long)t->width * t->rows, kSpecMovedMax);
        hipError_t e = hipGetLastError();
        if (e != hipSuccess) return hip_fail(ctx, e, "ort_sample_decide launch");
        e = launch_pixel_paths<1>(ctx, mode, deep, lds_scene, lds, blocks * nch, as, s);
        if (e != hipSuccess) return hip_fail(ctx, e, "ort_pixel_paths (samples) launch");
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr1[fslot][0], s));
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr0[fslot][1], s));
        hipLaunchKernelGGL(ort_sample_resolve, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ort_sample_resolve launch");
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr1[fslot][1], s));
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr0[fslot][2], s));
        // the fixup list (the workgroups beyond what it needs leave at once); in a fall-back frame
        // every pixel's chain, then the count of the pixels that moved
        e = launch_pixel_paths<2>(ctx, mode, deep, lds_scene, lds, blocks, a, s);
        if (e != hipSuccess) return hip_fail(ctx, e, "ort_pixel_paths (fixup) launch");
        if (timed) HIPCHK(ctx, hipEventRecord(ctx->tr1[fslot][2], s));
        hipLaunchKernelGGL(ort_sample_moved, dim3((unsigned)((slots + 255) / 256)), dim3(256), 0, s, a, a.sp_ctl + 1);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ort_sample_moved launch");
        if (timed && ctx->sp_tune == 1) ctx->sp_tune = 2;  // auto: the first speculating frame (not measured)
        if (timed && ctx->sp_tune == 3) {  // auto: ... and this one's the speculating side
            ctx->sp_tslot[1] = fslot;
            ctx->sp_tune = 4;
        }
    }
    if (spec_on) {  // this frame's end states are the next frame's
        ctx->sp_par ^= 1;
        ctx->sp_sig = sig;
    }
    if (timed) {
        ctx->tseg[fslot] = nseg;
        ctx->frames += 1;
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev1, s));
    ctx->timed = true;
    ctx->sync_ok = true;
    return ORT_OK;
}

int render_impl(ort_ctx* ctx, const ort_params* p, const ort_tile* t, float* out, int out_is_device,
                void* stream, unsigned long long* dcounters) {
    const std::string bad = check_params(p, t);
    if (!bad.empty()) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_render: " + bad);
    if (!ctx->has_scene) return fail(ctx, ORT_ERR_NO_SCENE, "ort_render: no scene uploaded");
    const int mode = (p->use_octree == 1) ? (ctx->layout == ORT_LAYOUT_COMPACT ? 0 : 1) : 2;
    if (mode != 2 && ctx->n_nodes <= 0) return fail(ctx, ORT_ERR_NO_SCENE, "ort_render: scene has no octree");
    const size_t pix = (size_t)t->width * (size_t)t->rows;
    if (!out && pix > 0) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_render: null output");
    if (pix == 0) return ORT_OK;
    const int tilesX = (t->width + 15) / 16, tilesY = (t->rows + 15) / 16;
    // tile pairs (ORT_OPT_TILE_PAIRS; the compact layout, trees of 4+ levels: cost_order_pair's
    // scratch): the slot blocks of a pair are consecutive, a last odd column's second tile a hole
    // (auto: on large tiles, and on any tile whose caller turned the split walks off -- frames in
    // flight fill the tail, and pairs then pay on small tiles too: 1/4 band at 3 in flight +4 %)
    const bool pairs = mode == 0 && ctx->depth >= 4 &&
                       (ctx->tile_pairs > 0 ||
                        (ctx->tile_pairs < 0 && ((long long)pix >= kPairsAutoPixels || ctx->split_steps == 0)));
    const int gridX = pairs ? (tilesX + 1) / 2 : tilesX;
    const long long blocks = (long long)(pairs ? 2 * gridX : tilesX) * tilesY;
    if (blocks * kBlock > 0x7fffffffLL) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_render: tile too large");
    const size_t slots = (size_t)blocks * kBlock;
    HIPCHK(ctx, hipSetDevice(ctx->device));
    hipStream_t s = stream ? (hipStream_t)stream : ctx->stream;
    float* dout = out;
    int rc;
    if (!out_is_device) {
        if ((rc = ensure(ctx, ctx->scratch_out, 12 * pix))) return rc;
        dout = (float*)ctx->scratch_out.p;
    }
    const int ns = p->num_samples, maxd = p->max_depth;
    const bool direct = (ns == 1 && maxd == 1);
    if (!dcounters && use_pixel_paths(ctx, mode, ns, maxd)) {  // the frame in one launch
        if ((rc = ensure(ctx, ctx->defer_count, 128)) || (rc = render_pixel_paths(ctx, p, t, mode, dout, s))) return rc;
        if (!out_is_device) {
            HIPCHK(ctx, hipMemcpyAsync(out, dout, 12 * pix, hipMemcpyDeviceToHost, s));
            HIPCHK(ctx, hipStreamSynchronize(s));
        } else if (!stream) {
            HIPCHK(ctx, hipStreamSynchronize(s));
        }
        return ORT_OK;
    }
    if ((rc = ensure(ctx, ctx->hit, 8 * slots)) || (rc = ensure(ctx, ctx->defer_list, 4 * slots)) ||
        (rc = ensure(ctx, ctx->defer_count, 128)))
        return rc;
    if (!direct || ctx->persistent) {
        if ((rc = ensure(ctx, ctx->po, 16 * slots)) || (rc = ensure(ctx, ctx->pd, 16 * slots)) ||
            (rc = ensure(ctx, ctx->prng, 8 * slots)) || (rc = ensure(ctx, ctx->pc, 16 * slots)) ||
            (rc = ensure(ctx, ctx->pcol, 16 * slots)))
            return rc;
    }
    const bool pers_bounce = ctx->persistent == 2;  // persistent only for the bounce >= 1 lists
    const bool compact = !direct && p->max_depth > 1;
    // primary-ray mode (1 sample, 1 bounce) on the compact layout: the trace kernels shade
    const bool fuse = direct && mode == 0;
    const bool sorted = compact && ctx->sort_paths == 1;   // radix sort of every slot's key
    const bool listsort = compact && ctx->sort_paths == 2; // sort of the appended list (its length read back)
    // bounce 0 of a multi-bounce frame: the trace kernels shade their camera rays into the path
    // state and append the paths that go on (no hit records, no shade launch: C5 -0.7 ms)
    const bool fuse_first = compact && !sorted && mode == 0 && !dcounters;
    size_t qtemp_bytes = 0;
    if (compact) {
        qtemp_bytes = (sorted || listsort) ? ort::sortAliveTempBytes((int)slots) : 0;
        if ((rc = ensure(ctx, ctx->qlist, 4 * slots)) || (rc = ensure(ctx, ctx->qlist2, 4 * slots)) ||
            (rc = ensure(ctx, ctx->qcount, 64)) ||
            (rc = ensure(ctx, ctx->qtemp, std::max<size_t>(qtemp_bytes, 16))))
            return rc;
        if (sorted && ((rc = ensure(ctx, ctx->skeys, 4 * slots)) || (rc = ensure(ctx, ctx->skeys2, 4 * slots)) ||
                       (rc = ensure(ctx, ctx->svals, 4 * slots))))
            return rc;
        if (listsort && ((rc = ensure(ctx, ctx->skeys, 4 * slots)) || (rc = ensure(ctx, ctx->skeys2, 4 * slots)) ||
                         (rc = ensure(ctx, ctx->svals, 4 * slots))))
            return rc;
        if (listsort) {  // the list-length hints belong to one frame shape and scene
            const unsigned long long sig = frame_sig(ctx, p, t);
            if (sig != ctx->hint_sig) {
                int bank = -1;
                for (int i = 1; i <= ort_ctx::kHintBanks && bank < 0; ++i) {
                    const int c = (ctx->hint_bank + i) % ort_ctx::kHintBanks;
                    if (!ctx->hint_ev_used[c] || hipEventQuery(ctx->hint_ev[c]) == hipSuccess) bank = c;
                }
                if (bank < 0) {  // every bank still awaits copies (several shape changes in flight)
                    bank = (ctx->hint_bank + 1) % ort_ctx::kHintBanks;
                    HIPCHK(ctx, hipEventSynchronize(ctx->hint_ev[bank]));
                }
                ctx->hint_bank = bank;
                for (int i = 0; i < ort_ctx::kHints; ++i) ctx->alive_host[bank * ort_ctx::kHints + i] = -1;
                ctx->hint_sig = sig;
            }
        }
        if (sorted || listsort) {  // the key tables of the current root box (built once per scene)
            const float box[6] = {ctx->root_lo[0], ctx->root_lo[1], ctx->root_lo[2],
                                  ctx->root_hi[0], ctx->root_hi[1], ctx->root_hi[2]};
            if (!ctx->key_spread.p || std::memcmp(box, ctx->spread_box, sizeof box) != 0) {
                if ((rc = ensure(ctx, ctx->key_spread, 4 * (size_t)ort::kSpreadWords))) return rc;
                std::vector<uint32_t> tab((size_t)ort::kSpreadWords);
                ort::mortonSpread(ort::mortonPlan(ctx->root_lo, ctx->root_hi), tab.data());
                HIPCHK(ctx, hipMemcpy(ctx->key_spread.p, tab.data(), 4 * tab.size(), hipMemcpyHostToDevice));
                std::memcpy(ctx->spread_box, box, sizeof box);
            }
        }
    }
    PipeArgs a;
    std::memset(&a, 0, sizeof(a));
    a.pp = pixel_params(p);
    a.S = device_scene(ctx);
    a.tm = {t->x0, t->width, t->y0, t->rows, t->band_height, t->band_stride};
    a.tilesX = gridX;
    a.pair = pairs ? 1 : 0;
    a.tilesY = tilesY;
    a.swizzle = ctx->xcd_swizzle >= 0 ? ctx->xcd_swizzle : ((!pairs && (long long)pix <= kRasterAutoPixels) ? 0 : 2);
    a.xrun_log2 = xcd_run_log2(gridX);
    a.total = (int)slots;
    a.exact_only = ctx->exact_only || !ctx->ordered;
    a.refill = ctx->refill;
    a.hit = (int2*)ctx->hit.p;
    a.defer_list = (int*)ctx->defer_list.p;
    // two sets of 16 counters (deferred count, persistent cursor, heavy list): a launch uses one
    // and its exact kernel zeroes the other for the next launch; a memset re-zeroes both after a
    // failed render or a new buffer (sync_ok)
    if (!ctx->sync_ok) {
        HIPCHK(ctx, hipMemsetAsync(ctx->defer_count.p, 0, 128, s));
        ctx->sync_set = 0;
        ctx->pre_ok = false;  // a failed render may not have listed the next frame's heavy rays
    }
    ctx->sync_ok = false;  // until this render has enqueued all its launches
    a.sync = (int*)ctx->defer_count.p;
    a.po = (float4*)ctx->po.p;
    a.pd = (float4*)ctx->pd.p;
    a.pc = (float4*)ctx->pc.p;
    a.prng = (float2*)ctx->prng.p;
    a.pcol = (float4*)ctx->pcol.p;
    a.out = dout;
    a.counters = dcounters;
#if ORT_ANALYSIS
    a.wclock = (ulonglong4*)ctx->wclock;
    a.wclock_n = (int)ctx->wclock_n;
#endif
    a.mp = ort::mortonPlan(ctx->root_lo, ctx->root_hi);
    // with bounce 0 shaded in the trace kernels every pixel's path ends in a kernel that knows
    // its pixel, so the last sample writes the final pixels itself (no finalize pass)
    a.final_out = fuse_first ? 1 : 0;
    a.key_spread = (const uint32_t*)ctx->key_spread.p;
    // the cost order: the per-workgroup camera-ray kernels (ort_trace_compact[_deep]) only
    // the camera moved since this context's last rendered frame (counting renders leave the
    // record alone): heavy priority here and heavy-first's bounce classes below both gate on it,
    // whether or not the cost order is on
    const bool cam_moved = mode == 0 && std::memcmp(&ctx->prio_cam, &a.pp.cam, sizeof(ort::KCamera)) != 0;
    if (mode == 0 && !dcounters) ctx->prio_cam = a.pp.cam;
    if (mode == 0 && ctx->cost_order && ctx->depth >= 2) {
        if ((rc = ensure(ctx, ctx->pcost, 2 * slots))) return rc;
        const unsigned long long sig = frame_sig(ctx, p, t);
        if (sig != ctx->cost_sig) {  // a new shape: tile order for the first frame
            HIPCHK(ctx, hipMemsetAsync(ctx->pcost.p, 0, 2 * slots, s));
            ctx->cost_sig = sig;
        }
        a.pcost = (uint16_t*)ctx->pcost.p;
        // heavy priority only for a camera that has not moved since this context's last frame:
        // after a move the per-slot steps are one frame stale (a pixel's walk cost follows its
        // pixel-seeded lens/jitter sample more than the scene: same-slot hints keep an in-block
        // correlation of 0.82 with the new walks, reprojected ones 0.05 -- profiles/r05_moving_*),
        // and raising the wrong waves costs: C3 moving frames 1.855 -> 1.798 ms without it
        // (profiles/r05_moving_shift_c3.log), static frames unchanged
        a.prio_steps = cam_moved ? 0 : ctx->heavy_prio;
    }
    // split walks of the heavy camera rays (1 sample; the production kernels, bounce 0)
    const int split_steps = ctx->split_steps >= 0 ? ctx->split_steps
                                                  : ((long long)pix <= kSplitAutoPixels ? kSplitAutoSteps : 0);
    const bool split = (fuse || fuse_first) && a.pcost && split_steps > 0 && !dcounters && ns == 1;
    if (!split) ctx->pre_ok = false;  // (a queued heavy list is only for the next split frame)
    if (split) {
        if (!ctx->aux_stream) HIPCHK(ctx, hipStreamCreateWithFlags(&ctx->aux_stream, hipStreamNonBlocking));
        if ((rc = ensure(ctx, ctx->hbits, 4 * (slots / 32 + 1))) || (rc = ensure(ctx, ctx->hlist, 4 * (size_t)ort_ctx::kSplitCap)) ||
            (rc = ensure(ctx, ctx->hcnt, 64)))
            return rc;
        a.hlist = (const int*)ctx->hlist.p;
        a.hcap = ort_ctx::kSplitCap;
        // the subtrees dealt to the lanes: ~5 levels above the leaves (a depth-8 tree: level 3)
        a.split_level = ctx->split_level > 0 ? ctx->split_level : std::max(1, ctx->depth - 5);
    }
    // heavy first: the bounce >= 1 lists of the persistent trace (sorted, default path)
    const int nbc = std::min(ns * (maxd > 0 ? maxd : 1), ort_ctx::kCostBounces);  // recorded bounce indices
    uint16_t* bcost = nullptr;
    if (listsort && mode == 0 && pers_bounce && ctx->heavy_first > 0) {
        if ((rc = ensure(ctx, ctx->bcost, 2 * slots * (size_t)nbc))) return rc;
        const unsigned long long sig = frame_sig(ctx, p, t);
        if (sig != ctx->bcost_sig) {  // a new shape: no heavy walks known
            HIPCHK(ctx, hipMemsetAsync(ctx->bcost.p, 0, 2 * slots * (size_t)nbc, s));
            ctx->bcost_sig = sig;
        }
        bcost = (uint16_t*)ctx->bcost.p;
        a.heavy = ctx->heavy_first;
    }
    // ... whose classes are read only while the camera stands still (the steps are recorded
    // always): after a move last frame's bounce walks are not this frame's, and sorting stale
    // heavy paths first cost C5's moving frames 0.8 % (1568 -> 1556 Mrays/s, bench --opt HEAVY_FIRST=0)
#ifndef ORT_HEAVY_FIRST_STATIC_ONLY
#define ORT_HEAVY_FIRST_STATIC_ONLY 1
#endif
#ifndef ORT_GEO_ALWAYS
#define ORT_GEO_ALWAYS 0  // analysis: the rays' own classes on every frame (tools/ab_stream.py)
#endif
    const uint16_t* bcost_rd = ((ORT_HEAVY_FIRST_STATIC_ONLY && cam_moved) || ORT_GEO_ALWAYS) ? nullptr : bcost;
#ifndef ORT_GEO_HEAVY
#define ORT_GEO_HEAVY 1
#endif
    if (ORT_GEO_HEAVY && bcost && !bcost_rd) {  // moved: classes from the rays themselves (geo_class_bits)
        a.geo_heavy = 1;
        float m = 3.0e38f;
        for (int q = 0; q < 3; ++q) {
            a.gbox[q] = ctx->root_lo[q];
            a.gbox[3 + q] = ctx->root_hi[q];
            m = std::min(m, ctx->root_hi[q] - ctx->root_lo[q]);
        }
#ifndef ORT_GEO_T
#define ORT_GEO_T 1.2f, 2.7f, 6.8f  // the class thresholds, in units of the box's smallest extent
#endif
        const float gt[3] = {ORT_GEO_T};
        for (int q = 0; q < 3; ++q) a.gthr[q] = gt[q] * m;
    }
    const int key_bits = bcost ? ort::kPathKeyBits + kHeavyKeyBits : ort::kPathKeyBits;
    const size_t lds = lds_bytes(mode, ctx->depth, false);
    const size_t lds_exact = lds_bytes(mode, ctx->depth, true);
    const int pblocks = (mode == 0 && ctx->persistent) ? persistent_blocks(ctx->device, dcounters != nullptr, ctx->depth > 8, ctx->depth, lds, blocks) : 0;
    // the exact kernel: a grid-stride loop over the (usually no) deferred rays; a small grid
    // dispatches fast
    const int exact_blocks = 256;
    hipError_t e;
    const int fslot = (int)(ctx->frames % ort_ctx::kRing);  // this frame's timing slot
    ctx->tseg[fslot] = 0;
    // the frame's start: also the start of its first trace launch when that is timed (nothing is
    // enqueued between them), which saves an event packet per frame (~1 % of a 1/8 band frame)
    const bool no_times = (ctx->debug_flags & 1) || !ctx->launch_times;  // no per-launch events
    const bool start_is_tr0 = maxd > 0 && !no_times;
    ctx->ev0_last = start_is_tr0 ? ctx->tr0[fslot][0] : ctx->ev0;
    HIPCHK(ctx, hipEventRecord(ctx->ev0_last, s));
    for (int smp = 0; smp < ns; ++smp) {
        a.sample = smp;
        a.qlist = nullptr;  // bounce 0: every slot
        a.qcount = nullptr;
        // the alive paths of the current bounce in append order, and the buffer the next
        // bounce's are appended to: qbuf[cur] / qcnt[cur] and qbuf[cur ^ 1] / qcnt[cur ^ 1]
        int* qbuf[2] = {(int*)ctx->qlist.p, (int*)ctx->qlist2.p};
        int* qcnt[2] = {(int*)ctx->qcount.p, (int*)ctx->qcount.p + 4};
        int cur = 1;  // bounce 0 appends to qbuf[0]
        const int bounces = maxd > 0 ? maxd : 1;
        a.nobounce = maxd <= 0;
        for (int b = 0; b < bounces; ++b) {
            a.last = (b == bounces - 1);
            const int fmode = fuse ? 1 : ((b == 0 && fuse_first) ? 2 : 0);
            if (!a.nobounce) {
                {   // this launch's counter set; mode 0 launches ort_trace_exact, which zeroes the other
                    int* const set = (int*)ctx->defer_count.p + 16 * ctx->sync_set;
                    a.sync = set;
                    if (mode == 0) a.sync_next = (int*)ctx->defer_count.p + 16 * (ctx->sync_set ^ 1);
                    else HIPCHK(ctx, hipMemsetAsync(set, 0, 64, s));
                }
                const int slot = fslot;
                const int seg = ctx->tseg[slot];
                // every trace launch of the frame, up to kSeg (analysis flag 1: none)
                const bool timed = seg < ort_ctx::kSeg && !no_times;
                if (timed && !ctx->tr0[slot][seg]) {
                    HIPCHK(ctx, hipEventCreate(&ctx->tr0[slot][seg]));
                    HIPCHK(ctx, hipEventCreate(&ctx->tr1[slot][seg]));
                }
                if (timed && !(seg == 0 && start_is_tr0)) HIPCHK(ctx, hipEventRecord(ctx->tr0[slot][seg], s));
                const bool prim = b == 0;
                const int pb = (pers_bounce && b > 0) ? pblocks : 0;
                PipeArgs at = a;
#if ORT_ANALYSIS
                if (pb > 0 && a.wclock) {  // analysis (ORT_PERSIST_CLOCK): a record range per launch
                    const long long nw = (long long)pb * (ctx->depth > 8 ? kPersistDeepBlock : kBlock) / 64 *
                                         (ORT_PERSIST_STATS ? 2 : 1);  // records per launch
                    at.wclock = (seg + 1) * nw <= ctx->wclock_n ? a.wclock + seg * nw : nullptr;
                    at.wclock_n = (int)nw;
                }
#endif
                if (fmode == 2) {  // the trace kernels append bounce 1's list (as ort_shade_kernel would)
                    HIPCHK(ctx, hipMemsetAsync(qcnt[cur ^ 1], 0, sizeof(int), s));
                    at.qnext = qbuf[cur ^ 1];
                    at.qnext_count = qcnt[cur ^ 1];
                    at.qnext_keys = listsort ? (uint32_t*)ctx->skeys.p : nullptr;
                }
                {   // heavy first: record index smp * bounces + b (bounces >= 1 only)
                    const int hi = smp * bounces + b;
                    if (bcost && pb > 0 && b > 0 && hi < nbc) at.bcost_w = bcost + (size_t)hi * slots;
                    if (bcost_rd && fmode == 2 && hi + 1 < nbc && b + 1 < bounces) at.bcost_r = bcost_rd + (size_t)(hi + 1) * slots;
                }
                const bool do_split = split && (fmode == 1 || fmode == 2);
                const unsigned long long fsig = do_split ? frame_sig(ctx, p, t) : 0ull;
                if (do_split) {
                    // the heavy rays of this frame (last frame's steps) -- listed by the scan the last
                    // frame of this shape queued on the second stream, or by one here -- then their
                    // split walks there, beside the per-tile kernel (which passes over them)
                    const bool pre = ctx->pre_ok && ctx->pre_sig == fsig && ctx->pre_steps == split_steps &&
                                     !(ctx->debug_flags & 2);
                    ctx->pre_ok = false;
                    int* hc = (int*)ctx->hcnt.p;
                    // the second stream follows this one up to here: with shading fused (1 bounce)
                    // nothing of this frame precedes the split walks on it but ev0 (event packets
                    // cost the frame ~1 % each); bounce 0 of a longer path needs the list memset too
                    if (fmode == 1) {
                        HIPCHK(ctx, hipStreamWaitEvent(ctx->aux_stream, ctx->ev0_last, 0));
                    } else {
                        HIPCHK(ctx, hipEventRecord(ctx->ev_scan, s));
                        HIPCHK(ctx, hipStreamWaitEvent(ctx->aux_stream, ctx->ev_scan, 0));
                    }
                    if (!pre) {  // (with pre, the last frame's exact kernel listed them, in this stream's order)
                        HIPCHK(ctx, hipMemsetAsync(hc, 0, 64, ctx->aux_stream));
                        ctx->hpar = 0;
                        const HeavyScan H{(const uint16_t*)a.pcost, (int)slots, split_steps, ort_ctx::kSplitCap,
                                          (uint32_t*)ctx->hbits.p, (int*)ctx->hlist.p, hc};
                        hipLaunchKernelGGL(k_heavy_scan, dim3((unsigned)((slots + 4095) / 4096)), dim3(kBlock), 0,
                                           ctx->aux_stream, H);
                        HIPCHK(ctx, hipGetLastError());
                        HIPCHK(ctx, hipEventRecord(ctx->ev_pre, ctx->aux_stream));
                        HIPCHK(ctx, hipStreamWaitEvent(s, ctx->ev_pre, 0));  // the tile kernel reads hbits
                    }
                    at.hsync = hc + 8 * ctx->hpar;
                    at.hsync_next = hc + 8 * (ctx->hpar ^ 1);
#ifndef ORT_SPLIT_BLOCKS
#define ORT_SPLIT_BLOCKS 32
#endif
                    const int hblocks = ORT_SPLIT_BLOCKS;  // 1024 heavy rays in flight; more loop
                    const dim3 hg(hblocks), ht(kBlock);
                    if (ctx->depth > 8 && fmode == 1) hipLaunchKernelGGL((ort_trace_split<true, 1>), hg, ht, lds, ctx->aux_stream, at);
                    else if (ctx->depth > 8) hipLaunchKernelGGL((ort_trace_split<true, 2>), hg, ht, lds, ctx->aux_stream, at);
                    else if (fmode == 1) hipLaunchKernelGGL((ort_trace_split<false, 1>), hg, ht, lds, ctx->aux_stream, at);
                    else hipLaunchKernelGGL((ort_trace_split<false, 2>), hg, ht, lds, ctx->aux_stream, at);
                    HIPCHK(ctx, hipGetLastError());
                    HIPCHK(ctx, hipEventRecord(ctx->ev_split, ctx->aux_stream));
                    at.hbits = (const uint32_t*)ctx->hbits.p;
                }
                const int tblocks = (prim && pairs) ? (int)(blocks / 2) : (int)blocks;  // a workgroup per tile pair
                e = dcounters ? launch_trace<true>(mode, prim, at, tblocks, pb, lds, s, fmode)
                              : launch_trace<false>(mode, prim, at, tblocks, pb, lds, s, fmode);
                if (e != hipSuccess) return hip_fail(ctx, e, "trace kernel launch");
                if (do_split) {
                    HIPCHK(ctx, hipStreamWaitEvent(s, ctx->ev_split, 0));  // joined before the exact kernel
                    if (timed) {
                        HIPCHK(ctx, hipEventRecord(ctx->tr1[slot][seg], s));
                        ctx->tseg[slot] = seg + 1;
                    }
                    // the exact kernel also lists the next frame's heavy rays, from this frame's
                    // steps (final now) -- no scan launch or cross-stream wait opens the next frame;
                    // ort_trace_split zeroed the other count pair
                    ctx->hpar ^= 1;
                    at.scan_pcost = a.pcost;
                    at.scan_T = split_steps;
                    at.scan_bits = (uint32_t*)ctx->hbits.p;
                    at.scan_list = (int*)ctx->hlist.p;
                    at.scan_count = (int*)ctx->hcnt.p + 8 * ctx->hpar;
                    ctx->pre_sig = fsig;
                    ctx->pre_steps = split_steps;
                } else if (timed) {
                    HIPCHK(ctx, hipEventRecord(ctx->tr1[slot][seg], s));
                    ctx->tseg[slot] = seg + 1;
                }
                if (mode == 0) {
                    const bool prim = b == 0;
                    const dim3 g(exact_blocks), t(kBlock);
                    if (dcounters && fuse) hipLaunchKernelGGL((ort_trace_exact<true, true, 1>), g, t, lds_exact, s, at);
                    else if (dcounters && prim) hipLaunchKernelGGL((ort_trace_exact<true, true, 0>), g, t, lds_exact, s, at);
                    else if (dcounters) hipLaunchKernelGGL((ort_trace_exact<true, false, 0>), g, t, lds_exact, s, at);
                    else if (fuse) hipLaunchKernelGGL((ort_trace_exact<false, true, 1>), g, t, lds_exact, s, at);
                    else if (fmode == 2) hipLaunchKernelGGL((ort_trace_exact<false, true, 2>), g, t, lds_exact, s, at);
                    else if (prim) hipLaunchKernelGGL((ort_trace_exact<false, true, 0>), g, t, lds_exact, s, at);
                    else hipLaunchKernelGGL((ort_trace_exact<false, false, 0>), g, t, lds_exact, s, at);
                    if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ort_trace_exact launch");
                    ctx->sync_set ^= 1;  // it zeroes the other set for the next launch
                    // it listed the next frame's heavy rays: only now may that frame skip its scan
                    if (do_split) ctx->pre_ok = true;
                }
            }
            if (!fuse && fmode != 2) {
                // bounce >= 1: the bounce's alive paths in APPEND order (about slot order: the
                // path-state reads and writes coalesce; the sorted trace list scattered them, C5
                // 65.4 -> 63.0 ms) -- or, with the every-slot sort (sort_paths 1), every slot
                PipeArgs a2 = a;
                a2.qlist = nullptr;
                a2.qcount = nullptr;
                if (compact && !sorted && b > 0) {
                    a2.qlist = qbuf[cur];
                    a2.qcount = qcnt[cur];
                }
                if (compact && !sorted && !a.nobounce && b + 1 < bounces) {
                    // the compaction: the shade kernel appends the paths that go on, one atomic
                    // per workgroup (a separate rocprim::select pass over the slots cost 0.55 ms
                    // per C5 bounce), into the other list buffer
                    HIPCHK(ctx, hipMemsetAsync(qcnt[cur ^ 1], 0, sizeof(int), s));
                    a2.qnext = qbuf[cur ^ 1];
                    a2.qnext_count = qcnt[cur ^ 1];
                    a2.qnext_keys = listsort ? (uint32_t*)ctx->skeys.p : nullptr;
                    const int hn = smp * bounces + b + 1;  // the next bounce's record
                    if (bcost_rd && hn < nbc) a2.bcost_r = bcost_rd + (size_t)hn * slots;
                }
                e = launch_shade(mode, b == 0, direct, a2, (int)blocks, s);
                if (e != hipSuccess) return hip_fail(ctx, e, "ort_shade_kernel launch");
            }
            if (compact && !a.nobounce && b + 1 < bounces) {  // the next bounce walks only the alive paths
                if (sorted) {
                    const ort::SortBuffers sb{(uint32_t*)ctx->skeys.p, (uint32_t*)ctx->skeys2.p, (int*)ctx->svals.p,
                                              (int*)ctx->qlist.p};
                    e = ort::sortAlive(ctx->qtemp.p, qtemp_bytes, (const float4*)ctx->po.p, (const float4*)ctx->pd.p,
                                       (int)slots, ctx->root_lo, ctx->root_hi, (const uint32_t*)ctx->key_spread.p, sb,
                                       (int*)ctx->qcount.p, s);
                    if (e != hipSuccess) return hip_fail(ctx, e, "path compaction");
                }  // else the shade kernel appended them
                if (sorted) {
                    a.qlist = (const int*)ctx->qlist.p;
                    a.qcount = (const int*)ctx->qcount.p;
                } else {
                    cur ^= 1;  // the list just appended is the next bounce's
                    if (listsort) {
                        // sort only about the alive paths, not every slot (C5: 36.6 M keys, not
                        // 99.6 M), without reading the length back: the bound is this bounce's
                        // length in an earlier frame of the same shape plus 1/64 + 1024 (the
                        // same camera gives the same length), every slot when there is none
                        const int hi = smp * bounces + b;
                        long long bound = (long long)slots;
                        if (ctx->sort_bound > 0) bound = ctx->sort_bound;
                        else if (hi < ort_ctx::kHints) {
                            const int h = ((volatile int*)ctx->alive_host)[ctx->hint_bank * ort_ctx::kHints + hi];
                            if (h >= 0) bound = (long long)h + (h >> 6) + 1024;
                        }
                        bound = std::min<long long>(bound, (long long)slots);
                        // (key, path) pairs as the shade / trace kernels appended them
                        const ort::SortBuffers sb{(uint32_t*)ctx->skeys.p, (uint32_t*)ctx->skeys2.p, qbuf[cur],
                                                  (int*)ctx->svals.p};
                        e = ort::sortListBounded(ctx->qtemp.p, qtemp_bytes, (int)bound, qcnt[cur], sb, s, key_bits);
                        if (e != hipSuccess) return hip_fail(ctx, e, "path list sort");
                        if (hi < ort_ctx::kHints)  // the next frame's bound (pinned: no host wait)
                            HIPCHK(ctx, hipMemcpyAsync(ctx->alive_host + ctx->hint_bank * ort_ctx::kHints + hi, qcnt[cur], sizeof(int),
                                                       hipMemcpyDeviceToHost, s));
                    }
                    a.qlist = listsort ? (const int*)ctx->svals.p : qbuf[cur];
                    a.qcount = qcnt[cur];
                }
            }
        }
    }
    if (ctx->tseg[fslot] > 0) ctx->frames += 1;
    if (listsort) {  // after this frame's hint copies: the bank is free once this completes
        HIPCHK(ctx, hipEventRecord(ctx->hint_ev[ctx->hint_bank], s));
        ctx->hint_ev_used[ctx->hint_bank] = true;
    }
    if (!direct && !a.final_out) {
        hipLaunchKernelGGL(ort_finalize_kernel, dim3((unsigned)blocks), dim3(kBlock), 0, s, a);
        if ((e = hipGetLastError()) != hipSuccess) return hip_fail(ctx, e, "ort_finalize_kernel launch");
    }
    HIPCHK(ctx, hipEventRecord(ctx->ev1, s));
    ctx->timed = true;
    ctx->sync_ok = true;  // every launch enqueued: the counter sets are in step again
    if (!out_is_device) {
        HIPCHK(ctx, hipMemcpyAsync(out, dout, 12 * pix, hipMemcpyDeviceToHost, s));
        HIPCHK(ctx, hipStreamSynchronize(s));
    } else if (!stream) {
        HIPCHK(ctx, hipStreamSynchronize(s));
    }
    return ORT_OK;
}

}  // namespace

extern "C" {

int ort_create(int device, ort_ctx** out) {
    if (!out) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_create: null out");
    *out = nullptr;
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) return hip_fail(nullptr, e, "hipGetDeviceCount");
    if (device < 0 || device >= n)
        return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_create: device " + std::to_string(device) + " not present (" +
                                                      std::to_string(n) + " visible)");
    ort_ctx* c = new (std::nothrow) ort_ctx();
    if (!c) return fail(nullptr, ORT_ERR_OUT_OF_MEMORY, "ort_create: out of host memory");
    c->device = device;
    if ((e = hipSetDevice(device)) != hipSuccess || (e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipEventCreate(&c->ev0)) != hipSuccess || (e = hipEventCreate(&c->ev1)) != hipSuccess) {
        const int rc = hip_fail(nullptr, e, "ort_create");
        delete c;
        return rc;
    }
    for (int i = 0; i < ort_ctx::kRing; ++i) {
        if ((e = hipEventCreate(&c->tr0[i][0])) != hipSuccess || (e = hipEventCreate(&c->tr1[i][0])) != hipSuccess) {
            const int rc = hip_fail(nullptr, e, "ort_create: events");
            ort_destroy(c);
            return rc;
        }
    }
    if ((e = hipHostMalloc((void**)&c->alive_host, sizeof(int) * ort_ctx::kHints * ort_ctx::kHintBanks,
                           hipHostMallocDefault)) != hipSuccess) {
        c->alive_host = nullptr;
        const int rc = hip_fail(nullptr, e, "ort_create: pinned hint buffer");
        ort_destroy(c);
        return rc;
    }
    for (int i = 0; i < ort_ctx::kHints * ort_ctx::kHintBanks; ++i) c->alive_host[i] = -1;
    for (int i = 0; i < ort_ctx::kHintBanks; ++i)
        if ((e = hipEventCreateWithFlags(&c->hint_ev[i], hipEventDisableTiming)) != hipSuccess) {
            const int rc = hip_fail(nullptr, e, "ort_create: hint events");
            ort_destroy(c);
            return rc;
        }
    // (the second stream itself is created with the first split frame: a stream takes one of the
    // process's few hardware queues, and contexts that never split -- group ranks sharing a
    // device -- should not crowd the others' queues)
    if ((e = hipEventCreateWithFlags(&c->ev_scan, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_split, hipEventDisableTiming)) != hipSuccess ||
        (e = hipEventCreateWithFlags(&c->ev_pre, hipEventDisableTiming)) != hipSuccess) {
        const int rc = hip_fail(nullptr, e, "ort_create: second stream");
        ort_destroy(c);
        return rc;
    }
    *out = c;
    return ORT_OK;
}

int ort_destroy(ort_ctx* ctx) {
    if (!ctx) return ORT_OK;
    (void)hipSetDevice(ctx->device);
    if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
    free_scene(ctx);
    free_buf(ctx->scratch_out);
    free_buf(ctx->counters);
    DevBuf* pipe[] = {&ctx->hit, &ctx->defer_list, &ctx->defer_count, &ctx->po, &ctx->pd, &ctx->pc, &ctx->prng, &ctx->pcol,
                      &ctx->qlist, &ctx->qlist2, &ctx->qcount, &ctx->qtemp, &ctx->skeys, &ctx->skeys2, &ctx->svals, &ctx->key_spread,
                      &ctx->pcost, &ctx->bcost, &ctx->hbits, &ctx->hlist, &ctx->hcnt, &ctx->pplist, &ctx->ppcnt, &ctx->ppcost, &ctx->spst, &ctx->spcol, &ctx->spfix, &ctx->spfixn};
    for (DevBuf* b : pipe) free_buf(*b);
    if (ctx->ev0) (void)hipEventDestroy(ctx->ev0);
    if (ctx->ev1) (void)hipEventDestroy(ctx->ev1);
    for (int i = 0; i < ort_ctx::kRing; ++i)
        for (int j = 0; j < ort_ctx::kSeg; ++j) {
            if (ctx->tr0[i][j]) (void)hipEventDestroy(ctx->tr0[i][j]);
            if (ctx->tr1[i][j]) (void)hipEventDestroy(ctx->tr1[i][j]);
        }
    if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    if (ctx->alive_host) (void)hipHostFree(ctx->alive_host);
    for (hipEvent_t ev : ctx->hint_ev)
        if (ev) (void)hipEventDestroy(ev);
    if (ctx->aux_stream) {
        (void)hipStreamSynchronize(ctx->aux_stream);
        (void)hipStreamDestroy(ctx->aux_stream);
    }
    if (ctx->ev_scan) (void)hipEventDestroy(ctx->ev_scan);
    if (ctx->ev_split) (void)hipEventDestroy(ctx->ev_split);
    if (ctx->ev_pre) (void)hipEventDestroy(ctx->ev_pre);
    delete ctx;
    return ORT_OK;
}

const char* ort_last_error(const ort_ctx* ctx) { return ctx ? ctx->err.c_str() : ort::thread_error(); }

int ort_set_option(ort_ctx* ctx, int option, int value) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_set_option: null ctx");
    if (option == ORT_OPT_FORCE_LAYOUT) {
        if (value < -1 || value > ORT_LAYOUT_EXPLICIT) return fail(ctx, ORT_ERR_INVALID_ARG, "bad layout");
        ctx->force_layout = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_PERSISTENT) {
        if (value == 1)  // removed in round 4
            return fail(ctx, ORT_ERR_UNSUPPORTED, "ORT_OPT_PERSISTENT 1 (every trace persistent) was removed (C5 -19 %)");
        if (value != 0 && value != 2) return fail(ctx, ORT_ERR_INVALID_ARG, "persistent must be 0 or 2");
        ctx->persistent = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_KID_SKIP) {
        if (value < 0 || value > 2) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_KID_SKIP: 0, 1 or 2");
        ctx->kid_skip = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_XCD_SWIZZLE) {
        if (value < -1 || value > 2) return fail(ctx, ORT_ERR_INVALID_ARG, "xcd swizzle must be -1 (auto), 0, 1 or 2");
        ctx->xcd_swizzle = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_SORT_PATHS) {
        if (value < 0 || value > 2) return fail(ctx, ORT_ERR_INVALID_ARG, "sort_paths must be 0, 1 or 2");
        ctx->sort_paths = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_HEAVY_FIRST) {
        if (value < 0 || value > 65535) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_HEAVY_FIRST: 0 (off) .. 65535 steps");
        ctx->heavy_first = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_TILE_PAIRS) {
        if (value < -1 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_TILE_PAIRS: -1 (auto), 0 or 1");
        ctx->tile_pairs = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_SPLIT_HEAVY) {
        if (value < -1 || value > 65535) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_SPLIT_HEAVY: -1 (auto), 0 (off) .. 65535 steps");
        ctx->split_steps = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_SPLIT_LEVEL) {
        if (value < 0 || value > ORT_COMPACT_MAX_DEPTH) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_SPLIT_LEVEL: 0 (auto) .. 10");
        ctx->split_level = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_PIXEL_PATHS) {
        if (value < -1 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_PIXEL_PATHS: -1 (auto), 0 or 1");
        ctx->pixel_paths = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_PIXEL_SPECULATE) {
        if (value < -1 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_PIXEL_SPECULATE: -1 (auto), 0 or 1");
        ctx->pixel_spec = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_PIXEL_HEAVY_FIRST) {
        if (value < -1 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_PIXEL_HEAVY_FIRST: -1 (auto), 0 or 1");
        ctx->pixel_heavy_first = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_PIXEL_LDS_SCENE) {
        if (value < 0 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_PIXEL_LDS_SCENE: 0 or 1");
        ctx->pixel_lds_scene = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_LAUNCH_TIMES) {
        if (value < 0 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_LAUNCH_TIMES: 0 or 1");
        ctx->launch_times = value;
        return ORT_OK;
    }
#if ORT_ANALYSIS
    if (option == ORT_OPT_DEBUG_FLAGS) {  // analysis: 1 no trace-timing events, 2 no queued heavy scan
        if (value < 0 || value > 3) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_DEBUG_FLAGS: 0 .. 3");
        ctx->debug_flags = value;
        return ORT_OK;
    }
#else
    if (option == ORT_OPT_DEBUG_FLAGS)
        return fail(ctx, ORT_ERR_UNSUPPORTED, "ORT_OPT_DEBUG_FLAGS: analysis library only (libort_analysis.so)");
#endif
    if (ORT_OPT_IS_RETIRED(option))  // removed options
        return fail(ctx, ORT_ERR_UNSUPPORTED, "option " + std::to_string(option) + " is retired (" +
                                                  (option == 5 ? "packet walk" : option == 7 ? "wave queue"
                                                                                             : "longest-first workgroups") +
                                                  ": measured slower, DESIGN.md 4)");
    if (option == ORT_OPT_HEAVY_PRIO) {
        if (value < 0 || value > 65535) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_HEAVY_PRIO: 0 (off) .. 65535 steps");
        ctx->heavy_prio = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_COST_ORDER) {
        if (value < 0 || value > 1) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_COST_ORDER: 0 or 1");
        ctx->cost_order = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_SORT_BOUND) {
        if (value < 0) return fail(ctx, ORT_ERR_INVALID_ARG, "ORT_OPT_SORT_BOUND must be >= 0");
        ctx->sort_bound = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_REFILL) {
        if (value < 1 || value > 64) return fail(ctx, ORT_ERR_INVALID_ARG, "refill must be 1..64");
        ctx->refill = value;
        return ORT_OK;
    }
    if (option == ORT_OPT_EXACT_TRAVERSAL) {
        ctx->exact_only = value ? 1 : 0;
        return ORT_OK;
    }
    return fail(ctx, ORT_ERR_INVALID_ARG, "unknown option");
}

int ort_upload_scene(ort_ctx* ctx, const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                     const float* node_min, const float* node_max, const int32_t* co, const int32_t* oo,
                     const int32_t* cnt, int32_t n_nodes, const int32_t* idx, int64_t n_indices) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_upload_scene: null ctx");
    try {
        ort::SceneInput in{cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        return upload_impl(ctx, in);
    } catch (const std::bad_alloc&) {
        return fail(ctx, ORT_ERR_OUT_OF_MEMORY, "ort_upload_scene: out of host memory");
    } catch (const std::exception& ex) {
        return fail(ctx, ORT_ERR_INTERNAL, std::string("ort_upload_scene: ") + ex.what());
    }
}

int ort_upload_octree_nodes(ort_ctx* ctx, const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                            const void* nodes, int32_t n_nodes, const int32_t* idx, int64_t n_indices) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_upload_octree_nodes: null ctx");
    if (n_nodes < 0 || (n_nodes > 0 && !nodes)) return fail(ctx, ORT_ERR_INVALID_ARG, "ort_upload_octree_nodes: bad nodes");
    try {
        struct Rec { float mn[3], mx[3]; int32_t co, oo, cnt; };
        static_assert(sizeof(Rec) == 36, "GPUOctreeNode layout");
        const Rec* r = (const Rec*)nodes;
        std::vector<float> mn(3 * (size_t)n_nodes), mx(3 * (size_t)n_nodes);
        std::vector<int32_t> co((size_t)n_nodes), oo((size_t)n_nodes), cn((size_t)n_nodes);
        for (int32_t i = 0; i < n_nodes; ++i) {
            std::memcpy(&mn[3 * (size_t)i], r[i].mn, 12);
            std::memcpy(&mx[3 * (size_t)i], r[i].mx, 12);
            co[i] = r[i].co;
            oo[i] = r[i].oo;
            cn[i] = r[i].cnt;
        }
        ort::SceneInput in{cr, ma, fr, n_spheres, mn.data(), mx.data(), co.data(), oo.data(), cn.data(), n_nodes, idx, n_indices};
        return upload_impl(ctx, in);
    } catch (const std::bad_alloc&) {
        return fail(ctx, ORT_ERR_OUT_OF_MEMORY, "ort_upload_octree_nodes: out of host memory");
    } catch (const std::exception& ex) {
        return fail(ctx, ORT_ERR_INTERNAL, std::string("ort_upload_octree_nodes: ") + ex.what());
    }
}

int ort_scene_get_info(const ort_ctx* ctx, ort_scene_info* info) {
    if (!ctx || !info) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_scene_get_info: null argument");
    if (!ctx->has_scene) return fail(const_cast<ort_ctx*>(ctx), ORT_ERR_NO_SCENE, "no scene uploaded");
    info->n_spheres = ctx->n_spheres;
    info->n_nodes = ctx->n_nodes;
    info->n_indices = ctx->n_indices;
    info->layout = ctx->layout;
    info->tree_depth = ctx->depth;
    const DevBuf* all[] = {&ctx->sph_cr, &ctx->sph_ma, &ctx->sph_fr, &ctx->node, &ctx->kid, &ctx->nk, &ctx->leaf_sph, &ctx->leaf_idx,
                           &ctx->planes, &ctx->lds_img, &ctx->lds_rev, &ctx->nodeA, &ctx->nodeB, &ctx->cnt, &ctx->indices};
    int64_t b = 0;
    for (const DevBuf* d : all) b += (int64_t)d->bytes;
    info->device_bytes = b;
    return ORT_OK;
}

int ort_build_scene(ort_ctx* ctx, const float* sphere_center_radius, const float* sphere_mat_albedo,
                    const float* sphere_fuzz_ri, int32_t n_spheres, int32_t max_depth, int32_t max_spheres_per_node,
                    int32_t keep_tree) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_build_scene: null ctx");
    try {
        return build_impl(ctx, sphere_center_radius, sphere_mat_albedo, sphere_fuzz_ri, n_spheres, max_depth,
                          max_spheres_per_node, keep_tree);
    } catch (const std::exception& ex) {
        return fail(ctx, ORT_ERR_INTERNAL, std::string("ort_build_scene: ") + ex.what());
    }
}

int ort_scene_export_octree(ort_ctx* ctx, float* node_min, float* node_max, int32_t* children_offset,
                            int32_t* objects_offset, int32_t* object_count, int32_t* object_indices) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_scene_export_octree: null ctx");
    const ort::GpuTree& t = ctx->tree;
    if (!ctx->has_scene || !t.co)
        return fail(ctx, ORT_ERR_NO_SCENE, "ort_scene_export_octree: no GPU-built tree kept (ort_build_scene keep_tree)");
    if (!node_min || !node_max || !children_offset || !objects_offset || !object_count || (!object_indices && t.n_indices))
        return fail(ctx, ORT_ERR_INVALID_ARG, "ort_scene_export_octree: null output");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    const size_t n = (size_t)t.n_nodes;
    HIPCHK(ctx, hipMemcpy(node_min, t.node_min, 12 * n, hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(node_max, t.node_max, 12 * n, hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(children_offset, t.co, 4 * n, hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(objects_offset, t.oo, 4 * n, hipMemcpyDeviceToHost));
    HIPCHK(ctx, hipMemcpy(object_count, t.cnt, 4 * n, hipMemcpyDeviceToHost));
    if (t.n_indices) HIPCHK(ctx, hipMemcpy(object_indices, t.idx, 4 * (size_t)t.n_indices, hipMemcpyDeviceToHost));
    return ORT_OK;
}

int ort_get_stream(const ort_ctx* ctx, void** stream) {
    if (!ctx || !stream) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_get_stream: null argument");
    *stream = (void*)ctx->stream;
    return ORT_OK;
}

int ort_last_build_ms(const ort_ctx* ctx, float* ms) {
    if (!ctx || !ms) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_last_build_ms: null argument");
    *ms = ctx->build_ms;
    return ORT_OK;
}

int ort_render(ort_ctx* ctx, const ort_params* params, const ort_tile* tile, float* rgb_out, int out_is_device,
               void* stream) {
    if (!ctx) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_render: null ctx");
    return render_impl(ctx, params, tile, rgb_out, out_is_device, stream, nullptr);
}

int ort_last_kernel_ms(ort_ctx* ctx, float* ms) {
    if (!ctx || !ms) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_last_kernel_ms: null argument");
    if (!ctx->timed) return fail(ctx, ORT_ERR_NO_SCENE, "no kernel launched yet");
    HIPCHK(ctx, hipEventSynchronize(ctx->ev1));
    HIPCHK(ctx, hipEventElapsedTime(ms, ctx->ev0_last, ctx->ev1));
    return ORT_OK;
}

int ort_last_trace_ms(ort_ctx* ctx, float* ms) {
    if (!ctx || !ms) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_last_trace_ms: null argument");
    return ort_trace_times_ms(ctx, 1, ms) == 1 ? ORT_OK : fail(ctx, ORT_ERR_NO_SCENE, "no trace kernel timed yet");
}

int ort_trace_times_ms(ort_ctx* ctx, int n, float* ms) {
    if (!ctx || !ms || n < 0) return -ORT_ERR_INVALID_ARG;
    const long long have = std::min<long long>(ctx->frames, ort_ctx::kRing);
    const int k = (int)std::min<long long>(n, have);
    for (int i = 0; i < k; ++i) {
        const int slot = (int)((ctx->frames - k + i) % ort_ctx::kRing);
        if (hipEventSynchronize(ctx->tr1[slot][0]) != hipSuccess ||
            hipEventElapsedTime(&ms[i], ctx->tr0[slot][0], ctx->tr1[slot][0]) != hipSuccess)
            return -ORT_ERR_HIP;
    }
    return k;
}

int ort_frame_trace_times_ms(ort_ctx* ctx, int n, float* ms, int32_t* launches) {
    if (!ctx || !ms || n < 0) return -ORT_ERR_INVALID_ARG;
    const long long have = std::min<long long>(ctx->frames, ort_ctx::kRing);
    const int k = (int)std::min<long long>(n, have);
    for (int i = 0; i < k; ++i) {
        const int slot = (int)((ctx->frames - k + i) % ort_ctx::kRing);
        float sum = 0.0f;
        for (int j = 0; j < ctx->tseg[slot]; ++j) {
            float t = 0.0f;
            if (hipEventSynchronize(ctx->tr1[slot][j]) != hipSuccess ||
                hipEventElapsedTime(&t, ctx->tr0[slot][j], ctx->tr1[slot][j]) != hipSuccess)
                return -ORT_ERR_HIP;
            sum += t;
        }
        ms[i] = sum;
        if (launches) launches[i] = ctx->tseg[slot];
    }
    return k;
}

int ort_count_traffic(ort_ctx* ctx, const ort_params* params, const ort_tile* tile, uint64_t* counts) {
    if (!ctx || !counts) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_count_traffic: null argument");
    HIPCHK(ctx, hipSetDevice(ctx->device));
    if (!ctx->counters.p) {
        HIPCHK(ctx, hipMalloc(&ctx->counters.p, 64));
        ctx->counters.bytes = 64;
    }
    HIPCHK(ctx, hipMemsetAsync(ctx->counters.p, 0, 64, ctx->stream));
    const size_t pix = tile ? (size_t)tile->width * (size_t)tile->rows : 0;
    DevBuf tmp;
    if (pix) HIPCHK(ctx, hipMalloc(&tmp.p, 12 * pix));
    const int rc = render_impl(ctx, params, tile, (float*)tmp.p, 1, nullptr, (unsigned long long*)ctx->counters.p);
    if (rc == ORT_OK) {
        unsigned long long h[8] = {0};
        hipError_t e = hipMemcpy(h, ctx->counters.p, 64, hipMemcpyDeviceToHost);
        if (e != hipSuccess) { free_buf(tmp); return hip_fail(ctx, e, "ort_count_traffic: copy counters"); }
        for (int k = 0; k < ORT_COUNT_N; ++k) counts[k] = h[k];
        // pixels inside the frame (main() runs once per fragment)
        const TileMap tm = {tile->x0, tile->width, tile->y0, tile->rows, tile->band_height, tile->band_stride};
        uint64_t px = 0;
        for (int j = 0; j < tile->rows; ++j)
            if (tile_row_to_y(tm, j) < params->height) px += (uint64_t)tile->width;
        counts[ORT_COUNT_PIXELS] = px;
    }
    free_buf(tmp);
    return rc;
}

#if ORT_ANALYSIS  // the analysis library only (libort_analysis.so)

// ---- TEST-ONLY host emulation (see ort_internal.h) ----------------------------------
int ort_debug_trace_rays(const float* cr, int32_t n_spheres, const float* node_min, const float* node_max,
                         const int32_t* co, const int32_t* oo, const int32_t* cnt, int32_t n_nodes, const int32_t* idx,
                         int64_t n_indices, const float* rays, int32_t n_rays, int32_t bounce, int32_t* out) {
    try {
        std::vector<float> ma((size_t)n_spheres * 4, 0.0f), fr((size_t)n_spheres * 4, 0.0f);
        ort::SceneInput in{cr, ma.data(), fr.data(), n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        const std::string vbad = ort::validateScene(in);
        if (!vbad.empty()) return fail(nullptr, ORT_ERR_INVALID_ARG, vbad);
        ort::CompactLayout cl;
        std::string why;
        if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why)) return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
        if (!cl.ordered) return fail(nullptr, ORT_ERR_UNSUPPORTED, "unordered tree");
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        S.node = (const uint2*)cl.node.data();
        S.kid = (const uint2*)cl.kid.data();
        S.tail_base = (uint32_t)in.n_indices;
        S.leaf_sph = (const float4*)cl.leaf_sph.data();
        S.leaf_idx = cl.leaf_idx.data();
        S.planes = cl.planes.data();
        S.depth = cl.depth;
        std::vector<float> fplanes(ort::fast_plane_floats(cl.depth));
        ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
        const bool rev_b = ort::Masks96Lean::kRevPlanes || ort::fast_rev_planes(cl.depth);
        std::vector<float> fplanes_b(ort::fast_plane_floats(cl.depth, rev_b));
        ort::fill_fast_planes(cl.planes.data(), fplanes_b.data(), cl.depth, rev_b);
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        ort::LocalFrames lf;
        for (int32_t i = 0; i < n_rays; ++i) {
            ort::Ray r;
            r.o = ort::mk(rays[6 * (size_t)i], rays[6 * (size_t)i + 1], rays[6 * (size_t)i + 2]);
            r.d = ort::mk(rays[6 * (size_t)i + 3], rays[6 * (size_t)i + 4], rays[6 * (size_t)i + 5]);
            ort::Counters cc;
            for (int k = 0; k < 6; ++k) cc.v[k] = 0;
            float tf = 0.0f, tx = 0.0f;
            int ef = -1, ex = -1;
            // the kernels' choice: the fast walk when fast_prepare takes the ray, else deferred
            ort::V3 inv = ort::mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
            const bool fast = ort::fast_prepare(S, r, inv);
            if (fast) {
                if (!bounce) ort::traverse_fast<false>(S, fplanes.data(), lut.data(), r, inv, 0.001f, ORT_MAXFLOAT, ef, tf, lf, cc);
                else if (S.depth <= 8)
                    ort::traverse_fast_t<false, ort::Masks64Plain>(S, fplanes.data(), lut.data(), r, inv, 0.001f, ORT_MAXFLOAT,
                                                                 ef, tf, lf, cc);
                else
                    ort::traverse_fast_t<false, ort::Masks96Lean>(S, fplanes_b.data(), lut.data(), r, inv, 0.001f,
                                                                ORT_MAXFLOAT, ef, tf, lf, cc);
            }
            ort::traverse_compact<false>(S, fplanes.data(), r, 0.001f, ORT_MAXFLOAT, ex, tx, lf, cc);
            int32_t* o = out + 5 * (size_t)i;
            o[0] = fast ? 1 : 0;
            o[1] = ef;
            o[2] = (int32_t)ort::f2u(tf);
            o[3] = ex;
            o[4] = (int32_t)ort::f2u(tx);
        }
        return ORT_OK;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}

int ort_debug_split_rays(const float* cr, int32_t n_spheres, const float* node_min, const float* node_max,
                         const int32_t* co, const int32_t* oo, const int32_t* cnt, int32_t n_nodes, const int32_t* idx,
                         int64_t n_indices, const float* rays, int32_t n_rays, int32_t level, int32_t lanes, int32_t* out) {
    try {
        if (lanes < 1 || level < 1) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_debug_split_rays: lanes, level >= 1");
        std::vector<float> ma((size_t)n_spheres * 4, 0.0f), fr((size_t)n_spheres * 4, 0.0f);
        ort::SceneInput in{cr, ma.data(), fr.data(), n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        const std::string vbad = ort::validateScene(in);
        if (!vbad.empty()) return fail(nullptr, ORT_ERR_INVALID_ARG, vbad);
        ort::CompactLayout cl;
        std::string why;
        if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why)) return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
        if (!cl.ordered) return fail(nullptr, ORT_ERR_UNSUPPORTED, "unordered tree");
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        S.node = (const uint2*)cl.node.data();
        S.kid = (const uint2*)cl.kid.data();
        S.tail_base = (uint32_t)in.n_indices;
        S.leaf_sph = (const float4*)cl.leaf_sph.data();
        S.leaf_idx = cl.leaf_idx.data();
        S.planes = cl.planes.data();
        S.depth = cl.depth;
        std::vector<float> fplanes(ort::fast_plane_floats(cl.depth));  // the default image's layout
        ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        ort::LocalFrames lf;
        for (int32_t i = 0; i < n_rays; ++i) {
            ort::Ray r;
            r.o = ort::mk(rays[6 * (size_t)i], rays[6 * (size_t)i + 1], rays[6 * (size_t)i + 2]);
            r.d = ort::mk(rays[6 * (size_t)i + 3], rays[6 * (size_t)i + 4], rays[6 * (size_t)i + 5]);
            const ort::V3 inv = ort::mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
            int32_t* o = out + 4 * (size_t)i;
            o[0] = -1;
            o[1] = 0;
            o[2] = 0x7fffffff;
            o[3] = 0;
            if (!ort::fast_path_ok(r, inv, 0.001f, ORT_MAXFLOAT)) continue;
            // the lanes of one group one after another; the lowest DFS position wins
            int best = 0x7fffffff, be = -1, top = 0, owns = 0;  // steps as ort_trace_split records them
            float bt = 0.0f;
            for (int j = 0; j < lanes; ++j) {
                int pos = 0x7fffffff, e = -1, st = 0, own = 0;
                float t = 0.0f;
                if (S.depth > 8)
                    ort::traverse_split<ort::Masks96Split>(S, fplanes.data(), lut.data(), r, inv, level, lanes, j, pos, e, t, lf, st, own);
                else
                    ort::traverse_split<ort::Masks64Split>(S, fplanes.data(), lut.data(), r, inv, level, lanes, j, pos, e, t, lf, st, own);
                top = std::max(top, st - own);
                owns += own;
                if (pos < best) {
                    best = pos;
                    be = e;
                    bt = t;
                }
            }
            o[0] = be;
            o[1] = (int32_t)ort::f2u(bt);
            o[2] = best;
            o[3] = top + owns;
        }
        return ORT_OK;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}

int ort_debug_fast_order(int32_t m, int32_t* order8, uint8_t* lut256) {
    if (m < 0 || m > 7 || !order8) return fail(nullptr, ORT_ERR_INVALID_ARG, "ort_debug_fast_order: m in 0..7");
    for (uint32_t r = 0; r < 8; ++r) order8[r] = (int32_t)ort::rank_perm(r, (uint32_t)m);
    if (lut256)
        for (uint32_t c = 0; c < 256; ++c) lut256[c] = ort::rank_lut_entry((uint32_t)m, c);
    return ORT_OK;
}

int ort_debug_emulate_render(const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                             const float* node_min, const float* node_max, const int32_t* co, const int32_t* oo,
                             const int32_t* cnt, int32_t n_nodes, const int32_t* idx, int64_t n_indices,
                             int32_t layout, const ort_params* p, const ort_tile* t, float* out, uint64_t* counts) {
    try {
        const std::string bad = check_params(p, t);
        if (!bad.empty()) return fail(nullptr, ORT_ERR_INVALID_ARG, bad);
        ort::SceneInput in{cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        const std::string vbad = ort::validateScene(in);
        if (!vbad.empty()) return fail(nullptr, ORT_ERR_INVALID_ARG, vbad);
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        std::vector<float> fr2((size_t)n_spheres * 2);
        for (int32_t i = 0; i < n_spheres; ++i) {
            fr2[2 * (size_t)i] = fr[4 * (size_t)i];
            fr2[2 * (size_t)i + 1] = fr[4 * (size_t)i + 1];
        }
        S.sph_cr = (const float4*)cr;
        S.sph_ma = (const float4*)ma;
        S.sph_fr = (const float2*)fr2.data();
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        ort::CompactLayout cl;
        std::vector<float> fplanes;  // fast-walk plane tables (forward + reversed)
        std::vector<float> fplanes_b;  // ... of the bounce walk (Masks96Lean's reversed tables at depth 9-10)
        std::vector<float> A, B;
        int mode = 2;
        if (p->use_octree == 1) {
            if (n_nodes <= 0) return fail(nullptr, ORT_ERR_NO_SCENE, "no octree");
            std::string why;
            if (layout == ORT_LAYOUT_COMPACT || layout == 2) {
                if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why))
                    return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
                mode = 0;
                S.node = (const uint2*)cl.node.data();
                S.kid = (const uint2*)cl.kid.data();
                S.tail_base = (uint32_t)in.n_indices;
                S.leaf_sph = (const float4*)cl.leaf_sph.data();
                S.leaf_idx = cl.leaf_idx.data();
                S.planes = cl.planes.data();
                S.depth = cl.depth;
                fplanes.resize(ort::fast_plane_floats(cl.depth));
                ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
                const bool rev_b = ort::Masks96Lean::kRevPlanes || ort::fast_rev_planes(cl.depth);
                fplanes_b.resize(ort::fast_plane_floats(cl.depth, rev_b));
                ort::fill_fast_planes(cl.planes.data(), fplanes_b.data(), cl.depth, rev_b);
            } else {
                mode = 1;
                A.resize(4 * (size_t)n_nodes);
                B.resize(4 * (size_t)n_nodes);
                for (int32_t i = 0; i < n_nodes; ++i) {
                    for (int k = 0; k < 3; ++k) {
                        A[4 * (size_t)i + k] = node_min[3 * (size_t)i + k];
                        B[4 * (size_t)i + k] = node_max[3 * (size_t)i + k];
                    }
                    std::memcpy(&A[4 * (size_t)i + 3], &co[i], 4);
                    std::memcpy(&B[4 * (size_t)i + 3], &oo[i], 4);
                }
                S.nodeA = (const float4*)A.data();
                S.nodeB = (const float4*)B.data();
                S.count = cnt;
                S.indices = idx;
            }
        }
        const ort::PixelParams pp = pixel_params(p);
        const TileMap tm = {t->x0, t->width, t->y0, t->rows, t->band_height, t->band_stride};
        ort::Counters total;
        for (int k = 0; k < 6; ++k) total.v[k] = 0;
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        const uint8_t* rank_lut = (layout == ORT_LAYOUT_COMPACT && cl.ordered) ? lut.data() : nullptr;
        std::vector<int> snode(ORT_MAX_STACK);
        std::vector<float> stmin(ORT_MAX_STACK);
        ort::LocalFrames lf;
        for (int row = 0; row < t->rows; ++row) {
            const int y = tile_row_to_y(tm, row);
            for (int c = 0; c < t->width; ++c) {
                float* o = out + 3 * ((size_t)row * t->width + c);
                if (y >= p->height) { o[0] = o[1] = o[2] = 0.0f; continue; }
                ort::Counters cc;
                for (int k = 0; k < 6; ++k) cc.v[k] = 0;
                ort::V3 v, vc;
                // pixels from the production walk (COUNT=false: with the rejected-sphere skip),
                // counters from the counting walk (the reference's work, no skip) -- and the two
                // pixels must agree bit for bit
                if (mode == 0) {
                    v = ort::shade_pixel<0, false>(pp, S, fplanes.data(), fplanes_b.data(), rank_lut, lf, nullptr, nullptr,
                                                   t->x0 + c, y, cc);
                    vc = ort::shade_pixel<0, true>(pp, S, fplanes.data(), fplanes_b.data(), rank_lut, lf, nullptr, nullptr,
                                                   t->x0 + c, y, cc);
                } else if (mode == 1) {
                    v = ort::shade_pixel<1, false>(pp, S, nullptr, nullptr, nullptr, lf, snode.data(), stmin.data(), t->x0 + c, y, cc);
                    vc = ort::shade_pixel<1, true>(pp, S, nullptr, nullptr, nullptr, lf, snode.data(), stmin.data(), t->x0 + c, y, cc);
                } else {
                    v = ort::shade_pixel<2, false>(pp, S, nullptr, nullptr, nullptr, lf, nullptr, nullptr, t->x0 + c, y, cc);
                    vc = ort::shade_pixel<2, true>(pp, S, nullptr, nullptr, nullptr, lf, nullptr, nullptr, t->x0 + c, y, cc);
                }
                if (ort::f2u(v.x) != ort::f2u(vc.x) || ort::f2u(v.y) != ort::f2u(vc.y) || ort::f2u(v.z) != ort::f2u(vc.z))
                    return fail(nullptr, ORT_ERR_INTERNAL, "emulation: production and counting walks differ at pixel (" +
                                                               std::to_string(t->x0 + c) + ", " + std::to_string(y) + ")");
                o[0] = v.x; o[1] = v.y; o[2] = v.z;
                cc.v[4] = 1;
                for (int k = 0; k < 6; ++k) total.v[k] += cc.v[k];
            }
        }
        if (counts) for (int k = 0; k < 6; ++k) counts[k] = total.v[k];
        return ORT_OK;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}


// Analysis builds only (ORT_PERSIST_CLOCK, tools/persist_clock.py): the persistent bounce
// kernel records a per-wave timeline {start, queue drained, end, XCC id | items << 8} into dev
// (n records of 4 x u64, one range per launch of a frame); null = off.
int ort_debug_wave_clock(ort_ctx* ctx, void* dev, int64_t n) {
    if (!ctx) return ORT_ERR_INVALID_ARG;
    ctx->wclock = dev;
    ctx->wclock_n = dev ? n : 0;
    return ORT_OK;
}

// ANALYSIS-ONLY (tools/wave_stats.py): walks sampled 8x8 pixel blocks (one wave each) of
// the primary-ray frame with the kernel's fast walk on the host and reports how the lanes'
// visited-node sets overlap, to price wave-level (packet) traversal against the per-lane
// loop.  stats: see tools/wave_stats.py for the field order.
int ort_debug_wave_stats(const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                         const float* node_min, const float* node_max, const int32_t* co, const int32_t* oo,
                         const int32_t* cnt, int32_t n_nodes, const int32_t* idx, int64_t n_indices,
                         const ort_params* p, int32_t block_step, double* stats, int32_t n_stats) {
    try {
        if (n_stats < 16 || block_step < 1) return fail(nullptr, ORT_ERR_INVALID_ARG, "bad stats args");
        ort::SceneInput in{cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        ort::CompactLayout cl;
        std::string why;
        if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why)) return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        S.node = (const uint2*)cl.node.data();
        S.kid = (const uint2*)cl.kid.data();
        S.tail_base = (uint32_t)in.n_indices;
        S.leaf_sph = (const float4*)cl.leaf_sph.data();
        S.leaf_idx = cl.leaf_idx.data();
        S.planes = cl.planes.data();
        S.depth = cl.depth;
        std::vector<float> fplanes(ort::fast_plane_floats(cl.depth));
        ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        const ort::PixelParams pp = pixel_params(p);
        ort::LocalFrames lf;
        ort::Counters cc;
        for (int k = 0; k < 6; ++k) cc.v[k] = 0;
        for (int k = 0; k < n_stats; ++k) stats[k] = 0.0;
        const int bw = (p->width + 7) / 8, bh = (p->height + 7) / 8;
        std::vector<std::vector<int>> seq(64);
        std::vector<int> all;
        for (int b = 0; b < bw * bh; b += block_step) {
            const int bx = b % bw, by = b / bw;
            bool uniform = true;
            int m0 = -1, lanes = 0;
            size_t maxlen = 0;
            for (int l = 0; l < 64; ++l) {
                seq[l].clear();
                const int px = bx * 8 + (l & 7), py = by * 8 + (l >> 3);
                if (px >= p->width || py >= p->height) continue;
                ort_rng st;
                ort::pixel_rng_init(pp, px, py, st);
                const ort::Ray ray = ort::primary_ray(pp, px, py, 0, st);
                const ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
                if (!ort::fast_path_ok(ray, inv, 0.001f, ORT_MAXFLOAT)) { uniform = false; continue; }
                lanes++;
                const int m = ((ray.d.z < 0.0f) << 2) | ((ray.d.x < 0.0f) << 1) | (ray.d.y < 0.0f);
                if (m0 < 0) m0 = m;
                else if (m != m0) uniform = false;
                ort::FastStateT<ort::Masks96> fs;
                if (!ort::fast_begin(S, fplanes.data(), lut.data(), ray, inv, 0.001f, ORT_MAXFLOAT, fs)) continue;
                for (;;) {
                    seq[l].push_back(fs.node);
                    if (ort::fast_step<false>(S, lut.data(), fs, lf, cc)) break;
                }
                maxlen = std::max(maxlen, seq[l].size());
            }
            stats[0] += 1;                  // waves
            stats[1] += uniform ? 0 : 1;    // waves with mixed order / non-fast lanes
            stats[2] += lanes;
            all.clear();
            for (int l = 0; l < 64; ++l)
                for (int nd : seq[l]) {
                    const bool leaf = !(cl.node[2 * (size_t)nd + 1] & ORT_INTERNAL_FLAG);
                    stats[leaf ? 4 : 3] += 1;  // individual internal / leaf visits
                    if (leaf) stats[5] += cl.node[2 * (size_t)nd + 1];  // individual sphere tests
                    all.push_back(nd);
                }
            std::sort(all.begin(), all.end());
            all.erase(std::unique(all.begin(), all.end()), all.end());
            for (int nd : all) {
                const bool leaf = !(cl.node[2 * (size_t)nd + 1] & ORT_INTERNAL_FLAG);
                stats[leaf ? 7 : 6] += 1;  // union internal / leaf visits
                if (leaf) stats[8] += cl.node[2 * (size_t)nd + 1];
            }
            // lockstep per-lane loop (the current kernel): iteration k runs the internal
            // block if any lane's k-th node is internal, the leaf block (max spheres) if any
            // is a leaf, and the pop for every lane still walking
            for (size_t k = 0; k < maxlen; ++k) {
                bool anyI = false, anyL = false;
                uint32_t maxS = 0;
                int act = 0;
                for (int l = 0; l < 64; ++l) {
                    if (k >= seq[l].size()) continue;
                    act++;
                    const uint32_t y = cl.node[2 * (size_t)seq[l][k] + 1];
                    if (y & ORT_INTERNAL_FLAG) anyI = true;
                    else { anyL = true; maxS = std::max(maxS, y); }
                }
                stats[9] += 1;            // lockstep iterations
                stats[10] += anyI;        // iterations running the internal block
                stats[11] += anyL;        // iterations running the leaf block
                stats[12] += maxS;        // sphere-loop trips
                stats[13] += act;         // lane-iterations
            }
            stats[14] += (double)maxlen;
            if (n_stats >= 18) {
                // wave-uniform iterations: every lane still walking pops the same node -- the
                // leading run of them (the shared descent) and all of them
                bool lead = true;
                for (size_t k = 0; k < maxlen; ++k) {
                    int nd = -1;
                    bool uni = true;
                    for (int l = 0; l < 64 && uni; ++l) {
                        if (k >= seq[l].size()) continue;
                        if (nd < 0) nd = seq[l][k];
                        else if (seq[l][k] != nd) uni = false;
                    }
                    lead = lead && uni;
                    stats[15] += lead ? 1 : 0;
                    stats[16] += uni ? 1 : 0;
                }
                stats[17] += 1;
            }
        }
        return ORT_OK;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}


// ANALYSIS-ONLY (tools/bounce_lines.py): the rays of bounce `bounce` (>= 1) of a tile's pixels,
// 1 sample (the host restatement of the path: trace_ray + shade_bounce per bounce, as
// shade_pixel), and per alive ray the loads of its bounce walk (the persistent kernel's walk,
// rejected-sphere skip on): per step {node popped, first object entry of a leaf or -1, objects}.
// rays: 8 floats per pixel {o.xyz, d.xyz, alive, steps}.  walks: 3 ints per step, ray after
// ray; n_out[0] = steps written (all steps if <= cap).
int ort_debug_bounce_walks(const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                           const float* node_min, const float* node_max, const int32_t* co, const int32_t* oo,
                           const int32_t* cnt, int32_t n_nodes, const int32_t* idx, int64_t n_indices,
                           const ort_params* p, const ort_tile* t, int32_t bounce, float* rays, int32_t* walks,
                           int64_t cap, int64_t* n_out) {
    try {
        const std::string bad = check_params(p, t);
        if (!bad.empty() || bounce < 1 || p->num_samples != 1) return fail(nullptr, ORT_ERR_INVALID_ARG, "bad args");
        ort::SceneInput in{cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        ort::CompactLayout cl;
        std::string why;
        if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why)) return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        std::vector<float> fr2((size_t)n_spheres * 2);
        for (int32_t i = 0; i < n_spheres; ++i) {
            fr2[2 * (size_t)i] = fr[4 * (size_t)i];
            fr2[2 * (size_t)i + 1] = fr[4 * (size_t)i + 1];
        }
        S.sph_cr = (const float4*)cr;
        S.sph_ma = (const float4*)ma;
        S.sph_fr = (const float2*)fr2.data();
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        S.node = (const uint2*)cl.node.data();
        S.kid = (const uint2*)cl.kid.data();
        S.tail_base = (uint32_t)in.n_indices;
        S.leaf_sph = (const float4*)cl.leaf_sph.data();
        S.leaf_idx = cl.leaf_idx.data();
        S.planes = cl.planes.data();
        S.depth = cl.depth;
        std::vector<float> fplanes(ort::fast_plane_floats(cl.depth));
        ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
        const bool rev_b = ort::Masks96Lean::kRevPlanes || ort::fast_rev_planes(cl.depth);
        std::vector<float> fplanes_b(ort::fast_plane_floats(cl.depth, rev_b));
        ort::fill_fast_planes(cl.planes.data(), fplanes_b.data(), cl.depth, rev_b);
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        const ort::PixelParams pp = pixel_params(p);
        const TileMap tm = {t->x0, t->width, t->y0, t->rows, t->band_height, t->band_stride};
        ort::LocalFrames lf;
        ort::Counters cc;
        for (int k = 0; k < 6; ++k) cc.v[k] = 0;
        int64_t n = 0;
        auto walk = [&](auto tag, const ort::Ray& ray, ort::V3 inv) -> int {
            using Masks = decltype(tag);
            ort::FastStateT<Masks> fs;
            const float* pl = cl.depth > 8 ? fplanes_b.data() : fplanes.data();
            if (!ort::fast_begin(S, pl, lut.data(), ray, inv, 0.001f, ORT_MAXFLOAT, fs)) return 0;
            int steps = 0;
            for (bool done = false; !done;) {
                const uint2 rec = fs.rec;
                const bool leaf = !(rec.y & ORT_INTERNAL_FLAG);
                if (n < cap) {
                    walks[3 * n] = fs.node;
                    walks[3 * n + 1] = leaf ? (int)rec.x : -1;
                    walks[3 * n + 2] = leaf ? (int)rec.y : 0;
                }
                ++n;
                ++steps;
                done = ort::fast_step<false>(S, lut.data(), fs, lf, cc);
            }
            return steps;
        };
        for (int row = 0; row < t->rows; ++row) {
            const int y = tile_row_to_y(tm, row);
            for (int c = 0; c < t->width; ++c) {
                float* o = rays + 8 * ((size_t)row * t->width + c);
                for (int k = 0; k < 8; ++k) o[k] = 0.0f;
                if (y >= p->height) continue;
                const int px = t->x0 + c;
                ort_rng st;
                ort::pixel_rng_init(pp, px, y, st);
                ort::Ray ray = ort::primary_ray(pp, px, y, 0, st);
                ort::V3 col = ort::mk(1.0f, 1.0f, 1.0f);
                float importance = 1.0f;
                bool alive = true;
                for (int b = 0; b < bounce && alive; ++b) {
                    if (importance < 0.01f) { alive = false; break; }
                    float th;
                    int entry;
                    const int tr = ort::trace_ray<0, false>(S, fplanes.data(), lut.data(), ray, false, th, entry, lf, nullptr,
                                                            nullptr, cc, b > 0, fplanes_b.data());
                    ort::HitRec h;
                    if (tr == ORT_TRACE_HIT) h = ort::hit_record<0>(S, ray, th, entry);
                    if (ort::shade_bounce(tr == ORT_TRACE_HIT, h, ray, col, importance, st)) alive = false;
                }
                if (!alive || importance < 0.01f) continue;
                ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
                o[0] = ray.o.x; o[1] = ray.o.y; o[2] = ray.o.z;
                o[3] = ray.d.x; o[4] = ray.d.y; o[5] = ray.d.z;
                o[6] = 1.0f;
                if (!ort::fast_prepare(S, ray, inv)) { o[6] = 2.0f; continue; }  // deferred (exact walk)
                o[7] = (float)(cl.depth > 8 ? walk(ort::Masks96Lean{}, ray, inv) : walk(ort::Masks64Plain{}, ray, inv));
            }
        }
        *n_out = n;
        return ORT_OK;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}

int64_t ort_debug_walk_steps(const float* cr, const float* ma, const float* fr, int32_t n_spheres,
                             const float* node_min, const float* node_max, const int32_t* co, const int32_t* oo,
                             const int32_t* cnt, int32_t n_nodes, const int32_t* idx, int64_t n_indices,
                             const ort_params* p, int32_t block_step, int32_t* lens, int64_t n_lens, uint16_t* steps,
                             int64_t cap) {
    try {
        if (block_step < 1) return fail(nullptr, ORT_ERR_INVALID_ARG, "bad block_step");
        ort::SceneInput in{cr, ma, fr, n_spheres, node_min, node_max, co, oo, cnt, n_nodes, idx, n_indices};
        ort::CompactLayout cl;
        std::string why;
        if (!ort::buildCompactLayout(in, ORT_COMPACT_MAX_DEPTH, cl, why)) return fail(nullptr, ORT_ERR_UNSUPPORTED, why);
        if (cl.depth > 8) return fail(nullptr, ORT_ERR_UNSUPPORTED, "walk_steps: depth <= 8 walk only");
        ort::KScene S;
        std::memset(&S, 0, sizeof(S));
        S.n_spheres = n_spheres;
        S.n_nodes = n_nodes;
        S.node = (const uint2*)cl.node.data();
        S.kid = (const uint2*)cl.kid.data();
        S.tail_base = (uint32_t)in.n_indices;
        S.leaf_sph = (const float4*)cl.leaf_sph.data();
        S.leaf_idx = cl.leaf_idx.data();
        S.planes = cl.planes.data();
        S.depth = cl.depth;
        std::vector<float> fplanes(ort::fast_plane_floats(cl.depth));
        ort::fill_fast_planes(cl.planes.data(), fplanes.data(), cl.depth);
        std::vector<uint8_t> lut(kRankLutBytes);
        for (size_t i = 0; i < lut.size(); ++i) lut[i] = ort::rank_lut_entry((uint32_t)i >> 8, (uint32_t)i & 255u);
        const ort::PixelParams pp = pixel_params(p);
        ort::LocalFrames lf;
        const int bw = (p->width + 7) / 8, bh = (p->height + 7) / 8;
        int64_t w = 0, n = 0;
        for (int b = 0; b < bw * bh; b += block_step, ++w) {
            const int bx = b % bw, by = b / bw;
            for (int l = 0; l < 64; ++l) {
                int32_t len = 0;
                const int px = bx * 8 + (l & 7), py = by * 8 + (l >> 3);
                if (px < p->width && py < p->height) {
                    ort_rng st;
                    ort::pixel_rng_init(pp, px, py, st);
                    const ort::Ray ray = ort::primary_ray(pp, px, py, 0, st);
                    const ort::V3 inv = ort::mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
                    ort::FastStateT<ort::Masks64> fs;
                    if (ort::fast_path_ok(ray, inv, 0.001f, ORT_MAXFLOAT) &&
                        ort::fast_begin(S, fplanes.data(), lut.data(), ray, inv, 0.001f, ORT_MAXFLOAT, fs)) {
                        for (bool done = false; !done;) {
                            ort::Counters cc;
                            for (int k = 0; k < 6; ++k) cc.v[k] = 0;
                            const uint32_t y = fs.rec.y;
                            done = ort::fast_step<true>(S, lut.data(), fs, lf, cc);
                            const uint64_t objs = cc.v[2] < 255 ? cc.v[2] : 255, kids = cc.v[0] - 1;
                            const bool lk = (y & ORT_INTERNAL_FLAG) && (y & ORT_LEAFKIDS_FLAG);
                            if (n < cap) steps[n] = (uint16_t)(objs | (kids < 15 ? kids : 15) << 8 | (lk ? 0x8000u : 0u));
                            ++n;
                            ++len;
                        }
                    }
                }
                if (64 * w + l < n_lens) lens[64 * w + l] = len;
            }
        }
        return n <= cap ? n : -n;
    } catch (const std::exception& ex) {
        return fail(nullptr, ORT_ERR_INTERNAL, ex.what());
    }
}

#endif  // ORT_ANALYSIS

}  // extern "C"
