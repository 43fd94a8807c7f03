// path_key.h -- the coherence key of an alive path between bounces (ORT_OPT_SORT_PATHS):
// computed where a path is appended to the next bounce's list (ort_kernel.hip shade/trace
// kernels) and by the every-slot sort (gpu_build.hip sortAlive).  Only orders work: pixels
// never depend on it.
//
// key = direction octant (3 bits) | origin code (kMortonBits) | direction (2 bits per axis of
// |d| / max|d|), < 2^30.  The origin code quantises the origin in the tree's root box and deals
// its bits one at a time to the axis whose cell is currently the longest (a k-d split order: a
// root box of 500 x 4.8 x 500, as at C5, gets its bits in x and z, not a third of them in y),
// most significant first.  Measured on C5 (tools/ab_stream.py): every one of these bits counts
// -- 24-bit keys (fewer origin bits), octant-only and octant + direction orders were all slower.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ort {

#ifndef ORT_MORTON_BITS
#define ORT_MORTON_BITS 21
#endif
constexpr int kMortonBits = ORT_MORTON_BITS;
#ifndef ORT_DIR_BITS
#define ORT_DIR_BITS 2  // direction bits per axis (C5: 3 bits with 18 origin bits -0.9 %, 1 with 24 -0.3 %)
#endif
constexpr int kDirBits = ORT_DIR_BITS;
constexpr int kPathKeyBits = 3 + kMortonBits + 3 * kDirBits;  // 30: alive keys < 2^30, dead = 0xffffffff
// origin-code bits above the direction bits (the rest below them): kMortonBits = origin first
#ifndef ORT_KEY_ORIGIN_HI
#define ORT_KEY_ORIGIN_HI ORT_MORTON_BITS
#endif
constexpr int kOriginHi = ORT_KEY_ORIGIN_HI, kOriginLo = kMortonBits - kOriginHi;
static_assert(kOriginHi >= 0 && kOriginLo >= 0, "ORT_KEY_ORIGIN_HI: 0 .. ORT_MORTON_BITS");
static_assert(kPathKeyBits <= 30, "the heavy-first class sits above the key");

struct MortonPlan {
    float lo[3], scale[3];      // q_a = (x - lo) * scale in [0, 2^bits_a)
    int bits[3];
    uint32_t axis_lo, axis_hi;  // 2 bits per split: axis of split i (i < 16 in lo)
};

// Host: the split plan of a root box.
inline MortonPlan mortonPlan(const float* root_lo, const float* root_hi) {
    MortonPlan mp{};
    float cell[3];
    for (int a = 0; a < 3; ++a) {
        const float ext = root_hi[a] - root_lo[a];
        cell[a] = (ext > 0.0f && ext < 3.0e38f) ? ext : 0.0f;
        mp.lo[a] = root_lo[a];
    }
    for (int i = 0; i < kMortonBits; ++i) {  // deal the splits to the longest current cell
        int a = 0;
        for (int j = 1; j < 3; ++j)
            if (cell[j] > cell[a]) a = j;
        cell[a] *= 0.5f;
        mp.bits[a] += 1;
        if (i < 16) mp.axis_lo |= (uint32_t)a << (2 * i);
        else mp.axis_hi |= (uint32_t)a << (2 * (i - 16));
    }
    for (int a = 0; a < 3; ++a) {
        const float ext = root_hi[a] - root_lo[a];
        mp.scale[a] = (ext > 0.0f && ext < 3.0e38f) ? (float)(1u << mp.bits[a]) / ext : 0.0f;
    }
    return mp;
}

// Host: the origin code as three table lookups per axis (spread[a][byte][v] = the code bits
// that byte `byte` of axis a's quantised coordinate contributes, v its value) -- the same
// code as dealing the kMortonBits bits one at a time, most significant first; ~9 loads
// instead of ~130 VALU per key.  kSpreadWords entries.
constexpr int kSpreadWords = 3 * 3 * 256;
inline void mortonSpread(const MortonPlan& mp, uint32_t* spread) {
    for (int i = 0; i < kSpreadWords; ++i) spread[i] = 0u;
    int rem[3] = {mp.bits[0], mp.bits[1], mp.bits[2]};
    for (int i = 0; i < kMortonBits; ++i) {  // split i puts bit r of axis a at code bit kMortonBits-1-i
        const int a = (int)(((i < 16 ? mp.axis_lo >> (2 * i) : mp.axis_hi >> (2 * (i - 16)))) & 3u);
        const int r = --rem[a];
        const uint32_t pos = 1u << (kMortonBits - 1 - i);
        const int byte = r >> 3, bit = r & 7;
        for (int v = 0; v < 256; ++v)
            if ((v >> bit) & 1) spread[(a * 3 + byte) * 256 + v] |= pos;
    }
}

__device__ __forceinline__ uint32_t key_quant(float x, float lo, float scale, int bits) {
    const float q = (x - lo) * scale;
    const float top = (float)((1u << bits) - 1u);
    return q <= 0.0f ? 0u : (q >= top ? (uint32_t)top : (uint32_t)q);  // NaN -> 0
}

// spread: mortonSpread's table (device memory).
__device__ __forceinline__ uint32_t path_key(const float4 o, const float4 d, const MortonPlan& mp,
                                             const uint32_t* spread) {
    const uint32_t m = ((uint32_t)(d.z < 0.0f) << 2) | ((uint32_t)(d.x < 0.0f) << 1) | (uint32_t)(d.y < 0.0f);
    const float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    const float inv = ((float)(1 << kDirBits) - 0.001f) / fmaxf(fmaxf(ax, ay), fmaxf(az, 1e-30f));
    const uint32_t dq = ((uint32_t)(ax * inv) << (2 * kDirBits)) | ((uint32_t)(ay * inv) << kDirBits) | (uint32_t)(az * inv);
    const float oa[3] = {o.x, o.y, o.z};
    uint32_t code = 0;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const uint32_t q = key_quant(oa[a], mp.lo[a], mp.scale[a], mp.bits[a]);  // < 2^21
        const uint32_t* t = spread + a * 768;
        code |= t[q & 255u] | t[256 + ((q >> 8) & 255u)] | t[512 + (q >> 16)];
    }
    const uint32_t lo = code & ((1u << kOriginLo) - 1u);
    return (m << (3 * kDirBits + kMortonBits)) | ((code >> kOriginLo) << (3 * kDirBits + kOriginLo)) | (dq << kOriginLo) | lo;
}

}  // namespace ort
