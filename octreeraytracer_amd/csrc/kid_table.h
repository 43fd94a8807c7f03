// kid_table.h -- the per-node "rejected-sphere skip" entries of the compact layout, shared by
// the host layout compiler (layout.cpp) and the device one (gpu_build.hip).
//
// The reference walk ends at the first leaf with an accepted hit, so until then every leaf it
// pops is a REJECTED sphere test over (leaf tmin, t_max).  A sphere s rejected over (e, t_max)
// is rejected over every (e', t_max) with e' >= e (same ray, same sphere: the same roots), so a
// later leaf that holds exactly s and whose pushed tmin is >= e cannot end the walk: skipping
// it changes no result.  In this scene shape (maxSpheresPerNode 1, thin octree cells) a sphere
// sits in ~170 leaves and a ray passing it walks through many of them in a row.
//
// Entry of internal node i (two words): up to two spheres held by one-sphere leaf children
// of i, each with the octant mask of the children holding it: word = id | mask << 24
// (id < 2^24; 0 = none).  The most frequent sphere first.  The walk keeps the last rejected
// one-sphere leaf's sphere and tmin per lane and drops matching children before pushing them
// (render_core.h fast_step), when the node's own tmin (a lower bound of every child's) is >=
// that tmin.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define ORT_KID_HD __host__ __device__
#else
#define ORT_KID_HD
#endif

#define ORT_KID_ID_LIMIT (1 << 24)

// sid[k]: the sphere of child k if it is a one-sphere leaf, else -1.
inline ORT_KID_HD void kid_entry(const int32_t sid[8], uint32_t& w0, uint32_t& w1) {
    int32_t b0 = -1, b1 = -1;
    int n0 = 0, n1 = 0;
    for (int k = 0; k < 8; ++k) {
        const int32_t s = sid[k];
        if (s < 0 || s >= ORT_KID_ID_LIMIT) continue;
        bool first = true;
        for (int j = 0; j < k; ++j) first = first && sid[j] != s;
        if (!first) continue;
        int c = 0;
        for (int j = k; j < 8; ++j) c += sid[j] == s ? 1 : 0;
        if (c > n0) {
            b1 = b0;
            n1 = n0;
            b0 = s;
            n0 = c;
        } else if (c > n1) {
            b1 = s;
            n1 = c;
        }
    }
    uint32_t m0 = 0, m1 = 0;
    for (int k = 0; k < 8; ++k) {
        if (b0 >= 0 && sid[k] == b0) m0 |= 1u << k;
        if (b1 >= 0 && sid[k] == b1) m1 |= 1u << k;
    }
    w0 = b0 >= 0 ? ((uint32_t)b0 | (m0 << 24)) : 0u;
    w1 = b1 >= 0 ? ((uint32_t)b1 | (m1 << 24)) : 0u;
}
