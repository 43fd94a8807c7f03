// leafkids_pack.h -- the packed record of a "leaf-children" node for the depth <= 8 camera
// walk (render_core.h leaf_kids_packed), shared by the host layout compiler (layout.cpp) and
// the device one (gpu_build.hip k_compact_nodes).
//
// A LEAFKIDS node (every existing child is a leaf) has its surviving leaf children tested
// inline in rank order.  With the plain record {childrenOffset, flags|mask} each child costs a
// dependent load of its own record {objectsOffset, objectCount} before its spheres can be
// fetched.  The reference builder numbers leaves breadth-first, so the object lists of a
// node's children are contiguous in octant order: objectsOffset of child k = that of the
// first existing child + the counts of the existing children before k.  The packed record
// carries exactly that:
//   x = objectsOffset of the first existing child (octant order)
//   y = INTERNAL | LEAFKIDS | (count - 1 of child k, 2 bits) << (8 + 2k) | existing-child mask
// so a child's sphere range is arithmetic on the node's own record.  Packable when every
// existing child holds 1..4 objects and the lists are contiguous; otherwise the node keeps
// its plain record with LEAFKIDS cleared (its children are then pushed and popped like any
// other node's).  The offsets point into the objectIndices-ordered entries (never into the
// per-sphere tail one-sphere leaves use, layout.h): the same spheres in the same order.
#pragma once
#include <stdint.h>

#include "render_core_flags.h"

#if defined(__HIPCC__)
#define ORT_LKP_HD __host__ __device__
#else
#define ORT_LKP_HD
#endif

#define ORT_LEAFKIDS_MAX_PACKED 4

// y: the node's compact record word (INTERNAL | LEAFKIDS | leafMask << 8 | childMask);
// co: its childrenOffset; oo / cnt: the reference arrays (objectsOffset / objectCount).
inline ORT_LKP_HD void pack_leafkids(uint32_t y, int32_t co, const int32_t* oo, const int32_t* cnt, uint32_t& px,
                                     uint32_t& py) {
    px = (uint32_t)co;
    py = y;
    if (!(y & ORT_INTERNAL_FLAG_HOST) || !(y & ORT_LEAFKIDS_FLAG_HOST)) return;
    const uint32_t mask = y & 0xffu;
    int64_t base = -1, next = 0;
    uint32_t fields = 0;
    bool ok = mask != 0;
    for (int k = 0; k < 8 && ok; ++k) {
        if (!((mask >> k) & 1u)) continue;
        const int64_t c = (int64_t)co + k;
        const int32_t n = cnt[c];
        if (n < 1 || n > ORT_LEAFKIDS_MAX_PACKED || oo[c] < 0) {
            ok = false;
            break;
        }
        if (base < 0) base = next = oo[c];
        if (oo[c] != next) ok = false;
        next += n;
        fields |= (uint32_t)(n - 1) << (2 * k);
    }
    if (!ok || base < 0 || base > 0x7fffffff) {
        py = y & ~ORT_LEAFKIDS_FLAG_HOST;
        return;
    }
    px = (uint32_t)base;
    py = ORT_INTERNAL_FLAG_HOST | ORT_LEAFKIDS_FLAG_HOST | (fields << 8) | mask;
}
