// gpu_build.h -- the reference octree builder on the GPU (see gpu_build.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "path_key.h"

#include <cstdint>
#include <string>
#include <vector>

namespace ort {

// The reference flattened tree (Octree::flattenedTree + objectIndices, src/octree.cpp:268-312)
// in device memory, SoA.  Owned by the caller of gpuBuildOctree (freeGpuTree).
struct GpuTree {
    int32_t n_nodes = 0;
    int64_t n_indices = 0;
    int32_t n_spheres = 0;              // spheres the tree was built over
    int depth = 0;                      // deepest node level (root = 0)
    std::vector<int64_t> level_start;   // BFS index of the first node of each level (+ end)
    float* node_min = nullptr;          // 3 per node
    float* node_max = nullptr;
    int32_t* co = nullptr;              // childrenOffset (-1 for leaves)
    int32_t* oo = nullptr;              // objectsOffset (-1 unless a leaf with objects)
    int32_t* cnt = nullptr;             // objectCount
    int32_t* idx = nullptr;             // objectIndices
    uint32_t* cell = nullptr;           // node cell, 10 bits per axis (x | y << 10 | z << 20)
    bool ordered = true;                // every box has min <= max (no NaN)
    double seconds = 0.0;               // device build time (events)
};

void freeGpuTree(GpuTree& t);

// Builds the tree of `spheres` (n x float4 center.xyz, radius; device memory) exactly as
// Octree::build(maxDepth, maxSpheresPerNode) does.  Synchronous on `s`.  Returns "" or an error.
std::string gpuBuildOctree(const float4* spheres, int32_t n, int32_t maxDepth, int32_t maxSpheresPerNode, hipStream_t s,
                           GpuTree& out);

// Device-side conversions of a built tree into the kernel layouts (ort_kernel.hip).  The
// caller owns the outputs (hipMalloc'd here).  Compact: returns false with `why` when the
// tree does not fit the compact layout (depth, 4 GiB offsets, plane check).
struct CompactDev {
    uint2* node = nullptr;
    uint2* kid = nullptr;  // rejected-sphere skip entries (kid_table.h), one per node
    float4* leaf_sph = nullptr;
    int32_t* leaf_idx = nullptr;
    float* planes = nullptr;
    size_t node_bytes = 0, leaf_bytes = 0, idx_bytes = 0, plane_bytes = 0;
};
bool gpuCompactLayout(const GpuTree& t, const float4* spheres, int maxDepth, hipStream_t s, CompactDev& out,
                      std::string& why);
struct ExplicitDev {
    float4* nodeA = nullptr;
    float4* nodeB = nullptr;
    int32_t* cnt = nullptr;
    int32_t* indices = nullptr;
};
std::string gpuExplicitLayout(const GpuTree& t, hipStream_t s, ExplicitDev& out);

}  // namespace ort

namespace ort {
// Coherence sort of the alive paths (ORT_OPT_SORT_PATHS): key = direction octant (3 bits) |
// Morton code of the origin in the root box (7 bits per axis) | 2 bits per axis of the
// normalised direction magnitude; dead slots get the largest
// key, so the sorted values are the alive slots first, *count of them (device).
struct SortBuffers {
    uint32_t* keys_in;
    uint32_t* keys_out;
    int* vals_in;
    int* vals_out;  // = the list the next bounce walks
};
// Coherence sort of the alive list itself (ORT_OPT_SORT_PATHS 2): n (key, path) pairs, keys
// written by the kernels that appended the list (path_key.h) -> b.vals_out in key order.
// Temp storage as for sortAlive with the same n bound.
hipError_t sortList(void* temp, size_t temp_bytes, int n, const SortBuffers& b, hipStream_t s);
// The same, stream-ordered: the list's length n is only on the device (*count).  `bound` is a
// host-side size (a hint: last frame's length plus a margin).  Keys [n, bound) are padded with
// the all-ones key, so the stable radix sort of `bound` pairs puts the n real ones first, in
// key order.  If n > bound (the hint was short) the sort's output is replaced by the list in
// append order -- the same paths, a different order, so the same pixels.  No host wait.
// key_bits: the keys' width (kPathKeyBits, or one more with the heavy-first bit).
hipError_t sortListBounded(void* temp, size_t temp_bytes, int bound, const int* count, const SortBuffers& b,
                           hipStream_t s, int key_bits = kPathKeyBits);
size_t sortAliveTempBytes(int n);
hipError_t sortAlive(void* temp, size_t temp_bytes, const float4* po, const float4* pd, int n, const float* root_lo,
                     const float* root_hi, const uint32_t* spread, const SortBuffers& b, int* count, hipStream_t s);
}  // namespace ort
