// layout.h -- host-side conversion of the reference buffer layout into the kernel's
// compact layout (the "layout compiler" run once per ort_upload_*).
//
// Reference layout (src/raytracer.cpp:87-101): per node min.xyz/childrenOffset and
// max.xyz/objectsOffset vec4s + objectCount; objectIndices; 36 B read per node popped plus
// 32 B per child box examined (glsl:318-324, 459-462).
//
// Compact layout (MI355X):
//   node[i] (8 B):  internal -> {childrenOffset, 0x80000000 | leafKids << 30 | leafMask << 8 | childMask}
//     leafKids: every existing child is a leaf (the kernel then tests them inline)
//     leafMask bit k = child k is in childMask and is a leaf (deep walks test a node's leading
//     leaf children inline: render_core.h fast_step)
//                   leaf     -> {objectsOffset, objectCount}
//     childMask bit k = child (childrenOffset + k) is in range and is not an empty leaf
//     (the glsl:456 and glsl:467 skip tests, precomputed).
//   leaf_sph[e] = spheres[objectIndices[e]] with .w = radius * radius (16 B): one gather
//   instead of index + sphere, and the sphere test's r * r precomputed (rounded as it would be).
//   leaf_idx[e] = objectIndices[e], read only for the final hit (material lookup).
//   kid[i] (8 B): internal node i's rejected-sphere skip entry (kid_table.h).
//   Both arrays carry a per-sphere TAIL after the n_indices entries: entry n_indices + s is
//   sphere s.  A leaf holding exactly one sphere s records objectsOffset = n_indices + s, so
//   its test reads the sphere table (16 B x spheres: cache-resident even at 1M spheres)
//   instead of its own copy inside the n_indices-entry array (2.8 GB at C5, where each
//   sphere sits in ~170 leaves and the copies are HBM misses for scattered bounce rays).
//   Same sphere, same order, same hit: the records only point elsewhere.
//   planes[a][k], k = 0..2^D: coordinate of the axis-a split plane at dyadic position
//     k / 2^D.  The reference builder derives every child box from its parent by
//     mid = (min+max)*0.5f and copies min/mid/max verbatim (src/octree.cpp:97-187, 197),
//     so the box of the node at depth d, cell (cx,cy,cz) is exactly
//     [planes[x][cx<<(D-d)], planes[x][(cx+1)<<(D-d)]] x ...; boxes are therefore
//     re-derived bit-exactly in the kernel instead of being read (8 x 32 B per node).
//     The conversion VERIFIES this for every reachable node; a tree that does not
//     satisfy it (e.g. hand-made) is uploaded in the explicit reference layout instead.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

namespace ort {

struct SceneInput {
    const float* sph_cr;
    const float* sph_ma;
    const float* sph_fr;
    int32_t n_spheres;
    const float* node_min;  // 3 per node
    const float* node_max;
    const int32_t* co;
    const int32_t* oo;
    const int32_t* cnt;
    int32_t n_nodes;
    const int32_t* indices;
    int64_t n_indices;
};

struct CompactLayout {
    int depth = 0;                 // D
    std::vector<float> planes;     // 3 * (2^D + 1)
    std::vector<uint32_t> node;    // 2 per node
    std::vector<float> leaf_sph;   // 4 per index entry
    std::vector<int32_t> leaf_idx; // 1 per index entry
    std::vector<uint32_t> kid;     // 2 per node: rejected-sphere skip entries (kid_table.h)
    // Every reachable box has min <= max and no NaN coordinate: then the plane tables are
    // monotone and the kernel's sign-decided fast walk applies; otherwise every ray takes
    // the exact (GLSL min/max) walk.
    bool ordered = true;
};

// Validates the scene like the reference would need (index ranges); returns "" or a message.
std::string validateScene(const SceneInput& in);

// Builds the compact layout; returns false (with `why`) if the tree is not representable
// (boxes not derivable by midpoint splits, node reachable twice, depth > maxDepth).
bool buildCompactLayout(const SceneInput& in, int maxDepth, CompactLayout& out, std::string& why);

// Maximum node depth reachable from the root (BFS), or -1 if a node is reached twice.
int treeDepth(const SceneInput& in);

}  // namespace ort
