// octree.h -- the reference's Octree API (src/octree.h:10-79), rebuilt from scratch.
//
// Kept: OctantPosition (octant = (z<<2)|(x<<1)|y), GPUOctreeNode (36-byte AoS record),
// Octree(maxDepth, maxSpheresPerNode), build(spheres, debug), setGPUData(),
// printFlattenedTree(), the public flattenedTree / objectIndices / buildTime members,
// and the thrown std::invalid_argument on an empty scene (src/octree.cpp:50-52).
//
// Changed (internals only): the reference grows a pointer tree depth-first and then
// flattens it with std::queue + std::map (src/octree.cpp:189-229, 268-312).  This
// builder grows the tree level by level straight into the BFS layout -- the same node
// order, boxes, offsets and index lists, byte for byte -- without per-node heap objects,
// so 10^6-sphere / depth-10 scenes (2.4e8 nodes) build in bounded memory and time.
#pragma once
#include <cstdint>
#include <vector>
#include "sphere.h"

enum OctantPosition {
    // Binary: zxy (0 = min, 1 = max for each dimension)
    BottomLeftBack = 0,
    BottomLeftFront = 1,
    BottomRightBack = 2,
    BottomRightFront = 3,
    TopLeftBack = 4,
    TopLeftFront = 5,
    TopRightBack = 6,
    TopRightFront = 7
};

// Same record as the reference (src/octree.h:24-30).
struct GPUOctreeNode {
    ortm::vec3 min;      // Bottom Left Back
    ortm::vec3 max;      // Top Right Front
    int childrenOffset;  // index of child octant 0, -1 for leaves
    int objectsOffset;   // first entry in objectIndices, -1 when the leaf is empty or internal
    int objectCount;     // entries in objectIndices (0 for internal nodes)
};
static_assert(sizeof(GPUOctreeNode) == 36, "GPUOctreeNode must match the reference's 36-byte layout");

class Octree {
public:
    Octree(int maxDepth = 8, int maxSpheresPerNode = 8);
    ~Octree() = default;

    // Vectors for the GPU (BFS order; children of a node are contiguous at childrenOffset + octant)
    std::vector<GPUOctreeNode> flattenedTree;
    std::vector<int> objectIndices;

    // seconds, as the reference's (src/octree.cpp:82-85): the root box and the subdivision, not
    // the flatten -- the saveStats "Octree Build Time" column
    double buildTime = 0.0;
    double flattenTime = 0.0;  // seconds: emitting the BFS records and leaf lists (the reference's setGPUData)

    // Throws std::invalid_argument("Sphere list is empty") like the reference.
    void build(const std::vector<Sphere>& spheres, const int debug = 0);

    // The reference flattens here; this builder already emits the flattened arrays, so
    // setGPUData() only re-validates them (kept for API compatibility).
    void setGPUData();

    void printFlattenedTree();

    int getMaxDepth() const { return maxDepth; }
    int getMaxSpheresPerNode() const { return maxSpheresPerNode; }

    // Sphere-vs-box closest-point test (src/octree.cpp:231-242).
    static bool sphereIntersectsBox(const Sphere& sphere, const ortm::vec3& boxMin, const ortm::vec3& boxMax);
    // Box of child `octant` of [min, max] split at mid (src/octree.cpp:97-187).
    static void childBox(int octant, const ortm::vec3& min, const ortm::vec3& max, const ortm::vec3& mid,
                         ortm::vec3& cmin, ortm::vec3& cmax);

private:
    int maxDepth;
    int maxSpheresPerNode;
};
