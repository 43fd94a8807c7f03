// octree.cpp -- level-synchronous octree builder emitting the reference's BFS layout.
//
// Semantics restated from the reference (all paths relative to the reference repo):
//   root box = union of sphere AABBs, glm::min/max fold      src/octree.cpp:54-63
//   stop when depth >= maxDepth || count <= maxSpheresPerNode src/octree.cpp:191
//   mid = (min + max) * 0.5f, 8 children by octant           src/octree.cpp:197-204, 97-187
//   spheres distributed in list order, children 0..7 tested  src/octree.cpp:207-217
//   empty children are never subdivided                       src/octree.cpp:224-228
//   closest-point sphere/box test, dist^2 <= r^2              src/octree.cpp:231-242
//   BFS flatten: childrenOffset = BFS index of child 0;       src/octree.cpp:268-312
//     leaves with objects get consecutive objectsOffset in BFS order.
// Because BFS visits level L completely before level L+1, in parent order and octant
// order within a parent, growing the tree one level at a time reproduces the exact
// node order of the reference's queue walk.
#include "octree.h"

#include <chrono>
#include <climits>
#include <iostream>
#include <stdexcept>
#include <string>

using ortm::vec3;

Octree::Octree(int maxDepth_, int maxSpheresPerNode_) : maxDepth(maxDepth_), maxSpheresPerNode(maxSpheresPerNode_) {}

bool Octree::sphereIntersectsBox(const Sphere& sphere, const vec3& boxMin, const vec3& boxMax) {
    vec3 closest;
    for (int i = 0; i < 3; ++i) {
        // std::max(boxMin, std::min(center, boxMax)) with libstdc++'s comparison order
        const float c = sphere.center[i];
        const float lo = boxMin[i], hi = boxMax[i];
        const float m = (hi < c) ? hi : c;   // std::min(c, hi)
        closest[i] = (lo < m) ? m : lo;      // std::max(lo, m)
    }
    const vec3 d = closest - sphere.center;
    const float distSquared = ortm::dot(d, d);
    return distSquared <= (sphere.radius * sphere.radius);
}

void Octree::childBox(int octant, const vec3& min, const vec3& max, const vec3& mid, vec3& cmin, vec3& cmax) {
    const bool zb = (octant >> 2) & 1, xb = (octant >> 1) & 1, yb = octant & 1;
    cmin.x = xb ? mid.x : min.x;
    cmax.x = xb ? max.x : mid.x;
    cmin.y = yb ? mid.y : min.y;
    cmax.y = yb ? max.y : mid.y;
    cmin.z = zb ? mid.z : min.z;
    cmax.z = zb ? max.z : mid.z;
}

namespace {
struct LevelNode {
    vec3 min, max;
    int64_t begin;  // into the level's index buffer
    int64_t count;
};
}  // namespace

void Octree::build(const std::vector<Sphere>& spheres, const int debug) {
    const auto start = std::chrono::steady_clock::now();
    if (spheres.empty()) throw std::invalid_argument("Sphere list is empty");
    if (spheres.size() > (size_t)INT_MAX) throw std::length_error("too many spheres for int32 indices");

    flattenedTree.clear();
    objectIndices.clear();

    vec3 rmin = spheres[0].center - vec3(spheres[0].radius, spheres[0].radius, spheres[0].radius);
    vec3 rmax = spheres[0].center + vec3(spheres[0].radius, spheres[0].radius, spheres[0].radius);
    for (const Sphere& s : spheres) {
        const vec3 smin = s.center - vec3(s.radius, s.radius, s.radius);
        const vec3 smax = s.center + vec3(s.radius, s.radius, s.radius);
        rmin = ortm::min(rmin, smin);
        rmax = ortm::max(rmax, smax);
    }
    if (debug) {
        std::cout << "Sphere Min: " << rmin.x << ", " << rmin.y << ", " << rmin.z << std::endl;
        std::cout << "Sphere Max: " << rmax.x << ", " << rmax.y << ", " << rmax.z << std::endl;
        std::cout << "Root Node Object Count: " << spheres.size() << std::endl;
    }

    std::vector<LevelNode> cur(1), next;
    std::vector<int> curIdx(spheres.size()), nextIdx;
    for (size_t i = 0; i < spheres.size(); ++i) curIdx[i] = (int)i;
    cur[0] = {rmin, rmax, 0, (int64_t)spheres.size()};

    int64_t levelBase = 0;   // BFS index of cur[0]
    int64_t objectCursor = 0;
    std::vector<int> childLists[8];
    // The reference's buildTime covers the root box and the subdivision only, not the BFS
    // flatten (src/octree.cpp:82-85, setGPUData after it): each level here runs the
    // subdivision (children's boxes and sphere lists) and then emits the level's records and
    // leaf lists, and the two are timed apart -- buildTime the first, flattenTime the second.
    double subdivideSeconds = 0.0, emitSeconds = 0.0;
    auto t = std::chrono::steady_clock::now();
    subdivideSeconds += std::chrono::duration<double>(t - start).count();  // root box
    // size_t comparison like the reference (a negative maxSpheresPerNode stops at the root)
    const size_t mcap = static_cast<size_t>(maxSpheresPerNode);

    for (int depth = 0; !cur.empty(); ++depth) {
        next.clear();
        nextIdx.clear();
        const int64_t nextBase = levelBase + (int64_t)cur.size();
        if (nextBase > (int64_t)INT_MAX) throw std::length_error("octree exceeds int32 node offsets");
        // The reference only recurses into non-empty nodes; an empty node is a leaf whatever
        // maxSpheresPerNode says (it can only be empty below the root).
        auto isLeaf = [&](const LevelNode& n) { return depth >= maxDepth || (size_t)n.count <= mcap || n.count == 0; };
        // 1. subdivision: the children of every internal node of the level, in BFS order
        for (const LevelNode& n : cur) {
            if (isLeaf(n)) continue;
            const vec3 mid = (n.min + n.max) * 0.5f;
            vec3 cmin[8], cmax[8];
            for (int i = 0; i < 8; ++i) {
                childBox(i, n.min, n.max, mid, cmin[i], cmax[i]);
                childLists[i].clear();
            }
            for (int64_t k = 0; k < n.count; ++k) {
                const int sIdx = curIdx[n.begin + k];
                const Sphere& s = spheres[sIdx];
                for (int i = 0; i < 8; ++i)
                    if (sphereIntersectsBox(s, cmin[i], cmax[i])) childLists[i].push_back(sIdx);
            }
            for (int i = 0; i < 8; ++i) {
                const int64_t b = (int64_t)nextIdx.size();
                nextIdx.insert(nextIdx.end(), childLists[i].begin(), childLists[i].end());
                next.push_back({cmin[i], cmax[i], b, (int64_t)childLists[i].size()});
            }
        }
        const auto t1 = std::chrono::steady_clock::now();
        // 2. flatten: the level's records and leaf object lists
        int64_t splitRank = 0;
        for (const LevelNode& n : cur) {
            GPUOctreeNode g;
            g.min = n.min;
            g.max = n.max;
            if (isLeaf(n)) {
                g.childrenOffset = -1;
                if (n.count > 0) {
                    g.objectsOffset = (int)objectCursor;
                    g.objectCount = (int)n.count;
                    objectIndices.insert(objectIndices.end(), curIdx.begin() + n.begin,
                                         curIdx.begin() + n.begin + n.count);
                    objectCursor += n.count;
                    if (objectCursor > (int64_t)INT_MAX) throw std::length_error("object index list exceeds int32");
                } else {
                    g.objectsOffset = -1;
                    g.objectCount = 0;
                }
                if (debug) std::cout << "Stopping subdivision at depth " << depth << " with " << n.count << " objects." << std::endl;
            } else {
                g.childrenOffset = (int)(nextBase + 8 * splitRank);
                g.objectsOffset = -1;
                g.objectCount = 0;
                ++splitRank;
            }
            flattenedTree.push_back(g);
        }
        const auto t2 = std::chrono::steady_clock::now();
        subdivideSeconds += std::chrono::duration<double>(t1 - t).count();
        emitSeconds += std::chrono::duration<double>(t2 - t1).count();
        t = t2;
        levelBase = nextBase;
        cur.swap(next);
        curIdx.swap(nextIdx);
    }

    buildTime = subdivideSeconds;
    flattenTime = emitSeconds;
    if (debug) std::cout << "Total build time: " << buildTime << "s" << std::endl;
}

void Octree::setGPUData() {
    // Validation only (see header): every internal node's 8 children are in range and
    // every leaf's index range lies inside objectIndices.
    const int64_t n = (int64_t)flattenedTree.size();
    for (int64_t i = 0; i < n; ++i) {
        const GPUOctreeNode& g = flattenedTree[i];
        if (g.childrenOffset != -1 && (g.childrenOffset <= i || (int64_t)g.childrenOffset + 8 > n))
            throw std::invalid_argument("Child node is null on non-leaf node");
        if (g.childrenOffset == -1 && g.objectCount > 0 &&
            (g.objectsOffset < 0 || (int64_t)g.objectsOffset + g.objectCount > (int64_t)objectIndices.size()))
            throw std::invalid_argument("leaf object range outside objectIndices");
    }
}

void Octree::printFlattenedTree() {
    int i = 0;
    std::cout << std::endl;
    for (const GPUOctreeNode& node : flattenedTree) {
        std::cout << "Node " << i++ << ":" << std::endl;
        std::cout << "Node Min: " << node.min.x << ", " << node.min.y << ", " << node.min.z << std::endl;
        std::cout << "Node Max: " << node.max.x << ", " << node.max.y << ", " << node.max.z << std::endl;
        std::cout << "Children Offset: " << node.childrenOffset << std::endl;
        std::cout << "Objects Offset: " << node.objectsOffset << std::endl;
        std::cout << "Object Count: " << node.objectCount << std::endl;
        if (node.objectCount > 0) {
            // prints the whole list, exactly like the reference (src/octree.cpp:254-258)
            std::cout << "Object Indices: ";
            for (int index : objectIndices) std::cout << index << " ";
            std::cout << std::endl;
        }
        std::cout << std::endl;
    }
}
