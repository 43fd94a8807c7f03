// ref_octree_driver.cpp -- TEST INFRASTRUCTURE ONLY.
// Links the reference's OWN src/octree.cpp (compiled from /root/reference, never copied)
// and dumps Octree::flattenedTree / objectIndices for a sphere set, so that tests can
// pin this repo's builder byte-for-byte against the reference builder.
//
// usage: ref_octree <in.bin> <out.bin>
//   in.bin : int32 n, int32 maxDepth, int32 maxSpheresPerNode, n x float4 (cx, cy, cz, r)
//   out.bin: int64 n_nodes, int64 n_indices, double buildTime,
//            n_nodes x 36-byte GPUOctreeNode, n_indices x int32
#include <cstdio>
#include <cstdint>
#include <vector>
#include "octree.h"   // the reference's src/octree.h (via -I/root/reference/src)

int main(int argc, char** argv) {
    if (argc != 3) { std::fprintf(stderr, "usage: %s in.bin out.bin\n", argv[0]); return 2; }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    int32_t hdr[3];
    if (std::fread(hdr, 4, 3, f) != 3) return 4;
    std::vector<float> cr((size_t)hdr[0] * 4);
    if (std::fread(cr.data(), 4, cr.size(), f) != cr.size()) return 5;
    std::fclose(f);
    std::vector<Sphere> spheres;
    spheres.reserve(hdr[0]);
    for (int i = 0; i < hdr[0]; ++i)
        spheres.push_back(Sphere(glm::vec3(cr[4 * i], cr[4 * i + 1], cr[4 * i + 2]), cr[4 * i + 3]));
    Octree tree(hdr[1], hdr[2]);
    tree.build(spheres, 0);
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 6;
    int64_t nn = (int64_t)tree.flattenedTree.size(), ni = (int64_t)tree.objectIndices.size();
    std::fwrite(&nn, 8, 1, o);
    std::fwrite(&ni, 8, 1, o);
    std::fwrite(&tree.buildTime, 8, 1, o);
    static_assert(sizeof(GPUOctreeNode) == 36, "layout");
    std::fwrite(tree.flattenedTree.data(), sizeof(GPUOctreeNode), tree.flattenedTree.size(), o);
    std::fwrite(tree.objectIndices.data(), 4, tree.objectIndices.size(), o);
    std::fclose(o);
    return 0;
}
