// gpu_build.hip -- the reference octree builder (src/octree.cpp Octree::build, subdivideNode,
// sphereIntersectsBox, setGPUData) as a level-synchronous GPU build, byte-identical output
// (SURVEY.md 8(f) item 2).
//
// Reference semantics restated:
//  * root box = glm::min/max over every sphere's center -+ radius (src/octree.cpp:54-63);
//  * a node at depth d with list L subdivides iff d < maxDepth and |L| > (size_t)
//    maxSpheresPerNode (:191); then all 8 children exist (octant = z<<2 | x<<1 | y, boxes from
//    mid = (min+max)*0.5f, :97-187, :197-204), child k's list = the spheres of L (in L's
//    order) that sphereIntersectsBox its box (:206-216), and L is cleared (:219-220);
//  * flatten (:268-312): node index = BFS order over all nodes (each internal node's 8
//    children consecutive, octant order), childrenOffset = index of child 0, leaves with
//    objects append their lists to objectIndices in BFS order.
// The root list is 0..N-1 and children filter in order, so every list is ascending.
//
// GPU formulation, per level d (the nodes of a level are consecutive in BFS order):
//  * the level's (node, sphere) pairs, in a deterministic order;
//  * counts[node] (atomics) -> subdivide flag -> rank of the subdividing nodes (scan) ->
//    child index = levelStart[d+1] + 8*rank + octant, child boxes and cells;
//  * per pair: the 8-bit mask of children its sphere touches (subdividing node), or a leaf
//    key (BFS node << 32 | sphere); one scan over (popcount(mask), is-leaf) gives every slot;
// then objectsOffset = scan of the leaf counts in BFS order, and one radix sort of the leaf
// keys yields objectIndices (BFS node, then ascending sphere: the reference order).
// Arithmetic is the reference's, operation for operation, with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <rocprim/rocprim.hpp>

#include "gpu_build.h"
#include "kid_table.h"
#include "path_key.h"

namespace ort {
namespace {

constexpr int kB = 256;

__device__ __forceinline__ float gmin(float x, float y) { return (y < x) ? y : x; }  // glm::min
__device__ __forceinline__ float gmax(float x, float y) { return (x < y) ? y : x; }  // glm::max

// Octree::sphereIntersectsBox (src/octree.cpp:231-242): std::max(lo, std::min(c, hi)) per
// axis, glm::dot((closest - c), (closest - c)) <= r*r.
__device__ __forceinline__ bool sphere_box(float4 s, const float* lo, const float* hi) {
    const float c[3] = {s.x, s.y, s.z};
    float d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
        const float m = (hi[i] < c[i]) ? hi[i] : c[i];
        const float cl = (lo[i] < m) ? m : lo[i];
        d[i] = cl - c[i];
    }
    const float dist2 = (d[0] * d[0] + d[1] * d[1]) + d[2] * d[2];
    return dist2 <= s.w * s.w;
}

// createSubnodes (src/octree.cpp:97-187): octant bit 1 = x, bit 0 = y, bit 2 = z.
__device__ __forceinline__ void child_box(int k, const float* lo, const float* hi, const float* mid, float* clo,
                                          float* chi) {
    const bool xb = (k >> 1) & 1, yb = k & 1, zb = (k >> 2) & 1;
    clo[0] = xb ? mid[0] : lo[0];
    chi[0] = xb ? hi[0] : mid[0];
    clo[1] = yb ? mid[1] : lo[1];
    chi[1] = yb ? hi[1] : mid[1];
    clo[2] = zb ? mid[2] : lo[2];
    chi[2] = zb ? hi[2] : mid[2];
}

__device__ __forceinline__ bool subdivides(int32_t count, int depth, int maxDepth, unsigned long long mspn) {
    return depth < maxDepth && (unsigned long long)(uint32_t)count > mspn;  // :191, size_t compare
}

// Root box partials: every thread folds its spheres starting from sphere 0's box (like :54-63).
__global__ void k_bounds(const float4* sp, int n, float* part) {
    __shared__ float sh[6][kB];
    const float4 s0 = sp[0];
    float v[6] = {s0.x - s0.w, s0.y - s0.w, s0.z - s0.w, s0.x + s0.w, s0.y + s0.w, s0.z + s0.w};
    for (int i = blockIdx.x * kB + threadIdx.x; i < n; i += gridDim.x * kB) {
        const float4 s = sp[i];
        v[0] = gmin(v[0], s.x - s.w);
        v[1] = gmin(v[1], s.y - s.w);
        v[2] = gmin(v[2], s.z - s.w);
        v[3] = gmax(v[3], s.x + s.w);
        v[4] = gmax(v[4], s.y + s.w);
        v[5] = gmax(v[5], s.z + s.w);
    }
    for (int j = 0; j < 6; ++j) sh[j][threadIdx.x] = v[j];
    __syncthreads();
    for (int w = kB / 2; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            for (int j = 0; j < 3; ++j) sh[j][threadIdx.x] = gmin(sh[j][threadIdx.x], sh[j][threadIdx.x + w]);
            for (int j = 3; j < 6; ++j) sh[j][threadIdx.x] = gmax(sh[j][threadIdx.x], sh[j][threadIdx.x + w]);
        }
        __syncthreads();
    }
    if (threadIdx.x == 0)
        for (int j = 0; j < 6; ++j) part[6 * blockIdx.x + j] = sh[j][0];
}

// Final fold of the partials into the root record (node 0 of level 0).
__global__ void k_root(const float* part, int nb, float* lmin, float* lmax, uint32_t* lcell) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    float v[6];
    for (int j = 0; j < 6; ++j) v[j] = part[j];
    for (int b = 1; b < nb; ++b) {
        for (int j = 0; j < 3; ++j) v[j] = gmin(v[j], part[6 * b + j]);
        for (int j = 3; j < 6; ++j) v[j] = gmax(v[j], part[6 * b + j]);
    }
    for (int j = 0; j < 3; ++j) {
        lmin[j] = v[j];
        lmax[j] = v[3 + j];
    }
    lcell[0] = 0;
}

__global__ void k_iota_pairs(int32_t* pnode, int32_t* psph, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        pnode[i] = 0;
        psph[i] = (int32_t)i;
    }
}

__global__ void k_count(const int32_t* pnode, int64_t np, int32_t* lcnt) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < np; i += (int64_t)gridDim.x * kB)
        atomicAdd(lcnt + pnode[i], 1);
}

__global__ void k_flags(const int32_t* lcnt, int64_t nn, int depth, int maxDepth, unsigned long long mspn,
                        uint32_t* flag) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < nn; i += (int64_t)gridDim.x * kB)
        flag[i] = subdivides(lcnt[i], depth, maxDepth, mspn) ? 1u : 0u;
}

// Level records: childrenOffset, cleared count of subdividing nodes, box order check, and
// the 8 children's boxes and cells in the next level's buffers.
__global__ void k_level(int64_t nn, int depth, int maxDepth, unsigned long long mspn, int64_t next_start,
                        const uint32_t* rank, const float* lmin, const float* lmax, const uint32_t* lcell,
                        int32_t* lco, int32_t* lcnt, float* nmin, float* nmax, uint32_t* ncell, int* unordered) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < nn; i += (int64_t)gridDim.x * kB) {
        const float lo[3] = {lmin[3 * i], lmin[3 * i + 1], lmin[3 * i + 2]};
        const float hi[3] = {lmax[3 * i], lmax[3 * i + 1], lmax[3 * i + 2]};
        if (!(lo[0] <= hi[0]) || !(lo[1] <= hi[1]) || !(lo[2] <= hi[2])) atomicOr(unordered, 1);
        if (!subdivides(lcnt[i], depth, maxDepth, mspn)) {
            lco[i] = -1;
            continue;
        }
        const int64_t c0 = 8 * (int64_t)rank[i];
        lco[i] = (int32_t)(next_start + c0);
        lcnt[i] = 0;  // :219-220
        const float mid[3] = {(lo[0] + hi[0]) * 0.5f, (lo[1] + hi[1]) * 0.5f, (lo[2] + hi[2]) * 0.5f};
        const uint32_t cl = lcell[i];
        const uint32_t cx = cl & 1023u, cy = (cl >> 10) & 1023u, cz = (cl >> 20) & 1023u;
        for (int k = 0; k < 8; ++k) {
            float clo[3], chi[3];
            child_box(k, lo, hi, mid, clo, chi);
            const int64_t j = c0 + k;
            for (int a = 0; a < 3; ++a) {
                nmin[3 * j + a] = clo[a];
                nmax[3 * j + a] = chi[a];
            }
            const uint32_t nx = ((cx << 1) | (uint32_t)((k >> 1) & 1)) & 1023u;
            const uint32_t ny = ((cy << 1) | (uint32_t)(k & 1)) & 1023u;
            const uint32_t nz = ((cz << 1) | (uint32_t)((k >> 2) & 1)) & 1023u;
            ncell[j] = nx | (ny << 10) | (nz << 20);
        }
    }
}

// Per pair: child mask of a subdividing node (bits 0-7) or the leaf flag (bit 8).
__global__ void k_codes(const int32_t* pnode, const int32_t* psph, int64_t np, const int32_t* lco, const float* lmin,
                        const float* lmax, const float4* sp, uint16_t* code) {
    for (int64_t p = blockIdx.x * (int64_t)kB + threadIdx.x; p < np; p += (int64_t)gridDim.x * kB) {
        const int32_t i = pnode[p];
        if (lco[i] < 0) {
            code[p] = 0x100;
            continue;
        }
        const float lo[3] = {lmin[3 * i], lmin[3 * i + 1], lmin[3 * i + 2]};
        const float hi[3] = {lmax[3 * i], lmax[3 * i + 1], lmax[3 * i + 2]};
        const float mid[3] = {(lo[0] + hi[0]) * 0.5f, (lo[1] + hi[1]) * 0.5f, (lo[2] + hi[2]) * 0.5f};
        const float4 s = sp[psph[p]];
        uint32_t m = 0;
        for (int k = 0; k < 8; ++k) {
            float clo[3], chi[3];
            child_box(k, lo, hi, mid, clo, chi);
            if (sphere_box(s, clo, chi)) m |= 1u << k;
        }
        code[p] = (uint16_t)m;
    }
}

struct CodeCounts {
    __host__ __device__ unsigned long long operator()(uint16_t c) const {
        return (unsigned long long)__builtin_popcount(c & 0xffu) | ((unsigned long long)(c >> 8) << 32);
    }
};

// Writes the next level's pairs (child-local index, sphere) and this level's leaf keys.
__global__ void k_emit(const int32_t* pnode, const int32_t* psph, int64_t np, const uint16_t* code,
                       const unsigned long long* off, const int32_t* lco, int64_t level_start, int64_t next_start,
                       int64_t leaf_base, int32_t* qnode, int32_t* qsph, unsigned long long* leaf_keys) {
    for (int64_t p = blockIdx.x * (int64_t)kB + threadIdx.x; p < np; p += (int64_t)gridDim.x * kB) {
        const uint32_t c = code[p];
        const unsigned long long o = off[p];
        const int32_t i = pnode[p];
        const int32_t s = psph[p];
        if (c & 0x100u) {
            leaf_keys[leaf_base + (int64_t)(o >> 32)] = ((unsigned long long)(level_start + i) << 32) | (uint32_t)s;
            continue;
        }
        int64_t q = (int64_t)(o & 0xffffffffull);
        const int32_t c0 = (int32_t)(lco[i] - next_start);  // 8 * rank
        for (int k = 0; k < 8; ++k)
            if ((c >> k) & 1u) {
                qnode[q] = c0 + k;
                qsph[q] = s;
                ++q;
            }
    }
}

__global__ void k_oo(const int32_t* cnt, const unsigned long long* scan, int64_t n, int32_t* oo) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        oo[i] = cnt[i] > 0 ? (int32_t)scan[i] : -1;
}

__global__ void k_keys_to_idx(const unsigned long long* keys, int64_t n, int32_t* idx) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        idx[i] = (int32_t)(uint32_t)(keys[i] & 0xffffffffull);
}

// ---- compact / explicit layouts on the device (see layout.h for the compact format) ----
__global__ void k_compact_nodes(const int32_t* co, const int32_t* oo, const int32_t* cnt, const int32_t* idx, int64_t n,
                                int64_t ni, uint2* node, uint2* kid) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        const int32_t c = co[i];
        if (c != -1) {
            uint32_t mask = 0, leaves = 0;
            bool leafkids = true;
            for (int k = 0; k < 8; ++k) {
                const int64_t j = (int64_t)c + k;
                if (j >= n) continue;
                if (co[j] != -1) leafkids = false;
                if (co[j] == -1 && oo[j] == -1) continue;  // empty leaf, glsl:467
                mask |= 1u << k;
                if (co[j] == -1) leaves |= 1u << k;
            }
            // bits 8-15: the existing children that are leaves (render_core.h ORT_LEAFMASK_SHIFT)
            node[i] = make_uint2((uint32_t)c, 0x80000000u | (leafkids ? 0x40000000u : 0u) | (leaves << 8) | mask);
            int32_t sid[8];
            for (int k = 0; k < 8; ++k) {
                const int64_t j = (int64_t)c + k;
                sid[k] = (j < n && co[j] == -1 && cnt[j] == 1) ? idx[oo[j]] : -1;
            }
            uint32_t w0, w1;
            kid_entry(sid, w0, w1);  // rejected-sphere skip entry (kid_table.h)
            kid[i] = make_uint2(w0, w1);
        } else {
            kid[i] = make_uint2(0u, 0u);
            const int32_t v = cnt[i] > 0 ? cnt[i] : 0;
            // one-sphere leaves point into the per-sphere tail (layout.h)
            node[i] = make_uint2(v == 1 ? (uint32_t)(ni + idx[oo[i]]) : (v > 0 ? (uint32_t)oo[i] : 0u), (uint32_t)v);
        }
    }
}

// entries 0..ni-1: objectIndices; ni..ni+nsph-1: the per-sphere tail (layout.h)
__global__ void k_leaf_gather(const int32_t* idx, int64_t ni, int64_t n, const float4* sp, float4* leaf_sph,
                              int32_t* leaf_idx) {
    for (int64_t e = blockIdx.x * (int64_t)kB + threadIdx.x; e < n; e += (int64_t)gridDim.x * kB) {
        const int32_t s = e < ni ? idx[e] : (int32_t)(e - ni);
        const float4 v = sp[s];
        leaf_sph[e] = make_float4(v.x, v.y, v.z, v.w * v.w);  // radius^2 (layout.h)
        leaf_idx[e] = s;
    }
}

__global__ void k_fill_nan(float* p, int64_t n) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB)
        p[i] = __uint_as_float(0x7fc00000u);
}

// Planes of the nodes [start, end) at depth d (tree depth D): box = planes[cell << s ...].
template <bool CHECK>
__global__ void k_planes(int64_t start, int64_t end, int d, int D, const float* nmin, const float* nmax,
                         const uint32_t* cell, float* planes, int* bad) {
    const int64_t P1 = ((int64_t)1 << D) + 1;
    const int s = D - d;
    for (int64_t i = start + blockIdx.x * (int64_t)kB + threadIdx.x; i < end; i += (int64_t)gridDim.x * kB) {
        const uint32_t cl = cell[i];
        const uint32_t c[3] = {cl & 1023u, (cl >> 10) & 1023u, (cl >> 20) & 1023u};
        for (int a = 0; a < 3; ++a) {
            const int64_t lo = a * P1 + ((int64_t)c[a] << s);
            const int64_t hi = a * P1 + ((int64_t)(c[a] + 1) << s);
            if (CHECK) {
                if (__float_as_uint(planes[lo]) != __float_as_uint(nmin[3 * i + a]) ||
                    __float_as_uint(planes[hi]) != __float_as_uint(nmax[3 * i + a]))
                    atomicOr(bad, 1);
            } else {
                planes[lo] = nmin[3 * i + a];
                planes[hi] = nmax[3 * i + a];
            }
        }
    }
}

__global__ void k_explicit(const float* nmin, const float* nmax, const int32_t* co, const int32_t* oo, int64_t n,
                           float4* A, float4* B) {
    for (int64_t i = blockIdx.x * (int64_t)kB + threadIdx.x; i < n; i += (int64_t)gridDim.x * kB) {
        A[i] = make_float4(nmin[3 * i], nmin[3 * i + 1], nmin[3 * i + 2], __int_as_float(co[i]));
        B[i] = make_float4(nmax[3 * i], nmax[3 * i + 1], nmax[3 * i + 2], __int_as_float(oo[i]));
    }
}

int grid_for(int64_t n) {
    const int64_t b = (n + kB - 1) / kB;
    return (int)std::max<int64_t>(1, std::min<int64_t>(b, 65536));
}

struct Level {  // one level's node arrays (device)
    int64_t n = 0;
    float* nmin = nullptr;
    float* nmax = nullptr;
    int32_t* co = nullptr;
    int32_t* cnt = nullptr;
    uint32_t* cell = nullptr;
};

#define GB_CHK(expr)                                                                     \
    do {                                                                                 \
        hipError_t _e = (expr);                                                          \
        if (_e != hipSuccess) return std::string(#expr ": ") + hipGetErrorString(_e);    \
    } while (0)

template <class T>
std::string dalloc(T*& p, int64_t n) {
    p = nullptr;
    GB_CHK(hipMalloc((void**)&p, (size_t)std::max<int64_t>(n, 1) * sizeof(T)));
    return "";
}

// Scratch that frees itself; every free first drains the stream (kernels already queued
// may still read the buffer).
struct Scratch {
    hipStream_t s;
    std::vector<void*> ptrs;
    explicit Scratch(hipStream_t st) : s(st) {}
    ~Scratch() {
        (void)hipStreamSynchronize(s);
        for (void* p : ptrs) (void)hipFree(p);
    }
    template <class T>
    std::string get(T*& p, int64_t n) {
        std::string e = dalloc(p, n);
        if (e.empty()) ptrs.push_back(p);
        return e;
    }
    void release(void* p) {
        if (!p) return;
        (void)hipStreamSynchronize(s);
        for (auto& q : ptrs)
            if (q == p) {
                (void)hipFree(q);
                q = nullptr;
            }
    }
};

std::string alloc_level(Level& L, int64_t n, Scratch& sc) {
    L.n = n;
    std::string e;
    if (!(e = sc.get(L.nmin, 3 * n)).empty() || !(e = sc.get(L.nmax, 3 * n)).empty() || !(e = sc.get(L.co, n)).empty() ||
        !(e = sc.get(L.cnt, n)).empty() || !(e = sc.get(L.cell, n)).empty())
        return e;
    return "";
}

}  // namespace

void freeGpuTree(GpuTree& t) {
    void* all[] = {t.node_min, t.node_max, t.co, t.oo, t.cnt, t.idx, t.cell};
    for (void* p : all)
        if (p) (void)hipFree(p);
    t = GpuTree();
}

std::string gpuBuildOctree(const float4* sp, int32_t n, int32_t maxDepth, int32_t mspn, hipStream_t s, GpuTree& out) {
    freeGpuTree(out);
    if (n <= 0) return "Sphere list is empty";  // src/octree.cpp:50-52
    hipEvent_t e0, e1;
    GB_CHK(hipEventCreate(&e0));
    GB_CHK(hipEventCreate(&e1));
    struct EvGuard {
        hipEvent_t a, b;
        ~EvGuard() {
            (void)hipEventDestroy(a);
            (void)hipEventDestroy(b);
        }
    } evg{e0, e1};
    GB_CHK(hipEventRecord(e0, s));
    const unsigned long long mspnSz = (unsigned long long)(int64_t)mspn;  // (size_t)maxSpheresPerNode
    Scratch sc(s);
    std::string err;
    std::vector<Level> levels;
    levels.emplace_back();
    if (!(err = alloc_level(levels[0], 1, sc)).empty()) return err;
    {
        const int nb = std::min(1024, grid_for(n));
        float* part;
        if (!(err = sc.get(part, 6 * (int64_t)nb)).empty()) return err;
        hipLaunchKernelGGL(k_bounds, dim3(nb), dim3(kB), 0, s, sp, n, part);
        hipLaunchKernelGGL(k_root, dim3(1), dim3(1), 0, s, part, nb, levels[0].nmin, levels[0].nmax, levels[0].cell);
        GB_CHK(hipGetLastError());
    }
    int* d_unordered;
    if (!(err = sc.get(d_unordered, 1)).empty()) return err;
    GB_CHK(hipMemsetAsync(d_unordered, 0, sizeof(int), s));
    // level-0 pairs: (root, every sphere)
    int64_t np = n;
    int32_t *pnode, *psph;
    if (!(err = sc.get(pnode, np)).empty() || !(err = sc.get(psph, np)).empty()) return err;
    hipLaunchKernelGGL(k_iota_pairs, dim3(grid_for(np)), dim3(kB), 0, s, pnode, psph, np);
    // leaf keys, grown as levels add leaves
    unsigned long long* leaf_keys = nullptr;
    int64_t leaf_cap = 0, leaf_n = 0;
    std::vector<int64_t> starts = {0};
    for (int d = 0;; ++d) {
        Level& L = levels[d];
        const int64_t start = starts[d];
        GB_CHK(hipMemsetAsync(L.cnt, 0, (size_t)L.n * 4, s));
        if (np > 0) hipLaunchKernelGGL(k_count, dim3(grid_for(np)), dim3(kB), 0, s, pnode, np, L.cnt);
        // ranks of the subdividing nodes
        uint32_t *flag, *rank;
        if (!(err = sc.get(flag, L.n)).empty() || !(err = sc.get(rank, L.n)).empty()) return err;
        hipLaunchKernelGGL(k_flags, dim3(grid_for(L.n)), dim3(kB), 0, s, L.cnt, L.n, d, maxDepth, mspnSz, flag);
        size_t tb = 0;
        GB_CHK(rocprim::exclusive_scan(nullptr, tb, flag, rank, 0u, (size_t)L.n, rocprim::plus<uint32_t>(), s));
        char* tmp;
        if (!(err = sc.get(tmp, (int64_t)tb)).empty()) return err;
        GB_CHK(rocprim::exclusive_scan(tmp, tb, flag, rank, 0u, (size_t)L.n, rocprim::plus<uint32_t>(), s));
        uint32_t tail[2];
        GB_CHK(hipMemcpyAsync(&tail[0], rank + (L.n - 1), 4, hipMemcpyDeviceToHost, s));
        GB_CHK(hipMemcpyAsync(&tail[1], flag + (L.n - 1), 4, hipMemcpyDeviceToHost, s));
        GB_CHK(hipStreamSynchronize(s));
        sc.release(tmp);
        const int64_t n_int = (int64_t)tail[0] + tail[1];
        const int64_t next_start = start + L.n;
        if (next_start + 8 * n_int > (int64_t)INT32_MAX) return "tree has more than 2^31 nodes";
        Level next;
        if (n_int > 0) {
            if (!(err = alloc_level(next, 8 * n_int, sc)).empty()) return err;
        }
        hipLaunchKernelGGL(k_level, dim3(grid_for(L.n)), dim3(kB), 0, s, L.n, d, maxDepth, mspnSz, next_start, rank,
                           L.nmin, L.nmax, L.cell, L.co, L.cnt, next.nmin, next.nmax, next.cell, d_unordered);
        GB_CHK(hipGetLastError());
        sc.release(flag);
        sc.release(rank);
        // pair codes and their slots
        int64_t nq = 0, nleaf = 0;
        int32_t *qnode = nullptr, *qsph = nullptr;
        if (np > 0) {
            uint16_t* code;
            unsigned long long* off;
            if (!(err = sc.get(code, np)).empty() || !(err = sc.get(off, np)).empty()) return err;
            hipLaunchKernelGGL(k_codes, dim3(grid_for(np)), dim3(kB), 0, s, pnode, psph, np, L.co, L.nmin, L.nmax, sp,
                               code);
            auto it = rocprim::make_transform_iterator(code, CodeCounts());
            tb = 0;
            GB_CHK(rocprim::exclusive_scan(nullptr, tb, it, off, 0ull, (size_t)np, rocprim::plus<unsigned long long>(), s));
            if (!(err = sc.get(tmp, (int64_t)tb)).empty()) return err;
            GB_CHK(rocprim::exclusive_scan(tmp, tb, it, off, 0ull, (size_t)np, rocprim::plus<unsigned long long>(), s));
            unsigned long long lastOff;
            uint16_t lastCode;
            GB_CHK(hipMemcpyAsync(&lastOff, off + (np - 1), 8, hipMemcpyDeviceToHost, s));
            GB_CHK(hipMemcpyAsync(&lastCode, code + (np - 1), 2, hipMemcpyDeviceToHost, s));
            GB_CHK(hipStreamSynchronize(s));
            sc.release(tmp);
            const unsigned long long lastCnt = CodeCounts()(lastCode);
            nq = (int64_t)((lastOff & 0xffffffffull) + (lastCnt & 0xffffffffull));
            nleaf = (int64_t)((lastOff >> 32) + (lastCnt >> 32));
            if (nq > 0xffffffffll || leaf_n + nleaf > (int64_t)INT32_MAX) return "too many (node, sphere) pairs";
            if (leaf_n + nleaf > leaf_cap) {  // grow the leaf-key buffer
                const int64_t cap = std::max<int64_t>(leaf_n + nleaf, 2 * leaf_cap);
                unsigned long long* nk;
                if (!(err = sc.get(nk, cap)).empty()) return err;
                if (leaf_n > 0) GB_CHK(hipMemcpyAsync(nk, leaf_keys, (size_t)leaf_n * 8, hipMemcpyDeviceToDevice, s));
                if (leaf_keys) sc.release(leaf_keys);
                leaf_keys = nk;
                leaf_cap = cap;
            }
            if (nq > 0) {
                if (!(err = sc.get(qnode, nq)).empty() || !(err = sc.get(qsph, nq)).empty()) return err;
            }
            hipLaunchKernelGGL(k_emit, dim3(grid_for(np)), dim3(kB), 0, s, pnode, psph, np, code, off, L.co, start,
                               next_start, leaf_n, qnode, qsph, leaf_keys);
            GB_CHK(hipGetLastError());
            sc.release(code);
            sc.release(off);
        }
        sc.release(pnode);
        sc.release(psph);
        pnode = qnode;
        psph = qsph;
        np = nq;
        leaf_n += nleaf;
        if (n_int == 0) break;
        starts.push_back(next_start);
        levels.push_back(next);
    }
    // concatenate the levels (BFS order) into the output arrays
    const int64_t total = starts.back() + levels.back().n;
    out.n_nodes = (int32_t)total;
    out.depth = (int)levels.size() - 1;
    out.level_start = starts;
    out.level_start.push_back(total);
    if (!(err = dalloc(out.node_min, 3 * total)).empty() || !(err = dalloc(out.node_max, 3 * total)).empty() ||
        !(err = dalloc(out.co, total)).empty() || !(err = dalloc(out.oo, total)).empty() ||
        !(err = dalloc(out.cnt, total)).empty() || !(err = dalloc(out.cell, total)).empty()) {
        freeGpuTree(out);
        return err;
    }
    for (size_t d = 0; d < levels.size(); ++d) {
        const Level& L = levels[d];
        const int64_t st = starts[d];
        GB_CHK(hipMemcpyAsync(out.node_min + 3 * st, L.nmin, (size_t)L.n * 12, hipMemcpyDeviceToDevice, s));
        GB_CHK(hipMemcpyAsync(out.node_max + 3 * st, L.nmax, (size_t)L.n * 12, hipMemcpyDeviceToDevice, s));
        GB_CHK(hipMemcpyAsync(out.co + st, L.co, (size_t)L.n * 4, hipMemcpyDeviceToDevice, s));
        GB_CHK(hipMemcpyAsync(out.cnt + st, L.cnt, (size_t)L.n * 4, hipMemcpyDeviceToDevice, s));
        GB_CHK(hipMemcpyAsync(out.cell + st, L.cell, (size_t)L.n * 4, hipMemcpyDeviceToDevice, s));
    }
    GB_CHK(hipStreamSynchronize(s));
    for (Level& L : levels) {
        sc.release(L.nmin);
        sc.release(L.nmax);
        sc.release(L.co);
        sc.release(L.cnt);
        sc.release(L.cell);
    }
    // objectsOffset = exclusive scan of the leaf counts (internal counts are 0)
    {
        unsigned long long* scan;
        if (!(err = sc.get(scan, total)).empty()) return err;
        auto it = rocprim::make_transform_iterator(out.cnt, [] __host__ __device__(int32_t c) {
            return (unsigned long long)(c > 0 ? c : 0);
        });
        size_t tb = 0;
        GB_CHK(rocprim::exclusive_scan(nullptr, tb, it, scan, 0ull, (size_t)total, rocprim::plus<unsigned long long>(), s));
        char* tmp;
        if (!(err = sc.get(tmp, (int64_t)tb)).empty()) return err;
        GB_CHK(rocprim::exclusive_scan(tmp, tb, it, scan, 0ull, (size_t)total, rocprim::plus<unsigned long long>(), s));
        hipLaunchKernelGGL(k_oo, dim3(grid_for(total)), dim3(kB), 0, s, out.cnt, scan, total, out.oo);
        GB_CHK(hipGetLastError());
    }
    // objectIndices: leaf keys sorted by (BFS node, sphere)
    out.n_indices = leaf_n;
    out.n_spheres = n;
    if (!(err = dalloc(out.idx, leaf_n)).empty()) {
        freeGpuTree(out);
        return err;
    }
    if (leaf_n > 0) {
        unsigned long long* sorted;
        if (!(err = sc.get(sorted, leaf_n)).empty()) return err;
        int nbits = 1;
        while (nbits < 32 && ((int64_t)1 << nbits) < total) ++nbits;
        size_t tb = 0;
        GB_CHK(rocprim::radix_sort_keys(nullptr, tb, leaf_keys, sorted, (size_t)leaf_n, 0, 32 + nbits, s));
        char* tmp;
        if (!(err = sc.get(tmp, (int64_t)tb)).empty()) return err;
        GB_CHK(rocprim::radix_sort_keys(tmp, tb, leaf_keys, sorted, (size_t)leaf_n, 0, 32 + nbits, s));
        hipLaunchKernelGGL(k_keys_to_idx, dim3(grid_for(leaf_n)), dim3(kB), 0, s, sorted, leaf_n, out.idx);
        GB_CHK(hipGetLastError());
    }
    int unordered = 0;
    GB_CHK(hipMemcpyAsync(&unordered, d_unordered, 4, hipMemcpyDeviceToHost, s));
    GB_CHK(hipEventRecord(e1, s));
    GB_CHK(hipStreamSynchronize(s));
    out.ordered = unordered == 0;
    float ms = 0.0f;
    GB_CHK(hipEventElapsedTime(&ms, e0, e1));
    out.seconds = ms * 1e-3;
    return "";
}

bool gpuCompactLayout(const GpuTree& t, const float4* sp, int maxDepth, hipStream_t s, CompactDev& out,
                      std::string& why) {
    out = CompactDev();
    if (t.depth > maxDepth) {
        why = "tree deeper than the compact layout supports";
        return false;
    }
    if (8 * (uint64_t)t.n_nodes >= ((uint64_t)1 << 32) ||
        16 * ((uint64_t)t.n_indices + (uint64_t)t.n_spheres) >= ((uint64_t)1 << 32)) {
        why = "compact buffers exceed 4 GiB";
        return false;
    }
    auto fail = [&](const std::string& e) {
        why = e;
        void* all[] = {out.node, out.leaf_sph, out.leaf_idx, out.planes, out.kid};
        for (void* p : all)
            if (p) (void)hipFree(p);
        out = CompactDev();
        return false;
    };
    const int64_t n = t.n_nodes, ni = t.n_indices, ne = t.n_indices + t.n_spheres;
    const int D = t.depth;
    const int64_t np = 3 * (((int64_t)1 << D) + 1);
    std::string e;
    if (!(e = dalloc(out.node, n)).empty() || !(e = dalloc(out.kid, n)).empty() || !(e = dalloc(out.leaf_sph, ne)).empty() ||
        !(e = dalloc(out.leaf_idx, ne)).empty() || !(e = dalloc(out.planes, np)).empty())
        return fail(e);
    out.node_bytes = (size_t)n * 8;
    out.leaf_bytes = (size_t)std::max<int64_t>(ne, 1) * 16;
    out.idx_bytes = (size_t)std::max<int64_t>(ne, 1) * 4;
    out.plane_bytes = (size_t)np * 4;
    int* bad;
    if (!(e = dalloc(bad, 1)).empty()) return fail(e);
    struct Free {
        int* p;
        ~Free() { (void)hipFree(p); }
    } fb{bad};
    hipLaunchKernelGGL(k_compact_nodes, dim3(grid_for(n)), dim3(kB), 0, s, t.co, t.oo, t.cnt, t.idx, n, ni, out.node,
                       out.kid);
    if (ne > 0)
        hipLaunchKernelGGL(k_leaf_gather, dim3(grid_for(ne)), dim3(kB), 0, s, t.idx, ni, ne, sp, out.leaf_sph,
                           out.leaf_idx);
    hipLaunchKernelGGL(k_fill_nan, dim3(grid_for(np)), dim3(kB), 0, s, out.planes, np);
    if (hipMemsetAsync(bad, 0, 4, s) != hipSuccess) return fail("hipMemsetAsync");
    for (int d = 0; d <= D; ++d) {
        const int64_t a = t.level_start[d], b = t.level_start[d + 1];
        hipLaunchKernelGGL((k_planes<false>), dim3(grid_for(b - a)), dim3(kB), 0, s, a, b, d, D, t.node_min, t.node_max,
                           t.cell, out.planes, bad);
    }
    for (int d = 0; d <= D; ++d) {  // every node's box must read back from the tables
        const int64_t a = t.level_start[d], b = t.level_start[d + 1];
        hipLaunchKernelGGL((k_planes<true>), dim3(grid_for(b - a)), dim3(kB), 0, s, a, b, d, D, t.node_min, t.node_max,
                           t.cell, out.planes, bad);
    }
    if (hipGetLastError() != hipSuccess) return fail("compact layout kernels");
    int hbad = 0;
    if (hipMemcpyAsync(&hbad, bad, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
        return fail("compact layout readback");
    if (hbad) return fail("node box not derivable from split planes");
    return true;
}

std::string gpuExplicitLayout(const GpuTree& t, hipStream_t s, ExplicitDev& out) {
    out = ExplicitDev();
    const int64_t n = t.n_nodes, ni = t.n_indices;
    std::string e;
    if (!(e = dalloc(out.nodeA, n)).empty() || !(e = dalloc(out.nodeB, n)).empty() || !(e = dalloc(out.cnt, n)).empty() ||
        !(e = dalloc(out.indices, ni)).empty())
        return e;
    hipLaunchKernelGGL(k_explicit, dim3(grid_for(n)), dim3(kB), 0, s, t.node_min, t.node_max, t.co, t.oo, n, out.nodeA,
                       out.nodeB);
    GB_CHK(hipGetLastError());
    GB_CHK(hipMemcpyAsync(out.cnt, t.cnt, (size_t)n * 4, hipMemcpyDeviceToDevice, s));
    if (ni > 0) GB_CHK(hipMemcpyAsync(out.indices, t.idx, (size_t)ni * 4, hipMemcpyDeviceToDevice, s));
    GB_CHK(hipStreamSynchronize(s));
    return "";
}

namespace {
// Grid-stride, one atomic per block: an atomic per wave on the one counter serialised
// (~0.5 M atomics at C5 took 3.8 ms per bounce).
__global__ void k_path_keys(const float4* po, const float4* pd, int n, MortonPlan mp, const uint32_t* spread,
                            uint32_t* keys, int* vals, int* count) {
    __shared__ int wave_alive[kB / 64];
    int alive_n = 0;
    for (int k = blockIdx.x * kB + threadIdx.x; k < n; k += gridDim.x * kB) {
        const float4 d = pd[k];
        const bool alive = d.w != 0.0f;
        uint32_t key = 0xffffffffu;
        if (alive) key = path_key(po[k], d, mp, spread);
        keys[k] = key;
        vals[k] = k;
        alive_n += alive ? 1 : 0;
    }
    // block sum: wave reduction by ballot counts is not possible for per-lane sums, so LDS
    int v = alive_n;
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off);
    if ((threadIdx.x & 63) == 0) wave_alive[threadIdx.x >> 6] = v;
    __syncthreads();
    if (threadIdx.x == 0) {
        int t = 0;
        for (int w = 0; w < kB / 64; ++w) t += wave_alive[w];
        if (t) atomicAdd(count, t);
    }
}

// sortListBounded, before the sort: keys [*count, bound) <- all ones (grid-stride; the grid
// is sized on the host, the range on the device)
__global__ void __launch_bounds__(kB) k_pad_keys(uint32_t* keys, const int* count, int bound) {
    const int n = *count;
    for (int i = n + (int)(blockIdx.x * kB + threadIdx.x); i < bound; i += (int)(gridDim.x * kB)) keys[i] = 0xffffffffu;
}

// ... after it: a list longer than the bound goes on in append order (vals_in -> vals_out)
__global__ void __launch_bounds__(kB) k_overflow_copy(const int* vals_in, int* vals_out, const int* count, int bound) {
    const int n = *count;
    if (n <= bound) return;
    for (int i = (int)(blockIdx.x * kB + threadIdx.x); i < n; i += (int)(gridDim.x * kB)) vals_out[i] = vals_in[i];
}

}  // namespace

// The path-list sorts' rocPRIM configuration.  rocPRIM 4.2 has no tuned onesweep entry for
// gfx950 and falls back to 4 radix bits per pass (eight passes over a 32-bit key); this is its
// gfx942 entry for 4-byte keys with 4-byte values: 8 bits per pass, 1024 x 8 items per block.
#ifndef ORT_SORT_RADIX_BITS
#define ORT_SORT_RADIX_BITS 8
#endif
#if ORT_SORT_RADIX_BITS > 0
using ListSortConfig = rocprim::radix_sort_config<
    rocprim::default_config, rocprim::default_config,
    rocprim::radix_sort_onesweep_config<rocprim::kernel_config<1024, 8>, rocprim::kernel_config<1024, 8>,
                                        ORT_SORT_RADIX_BITS, rocprim::block_radix_rank_algorithm::match>>;
#else
using ListSortConfig = rocprim::default_config;
#endif

hipError_t sortList(void* temp, size_t temp_bytes, int n, const SortBuffers& b, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    return rocprim::radix_sort_pairs<ListSortConfig>(temp, temp_bytes, b.keys_in, b.keys_out, b.vals_in, b.vals_out, (size_t)n, 0,
                                     kPathKeyBits, s);
}

hipError_t sortListBounded(void* temp, size_t temp_bytes, int bound, const int* count, const SortBuffers& b,
                           hipStream_t s, int key_bits) {
    if (bound <= 0) return hipSuccess;
    constexpr int kGrid = 512;  // 128 k lanes: the pad (usually < 2 % of the list) and the rare copy
    hipLaunchKernelGGL(k_pad_keys, dim3(kGrid), dim3(kB), 0, s, b.keys_in, count, bound);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    // stable LSD sort: a real key equal to the pad's low key_bits stays ahead of the pads
    e = rocprim::radix_sort_pairs<ListSortConfig>(temp, temp_bytes, b.keys_in, b.keys_out, b.vals_in, b.vals_out, (size_t)bound, 0,
                                  key_bits, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_overflow_copy, dim3(kGrid), dim3(kB), 0, s, (const int*)b.vals_in, b.vals_out, count, bound);
    return hipGetLastError();
}

size_t sortAliveTempBytes(int n) {
    size_t tb = 0;
    (void)rocprim::radix_sort_pairs<ListSortConfig>(nullptr, tb, (uint32_t*)nullptr, (uint32_t*)nullptr, (int*)nullptr, (int*)nullptr,
                                    (size_t)std::max(n, 1), 0, 31);
    return tb;
}

hipError_t sortAlive(void* temp, size_t temp_bytes, const float4* po, const float4* pd, int n, const float* root_lo,
                     const float* root_hi, const uint32_t* spread, const SortBuffers& b, int* count, hipStream_t s) {
    hipError_t e = hipMemsetAsync(count, 0, sizeof(int), s);
    if (e != hipSuccess) return e;
    const MortonPlan mp = mortonPlan(root_lo, root_hi);
    hipLaunchKernelGGL(k_path_keys, dim3(std::min((n + kB - 1) / kB, 2048)), dim3(kB), 0, s, po, pd, n, mp, spread,
                       b.keys_in, b.vals_in, count);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // alive keys are < 2^30, dead keys 0xffffffff: on bits [0, 31) every dead key sorts after
    // every alive one
    return rocprim::radix_sort_pairs<ListSortConfig>(temp, temp_bytes, b.keys_in, b.keys_out, b.vals_in, b.vals_out, (size_t)n, 0, 31, s);
}

}  // namespace ort
