// layout.cpp -- see layout.h.
#include "layout.h"

#include <cstring>

#include "kid_table.h"
#include "render_core_flags.h"

namespace ort {

static inline bool same_bits(float a, float b) {
    uint32_t x, y;
    std::memcpy(&x, &a, 4);
    std::memcpy(&y, &b, 4);
    return x == y;
}

std::string validateScene(const SceneInput& in) {
    if (in.n_spheres < 0 || in.n_nodes < 0 || in.n_indices < 0) return "negative count";
    if (in.n_spheres > 0 && (!in.sph_cr || !in.sph_ma || !in.sph_fr)) return "null sphere array";
    if (in.n_nodes > 0 && (!in.node_min || !in.node_max || !in.co || !in.oo || !in.cnt)) return "null node array";
    if (in.n_indices > 0 && !in.indices) return "null object_indices";
    if (in.n_indices > (int64_t)INT32_MAX) return "object_indices exceeds int32 range";
    for (int64_t e = 0; e < in.n_indices; ++e)
        if (in.indices[e] < 0 || in.indices[e] >= in.n_spheres) return "object index out of range at entry " + std::to_string(e);
    for (int32_t i = 0; i < in.n_nodes; ++i) {
        if (in.co[i] < -1) return "children_offset < -1 at node " + std::to_string(i);
        if (in.co[i] == -1 && in.cnt[i] > 0) {
            if (in.oo[i] < 0 || (int64_t)in.oo[i] + in.cnt[i] > in.n_indices)
                return "leaf object range outside object_indices at node " + std::to_string(i);
        }
    }
    return "";
}

int treeDepth(const SceneInput& in) {
    if (in.n_nodes <= 0) return -1;
    std::vector<int8_t> depth((size_t)in.n_nodes, -1);
    std::vector<int32_t> queue;
    queue.reserve((size_t)in.n_nodes);
    queue.push_back(0);
    depth[0] = 0;
    int maxd = 0;
    for (size_t h = 0; h < queue.size(); ++h) {
        const int32_t i = queue[h];
        const int32_t co = in.co[i];
        if (co == -1) continue;
        for (int k = 0; k < 8; ++k) {
            const int64_t c = (int64_t)co + k;
            if (c >= in.n_nodes) continue;
            if (depth[c] != -1) return -1;
            if (depth[i] >= 126) return -1;
            depth[c] = (int8_t)(depth[i] + 1);
            if (depth[c] > maxd) maxd = depth[c];
            queue.push_back((int32_t)c);
        }
    }
    return maxd;
}

bool buildCompactLayout(const SceneInput& in, int maxDepth, CompactLayout& out, std::string& why) {
    const int32_t n = in.n_nodes;
    if (n <= 0) { why = "no nodes"; return false; }
    // the kernel addresses node records and leaf spheres with 32-bit byte offsets
    if (8 * (uint64_t)n >= ((uint64_t)1 << 32) ||
        16 * ((uint64_t)in.n_indices + (uint64_t)in.n_spheres) >= ((uint64_t)1 << 32)) {
        why = "compact buffers exceed 4 GiB";
        return false;
    }
    // Pass 1: BFS for depth and cell coordinates of every reachable node.
    std::vector<int8_t> depth((size_t)n, -1);
    std::vector<uint32_t> cell((size_t)n, 0);  // 10 bits per axis: x | y << 10 | z << 20
    std::vector<int32_t> order;
    order.reserve((size_t)n);
    order.push_back(0);
    depth[0] = 0;
    int D = 0;
    for (size_t h = 0; h < order.size(); ++h) {
        const int32_t i = order[h];
        const int32_t co = in.co[i];
        if (co == -1) continue;
        const uint32_t cx = cell[i] & 1023u, cy = (cell[i] >> 10) & 1023u, cz = (cell[i] >> 20) & 1023u;
        for (int k = 0; k < 8; ++k) {
            const int64_t c = (int64_t)co + k;
            if (c >= n) continue;
            if (depth[c] != -1) { why = "node reachable twice"; return false; }
            const int d = depth[i] + 1;
            if (d > maxDepth) { why = "tree deeper than the compact layout supports"; return false; }
            depth[c] = (int8_t)d;
            if (d > D) D = d;
            const uint32_t nx = (cx << 1) | (uint32_t)((k >> 1) & 1);
            const uint32_t ny = (cy << 1) | (uint32_t)(k & 1);
            const uint32_t nz = (cz << 1) | (uint32_t)((k >> 2) & 1);
            cell[c] = nx | (ny << 10) | (nz << 20);
            order.push_back((int32_t)c);
        }
    }
    // Pass 2: the split-plane tables, checked against every reachable node's stored box.
    const size_t P1 = ((size_t)1 << D) + 1;
    out.depth = D;
    out.ordered = true;
    out.planes.assign(3 * P1, 0.0f);
    std::vector<uint8_t> set(3 * P1, 0);
    for (int32_t i : order) {
        const int s = D - depth[i];
        const uint32_t c[3] = {cell[i] & 1023u, (cell[i] >> 10) & 1023u, (cell[i] >> 20) & 1023u};
        for (int a = 0; a < 3; ++a) {
            const size_t lo = a * P1 + ((size_t)c[a] << s);
            const size_t hi = a * P1 + ((size_t)(c[a] + 1) << s);
            const float vlo = in.node_min[3 * (size_t)i + a];
            const float vhi = in.node_max[3 * (size_t)i + a];
            if (!(vlo <= vhi)) out.ordered = false;  // also false for NaN
            if (!set[lo]) { out.planes[lo] = vlo; set[lo] = 1; }
            else if (!same_bits(out.planes[lo], vlo)) { why = "node box not derivable from split planes"; return false; }
            if (!set[hi]) { out.planes[hi] = vhi; set[hi] = 1; }
            else if (!same_bits(out.planes[hi], vhi)) { why = "node box not derivable from split planes"; return false; }
        }
    }
    // Unset planes belong to splits of nodes whose children are all out of range: never
    // read for a pushed child.  Fill with NaN so a logic error would show.
    for (size_t k = 0; k < set.size(); ++k)
        if (!set[k]) {
            const uint32_t qnan = 0x7fc00000u;
            std::memcpy(&out.planes[k], &qnan, 4);
        }
    // Node records, and the rejected-sphere skip entries (kid_table.h).
    out.node.assign(2 * (size_t)n, 0u);
    out.kid.assign(2 * (size_t)n, 0u);
    for (int32_t i = 0; i < n; ++i) {
        const int32_t co = in.co[i];
        if (co != -1) {
            uint32_t mask = 0, leaves = 0;
            bool leafkids = true;
            for (int k = 0; k < 8; ++k) {
                const int64_t c = (int64_t)co + k;
                if (c >= n) continue;
                if (in.co[c] != -1) leafkids = false;
                if (in.co[c] == -1 && in.oo[c] == -1) continue;  // empty leaf, glsl:467
                mask |= 1u << k;
                if (in.co[c] == -1) leaves |= 1u << k;
            }
            out.node[2 * (size_t)i] = (uint32_t)co;
            out.node[2 * (size_t)i + 1] = ORT_INTERNAL_FLAG_HOST | (leafkids ? ORT_LEAFKIDS_FLAG_HOST : 0u) |
                                          (leaves << ORT_LEAFMASK_SHIFT_HOST) | mask;
            int32_t sid[8];
            for (int k = 0; k < 8; ++k) {
                const int64_t c = (int64_t)co + k;
                sid[k] = (c < n && in.co[c] == -1 && in.cnt[c] == 1) ? in.indices[in.oo[c]] : -1;
            }
            kid_entry(sid, out.kid[2 * (size_t)i], out.kid[2 * (size_t)i + 1]);
        } else {
            const int32_t cntv = in.cnt[i] > 0 ? in.cnt[i] : 0;
            // one-sphere leaves point into the per-sphere tail (layout.h)
            out.node[2 * (size_t)i] = cntv == 1 ? (uint32_t)(in.n_indices + in.indices[in.oo[i]])
                                               : (cntv > 0 ? (uint32_t)in.oo[i] : 0u);
            out.node[2 * (size_t)i + 1] = (uint32_t)cntv;
        }
    }
    // Leaf entries, then the per-sphere tail (entry n_indices + s = sphere s).
    const int64_t ne = in.n_indices + in.n_spheres;
    out.leaf_sph.resize(4 * (size_t)ne);
    out.leaf_idx.resize((size_t)ne);
    for (int64_t e = 0; e < ne; ++e) {
        const int32_t s = e < in.n_indices ? in.indices[e] : (int32_t)(e - in.n_indices);
        std::memcpy(&out.leaf_sph[4 * (size_t)e], in.sph_cr + 4 * (size_t)s, 12);
        const float rad = in.sph_cr[4 * (size_t)s + 3];
        out.leaf_sph[4 * (size_t)e + 3] = rad * rad;  // the kernel's r * r, rounded once (fp32)
        out.leaf_idx[(size_t)e] = s;
    }
    return true;
}

}  // namespace ort
