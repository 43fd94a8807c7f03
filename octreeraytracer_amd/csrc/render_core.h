// render_core.h -- per-pixel path of the MI355X kernel (__host__ __device__).
//
// Restates shaders/octree_fragment_shader.glsl for one pixel:
//   main()                    glsl:636-664   -> shade_pixel
//   radiance()                glsl:597-633   -> radiance
//   Material_bsdf/refract/    glsl:508-589   -> bsdf
//     schlick
//   skyColor                  glsl:592-595
//   Camera_getRay             glsl:205-221   -> camera_ray
//   random_in_unit_*/cosine   glsl:104-173
//   Sphere_hit                glsl:224-273   -> sphere_hit_t
//   traverseOctree            glsl:290-481   -> traverse_compact (fast layout) /
//                                               traverse_explicit (reference layout)
//   bruteForceIntersect       glsl:484-498   -> traverse_brute
//
// traverse_compact reproduces the reference's stack DFS exactly but stores it as one
// FRAME per tree level (children offset, parent tmin, and an 8-bit mask of the children
// still to visit, in traversal-order rank), and re-derives every box from per-axis split
// planes (see layout.h).  The reference pushes the surviving children of a node in
// reverse traversal order and always pops the top, so its stack is exactly "for every
// ancestor level, the not-yet-visited surviving siblings in traversal order": popping
// the lowest rank bit of the deepest non-empty frame pops the same node with the same
// tmin.  A hit ends the walk after its leaf (glsl:336), so `closest` is still t_max at
// every push, and the 200-entry cap (glsl:471) cannot bind for depth <= 28 (<= 7d+1
// entries); the compact layout is only used for depth <= ORT_COMPACT_MAX_DEPTH.
#pragma once

#include <stdint.h>

#include "../../include/ort_math.h"


#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define ORT_FN __host__ __device__ __forceinline__
#else
#define ORT_FN static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

#define ORT_COMPACT_MAX_DEPTH 10
#define ORT_MAX_STACK 200
#define ORT_INTERNAL_FLAG 0x80000000u
#define ORT_LEAFKIDS_FLAG 0x40000000u  // internal node whose existing children are all leaves
// internal record bits 8-15: which existing (pushable) children are leaves, octant space
#define ORT_LEAFMASK_SHIFT 8
#define ORT_MAXFLOAT 3.402823466e+38f

namespace ort {

struct V3 {
    float x, y, z;
};
ORT_FN int f2i(float f) { int i; __builtin_memcpy(&i, &f, 4); return i; }
ORT_FN uint32_t f2u(float f) { uint32_t i; __builtin_memcpy(&i, &f, 4); return i; }
ORT_FN float u2f(uint32_t i) { float f; __builtin_memcpy(&f, &i, 4); return f; }
ORT_FN V3 mk(float x, float y, float z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
ORT_FN V3 add(V3 a, V3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
ORT_FN V3 sub(V3 a, V3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
ORT_FN V3 mul(V3 a, V3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
ORT_FN V3 scl(float s, V3 a) { return mk(s * a.x, s * a.y, s * a.z); }
ORT_FN float dot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
ORT_FN V3 normalize(V3 v) {
    const float s = 1.0f / sqrtf(dot(v, v));
    return mk(v.x * s, v.y * s, v.z * s);
}
ORT_FN float length(V3 v) { return sqrtf(dot(v, v)); }
ORT_FN V3 cross(V3 a, V3 b) { return mk(a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y); }
// GLSL reflect(I, N) = I - 2.0 * dot(N, I) * N
ORT_FN V3 reflect(V3 I, V3 N) {
    const float k = 2.0f * dot(N, I);
    return mk(I.x - k * N.x, I.y - k * N.y, I.z - k * N.z);
}

struct KCamera {
    V3 origin, lowerLeft, horizontal, vertical, u, v, w;
    float lensRadius;
};

struct Ray {
    V3 o, d;
};

// Device view of an uploaded scene (pointers into one context's buffers).
struct KScene {
    const float4* sph_cr;    // center.xyz, radius          (binding 0)
    const float4* sph_ma;    // float(material), albedo     (binding 1)
    const float2* sph_fr;    // fuzz, refraction index      (binding 2 .xy)
    int n_spheres;
    int n_nodes;
    // compact layout
    const uint2* node;       // internal: {childrenOffset, FLAG|childMask}; leaf: {objectsOffset, objectCount}
    const float4* leaf_sph;  // per objectIndices entry: the sphere's center.xyz, radius^2 (as float r*r)
    const int* leaf_idx;     // per entry: sphere index (= objectIndices)
    const float* planes;     // 3 x (2^depth + 1) split-plane coordinates (global copy)
    const uint4* lds_img;    // the workgroup LDS image (fast plane tables | rank LUT), built once
    int lds_img_n16;         // per scene; its size in 16-byte chunks (planes part: lds_img_p16)
    int lds_img_p16;
    const uint4* lds_rev;    // depth 9-10: the reversed-table image (fast_rev_planes), lds_rev_n16 chunks
    int lds_rev_n16;
    int depth;               // tree depth D (root = 0)
    uint32_t node_bytes;     // buffer sizes for the range-checked buffer loads (< 2^32)
    uint32_t leaf_bytes;
    const uint2* kid;        // per node: rejected-sphere skip entry (kid_table.h), or null (off)
    const uint4* nk;         // per node: {record, kid entry} interleaved (one 16-byte load), or null
    uint32_t nk_bytes;
    uint32_t tail_base;      // = n_indices: a one-sphere leaf's objectsOffset is tail_base + sphere
    // walks with Masks::kLdsScene (ort_pixel_paths on small scenes): LDS byte addresses of
    // workgroup copies of nk[] and leaf_sph[] (set inside the kernel)
    uint32_t lds_nk, lds_sph;
    // explicit (reference) layout
    const float4* nodeA;     // min.xyz, int bits of childrenOffset (binding 3)
    const float4* nodeB;     // max.xyz, int bits of objectsOffset  (binding 4)
    const int* count;        // objectCount                         (binding 5)
    const int* indices;      // objectIndices                       (binding 6)
};

struct Counters {
    unsigned long long v[6];
};

// Sign-vector -> octant traversal order, glsl:341-447, as 8 x 3-bit codes (rank r at bits 3r).
// Index = (sx+1)*9 + (sy+1)*3 + (sz+1), s in {-1,0,1}.  (0,0,0) cannot occur for a normalised
// direction; the reference leaves traversalOrder uninitialised there, we use the identity.
ORT_FN uint32_t pack_order(int a, int b, int c, int d, int e, int f, int g, int h) {
    return (uint32_t)a | ((uint32_t)b << 3) | ((uint32_t)c << 6) | ((uint32_t)d << 9) | ((uint32_t)e << 12) |
           ((uint32_t)f << 15) | ((uint32_t)g << 18) | ((uint32_t)h << 21);
}
ORT_FN uint32_t order_code(V3 d) {
    const int sx = (d.x < 0.0f) ? -1 : ((d.x > 0.0f) ? 1 : 0);
    const int sy = (d.y < 0.0f) ? -1 : ((d.y > 0.0f) ? 1 : 0);
    const int sz = (d.z < 0.0f) ? -1 : ((d.z > 0.0f) ? 1 : 0);
    const uint32_t CYAN = pack_order(0, 1, 2, 3, 4, 5, 6, 7);
    const uint32_t YELLOW = pack_order(2, 0, 3, 1, 6, 4, 7, 5);
    const uint32_t RED = pack_order(3, 1, 2, 0, 7, 5, 6, 4);
    const uint32_t DPURPLE = pack_order(1, 0, 3, 2, 5, 4, 7, 6);
    const uint32_t BLUE = pack_order(4, 5, 6, 7, 0, 1, 2, 3);
    const uint32_t PURPLE = pack_order(6, 4, 7, 5, 2, 0, 3, 1);
    const uint32_t GREEN = pack_order(7, 5, 6, 4, 3, 1, 2, 0);
    const uint32_t BLACK = pack_order(5, 4, 7, 6, 1, 0, 3, 2);
    // the if/else-if chain of glsl:352-447, in the same order
    if (sx == 1 && sy == 1 && sz == 1) return CYAN;
    if ((sx == -1 && sy == 1 && sz == 1) || (sx == -1 && sy == 1 && sz == 0) || (sx == 0 && sy == 1 && sz == 0) ||
        (sx == 0 && sy == 1 && sz == 1))
        return YELLOW;
    if ((sx == -1 && sy == -1 && sz == 1) || (sx == -1 && sy == 0 && sz == 1) || (sx == 0 && sy == 0 && sz == 1) ||
        (sx == 0 && sy == -1 && sz == 1) || (sx == -1 && sy == -1 && sz == 0) || (sx == 0 && sy == -1 && sz == 0) ||
        (sx == -1 && sy == 0 && sz == 0))
        return RED;
    if ((sx == 1 && sy == -1 && sz == 1) || (sx == 1 && sy == 0 && sz == 1) || (sx == 1 && sy == -1 && sz == 0) ||
        (sx == 1 && sy == 0 && sz == 0))
        return DPURPLE;
    if ((sx == 1 && sy == 1 && sz == -1) || (sx == 1 && sy == 0 && sz == -1) || (sx == 0 && sy == 1 && sz == -1) ||
        (sx == 1 && sy == 1 && sz == 0))
        return BLUE;
    if (sx == -1 && sy == 1 && sz == -1) return PURPLE;
    if ((sx == -1 && sy == -1 && sz == -1) || (sx == -1 && sy == 0 && sz == -1) || (sx == 0 && sy == -1 && sz == -1) ||
        (sx == 0 && sy == 0 && sz == -1))
        return GREEN;
    if (sx == 1 && sy == -1 && sz == -1) return BLACK;
    return CYAN;
}

// rayBoxIntersection (glsl:276-288) on one axis: GLSL min/max semantics, bot/top order kept.
ORT_FN void slab(float tbot, float ttop, float& tmin, float& tmax) {
    tmin = ort_minf(tbot, ttop);
    tmax = ort_maxf(tbot, ttop);
}
ORT_FN bool ray_box(const Ray& r, V3 inv, V3 bmin, V3 bmax, float& tmin, float& tmax) {
    const float bx = inv.x * (bmin.x - r.o.x), by = inv.y * (bmin.y - r.o.y), bz = inv.z * (bmin.z - r.o.z);
    const float ux = inv.x * (bmax.x - r.o.x), uy = inv.y * (bmax.y - r.o.y), uz = inv.z * (bmax.z - r.o.z);
    float x0, x1, y0, y1, z0, z1;
    slab(bx, ux, x0, x1);
    slab(by, uy, y0, y1);
    slab(bz, uz, z0, z1);
    tmin = ort_maxf(ort_maxf(x0, y0), z0);
    tmax = ort_minf(ort_minf(x1, y1), z1);
    return tmax >= tmin;
}

// Sphere_hit (glsl:224-273) returning only the accepted t; a = dot(d,d) precomputed.
// R2: sp.w already holds radius * radius (the compact layout's leaf_sph), else the radius.
template <bool R2 = false>
ORT_FN bool sphere_hit_t(const Ray& r, float a, float4 sp, float t_min, float t_max, float& t) {
    const V3 oc = mk(r.o.x - sp.x, r.o.y - sp.y, r.o.z - sp.z);
    const float half_b = dot(oc, r.d);
    const float c = dot(oc, oc) - (R2 ? sp.w : sp.w * sp.w);
    const float disc = half_b * half_b - a * c;
    if (disc > 0.0f) {
        const float sq = sqrtf(disc);
        float temp = (-half_b - sq) / a;
        if (temp < t_max && temp > t_min) { t = temp; return true; }
        temp = (-half_b + sq) / a;
        if (temp < t_max && temp > t_min) { t = temp; return true; }
    }
    return false;
}

// Frame storage for traverse_compact: device = LDS columns, host = local arrays.
struct LdsFrames {
    int* co;     // co[level * stride + lane]
    float* tm;
    int stride;
    int lane;
    ORT_FN void set(int L, int c, float t) { co[L * stride + lane] = c; tm[L * stride + lane] = t; }
    ORT_FN void setCo(int L, int c) { co[L * stride + lane] = c; }
    ORT_FN int getCo(int L) const { return co[L * stride + lane]; }
    ORT_FN float getTm(int L) const { return tm[L * stride + lane]; }
};
struct LocalFrames {
    int co[ORT_COMPACT_MAX_DEPTH + 1];
    float tm[ORT_COMPACT_MAX_DEPTH + 1];
    ORT_FN void set(int L, int c, float t) { co[L] = c; tm[L] = t; }
    ORT_FN void setCo(int L, int c) { co[L] = c; }
    ORT_FN int getCo(int L) const { return co[L]; }
    ORT_FN float getTm(int L) const { return tm[L]; }
};

// Per-level masks of remaining children (rank space), levels 0..11 in 96 bits.
struct LevelMasks {
    uint64_t lo;  // levels 0..7, one byte each
    uint32_t hi;  // levels 8..11
    ORT_FN void clear() { lo = 0; hi = 0; }
    ORT_FN void put(int L, uint32_t m) {
        if (L < 8) lo |= (uint64_t)m << (8 * L);
        else hi |= m << (8 * (L - 8));
    }
    ORT_FN int top() const {
        if (hi) return 8 + ((31 - __builtin_clz(hi)) >> 3);
        if (lo) return (63 - __builtin_clzll(lo)) >> 3;
        return -1;
    }
    // pops the lowest rank of level L; returns the rank
    ORT_FN int pop(int L) {
        if (L < 8) {
            const uint32_t m = (uint32_t)(lo >> (8 * L)) & 0xffu;
            const int r = __builtin_ctz(m);
            lo &= ~((uint64_t)1 << (8 * L + r));
            return r;
        }
        const uint32_t m = (hi >> (8 * (L - 8))) & 0xffu;
        const int r = __builtin_ctz(m);
        hi &= ~(1u << (8 * (L - 8) + r));
        return r;
    }
};

// The fast walk's split-plane tables.  Reversed layout (every kernel at depth <= 8; the
// persistent bounce kernel at depth 9-10): with T = max(256, 2^D) floats, per axis a block
// of 3T floats at float 3T a -- the layout's forward table (entry i = plane i) at its start
// and the same table reversed (entry i = plane 2^D - i) T floats further -- so that a ray
// walking an axis downwards indexes its planes upwards like every other ray (no per-ray
// stride), and every table starts at a multiple of 4T bytes: a node's near plane (index < T)
// is then a byte offset whose low bits are 4 x the index, and the pop moves it to a child's
// with one and/or (fast_step).  The forward table's last entry is the reversed one's first
// (the same plane); the last axis block ends with its reversed table (7T + 2^D + 1 floats in
// all).  Forward layout (the other kernels at depth 9-10, whose LDS holds 256 lanes'
// frames): the forward tables back to back, 2^D + 1 floats each, and a +-4 byte stride per
// axis.  The image a workgroup copies into LDS (lds_layout) is the tables, the rank LUT
// (8 x 256 bytes: in the gap after axis 0's reversed table where it fits, at depth 10) and
// then the frame columns.
ORT_FN bool fast_rev_planes(int depth) { return depth <= 8; }  // the default image's layout
ORT_FN int fast_rev_T(int depth) { return depth <= 8 ? 256 : 1 << depth; }
ORT_FN int fast_axis_floats(int depth, bool rev) { return rev ? 3 * fast_rev_T(depth) : (1 << depth) + 1; }
ORT_FN int fast_axis_floats(int depth) { return fast_axis_floats(depth, fast_rev_planes(depth)); }
ORT_FN int fast_plane_floats(int depth, bool rev) {
    return rev ? 7 * fast_rev_T(depth) + (1 << depth) + 1 : 3 * fast_axis_floats(depth, false);
}
ORT_FN int fast_plane_floats(int depth) { return fast_plane_floats(depth, fast_rev_planes(depth)); }
struct LdsLayout {
    int lut;     // byte offset of the rank LUT
    int frames;  // byte offset of the frame columns (= the image's size; a multiple of 16)
};
ORT_FN LdsLayout lds_layout(int depth, bool rev) {
    const int pb = (4 * fast_plane_floats(depth, rev) + 15) & ~15;
    const int T = fast_rev_T(depth);
    LdsLayout l;
    if (rev && 4 * (2 * T - (1 << depth) - 1) >= 2048) {  // the gap after axis 0's reversed table
        l.lut = 12 * T - 2048;
        l.frames = pb;
    } else {
        l.lut = pb;
        l.frames = pb + 2048;
    }
    return l;
}
ORT_FN void fill_fast_planes(const float* fwd, float* out, int depth, bool rev, int i0 = 0, int step = 1) {
    const int P1 = (1 << depth) + 1;
    const int S = fast_axis_floats(depth, rev);
    const int T = fast_rev_T(depth);
    const int n = fast_plane_floats(depth, rev);
    for (int o = i0; o < n; o += step) {  // gather form: one writer per entry
        const int a = o / S, r = o - a * S;
        float v = 0.0f;  // the gaps: never read as planes
        if (r < P1) v = fwd[a * P1 + r];
        else if (rev && r >= T && r - T < P1) v = fwd[a * P1 + (P1 - 1 - (r - T))];
        out[o] = v;
    }
}
ORT_FN void fill_fast_planes(const float* fwd, float* out, int depth) {
    fill_fast_planes(fwd, out, depth, fast_rev_planes(depth));
}

// Child-box entry t of octant `oct` for a node at depth `dep` with cell (cx,cy,cz):
// recomputes the reference's rayBoxIntersection for that child (tmin only + hit flag).
ORT_FN float plane_t(float inv, float p, float o) { return inv * (p - o); }

template <bool COUNT, class Frames>
ORT_FN bool traverse_compact(const KScene& S, const float* planes, const Ray& r, float t_min, float t_max,
                             int& hitEntry, float& hitT, Frames& fr, Counters& cnt) {
    const int D = S.depth;
    const int S1 = fast_axis_floats(D);  // fast_plane_floats layout: forward tables at a * S1
    const float* PX = planes;
    const float* PY = planes + S1;
    const float* PZ = planes + 2 * S1;
    const V3 inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    const float a = dot(r.d, r.d);
    {
        float t0, t1;
        const V3 bmin = mk(PX[0], PY[0], PZ[0]);
        const V3 bmax = mk(PX[1 << D], PY[1 << D], PZ[1 << D]);
        if (!ray_box(r, inv, bmin, bmax, t0, t1)) return false;
    }
    const uint32_t ocode = order_code(r.d);
    int node = 0, depth = 0;
    uint32_t cx = 0, cy = 0, cz = 0;
    float ntmin = t_min;
    const float closest0 = t_max;
    float closest = t_max;
    bool hit = false;
    LevelMasks masks;
    masks.clear();
    for (;;) {
        const uint2 rec = S.node[node];
        if (COUNT) cnt.v[0] += 1;
        if (rec.y & ORT_INTERNAL_FLAG) {
            const int co = (int)rec.x;
            const uint32_t cmask = rec.y & 0xffu;
            if (COUNT) {
                const long long rem = (long long)S.n_nodes - (long long)co;
                cnt.v[1] += (unsigned long long)(rem >= 8 ? 8 : (rem > 0 ? rem : 0));
            }
            const int s = D - depth;  // >= 1 for an internal node
            const float tx0 = plane_t(inv.x, PX[cx << s], r.o.x);
            const float tx1 = plane_t(inv.x, PX[(2 * cx + 1) << (s - 1)], r.o.x);
            const float tx2 = plane_t(inv.x, PX[(cx + 1) << s], r.o.x);
            const float ty0 = plane_t(inv.y, PY[cy << s], r.o.y);
            const float ty1 = plane_t(inv.y, PY[(2 * cy + 1) << (s - 1)], r.o.y);
            const float ty2 = plane_t(inv.y, PY[(cy + 1) << s], r.o.y);
            const float tz0 = plane_t(inv.z, PZ[cz << s], r.o.z);
            const float tz1 = plane_t(inv.z, PZ[(2 * cz + 1) << (s - 1)], r.o.z);
            const float tz2 = plane_t(inv.z, PZ[(cz + 1) << s], r.o.z);
            float xa0, xa1, xb0, xb1, ya0, ya1, yb0, yb1, za0, za1, zb0, zb1;
            slab(tx0, tx1, xa0, xa1);  // lower x half: min = mid-split plane order bot/top
            slab(tx1, tx2, xb0, xb1);
            slab(ty0, ty1, ya0, ya1);
            slab(ty1, ty2, yb0, yb1);
            slab(tz0, tz1, za0, za1);
            slab(tz1, tz2, zb0, zb1);
            uint32_t rmask = 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const int oct = (int)((ocode >> (3 * k)) & 7u);
                if ((cmask >> oct) & 1u) {
                    const bool xh = (oct >> 1) & 1, yh = oct & 1, zh = (oct >> 2) & 1;
                    const float cmin = ort_maxf(ort_maxf(xh ? xb0 : xa0, yh ? yb0 : ya0), zh ? zb0 : za0);
                    const float cmax = ort_minf(ort_minf(xh ? xb1 : xa1, yh ? yb1 : ya1), zh ? zb1 : za1);
                    const bool keep = (cmax >= cmin) && !(cmax < ntmin) && !(cmin > closest0);
                    if (keep) rmask |= 1u << k;
                }
            }
            if (rmask) {
                masks.put(depth, rmask);
                fr.set(depth, co, ntmin);
            }
        } else {
            const int off = (int)rec.x;
            const int n = (int)rec.y;
            for (int i = 0; i < n; ++i) {
                const float4 sp = S.leaf_sph[off + i];
                if (COUNT) cnt.v[2] += 1;
                float t;
                if (sphere_hit_t<true>(r, a, sp, ntmin, closest, t)) {  // leaf_sph: .w = r^2
                    hit = true;
                    closest = t;
                    hitEntry = off + i;
                    if (COUNT) cnt.v[3] += 1;
                }
            }
            if (hit) break;  // glsl:336: the walk ends after the leaf that produced a hit
        }
        const int L = masks.top();
        if (L < 0) break;
        const int rk = masks.pop(L);
        const int oct = (int)((ocode >> (3 * rk)) & 7u);
        const int sh = depth - L;  // current node is at `depth`; its ancestor at level L
        cx = ((cx >> sh) << 1) | (uint32_t)((oct >> 1) & 1);
        cy = ((cy >> sh) << 1) | (uint32_t)(oct & 1);
        cz = ((cz >> sh) << 1) | (uint32_t)((oct >> 2) & 1);
        depth = L + 1;
        node = fr.getCo(L) + oct;
        // the tmin the reference pushed: max(childTMin, parent node_tmin) (glsl:474)
        const int s = D - depth;
        float xl, xu, yl, yu, zl, zu;
        slab(plane_t(inv.x, PX[cx << s], r.o.x), plane_t(inv.x, PX[(cx + 1) << s], r.o.x), xl, xu);
        slab(plane_t(inv.y, PY[cy << s], r.o.y), plane_t(inv.y, PY[(cy + 1) << s], r.o.y), yl, yu);
        slab(plane_t(inv.z, PZ[cz << s], r.o.z), plane_t(inv.z, PZ[(cz + 1) << s], r.o.z), zl, zu);
        const float cmin = ort_maxf(ort_maxf(xl, yl), zl);
        ntmin = ort_maxf(cmin, fr.getTm(L));
    }
    hitT = closest;
    return hit;
}

// ---------------------------------------------------------------------------------------
// Fast path of traverse_compact for rays whose direction has no zero (or denormal-reciprocal)
// component, i.e. 1/d is finite on every axis.  Then no slab value can be NaN and, per
// axis, t(p) = inv*(p - o) is monotone in p, so every GLSL min/max of the reference is
// decided by the sign of d alone:
//   * the entry/exit of a child slab are its near/far planes' t (no compare needed); the
//     plane tables are read in ray order (index i -> table[g ? 2^D - i : i], g = d < 0), so
//     a node's near plane is its lower ray-order index and rank bit = "far half";
//   * the traversal order (glsl:352-447) of an all-non-zero sign vector is
//     order[r] = perm(r) ^ m, m = (d.z<0)<<2 | (d.x<0)<<1 | (d.y<0), perm = identity for
//     d.x > 0 and "swap bits 0,1" for d.x < 0 (checked for all 8 tables), so children are
//     evaluated directly in traversal-rank space with static role axes
//     A = rank bit 1 (x, or y when swapped), B = rank bit 0, C = rank bit 2 (z);
//   * IEEE max3/min3 equal the GLSL chains (no NaN); a +0/-0 tie can pick the other zero,
//     which is harmless because every tmin is only ever compared (never divided by).
// The reference pushes max(childTMin, node_tmin).  A child box lies inside its parent's
// (midpoint splits; checked at upload, layout.cpp), so its entry t on every axis is >= the
// parent's (fl is monotone), hence by induction node_tmin = max(max3(entries), t_min) for
// every node below the root: no per-level tmin has to be kept, and the push test
// (tmax >= tmin && !(tmax < node_tmin) && !(tmin > closest)) becomes
// min(tmax, t_max) >= max(tmin, t_min).  Results are bit-identical to the exact walk
// (tests/test_emulation.py forces both on the same rays).
//
// Stack: the reference stack holds exactly the unvisited surviving siblings of every
// ancestor in traversal order, i.e. per tree level a set of ranks plus the level's children
// offset.  Ranks are kept as "rank-reversed" bytes (rank r of level L = bit 8L + 7 - r) so the
// next node -- lowest rank of the deepest non-empty level -- is the highest set bit, and a
// descent is the same pop as a backtrack: every visited internal node pushes all its
// surviving children, then one uniform pop picks the next node.
//
// rank_lut[m*256 + childMask] maps the node's octant-space child mask to reversed rank space.
ORT_FN uint32_t rank_perm(uint32_t r, uint32_t m) {
    const uint32_t swap = (m >> 1) & 1u;  // perm = swap bits 0,1 when d.x < 0
    const uint32_t p = swap ? ((r & 4u) | ((r & 1u) << 1) | ((r >> 1) & 1u)) : r;
    return p ^ m;
}
ORT_FN uint8_t rank_lut_entry(uint32_t m, uint32_t cmask) {
    uint32_t out = 0;
    for (uint32_t r = 0; r < 8; ++r)
        if ((cmask >> rank_perm(r, m)) & 1u) out |= 0x80u >> r;
    return (uint8_t)out;
}

ORT_FN bool a_in_qdiv_range(float a) { return a >= 0.125f && a <= 8.0f; }
// The fast walk's t_min (the shader's only one, glsl:hit(r, 0.001, ...)) is a literal in the
// instruction stream rather than a per-ray register.
constexpr float kFastTMin = 0.001f;
// The fast walk's preconditions: finite 1/d and origin (no slab value can be NaN), a
// positive t_min and finite t_max (the push test below relies on both), dot(d,d) in
// qdiv's range.
ORT_FN bool fast_path_ok(const Ray& r, V3 inv, float t_min, float t_max) {
    return fabsf(inv.x) <= ORT_MAXFLOAT && fabsf(inv.y) <= ORT_MAXFLOAT && fabsf(inv.z) <= ORT_MAXFLOAT &&
           fabsf(r.o.x) <= ORT_MAXFLOAT && fabsf(r.o.y) <= ORT_MAXFLOAT && fabsf(r.o.z) <= ORT_MAXFLOAT &&
           t_min == kFastTMin && t_max <= ORT_MAXFLOAT && a_in_qdiv_range(dot(r.d, r.d));
}

// Rays with a zero (or tiny denormal) direction component have an infinite 1/d there.  Their
// slab values on that axis are +-inf (never NaN unless the origin lies exactly on one of the
// axis's split planes), and a box's [min, max] interval on it is (-inf, +inf) or empty
// whichever sign the infinity has -- so the box tests do not depend on that sign.  What does
// depend on it is the traversal order: the shader picks it from the sign vector with zeros
// (glsl:342-447), and each of those 26 vectors' table equals perm(r) ^ m' for one full sign
// mask m' whose non-zero components agree with the ray's (checked against the shader's tables,
// tests/test_math.py).  So such a ray walks the fast path with inv = +-inf on its zero axes,
// signed by m'.  kGlslOrderM: m' by (sx+1)*9 + (sy+1)*3 + (sz+1), 3 bits each, 9 per word.
constexpr uint32_t kGlslOrderM[3] = {0x259bedfu, 0x2518edfu, 0x90984du};
ORT_FN uint32_t glsl_order_m(float dx, float dy, float dz) {
    const int sx = dx < 0.0f ? 0 : (dx > 0.0f ? 2 : 1), sy = dy < 0.0f ? 0 : (dy > 0.0f ? 2 : 1),
              sz = dz < 0.0f ? 0 : (dz > 0.0f ? 2 : 1);
    const int idx = sx * 9 + sy * 3 + sz;
    return (kGlslOrderM[idx / 9] >> (3 * (idx % 9))) & 7u;
}
// Is v exactly one of the split planes of one axis (2^D + 1 entries)?  The table holds NaN
// where no node uses a plane (layout.cpp), so search it like the tree splits it: the planes
// inside (lo, hi) can be used only if the interval's mid plane is (a node with a boundary
// inside has an ancestor spanning (lo, hi) that was split there), and the used planes are
// ascending.  D steps; run only for the rare rays with a zero direction component.
ORT_FN bool on_split_plane(const float* P, int D, float v) {
    int lo = 0, hi = 1 << D;
    if (P[lo] == v || P[hi] == v) return true;
    if (!(v > P[lo] && v < P[hi])) return false;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        const float pm = P[mid];
        if (!(pm == pm)) return false;
        if (pm == v) return true;
        if (v < pm) hi = mid;
        else lo = mid;
    }
    return false;
}
// The fast walk for a ray fast_path_ok refused only because some 1/d component is infinite:
// returns whether it may take the fast walk, with those components of inv signed by the
// shader's order (see above).  Refused: a zero direction vector (the shader leaves its order
// undefined), an origin on a split plane of a zero axis (NaN slabs), the other fast_path_ok
// conditions.
ORT_FN bool fast_zero_axes(const KScene& S, const Ray& r, V3& inv, float t_min, float t_max) {
    if (!(fabsf(r.o.x) <= ORT_MAXFLOAT && fabsf(r.o.y) <= ORT_MAXFLOAT && fabsf(r.o.z) <= ORT_MAXFLOAT) ||
        t_min != kFastTMin || !(t_max <= ORT_MAXFLOAT) || !a_in_qdiv_range(dot(r.d, r.d)))
        return false;
    if (r.d.x == 0.0f && r.d.y == 0.0f && r.d.z == 0.0f) return false;
    if (!(inv.x == inv.x) || !(inv.y == inv.y) || !(inv.z == inv.z)) return false;
    const uint32_t m = glsl_order_m(r.d.x, r.d.y, r.d.z);
    const int P1 = (1 << S.depth) + 1;
    float inf;
    const uint32_t inf_bits = 0x7f800000u;
    __builtin_memcpy(&inf, &inf_bits, 4);
    float* c[3] = {&inv.x, &inv.y, &inv.z};
    const float o[3] = {r.o.x, r.o.y, r.o.z};
    const uint32_t neg[3] = {(m >> 1) & 1u, m & 1u, (m >> 2) & 1u};
    for (int a = 0; a < 3; ++a) {
        if (fabsf(*c[a]) <= ORT_MAXFLOAT) continue;
        if (on_split_plane(S.planes + a * P1, S.depth, o[a])) return false;
        *c[a] = neg[a] ? -inf : inf;
    }
    return true;
}

// fast_path_ok, or else fast_zero_axes (rare: a zero direction component): inv may be re-signed.
ORT_FN bool fast_prepare(const KScene& S, const Ray& r, V3& inv) {
    if (fast_path_ok(r, inv, kFastTMin, ORT_MAXFLOAT)) return true;
    return fast_zero_axes(S, r, inv, kFastTMin, ORT_MAXFLOAT);
}

// 24-bit signed multiply (plane indices are < 2^11): one full-rate VALU op on the device.
ORT_FN int imul24(int a, int b) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __mul24(a, b);
#else
    return a * b;
#endif
}

// min/max for NaN-free operands.  On the device these are the raw VALU instructions: the
// libm-style fmaxf would first canonicalise every operand the compiler cannot prove
// canonical (one v_max x,x each), which the fast walk never needs.
#if defined(__HIP_DEVICE_COMPILE__)
ORT_FN float fmax2(float a, float b) { float r; asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
ORT_FN float fmin2(float a, float b) { float r; asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b)); return r; }
ORT_FN float fmax3(float a, float b, float c) {
    float r;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
ORT_FN float fmin3(float a, float b, float c) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
}
// max(x, kFastTMin) with the constant as an instruction literal (0x3a83126f = 0.001f)
ORT_FN float fmax_tmin(float x) { float r; asm("v_max_f32 %0, 0x3a83126f, %1" : "=v"(r) : "v"(x)); return r; }
#else
ORT_FN float fmax_tmin(float x) { return fmaxf(x, kFastTMin); }
ORT_FN float fmax2(float a, float b) { return fmaxf(a, b); }
ORT_FN float fmin2(float a, float b) { return fminf(a, b); }
ORT_FN float fmax3(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
ORT_FN float fmin3(float a, float b, float c) { return fminf(fminf(a, b), c); }
#endif

// Correctly rounded n / a given y = RN(1/a): q0 = n*y is faithful, r = n - a*q0 is exact
// (fma), and RN(q0 + r*y) = RN(n/a) (Markstein's theorem; no division is ever exactly a
// midpoint).  Valid without underflow/overflow in r and q: |n| in [2^-60, 2^100] and
// a in [2^-3, 2^3] (checked per ray by fast_path_ok); otherwise the IEEE division.
// 2.56e9 random (n, a) pairs in those ranges were checked bitwise against n / a on the host.
// any_lane(p): p on any active lane of the wave (a wave-uniform branch: no exec-mask juggling
// around a path that is almost never taken); p itself on the host.
ORT_FN bool any_lane(bool p) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_ballot_w64(p) != 0;
#else
    return p;
#endif
}
// n / a for the fast walk's sphere roots (callers: t_min >= kFastTMin).  Below |n| = 2^-60 the
// Markstein step may miss the correct rounding, but then |n / a| < 2^-57 (a >= 1/8) is far
// below t_min and the root is rejected whatever its last bit, so only |n| > 2^100 (and NaN)
// takes the IEEE division.
ORT_FN float qdiv(float n, float a, float y) {
    const float q0 = n * y;
    float q = fmaf(fmaf(-q0, a, n), y, q0);
    const float an = fabsf(n);
    const bool slow = !(an <= 0x1p100f);
    if (any_lane(slow)) q = slow ? n / a : q;
    return q;
}
// Correctly rounded sqrt for x in [2^-96, 2^100]: the hardware estimate corrected by the
// two residual tests of the compiler's own IEEE expansion, minus its denormal scaling and
// special-value handling (not needed in that range); otherwise sqrtf.
ORT_FN float qsqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u);
    const float sp = __uint_as_float(__float_as_uint(s) + 1u);
    float r = (fmaf(-sm, s, x) <= 0.0f) ? sm : s;
    r = (fmaf(-sp, s, x) > 0.0f) ? sp : r;
    // x in [2^-96, 2^100] as one unsigned compare of the bits (x > 0 here: disc > 0)
    const bool slow = f2u(x) - f2u(0x1p-96f) > f2u(0x1p100f) - f2u(0x1p-96f);
    if (any_lane(slow)) {
        // the volatile asm keeps this a real (wave-uniform) branch: left alone, the compiler
        // if-converts it and evaluates sqrtf's IEEE expansion on every call
        asm volatile("" ::: "memory");
        r = slow ? sqrtf(x) : r;
    }
    return r;
#else
    return sqrtf(x);
#endif
}

// Sphere_hit_t with the fast division/sqrt (ya = RN(1 / a)); same results.
ORT_FN bool sphere_hit_fast(const Ray& r, float a, float ya, float4 sp, float t_min, float t_max, float& t) {
    const V3 oc = mk(r.o.x - sp.x, r.o.y - sp.y, r.o.z - sp.z);
    const float half_b = dot(oc, r.d);
    const float c = dot(oc, oc) - sp.w;  // leaf_sph: .w = radius * radius
    const float disc = half_b * half_b - a * c;
    if (disc > 0.0f) {
        // both roots, no branch between them: the near one if in range, else the far one
        const float sq = qsqrt(disc);
        const float t1 = qdiv(-half_b - sq, a, ya);
        const float t2 = qdiv(-half_b + sq, a, ya);
        const bool ok1 = t1 < t_max && t1 > t_min;
        const bool ok2 = t2 < t_max && t2 > t_min;
        t = ok1 ? t1 : t2;
        return ok1 || ok2;
    }
    return false;
}

// Node record / leaf sphere loads of the fast walk.  On the device: buffer loads with a
// 32-bit byte offset (descriptor from the kernel arguments, so it stays in SGPRs) instead of
// 64-bit flat addresses -- fewer VALU ops and VGPRs per fetch (cdna_hip_programming.md T8).
ORT_FN uint2 fetch_node(const KScene& S, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.node, 0, (int)S.node_bytes, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (uint32_t)i * 8u, 0, 0);
    return make_uint2(v[0], v[1]);
#else
    return S.node[i];
#endif
}
ORT_FN uint2 fetch_kid(const KScene& S, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.kid, 0, (int)S.node_bytes, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(rs, (uint32_t)i * 8u, 0, 0);
    return make_uint2(v[0], v[1]);
#else
    return S.kid[i];
#endif
}
ORT_FN uint4 fetch_nk(const KScene& S, int i) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.nk, 0, (int)S.nk_bytes, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)i * 16u, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
#else
    return S.nk[i];
#endif
}
ORT_FN float4 fetch_sphere(const KScene& S, int e) {
#if defined(__HIP_DEVICE_COMPILE__)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)S.leaf_sph, 0, (int)S.leaf_bytes, 0x00020000);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (uint32_t)e * 16u, 0, 0);
    return make_float4(__uint_as_float(v[0]), __uint_as_float(v[1]), __uint_as_float(v[2]), __uint_as_float(v[3]));
#else
    return S.leaf_sph[e];
#endif
}

// The rejected-sphere skip's kid entry of a popped node loaded in the pop beside its record
// (its latency hidden behind the pop's plane reads) instead of in the node's step.
#ifndef ORT_KID_PREFETCH
#define ORT_KID_PREFETCH 1
#endif
constexpr bool kKidPrefetch = ORT_KID_PREFETCH;
// The skip folded into the child mask before the node's rank-LUT read (fast_step).
#ifndef ORT_KID_SKIP_FOLD
#define ORT_KID_SKIP_FOLD 1
#endif

// Plane idx of a ray-order table (base[idx]; see fast_begin for the reversed copies).
ORT_FN float plane_at(const float* base, int idx) { return base[idx]; }

// Rank-reversed level masks (see above).  pop() returns hb = 8L + 7 - rank.
struct Masks64 {  // levels 0..7: trees of depth <= 8
    static constexpr bool kLdsScene = false;  // records / leaf spheres from global memory
    // test the leaf children of a LEAFKIDS node inline (fast_step); pays for its registers on
    // depth <= 8 trees (all leaves at the bottom level with maxSpheresPerNode 0), not deeper
    static constexpr bool kInlineLeaves = true;
    // test a node's LEADING leaf children inline (see fast_step): deep trees
    static constexpr bool kLeadLeaves = false;
    static constexpr bool kRevPlanes = true;  // depth <= 8: reversed plane tables (fast_rev_planes)
    static constexpr bool kKeepNear = true;   // keep the node's near-plane pointers (FastStateT::nA..)
    // the pop also reads the popped node's mid planes (FastStateT::tMA..), so their LDS reads
    // overlap the record load instead of following it (most pops here are internal nodes: the
    // leaves are tested inline)
#ifndef ORT_PRE_MID
#define ORT_PRE_MID 1
#endif
    static constexpr bool kPreMid = ORT_PRE_MID;
    static_assert(!kPreMid || kInlineLeaves, "the pop's mid-plane reads rely on never popping a level-D leaf");
    // rejected-sphere skip (kid_table.h): off in the depth <= 8 camera-ray walk, whose inline
    // leaf children already avoid most leaf pops (C3 5 % slower with it); on in the bounce
    // walks and the deep camera walk (Masks96)
#ifndef ORT_KID_SKIP_CAMERA8
#define ORT_KID_SKIP_CAMERA8 0
#endif
    static constexpr bool kKidSkip = ORT_KID_SKIP_CAMERA8;
    uint64_t m;
    ORT_FN void clear() { m = 0; }
    ORT_FN bool empty() const { return m == 0; }
    ORT_FN void put(int L, uint32_t rev) { m |= (uint64_t)rev << (8 * L); }
    ORT_FN int pop() {
        const int hb = 63 - __builtin_clzll(m);
        m ^= (uint64_t)1 << hb;
        return hb;
    }
    // clears bit hb (= 8L + 7 - rank) and returns whether it was set
    ORT_FN bool take(int hb) {
        const uint64_t b = (uint64_t)1 << hb;
        const bool t = (m & b) != 0;
        m &= ~b;
        return t;
    }    // device: re-assert wave-uniformity (the value is uniform; this only helps the compiler)
    ORT_FN void uniform() {
#if defined(__HIP_DEVICE_COMPILE__)
        m = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(m >> 32)) << 32) |
            (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)m);
#endif
    }
};
struct Masks96 {  // levels 0..9 (ORT_COMPACT_MAX_DEPTH 10)
    static constexpr bool kLdsScene = false;
    // a leaf-children node's leaves tested inline (as in the depth <= 8 walk): C5 camera rays
    // 14.11 -> 14.86 ms (the rejected-sphere skip already drops most of them): off
#ifndef ORT_INLINE_LEAVES_DEEP
#define ORT_INLINE_LEAVES_DEEP 0
#endif
    static constexpr bool kInlineLeaves = ORT_INLINE_LEAVES_DEEP;
#ifndef ORT_PRE_MID_DEEP
#define ORT_PRE_MID_DEEP 0
#endif
    static constexpr bool kPreMid = ORT_PRE_MID_DEEP;
    // leading leaf children tested inline: C5 camera walk 19.45 -> 17.62 ms when added, but
    // with the rejected-sphere skip on (which drops most of those leaves before they are
    // pushed) 16.60 -> 15.37 ms without them (tools/ab_stream.py): off
#ifndef ORT_LEAD_LEAVES_DEEP
#define ORT_LEAD_LEAVES_DEEP 0
#endif
    static constexpr bool kLeadLeaves = ORT_LEAD_LEAVES_DEEP;
    static constexpr bool kRevPlanes = false;
    static constexpr bool kKeepNear = true;
    // the rejected-sphere skip here too: with the kid entry loaded in the pop, C5's camera
    // walk 17.52 -> 16.41 ms in A/B (no gain while the entry was loaded in the node's step)
#ifndef ORT_KID_SKIP_DEEP_CAMERA
#define ORT_KID_SKIP_DEEP_CAMERA 1
#endif
    static constexpr bool kKidSkip = ORT_KID_SKIP_DEEP_CAMERA;
    // levels 2..9 in lo (bits 8(L-2)..), levels 0..1 in hi: the deep levels a walk spends
    // nearly all its steps at share one word, so the put/pop branches below are taken alike
    // by almost every lane of a wave (with levels 8.. in hi, lanes split over them often)
#ifndef ORT_MASKS_SPLIT_AT
#define ORT_MASKS_SPLIT_AT 2
#endif
    static constexpr int kSplit = ORT_MASKS_SPLIT_AT;  // first level held in lo
    uint64_t lo;
    uint32_t hi;
    ORT_FN void clear() { lo = 0; hi = 0; }
    ORT_FN bool empty() const { return (lo | hi) == 0; }
    ORT_FN void put(int L, uint32_t rev) {
        if (L >= kSplit) lo |= (uint64_t)rev << (8 * (L - kSplit));
        else hi |= rev << (8 * L);
    }
    ORT_FN int pop() {
        if (lo) {
            const int hb = 63 - __builtin_clzll(lo);
            lo ^= (uint64_t)1 << hb;
            return 8 * kSplit + hb;
        }
        const int hb = 31 - __builtin_clz(hi);
        hi ^= 1u << hb;
        return hb;
    }
    ORT_FN bool take(int hb) {
        if (hb >= 8 * kSplit) {
            const uint64_t b = (uint64_t)1 << (hb - 8 * kSplit);
            const bool t = (lo & b) != 0;
            lo &= ~b;
            return t;
        }
        const uint32_t b = 1u << hb;
        const bool t = (hi & b) != 0;
        hi &= ~b;
        return t;
    }    ORT_FN void uniform() {
#if defined(__HIP_DEVICE_COMPILE__)
        lo = ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(lo >> 32)) << 32) |
             (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)lo);
        hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)hi);
#endif
    }
};

// Resumable per-lane state of the fast walk (so a persistent kernel can interleave rays).
// Registers are what limits the walk (7 waves/SIMD at 72 VGPRs), so nothing derivable is
// kept: the world-axis origin comes back from the role-axis one (swap = bit 1 of otab's
// nibble 0, which is m), dot(d, d) is recomputed per leaf, the half width from depth, the
// LUT row from m, and "hit" is hitEntry >= 0.
template <class Masks>
struct FastStateT {
    V3 d;            // original-axis direction (Sphere_hit)
    float ya;        // RN(1 / dot(d, d))
    float oA, oB, oC, iA, iB, iC;  // role-axis origin / 1/d
    // kRevPlanes: byte offsets from pl0 of the current node's near plane per role axis (table
    // start, a multiple of 4T bytes, + 4 * index; see fast_rev_planes)
    const float* pl0;
    uint32_t aA, aB, aC;
    uint32_t h4;      // half the current node's width, in bytes of plane table (4 * 2^(D-1-depth))
#if defined(__HIP_DEVICE_COMPILE__)
    // device: the offsets are absolute LDS byte addresses (the table image sits in LDS, at a
    // 1 KiB-aligned start), so a read is one ds_read with no base add -- the dynamic LDS
    // symbol's address is a link-time constant the compiler would otherwise add every time
    ORT_FN float plane(uint32_t a) const { return *(const __attribute__((address_space(3))) float*)(size_t)a; }
    static ORT_FN uint32_t table_base(const float* planes) {
        return (uint32_t)(size_t)(const __attribute__((address_space(3))) float*)planes;
    }
#else
    ORT_FN float plane(uint32_t off) const { return *(const float*)((const char*)pl0 + off); }
    static ORT_FN uint32_t table_base(const float*) { return 0u; }
#endif
    // otherwise: the ray-order plane table of each role axis, plane(i) = *(pA + sA * i bytes)
    const float* pA;
    const float* pB;
    const float* pC;
    int sA, sB, sC;   // +-4
    float tNA, tFA, tNB, tFB, tNC, tFC;  // near/far plane t of the current node's box
    float tMA, tMB, tMC;                 // (kPreMid) its mid planes' t
    uint32_t cP;     // (not kRevPlanes) ray-order index of the current node's near plane, 10 bits per axis
    uint32_t otab;   // nibble r = octant of rank r; nibble 0 = m
    int node, depth;
    uint2 kd;        // (kKidSkip, ORT_KID_PREFETCH) kid entry of `node`, loaded with rec
    uint2 rec;       // node record of `node`, loaded as soon as the pop knows it (its latency
                     // overlaps the pop's plane reads instead of opening the next step)
    float closest;   // (t_min is kFastTMin)
    int hitEntry;    // -1: no hit yet
    // the last rejected one-sphere leaf: its sphere and tmin (kid_table.h; ~0u = none)
    uint32_t kc_id;
    float kc_e;
    Masks masks;
    ORT_FN bool hit() const { return hitEntry >= 0; }
    ORT_FN float pl(const float* p, int s, int idx) const {
        return Masks::kRevPlanes ? p[idx] : *(const float*)((const char*)p + imul24(s, idx));
    }
    // near planes of the current node (set by the pop): its mid plane is h steps further
    const float* nA;
    const float* nB;
    const float* nC;
    ORT_FN const float* at(const float* p, int s, int idx) const {
        return Masks::kRevPlanes ? p + idx : (const float*)((const char*)p + imul24(s, idx));
    }
    ORT_FN float plA(int idx) const { return pl(pA, sA, idx); }
    ORT_FN float plB(int idx) const { return pl(pB, sB, idx); }
    ORT_FN float plC(int idx) const { return pl(pC, sC, idx); }
    ORT_FN int cA() const { return (int)(cP & 1023u); }
    ORT_FN int cB() const { return (int)((cP >> 10) & 1023u); }
    ORT_FN int cC() const { return (int)(cP >> 20); }
    ORT_FN Ray ray() const {
        const bool swap = (otab >> 1) & 1u;
        Ray r;
        r.o = mk(swap ? oB : oA, swap ? oA : oB, oC);
        r.d = d;
        return r;
    }
};
using FastState = FastStateT<Masks96>;
// The persistent kernel keeps a lane's state across refills; there three more registers for
// the near-plane pointers cost occupancy, so it re-derives them from cP.
struct Masks96Lean : Masks96 {
    static constexpr bool kInlineLeaves = false;
    static constexpr bool kKeepNear = false;
#ifndef ORT_PRE_MID_BOUNCE
#define ORT_PRE_MID_BOUNCE 0
#endif
    static constexpr bool kPreMid = ORT_PRE_MID_BOUNCE;
    // leading leaf children inline: C5 camera rays (deep kernel) 19.45 -> 17.62 ms, but the
    // persistent bounce kernel 4.8 ms slower per frame (tools/ab_stream.py): off there
#ifndef ORT_LEAD_LEAVES_PERSISTENT
#define ORT_LEAD_LEAVES_PERSISTENT 0
#endif
    static constexpr bool kLeadLeaves = ORT_LEAD_LEAVES_PERSISTENT;
    static constexpr bool kKidSkip = true;
    // the reversed plane tables (fast_rev_planes) at depth 9-10 too: the persistent kernel
    // runs 512-thread workgroups, whose LDS holds them at 6 waves/SIMD
#ifndef ORT_REV_BOUNCE
#define ORT_REV_BOUNCE 1
#endif
    static constexpr bool kRevPlanes = ORT_REV_BOUNCE;
};
// Depth <= 8 walk without the inline leaf children: the persistent bounce kernel's walk
// (inline leaves pay off on coherent camera rays, not on scattered bounce rays).
struct Masks64Plain : Masks64 {
    static constexpr bool kInlineLeaves = false;
    static constexpr bool kPreMid = false;
    static constexpr bool kKidSkip = true;
};
// ... reading node records and leaf spheres from the workgroup's LDS copies of nk[] / leaf_sph[]
// (KScene::lds_nk / lds_sph): whole-pixel paths on scenes that fit (ort_pixel_paths)
struct Masks64PlainLds : Masks64Plain {
    static constexpr bool kLdsScene = true;
};

// The split walk's level masks (traverse_split): no leaf children tested inline (the lanes
// must pop every level-`level` node themselves, to count it) and no rejected-sphere skip (each
// lane's skip state depends on the subtrees it walked, and a skipped level-`level` leaf would
// shift that lane's subtree count against the others').
struct Masks64Split : Masks64Plain {
    static constexpr bool kKidSkip = false;
};
struct Masks96Split : Masks96 {
    static constexpr bool kInlineLeaves = false;
    static constexpr bool kLeadLeaves = false;
    static constexpr bool kKidSkip = false;
};

// Node i's record into st.rec and, with kid (the rejected-sphere skip), its kid entry into
// st.kd: both from the interleaved copy S.nk in one 16-byte load when the context built it
// (ORT_NODE_KID), else from the two arrays.
#ifndef ORT_NODE_KID
#define ORT_NODE_KID 1
#endif
#if defined(__HIP_DEVICE_COMPILE__)
ORT_FN uint4 lds_u4(uint32_t a) { return *(const __attribute__((address_space(3))) uint4*)(size_t)a; }
#endif
template <class Masks>
ORT_FN void fetch_rec(const KScene& S, int i, bool kid, FastStateT<Masks>& st) {
#if defined(__HIP_DEVICE_COMPILE__)
    if constexpr (Masks::kLdsScene) {  // the workgroup's copy of nk[] (ort_pixel_paths)
        const uint4 v = lds_u4(S.lds_nk + 16u * (uint32_t)i);
        st.rec = make_uint2(v.x, v.y);
        st.kd = make_uint2(v.z, v.w);
        return;
    }
#endif
    if (ORT_NODE_KID && Masks::kKidSkip && kid && S.nk) {
        const uint4 v = fetch_nk(S, i);
        st.rec = make_uint2(v.x, v.y);
        st.kd = make_uint2(v.z, v.w);
        return;
    }
    st.rec = fetch_node(S, i);
    if (kid) st.kd = fetch_kid(S, i);
}

// Root test and state setup (glsl:296-311).  Returns false when the root box is missed.
template <class Masks>
ORT_FN bool fast_begin(const KScene& S, const float* planes, const uint8_t* rank_lut, const Ray& r, V3 inv, float t_min,
                       float t_max, FastStateT<Masks>& st) {
    const int D = S.depth;
    const int top = 1 << D;
    // the signs of 1/d (= of d, except on zero axes, where fast_zero_axes chose them)
    const uint32_t nx = f2u(inv.x) >> 31, ny = f2u(inv.y) >> 31, nz = f2u(inv.z) >> 31;
    const uint32_t m = (nz << 2) | (nx << 1) | ny;
    const bool swap = nx != 0;
    const uint32_t gA = swap ? ny : nx, gB = swap ? nx : ny, gC = nz;
    st.d = r.d;
    st.ya = 1.0f / dot(r.d, r.d);
    st.oA = swap ? r.o.y : r.o.x;
    st.oB = swap ? r.o.x : r.o.y;
    st.oC = r.o.z;
    st.iA = swap ? inv.y : inv.x;
    st.iB = swap ? inv.x : inv.y;
    st.iC = inv.z;
    // nibble k = rank_perm(k, m): the identity (or, swap, bits 0/1 exchanged) XOR m per nibble
    st.otab = (swap ? 0x75643120u : 0x76543210u) ^ (m * 0x11111111u);
    // planes: fast_plane_floats(D) floats (fill_fast_planes)
    if (Masks::kRevPlanes) {  // per axis: forward table, reversed one T floats further
        st.pl0 = planes;
        const uint32_t b0 = FastStateT<Masks>::table_base(planes);  // 4T-byte-aligned (ort_kernel.hip)
        const uint32_t T = (uint32_t)fast_rev_T(D), S3 = 3u * T;
        st.aA = b0 + 4u * ((swap ? S3 : 0u) + (gA ? T : 0u));
        st.aB = b0 + 4u * ((swap ? 0u : S3) + (gB ? T : 0u));
        st.aC = b0 + 4u * (2u * S3 + (gC ? T : 0u));
        st.h4 = 2u * (uint32_t)top;
        const uint32_t t4 = 4u * (uint32_t)top;
        st.tNA = st.iA * (st.plane(st.aA) - st.oA);
        st.tFA = st.iA * (st.plane(st.aA + t4) - st.oA);
        st.tNB = st.iB * (st.plane(st.aB) - st.oB);
        st.tFB = st.iB * (st.plane(st.aB + t4) - st.oB);
        st.tNC = st.iC * (st.plane(st.aC) - st.oC);
        st.tFC = st.iC * (st.plane(st.aC + t4) - st.oC);
        if (Masks::kPreMid) {
            const uint32_t hm = st.h4 & ~3u;  // (a depth-0 root is a leaf: 2 bytes, unused)
            st.tMA = st.iA * (st.plane(st.aA + hm) - st.oA);
            st.tMB = st.iB * (st.plane(st.aB + hm) - st.oB);
            st.tMC = st.iC * (st.plane(st.aC + hm) - st.oC);
        }
    } else {
        const int S1 = fast_axis_floats(D);
        st.pA = planes + (swap ? S1 : 0) + (gA ? top : 0);
        st.pB = planes + (swap ? 0 : S1) + (gB ? top : 0);
        st.pC = planes + 2 * S1 + (gC ? top : 0);
        st.sA = gA ? -4 : 4;
        st.sB = gB ? -4 : 4;
        st.sC = gC ? -4 : 4;
        st.tNA = st.iA * (st.plA(0) - st.oA);
        st.tFA = st.iA * (st.plA(top) - st.oA);
        st.tNB = st.iB * (st.plB(0) - st.oB);
        st.tFB = st.iB * (st.plB(top) - st.oB);
        st.tNC = st.iC * (st.plC(0) - st.oC);
        st.tFC = st.iC * (st.plC(top) - st.oC);
        if (Masks::kPreMid) {
            st.tMA = st.iA * (st.plA(top >> 1) - st.oA);
            st.tMB = st.iB * (st.plB(top >> 1) - st.oB);
            st.tMC = st.iC * (st.plC(top >> 1) - st.oC);
        }
        st.cP = 0;
        if (Masks::kKeepNear) {
            st.nA = st.pA;
            st.nB = st.pB;
            st.nC = st.pC;
        }
    }
    st.node = 0;
    fetch_rec(S, 0, kKidPrefetch && Masks::kKidSkip && S.kid, st);
    st.depth = 0;
    st.closest = t_max;
    st.hitEntry = -1;
    st.kc_id = ~0u;
    st.kc_e = 0.0f;
    st.masks.clear();
    return fmin3(st.tFA, st.tFB, st.tFC) >= fmax3(st.tNA, st.tNB, st.tNC);
}

// Sphere_hit over one leaf's objects (glsl:327-338) in the range (ntmin, closest); returns
// true if one was accepted (the walk then ends after this leaf).
template <bool COUNT, class Masks>
ORT_FN bool leaf_tests(const KScene& S, FastStateT<Masks>& st, int off, int n, float ntmin, Counters& cnt) {
    const Ray r = st.ray();
    const float a = dot(r.d, r.d);  // as fast_begin computed it
    for (int i = 0; i < n; ++i) {
#if defined(__HIP_DEVICE_COMPILE__)
        float4 sp;
        if constexpr (Masks::kLdsScene) {
            const uint4 v = lds_u4(S.lds_sph + 16u * (uint32_t)(off + i));
            sp = make_float4(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z), __uint_as_float(v.w));
        } else {
            sp = fetch_sphere(S, off + i);
        }
#else
        const float4 sp = fetch_sphere(S, off + i);
#endif
        if (COUNT) cnt.v[2] += 1;
        float t;
        if (sphere_hit_fast(r, a, st.ya, sp, ntmin, st.closest, t)) {
            st.closest = t;
            st.hitEntry = off + i;
            if (COUNT) cnt.v[3] += 1;
        }
    }
    if (!COUNT && Masks::kKidSkip) {  // a rejected one-sphere leaf: remember its sphere (kid_table.h)
        const bool rej = n == 1 && !st.hit();
        st.kc_id = rej ? (uint32_t)off - S.tail_base : st.kc_id;
        st.kc_e = rej ? ntmin : st.kc_e;
    }
    return st.hit();
}

// Drop bits of a node's eight children, rank order (rank 0 ends at bit 7: the reversed
// layout), from its per-axis slab values N (near), M (mid), F (far); t_min is folded into the
// C entries (nN, nF) and t_max into the C exits (cN, cF).  Keep child R <=> exit >= entry, with
// entry >= t_min > 0 and exit <= t_max finite, so exit - entry is never NaN and is +0 when
// equal: its sign bit is "drop" -- one v_max3 + v_min3 + v_sub + v_alignbit per child.
ORT_FN uint32_t child_drops(float tNA, float tNB, float tMA, float tMB, float tFA, float tFB, float nN, float nF,
                            float cN, float cF) {
    uint32_t drop = 0;
#if defined(__HIP_DEVICE_COMPILE__)
    // the eight tests as ONE asm block: separate min3/max3 asm statements each made the
    // compiler's hazard recognizer put an s_nop before their consumer
    float e, x;
#define ORT_C(EA, EB, EC, XA, XB, XC)                                                         \
    "v_max3_f32 %[e], " EA ", " EB ", " EC "\n\tv_min3_f32 %[x], " XA ", " XB ", " XC "\n\t" \
    "v_sub_f32 %[x], %[x], %[e]\n\tv_alignbit_b32 %[d], %[d], %[x], 31\n\t"
    asm("v_mov_b32 %[d], 0\n\t"
        ORT_C("%[NA]", "%[NB]", "%[nN]", "%[MA]", "%[MB]", "%[cN]")  // rank 0: A near, B near, C near
        ORT_C("%[NA]", "%[MB]", "%[nN]", "%[MA]", "%[FB]", "%[cN]")  // rank 1: B far
        ORT_C("%[MA]", "%[NB]", "%[nN]", "%[FA]", "%[MB]", "%[cN]")  // rank 2: A far
        ORT_C("%[MA]", "%[MB]", "%[nN]", "%[FA]", "%[FB]", "%[cN]")  // rank 3
        ORT_C("%[NA]", "%[NB]", "%[nF]", "%[MA]", "%[MB]", "%[cF]")  // ranks 4-7: C far
        ORT_C("%[NA]", "%[MB]", "%[nF]", "%[MA]", "%[FB]", "%[cF]")
        ORT_C("%[MA]", "%[NB]", "%[nF]", "%[FA]", "%[MB]", "%[cF]")
        ORT_C("%[MA]", "%[MB]", "%[nF]", "%[FA]", "%[FB]", "%[cF]")
        : [d] "=&v"(drop), [e] "=&v"(e), [x] "=&v"(x)
        : [NA] "v"(tNA), [NB] "v"(tNB), [MA] "v"(tMA), [MB] "v"(tMB), [FA] "v"(tFA), [FB] "v"(tFB), [nN] "v"(nN),
          [nF] "v"(nF), [cN] "v"(cN), [cF] "v"(cF));
#undef ORT_C
#else
#define ORT_CHILD(EA, EB, EC, XA, XB, XC) drop = (drop << 1) | (f2u(fmin3(XA, XB, XC) - fmax3(EA, EB, EC)) >> 31);
    ORT_CHILD(tNA, tNB, nN, tMA, tMB, cN)  // rank 0: A near, B near, C near
    ORT_CHILD(tNA, tMB, nN, tMA, tFB, cN)  // rank 1: B far
    ORT_CHILD(tMA, tNB, nN, tFA, tMB, cN)  // rank 2: A far
    ORT_CHILD(tMA, tMB, nN, tFA, tFB, cN)  // rank 3
    ORT_CHILD(tNA, tNB, nF, tMA, tMB, cF)  // ranks 4-7: C far
    ORT_CHILD(tNA, tMB, nF, tMA, tFB, cF)
    ORT_CHILD(tMA, tNB, nF, tFA, tMB, cF)
    ORT_CHILD(tMA, tMB, nF, tFA, tFB, cF)
#undef ORT_CHILD
#endif
    return drop;
}

// The surviving leaf children (keep, rank-reversed bits) of a leaf-children node whose
// children start at co, tested in rank order -- the order the reference pops them -- each
// with the tmin the reference pushed for it (max(max3(child entries), t_min), t_min folded
// into the C entries nN / nF; max is exact, so the order does not matter).  A hit ends the
// walk after its leaf (glsl:336): no later sibling is tested.  Returns whether one hit.
template <bool COUNT, class Masks>
ORT_FN bool leaf_kids(const KScene& S, FastStateT<Masks>& st, int co, uint32_t keep, float tNA, float tMA, float tNB,
                      float tMB, float nN, float nF, Counters& cnt) {
    uint32_t todo = keep;
    while (todo) {
        const int hb = 31 - __builtin_clz(todo);
        todo ^= 1u << hb;
        const uint32_t R = 7u - (uint32_t)hb;
        const uint2 lrec = fetch_node(S, co + (int)((st.otab >> (4 * R)) & 15u));
        if (COUNT) cnt.v[0] += 1;
#if defined(__HIP_DEVICE_COMPILE__)
        // bitwise selects (v_bfe_i32 + v_bfi_b32) in one asm block: the compiler turns a
        // plain select into v_cmp + s_nop + v_cndmask
        float eA, eB, eC;
        {
            uint32_t m;
            asm("v_bfe_i32 %[m], %[R], 1, 1\n\tv_bfi_b32 %[a], %[m], %[MA], %[NA]\n\t"
                "v_bfe_i32 %[m], %[R], 0, 1\n\tv_bfi_b32 %[b], %[m], %[MB], %[NB]\n\t"
                "v_bfe_i32 %[m], %[R], 2, 1\n\tv_bfi_b32 %[c], %[m], %[CF], %[CN]"
                : [a] "=&v"(eA), [b] "=&v"(eB), [c] "=&v"(eC), [m] "=&v"(m)
                : [R] "v"(R), [MA] "v"(tMA), [NA] "v"(tNA), [MB] "v"(tMB), [NB] "v"(tNB), [CF] "v"(nF), [CN] "v"(nN));
        }
#else
        const float eA = (R & 2u) ? tMA : tNA, eB = (R & 1u) ? tMB : tNB, eC = (R & 4u) ? nF : nN;
#endif
        const bool h = leaf_tests<COUNT>(S, st, (int)lrec.x, (int)lrec.y, fmax3(eA, eB, eC), cnt);
        todo = h ? 0u : todo;
    }
    return st.hit();
}

// Visit st.node: push its surviving children, or test its spheres.  Returns true when a hit
// ends the walk (glsl:336).
template <bool COUNT, class Masks, class Frames>
ORT_FN bool fast_visit(const KScene& S, const uint8_t* rank_lut, FastStateT<Masks>& st, Frames& fr, Counters& cnt) {
    const int D = S.depth;
    const uint2 rec = st.rec;
    if (COUNT) cnt.v[0] += 1;
    if (rec.y & ORT_INTERNAL_FLAG) {
        const int co = (int)rec.x;
        if (COUNT) {
            const long long rem = (long long)S.n_nodes - (long long)co;
            cnt.v[1] += (unsigned long long)(rem >= 8 ? 8 : (rem > 0 ? rem : 0));
        }
        // rejected-sphere skip (kid_table.h): one-sphere leaf children holding the sphere this
        // lane last rejected, at a tmin <= this node's (<= theirs), cannot end the walk; not
        // in the counting kernels, which count the reference walk's work.  The LUT maps octant
        // bits to rank bits one for one, so the skipped octants are cleared from the child mask
        // before its one LUT read (lut[c & ~s] = lut[c] & ~lut[s]), branch-free.
        uint32_t cm = rec.y & 0xffu;
        if (ORT_KID_SKIP_FOLD && !COUNT && Masks::kKidSkip && S.kid) {
            const uint2 kd = kKidPrefetch ? st.kd : fetch_kid(S, st.node);
            const uint32_t m = (((kd.x & 0xffffffu) == st.kc_id) ? (kd.x >> 24) : 0u) |
                               (((kd.y & 0xffffffu) == st.kc_id) ? (kd.y >> 24) : 0u);
            const float ptmin = fmax_tmin(fmax3(st.tNA, st.tNB, st.tNC));
            cm &= ~(m & (0u - (uint32_t)(st.kc_e <= ptmin)));
        }
        const uint32_t rcm = rank_lut[((st.otab & 7u) << 8) | cm];  // LUT row m
        const int h = 1 << (D - 1 - st.depth);  // half the node's width, in plane steps
        float tMA, tMB, tMC;
        if (Masks::kPreMid) {
            tMA = st.tMA;
            tMB = st.tMB;
            tMC = st.tMC;
        } else if (Masks::kRevPlanes) {
            const uint32_t h4 = st.h4;
            tMA = st.iA * (st.plane(st.aA + h4) - st.oA);
            tMB = st.iB * (st.plane(st.aB + h4) - st.oB);
            tMC = st.iC * (st.plane(st.aC + h4) - st.oC);
        } else {
            const float* nA = Masks::kKeepNear ? st.nA : st.at(st.pA, st.sA, st.cA());
            const float* nB = Masks::kKeepNear ? st.nB : st.at(st.pB, st.sB, st.cB());
            const float* nC = Masks::kKeepNear ? st.nC : st.at(st.pC, st.sC, st.cC());
            tMA = st.iA * (*st.at(nA, st.sA, h) - st.oA);
            tMB = st.iB * (*st.at(nB, st.sB, h) - st.oB);
            tMC = st.iC * (*st.at(nC, st.sC, h) - st.oC);
        }
        const float tNA = st.tNA, tNB = st.tNB, tNC = st.tNC, tFA = st.tFA, tFB = st.tFB, tFC = st.tFC;
        // child R enters at max3 of its axis entries (near half: tN, far half: tM) and exits at
        // min3 of its exits (tM / tF); t_min and t_max are folded into the C axis.
        const float nN = fmax_tmin(tNC), nF = fmax_tmin(tMC);
        const float cN = fmin2(tMC, st.closest), cF = fmin2(tFC, st.closest);  // closest == t_max here
        // keep child R <=> exit >= entry, with entry >= t_min > 0 and exit <= t_max finite, so
        // exit - entry is never NaN and is +0 when equal: its sign bit is "drop".  The drop
        // bits are shifted in rank order (rank 0 ends at bit 7: the reversed layout) -- one
        // v_max3 + v_min3 + v_sub + v_alignbit per child, no compare/select.
        uint32_t skip = 0;
        if (!ORT_KID_SKIP_FOLD && !COUNT && Masks::kKidSkip && S.kid) {
            const uint2 kd = kKidPrefetch ? st.kd : fetch_kid(S, st.node);
            const uint32_t m = (((kd.x & 0xffffffu) == st.kc_id) ? (kd.x >> 24) : 0u) |
                               (((kd.y & 0xffffffu) == st.kc_id) ? (kd.y >> 24) : 0u);
            const float ptmin = fmax_tmin(fmax3(tNA, tNB, tNC));
            skip = st.kc_e <= ptmin ? (uint32_t)rank_lut[((st.otab & 7u) << 8) | m] : 0u;
        }
        const uint32_t keep = rcm & ~skip & ~child_drops(tNA, tNB, tMA, tMB, tFA, tFB, nN, nF, cN, cF) & 0xffu;
        if (Masks::kInlineLeaves && (rec.y & ORT_LEAFKIDS_FLAG)) {
            // Every existing child is a leaf, so the reference pops the surviving ones next,
            // consecutively in rank order (a leaf pushes nothing): test them right here.
            if (leaf_kids<COUNT>(S, st, co, keep, tNA, tMA, tNB, tMB, nN, nF, cnt)) return true;
        } else if (Masks::kLeadLeaves) {
            // The surviving leaf children ranked before every surviving internal child are the
            // nodes the reference pops next, consecutively (a leaf pushes nothing): test them
            // here, push the rest.  Reversed rank bits: "before" = higher bits.
            const uint32_t rl = rank_lut[((st.otab & 7u) << 8) | ((rec.y >> ORT_LEAFMASK_SHIFT) & 0xffu)];
            const uint32_t kl = keep & rl, ki = keep & ~rl;
            const uint32_t lead = ki ? kl & ~((2u << (31 - __builtin_clz(ki))) - 1u) : kl;
            st.masks.put(st.depth, keep ^ lead);
            fr.setCo(st.depth, co);
            if (lead && leaf_kids<COUNT>(S, st, co, lead, tNA, tMA, tNB, tMB, nN, nF, cnt)) return true;
        } else {
            // level depth holds nothing yet (every deeper level is empty), so both writes are
            // harmless when no child survives
            st.masks.put(st.depth, keep);
            fr.setCo(st.depth, co);
        }
    } else {
        const float ntmin = st.depth == 0 ? kFastTMin : fmax_tmin(fmax3(st.tNA, st.tNB, st.tNC));
        if (leaf_tests<COUNT>(S, st, (int)rec.x, (int)rec.y, ntmin, cnt)) return true;  // glsl:336
    }
    return false;
}

// Pop the next node -- the lowest remaining rank of the deepest level with one left (the masks
// must not be empty) -- and load its record and box planes.
template <bool COUNT, class Masks, class Frames>
ORT_FN void fast_pop(const KScene& S, FastStateT<Masks>& st, Frames& fr);

// One node of the walk: visit st.node (push its surviving children, or test its spheres),
// then pop the next node.  Returns true when the walk is over (hit found, or stack empty).
template <bool COUNT, class Masks, class Frames>
ORT_FN bool fast_step(const KScene& S, const uint8_t* rank_lut, FastStateT<Masks>& st, Frames& fr, Counters& cnt) {
    if (fast_visit<COUNT>(S, rank_lut, st, fr, cnt)) return true;
    if (st.masks.empty()) return true;
#if defined(__HIP_DEVICE_COMPILE__) && defined(ORT_PAD_VALU)
    {   // issue-sensitivity experiment only (tools): ORT_PAD_VALU extra VALU per step
        float pv = 0.0f;
        for (int q = 0; q < ORT_PAD_VALU; ++q) asm volatile("v_mov_b32 %0, %0" : "+v"(pv));
    }
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(ORT_PAD_SALU)
    {   // issue-sensitivity experiment only (tools): ORT_PAD_SALU extra SALU per step
        int ps = 0;
        for (int q = 0; q < ORT_PAD_SALU; ++q) asm volatile("s_mov_b32 %0, %0" : "+s"(ps));
    }
#endif
    fast_pop<COUNT>(S, st, fr);
    return false;
}

template <bool COUNT, class Masks, class Frames>
ORT_FN void fast_pop(const KScene& S, FastStateT<Masks>& st, Frames& fr) {
    const int D = S.depth;
    // next node: lowest remaining rank of the deepest level with one left
    const int hb = st.masks.pop();
    const int L = hb >> 3;
    const uint32_t rk = (uint32_t)(~hb) & 7u;
    const int w = 1 << (D - 1 - L);  // child width in plane steps
    st.depth = L + 1;
    st.node = fr.getCo(L) + (int)((st.otab >> (4 * rk)) & 15u);
    fetch_rec(S, st.node, kKidPrefetch && !COUNT && Masks::kKidSkip && S.kid, st);
    if (Masks::kRevPlanes) {
        // near plane of the level-(L+1) child: the level-L ancestor's (offset bits below 8w
        // cleared; the table start is a multiple of 4T >= 8w bytes) plus w planes on the axes
        // where the child is the far half
        const uint32_t w4 = 4u << (D - 1 - L);
        st.h4 = w4 >> 1;
        const uint32_t m8 = ~(2u * w4 - 1u);
        const uint32_t s = (uint32_t)(D + 1 - L);  // log2(w4)
        st.aA = (st.aA & m8) | (((rk >> 1) & 1u) << s);
        st.aB = (st.aB & m8) | ((rk & 1u) << s);
        st.aC = (st.aC & m8) | (((rk >> 2) & 1u) << s);
        st.tNA = st.iA * (st.plane(st.aA) - st.oA);
        st.tFA = st.iA * (st.plane(st.aA + w4) - st.oA);
        st.tNB = st.iB * (st.plane(st.aB) - st.oB);
        st.tFB = st.iB * (st.plane(st.aB + w4) - st.oB);
        st.tNC = st.iC * (st.plane(st.aC) - st.oC);
        st.tFC = st.iC * (st.plane(st.aC + w4) - st.oC);
        if (Masks::kPreMid) {
            // h4 is 2 bytes (a misaligned plane offset) only for a level-D node, a leaf; the
            // kPreMid walk tests its leaves inline (kInlineLeaves), so it never pops one
            st.tMA = st.iA * (st.plane(st.aA + st.h4) - st.oA);
            st.tMB = st.iB * (st.plane(st.aB + st.h4) - st.oB);
            st.tMC = st.iC * (st.plane(st.aC + st.h4) - st.oC);
        }
    } else {
        const int keep = -2 * w;  // clears the offsets below the level-L ancestor
        {   // per 10-bit field: (c & keep) | (axis bit of rk ? w : 0)
            const uint32_t k3 = ((uint32_t)keep & 1023u) * 0x100401u;
            const uint32_t bits = ((rk >> 1) & 1u) | ((rk & 1u) << 10) | (((rk >> 2) & 1u) << 20);
            st.cP = (st.cP & k3) | bits * (uint32_t)w;
        }
        const float* nA = st.at(st.pA, st.sA, st.cA());
        const float* nB = st.at(st.pB, st.sB, st.cB());
        const float* nC = st.at(st.pC, st.sC, st.cC());
        if (Masks::kKeepNear) {
            st.nA = nA;
            st.nB = nB;
            st.nC = nC;
        }
        st.tNA = st.iA * (nA[0] - st.oA);
        st.tFA = st.iA * (*st.at(nA, st.sA, w) - st.oA);
        st.tNB = st.iB * (nB[0] - st.oB);
        st.tFB = st.iB * (*st.at(nB, st.sB, w) - st.oB);
        st.tNC = st.iC * (nC[0] - st.oC);
        st.tFC = st.iC * (*st.at(nC, st.sC, w) - st.oC);
        if (Masks::kPreMid) {  // (a leaf's half width is 0: its "mid" is never used)
            st.tMA = st.iA * (*st.at(nA, st.sA, w >> 1) - st.oA);
            st.tMB = st.iB * (*st.at(nB, st.sB, w >> 1) - st.oB);
            st.tMC = st.iC * (*st.at(nC, st.sC, w >> 1) - st.oC);
        }
    }
}

template <bool COUNT, class Masks, class Frames>
ORT_FN bool traverse_fast_t(const KScene& S, const float* planes, const uint8_t* rank_lut, const Ray& r, V3 inv,
                            float t_min, float t_max, int& hitEntry, float& hitT, Frames& fr, Counters& cnt,
                            Ray* walked = nullptr, int* steps = nullptr) {
    FastStateT<Masks> st;
    const bool in = fast_begin(S, planes, rank_lut, r, inv, t_min, t_max, st);
    int n = 0;  // walk steps (steps: the cost order's record; folds away without it)
    // (a leaf hold as in the deep bounce walk, lanes at a leaf waiting for company, cost the deep
    // camera walk 10-14 % at 8-16 lanes: the coherent camera rays reach leaves together anyway)
    if (in)
        while (!fast_step<COUNT>(S, rank_lut, st, fr, cnt)) {
            ++n;
        }
    if (steps) *steps = in ? n + 1 : 0;
    // the ray back from the walk state (bit-identical to r; no extra registers across the walk)
    if (walked) *walked = st.ray();
    if (!in) return false;
    hitEntry = st.hitEntry;
    hitT = st.closest;
    return st.hit();
}

// Split walk (the heavy camera rays of ort_trace_split): ONE ray's walk dealt over G lanes by
// its level-`level` subtrees.  The reference DFS (glsl:312-479) walks the subtree of a node
// completely before its next sibling, so the nodes of the walk's level-`level` subtrees are
// contiguous, in DFS order, and a hit ends the walk (glsl:336): the walk's result is the first
// hit of the lowest-ordered subtree holding one, unless a leaf above that level, visited before
// it, holds one.  Lane j walks the nodes above the level and the subtrees i with i % G == j,
// popping the others without visiting them, and stops at its first hit; `pos` orders the lanes'
// hits by their place in the DFS -- 2i + 1 for a hit inside subtree i, 2c for a hit in a leaf
// above the level visited after c subtrees -- and the lowest `pos` of the G lanes is the result
// of the whole walk (bit-identical: each lane's visits are the reference walk's own).
// Returns whether this lane found a hit; steps = the nodes it visited, own = those of them inside
// its own subtrees (the rest, above the level, every lane visits up to where it stops: a single
// walk's length is about the largest `steps - own` of the lanes plus the sum of their `own`).
template <class Masks, class Frames>
ORT_FN bool traverse_split(const KScene& S, const float* planes, const uint8_t* rank_lut, const Ray& r, V3 inv,
                           int level, int G, int j, int& pos, int& hitEntry, float& hitT, Frames& fr, int& steps,
                           int& own) {
    FastStateT<Masks> st;
    Counters cnt;  // (COUNT = false: untouched)
    steps = 0;
    own = 0;
    if (!fast_begin(S, planes, rank_lut, r, inv, kFastTMin, ORT_MAXFLOAT, st)) return false;
    int sub = -1, seen = 0;  // the level-`level` subtree the walk is in; how many were popped
    for (;;) {
        ++steps;
        own += st.depth >= level ? 1 : 0;
        if (fast_visit<false>(S, rank_lut, st, fr, cnt)) {
            pos = st.depth >= level ? 2 * sub + 1 : 2 * seen;
            hitEntry = st.hitEntry;
            hitT = st.closest;
            return true;
        }
        bool more = false;
        while (!st.masks.empty()) {  // the next node, passing over other lanes' subtrees
            fast_pop<false>(S, st, fr);
            if (st.depth != level) {
                more = true;
                break;
            }
            sub = seen++;
            if (sub % G == j) {
                more = true;
                break;
            }
        }
        if (!more) return false;
    }
}

template <bool COUNT, class Frames>
ORT_FN bool traverse_fast(const KScene& S, const float* planes, const uint8_t* rank_lut, const Ray& r, V3 inv,
                          float t_min, float t_max, int& hitEntry, float& hitT, Frames& fr, Counters& cnt) {
    if (S.depth <= 8) return traverse_fast_t<COUNT, Masks64>(S, planes, rank_lut, r, inv, t_min, t_max, hitEntry, hitT, fr, cnt);
    return traverse_fast_t<COUNT, Masks96>(S, planes, rank_lut, r, inv, t_min, t_max, hitEntry, hitT, fr, cnt);
}

// Literal restatement of traverseOctree (glsl:290-481) over the reference record layout
// (boxes read from memory, 200-entry stack).  Used for trees the compact layout cannot
// represent.  `stack_node`/`stack_tmin` point at ORT_MAX_STACK entries owned by the lane.
template <bool COUNT>
ORT_FN bool traverse_explicit(const KScene& S, const Ray& r, float t_min, float t_max, int& hitEntry, float& hitT,
                              int* stack_node, float* stack_tmin, Counters& cnt) {
    const V3 inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
    const float a = dot(r.d, r.d);
    int sp = 0;
    stack_node[0] = 0;
    stack_tmin[0] = t_min;
    bool hit = false;
    float closest = t_max;
    {
        const float4 A = S.nodeA[0], B = S.nodeB[0];
        float t0, t1;
        if (!ray_box(r, inv, mk(A.x, A.y, A.z), mk(B.x, B.y, B.z), t0, t1)) return false;
    }
    const uint32_t ocode = order_code(r.d);
    // bounded so that a malformed (cyclic) upload cannot hang the GPU
    for (long long guard = 0; sp >= 0 && guard < (1ll << 26); ++guard) {
        const int nodeIdx = stack_node[sp];
        const float ntmin = stack_tmin[sp];
        --sp;
        if (COUNT) cnt.v[0] += 1;
        const float4 A = S.nodeA[nodeIdx], B = S.nodeB[nodeIdx];
        const int co = f2i(A.w);
        const int oo = f2i(B.w);
        const int objectCount = S.count[nodeIdx];
        if (co == -1) {
            for (int i = 0; i < objectCount; ++i) {
                const int e = oo + i;
                const float4 spr = S.sph_cr[S.indices[e]];
                if (COUNT) cnt.v[2] += 1;
                float t;
                if (sphere_hit_t(r, a, spr, ntmin, closest, t)) {
                    hit = true;
                    closest = t;
                    hitEntry = e;
                    sp = -1;
                    if (COUNT) cnt.v[3] += 1;
                }
            }
        } else {
            for (int i = 7; i >= 0; --i) {
                const int oct = (int)((ocode >> (3 * i)) & 7u);
                const int childIdx = co + oct;
                if (childIdx >= S.n_nodes) continue;
                if (COUNT) cnt.v[1] += 1;
                const float4 CA = S.nodeA[childIdx], CB = S.nodeB[childIdx];
                float cmin, cmax;
                const bool boxhit = ray_box(r, inv, mk(CA.x, CA.y, CA.z), mk(CB.x, CB.y, CB.z), cmin, cmax);
                if (!boxhit || cmax < ntmin || cmin > closest ||
                    (f2i(CA.w) == -1 && f2i(CB.w) == -1))
                    continue;
                if (sp < ORT_MAX_STACK - 1) {
                    ++sp;
                    stack_node[sp] = childIdx;
                    stack_tmin[sp] = ort_maxf(cmin, ntmin);
                }
            }
        }
    }
    hitT = closest;
    return hit;
}

// bruteForceIntersect (glsl:484-498): exact closest hit over all spheres.
template <bool COUNT>
ORT_FN bool traverse_brute(const KScene& S, const Ray& r, float t_min, float t_max, int& hitSphere, float& hitT,
                           Counters& cnt) {
    const float a = dot(r.d, r.d);
    bool hit = false;
    float closest = t_max;
#ifndef ORT_BRUTE_FAST
#define ORT_BRUTE_FAST 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && ORT_BRUTE_FAST
    // the fast walk's sphere test (per-ray correctly rounded 1/a, Markstein quotient, guarded
    // sqrt: the same roots) whenever its preconditions hold for the wave, and the spheres read
    // with scalar loads -- every lane tests sphere i at once, so the address is wave-uniform
    if (!COUNT && !any_lane(!(t_min == kFastTMin && a_in_qdiv_range(a)))) {
        const float ya = 1.0f / a;
        typedef __attribute__((address_space(4))) const float4 ConstF4;
        ConstF4* sph = (ConstF4*)S.sph_cr;
        for (int i = 0; i < S.n_spheres; ++i) {
            const float4 s4 = sph[i];
            float t;
            // (radius^2 as sphere_hit_t computes it: one rounded product)
            if (sphere_hit_fast(r, a, ya, make_float4(s4.x, s4.y, s4.z, s4.w * s4.w), t_min, closest, t)) {
                hit = true;
                closest = t;
                hitSphere = i;
            }
        }
        hitT = closest;
        return hit;
    }
#endif
    for (int i = 0; i < S.n_spheres; ++i) {
        float t;
        if (COUNT) cnt.v[2] += 1;
        if (sphere_hit_t(r, a, S.sph_cr[i], t_min, closest, t)) {
            hit = true;
            closest = t;
            hitSphere = i;
            if (COUNT) cnt.v[3] += 1;
        }
    }
    hitT = closest;
    return hit;
}

struct HitRec {
    float t;
    V3 point, normal;
    int mat;
    V3 albedo;
    float fuzz, ri;
};

// --- random directions (glsl:104-173) ---
ORT_FN V3 random_in_unit_disk(ort_rng& st) {
    const float PI_F = (float)3.14159265359;
    const float spx = 2.0f * ort_rand2D(&st) - 1.0f;
    const float spy = 2.0f * ort_rand2D(&st) - 1.0f;
    // the four branches of glsl:109-131 with their one division hoisted out (divergent
    // branches each ran a full IEEE division): q = num / den, then the branch's phi from q
    const bool right = spx > -spy;
    const bool xbig = right ? (spx > spy) : (spx < spy);  // |spx| dominates: phi from spy / spx
    const float r = right ? (xbig ? spx : spy) : (xbig ? -spx : -spy);
    const float q = (xbig ? spy : spx) / (xbig ? spx : spy);
    float phi;
    if (xbig) phi = right ? q : 4.0f + q;
    else phi = right ? 2.0f - q : (spy != 0.0f ? 6.0f - q : 0.0f);
    phi *= PI_F / 4.0f;
    float sp, cp;
    ort_sincosf(phi, &sp, &cp);  // = ort_sinf(phi), ort_cosf(phi): one reduction
    return mk(r * cp, r * sp, 0.0f);
}
ORT_FN V3 random_in_unit_sphere(ort_rng& st) {
    const float PI_F = (float)3.14159265359;
    const float z = 2.0f * ort_rand2D(&st) - 1.0f;
    const float phi = 2.0f * PI_F * ort_rand2D(&st);
    const float r = ort_powf(ort_rand2D(&st), 1.0f / 3.0f);
    const float s = sqrtf(1.0f - z * z);
    float sp, cp;
    ort_sincosf(phi, &sp, &cp);
    return mk(r * s * cp, r * s * sp, r * z);
}
ORT_FN V3 random_cosine_direction(ort_rng& st) {
    const float PI_F = (float)3.14159265359;
    const float r1 = ort_rand2D(&st);
    const float r2 = ort_rand2D(&st);
    const float phi = 2.0f * PI_F * r1;
    const float sr2 = sqrtf(r2);
    float sp, cp;
    ort_sincosf(phi, &sp, &cp);
    return mk(cp * sr2, sp * sr2, sqrtf(1.0f - r2));
}

ORT_FN bool refract_vec(V3 v, V3 n, float ni_over_nt, V3& refracted) {
    const V3 uv = normalize(v);
    const float dt = dot(uv, n);
    const float disc = 1.0f - ni_over_nt * ni_over_nt * (1.0f - dt * dt);
    if (disc > 0.0f) {
        const float sq = sqrtf(disc);
        refracted = mk(ni_over_nt * (uv.x - n.x * dt) - n.x * sq, ni_over_nt * (uv.y - n.y * dt) - n.y * sq,
                       ni_over_nt * (uv.z - n.z * dt) - n.z * sq);
        return true;
    }
    return false;
}
ORT_FN float schlick(float cosine, float ri) {
    float r0 = (1.0f - ri) / (1.0f + ri);
    r0 = r0 * r0;
    return r0 + (1.0f - r0) * ort_powf(1.0f - cosine, 5.0f);
}

// Material_bsdf (glsl:525-589)
// FINAL: nothing after this bounce reads the scattered ray or the RNG state (last bounce of
// the last sample), so only what reaches the pixel is computed: Lambert and dielectric
// attenuations do not depend on the sampled direction (their sampling is skipped); metal
// still samples, its absorption test needs the direction.
template <bool FINAL = false>
ORT_FN bool bsdf(const HitRec& h, const Ray& wo, Ray& wi, V3& att, ort_rng& st) {
    wi.o = h.point;
    if (FINAL && (h.mat == 0 || h.mat == 2)) {
        att = h.mat == 0 ? h.albedo : mk(1.0f, 1.0f, 1.0f);
        wi.d = wo.d;
        return true;
    }
    switch (h.mat) {
        case 0: {
            const V3 ld = random_cosine_direction(st);
            const V3 w = h.normal;
            const V3 a = (fabsf(w.x) > 0.1f) ? mk(0.0f, 1.0f, 0.0f) : mk(1.0f, 0.0f, 0.0f);
            const V3 u = normalize(cross(a, w));
            const V3 v = cross(w, u);
            wi.d = normalize(mk((ld.x * u.x + ld.y * v.x) + ld.z * w.x, (ld.x * u.y + ld.y * v.y) + ld.z * w.y,
                                (ld.x * u.z + ld.y * v.z) + ld.z * w.z));
            att = h.albedo;
            return true;
        }
        case 1: {
            const float fuzz = h.fuzz;
            const V3 refl = reflect(normalize(wo.d), h.normal);
            const V3 rs = random_in_unit_sphere(st);
            wi.d = mk(refl.x + fuzz * rs.x, refl.y + fuzz * rs.y, refl.z + fuzz * rs.z);
            att = h.albedo;
            return dot(wi.d, h.normal) > 0.0f;
        }
        case 2: {
            V3 outward;
            float ni_over_nt, cosine;
            const float ri = h.ri;
            att = mk(1.0f, 1.0f, 1.0f);
            if (dot(wo.d, h.normal) > 0.0f) {
                outward = mk(-h.normal.x, -h.normal.y, -h.normal.z);
                ni_over_nt = ri;
                cosine = dot(wo.d, h.normal) / length(wo.d);
                cosine = sqrtf(1.0f - ri * ri * (1.0f - cosine * cosine));
            } else {
                outward = h.normal;
                ni_over_nt = 1.0f / ri;
                cosine = -dot(wo.d, h.normal) / length(wo.d);
            }
            V3 refracted = mk(0.0f, 0.0f, 0.0f);
            const bool can = refract_vec(wo.d, outward, ni_over_nt, refracted);
            const float prob = can ? schlick(cosine, ri) : 1.0f;
            if (ort_rand2D(&st) < prob) wi.d = reflect(wo.d, h.normal);
            else wi.d = refracted;
            return true;
        }
        default:
            return false;
    }
}

ORT_FN V3 sky_color(const Ray& r) {
    const float t = 0.5f * (r.d.y + 1.0f);
    return mk((1.0f - t) * 1.0f + t * 0.5f, (1.0f - t) * 1.0f + t * 0.7f, (1.0f - t) * 1.0f + t * 1.0f);
}

// Camera_getRay (glsl:205-221)
ORT_FN Ray camera_ray(const KCamera& c, float s, float t, float W, float H, ort_rng& st) {
    const float pixelRadius = 0.5f / ort_maxf(W, H);
    const float jx = pixelRadius * (ort_rand2D(&st) - 0.5f);
    const float jy = pixelRadius * (ort_rand2D(&st) - 0.5f);
    const V3 rdd = random_in_unit_disk(st);
    const V3 rd = mk(c.lensRadius * rdd.x, c.lensRadius * rdd.y, c.lensRadius * rdd.z);
    const V3 off = mk(c.u.x * rd.x + c.v.x * rd.y, c.u.y * rd.x + c.v.y * rd.y, c.u.z * rd.x + c.v.z * rd.y);
    Ray r;
    r.o = add(c.origin, off);
    const float a = s + jx, b = t + jy;
    r.d = normalize(mk((((c.lowerLeft.x + a * c.horizontal.x) + b * c.vertical.x) - c.origin.x) - off.x,
                       (((c.lowerLeft.y + a * c.horizontal.y) + b * c.vertical.y) - c.origin.y) - off.y,
                       (((c.lowerLeft.z + a * c.horizontal.z) + b * c.vertical.z) - c.origin.z) - off.z));
    return r;
}

// ---------------------------------------------------------------------------------------
// Path steps.  The GPU runs them as a wavefront pipeline (ort_kernel.hip: trace kernel ->
// rare exact-walk kernel -> shade kernel, per bounce); shade_pixel below chains the same
// steps for one pixel (host emulation / reference order).  Both orders give identical
// pixels because every path is independent and each step is a pure function of its state.

struct PixelParams {
    KCamera cam;
    int W, H, ns, maxDepth;
};

// main() prologue + the sample-s part of its loop up to radiance()'s first line
// (glsl:640, 647-654, 602): consumes 2 + 4 rand2D, returns the normalised camera ray.
// st must hold the pixel's RNG state at the start of sample s (FragCoord/iResolution for s=0).
ORT_FN void pixel_rng_init(const PixelParams& P, int px, int py, ort_rng& st) {
    st.x = ((float)px + 0.5f) / (float)P.W;
    st.y = ((float)py + 0.5f) / (float)P.H;
}
ORT_FN Ray primary_ray(const PixelParams& P, int px, int py, int s, ort_rng& st) {
    const float W = (float)P.W, H = (float)P.H;
    const float fx = (float)px + 0.5f, fy = (float)py + 0.5f;
    const int sqrt_ns = (int)sqrtf((float)P.ns);
    const int i = s % sqrt_ns;
    const int j = s / sqrt_ns;
    // x / 1.0f == x exactly: one sample per pixel (the benchmark) skips both divisions
    const float ru = (float)i + ort_rand2D(&st);
    const float u = (fx + (sqrt_ns == 1 ? ru : ru / (float)sqrt_ns)) / W;
    const float rv = (float)j + ort_rand2D(&st);
    const float v = (fy + (sqrt_ns == 1 ? rv : rv / (float)sqrt_ns)) / H;
    Ray ray = camera_ray(P.cam, u, v, W, H, st);
    ray.d = normalize(ray.d);
    return ray;
}

#define ORT_TRACE_MISS 0
#define ORT_TRACE_HIT 1
#define ORT_TRACE_DEFER 2

// intersectScene(ray, 0.001, MAXFLOAT) (glsl:500-506, 607).  MODE: 0 compact octree,
// 1 explicit octree, 2 brute force.  With MODE 0 and allow_defer, a ray the fast walk
// cannot take (some 1/d component not finite) is reported as DEFER instead of walking
// it exactly here, so the exact walk's registers stay out of the hot kernel.
// bounce: the ray of a bounce >= 1 -- walked like the GPU's bounce kernel does (Masks64Plain /
// Masks96Lean: no inline leaf children, the rejected-sphere skip; at depth 9-10 over the plane
// tables planes_b in the Masks96Lean layout), same result.
template <int MODE, bool COUNT, class Frames>
ORT_FN int trace_ray(const KScene& S, const float* planes, const uint8_t* rank_lut, const Ray& r, bool allow_defer,
                     float& t, int& entry, Frames& fr, int* snode, float* stmin, Counters& cnt, bool bounce = false,
                     const float* planes_b = nullptr) {
    bool hit;
    entry = -1;
    t = 0.0f;
    if (MODE == 0) {
        V3 inv = mk(1.0f / r.d.x, 1.0f / r.d.y, 1.0f / r.d.z);
        if (rank_lut && fast_prepare(S, r, inv)) {
            if (COUNT) cnt.v[5] += 1;
            if (!bounce)
                hit = traverse_fast<COUNT>(S, planes, rank_lut, r, inv, 0.001f, ORT_MAXFLOAT, entry, t, fr, cnt);
            else if (S.depth <= 8)
                hit = traverse_fast_t<COUNT, Masks64Plain>(S, planes, rank_lut, r, inv, 0.001f, ORT_MAXFLOAT, entry, t, fr, cnt);
            else
                hit = traverse_fast_t<COUNT, Masks96Lean>(S, planes_b, rank_lut, r, inv, 0.001f, ORT_MAXFLOAT, entry, t, fr, cnt);
        } else if (allow_defer) {
            return ORT_TRACE_DEFER;
        } else {
            if (COUNT) cnt.v[5] += 1;
            hit = traverse_compact<COUNT>(S, planes, r, 0.001f, ORT_MAXFLOAT, entry, t, fr, cnt);
        }
    } else if (MODE == 1) {
        if (COUNT) cnt.v[5] += 1;
        hit = traverse_explicit<COUNT>(S, r, 0.001f, ORT_MAXFLOAT, entry, t, snode, stmin, cnt);
    } else {
        if (COUNT) cnt.v[5] += 1;
        hit = traverse_brute<COUNT>(S, r, 0.001f, ORT_MAXFLOAT, entry, t, cnt);
    }
    return hit ? ORT_TRACE_HIT : ORT_TRACE_MISS;
}

// The IntersectInfo Sphere_hit fills for the accepted hit (glsl:240-251).
template <int MODE>
ORT_FN HitRec hit_record(const KScene& S, const Ray& r, float t, int entry) {
    int sidx;
    float4 sp;
    if (MODE == 0) {
        sidx = S.leaf_idx[entry];
        sp = S.sph_cr[sidx];  // (leaf_sph holds radius^2)
    } else if (MODE == 1) {
        sidx = S.indices[entry];
        sp = S.sph_cr[sidx];
    } else {
        sidx = entry;
        sp = S.sph_cr[sidx];
    }
    HitRec h;
    h.t = t;
    h.point = mk(r.o.x + t * r.d.x, r.o.y + t * r.d.y, r.o.z + t * r.d.z);
    h.normal = mk((h.point.x - sp.x) / sp.w, (h.point.y - sp.y) / sp.w, (h.point.z - sp.z) / sp.w);
    const float4 ma = S.sph_ma[sidx];
    const float2 fr2 = S.sph_fr[sidx];
    h.mat = (int)ma.x;
    h.albedo = mk(ma.y, ma.z, ma.w);
    h.fuzz = fr2.x;
    h.ri = fr2.y;
    return h;
}

// One iteration of radiance()'s bounce loop after intersectScene (glsl:607-627).
// Returns true when the path ends here (absorbed, or escaped to the sky).
template <bool FINAL = false>
ORT_FN bool shade_bounce(bool hit, const HitRec& h, Ray& ray, V3& c, float& importance, ort_rng& st) {
    if (hit) {
        Ray wi;
        wi.d = ray.d;
        V3 att = mk(0.0f, 0.0f, 0.0f);
        const bool scattered = bsdf<FINAL>(h, ray, wi, att, st);
        ray.o = wi.o;
        ray.d = wi.d;
        if (!scattered) {
            c = mul(c, mk(0.0f, 0.0f, 0.0f));
            return true;
        }
        c = mul(c, att);
        importance *= ort_maxf(att.x, ort_maxf(att.y, att.z));
        return false;
    }
    c = mul(c, sky_color(ray));
    return true;
}

// col /= float(numSamples); pow(col, 1/2.2) (glsl:659-661)
ORT_FN V3 finish_pixel(V3 col, int ns) {
    const float fns = (float)ns;
    if (ns != 1) col = mk(col.x / fns, col.y / fns, col.z / fns);  // x / 1.0f == x exactly
    const float g = 1.0f / 2.2f;
    return mk(ort_powf(col.x, g), ort_powf(col.y, g), ort_powf(col.z, g));
}

// main() of the fragment shader (glsl:636-664) for pixel (px, py), py = 0 the bottom row,
// as one sequential chain of the steps above (host emulation).
// planes_b: the bounce walk's plane tables (trace_ray).
template <int MODE, bool COUNT, class Frames>
ORT_FN V3 shade_pixel(const PixelParams& P, const KScene& S, const float* planes, const float* planes_b,
                      const uint8_t* rank_lut, Frames& fr, int* snode, float* stmin, int px, int py, Counters& cnt) {
    ort_rng st;
    pixel_rng_init(P, px, py, st);
    V3 col = mk(0.0f, 0.0f, 0.0f);
    for (int s = 0; s < P.ns; ++s) {
        Ray ray = primary_ray(P, px, py, s, st);
        V3 c = mk(1.0f, 1.0f, 1.0f);
        float importance = 1.0f;
        for (int b = 0; b < P.maxDepth; ++b) {
            if (importance < 0.01f) break;
            float t;
            int entry;
            const int tr = trace_ray<MODE, COUNT>(S, planes, rank_lut, ray, false, t, entry, fr, snode, stmin, cnt, b > 0, planes_b);
            HitRec h;
            if (tr == ORT_TRACE_HIT) h = hit_record<MODE>(S, ray, t, entry);
            const bool hit = tr == ORT_TRACE_HIT;
            const bool fin = b == P.maxDepth - 1 && s == P.ns - 1;  // the RNG state is dead after it
            if (fin ? shade_bounce<true>(hit, h, ray, c, importance, st) : shade_bounce(hit, h, ray, c, importance, st))
                break;
        }
        col = add(col, c);
    }
    return finish_pixel(col, P.ns);
}

}  // namespace ort
