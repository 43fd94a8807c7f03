// prune_sim.cpp -- analysis only (not part of the product): replays the reference's DFS
// (glsl:290-481, explicit stack, early exit after the first hitting leaf) for a batch of
// rays and counts how many node visits a per-node bound of the subtree's SPHERES would let a
// kernel skip without changing any result: a leaf only reports a hit on one of its own
// spheres, so a subtree whose sphere-union box the ray's half-line (t > t_min) misses cannot
// hold the first hitting leaf -- skipping it leaves every later leaf's test unchanged.
// Build: g++ -O2 -shared -fPIC -o tools/libprune_sim.so tools/prune_sim.cpp
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <vector>

namespace {
struct V3 { float x, y, z; };
inline float fminr(float a, float b) { return (b < a) ? b : a; }
inline float fmaxr(float a, float b) { return (a < b) ? b : a; }

bool ray_box(V3 o, V3 inv, const float* mn, const float* mx, float& tmin, float& tmax) {
    const float tb[3] = {(mn[0] - o.x) * inv.x, (mn[1] - o.y) * inv.y, (mn[2] - o.z) * inv.z};
    const float tt[3] = {(mx[0] - o.x) * inv.x, (mx[1] - o.y) * inv.y, (mx[2] - o.z) * inv.z};
    tmin = fmaxr(fmaxr(fminr(tb[0], tt[0]), fminr(tb[1], tt[1])), fminr(tb[2], tt[2]));
    tmax = fminr(fminr(fmaxr(tb[0], tt[0]), fmaxr(tb[1], tt[1])), fmaxr(tb[2], tt[2]));
    return tmax >= tmin;
}

bool sphere_hit(V3 o, V3 d, const float* s, float tmn, float tmx, float& t) {
    const V3 oc = {o.x - s[0], o.y - s[1], o.z - s[2]};
    const float a = d.x * d.x + d.y * d.y + d.z * d.z;
    const float hb = oc.x * d.x + oc.y * d.y + oc.z * d.z;
    const float c = oc.x * oc.x + oc.y * oc.y + oc.z * oc.z - s[3] * s[3];
    const float disc = hb * hb - a * c;
    if (disc > 0) {
        const float r = sqrtf(disc);
        float tt = (-hb - r) / a;
        if (tt < tmx && tt > tmn) { t = tt; return true; }
        tt = (-hb + r) / a;
        if (tt < tmx && tt > tmn) { t = tt; return true; }
    }
    return false;
}

void order_for(V3 d, int ord[8]) {
    const int nx = d.x < 0, ny = d.y < 0, nz = d.z < 0;
    const int m = (nz << 2) | (nx << 1) | ny;
    for (int r = 0; r < 8; ++r) {
        int p = r;
        if (nx) p = (r & 4) | ((r & 1) << 1) | ((r >> 1) & 1);
        ord[r] = p ^ m;
    }
}
}  // namespace

extern "C" {

// bounds[6*i] = min xyz, max xyz of the union of the spheres of node i's subtree, inflated by
// `margin`; a node without spheres gets an empty box (min > max).  Children have larger BFS
// indices, so one backwards sweep.
void prune_sim_bounds(const int32_t* co, const int32_t* oo, const int32_t* cnt, const int32_t* idx, int32_t n,
                      const float* sph, float margin, float* b) {
    for (int64_t i = (int64_t)n - 1; i >= 0; --i) {
        float lo[3] = {INFINITY, INFINITY, INFINITY}, hi[3] = {-INFINITY, -INFINITY, -INFINITY};
        if (co[i] == -1) {
            for (int j = 0; j < cnt[i]; ++j) {
                const float* s = sph + 4 * idx[oo[i] + j];
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fminf(lo[a], s[a] - s[3] - margin);
                    hi[a] = fmaxf(hi[a], s[a] + s[3] + margin);
                }
            }
        } else {
            for (int k = 0; k < 8; ++k) {
                const int64_t c = (int64_t)co[i] + k;
                if (c >= n) continue;
                for (int a = 0; a < 3; ++a) {
                    lo[a] = fminf(lo[a], b[6 * c + a]);
                    hi[a] = fmaxf(hi[a], b[6 * c + 3 + a]);
                }
            }
        }
        for (int a = 0; a < 3; ++a) {
            b[6 * i + a] = lo[a];
            b[6 * i + 3 + a] = hi[a];
        }
    }
}

// per_ray[8*r]: reference pops (internal + leaf), [+1] internal pops, [+2] pops with the
// prune (a pruned node still costs its pop), [+3] pruned pops, [+4] internal pops with the
// prune (not pruned ones), [+5] sphere tests, [+6] sphere tests with the prune, [+7] pruned
// internal nodes.  prune_from: only nodes at
// depth >= prune_from are tested.  Returns the number of rays whose result differs (must be 0).
int64_t prune_sim_run(const float* nmin, const float* nmax, const int32_t* co, const int32_t* oo, const int32_t* cnt,
                      const int32_t* idx, int32_t n, const float* sph, const float* bounds, int prune_from, int mode,
                      const float* rays, int64_t nrays, int32_t* per_ray, float* hit_t, int32_t* hit_s) {
    std::vector<int32_t> stk(1024), std_(1024);
    std::vector<float> stt(1024);
    int64_t bad = 0;
    for (int64_t r = 0; r < nrays; ++r) {
        const V3 o = {rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]};
        const V3 d = {rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]};
        const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        int32_t* pr = per_ray + 8 * r;
        for (int q = 0; q < 8; ++q) pr[q] = 0;
        float res[2] = {-1.0f, -1.0f};
        float t0, t1;
        if (!ray_box(o, inv, nmin, nmax, t0, t1)) {
            if (hit_t) hit_t[r] = -1.0f;
            if (hit_s) hit_s[r] = -1;
            continue;
        }
        int ord[8];
        order_for(d, ord);
        for (int pass = 0; pass < 2; ++pass) {
            int sp = 0;
            stk[0] = 0;
            stt[0] = 0.001f;
            std_[0] = 0;
            float closest = 3.402823466e+38f;
            bool hit = false;
            int hs = -1;
            while (sp >= 0) {
                const int32_t ni = stk[sp];
                const float ntmin = stt[sp];
                const int dep = std_[sp];
                --sp;
                pr[pass ? 2 : 0] += 1;
                if (pass && dep >= prune_from) {
                    const float* bl = bounds + 6 * ni;
                    const float* bh = bl + 3;
                    bool miss;
                    if (mode == 0) {  // half-line (t > t_min) vs the sphere-union box
                        float a, b;
                        miss = !ray_box(o, inv, bl, bh, a, b) || b < 0.001f;
                    } else {  // the origin past the box along the direction of travel: 3 axes / y only
                        const float oo3[3] = {o.x, o.y, o.z}, dd3[3] = {d.x, d.y, d.z};
                        miss = false;
                        for (int a = (mode == 2 ? 1 : 0); a < (mode == 2 ? 2 : 3); ++a)
                            miss = miss || (dd3[a] > 0 ? oo3[a] > bh[a] : oo3[a] < bl[a]);
                    }
                    if (miss) {
                        pr[3] += 1;
                        pr[7] += co[ni] != -1;
                        continue;
                    }
                }
                if (co[ni] == -1) {
                    for (int j = 0; j < cnt[ni]; ++j) {
                        pr[pass ? 6 : 5] += 1;
                        float t;
                        if (sphere_hit(o, d, sph + 4 * idx[oo[ni] + j], ntmin, closest, t)) {
                            closest = t;
                            hit = true;
                            hs = idx[oo[ni] + j];
                            sp = -1;
                        }
                    }
                } else {
                    pr[pass ? 4 : 1] += 1;
                    for (int i = 7; i >= 0; --i) {
                        const int64_t c = (int64_t)co[ni] + ord[i];
                        if (c >= n) continue;
                        float cmin, cmax;
                        if (!ray_box(o, inv, nmin + 3 * c, nmax + 3 * c, cmin, cmax) || cmax < ntmin || cmin > closest ||
                            (co[c] == -1 && oo[c] == -1))
                            continue;
                        if (sp < 1022) {
                            ++sp;
                            stk[sp] = (int32_t)c;
                            stt[sp] = fmaxr(cmin, ntmin);
                            std_[sp] = dep + 1;
                        }
                    }
                }
            }
            res[pass] = hit ? closest : -1.0f;
            if (!pass && hit_s) hit_s[r] = hs;
        }
        if (hit_t) hit_t[r] = res[0];
        if (res[0] != res[1]) ++bad;
    }
    return bad;
}
}

// ---- lockstep cost model ---------------------------------------------------------------
// Quantized bound per INTERNAL node, relative to its own cell: per face an offset of k/8 of
// the cell width along the face normal, k in [-3, 3] (positive = outward), or unbounded
// (code 127) when the spheres reach further out than 3/8 of the width.  Rounded outward.
extern "C" void prune_sim_quantize(const float* nmin, const float* nmax, const int32_t* co, int32_t n, const float* bounds,
                                   int8_t* q /* 6 per node */) {
    for (int64_t i = 0; i < n; ++i) {
        for (int a = 0; a < 3; ++a) {
            const float lo = nmin[3 * i + a], hi = nmax[3 * i + a], w = hi - lo;
            const float blo = bounds[6 * i + a], bhi = bounds[6 * i + 3 + a];
            int8_t klo = 127, khi = 127;
            if (co[i] != -1 && w > 0 && blo <= bhi) {
                const float out_lo = (lo - blo) / w * 8.0f, out_hi = (bhi - hi) / w * 8.0f;  // outward, in w/8
                const int kl = (int)ceilf(out_lo), kh = (int)ceilf(out_hi);
                klo = kl > 3 ? 127 : (int8_t)(kl < -3 ? -3 : kl);
                khi = kh > 3 ? 127 : (int8_t)(kh < -3 ? -3 : kh);
            }
            q[6 * i + a] = klo;
            q[6 * i + 3 + a] = khi;
        }
    }
}

namespace {
struct Lane {
    std::vector<int32_t> stk;
    std::vector<float> stt;
    int sp = -1;
    float closest = 3.402823466e+38f;
    bool done = true;
    V3 o, d, inv;
    int ord[8];
};

bool quant_miss(const Lane& L, const float* nmin, const float* nmax, const int8_t* q, int64_t ni) {
    float lo[3], hi[3];
    for (int a = 0; a < 3; ++a) {
        const float cl = nmin[3 * ni + a], ch = nmax[3 * ni + a], w = ch - cl;
        lo[a] = q[6 * ni + a] == 127 ? -INFINITY : cl - q[6 * ni + a] * w / 8.0f;
        hi[a] = q[6 * ni + 3 + a] == 127 ? INFINITY : ch + q[6 * ni + 3 + a] * w / 8.0f;
    }
    float a, b;
    return !ray_box(L.o, L.inv, lo, hi, a, b) || b < 0.001f;
}
}  // namespace

// Per wave of 64 rays: the kernel's loop in lockstep.  Each iteration every walking lane pops
// one node: cost P (+T with the prune test); a pruned internal node ends the lane's iteration
// (prune 1: at the pop, tested on the quantized bound); otherwise internal block I if any lane
// has an internal node; with inline_leaves a leaf-children node tests its surviving leaf
// children in that iteration (K per kid iteration + S per object iteration, lockstep over
// lanes); a popped leaf costs S per object iteration.  costs = {P, I, K, S, T}.
// out[2*w] = VALU model cost of wave w, out[2*w+1] = its iterations.
extern "C" void prune_sim_lockstep(const float* nmin, const float* nmax, const int32_t* co, const int32_t* oo,
                                   const int32_t* cnt, const int32_t* idx, int32_t n, const float* sph, const int8_t* q,
                                   int prune, int inline_leaves, const float* costs, const float* rays, int64_t nwaves,
                                   double* out) {
    const float P = costs[0], I = costs[1], K = costs[2], S = costs[3], T = costs[4];
    std::vector<Lane> lanes(64);
    for (auto& L : lanes) { L.stk.resize(1024); L.stt.resize(1024); }
    auto is_leafkids = [&](int64_t ni) {
        if (co[ni] == -1) return false;
        bool any = false;
        for (int k = 0; k < 8; ++k) {
            const int64_t c = (int64_t)co[ni] + k;
            if (c >= n) continue;
            if (co[c] != -1) return false;
            any = true;
        }
        return any;
    };
    for (int64_t w = 0; w < nwaves; ++w) {
        for (int l = 0; l < 64; ++l) {
            Lane& L = lanes[l];
            const float* r = rays + 6 * (64 * w + l);
            L.o = {r[0], r[1], r[2]};
            L.d = {r[3], r[4], r[5]};
            L.inv = {1.0f / L.d.x, 1.0f / L.d.y, 1.0f / L.d.z};
            float t0, t1;
            L.done = !ray_box(L.o, L.inv, nmin, nmax, t0, t1);
            L.sp = 0;
            L.stk[0] = 0;
            L.stt[0] = 0.001f;
            L.closest = 3.402823466e+38f;
            order_for(L.d, L.ord);
        }
        double cost = 0;
        int64_t iters = 0;
        for (;;) {
            bool any = false;
            for (auto& L : lanes) any = any || !L.done;
            if (!any) break;
            ++iters;
            cost += P + (prune == 1 ? T : 0.0f);
            bool any_internal = false;
            int max_leaf_objs = 0;
            // per lane: inline leaf children to test this iteration (leaf node, ntmin)
            std::vector<std::vector<std::pair<int64_t, float>>> kids(64);
            for (int l = 0; l < 64; ++l) {
                Lane& L = lanes[l];
                if (L.done) continue;
                const int64_t ni = L.stk[L.sp];
                const float ntmin = L.stt[L.sp];
                --L.sp;
                if (co[ni] == -1) {  // a leaf reached by the pop
                    max_leaf_objs = cnt[ni] > max_leaf_objs ? cnt[ni] : max_leaf_objs;
                    for (int j = 0; j < cnt[ni]; ++j) {
                        float t;
                        if (sphere_hit(L.o, L.d, sph + 4 * idx[oo[ni] + j], ntmin, L.closest, t)) {
                            L.closest = t;
                            L.done = true;
                        }
                    }
                } else if (prune == 1 && quant_miss(L, nmin, nmax, q, ni)) {
                    // pruned: nothing more this iteration
                } else {
                    any_internal = true;
                    const bool lk = inline_leaves == 1 && is_leafkids(ni);
                    // surviving children in rank order
                    int64_t sc[8];
                    float st[8];
                    int ns = 0;
                    for (int i = 0; i < 8; ++i) {
                        const int64_t c = (int64_t)co[ni] + L.ord[i];
                        if (c >= n) continue;
                        float cmin, cmax;
                        if (!ray_box(L.o, L.inv, nmin + 3 * c, nmax + 3 * c, cmin, cmax) || cmax < ntmin ||
                            cmin > L.closest || (co[c] == -1 && oo[c] == -1))
                            continue;
                        if (prune == 2 && co[c] != -1 && quant_miss(L, nmin, nmax, q, c)) continue;  // at the push
                        sc[ns] = c;
                        st[ns++] = fmaxr(cmin, ntmin);
                    }
                    int lead = 0;  // inline_leaves 2: the leading leaf children (popped next, consecutively)
                    if (lk) lead = ns;
                    else if (inline_leaves == 2)
                        while (lead < ns && co[sc[lead]] == -1) ++lead;
                    for (int i = 0; i < lead; ++i) kids[l].push_back({sc[i], st[i]});
                    for (int i = ns - 1; i >= lead; --i) {
                        ++L.sp;
                        L.stk[L.sp] = (int32_t)sc[i];
                        L.stt[L.sp] = st[i];
                    }
                }
                if (!L.done && L.sp < 0 && kids[l].empty()) L.done = true;
            }
            if (any_internal) cost += I + (prune == 2 ? T : 0.0f);
            if (max_leaf_objs) cost += S * max_leaf_objs;
            // inline leaf children, lockstep: kid iteration j, then its object iterations
            for (size_t j = 0;; ++j) {
                bool more = false;
                int mo = 0;
                for (int l = 0; l < 64; ++l) {
                    Lane& L = lanes[l];
                    if (j >= kids[l].size() || L.closest < 3.402823466e+38f) continue;
                    more = true;
                    const int64_t c = kids[l][j].first;
                    mo = cnt[c] > mo ? cnt[c] : mo;
                    for (int k = 0; k < cnt[c]; ++k) {
                        float t;
                        if (sphere_hit(L.o, L.d, sph + 4 * idx[oo[c] + k], kids[l][j].second, L.closest, t)) L.closest = t;
                    }
                }
                if (!more) break;
                cost += K + S * mo;
            }
            for (int l = 0; l < 64; ++l) {
                Lane& L = lanes[l];
                if (!kids[l].empty() && L.closest < 3.402823466e+38f) L.done = true;
                if (!L.done && L.sp < 0) L.done = true;
            }
        }
        out[2 * w] = cost;
        out[2 * w + 1] = (double)iters;
    }
}
