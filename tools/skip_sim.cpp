// skip_sim.cpp -- analysis only (not part of the product): replays the reference's DFS
// (glsl:290-481, explicit stack, early exit after the first hitting leaf) for a batch of
// rays and counts how much of the walk a per-ray cache of REJECTED sphere tests would let a
// kernel skip without changing any result:
//   * a sphere test rejected over the range (e, t_max) is rejected over every (e', t_max)
//     with e' >= e, so a later leaf holding the same sphere need not test it again;
//   * a subtree whose spheres (<= K distinct) were all rejected with e <= the subtree's
//     pushed tmin can be skipped whole.
// Build: g++ -O2 -shared -fPIC -o tools/libskip_sim.so tools/skip_sim.cpp
#include <math.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
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

// sign-vector traversal order (glsl:352-447) for non-zero components: perm(r) ^ m
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

// sum_k: per node, distinct sphere ids of its subtree if <= K (else count = K+1), K <= 4.
// Computed bottom-up (children have larger BFS indices).
void skip_sim_summaries(const int32_t* co, const int32_t* oo, const int32_t* cnt, const int32_t* idx, int32_t n, int K,
                        int32_t* sum_ids /* n*K */, int8_t* sum_n) {
    for (int64_t i = (int64_t)n - 1; i >= 0; --i) {
        int32_t ids[8];
        int m = 0;
        bool many = false;
        auto add = [&](int32_t s) {
            for (int j = 0; j < m; ++j) if (ids[j] == s) return;
            if (m < K) ids[m++] = s; else many = true;
        };
        if (co[i] == -1) {
            for (int j = 0; j < cnt[i] && !many; ++j) add(idx[oo[i] + j]);
        } else {
            for (int k = 0; k < 8 && !many; ++k) {
                const int64_t c = (int64_t)co[i] + k;
                if (c >= n) continue;
                if (sum_n[c] > K) { many = true; break; }
                for (int j = 0; j < sum_n[c]; ++j) add(sum_ids[c * K + j]);
            }
        }
        sum_n[i] = many ? (int8_t)(K + 1) : (int8_t)m;
        for (int j = 0; j < m; ++j) sum_ids[(int64_t)i * K + j] = ids[j];
    }
}

// stats[0] rays, [1] pops, [2] internal pops, [3] leaf pops, [4] sphere tests,
// [5] tests skipped by the CACHE-entry rejection cache, [7] sphere tests remaining with both skips,
// [8] hits, [9] pops with both skips, [10] rays whose result differs (must be 0)
// per_ray (optional, 4 per ray): internal pops base, all pops base, internal steps with skip
// (skipped internal nodes still cost their step), all steps with skip (skipped nodes included)
void skip_sim_run(const float* nmin, const float* nmax, const int32_t* co, const int32_t* oo, const int32_t* cnt,
                  const int32_t* idx, int32_t n, const float* sph, const int32_t* sum_ids, const int8_t* sum_n, int K,
                  int cache, const float* rays /* 6 per ray */, int64_t nrays, int64_t* stats, int32_t* per_ray) {
    std::vector<int32_t> stk(512);
    std::vector<float> stt(512);
    for (int64_t r = 0; r < nrays; ++r) {
        const V3 o = {rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]};
        const V3 d = {rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]};
        const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        stats[0] += 1;
        float t0, t1;
        if (!ray_box(o, inv, nmin, nmax, t0, t1)) continue;
        int ord[8];
        order_for(d, ord);
        // two walks in lockstep of logic: A = reference (counts), B = with skips (must agree)
        float res[2] = {0, 0};
        bool rhit[2] = {false, false};
        for (int pass = 0; pass < 2; ++pass) {
            const bool skip = pass == 1;
            int32_t cid[8];
            float ce[8];
            int cn = 0;  // LRU: most recent at the end
            auto cache_find = [&](int32_t s) { for (int j = 0; j < cn; ++j) if (cid[j] == s) return j; return -1; };
            auto cache_put = [&](int32_t s, float e) {
                int j = cache_find(s);
                if (j >= 0) { for (int q = j; q + 1 < cn; ++q) { cid[q] = cid[q + 1]; ce[q] = ce[q + 1]; } --cn; }
                if (cn == cache) { for (int q = 0; q + 1 < cn; ++q) { cid[q] = cid[q + 1]; ce[q] = ce[q + 1]; } --cn; }
                if (cache > 0) { cid[cn] = s; ce[cn] = e; ++cn; }
            };
            int sp = 0;
            stk[0] = 0;
            stt[0] = 0.001f;
            float closest = 3.402823466e+38f;
            bool hit = false;
            int64_t pops = 0, ipops = 0, lpops = 0, tests = 0, skipped = 0, iskip = 0, askip = 0;
            while (sp >= 0) {
                const int32_t ni = stk[sp];
                const float ntmin = stt[sp];
                --sp;
                if (skip && sum_n[ni] <= K && sum_n[ni] > 0) {  // subtree of known, all-rejected spheres?
                    bool all = true;
                    for (int j = 0; j < sum_n[ni] && all; ++j) {
                        const int q = cache_find(sum_ids[(int64_t)ni * K + j]);
                        all = q >= 0 && ce[q] <= ntmin;
                    }
                    if (all) {
                        ++askip;
                        if (co[ni] != -1) ++iskip;
                        continue;
                    }
                }
                ++pops;
                if (co[ni] == -1) {
                    ++lpops;
                    for (int j = 0; j < cnt[ni]; ++j) {
                        const int32_t s = idx[oo[ni] + j];
                        if (skip) {
                            const int q = cache_find(s);
                            if (q >= 0 && ce[q] <= ntmin) { ++skipped; continue; }
                        }
                        ++tests;
                        float t;
                        if (sphere_hit(o, d, sph + 4 * s, ntmin, closest, t)) { closest = t; hit = true; sp = -1; }
                        else if (skip) cache_put(s, ntmin);
                    }
                } else {
                    ++ipops;
                    for (int i = 7; i >= 0; --i) {
                        const int64_t c = (int64_t)co[ni] + ord[i];
                        if (c >= n) continue;
                        float cmin, cmax;
                        if (!ray_box(o, inv, nmin + 3 * c, nmax + 3 * c, cmin, cmax) || cmax < ntmin || cmin > closest ||
                            (co[c] == -1 && oo[c] == -1))
                            continue;
                        if (sp < 510) { ++sp; stk[sp] = (int32_t)c; stt[sp] = fmaxr(cmin, ntmin); }
                    }
                }
            }
            res[pass] = closest;
            rhit[pass] = hit;
            if (per_ray) {
                if (!skip) { per_ray[4 * r] = (int32_t)ipops; per_ray[4 * r + 1] = (int32_t)pops; }
                else { per_ray[4 * r + 2] = (int32_t)(ipops + iskip); per_ray[4 * r + 3] = (int32_t)(pops + askip); }
            }
            if (!skip) {
                stats[1] += pops; stats[2] += ipops; stats[3] += lpops; stats[4] += tests; stats[8] += hit;
            } else {
                stats[5] += skipped;
                stats[7] += tests;
                stats[9] += pops;  // pops with both skips
            }
        }
        if (res[0] != res[1] || rhit[0] != rhit[1]) stats[10] += 1;  // must never happen
    }
}
// Push-time variant: an internal node does not push a leaf child that holds exactly one
// sphere s when the lane's rejection cache (the last `cache` rejected spheres, LRU) has s with
// e <= the child's pushed tmin -- the child is never popped.  A parent can name at most
// `kids_k` distinct such spheres (the record's budget); others are pushed as usual.
// stats: [0] rays, [1] pops (reference), [2] pops with push skips, [3] leaf children skipped,
// [4] sphere tests with skips, [5] rays whose result differs (must be 0)
// per_ray (2 per ray): pops reference, pops with skips
static int kids_k_parent = 0;
void skip_sim_push_parent(int v) { kids_k_parent = v; }
// Subtree mode: a child also qualifies when its whole subtree holds one distinct sphere
// (skip_sim_summaries with K >= 1); null = leaf children only.
static const int32_t* g_sum_ids = nullptr;
static const int8_t* g_sum_n = nullptr;
static int g_sum_k = 1;
void skip_sim_push_subtree(const int32_t* sum_ids, const int8_t* sum_n, int K) {
    g_sum_ids = sum_ids;
    g_sum_n = sum_n;
    g_sum_k = K;
}
void skip_sim_push(const float* nmin, const float* nmax, const int32_t* co, const int32_t* oo, const int32_t* cnt,
                   const int32_t* idx, int32_t n, const float* sph, int cache, int kids_k, const float* rays,
                   int64_t nrays, int64_t* stats, int32_t* per_ray) {
    std::vector<int32_t> stk(512);
    std::vector<float> stt(512);
    for (int64_t r = 0; r < nrays; ++r) {
        const V3 o = {rays[6 * r], rays[6 * r + 1], rays[6 * r + 2]};
        const V3 d = {rays[6 * r + 3], rays[6 * r + 4], rays[6 * r + 5]};
        const V3 inv = {1.0f / d.x, 1.0f / d.y, 1.0f / d.z};
        stats[0] += 1;
        float t0, t1;
        if (!ray_box(o, inv, nmin, nmax, t0, t1)) continue;
        int ord[8];
        order_for(d, ord);
        float res[2] = {0, 0};
        bool rhit[2] = {false, false};
        for (int pass = 0; pass < 2; ++pass) {
            const bool skip = pass == 1;
            int32_t cid[8];
            float ce[8];
            int cn = 0;
            auto cache_find = [&](int32_t s) { for (int j = 0; j < cn; ++j) if (cid[j] == s) return j; return -1; };
            auto cache_put = [&](int32_t s, float e) {
                int j = cache_find(s);
                if (j >= 0) { for (int q = j; q + 1 < cn; ++q) { cid[q] = cid[q + 1]; ce[q] = ce[q + 1]; } --cn; }
                if (cn == cache) { for (int q = 0; q + 1 < cn; ++q) { cid[q] = cid[q + 1]; ce[q] = ce[q + 1]; } --cn; }
                if (cache > 0) { cid[cn] = s; ce[cn] = e; ++cn; }
            };
            int sp = 0;
            stk[0] = 0;
            stt[0] = 0.001f;
            float closest = 3.402823466e+38f;
            bool hit = false;
            int64_t pops = 0, kskip = 0, tests = 0;
            while (sp >= 0) {
                const int32_t ni = stk[sp];
                const float ntmin = stt[sp];
                --sp;
                ++pops;
                if (co[ni] == -1) {
                    for (int j = 0; j < cnt[ni]; ++j) {
                        const int32_t s = idx[oo[ni] + j];
                        ++tests;
                        float t;
                        if (sphere_hit(o, d, sph + 4 * s, ntmin, closest, t)) { closest = t; hit = true; sp = -1; }
                        else if (skip) cache_put(s, ntmin);
                    }
                } else {
                    // distinct one-sphere-leaf spheres among the children (the parent's budget)
                    int32_t ks[8];
                    int kn = 0;
                    auto one = [&](int64_t c, int32_t& s) {
                        if (co[c] == -1 && cnt[c] == 1) { s = idx[oo[c]]; return true; }
                        if (g_sum_n && co[c] != -1 && g_sum_n[c] == 1) { s = g_sum_ids[c * g_sum_k]; return true; }
                        return false;
                    };
                    for (int i = 0; i < 8; ++i) {
                        const int64_t c = (int64_t)co[ni] + i;
                        int32_t s;
                        if (c >= n || !one(c, s)) continue;
                        bool seen = false;
                        for (int q = 0; q < kn; ++q) seen = seen || ks[q] == s;
                        if (!seen) ks[kn++] = s;
                    }
                    for (int i = 7; i >= 0; --i) {
                        const int64_t c = (int64_t)co[ni] + ord[i];
                        if (c >= n) continue;
                        float cmin, cmax;
                        if (!ray_box(o, inv, nmin + 3 * c, nmax + 3 * c, cmin, cmax) || cmax < ntmin || cmin > closest ||
                            (co[c] == -1 && oo[c] == -1))
                            continue;
                        const float ct = fmaxr(cmin, ntmin);
                        int32_t s1;
                        if (skip && one(c, s1)) {
                            const int32_t s = s1;
                            int pos = -1;
                            for (int q = 0; q < kn; ++q) if (ks[q] == s) pos = q;
                            const int qc = cache_find(s);
                            if (pos >= 0 && pos < kids_k && qc >= 0 && ce[qc] <= (kids_k_parent ? ntmin : ct)) { ++kskip; continue; }
                        }
                        if (sp < 510) { ++sp; stk[sp] = (int32_t)c; stt[sp] = ct; }
                    }
                }
            }
            res[pass] = closest;
            rhit[pass] = hit;
            if (per_ray) per_ray[2 * r + pass] = (int32_t)pops;
            if (!skip) stats[1] += pops;
            else { stats[2] += pops; stats[3] += kskip; stats[4] += tests; }
        }
        if (res[0] != res[1] || rhit[0] != rhit[1]) stats[5] += 1;
    }
}
}
