// tests/cpp/san_check.cpp -- host ASan/UBSan run of the scene stage (scene.cpp: the
// reference's sphere generators), the octree builder (octree.cpp), the layout compilers
// (layout.cpp, via the emulation), the C ABI's host side (host_abi.cpp), the kernel's
// per-pixel code compiled for the host (ort_debug_emulate_render, render_core.h), the group
// partition/assembly (ort_debug_group_emulate) and the oracle (oracle/ort_oracle.c).
// Built by `make san` (every object instrumented, clang's runtime); no GPU is touched.
// Each case renders a small frame through the emulation (compact and explicit layouts) and
// through the oracle and requires identical bits, like tests/test_emulation.py.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "ort_internal.h"

extern "C" {
#include "ort_oracle.h"
}

namespace {

struct Scene {
    std::vector<float> cr, ma, fr;
    int n = 0;
};

struct Tree {
    std::vector<float> mn, mx;
    std::vector<int32_t> co, oo, cnt, idx;
};

int failures = 0;

void check(bool ok, const char* what, const char* name) {
    if (!ok) {
        std::printf("FAIL %s: %s (%s)\n", name, what, ort_last_error(nullptr));
        ++failures;
    }
}

bool build(const Scene& s, int depth, int mspn, Tree& t) {
    ort_octree* o = nullptr;
    if (ort_octree_build(s.cr.data(), s.n, depth, mspn, &o) != ORT_OK) return false;
    int64_t nn = 0, ni = 0;
    double secs = 0;
    ort_octree_sizes(o, &nn, &ni, &secs);
    t.mn.resize(3 * nn);
    t.mx.resize(3 * nn);
    t.co.resize(nn);
    t.oo.resize(nn);
    t.cnt.resize(nn);
    t.idx.resize(ni > 0 ? ni : 1);
    const int rc = ort_octree_export(o, t.mn.data(), t.mx.data(), t.co.data(), t.oo.data(), t.cnt.data(), t.idx.data());
    t.idx.resize(ni);
    ort_octree_free(o);
    return rc == ORT_OK;
}

ort_params camera(int w, int h, int spp, int bounces, int use_octree) {
    ort_params p{};
    p.width = w;
    p.height = h;
    p.num_samples = spp;
    p.max_depth = bounces;
    p.use_octree = use_octree;
    const float pos[3] = {0.0f, 2.5f, -10.0f}, up[3] = {0.0f, 1.0f, 0.0f};
    ort_camera_view(pos, up, -90.0f, 0.0f, p.view);
    std::memcpy(p.camera_position, pos, sizeof pos);
    p.camera_zoom = 45.0f;
    return p;
}

void render_case(const char* name, const Scene& s, int depth, int mspn, int w, int h, int spp, int bounces) {
    Tree t;
    if (!build(s, depth, mspn, t)) {
        check(false, "octree build", name);
        return;
    }
    const int nn = (int)t.co.size();
    const size_t px = (size_t)w * h;
    for (int use_octree = 1; use_octree >= 0; --use_octree) {
        const ort_params p = camera(w, h, spp, bounces, use_octree);
        oracle_scene os{s.cr.data(), s.ma.data(), s.fr.data(), s.n, t.mn.data(), t.mx.data(), t.co.data(),
                        t.oo.data(), t.cnt.data(), nn, t.idx.data(), (long long)t.idx.size()};
        oracle_params op;
        std::memcpy(&op, &p, sizeof op);
        std::vector<float> ref(3 * px);
        uint64_t rc[ORACLE_COUNT_N] = {0};
        check(oracle_render(&os, &op, 0, 0, w, h, 0, 0, ref.data(), rc, 1) == 0, "oracle render", name);
        const ort_tile tile{0, w, 0, h, 0, 0};
        for (int layout = 0; layout < (use_octree ? 2 : 1); ++layout) {
            std::vector<float> out(3 * px, -1.0f);
            uint64_t cnt[ORT_COUNT_N] = {0};
            const int e = ort_debug_emulate_render(s.cr.data(), s.ma.data(), s.fr.data(), s.n, t.mn.data(), t.mx.data(),
                                                   t.co.data(), t.oo.data(), t.cnt.data(), nn, t.idx.data(),
                                                   (int64_t)t.idx.size(), layout, &p, &tile, out.data(), cnt);
            check(e == ORT_OK, "emulated render", name);
            check(std::memcmp(out.data(), ref.data(), 4 * out.size()) == 0, "emulation != oracle bits", name);
            for (int k = 0; k < ORT_COUNT_N; ++k) check(cnt[k] == rc[k], "reference-walk work counters", name);
        }
        if (use_octree) {  // 3 band tiles, in-memory transport, assembled by the group's row map
            std::vector<float> g(3 * px, -1.0f);
            check(ort_debug_group_emulate(s.cr.data(), s.ma.data(), s.fr.data(), s.n, t.mn.data(), t.mx.data(),
                                          t.co.data(), t.oo.data(), t.cnt.data(), nn, t.idx.data(),
                                          (int64_t)t.idx.size(), 3, &p, g.data()) == ORT_OK,
                  "group emulation", name);
            check(std::memcmp(g.data(), ref.data(), 4 * g.size()) == 0, "group frame != oracle bits", name);
        }
    }
    std::printf("ok %s: %d nodes, %zu indices\n", name, nn, t.idx.size());
}

Scene random_scene(int n, uint32_t seed) {
    Scene s;
    s.n = n;
    s.cr.resize(4 * (size_t)n + 4);
    s.ma.resize(4 * (size_t)n + 4);
    s.fr.resize(4 * (size_t)n + 4);
    if (ort_scene_random(n, seed, s.cr.data(), s.ma.data(), s.fr.data()) != ORT_OK) ++failures;
    return s;
}

}  // namespace

int main() {
    render_case("c1 100 spheres d4 m0, 2 spp 3 bounces", random_scene(100, 42), 4, 0, 40, 30, 2, 3);
    render_case("1000 spheres d5 m1", random_scene(1000, 7), 5, 1, 48, 27, 1, 4);
    render_case("300 spheres d3 m2", random_scene(300, 3), 3, 2, 32, 24, 1, 2);
    render_case("depth 0", random_scene(50, 1), 0, 0, 24, 16, 1, 2);
    render_case("negative maxSpheresPerNode", random_scene(64, 9), 6, -1, 24, 16, 1, 2);
    render_case("depth 9 (96-bit walk)", random_scene(2000, 5), 9, 1, 32, 18, 1, 3);
    {
        Scene s;
        int32_t n = 0;
        ort_scene_prebuilt(nullptr, nullptr, nullptr, &n);
        s.n = n;
        s.cr.resize(4 * n);
        s.ma.resize(4 * n);
        s.fr.resize(4 * n);
        check(ort_scene_prebuilt(s.cr.data(), s.ma.data(), s.fr.data(), &n) == ORT_OK, "prebuilt", "prebuilt");
        render_case("prebuilt scene d5", s, 5, 0, 32, 24, 2, 4);
        check(ort_scene_debug(s.cr.data(), s.ma.data(), s.fr.data(), &n) == ORT_OK && n == 3, "debug scene", "debug");
        s.n = n;
        render_case("debug scene d3 m2", s, 3, 2, 24, 16, 1, 3);
    }
    {  // coincident and tangent spheres
        Scene s = random_scene(40, 11);
        for (int i = 1; i < 10; ++i) std::memcpy(&s.cr[4 * i], &s.cr[0], 4 * sizeof(float));
        s.cr[4 * 10 + 0] = s.cr[0] + 2.0f * s.cr[3];
        s.cr[4 * 10 + 1] = s.cr[1];
        s.cr[4 * 10 + 2] = s.cr[2];
        s.cr[4 * 10 + 3] = s.cr[3];
        render_case("coincident + tangent spheres d5 m1", s, 5, 1, 24, 16, 1, 3);
    }
    {  // error paths of the host ABI
        ort_octree* o = nullptr;
        check(ort_octree_build(nullptr, 0, 3, 0, &o) != ORT_OK, "empty sphere list must fail", "errors");
        check(ort_scene_random(-1, 0, nullptr, nullptr, nullptr) != ORT_OK, "negative count must fail", "errors");
    }
    if (failures) {
        std::printf("san_check: %d FAILURES\n", failures);
        return 1;
    }
    std::printf("san_check: all cases passed\n");
    return 0;
}
