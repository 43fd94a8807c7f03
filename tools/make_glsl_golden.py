"""Generate tests/golden/glsl/*.npz: frames of the REFERENCE'S OWN shaders
(/root/reference/shaders/vertex_shader.glsl + octree_fragment_shader.glsl) executed by a real
GLSL 4.30 implementation, the image's Mesa llvmpipe, through oracle/_ref/glsl_run
(oracle/glsl_run.c: a headless DRI swrast loader; `make -C oracle glsl`).  Test infrastructure
only: the fixtures pin the CPU oracle's pixel arithmetic (tests/test_glsl_parity.py) and, through
it, the HIP kernels (tests/test_gpu_parity.py); nothing here runs on the GPU box.

Inputs are this repo's seeded sphere sets and the octrees of its builder, which is
byte-identical to the reference's own src/octree.cpp on every pinned tree
(tests/golden/manifest.json).  Each fixture holds the frame (float32 RGB, GL row order; the
shader's alpha is 1 everywhere and is checked, then dropped) and the case it was made from.

With --canonical the same shaders run with oracle/glsl_canonical_builtins.glsl inserted after
the fragment shader's #version line (glsl_run's PRELUDE, in memory): the oracle's canonical
builtins (include/ort_math.h) in place of llvmpipe's sin/cos/tan/pow/normalize/dot/length/cross/
reflect/min/max -- GLSL leaves their precision to the implementation, and this is one
implementation of them.  Those frames are stored as SHA-256 only (tests/golden/glsl/
canonical.json): the oracle and the HIP kernels must reproduce them bit for bit.

usage: python tools/make_glsl_golden.py [case ...]
       python tools/make_glsl_golden.py --canonical [case ...]
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd.scene import DEFAULT_CAMERA_POSITION, DEFAULT_PITCH, DEFAULT_YAW, DEFAULT_ZOOM  # noqa: E402

OUT = ROOT / "tests" / "golden" / "glsl"
RUNNER = ROOT / "oracle" / "_ref" / "glsl_run"
SHADERS = Path(os.environ.get("ORT_REF", "/root/reference")) / "shaders"

# name: scene, (n, seed), tree depth, maxSpheresPerNode, frame (W, H, spp, maxDepth, useOctree),
# camera (yaw, pitch offsets from the default camera), kind (primary: one traversal per pixel)
CASES = {
    "c1": dict(scene="random", n=100, depth=4, m=0, W=256, H=256, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "c1_turned": dict(scene="random", n=100, depth=4, m=0, W=192, H=144, spp=1, md=1, oct=1, dyaw=30.0, dpitch=-15.0),
    "debug": dict(scene="debug", n=3, depth=3, m=2, W=160, H=120, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "m1_d6": dict(scene="random", n=2000, depth=6, m=1, W=192, H=108, spp=1, md=1, oct=1, dyaw=-12.0, dpitch=4.0),
    "c2": dict(scene="random", n=10000, depth=6, m=0, W=320, H=180, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "c3": dict(scene="random", n=100000, depth=8, m=0, W=256, H=144, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "brute_d4": dict(scene="random", n=100, depth=4, m=0, W=128, H=96, spp=1, md=4, oct=0, dyaw=0.0, dpitch=0.0),
    "prebuilt_spp4_d8": dict(scene="prebuilt", n=83, depth=5, m=1, W=160, H=120, spp=4, md=8, oct=1, dyaw=0.0,
                             dpitch=0.0),
    "c2_spp2_d4": dict(scene="random", n=10000, depth=6, m=0, W=192, H=108, spp=2, md=4, oct=1, dyaw=20.0,
                       dpitch=-10.0),
    # sphere-root edge cases (tests/test_emulation.py extreme_root_scene): camera inside a sphere,
    # roots near 0, half_b^2 overflow, disc > 2^100.  Primary rays only: bounced off spheres of
    # radius 1e18-1e19 a path is chaotic at float precision (the 0.001 self-intersection bound is far
    # below the hit point's ULP there), and at maxDepth 4 llvmpipe and the oracle agree to 1e-6 on 0.07 % of pixels
    "extreme": dict(scene="extreme", n=7, depth=5, m=0, W=160, H=100, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    # the bench's C3 frame itself (3840x2160, 100k spheres, depth 8); 16 of its rows are kept (the
    # --canonical hashes cover the whole frame: c3_full)
    "c3_full_rows": dict(scene="random", n=100000, depth=8, m=0, W=3840, H=2160, spp=1, md=1, oct=1, dyaw=0.0,
                         dpitch=0.0, rows=[0, 135, 270, 405, 540, 675, 810, 945, 1080, 1215, 1350, 1485, 1620, 1755,
                                           1890, 2159]),
}


# --canonical only (hashes of whole frames): the bench's C2 and C3 frames (bench.py checks its own frame
# against them); C2 at 4 samples and 8 bounces
CANON_EXTRA = {
    "c2_full": dict(scene="random", n=10000, depth=6, m=0, W=1920, H=1080, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "c3_full": dict(scene="random", n=100000, depth=8, m=0, W=3840, H=2160, spp=1, md=1, oct=1, dyaw=0.0, dpitch=0.0),
    "c2_full_spp4_d8": dict(scene="random", n=10000, depth=6, m=0, W=1920, H=1080, spp=4, md=8, oct=1, dyaw=0.0,
                            dpitch=0.0),
    # trees deeper than 8 levels (C5's kind: depth 10, maxSpheresPerNode 1, 4 bounces) take the
    # HIP path's deep kernels (96-bit level masks, the depth 9-10 persistent bounce walk); C5's own
    # 239 M-node tree is too large for llvmpipe, these are not
    "deep_d10_m1_b4": dict(scene="random", n=50000, depth=10, m=1, W=640, H=360, spp=1, md=4, oct=1, dyaw=0.0,
                           dpitch=0.0),
    "deep_d9_m1_spp2_b3": dict(scene="random", n=20000, depth=9, m=1, W=320, H=180, spp=2, md=3, oct=1, dyaw=15.0,
                               dpitch=-6.0),
    # leaves of up to 8 spheres, an odd frame size (partial tiles on both axes), 2 bounces
    "m8_d7_odd_b2": dict(scene="random", n=30000, depth=7, m=8, W=333, H=177, spp=1, md=2, oct=1, dyaw=-25.0,
                         dpitch=8.0),
    # the C3 tree (depth 8) with bounces and samples: the depth <= 8 persistent bounce walk
    "c3tree_spp3_b5": dict(scene="random", n=100000, depth=8, m=0, W=200, H=120, spp=3, md=5, oct=1, dyaw=10.0,
                           dpitch=-20.0),
    # --- camera inputs (round 6): the reference moves Position by WASD (src/opengl/camera.h:70-81)
    # and Zoom by the scroll wheel (camera.h:106-113, clamped to [1, 45]); both reach
    # Camera_initFromViewMatrix (glsl:176-202) as the cameraPosition / cameraZoom uniforms.
    # The DEBUG scene from its own camera (src/main.cpp:31: Position (30, 20, -50)), bounced
    "debug_pose": dict(scene="debug", n=3, depth=3, m=2, W=320, H=240, spp=2, md=4, oct=1, dyaw=0.0, dpitch=0.0,
                       pos=[30.0, 20.0, -50.0]),
    # main.cpp:33's commented "centered" pose (0, 2.5, 0): inside the C3 field
    "c3tree_centered": dict(scene="random", n=100000, depth=8, m=0, W=320, H=180, spp=1, md=3, oct=1, dyaw=0.0,
                            dpitch=0.0, pos=[0.0, 2.5, 0.0]),
    # above the C2 field (half-width 30) at pitch -40 and +40 (the shader looks along -Front:
    # w = -normalize(view row 2), glsl:181, so +40 looks down onto the field, -40 up into the sky)
    "c2tree_above_m40": dict(scene="random", n=10000, depth=6, m=0, W=320, H=180, spp=1, md=2, oct=1, dyaw=0.0,
                             dpitch=-40.0, pos=[5.0, 25.0, -45.0]),
    "c2tree_above_p40": dict(scene="random", n=10000, depth=6, m=0, W=320, H=180, spp=1, md=2, oct=1, dyaw=12.0,
                             dpitch=40.0, pos=[5.0, 25.0, -45.0]),
    # zoom 20 and zoom 1 (the scroll clamp's lower end): narrow fields of view, tan(theta/2) of
    # small arguments
    "c2tree_zoom20": dict(scene="random", n=10000, depth=6, m=0, W=320, H=180, spp=2, md=3, oct=1, dyaw=0.0,
                          dpitch=0.0, zoom=20.0),
    "c2tree_zoom1": dict(scene="random", n=10000, depth=6, m=0, W=320, H=180, spp=1, md=2, oct=1, dyaw=3.0,
                         dpitch=-2.0, zoom=1.0),
    # a moved, turned and zoomed pose together
    "c3tree_moved_zoom30": dict(scene="random", n=100000, depth=8, m=0, W=256, H=192, spp=1, md=2, oct=1,
                                dyaw=-35.0, dpitch=12.0, pos=[-20.0, 6.0, 15.0], zoom=30.0),
    # --- the reference's own configurations
    # src/config.h:10-28 (the default build): 800x600, 100 spheres, depth 3, M=0, 16 spp x 8 bounces
    "config_default": dict(scene="random", n=100, depth=3, m=0, W=800, H=600, spp=16, md=8, oct=1, dyaw=0.0,
                           dpitch=0.0),
    # analysis/stats.csv:114's row: 1000 spheres, depth 5, M=1, 16 x 8, 1920x1080
    "stats114": dict(scene="random", n=1000, depth=5, m=1, W=1920, H=1080, spp=16, md=8, oct=1, dyaw=0.0,
                     dpitch=0.0),
    # analysis/stats_maxspheres0.csv:68's row: 2000 spheres, depth 3, M=0, 4 x 4, 800x600
    "ms0_row68": dict(scene="random", n=2000, depth=3, m=0, W=800, H=600, spp=4, md=4, oct=1, dyaw=0.0,
                      dpitch=0.0),
    # a depth-9 tree subdivided to the bottom (maxSpheresPerNode 0): the deep kernels without C5's
    # one-sphere leaves (at depth 10 such trees pass 2^24 nodes even at 2000 spheres: SURVEY F7,
    # the reference's float offsets then name wrong children)
    "deep_d9_m0_b2": dict(scene="random", n=10000, depth=9, m=0, W=320, H=180, spp=1, md=2, oct=1, dyaw=-8.0,
                          dpitch=3.0),
}
PRELUDE = ROOT / "oracle" / "glsl_canonical_builtins.glsl"


def canonical_cases():
    cc = {k: v for k, v in CASES.items() if "rows" not in v}
    cc.update(CANON_EXTRA)
    return cc


def case_inputs(c):
    if c["scene"] == "random":
        s = ort.random_spheres(c["n"], 42)
    elif c["scene"] == "prebuilt":
        s = ort.prebuilt_spheres()
    elif c["scene"] == "extreme":
        sys.path.insert(0, str(ROOT / "tests"))
        from test_emulation import extreme_root_scene
        s = extreme_root_scene(ort)
    else:
        s = ort.debug_spheres()
    t = ort.build_octree(s, c["depth"], c["m"])
    return s, t, case_params(c)


def case_params(c):
    """The frame of a case: size, samples, bounces and the camera -- yaw/pitch offsets from the
    default camera and, when the case names them, the position and zoom (else main.cpp's)."""
    return ort.FrameParams.default_camera(c["W"], c["H"], yaw=DEFAULT_YAW + c["dyaw"], pitch=DEFAULT_PITCH + c["dpitch"],
                                          num_samples=c["spp"], max_depth=c["md"], use_octree=c["oct"],
                                          position=tuple(c.get("pos", DEFAULT_CAMERA_POSITION)),
                                          zoom=c.get("zoom", DEFAULT_ZOOM))


def write_input(path, s, t, p):
    """glsl_run's input: the header, the frame's uniforms and setupBuffers' seven arrays."""
    c = p.to_c()
    hdr = np.array([c.width, c.height, c.num_samples, c.max_depth, c.use_octree, s.n, t.n_nodes, t.n_indices], np.int32)
    uni = np.array(list(c.view) + list(c.camera_position) + [c.camera_zoom], np.float32)
    # (glm::vec4(node.min, node.childrenOffset): the offsets travel as floats, src/raytracer.cpp:98-99)
    nmin = np.concatenate([t.node_min.astype(np.float32), t.children_offset.astype(np.float32)[:, None]], 1)
    nmax = np.concatenate([t.node_max.astype(np.float32), t.objects_offset.astype(np.float32)[:, None]], 1)
    with open(path, "wb") as f:
        for a in (hdr, uni, s.center_radius.astype(np.float32), s.mat_albedo.astype(np.float32),
                  s.fuzz_ri.astype(np.float32), nmin, nmax, t.object_count.astype(np.int32),
                  t.object_indices.astype(np.int32)):
            f.write(np.ascontiguousarray(a).tobytes())


def run_glsl(s, t, p, timing=None, prelude=None):
    """The frame (H, W, 3) and the renderer line; timing (a dict) gets the draw's wall ms;
    prelude: a GLSL file glsl_run inserts after the fragment shader's #version line."""
    with tempfile.TemporaryDirectory() as d:
        write_input(f"{d}/in.bin", s, t, p)
        cmd = [str(RUNNER), str(SHADERS), f"{d}/in.bin", f"{d}/out.bin"] + ([str(prelude)] if prelude else [])
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise SystemExit(f"glsl_run failed: {r.stderr}")
        img = np.fromfile(f"{d}/out.bin", np.float32).reshape(p.height, p.width, 4)
    if not (img[..., 3] == 1.0).all():
        raise SystemExit("FragColor alpha is not 1 everywhere")
    lines = r.stderr.strip().splitlines()
    if timing is not None:
        timing["draw_ms"] = float(next(x for x in lines if " draw " in x).split()[-2])
    return np.ascontiguousarray(img[..., :3]), next(x for x in lines if "Mesa" in x)


def frame_sha(img):
    return hashlib.sha256(np.ascontiguousarray(img, np.float32).tobytes()).hexdigest()


def canonical(names):
    import glsl_builtins_check as B
    PRELUDE.write_text(B.prelude())
    path = OUT / "canonical.json"
    doc = json.loads(path.read_text()) if path.exists() else {"cases": {}}
    doc["prelude"] = "oracle/glsl_canonical_builtins.glsl"
    doc["prelude_sha256"] = hashlib.sha256(PRELUDE.read_bytes()).hexdigest()
    cc = canonical_cases()
    for name in names or list(cc):
        t0 = time.time()
        s, t, p = case_inputs(cc[name])
        img, renderer = run_glsl(s, t, p, prelude=PRELUDE)
        doc["renderer"] = renderer
        doc["cases"][name] = dict(cc[name], sha256=frame_sha(img), n_nodes=int(t.n_nodes), n_indices=int(t.n_indices))
        print(f"{name}: {p.width}x{p.height} canonical builtins in {time.time() - t0:.1f} s", flush=True)
    path.write_text(json.dumps(doc, indent=1, sort_keys=True) + "\n")


def main():
    if not RUNNER.exists():
        raise SystemExit("build the runner first: make -C oracle glsl")
    OUT.mkdir(parents=True, exist_ok=True)
    if sys.argv[1:2] == ["--canonical"]:
        return canonical(sys.argv[2:])
    names = sys.argv[1:] or list(CASES)
    for name in names:
        c = CASES[name]
        t0 = time.time()
        s, t, p = case_inputs(c)
        img, renderer = run_glsl(s, t, p)
        if "rows" in c:  # a large frame: the listed rows (GL row order) only
            img = np.ascontiguousarray(img[c["rows"]])
        meta = dict(c, name=name, renderer=renderer, shaders="shaders/vertex_shader.glsl + shaders/octree_fragment_shader.glsl",
                    n_nodes=int(t.n_nodes), n_indices=int(t.n_indices))
        np.savez_compressed(OUT / f"{name}.npz", rgb=img, meta=json.dumps(meta))
        print(f"{name}: {p.width}x{p.height} in {time.time() - t0:.1f} s ({renderer})", flush=True)


if __name__ == "__main__":
    main()
