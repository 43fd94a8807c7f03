"""Parity pinned to the REFERENCE'S OWN shaders, in two steps.

1. Bit for bit.  GLSL leaves the precision of its builtins to the implementation.  With the
   oracle's canonical builtins (include/ort_math.h, as GLSL in oracle/glsl_canonical_builtins.glsl)
   in place of llvmpipe's, the reference's unmodified shaders produce frames BIT-IDENTICAL to the
   oracle's -- and so to the HIP kernels' -- on every case of tests/golden/glsl/canonical.json:
   C1, the DEBUG scene, M=1, C2, the whole 1920x1080 C2 and 3840x2160 C3 bench frames, brute force at 4 bounces,
   the prebuilt scene at 4 samples x 8 bounces, C2 at 2 x 4 and (1920x1080) 4 x 8, depth-9/10
   M=1 trees with bounces (the HIP deep kernels), the sphere-root edge cases, moved camera
   positions (the DEBUG pose, inside and above the field) and zooms 1-30, and the reference's own
   configurations (config.h's default 800x600 16 x 8, stats.csv:114, stats_maxspheres0.csv:68).
   Only SHA-256s are stored.

2. Within GLSL's tolerance, with llvmpipe's own builtins: tests/golden/glsl/*.npz are frames of
/root/reference/shaders/{vertex_shader,octree_fragment_shader}.glsl run unmodified by a real GLSL
4.30 implementation, the image's Mesa 23.2 llvmpipe (oracle/glsl_run.c, a headless DRI swrast
loader; tools/make_glsl_golden.py made them), on this repo's seeded scenes and builder trees
(byte-identical to the reference builder's on every pinned tree).  Here the CPU oracle is
checked against them; tests/test_gpu_parity.py checks the HIP kernels the same way.

Tolerances.  GLSL leaves sqrt, division, pow, sin and cos a few ULP of freedom and llvmpipe
uses its own approximations where the oracle takes the canonical choices of SURVEY Appendix
A, so frames agree to rounding, not bit for bit:
  * one traversal per pixel (maxDepth 1): at least 99.99 % of pixels within 1e-6 (in practice
    every pixel but a handful per frame), and every pixel off by more than 1e-3 sits on a
    sphere silhouette in one of the two frames (a 4-neighbour differs by > 0.02; a sphere
    smaller than a pixel is a silhouette of one pixel): a grazing ray whose hit a rounding
    difference flips;
  * bounced paths: the rounding differences of each scattered direction (sin/cos/pow) are
    amplified bounce by bounce, so the share of pixels within 1e-4 falls with maxDepth
    (C2 spp 2: 1.0 / 0.9955 / 0.984 / 0.969 / 0.951 at maxDepth 1 / 2 / 3 / 4 / 6); each case
    asserts its measured share less a small margin, and the median difference stays at the
    rounding level (<= 1e-6) -- a wrong formula in the oracle's bounce code would move most
    pixels, not a few percent."""
import json
from pathlib import Path

import numpy as np
import pytest

GOLD = Path(__file__).resolve().parent / "golden" / "glsl"
CASES = sorted(p.stem for p in GOLD.glob("*.npz"))

# bounced cases: minimum share of pixels within 1e-4 of the GLSL frame (measured less ~0.5 %)
BOUNCE_MIN_1E4 = {"brute_d4": 0.992, "prebuilt_spp4_d8": 0.994, "c2_spp2_d4": 0.964}


def load(name):
    z = np.load(GOLD / f"{name}.npz")
    return z["rgb"], json.loads(str(z["meta"]))


def inputs(ort, c):
    from octreeraytracer_amd.scene import DEFAULT_CAMERA_POSITION, DEFAULT_PITCH, DEFAULT_YAW, DEFAULT_ZOOM
    if c["scene"] == "random":
        s = ort.random_spheres(c["n"], 42)
    elif c["scene"] == "prebuilt":
        s = ort.prebuilt_spheres()
    elif c["scene"] == "extreme":
        from test_emulation import extreme_root_scene
        s = extreme_root_scene(ort)
    else:
        s = ort.debug_spheres()
    t = ort.build_octree(s, c["depth"], c["m"])
    # the camera: yaw/pitch offsets from main.cpp's camera; position and zoom when the case names them
    p = ort.FrameParams.default_camera(c["W"], c["H"], yaw=DEFAULT_YAW + c["dyaw"], pitch=DEFAULT_PITCH + c["dpitch"],
                                       num_samples=c["spp"], max_depth=c["md"], use_octree=c["oct"],
                                       position=tuple(c.get("pos", DEFAULT_CAMERA_POSITION)),
                                       zoom=c.get("zoom", DEFAULT_ZOOM))
    return s, t, p


def check_against_glsl(img, ref, meta, what):
    """img (H, W, 3) float32 against the GLSL frame ref under the tolerances above."""
    assert img.shape == ref.shape, what
    d = np.abs(img.astype(np.float64) - ref.astype(np.float64)).max(-1)
    assert np.isfinite(img).all(), what
    assert float(np.median(d)) <= 1e-6, f"{what}: median |diff| {np.median(d)}"
    if meta["md"] == 1:
        assert np.mean(d <= 1e-6) >= 0.9999, f"{what}: {np.mean(d <= 1e-6):.6f} of pixels within 1e-6"
        nbs = []
        for f in (ref, img):  # a silhouette in either frame (a sub-pixel sphere only one of them hits)
            pad = np.pad(f, ((1, 1), (1, 1), (0, 0)), mode="edge")
            nbs += [np.abs(pad[1:-1, 2:] - f), np.abs(pad[1:-1, :-2] - f)]
            if "rows" not in meta:  # (a fixture of separate rows: horizontal neighbours only)
                nbs += [np.abs(pad[2:, 1:-1] - f), np.abs(pad[:-2, 1:-1] - f)]
        nb = np.stack(nbs).max(axis=(0, 3))
        off = d > 1e-3
        assert not (off & (nb <= 0.02)).any(), f"{what}: {int((off & (nb <= 0.02)).sum())} off-silhouette pixels > 1e-3"
    else:
        share = float(np.mean(d <= 1e-4))
        assert share >= BOUNCE_MIN_1E4[meta["name"]], f"{what}: {share:.5f} of pixels within 1e-4"
    return d


def test_fixtures_are_reference_shader_frames():
    assert len(CASES) >= 9
    for name in CASES:
        rgb, meta = load(name)
        assert meta["name"] == name and "llvmpipe" in meta["renderer"] and rgb.dtype == np.float32
        assert rgb.shape == (len(meta["rows"]) if "rows" in meta else meta["H"], meta["W"], 3)
        assert "octree_fragment_shader.glsl" in meta["shaders"]


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_shader(ort, oracle, name):
    ref, meta = load(name)
    s, t, p = inputs(ort, meta)
    assert (t.n_nodes, t.n_indices) == (meta["n_nodes"], meta["n_indices"])
    tree = t if meta["oct"] else None
    if "rows" in meta:  # the fixture's rows of a large frame
        img = np.concatenate([oracle.render(s, tree, p, y0=r, rows=1) for r in meta["rows"]])
    else:
        img = oracle.render(s, tree, p)
    check_against_glsl(img, ref, meta, f"oracle vs GLSL {name}")


CANON = json.loads((GOLD / "canonical.json").read_text())
PRELUDE = Path(__file__).resolve().parents[1] / "oracle" / "glsl_canonical_builtins.glsl"


def frame_sha(img):
    import hashlib
    return hashlib.sha256(np.ascontiguousarray(img, np.float32).tobytes()).hexdigest()


def test_canonical_prelude_is_ort_math():
    """The committed prelude is include/ort_math.h's canonical builtins, as generated now."""
    import hashlib
    import sys
    sys.path.insert(0, str(PRELUDE.parents[1] / "tools"))
    import glsl_builtins_check as B
    assert B.prelude() == PRELUDE.read_text()
    assert hashlib.sha256(PRELUDE.read_bytes()).hexdigest() == CANON["prelude_sha256"]
    assert "llvmpipe" in CANON["renderer"] and len(CANON["cases"]) >= 28


@pytest.mark.parametrize("name", sorted(CANON["cases"]))
def test_oracle_bit_exact_to_reference_shader(ort, oracle, name):
    c = CANON["cases"][name]
    s, t, p = inputs(ort, c)
    assert (t.n_nodes, t.n_indices) == (c["n_nodes"], c["n_indices"])
    img = oracle.render(s, t if c["oct"] else None, p)
    assert frame_sha(img) == c["sha256"], f"{name}: the oracle's frame is not the reference shader's"


RUNNER = Path(__file__).resolve().parents[1] / "oracle" / "_ref" / "glsl_run"
SHADERS = Path("/root/reference/shaders")


@pytest.mark.skipif(not (RUNNER.exists() and SHADERS.exists()), reason="needs oracle/_ref/glsl_run and /root/reference")
@pytest.mark.parametrize("name", ["c1", "debug", "brute_d4"])
def test_fixtures_regenerate_bit_for_bit(name):
    """The fixtures are what the reference's shaders give now (llvmpipe is deterministic)."""
    import sys
    sys.path.insert(0, str(RUNNER.parents[2] / "tools"))
    import make_glsl_golden as M
    ref, meta = load(name)
    img, renderer = M.run_glsl(*M.case_inputs(M.CASES[name]))
    assert renderer == meta["renderer"]
    assert np.array_equal(img.view(np.uint32), ref.view(np.uint32))


@pytest.mark.skipif(not (RUNNER.exists() and SHADERS.exists()), reason="needs oracle/_ref/glsl_run and /root/reference")
@pytest.mark.parametrize("name", ["c1", "prebuilt_spp4_d8", "c2_spp2_d4", "m8_d7_odd_b2", "debug_pose", "c2tree_zoom1",
                                  "config_default"])
def test_canonical_hashes_regenerate(name):
    """The canonical-builtin hashes are what the reference's shaders give now."""
    import sys
    sys.path.insert(0, str(RUNNER.parents[2] / "tools"))
    import make_glsl_golden as M
    img, _ = M.run_glsl(*M.case_inputs(CANON["cases"][name]), prelude=PRELUDE)
    assert frame_sha(img) == CANON["cases"][name]["sha256"]


@pytest.mark.skipif(not (RUNNER.exists() and SHADERS.exists()), reason="needs oracle/_ref/glsl_run and /root/reference")
def test_interpolated_pixel_centre_is_implementation_defined():
    """Why the canonical prelude reads gl_FragCoord: at 333x177 llvmpipe's interpolated FragCoord
    varying misses the exact pixel centre by an ulp on part of the frame, which reseeds those
    pixels' RNG; with the builtins alone canonical (no //@replace line) the frame is not the
    oracle's, with the exact centre it is (canonical.json)."""
    import sys
    import tempfile
    sys.path.insert(0, str(RUNNER.parents[2] / "tools"))
    import make_glsl_golden as M
    c = CANON["cases"]["m8_d7_odd_b2"]
    text = PRELUDE.read_text()
    assert text.startswith("//@replace in vec2 FragCoord;\t#define FragCoord gl_FragCoord\n")
    with tempfile.TemporaryDirectory() as d:
        Path(f"{d}/pre.glsl").write_text(text.split("\n", 1)[1])  # the builtins without the replacement
        img, _ = M.run_glsl(*M.case_inputs(c), prelude=f"{d}/pre.glsl")
    assert frame_sha(img) != c["sha256"]
