"""Tile frontiers (include/ort.h ORT_OPT_FRONTIER; render_core.h build_frontier): the depth <= 8
camera-ray walks start from each 16x16 tile's list of depth-L nodes instead of walking the top L
levels.  The visits below L and the first hit are the reference walk's own (glsl:312-479, early
exit :336), so every frame must be bit-identical to the plain walk and to the oracle: frontier
depths 1..5 (auto), full frames, band tiles whose 16-row blocks span bands, ragged tiles, a
moving camera (lists rebuilt), several samples and bounces (bounce 0 only uses them), and
maxSpheresPerNode 1 trees (leaves above depth L in the lists)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n,d,m", [(10_000, 6, 0), (10_000, 8, 1), (100_000, 8, 0)])
def test_frontier_frames_identical(ort, oracle, n, d, m):
    from octreeraytracer_amd.scene import DEFAULT_YAW
    s = ort.random_spheres(n, 42)
    t = ort.build_octree(s, d, m)
    W, H = 1280, 720
    shots = [ort.FrameParams.default_camera(W, H), ort.FrameParams.default_camera(W, H),
             ort.FrameParams.default_camera(W, H, yaw=DEFAULT_YAW + 3.0, pitch=-4.0),
             ort.FrameParams.default_camera(W, H, num_samples=2, max_depth=3)]
    tiles = [ort.Tile(0, W, 0, H), ort.Tile(0, W, 0, H), ort.Tile(0, W, 0, H), ort.Tile(0, W, 0, H),
             ort.Tile(0, W, 8, 96, band_height=8, band_stride=40), ort.Tile(301, 517, 123, 211)]
    params = shots + [shots[0], shots[2]]
    got = {}
    for fr in (0, -1, 1, 3, 5):
        if fr > d - 1:
            continue
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_frontier(fr)
            got[fr] = [r.render(p, tl) for p, tl in zip(params, tiles)]
    for fr, frames in got.items():
        for i, (a, b) in enumerate(zip(frames, got[0])):
            assert_same(a, b, f"frontier {fr}, frame {i} vs the plain walk")
    ref = oracle.render(s, t, shots[2], y0=355, rows=10)
    assert_same(got[-1][2][355:365], ref, "frontier walk, turned camera, vs oracle")


def test_frontier_option_range(ort):
    with ort.Renderer(0) as r:
        for bad in (-2, 7):
            with pytest.raises(ort.OrtError):
                r.set_frontier(bad)
        r.set_frontier(0)
        r.set_frontier(-1)
