"""Cost order (include/ort.h ORT_OPT_COST_ORDER): the camera-ray trace deals each 16x16 tile's
pixels to its waves by the walk steps their rays took in the previous frame.  Only which lane
walks which pixel changes, so every frame -- the first (tile order), later ones (ordered by
exact costs), after a camera move (stale costs), after a shape change (costs cleared) -- must
be bit-identical to the fixed-block order, and to the oracle (reference: one invocation per
pixel, glsl:597-633, whatever the invocation order)."""
import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


def _frames(ort, r, s, t, params, tiles):
    out = []
    for p, tile in zip(params, tiles):
        out.append(r.render(p, tile))
    return out


@pytest.mark.parametrize("ns,md", [(1, 1), (2, 3)])
def test_cost_order_frames_match_block_order(ort, oracle, scene_c2, ns, md):
    """C2 scene at 640x360: a static camera (frames 1-2), a moved camera (3), a band tile (4,
    a new shape: costs cleared), the full frame again (5).  Cost order on vs off: bit-exact."""
    from octreeraytracer_amd.scene import DEFAULT_YAW, DEFAULT_PITCH
    s, t = scene_c2
    W, H = 640, 360
    p0 = ort.FrameParams.default_camera(W, H, num_samples=ns, max_depth=md)
    p1 = ort.FrameParams.default_camera(W, H, num_samples=ns, max_depth=md, yaw=DEFAULT_YAW + 4.0,
                                        pitch=DEFAULT_PITCH - 2.0)
    full = ort.Tile(0, W, 0, H)
    band = ort.Tile(0, W, 8, 64, band_height=8, band_stride=32)
    params = [p0, p0, p1, p0, p0]
    tiles = [full, full, full, band, full]
    got = {}
    for on in (1, 0):
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            r.set_cost_order(on)
            got[on] = _frames(ort, r, s, t, params, tiles)
    for i, (a, b) in enumerate(zip(got[1], got[0])):
        assert_same(a, b, f"frame {i}: cost order vs block order")
    ref = oracle.render(s, t, p1, 0, 200, W, 16, threads=0)
    assert_same(got[1][2][200:216], ref, "moved camera, stale costs vs oracle")


def test_cost_order_deep_tree(ort, oracle):
    """Depth 9 (the 96-bit-mask camera kernel, ort_trace_compact_deep, with shading fused into
    bounce 0 of a multi-bounce frame): two frames with cost order, bit-exact vs block order and
    the oracle."""
    s = ort.random_spheres(20000, 42)
    t = ort.build_octree(s, 9, 0)
    W, H = 480, 270
    p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=3)
    got = {}
    for on in (1, 0):
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            r.set_cost_order(on)
            got[on] = [r.render(p) for _ in range(2)]
    assert_same(got[1][1], got[0][1], "depth 9, second frame: cost order vs block order")
    assert_same(got[1][0], got[0][0], "depth 9, first frame")
    ref = oracle.render(s, t, p, 0, 100, W, 8, threads=0)
    assert_same(got[1][1][100:108], ref, "depth 9 cost order vs oracle")


def test_cost_order_option_range(ort):
    with ort.Renderer(0) as r:
        with pytest.raises(ort.OrtError):
            r.set_cost_order(2)
        r.set_cost_order(0)
        r.set_cost_order(1)


@pytest.mark.parametrize("depth", [6, 9])
def test_heavy_first_frames_match_coherence_order(ort, oracle, depth):
    """Heavy first (ORT_OPT_HEAVY_FIRST): a 4-bounce frame rendered three times (the second and
    third sort each bounce list with the previous frame's walk steps) at thresholds 0 (off), 8
    (most walks heavy) and 48, on the depth <= 8 and the depth 9-10 persistent kernel: every
    frame bit-identical, and to the oracle."""
    s = ort.random_spheres(20000, 42)
    t = ort.build_octree(s, depth, 0)
    W, H = 480, 270
    p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=4)
    got = {}
    for thr in (0, 8, 48):
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            r.set_heavy_first(thr)
            got[thr] = [r.render(p) for _ in range(3)]
    for thr in (8, 48):
        for i in range(3):
            assert_same(got[thr][i], got[0][i], f"depth {depth}, heavy >= {thr}, frame {i} vs coherence order")
    ref = oracle.render(s, t, p, 0, 120, W, 8, threads=0)
    assert_same(got[48][2][120:128], ref, f"depth {depth} heavy first vs oracle")


@pytest.mark.parametrize("depth", [8, 10])
def test_heavy_first_moving_camera(ort, oracle, depth):
    """Heavy first with the camera turning: a moved frame sorts its bounce lists by classes from
    the rays themselves (the root-box exit distance, geo_class_bits), a frame of an unmoved
    camera by last frame's walk steps -- the frames stay bit-identical to coherence order and to
    the oracle, on the depth <= 8 and the depth 9-10 persistent kernel."""
    from octreeraytracer_amd.scene import DEFAULT_YAW
    s = ort.random_spheres(20000, 42)
    t = ort.build_octree(s, depth, 1)
    W, H = 320, 180
    ps = [ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=4, yaw=DEFAULT_YAW + 0.5 * j)
          for j in (0, 0, 1, 2, 2)]  # static, moved, moved, static
    got = {}
    # (48, 0): heavy first with the cost order off -- the camera-moved test that gates the
    # bounce classes must not depend on the cost order (it did until round 6)
    for thr, cost_order in ((0, 1), (48, 1), (48, 0)):
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            r.set_cost_order(cost_order)
            r.set_heavy_first(thr)
            got[thr, cost_order] = [r.render(p) for p in ps]
    for i in range(len(ps)):
        assert_same(got[48, 1][i], got[0, 1][i], f"depth {depth}, frame {i}: heavy first vs coherence order")
        assert_same(got[48, 0][i], got[0, 1][i], f"depth {depth}, frame {i}: heavy first, cost order off")
    got[48] = got[48, 1]
    ref = oracle.render(s, t, ps[3], 0, 80, W, 8, threads=0)
    assert_same(got[48][3][80:88], ref, f"depth {depth}, moved frame vs oracle")


def test_heavy_first_option_range(ort):
    with ort.Renderer(0) as r:
        with pytest.raises(ort.OrtError):
            r.set_heavy_first(-1)
        with pytest.raises(ort.OrtError):
            r.set_heavy_first(70000)
        r.set_heavy_first(0)
        r.set_heavy_first(384)


def _plain(r):
    """The per-tile kernel alone: no heavy priority, split walks or tile pairs (the defaults turn
    them on by tile size)."""
    r.set_heavy_prio(0)
    r.set_split_heavy(0)
    r.set_tile_pairs(0)


@pytest.mark.parametrize("split,level,prio,md", [(40, 0, 150, 1), (20, 1, 0, 1), (60, 2, 60, 1), (30, 5, 0, 1),
                                                 (40, 0, 150, 3), (25, 2, 0, 4)])
def test_split_heavy_frames_match(ort, oracle, scene_c2, split, level, prio, md):
    """Split walks of the heavy camera rays (ORT_OPT_SPLIT_HEAVY: 8 lanes per ray on the second
    stream, subtrees of one level dealt round robin) and heavy-wave priority (ORT_OPT_HEAVY_PRIO):
    low thresholds make many rays heavy (up to the 4096-ray cap, the rest walked by the tiles).
    Static camera, moved camera (last frame's costs), a band tile, every split level: bit-exact
    vs the plain per-tile kernel and the oracle."""
    from octreeraytracer_amd.scene import DEFAULT_YAW
    s, t = scene_c2
    W, H = 960, 540
    p0 = ort.FrameParams.default_camera(W, H, max_depth=md)
    p1 = ort.FrameParams.default_camera(W, H, yaw=DEFAULT_YAW + 3.0, max_depth=md)
    full = ort.Tile(0, W, 0, H)
    band = ort.Tile(0, W, 0, 136, band_height=16, band_stride=128)
    params = [p0, p0, p1, p1, p0, p0, p0]
    tiles = [full, full, full, full, band, band, full]
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        _plain(r)
        want = _frames(ort, r, s, t, params, tiles)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        r.set_split_heavy(split)
        r.set_split_level(level)
        r.set_heavy_prio(prio)
        got = _frames(ort, r, s, t, params, tiles)
    for i, (a, b) in enumerate(zip(got, want)):
        assert_same(a, b, f"frame {i}: split {split} level {level} vs plain")
    ref = oracle.render(s, t, p1, 0, 300, W, 16)
    assert_same(got[3][300:316], ref, "moved camera, split walks vs oracle")


def test_split_heavy_deep_tree(ort, oracle):
    """The split walk over 96-bit masks (depth 9): bit-exact vs the plain kernel and the oracle."""
    s = ort.random_spheres(20000, 42)
    t = ort.build_octree(s, 9, 1)
    W, H = 480, 270
    p = ort.FrameParams.default_camera(W, H)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        _plain(r)
        want = [r.render(p) for _ in range(2)]
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        r.set_split_heavy(30)
        got = [r.render(p) for _ in range(3)]
    for g in got:
        assert_same(g, want[1], "deep split")
    assert_same(got[2][100:116], oracle.render(s, t, p, 0, 100, W, 16), "deep split vs oracle")


@pytest.mark.parametrize("ns,md,depth", [(1, 1, 6), (1, 3, 6), (2, 2, 6), (1, 1, 9), (1, 3, 9)])
def test_tile_pairs_frames_match(ort, oracle, ns, md, depth):
    """Tile pairs (ORT_OPT_TILE_PAIRS: a camera-ray workgroup renders two tiles, each wave a heavy
    and a light 64-pixel block by last frame's steps; every kernel of the frame maps slots to
    pixels through the pair grid): an odd tile count per row (a hole tile), band tiles, a moved
    camera, several samples and bounces, depth 6 and 9 -- bit-exact vs one tile per workgroup."""
    from octreeraytracer_amd.scene import DEFAULT_YAW
    s = ort.random_spheres(10_000 if depth == 6 else 20_000, 42)
    t = ort.build_octree(s, depth, 0 if depth == 6 else 1)
    W, H = 720, 400  # 45 tiles per row: the last pair holds a hole
    p0 = ort.FrameParams.default_camera(W, H, num_samples=ns, max_depth=md)
    p1 = ort.FrameParams.default_camera(W, H, num_samples=ns, max_depth=md, yaw=DEFAULT_YAW + 3.0)
    full = ort.Tile(0, W, 0, H)
    band = ort.Tile(0, W, 0, 104, band_height=16, band_stride=64)
    params = [p0, p0, p1, p0, p0]
    tiles = [full, full, full, band, band]
    got = {}
    for on in (1, 0):
        with ort.Renderer(0) as r:
            r.upload(s, t)
            r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            r.set_tile_pairs(on)
            r.set_heavy_prio(100)
            got[on] = _frames(ort, r, s, t, params, tiles)
    for i, (a, b) in enumerate(zip(got[1], got[0])):
        assert_same(a, b, f"frame {i}: tile pairs vs one tile per workgroup")
    assert_same(got[1][2][200:216], oracle.render(s, t, p1, 0, 200, W, 16), "tile pairs, moved camera vs oracle")


def test_split_heavy_queued_list_across_other_frames(ort, oracle, scene_c2):
    """The next frame's heavy list is queued on the second stream at the end of a split frame; a
    frame without split walks (another shape, a larger tile that regrows the buffers, the counting
    render, split off) in between must not let a stale list through: bit-exact vs the plain kernel."""
    s, t = scene_c2
    W, H = 960, 540
    p = ort.FrameParams.default_camera(W, H)
    band = ort.Tile(0, W, 0, 136, band_height=16, band_stride=128)
    full = ort.Tile(0, W, 0, H)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        _plain(r)
        want_band, want_full = r.render(p, band), r.render(p, full)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        _plain(r)
        r.set_split_heavy(30)
        got = [r.render(p, band) for _ in range(3)]
        r.set_split_heavy(0)
        got.append(r.render(p, band))            # same shape, no split walks
        r.set_split_heavy(30)
        got += [r.render(p, band) for _ in range(2)]
        got_full = r.render(p, full)             # another shape (larger: the buffers regrow)
        r.count_traffic(p, band)                 # the counting render
        got += [r.render(p, band) for _ in range(2)]
        got_full2 = r.render(p, full)
    for i, g in enumerate(got):
        assert_same(g, want_band, f"band frame {i}")
    assert_same(got_full, want_full, "full frame")
    assert_same(got_full2, want_full, "full frame again")
    assert_same(got[-1][0:16], oracle.render(s, t, p, 0, 0, W, 16), "band rows 0-15 vs oracle")

