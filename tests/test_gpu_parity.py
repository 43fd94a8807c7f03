"""GPU parity: the gfx950 kernel through the C ABI against the CPU oracle.

Bar: bit-exact (the float32 bits of every pixel equal), which implies the 1e-5 target of
BASELINE.json; the tolerance assertion is kept explicit as well.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

TOL = 1e-5  # BASELINE.json north_star: pixels within 1e-5 of the CPU reference


def assert_same(img, ref, what=""):
    assert img.shape == ref.shape
    diff = np.abs(img.astype(np.float64) - ref.astype(np.float64))
    bad = int((img.view(np.uint32) != ref.view(np.uint32)).any(axis=-1).sum())
    assert float(np.nanmax(diff)) <= TOL, f"{what}: max |diff| {np.nanmax(diff)}"
    assert bad == 0, f"{what}: {bad} pixels not bit-identical"


class pixel_paths:
    """ORT_OPT_PIXEL_PATHS for a block: 0 the per-bounce pipeline (the tests of its options), 1
    whole-pixel paths in one launch; the default (-1, auto) restored after."""

    def __init__(self, renderer, mode):
        self.r, self.mode = renderer, mode

    def __enter__(self):
        self.r.set_pixel_paths(self.mode)
        return self.r

    def __exit__(self, *exc):
        self.r.set_pixel_paths(-1)


@pytest.mark.parametrize("layout", [0, 1])
def test_c1_bit_exact(ort, oracle, renderer, scene_c1, layout):
    s, t = scene_c1
    renderer.set_layout(layout)
    renderer.upload(s, t)
    assert renderer.info()["layout"] == ("compact" if layout == 0 else "explicit")
    p = ort.FrameParams.default_camera(256, 256)
    assert_same(renderer.render(p), oracle.render(s, t, p), f"C1 layout {layout}")
    renderer.set_layout(-1)


@pytest.mark.parametrize("mode", [0, 1])
def test_c1_bounces_and_samples(ort, oracle, renderer, scene_c1, mode):
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(160, 120, num_samples=4, max_depth=8)
    with pixel_paths(renderer, mode):
        assert_same(renderer.render(p), oracle.render(s, t, p), f"C1 spp4 depth8 pixel_paths={mode}")


@pytest.mark.parametrize("mode", [0, 1])
def test_brute_force_mode(ort, oracle, renderer, scene_c1, mode):
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(128, 128, use_octree=0, max_depth=4, num_samples=2)
    with pixel_paths(renderer, mode):
        assert_same(renderer.render(p), oracle.render(s, None, p), f"brute force pixel_paths={mode}")


def test_prebuilt_scene(ort, oracle, renderer):
    s = ort.prebuilt_spheres()
    t = ort.build_octree(s, 5, 1)
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(200, 150, num_samples=2, max_depth=4)
    assert_same(renderer.render(p), oracle.render(s, t, p), "prebuilt")


def test_c2_full_frame(ort, oracle, renderer, scene_c2):
    s, t = scene_c2
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(1920, 1080)
    assert_same(renderer.render(p), oracle.render(s, t, p), "C2 1920x1080")


def test_counters_match_oracle(ort, oracle, renderer, scene_c1):
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(256, 256)
    _, want = oracle.render(s, t, p, counts=True)
    got = renderer.count_traffic(p)
    assert got == want


def test_tiles_and_bands_compose(ort, renderer, scene_c1):
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(200, 136)
    full = renderer.render(p)
    # contiguous sub-tile with odd sizes
    tile = ort.Tile(13, 77, 29, 51)
    sub = renderer.render(p, tile)
    assert np.array_equal(sub, full[29:29 + 51, 13:13 + 77])
    # 16-row bands dealt round-robin to 3 "ranks"
    for rank in range(3):
        nb = -(-136 // 16)
        mine = len(range(rank, nb, 3))
        tile = ort.Tile(0, 200, rank * 16, mine * 16, 16, 48)
        out = renderer.render(p, tile)
        ys = tile.pixel_rows(136)
        for j, y in enumerate(ys):
            if y < 136:
                assert np.array_equal(out[j], full[y]), (rank, j, y)
            else:
                assert not out[j].any()


def test_device_output_and_stream(ort, renderer, scene_c1):
    torch = pytest.importorskip("torch")
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(96, 64)
    host = renderer.render(p)
    dev = torch.empty((64, 96, 3), dtype=torch.float32, device="cuda:0")
    renderer.render(p, out=dev, stream=torch.cuda.current_stream().cuda_stream)  # null stream: synchronous
    torch.cuda.synchronize()
    assert np.array_equal(dev.cpu().numpy(), host)
    assert renderer.last_kernel_ms() > 0
    # stream-ordered on a caller stream: several frames queued back to back, then one sync
    st = torch.cuda.Stream()
    outs = [torch.full((64, 96, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(4)]
    with torch.cuda.stream(st):
        for o in outs:
            renderer.render(p, out=o, stream=st.cuda_stream)
    st.synchronize()
    for o in outs:
        assert np.array_equal(o.cpu().numpy(), host)


def test_frames_in_flight(ort, scene_c1):
    """bench.py --inflight: several contexts, each rendering on its own stream, frames
    overlapping on the GPU (1 and 3 bounces) -- every frame equals the synchronous render."""
    torch = pytest.importorskip("torch")
    s, t = scene_c1
    rs = [ort.Renderer(0) for _ in range(3)]
    try:
        for x in rs:
            x.upload(s, t)
        for md in (1, 3):
            p = ort.FrameParams.default_camera(200, 136, max_depth=md)
            host = rs[0].render(p)
            sts = [torch.cuda.ExternalStream(x.stream_handle()) for x in rs]
            assert all(st.cuda_stream != 0 for st in sts)
            outs = [torch.full((136, 200, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(9)]
            for k, o in enumerate(outs):
                rs[k % 3].render(p, out=o, stream=sts[k % 3].cuda_stream)
            torch.cuda.synchronize()
            for o in outs:
                assert np.array_equal(o.cpu().numpy(), host)
    finally:
        for x in rs:
            x.close()


def test_errors(ort, renderer, scene_c1):
    s, t = scene_c1
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(64, 64)
    with pytest.raises(ort.OrtError):
        renderer.render(p, ort.Tile(60, 10, 0, 4))  # columns outside the frame
    bad = ort.FlatOctree(t.node_min, t.node_max, t.children_offset, t.objects_offset, t.object_count,
                         t.object_indices + 1000)
    with pytest.raises(ort.OrtError):
        renderer.upload(s, bad)
    fresh = ort.Renderer(0)
    with pytest.raises(ort.OrtError):
        fresh.render(p)  # no scene
    fresh.close()


@pytest.mark.parametrize("persistent,exact,refill", [
    (0, False, 16), (0, True, 16), (2, False, 1), (2, False, 8), (2, True, 32), (2, False, 64)])
def test_kernel_variants_identical(ort, oracle, renderer, scene_c2, persistent, exact, refill):
    """Every trace-kernel variant (one ray per lane / persistent bounce walks with refill, fast
    / exact walk) produces the oracle's pixels, also with several samples and bounces."""
    s, t = scene_c2
    renderer.upload(s, t)
    renderer.set_persistent(persistent)
    renderer.set_exact_traversal(exact)
    renderer.set_refill(refill)
    renderer.set_pixel_paths(0)  # the pipeline's kernels (C2's small tree would take whole-pixel paths)
    try:
        p = ort.FrameParams.default_camera(1920, 1080, num_samples=2, max_depth=3)
        tile = ort.Tile(700, 200, 300, 120)
        got = renderer.render(p, tile)
        ref = oracle.render(s, t, p, 700, 300, 200, 120)
        assert_same(got, ref, f"variant persistent={persistent} exact={exact}")
        p1 = ort.FrameParams.default_camera(1920, 1080)
        assert_same(renderer.render(p1, tile), oracle.render(s, t, p1, 700, 300, 200, 120), "primary")
        with pixel_paths(renderer, 1):  # and whole-pixel paths, fast or exact walk
            assert_same(renderer.render(p, tile), ref, f"pixel paths exact={exact}")
    finally:
        renderer.set_persistent(2)  # the default
        renderer.set_exact_traversal(False)
        renderer.set_refill(16)  # the default
        renderer.set_pixel_paths(-1)


def test_removed_options_are_refused(ort, renderer):
    """The retired option codes (ort.h ORT_OPT_IS_RETIRED: packet walk 5, wave queue 7,
    longest-first workgroups 17), every-trace persistent and, in the product library, the
    analysis-only ORT_OPT_DEBUG_FLAGS fail loudly (ORT_ERR_UNSUPPORTED) instead of silently
    rendering another way."""
    from octreeraytracer_amd import _lib as L
    for opt, val in ((L.ORT_OPT_RETIRED[0], 1), (L.ORT_OPT_RETIRED[1], 1), (L.ORT_OPT_PERSISTENT, 1),
                     (L.ORT_OPT_RETIRED[2], 1), (L.ORT_OPT_DEBUG_FLAGS, 1)):
        with pytest.raises(ort.OrtError) as e:
            renderer._check(renderer._lib.ort_set_option(renderer._ctx, opt, val))
        assert e.value.code == L.ORT_ERR_UNSUPPORTED, opt


@pytest.mark.parametrize("kid_skip", [1, 2, 0])
@pytest.mark.parametrize("sort", [2, 1, 0])
@pytest.mark.parametrize("depth,mspn", [(6, 1), (10, 1)])
def test_bounce_orders_and_skip_identical(ort, oracle, renderer, depth, mspn, sort, kid_skip):
    """Every order of the alive paths between bounces (ORT_OPT_SORT_PATHS: list sort with the
    length read back, every-slot sort, slot order) and the rejected-sphere skip on (records and
    kid entries interleaved, or from their two arrays) and off give
    the oracle's pixels, on maxSpheresPerNode-1 trees (where the skip fires) of depth 6 (64-bit
    bounce walk) and 10 (96-bit), with several samples (path state carried across samples)."""
    s = ort.random_spheres(8000, 3)
    t = ort.build_octree(s, depth, mspn)
    renderer.upload(s, t)
    renderer.set_sort_paths(sort)
    renderer.set_kid_skip(kid_skip)
    renderer.set_pixel_paths(0)  # the pipeline's bounce lists
    try:
        p = ort.FrameParams.default_camera(960, 540, num_samples=2, max_depth=5)
        tile = ort.Tile(100, 400, 200, 96)
        got = renderer.render(p, tile)
        ref = oracle.render(s, t, p, tile.x0, tile.y0, tile.width, tile.rows)
        assert_same(got, ref, f"sort={sort} kid_skip={kid_skip} d{depth}")
        with pytest.raises(ort.OrtError):
            renderer.set_kid_skip(3)
        if sort == 2:  # whole-pixel paths, with and without the skip
            with pixel_paths(renderer, 1):
                assert_same(renderer.render(p, tile), ref, f"pixel paths kid_skip={kid_skip} d{depth}")
    finally:
        renderer.set_sort_paths(2)  # the defaults
        renderer.set_kid_skip(1)
        renderer.set_pixel_paths(-1)


@pytest.mark.parametrize("mode", [0, 1])
@pytest.mark.parametrize("ns", [1, 2])
def test_band_padding_rows_with_bounces(ort, oracle, renderer, scene_c2, ns, mode):
    """Band tiles whose rows run past the frame (the multi-GPU partition's padding) in the
    multi-bounce pipeline, where the last shading writes the final pixels itself: the padding
    rows come back as zeros and every other pixel as the oracle's."""
    s, t = scene_c2
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(320, 180, num_samples=ns, max_depth=4)
    tile = ort.Tile(0, 320, 150, 64, 16, 64)  # rows y = 150 + 64 (j / 16) + j % 16: most past 180
    with pixel_paths(renderer, mode):
        got = renderer.render(p, tile)
    ref = oracle.render(s, t, p, 0, 150, 320, 64, band_height=16, band_stride=64)
    assert_same(got, ref, f"band padding ns={ns} pixel_paths={mode}")
    assert float(np.abs(got[16:]).max()) == 0.0  # rows past the frame


@pytest.fixture(scope="module")
def scene_c3(ort):
    s = ort.random_spheres(100_000, 42)
    return s, ort.build_octree(s, 8, 0)


def test_c3_full_frame_bit_exact(ort, oracle, renderer, scene_c3):
    """BASELINE configs[2]: 3840x2160, 100k spheres, depth 8 -- every pixel against the oracle."""
    s, t = scene_c3
    renderer.upload(s, t)
    assert renderer.info()["layout"] == "compact" and renderer.info()["n_nodes"] == 10_953_681
    p = ort.FrameParams.default_camera(3840, 2160)
    img = renderer.render(p)
    ref = oracle.render(s, t, p)
    assert_same(img, ref, "C3 full frame")
    # deterministic across launches, and the 8-rank band partition reassembles the frame
    assert np.array_equal(renderer.render(p), img)
    from octreeraytracer_amd.distributed import assemble, rank_tile
    parts = [renderer.render(p, rank_tile(3840, 2160, r, 8)) for r in range(8)]
    assert np.array_equal(assemble(np.stack(parts), 2160, 8), img)


def test_c3_counters_match_oracle_on_rows(ort, oracle, renderer, scene_c3):
    s, t = scene_c3
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(3840, 2160)
    tile = ort.Tile(0, 3840, 7, 16 * 4, 4, 135)  # 64 rows spread over the frame
    _, want = oracle.render(s, t, p, 0, 7, 3840, 64, band_height=4, band_stride=135, counts=True)
    assert renderer.count_traffic(p, tile) == want


def test_bounce_compaction_after_larger_frames(ort, oracle, renderer, scene_c2):
    """Bounces >= 1 walk only the alive paths (compacted list).  Slots a previous, larger
    render left alive must never leak into a later, smaller tile."""
    s, t = scene_c2
    renderer.upload(s, t)
    with pixel_paths(renderer, 0):  # the pipeline's compacted lists
        big = ort.FrameParams.default_camera(1920, 1080, num_samples=1, max_depth=4)
        renderer.render(big, ort.Tile(0, 1920, 0, 256))
        p = ort.FrameParams.default_camera(1920, 1080, num_samples=2, max_depth=5)
        for tile in (ort.Tile(900, 70, 500, 30), ort.Tile(0, 1920, 3, 40, 8, 27)):
            got = renderer.render(p, tile)
            ref = oracle.render(s, t, p, tile.x0, tile.y0, tile.width, tile.rows, band_height=tile.band_height,
                                band_stride=tile.band_stride)
            assert_same(got, ref, f"compaction tile {tile}")
            with pixel_paths(renderer, 1):  # whole-pixel paths after pipeline frames, and back
                assert_same(renderer.render(p, tile), ref, f"pixel paths tile {tile}")
            renderer.set_pixel_paths(0)


@pytest.mark.parametrize("depth,mspn", [(9, 0), (10, 1)])
def test_deep_tree_kernel_bit_exact(ort, oracle, renderer, depth, mspn):
    """Depth 9-10 trees take ort_trace_compact_deep (96-bit level masks): primary frame and
    multi-bounce tiles (path compaction in slot order, with the coherence sort of every slot and
    of the compacted list) against the oracle."""
    s = ort.random_spheres(20_000, 7)
    t = ort.build_octree(s, depth, mspn)
    renderer.build_scene(s, depth, mspn)
    assert renderer.info()["layout"] == "compact" and renderer.info()["tree_depth"] == depth
    p = ort.FrameParams.default_camera(640, 360)
    assert_same(renderer.render(p), oracle.render(s, t, p), f"deep d{depth} primary")
    pb = ort.FrameParams.default_camera(1280, 720, num_samples=2, max_depth=4)
    try:
        for sort in (0, 1, 2, "pixel paths"):
            if sort == "pixel paths":  # the depth 9-10 whole-pixel kernel (96-bit masks)
                renderer.set_pixel_paths(1)
            else:
                renderer.set_pixel_paths(0)
                renderer.set_sort_paths(sort)
            for tile in (ort.Tile(300, 160, 200, 96), ort.Tile(0, 1280, 5, 48, 8, 90)):
                got = renderer.render(pb, tile)
                ref = oracle.render(s, t, pb, tile.x0, tile.y0, tile.width, tile.rows, band_height=tile.band_height,
                                    band_stride=tile.band_stride)
                assert_same(got, ref, f"deep d{depth} bounces {tile} sort={sort}")
    finally:
        renderer.set_sort_paths(2)  # the default
        renderer.set_pixel_paths(-1)


@pytest.mark.parametrize("mode", [0, 1, 2, -1])
def test_xcd_swizzle_orders_identical(ort, oracle, renderer, scene_c2, mode):
    """Every workgroup -> tile order (ORT_OPT_XCD_SWIZZLE) renders the oracle's pixels: a
    ragged tile (partial 512/64-workgroup groups, edge super-tiles), bounces included."""
    s, t = scene_c2
    renderer.upload(s, t)
    renderer.set_xcd_swizzle(mode)
    renderer.set_pixel_paths(0)  # the pipeline's per-tile kernels
    try:
        p = ort.FrameParams.default_camera(1920, 1080, num_samples=1, max_depth=3)
        tile = ort.Tile(13, 1900, 7, 1010)  # 119 x 64 tiles: ragged in both directions
        assert_same(renderer.render(p, tile), oracle.render(s, t, p, 13, 7, 1900, 1010), f"swizzle {mode}")
        small = ort.Tile(5, 1000, 3, 900)  # <= 1.5 M pixels: raster order under the auto mode
        assert_same(renderer.render(p, small), oracle.render(s, t, p, 5, 3, 1000, 900), f"swizzle {mode}, small")
        for bad in (3, -2):
            with pytest.raises(ort.OrtError):
                renderer.set_xcd_swizzle(bad)
    finally:
        renderer.set_xcd_swizzle(-1)
        renderer.set_pixel_paths(-1)


@pytest.mark.parametrize("use_octree", [1, 0])
def test_extreme_sphere_roots(ort, oracle, renderer, use_octree):
    """The kernel's quotient/sqrt shortcuts at their edges (tests/test_emulation.py
    extreme_root_scene): camera inside a sphere, roots near 0, half_b^2 overflow, disc > 2^100."""
    from test_emulation import extreme_root_scene
    s = extreme_root_scene(ort)
    t = ort.build_octree(s, 5, 0) if use_octree else None
    renderer.upload(s, t)
    p = ort.FrameParams.default_camera(64, 40, max_depth=4, use_octree=use_octree)
    ref = oracle.render(s, t, p)
    for mode in (0, 1):
        with pixel_paths(renderer, mode):
            assert_same(renderer.render(p), ref, f"extreme roots pixel_paths={mode}")
    p1 = ort.FrameParams.default_camera(64, 40, use_octree=use_octree)
    assert_same(renderer.render(p1), oracle.render(s, t, p1), "extreme roots, primary")


@pytest.mark.parametrize("name", sorted(p.stem for p in (__import__("pathlib").Path(__file__).parent / "golden" / "glsl").glob("*.npz")))
def test_kernel_matches_reference_shader(ort, oracle, renderer, name):
    """The HIP kernels against the reference's own shaders run by Mesa llvmpipe
    (tests/golden/glsl, tests/test_glsl_parity.py for the tolerances) -- and bit-exact against
    the oracle on the same frame."""
    from test_glsl_parity import check_against_glsl, inputs, load
    ref, meta = load(name)
    s, t, p = inputs(ort, meta)
    renderer.upload(s, t)
    tree = t if meta["oct"] else None
    if "rows" in meta:  # the fixture's rows of a large frame (the bench's C3 frame)
        img = np.concatenate([renderer.render(p, ort.Tile(0, p.width, r, 1)) for r in meta["rows"]])
        ref_o = np.concatenate([oracle.render(s, tree, p, y0=r, rows=1) for r in meta["rows"]])
    else:
        img, ref_o = renderer.render(p), oracle.render(s, tree, p)
    check_against_glsl(img, ref, meta, f"HIP vs GLSL {name}")
    assert_same(img, ref_o, f"HIP vs oracle {name}")


@pytest.mark.parametrize("name", sorted(__import__("json").loads(
    (__import__("pathlib").Path(__file__).parent / "golden" / "glsl" / "canonical.json").read_text())["cases"]))
def test_kernel_bit_exact_to_reference_shader(ort, renderer, name):
    """The HIP frame IS the reference shader's frame, bit for bit, once GLSL's implementation-
    defined builtins are the canonical ones (tests/test_glsl_parity.py, canonical.json): the
    whole 3840x2160 C3 bench frame and C2 at 4 samples x 8 bounces included."""
    from test_glsl_parity import CANON, frame_sha, inputs
    c = CANON["cases"][name]
    s, t, p = inputs(ort, c)
    renderer.upload(s, t)
    assert frame_sha(renderer.render(p)) == c["sha256"], f"{name}: HIP frame differs from the reference shader's"


def test_launch_times_option(ort, oracle, renderer, scene_c1):
    """ORT_OPT_LAUNCH_TIMES 0: no per-launch events, same pixels, the frame still timed -- and the
    per-launch queries report no newer launch (include/ort.h): on a context never timed
    ort_last_trace_ms is an error and ort_trace_times_ms returns nothing; after one timed frame,
    untimed frames leave that frame's launch time the newest."""
    s, t = scene_c1
    p = ort.FrameParams.default_camera(96, 64, num_samples=2, max_depth=3)
    with ort.Renderer(0) as fresh:
        fresh.upload(s, t)
        fresh.set_launch_times(0)
        assert_same(fresh.render(p), oracle.render(s, t, p), "launch times off, fresh context")
        assert fresh.last_kernel_ms() > 0.0
        with pytest.raises(ort.OrtError):
            fresh.last_trace_ms()
        assert fresh.trace_times_ms(4) == []
        fresh.set_launch_times(1)
        fresh.render(p)  # one timed frame
        timed = fresh.trace_times_ms(1)
        assert len(timed) == 1 and timed[0] > 0.0 and fresh.last_trace_ms() == timed[0]
        fresh.set_launch_times(0)
        for _ in range(3):
            fresh.render(p)
        assert fresh.trace_times_ms(1) == timed and fresh.last_trace_ms() == timed[0]
        assert len(fresh.trace_times_ms(8)) == 1
    renderer.upload(s, t)
    try:
        renderer.set_launch_times(0)
        got = renderer.render(p)
        assert_same(got, oracle.render(s, t, p), "launch times off")
        assert renderer.last_kernel_ms() > 0.0
        with pytest.raises(ort.OrtError):
            renderer.set_launch_times(2)
    finally:
        renderer.set_launch_times(1)
    renderer.render(p)
    assert renderer.last_trace_ms() > 0.0


def test_pixel_paths_option_and_auto(ort, oracle, scene_c1, scene_c3):
    """ORT_OPT_PIXEL_PATHS: -1 / 0 / 1 accepted, others refused; the auto mode renders a
    small tree's multi-bounce frame in ONE trace launch and the C3 tree's (10.9 M nodes) with
    the per-bounce pipeline; primary-ray frames (1 sample, 1 bounce) never take it."""
    s, t = scene_c1
    p = ort.FrameParams.default_camera(128, 96, num_samples=8, max_depth=6)
    with ort.Renderer(0) as r:
        for bad in (-2, 2):
            with pytest.raises(ort.OrtError):
                r.set_pixel_paths(bad)
        r.upload(s, t)
        ref = oracle.render(s, t, p)
        # the first whole-pixel frame of a shape: one launch; the next: samples in parallel
        # (ORT_OPT_PIXEL_SPECULATE), a resolve and the fixup list -- three
        for mode, launches in ((-1, 1), (1, 3), (0, None)):
            r.set_pixel_paths(mode)
            assert_same(r.render(p), ref, f"pixel_paths={mode}")
            n = r.frame_trace_times_ms(1)[0][1]
            assert n == launches if launches else n > 1, (mode, n)
        r.set_pixel_paths(1)
        p1 = ort.FrameParams.default_camera(128, 96)
        assert_same(r.render(p1), oracle.render(s, t, p1), "primary")
    s3, t3 = scene_c3
    with ort.Renderer(0) as r:
        r.upload(s3, t3)
        pb = ort.FrameParams.default_camera(256, 144, num_samples=2, max_depth=3)
        got = r.render(pb)
        assert r.frame_trace_times_ms(1)[0][1] > 1  # auto: the pipeline on a large tree
        assert_same(got, oracle.render(s3, t3, pb), "C3 tree, auto")
    # a 1.48 M-node tree (> 2^19): whole-pixel paths with 5 or 8 bounces, the pipeline with 3,
    # whatever the samples -- the rule's regimes (profiles/r06/grid/)
    sm = ort.random_spheres(30_000, 42)
    tm = ort.build_octree(sm, 7, 0)
    assert 2**19 < tm.n_nodes <= 2**23
    with ort.Renderer(0) as r:
        r.upload(sm, tm)
        for ns, maxd, one_launch in ((2, 3, False), (1, 3, False), (2, 5, True), (1, 8, True)):
            pm = ort.FrameParams.default_camera(192, 108, num_samples=ns, max_depth=maxd)
            got = r.render(pm)
            n = r.frame_trace_times_ms(1)[0][1]
            assert (n == 1) == one_launch, (ns, maxd, n)
            assert_same(got, oracle.render(sm, tm, pm), f"1.48 M-node tree, {ns} x {maxd}, auto")


@pytest.mark.parametrize("n,depth,mspn", [(100, 3, 0), (60, 5, 1), (10, 1, 1)])
def test_pixel_paths_lds_scene(ort, oracle, n, depth, mspn):
    """Whole-pixel paths on scenes small enough for the LDS-resident copy (ORT_OPT_PIXEL_LDS_SCENE):
    config.h's default scene, a depth-5 M=1 tree (the rejected-sphere skip from the LDS kid
    entries) and runner.py's 10-sphere tree -- LDS on and off, against the oracle."""
    s = ort.random_spheres(n, 42)
    t = ort.build_octree(s, depth, mspn)
    assert 16 * (t.n_nodes + t.n_indices + s.n) <= 32768
    p = ort.FrameParams.default_camera(200, 150, num_samples=4, max_depth=8)
    ref = oracle.render(s, t, p)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        for on in (1, 0):
            r.set_pixel_lds_scene(on)
            assert_same(r.render(p), ref, f"n{n} d{depth} lds_scene={on}")
        with pytest.raises(ort.OrtError):
            r.set_pixel_lds_scene(2)


@pytest.mark.parametrize("scene", ["c2", "lds", "deep", "brute"])
def test_pixel_speculate(ort, oracle, scene_c2, scene):
    """ORT_OPT_PIXEL_SPECULATE: from a shape's second frame on, every (pixel, sample) traced in
    parallel from last frame's per-sample RNG end states, checked, and the pixels whose states
    moved re-traced from the first moved sample on.  Static frames (every state holds), a camera
    turning by small and large steps (some / most pixels re-traced), shape changes, a band tile
    with padding rows, the LDS-resident and the depth-10 walks and brute force -- every frame the
    oracle's, with the option on and off."""
    if scene == "c2":
        s, t = scene_c2
    elif scene == "lds":
        s = ort.random_spheres(100, 42)
        t = ort.build_octree(s, 3, 0)
    else:  # deep; brute force over the same 1000 spheres (the uploaded tree unused)
        s = ort.random_spheres(1000, 42)
        t = ort.build_octree(s, 10, 1)
    bf = scene == "brute"
    t_up, t = t, (None if bf else t)

    def cam(W, H, ns, md, yaw=0.0):
        from octreeraytracer_amd.scene import DEFAULT_YAW
        return ort.FrameParams.default_camera(W, H, num_samples=ns, max_depth=md, yaw=DEFAULT_YAW + yaw,
                                              use_octree=0 if bf else 1)

    W, H = (96, 64) if bf else (160, 120)
    shots = [(cam(W, H, 8, 6), None)] * 3                                   # static (2 chunks of 4 samples)
    shots += [(cam(W, H, 8, 6, 0.3 * j), None) for j in (1, 2, 3)]          # small turns
    shots += [(cam(W, H, 8, 6, 25.0), None), (cam(W, H, 8, 6, -40.0), None)]  # large jumps
    shots += [(cam(W, H, 12, 4), None)] * 2                                 # another shape: 3 chunks
    shots += [(cam(320, 180, 9, 4), ort.Tile(0, 320, 150, 64, 16, 64))] * 2  # band padding, a 1-sample chunk
    with ort.Renderer(0) as r:
        for bad in (-2, 2):
            with pytest.raises(ort.OrtError):
                r.set_pixel_speculate(bad)
        r.upload(s, t_up)
        with pixel_paths(r, 1):
            for mode in (1, -1, 0):  # on, auto (timed per shape: either way), off
                r.set_pixel_speculate(mode)
                for i, (fp, tile) in enumerate(shots):
                    if tile is None:
                        got, ref = r.render(fp), oracle.render(s, t, fp)
                    else:
                        got = r.render(fp, tile)
                        ref = oracle.render(s, t, fp, tile.x0, tile.y0, tile.width, tile.rows,
                                            band_height=tile.band_height, band_stride=tile.band_stride)
                    assert_same(got, ref, f"{scene} speculate={mode} frame {i}")
                    # launches: 3 speculating, 1 running whole chains -- the first frame of a
                    # shape (0, 8, 10) and, while pixels move (frames 4-7: the camera turns; the
                    # frames are synchronous, so each one knows what the one before measured),
                    # frames after one that found moved pixels
                    n = r.frame_trace_times_ms(1)[0][1]
                    if mode == 0 or i in (0, 8, 10):
                        assert n == 1, (scene, mode, i, n)
                    elif mode == 1 and i in (1, 2, 3, 9, 11):
                        assert n == 3, (scene, mode, i, n)
                    else:
                        assert n in (1, 3), (scene, mode, i, n)
            r.set_pixel_speculate(-1)


def test_pixel_heavy_first(ort, oracle, scene_c2):
    """ORT_OPT_PIXEL_HEAVY_FIRST: whole-pixel paths taking the previous frame's heaviest 8x8
    blocks first.  Runs of frames of one shape (the second and later read the lists the one
    before wrote), shape changes (lists discarded), an odd frame size (slots past the tile) and a
    band tile with padding rows (slots past the frame) -- every frame the oracle's, in each mode."""
    s, t = scene_c2
    p = ort.FrameParams.default_camera(200, 150, num_samples=4, max_depth=6)
    p2 = ort.FrameParams.default_camera(136, 100, num_samples=2, max_depth=5)
    p3 = ort.FrameParams.default_camera(320, 180, num_samples=2, max_depth=4)
    p1 = ort.FrameParams.default_camera(200, 150, num_samples=1, max_depth=4)
    band = ort.Tile(0, 320, 150, 64, 16, 64)
    refs = {"p": oracle.render(s, t, p), "p2": oracle.render(s, t, p2), "p1": oracle.render(s, t, p1),
            "band": oracle.render(s, t, p3, 0, 150, 320, 64, band_height=16, band_stride=64)}
    frames = {"p": (p, None), "p2": (p2, None), "p1": (p1, None), "band": (p3, band)}
    with ort.Renderer(0) as r:
        for bad in (-2, 2):
            with pytest.raises(ort.OrtError):
                r.set_pixel_heavy_first(bad)
        r.upload(s, t)
        with pixel_paths(r, 1):
            for mode in (-1, 1, 0):
                r.set_pixel_heavy_first(mode)
                for name in ("p", "p", "p", "p2", "p2", "p", "band", "band", "band", "p1", "p1", "p"):
                    fp, tile = frames[name]
                    got = r.render(fp, tile) if tile else r.render(fp)
                    assert_same(got, refs[name], f"heavy_first={mode} {name}")
            r.set_pixel_heavy_first(-1)


def test_pixel_speculate_stream_ordered_and_group(ort, oracle, scene_c2):
    """Speculating frames queued back to back on a caller stream (device output, no host wait
    between them: the moved-pixel counts and the auto mode's timings are read only once their
    events completed), on two contexts alternating, and on a one-GPU render group's band
    contexts -- every frame the synchronous whole-chain render's."""
    torch = pytest.importorskip("torch")
    from octreeraytracer_amd.group import RenderGroup
    s, t = scene_c2
    W, H = 200, 136
    p = ort.FrameParams.default_camera(W, H, num_samples=8, max_depth=5)
    ref = oracle.render(s, t, p)
    rs = [ort.Renderer(0) for _ in range(2)]
    try:
        for x in rs:
            x.upload(s, t)
            x.set_pixel_paths(1)
        st = torch.cuda.Stream()
        outs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(12)]
        for k, o in enumerate(outs):
            rs[k % 2].render(p, out=o, stream=st.cuda_stream)
        st.synchronize()
        for k, o in enumerate(outs):
            assert_same(o.cpu().numpy(), ref, f"stream-ordered frame {k}")
        assert any(n == 3 for _, n in rs[0].frame_trace_times_ms(6))  # some of them speculated
    finally:
        for x in rs:
            x.close()
    with RenderGroup([0, 0, 0], 1) as g:
        g.upload(s, t)
        for k in range(5):
            assert_same(g.render(p), ref, f"group frame {k}")
