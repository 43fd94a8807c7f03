"""Multi-bounce ort_render is stream-ordered (include/ort.h ORT_OPT_SORT_PATHS 2): the list
sort between bounces takes its size from a host-side hint and its length from the device, so
no step of a frame waits on the host (the reference's per-frame launch returns at once too:
glDrawArrays, src/raytracer.cpp:499, with the bounce loop on the device, glsl:597-633).

Bar: bit-exact against the oracle and against other path orders (the order of the alive
paths never changes pixels: they are independent)."""
import time

import numpy as np
import pytest

from test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu

W, H = 1920, 1080


@pytest.fixture(scope="module")
def c2_bounce(ort, scene_c2):
    s, t = scene_c2
    r = ort.Renderer(0)
    r.upload(s, t)
    r.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
    yield s, t, r
    r.close()


def test_multibounce_render_returns_before_the_frame_ends(ort, oracle, c2_bounce):
    """A 4-bounce C2 frame under the default SORT_PATHS, rendered on a caller's stream that a
    spin kernel holds busy: ort_render returns while that stream has not even started the
    frame (a host wait inside the call would have blocked until the spin kernel and the first
    bounces finished).  The frame is then bit-exact."""
    torch = pytest.importorskip("torch")
    s, t, r = c2_bounce
    p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=4)
    stream = torch.cuda.Stream(device=0)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
    r.render(p, out=out, stream=stream.cuda_stream)  # first frame of this shape: allocations, hints
    stream.synchronize()
    for _ in range(2):  # the second frame sorts with the previous frame's lengths as bounds
        with torch.cuda.stream(stream):
            torch.cuda._sleep(400_000_000)  # hundreds of ms of spinning on `stream`
        end = torch.cuda.Event()
        t0 = time.perf_counter()
        r.render(p, out=out, stream=stream.cuda_stream)
        call_ms = (time.perf_counter() - t0) * 1e3
        end.record(stream)
        busy = not end.query()
        stream.synchronize()
        assert busy, "ort_render waited on the host for the frame"
        assert call_ms < 50.0, f"ort_render took {call_ms:.1f} ms on the host"
    img = out.cpu().numpy()
    with ort.Renderer(0) as r0:  # slot order, synchronous: an independent path order
        r0.upload(s, t)
        r0.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
        r0.set_sort_paths(0)
        assert_same(img, r0.render(p), "stream-ordered list sort vs slot order")
    ref = oracle.render(s, t, p, 0, 500, W, 40, threads=0)
    assert_same(img[500:540], ref, "stream-ordered 4-bounce C2 rows vs oracle")


@pytest.mark.parametrize("bound", [1, 1000, 300_000, 0])
def test_sort_bound_short_and_long(ort, oracle, c2_bounce, bound):
    """A bound below the list's length (the list goes on in append order), one around it, and
    the hint (0): the same pixels every time, across frames that reuse the hints."""
    s, t, r = c2_bounce
    p = ort.FrameParams.default_camera(W, H, num_samples=2, max_depth=3)
    tile = ort.Tile(0, W, 4, 96, 16, 270)
    r.set_sort_bound(bound)
    try:
        frames = [r.render(p, tile) for _ in range(3)]
    finally:
        r.set_sort_bound(0)
    ref = oracle.render(s, t, p, 0, 4, W, 96, band_height=16, band_stride=270, threads=0)
    for i, f in enumerate(frames):
        assert_same(f, ref, f"bound={bound} frame {i}")


def test_hints_follow_the_frame_shape(ort, c2_bounce):
    """Hints belong to one frame shape: alternating shapes (different list lengths) on one
    context stays bit-exact against fresh contexts."""
    s, t, r = c2_bounce
    shapes = [(ort.FrameParams.default_camera(W, H, max_depth=4), ort.Tile(0, W, 0, 256)),
              (ort.FrameParams.default_camera(W, H, max_depth=3), ort.Tile(300, 700, 200, 333)),
              (ort.FrameParams.default_camera(640, 360, num_samples=3, max_depth=4), None)]
    want = []
    for p, tl in shapes:
        with ort.Renderer(0) as fresh:
            fresh.upload(s, t)
            fresh.set_pixel_paths(0)  # the per-bounce pipeline (its options are under test)
            want.append(fresh.render(p, tl))
    for rep in range(2):
        for (p, tl), w in zip(shapes, want):
            assert_same(r.render(p, tl), w, f"shape {p.width}x{p.height} d{p.max_depth} rep {rep}")
