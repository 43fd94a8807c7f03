"""ort_group_*: several GPUs in one process behind the C ABI.

CPU: the group's band partition and row map with an in-memory ("fake") transport -- every
rank's band tile rendered one after another by the host emulation of the kernel, then
assembled by the device kernel's row map -- equal the oracle's single-context frame bit for
bit, for 1..8 ranks and heights that are not a multiple of the band.
GPU: the real group (RCCL over one device; device copies over one device listed several
times, which exercises the multi-rank gather and de-interleave on a one-GPU box) against
ort_render and the oracle."""
import numpy as np
import pytest


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_group_partition_emulated(ort, oracle, scene_c1, world):
    from octreeraytracer_amd.group import emulate_group_host
    s, t = scene_c1
    for W, H in ((96, 70), (64, 33)):
        p = ort.FrameParams.default_camera(W, H, max_depth=2)
        got = emulate_group_host(s, t, p, world)
        ref = oracle.render(s, t, p)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32)), (world, W, H)


def test_group_partition_matches_distributed_py(ort):
    """group_map.h and distributed.py deal the same bands (both paths shard the frame alike)."""
    from octreeraytracer_amd.distributed import rank_tile
    from octreeraytracer_amd.group import emulate_group_host  # noqa: F401  (library loads)
    for H in (70, 2160, 4320):
        for world in (1, 2, 3, 8):
            rows = set()
            for r in range(world):
                t = rank_tile(128, H, r, world)
                rows.update(int(y) for y in t.pixel_rows(H) if y < H)
            assert rows == set(range(H))


@pytest.mark.gpu
@pytest.mark.parametrize("devices,transport", [([0], 0), ([0], 1), ([0, 0], 1), ([0, 0, 0], 1)])
def test_group_render(ort, oracle, scene_c2, devices, transport):
    from octreeraytracer_amd.group import RenderGroup
    s, t = scene_c2
    with RenderGroup(devices, transport) as g:
        g.upload(s, t)
        for md, spp in ((1, 1), (3, 2)):
            p = ort.FrameParams.default_camera(1920, 1080, num_samples=spp, max_depth=md)
            img = g.render(p)
            assert g.last_frame_ms() > 0
            with ort.Renderer(0) as r:
                r.upload(s, t)
                single = r.render(p)
            assert np.array_equal(img.view(np.uint32), single.view(np.uint32)), (devices, transport, md)
        p = ort.FrameParams.default_camera(1920, 1080)
        img = g.render(p)
        ref = oracle.render(s, t, p, 0, 500, 1920, 40)  # rows 500..539 span three 16-row bands
        assert np.array_equal(img[500:540].view(np.uint32), ref.view(np.uint32))


@pytest.mark.gpu
def test_group_device_output_and_build(ort, oracle):
    torch = pytest.importorskip("torch")
    from octreeraytracer_amd.group import RenderGroup
    s = ort.random_spheres(10_000, 42)
    t = ort.build_octree(s, 6, 0)
    with RenderGroup([0, 0, 0, 0], 1) as g:
        g.build_scene(s, 6, 0)  # every context builds on its device
        p = ort.FrameParams.default_camera(1000, 600)
        dev = torch.empty((600, 1000, 3), dtype=torch.float32, device="cuda:0")
        g.render(p, out=dev)
        torch.cuda.synchronize()
        ref = oracle.render(s, t, p)
        assert np.array_equal(dev.cpu().numpy().view(np.uint32), ref.view(np.uint32))
        with pytest.raises(ValueError):
            g.render(p, out=torch.empty((600, 1000, 3), dtype=torch.float16, device="cuda:0"))


@pytest.mark.gpu
def test_group_errors(ort):
    from octreeraytracer_amd.group import RenderGroup
    with pytest.raises(ort.OrtError):
        RenderGroup([0, 0], 0)  # RCCL needs distinct devices
    with pytest.raises(ort.OrtError):
        RenderGroup([], 1)
    with pytest.raises(ort.OrtError):
        RenderGroup([0], 7)  # unknown transport


@pytest.mark.gpu
@pytest.mark.parametrize("inflight", [2, 3])
def test_group_pipelined_frames(ort, oracle, scene_c2, inflight):
    """ort_group_submit / ort_group_wait with frame slots on [0, 0, 0, 0] (copy transport): a
    stream of frames with changing cameras and bounce depths, several in flight, each equal to
    a single-context render bit for bit (the slot buffers are reused only after their frame)."""
    torch = pytest.importorskip("torch")
    from octreeraytracer_amd.group import RenderGroup
    s, t = scene_c2
    W, H = 1920, 1080
    shots = []
    for k in range(7):
        pos = (0.3 * k, 2.5, -10.0 + 0.5 * k)
        shots.append(ort.FrameParams.default_camera(W, H, max_depth=1 + (k % 3), position=pos, yaw=-90.0 + 2 * k))
    with ort.Renderer(0) as r:
        r.upload(s, t)
        want = [r.render(p) for p in shots]
    with RenderGroup([0, 0, 0, 0], 1, inflight=inflight) as g:
        g.upload(s, t)
        outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0") for _ in shots]
        host = np.empty((H, W, 3), np.float32)
        tickets = [g.submit(p, o) for p, o in zip(shots, outs)]
        assert tickets == list(range(len(shots)))
        g.wait(tickets[-1])
        ms_last = g.last_frame_ms()
        # frame 0's slot has been reused since: its time was kept when it completed (not the
        # time of the slot's later frame)
        g.wait(tickets[0])
        ms_first = g.last_frame_ms()
        assert ms_last > 0 and ms_first > 0
        for tk in tickets:
            g.wait(tk)
        assert g.last_frame_ms() > 0
        with pytest.raises(ValueError):
            g.submit(shots[0], None)  # the frame is written after submit returns: out is required
        for k, (o, w) in enumerate(zip(outs, want)):
            assert np.array_equal(o.cpu().numpy().view(np.uint32), w.view(np.uint32)), k
        tk = g.submit(shots[2], host)  # host output through a slot
        g.wait(tk)
        assert np.array_equal(host.view(np.uint32), want[2].view(np.uint32))
        ref = oracle.render(s, t, shots[0], 0, 500, W, 40)
        assert np.array_equal(outs[0].cpu().numpy()[500:540].view(np.uint32), ref.view(np.uint32))
        with pytest.raises(ort.OrtError):
            g.wait(99)


def test_group_submit_requires_out(ort):
    """submit() writes its frame asynchronously, so a missing output is refused before the ABI
    (no GPU needed: the check runs first)."""
    from octreeraytracer_amd.group import RenderGroup
    g = object.__new__(RenderGroup)
    g._g = None
    g._pending = {}
    with pytest.raises(ValueError):
        g.submit(ort.FrameParams.default_camera(64, 32), None)


@pytest.mark.gpu
def test_group_wait_is_bounded(ort, scene_c2):
    """ort_group_set_timeout: a wait that expires returns ORT_ERR_TIMEOUT naming the frame, its
    slot and what is still pending (instead of blocking: a first multi-GPU run that stalls says
    where); the frame stays submitted and a later wait sees it complete, bit-exact.

    Deterministic: rank 0's stream is held by a device-side gate the test owns
    (hipStreamWaitValue32 on a flag in mapped, coherent host memory, enqueued ahead of the
    submit), so the frame cannot complete before the zero-timeout poll whatever the GPU's
    speed; the host sets the flag after the poll, and in any case before the group is destroyed
    (a release from another stream could share the gated stream's hardware queue)."""
    import ctypes as C
    from octreeraytracer_amd.group import RenderGroup
    s, t = scene_c2
    p = ort.FrameParams.default_camera(320, 180, num_samples=2, max_depth=3)
    with ort.Renderer(0) as r:
        r.upload(s, t)
        want = r.render(p)
    torch = pytest.importorskip("torch")
    hip = C.CDLL("libamdhip64.so.7")  # the runtime libort.so is linked against (already loaded)
    assert hip.hipSetDevice(0) == 0
    flag, dflag = C.c_void_p(), C.c_void_p()
    assert hip.hipHostMalloc(C.byref(flag), C.c_size_t(64), C.c_uint(0x40000002)) == 0  # mapped | coherent
    gate = C.c_uint32.from_address(flag.value)
    gate.value = 0
    assert hip.hipHostGetDevicePointer(C.byref(dflag), flag, C.c_uint(0)) == 0

    def release():
        gate.value = 1

    try:
        with RenderGroup([0, 0], 1, inflight=2) as g:
            g.upload(s, t)
            out = torch.empty((180, 320, 3), dtype=torch.float32, device="cuda:0")  # device output: no host copy
            h = C.c_void_p()
            assert g._lib.ort_get_stream(g.context(0), C.byref(h)) == 0 and h.value  # slot 0, rank 0
            try:
                # hipStreamWaitValue32(stream, ptr, value, flags = hipStreamWaitValueGte, mask)
                assert hip.hipStreamWaitValue32(h, dflag, C.c_uint32(1), C.c_uint(0), C.c_uint32(0xFFFFFFFF)) == 0
                g.set_timeout(0)  # poll once
                tk = g.submit(p, out)  # ticket 0: slot 0, behind the gate
                with pytest.raises(ort.OrtError) as e:
                    g.wait(tk)
            finally:
                release()
            assert e.value.code == ort.ORT_ERR_TIMEOUT
            msg = str(e.value)
            assert "slot" in msg and "pending" in msg and "frame" in msg and "rank 0" in msg, msg
            g.set_timeout(120_000)
            g.wait(tk)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))
    finally:
        release()
        assert hip.hipDeviceSynchronize() == 0
        hip.hipHostFree(flag)


@pytest.mark.gpu
def test_group_frame_times_window(ort, scene_c1):
    """ort_group_last_frame_ms keeps the last 64 frames' times: waiting for an older ticket
    leaves the time unknown (an error), not an earlier frame's."""
    from octreeraytracer_amd.group import RenderGroup
    s, t = scene_c1
    p = ort.FrameParams.default_camera(64, 64)
    with RenderGroup([0], 1, inflight=2) as g:
        g.upload(s, t)
        outs = [np.empty((64, 64, 3), np.float32) for _ in range(3)]
        tks = []
        for k in range(70):
            tks.append(g.submit(p, outs[k % 3]))
            g.wait(tks[-1])
        assert g.last_frame_ms() > 0
        g.wait(tks[0])  # 70 frames ago: its time is gone
        with pytest.raises(ort.OrtError):
            g.last_frame_ms()
        g.wait(tks[-2])
        assert g.last_frame_ms() > 0
