"""Multi-rank partition + gather + assembly on CPU (gloo, world_size 2 and 3).  Each rank
renders its band tile with the host build of the kernel's per-pixel code; rank 0 gathers
with the same FrameGather the GPU bench uses and must reproduce the single-render frame."""
import os
import sys
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, W, H, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import octreeraytracer_amd as ort
    from octreeraytracer_amd.distributed import FrameGather, rank_tile
    from octreeraytracer_amd.renderer import emulate_render_host
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    p = ort.FrameParams.default_camera(W, H)
    tile = rank_tile(W, H, rank, world)
    local, _ = emulate_render_host(s, t, p, tile)
    g = FrameGather(dist, W, H, world, rank, "cpu")
    frame = g(torch.from_numpy(local))
    if rank == 0:
        q.put(frame.numpy().copy())
    dist.barrier()
    dist.destroy_process_group()


def worker_pipelined(rank, world, port, W, H, q):
    """bench.py's pipeline: two frames in flight (double-buffered tiles, async gathers)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import octreeraytracer_amd as ort
    from octreeraytracer_amd.distributed import FrameGather, rank_tile
    from octreeraytracer_amd.renderer import emulate_render_host
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    tile = rank_tile(W, H, rank, world)
    g = FrameGather(dist, W, H, world, rank, "cpu", depth=2)
    handles = []
    for slot, yaw in enumerate((-90.0, -80.0)):
        p = ort.FrameParams.default_camera(W, H, yaw=yaw)
        local, _ = emulate_render_host(s, t, p, tile)
        handles.append(g.submit(torch.from_numpy(local), slot))
    frames = []
    for h in handles:  # finish() assembles into one frame buffer: copy each frame out
        f = g.finish(h)
        if rank == 0:
            frames.append(f.numpy().copy())
    if rank == 0:
        q.put(frames)
    dist.barrier()
    dist.destroy_process_group()


def test_pipelined_gather_two_frames_in_flight(ort, oracle):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    W, H, world = 48, 40, 2
    procs = [ctx.Process(target=worker_pipelined, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    frames = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    for f, yaw in zip(frames, (-90.0, -80.0)):
        assert np.array_equal(f, oracle.render(s, t, ort.FrameParams.default_camera(W, H, yaw=yaw)))


@pytest.mark.parametrize("world,W,H", [(2, 64, 72), (3, 40, 100)])
def test_gather_assembles_full_frame(ort, oracle, world, W, H):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=worker, args=(r, world, port, W, H, q)) for r in range(world)]
    for p in procs:
        p.start()
    frame = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    ref = oracle.render(s, t, ort.FrameParams.default_camera(W, H))
    assert np.array_equal(frame, ref)


def test_partition_covers_every_row_once():
    from octreeraytracer_amd.distributed import assemble, rank_tile
    for H in (1, 15, 16, 17, 2160, 4320):
        for world in (1, 2, 3, 4, 8):
            rows = []
            tiles = [rank_tile(8, H, r, world) for r in range(world)]
            assert len({t.rows for t in tiles}) == 1
            for t in tiles:
                ys = t.pixel_rows(H)
                rows += [y for y in ys if y < H]
            assert sorted(rows) == list(range(H)), (H, world)
            # assembly inverts the partition
            g = np.stack([np.broadcast_to(np.array(t.pixel_rows(H), np.float32)[:, None, None], (t.rows, 8, 3))
                          for t in tiles])
            f = assemble(g, H, world)
            assert np.array_equal(f[:, 0, 0], np.arange(H, dtype=np.float32))


def _bench_line(out: str) -> dict:
    import json
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def worker_timeout(rank, world, port, q, done):
    """Rank 1 never sends its band: rank 0's bounded finish() must raise naming rank and slot."""
    try:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        from octreeraytracer_amd.distributed import FrameGather, GatherTimeout
        W, H = 8, 64
        g = FrameGather(dist, W, H, world, rank, "cpu", depth=2, timeout_s=2.0)
        if rank == 0:
            local = torch.zeros((g.slots[0].shape[1], W, 3))
            h = g.submit(local, 1)
            try:
                g.finish(h)
                q.put("no timeout")
            except GatherTimeout as e:
                q.put(str(e))
            done.set()
        else:
            done.wait(120)  # alive but sending nothing (a dead peer would end the gather with an error instead)
    except BaseException as e:  # any other failure reaches the test as its message
        q.put(f"rank {rank} failed: {e!r}")
        done.set()
    q.close()
    q.join_thread()  # the queue's feeder thread has written the message (os._exit would drop it)
    os._exit(0)  # the gather is still posted: leave without tearing the group down


def test_gather_wait_is_bounded():
    """FrameGather(timeout_s) bounds a frame's gather: a rank that never sends makes rank 0's
    finish() raise GatherTimeout naming the rank and the slot (bench.py then exits 3)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    done = ctx.Event()
    procs = [ctx.Process(target=worker_timeout, args=(r, 2, port, q, done)) for r in range(2)]
    for p in procs:
        p.start()
    msg = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        if p.exitcode is None:
            p.kill()
    assert "rank 0" in msg and "slot 1" in msg and "within 2.0 s" in msg, msg


@pytest.mark.parametrize("world", [2, 3, 8])
def test_bench_self_launch(world):
    """`bench.py --gpus N` with no launcher starts its own N ranks (torch.distributed.run as a
    child process) and prints rank 0's line only; --emulate renders on the host and gathers
    with gloo.  The assembled frame equals the oracle's single-process frame and the reference
    shaders' frame."""
    import hashlib
    import subprocess
    import sys
    from pathlib import Path
    root = Path(__file__).resolve().parents[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", str(world), "--emulate", "--config", "c1",
                        "--steps", "1", "--warmup", "0"], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = _bench_line(r.stdout)
    assert line["n_gpus"] == world and "EMULATION" in line["data"]
    import octreeraytracer_amd as ort
    from oracle import oracle
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    ref = oracle.render(s, t, ort.FrameParams.default_camera(256, 256))
    assert line["frame_sha256"] == hashlib.sha256(np.ascontiguousarray(ref).tobytes()).hexdigest()
    # ... and the reference's own shaders' frame (tests/test_glsl_parity.py), bit for bit
    assert line["parity"]["bit_identical"] and line["parity"]["frame_sha256"] == line["frame_sha256"]


def test_bench_group_arguments(monkeypatch):
    """`bench.py --group` runs in this process (no torch.distributed.run self-launch even with
    --gpus N) and reaches group_bench with the parsed options."""
    import bench
    seen = {}
    monkeypatch.setattr(sys, "argv", ["bench.py", "--group", "--gpus", "8", "--rehearse-one-gpu", "--config", "c1",
                                      "--inflight", "3", "--steps", "2"])
    monkeypatch.setattr(bench, "self_launch", lambda args: (_ for _ in ()).throw(AssertionError("self-launched")))
    monkeypatch.setattr(bench, "group_bench", lambda args: seen.update(vars(args)))
    bench.main()
    assert seen["group"] and seen["gpus"] == 8 and seen["rehearse_one_gpu"] and seen["inflight"] == 3
    assert seen["config"] == "c1" and seen["steps"] == 2
