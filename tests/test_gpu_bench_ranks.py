"""bench.py's N>1 path on the GPU (BASELINE configs[3], C4: the 3840x2160 / 100k-sphere /
depth-8 frame cut into 16-row bands dealt round-robin to N ranks, gathered to rank 0).

On a one-GPU box every rank runs on GPU 0 (`--rehearse-one-gpu`): the rank processes, their
two contexts each (frames in flight), the band tiles rendered by the HIP kernels, the
pipelined async gather and rank 0's de-interleave are bench.py's own code; only the transport
is gloo instead of RCCL (RCCL refuses two ranks on one device).  The frame rank 0 assembles
(saved as float32 PFM, lossless) must equal a single-GPU render of the whole frame bit for
bit -- pixels depend only on global coordinates.  N = 2, 4 and 8 (C4's own
partition: 17 bands of 16 rows per rank, the last ones padding); each rank process holds two
scene copies on the one card.
"""
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def c3_frame(ort):
    s = ort.random_spheres(100_000, 42)
    r = ort.Renderer(0)
    r.build_scene(s, 8, 0)
    frame = r.render(ort.FrameParams.default_camera(3840, 2160))
    r.close()
    return frame


@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_ranks_assemble_the_c3_frame(c3_frame, world, tmp_path):
    from octreeraytracer_amd import image
    out = tmp_path / "frame.pfm"
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", str(world), "--rehearse-one-gpu",
                        "--config", "c3", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--save", str(out)],
                       capture_output=True, text=True, env=env, timeout=100)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    import bench
    assert line["n_gpus"] == world and line["config"]["frames_in_flight"] == bench.default_inflight("c3", world)
    assert line["config"]["rays_per_step"] == 3840 * 2160
    got = image.read_pfm(out)
    assert got.shape == c3_frame.shape and got.dtype == np.float32
    assert np.array_equal(got.view(np.uint32), c3_frame.view(np.uint32))
    assert line["parity"]["bit_identical"], line["parity"]  # ... and the reference shaders' frame


@pytest.mark.parametrize("world,inflight", [(4, 2), (8, 0)])
def test_bench_group_rehearsal_is_bit_identical(world, inflight):
    """`bench.py --group --rehearse-one-gpu`: one process, the C-ABI group with `world` ranks on
    GPU 0 (device-copy gather), frames submitted with slots in flight; the line's frame check
    compares the last frame with a single-context render bit for bit."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, str(ROOT / "bench.py"), "--group", "--gpus", str(world), "--rehearse-one-gpu",
           "--config", "c3", "--steps", "4", "--warmup", "1", "--no-cpu-baseline"]
    if inflight:
        cmd += ["--inflight", str(inflight)]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=110)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["frame_check"].startswith("bit-identical"), line["frame_check"]
    assert line["parity"]["bit_identical"], line["parity"]  # the group's frame IS the reference shaders'
    assert line["n_gpus"] == world and line["config"]["devices"] == [0] * world
    assert line["config"]["rays_per_step"] == 3840 * 2160
    import bench
    assert line["config"]["frames_in_flight"] == (inflight or bench.default_inflight("c3", world))
    assert line["frame_latency_ms"] > 0 and line["single_frame"]["frame_latency_ms"] > 0
