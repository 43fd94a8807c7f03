"""The torch RCCL transport bench.py's N>1 path uses (backend "nccl" = RCCL), run for real on the
one-GPU box: a one-rank process group initialised exactly as bench.py does (device_id,
timeout), then FrameGather's gather calls -- the synchronous dist.gather and the async one
submit() issues, waited on as finish() waits -- moving a rendered band tile through RCCL into
rank 0's receive slot, de-interleaved by assemble(); the frame must equal a direct render bit
for bit.  (FrameGather itself skips the gather at world 1; the N>1 band logic is covered by the
gloo tests and the one-GPU rehearsals, test_gpu_bench_ranks.py.  RCCL refuses two ranks on one
device, so distinct devices stay the driver's scaling run.)"""
import os
import socket
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parents[1]

SCRIPT = r"""
import sys
from datetime import timedelta
import numpy as np
import torch
import torch.distributed as dist
sys.path.insert(0, sys.argv[1])
import octreeraytracer_amd as ort
from octreeraytracer_amd.distributed import assemble, rank_tile

torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), timeout=timedelta(seconds=60))
assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
W, H = 640, 360
s = ort.random_spheres(2000, 42)
with ort.Renderer(0) as r:
    r.build_scene(s, 5, 1)
    p = ort.FrameParams.default_camera(W, H, num_samples=2, max_depth=3)
    want = r.render(p)
    tile = rank_tile(W, H, 0, 1)
    local = torch.full((tile.rows, W, 3), -1.0, dtype=torch.float32, device="cuda")
    r.render(p, tile, out=local, stream=torch.cuda.current_stream().cuda_stream)
    for asynchronous in (False, True):
        slot = torch.full((1, tile.rows, W, 3), -2.0, dtype=torch.float32, device="cuda")
        work = dist.gather(local, list(slot.unbind(0)), dst=0, async_op=asynchronous)
        if asynchronous:
            work.wait(timeout=timedelta(seconds=30))
        frame = assemble(slot, H, 1)
        got = frame.cpu().numpy()
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), asynchronous
dist.barrier()
dist.destroy_process_group()
print("rccl gather ok")
"""


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def test_rccl_gather_one_rank():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", SCRIPT, str(ROOT)], capture_output=True, text=True, env=env,
                       timeout=110)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout[-1000:]
    assert "rccl gather ok" in r.stdout
