"""Interleaved A/B timing of libort.so builds in bench.py's steady state: scene built on the
GPU, device output, each build's frames back to back on its own stream (no host sync per
frame), builds alternating in blocks of --block frames in ABBA order so clock and thermal
drift hit every build alike.  Also checks that every build writes bit-identical frames.
usage: python tools/ab_stream.py LIB_A LIB_B [...] [--config c3] [--rounds 12] [--block 10]"""
import argparse
import ctypes as C
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=12)
ap.add_argument("--block", type=int, default=10)
args = ap.parse_args()
W, H, N, D, M, NS, MD = bench.CONFIGS[args.config]
s = ort.random_spheres(N, 42)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
libs, rs, outs, sts = [], [], [], []
for path in args.libs:
    lib = C.CDLL(str(Path(path).resolve()), mode=C.RTLD_LOCAL)
    L._declare(lib)
    L._lib = lib
    r = ort.Renderer(0)
    r.build_scene(s, D, M)
    libs.append(lib)
    rs.append(r)
    outs.append(torch.empty((H, W, 3), dtype=torch.float32, device="cuda"))
    sts.append(torch.cuda.ExternalStream(r.stream_handle()))
n = len(libs)
per_frame = [[] for _ in range(n)]
trace = [[] for _ in range(n)]


def block(i, record):
    L._lib = libs[i]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.block):
        rs[i].render(p, out=outs[i], stream=sts[i].cuda_stream)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.block * 1e3
    if record:
        per_frame[i].append(dt)
        trace[i].extend(rs[i].trace_times_ms(args.block))


for i in range(n):
    block(i, False)  # warm-up
for k in range(args.rounds):
    order = list(range(n)) if k % 2 == 0 else list(reversed(range(n)))
    for i in order:
        block(i, True)
ref = outs[0].cpu().numpy().view(np.uint32)
for i in range(1, n):
    assert np.array_equal(ref, outs[i].cpu().numpy().view(np.uint32)), f"build {args.libs[i]} differs"
base = np.median(per_frame[0])
for i, path in enumerate(args.libs):
    f, tr = np.median(per_frame[i]), np.median(trace[i])
    print(f"{args.config} {Path(path).name:14s} frame {f:.4f} ms (min {np.min(per_frame[i]):.4f})  "
          f"trace {tr:.4f} ms  -> {W * H * NS / f / 1e3:.1f} Mrays/s  ({base / f:.3f}x of {Path(args.libs[0]).name})")
