"""Interleaved A/B timing of builds of libort.so in one process (e.g. the committed HEAD
build against the working tree), frames alternating so clocks/thermals hit all alike.
Also checks that all builds produce bit-identical frames.
usage: python tools/ab_libs.py LIB_A LIB_B [LIB_C ...] [--config c3] [--rounds 10]"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("libs", nargs="+")
ap.add_argument("--config", default="c3")
ap.add_argument("--rounds", type=int, default=10)
args = ap.parse_args()
paths, cfg, rounds = args.libs, args.config, args.rounds
libs = []
for p in paths:
    lib = C.CDLL(str(Path(p).resolve()), mode=C.RTLD_LOCAL)
    L._declare(lib)
    libs.append(lib)
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
L._lib = libs[0]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
rs = []
for lib in libs:
    L._lib = lib
    r = ort.Renderer(0)
    r.upload(s, t)
    rs.append(r)
outs = [np.empty((H, W, 3), np.float32) for _ in libs]
frame = [[] for _ in libs]
trace = [[] for _ in libs]
for k in range(rounds + 1):
    for i, (lib, r) in enumerate(zip(libs, rs)):
        L._lib = lib
        r.render(p, out=outs[i])
        if k > 0:  # first round = warm-up
            frame[i].append(r.last_kernel_ms())
            trace[i].append(r.last_trace_ms())
    for i in range(1, len(libs)):
        assert np.array_equal(outs[0].view(np.uint32), outs[i].view(np.uint32)), f"build {paths[i]} differs"
for i, path in enumerate(paths):
    f, tr = np.median(frame[i]), np.median(trace[i])
    print(f"{cfg} {Path(path).name:18s} frame {f:.3f} ms (min {np.min(frame[i]):.3f})  trace {tr:.3f} ms"
          f"  -> {W * H * NS / f / 1e3:.1f} Mrays/s")
for i in range(1, len(libs)):
    print(f"speedup {Path(paths[i]).name} vs {Path(paths[0]).name}: frame "
          f"{np.median(frame[0]) / np.median(frame[i]):.3f}x, trace {np.median(trace[0]) / np.median(trace[i]):.3f}x")
