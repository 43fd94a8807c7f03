"""Interleaved A/B timing of kernel variants in one process (cdna_hip_programming.md 5.4
rule 24).  Variants: exact walk, per-lane walk, packet walk, persistent-trace refill thresholds.
usage: python tools/ab.py [config] [rounds] [refill,refill,...]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
refills = [int(x) for x in sys.argv[3].split(",")] if len(sys.argv) > 3 else [16]
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
r = ort.Renderer(0)
r.upload(s, t)
out = np.empty((H, W, 3), np.float32)
ref = None
# (name, exact walk, persistent refill threshold or 0, packet walk for camera rays)
variants = [("exact", True, 0, False), ("lane", False, 0, False), ("packet", False, 0, True)] + \
    [(f"refill{f}", False, f, False) for f in refills]
res = {v[0]: [] for v in variants}
tr = {v[0]: [] for v in variants}
for k in range(rounds):
    for name, exact, f, pk in variants:
        r.set_exact_traversal(exact)
        r.set_packet(pk)
        r.set_persistent(f > 0)
        if f > 0:
            r.set_refill(f)
        r.render(p, out=out)
        res[name].append(r.last_kernel_ms())
        tr[name].append(r.last_trace_ms())
        if ref is None:
            ref = out.copy()
        else:
            assert np.array_equal(ref, out), name
for name in res:
    v = res[name]
    print(f"{cfg} {name:9s} frame median {np.median(v):.3f} ms (min {np.min(v):.3f}; first trace {np.median(tr[name]):.3f})"
          f" -> {W*H*NS/np.median(v)/1e3:.1f} Mrays/s")
