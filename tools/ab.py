"""Interleaved A/B timing of kernel variants in one process (cdna_hip_programming.md 5.4
rule 24): frames of the variants alternate, and every variant must produce the same pixels.
usage: python tools/ab.py [config] [rounds] [variant,variant,...]
variants: exact (GLSL min/max walk), lane (the defaults: per-lane walk for camera rays,
persistent refill kernel for bounces >= 1), laneonly (per-lane walk everywhere), packet (wave-level walk
for camera rays), nosort (bounce paths compacted but not coherence-sorted), refillN
(persistent trace, refill threshold N), bounceN (persistent only for bounces >= 1)."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
names = sys.argv[3].split(",") if len(sys.argv) > 3 else ["exact", "lane", "packet", "refill16"]


def settings(name):
    s = {"exact": False, "refill": 0, "packet": False, "sort": True, "pmode": 1}
    if name == "exact":
        s["exact"] = True
    elif name == "packet":
        s["packet"] = True
    elif name == "nosort":
        s["sort"] = False
    elif name.startswith("refill"):
        s["refill"] = int(name[6:])
    elif name.startswith("bounce"):  # persistent kernel for the bounce >= 1 lists only
        s["refill"], s["pmode"] = int(name[6:]), 2
    elif name not in ("lane", "laneonly"):
        raise SystemExit(f"unknown variant {name}")
    return s


W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
r = ort.Renderer(0)
r.build_scene(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = np.empty((H, W, 3), np.float32)
ref = None
res = {n: [] for n in names}
tr = {n: [] for n in names}
for k in range(rounds + 1):
    for name in names:
        v = settings(name)
        r.set_exact_traversal(v["exact"])
        r.set_packet(v["packet"])
        r.set_sort_paths(v["sort"])
        r.set_persistent(v["pmode"] if v["refill"] > 0 else (2 if name == "lane" else 0))
        if v["refill"] > 0:
            r.set_refill(v["refill"])
        r.render(p, out=out)
        if k > 0:  # round 0 = warm-up
            res[name].append(r.last_kernel_ms())
            tr[name].append(r.last_trace_ms())
        if ref is None:
            ref = out.copy()
        else:
            assert np.array_equal(ref.view(np.uint32), out.view(np.uint32)), name
for name in names:
    v = res[name]
    print(f"{cfg} {name:9s} frame median {np.median(v):.3f} ms (min {np.min(v):.3f}; first trace {np.median(tr[name]):.3f})"
          f" -> {W*H*NS/np.median(v)/1e3:.1f} Mcamera-rays/s")
