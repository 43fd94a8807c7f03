"""Interleaved A/B timing of kernel variants in one process (cdna_hip_programming.md 5.4
rule 24): fast vs exact traversal (and layouts) on a bench config.
usage: python tools/ab.py [config] [rounds]"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 5
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
variants = {}
r = ort.Renderer(0)
r.upload(s, t)
out = np.empty((H, W, 3), np.float32)
ref = None
res = {"fast": [], "exact": []}
for k in range(rounds):
    for name in ("fast", "exact"):
        r.set_exact_traversal(name == "exact")
        r.render(p, out=out)
        res[name].append(r.last_kernel_ms())
        if ref is None:
            ref = out.copy()
        else:
            assert np.array_equal(ref, out), name
for name, v in res.items():
    print(f"{cfg} {name:6s} median {np.median(v):.3f} ms  min {np.min(v):.3f}  -> {W*H*NS/np.median(v)/1e3:.1f} Mrays/s")
