"""Deferred bounce rays of a frame (ANALYSIS-ONLY, ort_debug_defer_probe): per trace launch
the number of rays the fast walk could not take and what they look like (zero / denormal
direction components, |d|^2 outside the fast walk's [1/8, 8], non-finite values).
usage: python tools/defer_probe.py [config] [cap]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
cap = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
r = ort.Renderer(0)
r.build_scene(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=max(MD, 4))
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
r.render(p, out=out)
buf = torch.zeros((16, 1 + 2 * cap, 4), dtype=torch.float32, device="cuda")
f = r._lib.ort_debug_defer_probe
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int32]
assert f(r._ctx, C.c_void_p(buf.data_ptr()), cap) == 0
r.render(p, out=out)
torch.cuda.synchronize()
assert f(r._ctx, None, 0) == 0
b = buf.cpu().numpy()
for seg in range(16):
    n = int(b[seg, 0, 0].view(np.int32))
    if n == 0 and not b[seg, 1:].any():
        continue
    k = min(n, cap)
    o = b[seg, 1:1 + 2 * k:2, :3]
    d = b[seg, 2:2 + 2 * k:2, :3]
    dd = (d.astype(np.float64) ** 2).sum(1)
    zero = (np.abs(d) < 1.1754944e-38).any(1)
    nonfin = ~np.isfinite(d).all(1) | ~np.isfinite(o).all(1)
    print(f"launch {seg}: {n} deferred; of {k}: zero/denormal dir comp {zero.sum()}, |d|^2<1/8 {(dd < 0.125).sum()}, "
          f"|d|^2>8 {(dd > 8).sum()}, non-finite {nonfin.sum()}")
    for i in range(min(k, 6)):
        print("   o", o[i].tolist(), "d", d[i].tolist())
