"""Moving-camera frames, one context, one frame at a time: per-frame GPU time (ort_last_kernel_ms)
and the trace kernels' time, against the same context's static frames, under modes
"cost order:heavy priority" (analysis).  The reprojected-hint runs of
profiles/r05_moving_*.log used the reprojection build (git history: "Cost-hint reprojection
after camera moves") with a third mode field.
usage: python tools/moving_ab.py [config] [frames] [yaw_step] [modes, e.g. 1:150,0:150,1:0]"""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd.scene import DEFAULT_YAW  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20
ys = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
with ort.Renderer(0) as r:
    r.build_scene(s, D, M)
    import torch
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    # modes: cost order[:heavy priority], comma-separated
    for mode in (sys.argv[4] if len(sys.argv) > 4 else "1:150,0:150,1:0").split(","):
        co, hp = (list(map(int, mode.split(":"))) + [150])[:2]
        r.set_cost_order(co)
        r.set_heavy_prio(hp)
        poses = [ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD, yaw=DEFAULT_YAW + ys * k)
                 for k in range(nf)]
        for p in poses[:2]:
            r.render(p, out=out)
        ms, tr = [], []
        for p in poses:
            r.render(p, out=out)
            ms.append(r.last_kernel_ms())
            tr.append(r.frame_trace_times_ms(1)[0][0])
        stat = []
        for _ in range(5):
            r.render(poses[-1], out=out)
            stat.append(r.last_kernel_ms())
        print(f"{cfg} cost order {co} heavy prio {hp}: moving frame {np.mean(ms[2:]):.4f} ms (trace {np.mean(tr[2:]):.4f}), "
              f"static {np.mean(stat[1:]):.4f} ms", flush=True)
