"""Render --warm + N frames of a bench config with only the production kernels, then (untimed) the
counting pass: the command profiled by tools/profile_box.sh under rocprofv3 PMC passes.
--meta writes {frames, traversals_per_frame, lib_sha} for tools/summarize_profile.py."""
import argparse
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--config", default="c3")
ap.add_argument("--frames", type=int, default=3)
ap.add_argument("--warm", type=int, default=1,
                help="frames rendered first and left out of the PMC sums (the cost order's first frame "
                     "has no previous-frame costs; bench.py's timed frames all do)")
ap.add_argument("--layout", type=int, default=-1)
ap.add_argument("--meta", default="", help="write frames / traversals / build id here (JSON)")
a = ap.parse_args()
W, H, N, D, M, NS, MD = bench.CONFIGS[a.config]
s = ort.random_spheres(N, 42)
r = ort.Renderer(0)
r.set_layout(a.layout)
r.build_scene(s, D, M)  # GPU octree builder (same tree as the host builder)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = np.empty((H, W, 3), np.float32)
ms = []
for _ in range(a.warm + a.frames):
    r.render(p, out=out)
    ms.append(r.last_kernel_ms())
print(f"{a.config} layout={r.info()['layout']} kernel ms: {['%.3f' % m for m in ms]}", flush=True)
if a.meta:
    counts = r.count_traffic(p)  # COUNT=true kernel instances: excluded from the PMC sums by name
    Path(a.meta).write_text(json.dumps({"config": a.config, "frames": a.frames,
                                        "warm_frames": a.warm,
                                        "traversals_per_frame": counts["traversals"], "counts": counts,
                                        "lib_sha": bench.lib_sha(), "device_sha": bench.device_sha(), "tile_rows": H}))
r.close()
