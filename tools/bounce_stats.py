"""Analysis only: where a multi-bounce frame goes, per bounce -- traversals, node pops and leaf
objects per ray (ort_count_traffic at max_depth 1..B, differenced) and each trace launch's
HIP-event time (ort_frame_trace_times_ms of frames rendered at max_depth 1..B, differenced),
under the renderer options given.
usage: python tools/bounce_stats.py [config] [option=value ...]   (options: Renderer setters)"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
MD = max(MD, 4)
r = ort.Renderer(0)
for o in sys.argv[2:]:
    k, v = o.split("=")
    getattr(r, "set_" + k)(int(v))
t0 = time.time()
r.build_scene(ort.random_spheres(N, 42), D, M)
print(f"{cfg}: scene in {time.time() - t0:.1f} s", flush=True)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.ExternalStream(r.stream_handle())
prev_c, prev_t = None, None
for b in range(1, MD + 1):
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=b)
    c = r.count_traffic(p)
    for _ in range(3):
        r.render(p, out=out, stream=st.cuda_stream)
    torch.cuda.synchronize()
    nf = 5
    for _ in range(nf):
        r.render(p, out=out, stream=st.cuda_stream)
    torch.cuda.synchronize()
    fr = r.frame_trace_times_ms(nf)
    tt = float(np.median([f[0] for f in fr]))
    d = {k: c[k] - (prev_c[k] if prev_c else 0) for k in c}
    dt = tt - (prev_t or 0.0)
    n = max(d["traversals"], 1)
    print(f"bounce {b - 1}: rays {d['traversals'] / 1e6:7.2f} M  trace {dt:7.3f} ms  "
          f"{d['traversals'] / dt / 1e3:7.1f} Mrays/s  pops/ray {d['nodes_popped'] / n:6.1f}  "
          f"child recs/ray {d['child_records'] / n:6.1f}  leaf objs/ray {d['leaf_objects'] / n:6.1f}  "
          f"hits {d['accepted_hits'] / n:.3f}  (frame trace total {tt:.3f} ms, launches {fr[-1][1]})", flush=True)
    prev_c, prev_t = c, tt
