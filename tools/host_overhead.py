"""Host-side cost of ort_render (enqueue only) vs GPU time per frame, device output.
usage: python tools/host_overhead.py [config] [frames]"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 100
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
r = ort.Renderer(0)
r.upload(s, t)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()  # not the null stream (handle 0 = synchronous, see bench.py)
torch.cuda.set_stream(st)
for _ in range(5):
    r.render(p, out=out, stream=st.cuda_stream)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
t0 = time.perf_counter()
e0.record(st)
for _ in range(n):
    r.render(p, out=out, stream=st.cuda_stream)
e1.record(st)
t1 = time.perf_counter()
torch.cuda.synchronize()
t2 = time.perf_counter()
print(f"{cfg}: enqueue {1e3 * (t1 - t0) / n:.3f} ms/frame, wall {1e3 * (t2 - t0) / n:.3f} ms/frame, "
      f"gpu span {e0.elapsed_time(e1) / n:.3f} ms/frame, last frame pipeline {r.last_kernel_ms():.3f} ms, "
      f"trace {r.last_trace_ms():.3f} ms")
