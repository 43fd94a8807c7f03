"""Where a whole-pixel-paths frame's wave time goes (analysis only): needs a build with
-DORT_PIXEL_CLOCK=1 (tools/build_variant.sh pxclk -DORT_PIXEL_CLOCK=1).  Per wave of one frame's
ort_pixel_paths launch: shader-clock cycles in the refill (idle lanes taking pixels), the walk
(pixel_trace) and the rest of the bounce (hit record, shading, next ray, pixel end), loop
iterations, lanes walking per iteration, and the wave's start and end (100 MHz clock): the
spread of the wave ends is the frame's tail.
usage: python tools/pixel_clock.py LIB [config] [--samples S] [--max-depth D] [--spheres N] [--tree-depth D]"""
import argparse
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("lib")
ap.add_argument("config", nargs="?", default="ref_default")
ap.add_argument("--samples", type=int, default=0)
ap.add_argument("--max-depth", type=int, default=0)
ap.add_argument("--spheres", type=int, default=0)
ap.add_argument("--tree-depth", type=int, default=0)
ap.add_argument("--heavy-first", type=int, default=-1)
ap.add_argument("--speculate", type=int, default=-1)
args = ap.parse_args()
lib = C.CDLL(str(Path(args.lib).resolve()), mode=C.RTLD_LOCAL)
L._declare(lib, debug="present")
L._lib = lib
W, H, N, D, M, NS, MD = bench.CONFIGS[args.config]
N, D, NS, MD = args.spheres or N, args.tree_depth or D, args.samples or NS, args.max_depth or MD
r = ort.Renderer(0)
r.build_scene(ort.random_spheres(N, 42), D, M)
r.set_pixel_paths(1)
r.set_pixel_heavy_first(args.heavy_first)
r.set_pixel_speculate(args.speculate)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
tile = ort.Tile(0, W, 0, H)
out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
NREC = 2 * 65536
buf = torch.zeros((NREC, 4), dtype=torch.int64, device="cuda")
f = lib.ort_debug_wave_clock
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
for _ in range(3):
    r.render(p, tile, out=out, stream=st.cuda_stream)
assert f(r._ctx, C.c_void_p(buf.data_ptr()), NREC) == 0
r.render(p, tile, out=out, stream=st.cuda_stream)
torch.cuda.synchronize()
assert f(r._ctx, None, 0) == 0
rec = buf.cpu().numpy().astype(np.uint64).reshape(-1, 2, 4)
rec = rec[rec[:, 1, 3] == 1]
if not len(rec):
    raise SystemExit("no records: is this an ORT_PIXEL_CLOCK=1 build?")
refill, trace, shade, iters = (rec[:, 0, i].astype(np.float64) for i in range(4))
lanes = rec[:, 1, 0].astype(np.float64)
t0, t1 = rec[:, 1, 1].astype(np.int64), rec[:, 1, 2].astype(np.int64)
base = t0.min()
start, end = (t0 - base) / 100.0, (t1 - base) / 100.0  # us
tot = refill + trace + shade
ft = r.frame_trace_times_ms(1)[0]
print(f"{args.config} {W}x{H} {N} sph d{D} {NS}x{MD}: {len(rec)} waves, frame trace {ft[0]:.3f} ms in {ft[1]} launches, "
      f"the first {r.trace_times_ms(1)[0]:.3f} ms")
print(f"  wave cycles: refill {refill.sum() / tot.sum():.3f}, walk {trace.sum() / tot.sum():.3f}, "
      f"shade+rest {shade.sum() / tot.sum():.3f}")
print(f"  iterations per wave: mean {iters.mean():.0f}, p10 {np.percentile(iters, 10):.0f}, "
      f"p90 {np.percentile(iters, 90):.0f}, max {iters.max():.0f}; lanes walking per iteration {lanes.sum() / iters.sum():.1f} of 64")
print(f"  cycles per iteration: walk {trace.sum() / iters.sum():.0f}, shade+rest {shade.sum() / iters.sum():.0f}, "
      f"refill {refill.sum() / iters.sum():.0f}")
print(f"  wave ends (us): p10 {np.percentile(end, 10):.0f}, p50 {np.median(end):.0f}, p90 {np.percentile(end, 90):.0f}, "
      f"max {end.max():.0f}; starts max {start.max():.0f}")
busy = np.zeros(200)
span = end.max()
for s_, e_ in zip(start, end):
    a, b = int(s_ / span * 199), int(e_ / span * 199)
    busy[a:b + 1] += 1
q = [int(busy[int(x * 199)]) for x in (0.5, 0.8, 0.9, 0.95, 0.99)]
print(f"  waves alive at 50/80/90/95/99 % of the span: {q} (of {len(rec)})")
order = np.argsort(end)[::-1][:6]
print("  the last waves to end: end us, iterations, lanes/iteration, cycles/iteration walk / shade+rest / refill:")
for i in order:
    print(f"    {end[i]:7.0f} {iters[i]:5.0f} {lanes[i] / max(iters[i], 1):5.1f} "
          f"{trace[i] / max(iters[i], 1):8.0f} {shade[i] / max(iters[i], 1):8.0f} {refill[i] / max(iters[i], 1):8.0f}")
med = np.argsort(end)[len(end) // 2]
print(f"  the median wave: {end[med]:.0f} us, {iters[med]:.0f} iterations, {lanes[med] / max(iters[med], 1):.1f} lanes, "
      f"cycles/iteration {trace[med] / max(iters[med], 1):.0f} / {shade[med] / max(iters[med], 1):.0f} / "
      f"{refill[med] / max(iters[med], 1):.0f}")
