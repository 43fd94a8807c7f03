"""Per-wave timeline of the per-tile camera-ray kernel (analysis only): needs a build with
-DORT_TILE_CLOCK=1 (tools/build_variant.sh tclk -DORT_TILE_CLOCK=1).  Renders rank 0's band
tile of a `world`-GPU frame with one frame in flight and reports, for the last frame, the
kernel span, when waves start and end, and how the longest waves relate to their longest
walk -- what sets the single-frame tail of a small tile.
usage: python tools/tile_clock.py LIB [config] [world] [frames] [option=value ...]  (Renderer setters)"""
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
from octreeraytracer_amd.distributed import rank_tile  # noqa: E402

lib = C.CDLL(str(Path(sys.argv[1]).resolve()), mode=C.RTLD_LOCAL)
L._declare(lib, debug="present")
L._lib = lib
cfg = sys.argv[2] if len(sys.argv) > 2 else "c3"
world = int(sys.argv[3]) if len(sys.argv) > 3 else 8
frames = int(sys.argv[4]) if len(sys.argv) > 4 else 5
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
r = ort.Renderer(0)
for o in sys.argv[5:]:
    k, v = o.split("=")
    getattr(r, "set_" + k)(int(v))
r.build_scene(ort.random_spheres(N, 42), D, M)
tile = rank_tile(W, H, 0, world)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
nw = ((W + 15) // 16) * ((tile.rows + 15) // 16) * 4 + 1024  # + ort_trace_split's records at the end
buf = torch.zeros((nw, 4), dtype=torch.int64, device="cuda")
f = lib.ort_debug_wave_clock
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
for _ in range(3):
    r.render(p, tile, out=out, stream=st.cuda_stream)
torch.cuda.synchronize()
for fr in range(frames):
    buf.zero_()
    assert f(r._ctx, C.c_void_p(buf.data_ptr()), nw) == 0
    r.render(p, tile, out=out, stream=st.cuda_stream)
    torch.cuda.synchronize()
    assert f(r._ctx, None, 0) == 0
    rec = buf.cpu().numpy().astype(np.int64)
    sp = rec[:, 2] < 0  # ort_trace_split's records (bit 63 set), written from the end
    if sp.any():
        S = rec[sp]
        sbase = rec[(rec[:, 1] > 0)][:, 0].min()
        print(f"  split kernel: {len(S)} waves, {int(S[:, 3].sum())} rays, starts {(S[:, 0].min() - sbase) / 100:.0f} us, "
              f"ends max {(S[:, 1].max() - sbase) / 100:.0f} us (wave us max {(S[:, 1] - S[:, 0]).max() / 100:.0f})",
              flush=True)
    rec[sp] = 0
    ok = rec[:, 1] > 0
    if not ok.any():
        raise SystemExit("no records: is this an ORT_TILE_CLOCK=1 build?")
    R = rec[ok]
    base = R[:, 0].min()
    a, b = (R[:, 0] - base) / 100.0, (R[:, 1] - base) / 100.0  # us (s_memrealtime: 100 MHz)
    dur = b - a
    steps = R[:, 3]
    span = b.max()
    ft = r.frame_trace_times_ms(1)[0][0]
    late = b >= np.percentile(b, 99)
    print(f"{cfg} world={world} frame {fr}: {len(R)} waves, kernel span {span:.0f} us (HIP events {ft * 1e3:.0f} us); "
          f"starts p50 {np.median(a):.0f} p90 {np.percentile(a, 90):.0f} max {a.max():.0f} us; "
          f"ends p50 {np.median(b):.0f} p90 {np.percentile(b, 90):.0f} p99 {np.percentile(b, 99):.0f} us; "
          f"wave us p50 {np.median(dur):.0f} p99 {np.percentile(dur, 99):.0f} max {dur.max():.0f}; "
          f"longest walk per wave p50 {np.median(steps):.0f} p99 {np.percentile(steps, 99):.0f} max {steps.max()}; "
          f"last 1 % of waves to end: start p50 {np.median(a[late]):.0f} us, lasted p50 {np.median(dur[late]):.0f} us, "
          f"longest walk p50 {np.median(steps[late]):.0f}", flush=True)
    # workgroups (4 consecutive records): a workgroup holds its LDS until its slowest wave ends
    g = rec[: len(rec) // 4 * 4].reshape(-1, 4, 4)
    gok = (g[:, :, 1] > 0).all(1)
    gd = (g[gok, :, 1] - g[gok, :, 0]) / 100.0
    idle = (gd.max(1)[:, None] - gd).sum() / (4 * gd.max(1)).sum()
    print(f"  workgroups: {int(gok.sum())}, wave-slot time idle inside them (waiting for their slowest wave) "
          f"{idle:.3f}; slowest/mean wave per workgroup p50 {np.median(gd.max(1) / gd.mean(1)):.2f}", flush=True)
    # busy waves over time (10 us bins)
    bins = np.arange(0, span + 10, 10)
    busy = [int(((a <= t) & (b > t)).sum()) for t in bins]
    print("  resident waves every 10 us:", busy, flush=True)
r.close()
