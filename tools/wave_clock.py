"""Per-block timeline of the wave-queue trace kernel (analysis only, ort_debug_wave_clock):
each 64-slot block's start/end (s_memrealtime, 100 MHz) and the CU it ran on, for rank 0's
band tile of an N-GPU frame.  Shows whether a small tile's trace time is set by the tail
(a few long blocks started late), by slow ramp-up, or by blocks running slower overall.
usage: python tools/wave_clock.py [config] [world] [out.npy]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd.distributed import rank_tile  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
world = int(sys.argv[2]) if len(sys.argv) > 2 else 8
dump = sys.argv[3] if len(sys.argv) > 3 else None
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
r = ort.Renderer(0)
r.build_scene(s, D, M)
r.set_wave_queue(True)
tile = rank_tile(W, H, 0, world)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
nrec = (tile.rows + 15) // 16 * ((W + 15) // 16) * 4
buf = torch.zeros((nrec, 4), dtype=torch.int64, device="cuda")
f = r._lib.ort_debug_wave_clock
f.restype = C.c_int
f.argtypes = [C.c_void_p, C.c_void_p, C.c_int64]
for _ in range(3):
    r.render(p, tile, out=out, stream=st.cuda_stream)
assert f(r._ctx, C.c_void_p(buf.data_ptr()), nrec) == 0
r.render(p, tile, out=out, stream=st.cuda_stream)
torch.cuda.synchronize()
assert f(r._ctx, None, 0) == 0
rec = buf.cpu().numpy().astype(np.uint64)
ok = rec[:, 1] > 0
rec = rec[ok]
t0 = rec[:, 0].astype(np.int64)
t1 = rec[:, 1].astype(np.int64)
base = t0.min()
a, b = (t0 - base) / 100.0, (t1 - base) / 100.0  # us
dur = b - a
hw = rec[:, 2].astype(np.int64)
cu = (hw >> 8) & 15
se = (hw >> 13) & 7
xcc = rec[:, 3].astype(np.int64) & 15
print(f"{cfg} world={world}: {ok.sum()} blocks, kernel span {b.max():.1f} us (trace event {r.last_trace_ms() * 1e3:.1f} us)")
print(f"block duration us: mean {dur.mean():.1f} p50 {np.median(dur):.1f} p90 {np.percentile(dur, 90):.1f} "
      f"p99 {np.percentile(dur, 99):.1f} max {dur.max():.1f}")
print(f"last block start {a.max():.1f} us; blocks ending after 0.8*span: {(b > 0.8 * b.max()).sum()}")
edges = np.linspace(0, b.max(), 21)
act = [int(((a <= x) & (b > x)).sum()) for x in edges[:-1]]
print("concurrent blocks (waves busy) over time:", act)
for x in range(8):
    m = xcc == x
    if m.any():
        print(f"  xcc {x}: blocks {m.sum()}, last end {b[m].max():.1f} us, busy-sum {dur[m].sum():.0f} us")
if dump:
    np.save(dump, np.stack([a, b, cu + 16 * se, xcc], 1))
