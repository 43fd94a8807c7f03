"""Per-wave timeline of the persistent bounce kernel (analysis only): needs a build with
-DORT_PERSIST_CLOCK=1 (tools/build_variant.sh pclk -DORT_PERSIST_CLOCK=1).  For every
persistent launch of one frame: the span, when the item queue ran dry (the first wave that
found it empty), and how long the drain tail lasted -- the part of the launch in which waves
only finish their last walks, with ever fewer lanes busy.
usage: python tools/persist_clock.py LIB [config] [world]"""
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
cfg = sys.argv[2] if len(sys.argv) > 2 else "c5"
world = int(sys.argv[3]) if len(sys.argv) > 3 else 1
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
r = ort.Renderer(0)
r.build_scene(ort.random_spheres(N, 42), D, M)
tile = rank_tile(W, H, 0, world)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
NREC = 16 * 16384
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
rec = buf.cpu().numpy().astype(np.uint64)
ft = r.frame_trace_times_ms(1)
print(f"{cfg} world={world}: frame trace launches (ms, count): {ft}")
# records: launch seg occupies [seg * nw, (seg + 1) * nw); find the ranges with data
nz = np.nonzero(rec[:, 2])[0]
if not len(nz):
    raise SystemExit("no records: is this an ORT_PERSIST_CLOCK=1 build?")
# waves per launch (nw): launch seg's records start at seg * nw, and launch 0 (the camera
# rays' per-tile kernel) keeps none, so the first record sits at nw
nw = int(nz[0]) if nz[0] > 0 else len(nz)
for seg in range(NREC // nw):
    R = rec[seg * nw:(seg + 1) * nw]
    R = R[R[:, 2] > 0]
    if not len(R):
        continue
    t0, td, t1 = (R[:, 0].astype(np.int64), R[:, 1].astype(np.int64), R[:, 2].astype(np.int64))
    base = t0.min()
    a, d, b = (t0 - base) / 100.0, (td - base) / 100.0, (t1 - base) / 100.0  # us (100 MHz)
    items = (R[:, 3] >> 8).astype(np.int64)
    dry = d[td > 0].min() if (td > 0).any() else float("nan")
    span = b.max()
    busy_after = np.clip(b - dry, 0, None).sum()  # wave-us spent after the queue ran dry
    print(f" launch {seg}: {len(R)} waves, {items.sum()} items, span {span:.0f} us, queue dry at {dry:.0f} us, "
          f"tail {span - dry:.0f} us ({(span - dry) / span * 100:.1f} %); wave ends: p10 {np.percentile(b, 10):.0f} "
          f"p50 {np.median(b):.0f} p90 {np.percentile(b, 90):.0f} us; wave starts max {a.max():.0f} us; "
          f"mean busy share of the tail {busy_after / max(1e-9, len(R) * (span - dry)):.2f}")
