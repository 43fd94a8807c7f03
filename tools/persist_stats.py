"""How the persistent bounce kernel's loop iterations go (analysis only): needs a build with
-DORT_PERSIST_STATS=1 (tools/build_variant.sh pstat -DORT_PERSIST_STATS=1).  For every
persistent launch of one frame, summed over its waves: loop iterations, refill iterations,
step iterations, and of the steps how many lanes stepped an internal node or a leaf -- a step
runs the internal-node block and the leaf block one after the other, each with only its own
lanes, so their lane shares are the walk's SIMD efficiency.
usage: python tools/persist_stats.py LIB [config] [world] [option=value ...]"""
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
for o in sys.argv[4:]:
    k, v = o.split("=")
    getattr(r, "set_" + k)(int(v))
r.build_scene(ort.random_spheres(N, 42), D, M)
tile = rank_tile(W, H, 0, world)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
NREC = 16 * 16384 * 2
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
rec = buf.cpu().numpy().astype(np.int64).reshape(-1, 8)  # a wave's two records
print(f"{cfg} world={world}: frame trace launches (ms, count): {r.frame_trace_times_ms(1)}")
nz = np.nonzero(rec[:, 0])[0]
if not len(nz):
    raise SystemExit("no records: is this an ORT_PERSIST_STATS=1 build?")
nw = int(nz[0]) if nz[0] > 0 else len(nz)  # launch 0 (the camera-ray kernel) keeps none
for seg in range(len(rec) // nw):
    R = rec[seg * nw:(seg + 1) * nw]
    R = R[R[:, 0] > 0]
    if not len(R):
        continue
    it, rf, stp, li, ll, si, sl, sb = R.sum(0)
    print(f" launch {seg}: {len(R)} waves; iterations {it} ({it / len(R):.0f}/wave): refills {rf / it:.3f}, steps "
          f"{stp / it:.3f}; per step: lanes at internal nodes {li / stp:.1f}, at leaves {ll / stp:.1f} (of 64); "
          f"steps running the internal block {si / stp:.3f}, the leaf block {sl / stp:.3f}, both {sb / stp:.3f}; "
          f"lane share of the blocks run: internal {li / max(1, 64 * si):.3f}, leaf {ll / max(1, 64 * sl):.3f}",
          flush=True)
r.close()
