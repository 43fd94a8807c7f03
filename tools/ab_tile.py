"""Interleaved A/B of the wave queue (ORT_OPT_WAVE_QUEUE) on rank 0's band tile for several
world sizes: is the 1/N-frame tile traced at 1/N of the full frame's time?  Both settings
must produce the same pixels.
usage: python tools/ab_tile.py [config] [rounds] [worlds, e.g. 1,2,4,8]"""
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
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 20
worlds = [int(x) for x in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8").split(",")]
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
r = ort.Renderer(0)
r.build_scene(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
st = torch.cuda.Stream()
torch.cuda.set_stream(st)
full = {}
for world in worlds:
    tile = rank_tile(W, H, 0, world)
    out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
    res = {q: [] for q in (0, 1)}
    ref = None
    for k in range(rounds + 2):
        for q in (0, 1):
            r.set_wave_queue(bool(q))
            r.render(p, tile, out=out, stream=st.cuda_stream)
            torch.cuda.synchronize()
            if k >= 2:
                res[q].append((r.last_kernel_ms(), r.last_trace_ms()))
            img = out.cpu().numpy()
            if ref is None:
                ref = img
            else:
                assert np.array_equal(ref.view(np.uint32), img.view(np.uint32)), (world, q)
    for q in (0, 1):
        fr = float(np.median([a for a, _ in res[q]]))
        tr = float(np.median([b for _, b in res[q]]))
        if world == worlds[0]:
            full[q] = fr * world
        eff = full[q] / world / fr if q in full else float("nan")
        print(f"{cfg} world={world} queue={q}: frame {fr:.3f} ms, trace {tr:.3f} ms, "
              f"efficiency vs world {worlds[0]} x{worlds[0]}/{world}: {eff:.2f}")
