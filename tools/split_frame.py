"""Analysis only: does splitting ONE frame into K row parts rendered concurrently (each part on
its own context and stream) shorten the frame?  Each part's launches end in a tail of a few
long walks on an emptying GPU; another part's work can fill it.  Prints ms per frame for the
whole frame on one context and for K = 2, 3, 4 parts (contiguous row ranges), frames back to
back, and checks that the parts assemble the single-context frame bit for bit.
usage: python tools/split_frame.py [config] [frames]"""
import os
import sys
import time
from pathlib import Path

os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")  # before any HIP call: streams on their own queues
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 8
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
rs = [ort.Renderer(0) for _ in range(4)]
for r in rs:
    r.build_scene(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
full = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
streams = [torch.cuda.ExternalStream(r.stream_handle()) for r in rs]


def run(k):
    rows = [(H * i // k, H * (i + 1) // k) for i in range(k)]
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    tiles = [ort.Tile(0, W, y0, y1 - y0) for y0, y1 in rows]
    views = [out[y0:y1] for y0, y1 in rows]

    def frame():
        for i in range(k):
            rs[i].render(p, tiles[i], out=views[i], stream=streams[i].cuda_stream)

    for _ in range(2):
        frame()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(nf):
        frame()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / nf * 1e3, out


ref = None
for rep in range(2):
    for k in (1, 2, 3, 4):
        ms, img = run(k)
        if ref is None:
            ref = img.clone()
        same = bool(torch.equal(img, ref))
        print(f"{cfg} parts={k}: {ms:.3f} ms/frame  identical={same}", flush=True)
