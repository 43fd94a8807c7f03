"""One Renderer option at several values on one context, interleaved (ABAB... blocks of frames),
one frame in flight (device output, synchronous renders): ms per frame (best block, median)
and whether every value renders the first value's frame bit for bit.

usage: python tools/opt_ab.py CASE SETTER V1 V2 [...] [--rounds R] [--block B]
  CASE: a tools/pixel_paths_ab.py case or a bench.py config; SETTER: a Renderer set_* name
  without the prefix (e.g. pixel_lds_scene 1 0)."""
import argparse
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import torch  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from pixel_paths_ab import CASES  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("case")
    ap.add_argument("setter")
    ap.add_argument("values", nargs="+", type=int)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--block", type=int, default=10)
    a = ap.parse_args()
    if a.case in CASES:
        n, d, m, W, H, spp, md, oct_ = CASES[a.case]
    else:
        W, H, n, d, m, spp, md = bench.CONFIGS[a.case]
        oct_ = 1
    s = ort.random_spheres(n, 42)
    p = ort.FrameParams.default_camera(W, H, num_samples=spp, max_depth=md, use_octree=oct_)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    times = {v: [] for v in a.values}
    same = {v: True for v in a.values}
    ref = None
    with ort.Renderer(0) as r:
        if oct_:
            r.build_scene(s, d, m)
        else:
            r.upload(s, None)
        setter = getattr(r, "set_" + a.setter)
        for k in range(a.rounds):
            for v in (a.values if k % 2 == 0 else a.values[::-1]):
                setter(v)
                for _ in range(2):
                    r.render(p, out=out)  # warm-up of this setting
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(a.block):
                    r.render(p, out=out)
                times[v].append((time.perf_counter() - t0) / a.block * 1e3)
                img = out.cpu().numpy()
                if ref is None:
                    ref = img.copy()
                same[v] = same[v] and np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    base = min(times[a.values[0]])
    for v in a.values:
        print(f"{a.case} {a.setter}={v}: best {min(times[v]):.4f} ms  median {np.median(times[v]):.4f} ms  "
              f"x{base / min(times[v]):.3f} of {a.values[0]}  bit-identical {same[v]}", flush=True)


if __name__ == "__main__":
    main()
