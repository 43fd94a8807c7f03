"""Whole-pixel paths (ORT_OPT_PIXEL_PATHS 1) against the per-bounce pipeline (0) on the
reference's own configurations and the multi-bounce bench shapes: ms per frame at one frame in
flight (device output, synchronous renders, like Raytracer::render), traced rays per second,
and the two frames compared bit for bit.

usage: python tools/pixel_paths_ab.py [name ...]     (GPU)
"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import octreeraytracer_amd as ort  # noqa: E402

# name: spheres, depth, maxSpheresPerNode, W, H, spp, bounces, use_octree
CASES = {
    "config_default": (100, 3, 0, 800, 600, 16, 8, 1),        # src/config.h:10-28
    "stats114": (1000, 5, 1, 1920, 1080, 16, 8, 1),           # analysis/stats.csv:114
    "ms0_row68": (2000, 3, 0, 800, 600, 4, 4, 1),             # stats_maxspheres0.csv:68
    "runner_10_d1_32x16": (10, 1, 1, 800, 600, 32, 16, 1),    # runner.py's worst rows for the pipeline
    "runner_1000_d10_32x16_1080": (1000, 10, 1, 1920, 1080, 32, 16, 1),
    "brute_1000_16x8_1080": (1000, -1, 1, 1920, 1080, 16, 8, 0),
    "brute_100_32x16": (100, -1, 1, 800, 600, 32, 16, 0),
    "c2_spp4_d8": (10000, 6, 0, 1920, 1080, 4, 8, 1),
    "c2_spp1_d4": (10000, 6, 0, 1920, 1080, 1, 4, 1),
    "c3tree_spp1_d4": (100000, 8, 0, 3840, 2160, 1, 4, 1),
    "c3tree_spp3_d5": (100000, 8, 0, 1920, 1080, 3, 5, 1),
    # trees between C2's (209 k nodes) and C3's (11 M): where the auto rule's 2^21-node line sits
    "mid_30k_d7_spp4_d8": (30000, 7, 0, 1920, 1080, 4, 8, 1),     # 1.48 M nodes
    "mid_100k_d7_spp4_d8": (100000, 7, 0, 1920, 1080, 4, 8, 1),   # 1.94 M nodes
    "mid_20k_d8_spp4_d8": (20000, 8, 0, 1920, 1080, 4, 8, 1),     # 5.07 M nodes
    "mid_50k_d8_spp4_d8": (50000, 8, 0, 1920, 1080, 4, 8, 1),     # 8.26 M nodes
    "mid_100k_d7_spp1_d4": (100000, 7, 0, 3840, 2160, 1, 4, 1),   # 1.94 M nodes, C3's frame shape
}


def run(name, frames=10):
    n, d, m, W, H, spp, md, oct_ = CASES[name]
    s = ort.random_spheres(n, 42)
    out = torch.empty((H, W, 3), dtype=torch.float32, device="cuda")
    p = ort.FrameParams.default_camera(W, H, num_samples=spp, max_depth=md, use_octree=oct_)
    res = {}
    with ort.Renderer(0) as r:
        if oct_:
            r.build_scene(s, d, m)
        else:
            r.upload(s, None)
        rays = r.count_traffic(p)["traversals"]
        for mode in (0, 1, 0, 1):
            r.set_pixel_paths(mode)
            for _ in range(3):
                r.render(p, out=out)  # synchronous (null stream): warm-up
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(frames):
                r.render(p, out=out)
            ms = (time.perf_counter() - t0) / frames * 1e3
            res.setdefault(mode, []).append(ms)
            img = out.cpu().numpy().copy()
            if mode == 0:
                ref = img
            else:
                same = np.array_equal(img.view(np.uint32), ref.view(np.uint32))
    a, b = min(res[0]), min(res[1])
    print(f"{name:28s} {W}x{H} spp{spp} d{md} n{n} tree{d}: pipeline {a:8.3f} ms  pixel paths {b:8.3f} ms  "
          f"x{a / b:5.2f}  {rays / b / 1e3:8.1f} Mrays/s  bit-identical {same}", flush=True)
    return a, b, same


if __name__ == "__main__":
    names = sys.argv[1:] or list(CASES)
    for nm in names:
        run(nm)
