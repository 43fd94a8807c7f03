"""SHA-256 of the GPU builder's tree (ort_build_scene, exported whole), in the byte order
tools/make_golden.py and tools/hash_ref_tree.py hash the reference builder's output: the
36-byte GPUOctreeNode records, then objectIndices.  Needs a GPU.

usage: python tools/hash_gpu_tree.py [--n 1000000] [--depth 10] [--mspn 1] [--seed 42] [--out FILE]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import octreeraytracer_amd as ort  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--mspn", type=int, default=1)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--out", default="")
    args = ap.parse_args()
    s = ort.random_spheres(args.n, args.seed)
    with ort.Renderer(0) as r:
        r.build_scene(s, args.depth, args.mspn, keep_tree=True)
        build_ms = r.last_build_ms()
        t0 = time.time()
        t = r.export_octree()
        export_s = time.time() - t0
    t0 = time.time()
    h = hashlib.sha256()
    h.update(np.ascontiguousarray(t.gpu_records()).tobytes())
    h.update(np.ascontiguousarray(t.object_indices).tobytes())
    res = {"nodes": t.n_nodes, "indices": t.n_indices, "sha256": h.hexdigest(), "gpu_build_ms": round(build_ms, 2),
           "export_s": round(export_s, 2), "hash_s": round(time.time() - t0, 2)}
    print(json.dumps(res), flush=True)
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
