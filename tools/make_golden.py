"""Generate tests/golden/ fixtures.

Octree fixtures come from the REFERENCE's own builder (src/octree.cpp compiled from
/root/reference by oracle/Makefile into oracle/_ref/ref_octree) run on this repo's seeded
sphere sets: small trees are stored whole (.npz: 36-byte GPUOctreeNode records as int32
and objectIndices), large ones as SHA-256 + counts in manifest.json.  Image fixtures come
from the CPU oracle (oracle/ort_oracle.c) and pin it against regressions; they are not
reference outputs (the reference never reads pixels back).

usage: python tools/make_golden.py [--large]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import octreeraytracer_amd as ort  # noqa: E402
from oracle import oracle  # noqa: E402

G = ROOT / "tests" / "golden"


def sha(*arrays) -> str:
    h = hashlib.sha256()
    for a in arrays:
        h.update(np.ascontiguousarray(a).tobytes())
    return h.hexdigest()


def scene(name):
    if name == "debug":
        return ort.debug_spheres()
    if name == "prebuilt":
        return ort.prebuilt_spheres()
    n = int(name.replace("rand", "").replace("k", "000"))
    return ort.random_spheres(n, 42)


SMALL_TREES = [("debug", 3, 2), ("prebuilt", 5, 1), ("prebuilt", 3, 0), ("rand100", 3, 0), ("rand100", 4, 0),
               ("rand1000", 5, 1), ("rand1000", 4, 0)]
LARGE_TREES = [("rand10k", 6, 0), ("rand10k", 6, 1), ("rand100k", 8, 0), ("rand100k", 8, 1)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--large", action="store_true", help="also hash the 100k-sphere trees (slow)")
    args = ap.parse_args()
    if not oracle.ref_octree_available():
        raise SystemExit("oracle/_ref/ref_octree missing: build with `make ref` (needs /root/reference)")
    G.mkdir(parents=True, exist_ok=True)
    manifest = {"generator": "tools/make_golden.py", "spheres": {}, "trees": {}, "images": {}}

    for name in ("rand100", "rand1000", "rand10k", "rand100k"):
        s = scene(name)
        manifest["spheres"][name] = {"n": s.n, "seed": 42, "sha256": sha(s.center_radius, s.mat_albedo, s.fuzz_ri),
                                     "first": s.center_radius[0].tolist(), "last": s.center_radius[-1].tolist()}
    s = scene("rand100")
    np.savez(G / "spheres_rand100_seed42.npz", center_radius=s.center_radius, mat_albedo=s.mat_albedo,
             fuzz_ri=s.fuzz_ri)

    for name, d, m in SMALL_TREES + (LARGE_TREES if args.large else LARGE_TREES[:2]):
        s = scene(name)
        rec, idx, secs = oracle.ref_build_octree(s.center_radius, d, m)
        key = f"{name}_d{d}_m{m}"
        entry = {"nodes": int(rec.shape[0]), "indices": int(idx.shape[0]), "sha256": sha(rec, idx),
                 "reference_build_seconds": secs}
        if (name, d, m) in SMALL_TREES:
            np.savez(G / f"octree_{key}.npz", records=rec, indices=idx)
            entry["file"] = f"octree_{key}.npz"
        manifest["trees"][key] = entry
        print(key, entry["nodes"], entry["indices"])

    # oracle images (regression pins of the restatement)
    s = scene("rand100")
    t = ort.build_octree(s, 4, 0)
    p = ort.FrameParams.default_camera(256, 256)
    img = oracle.render(s, t, p)
    np.save(G / "image_c1_256x256.npy", img)
    manifest["images"]["c1_256x256"] = {"file": "image_c1_256x256.npy", "sha256": sha(img)}
    p2 = ort.FrameParams.default_camera(96, 64, num_samples=4, max_depth=8)
    img2 = oracle.render(s, t, p2)
    np.save(G / "image_c1_96x64_spp4_d8.npy", img2)
    manifest["images"]["c1_96x64_spp4_d8"] = {"file": "image_c1_96x64_spp4_d8.npy", "sha256": sha(img2)}
    s2 = scene("rand10k")
    t2 = ort.build_octree(s2, 6, 0)
    p3 = ort.FrameParams.default_camera(1920, 1080)
    img3 = oracle.render(s2, t2, p3, 0, 500, 1920, 40)
    manifest["images"]["c2_rows500_540"] = {"sha256": sha(img3), "x0": 0, "y0": 500, "width": 1920, "rows": 40}

    # math known answers: the canonical builtins (include/ort_math.h) at fixed points
    xs = np.array([0.0, 1e-6, 0.1, 0.5, 0.7853982, 1.0, 1.5707964, 2.0, 3.1415927, 4.0, 5.5, 6.2831855, -0.3, -2.5],
                  np.float32)
    manifest["math"] = {
        "x": xs.tolist(),
        "sin": [float(oracle.lib().oracle_sin(float(x))) for x in xs],
        "cos": [float(oracle.lib().oracle_cos(float(x))) for x in xs],
        "pow_gamma": [float(oracle.lib().oracle_pow(float(abs(x)) / 7.0, 1.0 / 2.2)) for x in xs],
    }
    manifest["rand2D"] = {f"{sx},{sy}": oracle.rand_sequence(sx, sy, 16).tolist()
                          for sx, sy in ((0.5 / 256, 0.5 / 256), (0.25, 0.75), (0.999, 0.001))}
    (G / "manifest.json").write_text(json.dumps(manifest, indent=1))
    print("wrote", G / "manifest.json")


if __name__ == "__main__":
    main()
