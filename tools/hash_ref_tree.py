"""Pin a large tree to the REFERENCE builder by SHA-256 (test infrastructure).

Runs oracle/_ref/ref_octree (the reference's own src/octree.cpp, compiled from
/root/reference by oracle/Makefile) on a seeded sphere set and hashes its output without
holding it in memory: the dump is written to a temporary file and streamed through SHA-256
(the 36-byte GPUOctreeNode records, then objectIndices -- the same byte sequence
tools/make_golden.py's sha(records, indices) hashes).  The entry is merged into
tests/golden/manifest.json under "trees" with "hash_only": true, so that
tests/test_gpu_build.py leaves it to tests/test_gpu_c5.py (which exports the C5 tree once).

usage: python tools/hash_ref_tree.py [--n 1000000] [--depth 10] [--mspn 1] [--seed 42] [--key rand1M_d10_m1]
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import resource
import struct
import subprocess
import sys
import tempfile
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import octreeraytracer_amd as ort  # noqa: E402
from oracle import oracle  # noqa: E402

MANIFEST = ROOT / "tests" / "golden" / "manifest.json"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--depth", type=int, default=10)
    ap.add_argument("--mspn", type=int, default=1)
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--key", default="rand1M_d10_m1")
    ap.add_argument("--tmp", default="/tmp")
    ap.add_argument("--out", default="", help="also write the entry to this JSON file (a GPU box's gpurun_out/: "
                    "the build needs ~60 GB of host memory, more than this container has)")
    ap.add_argument("--no-manifest", action="store_true", help="do not merge into tests/golden/manifest.json")
    ap.add_argument("--verify", action="store_true", help="compare with the manifest's entry for --key, write nothing")
    args = ap.parse_args()
    if not oracle.ref_octree_available():
        raise SystemExit("oracle/_ref/ref_octree missing: build with `make -C oracle ref` (needs /root/reference)")
    s = ort.random_spheres(args.n, args.seed)
    cr = np.ascontiguousarray(s.center_radius, np.float32)
    with tempfile.TemporaryDirectory(dir=args.tmp) as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            np.array([cr.shape[0], args.depth, args.mspn], np.int32).tofile(f)
            cr.tofile(f)
        t0 = time.time()
        proc = subprocess.Popen([str(oracle.REF_OCTREE), fin, fout], stdout=subprocess.DEVNULL)
        while proc.poll() is None:  # a heartbeat: the build is silent for minutes
            try:
                proc.wait(timeout=30)
            except subprocess.TimeoutExpired:
                print(f"reference build running, {time.time() - t0:.0f} s", flush=True)
        if proc.returncode != 0:
            raise SystemExit(f"ref_octree failed with status {proc.returncode}")
        wall = time.time() - t0
        peak_gb = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 2**20
        h = hashlib.sha256()
        with open(fout, "rb") as f:
            nn, ni, secs = struct.unpack("<qqd", f.read(24))
            while True:
                b = f.read(1 << 26)
                if not b:
                    break
                h.update(b)
    entry = {"nodes": int(nn), "indices": int(ni), "sha256": h.hexdigest(), "reference_build_seconds": secs,
             "reference_wall_seconds": round(wall, 1), "reference_peak_rss_gb": round(peak_gb, 1),
             "spheres": {"n": args.n, "seed": args.seed, "sha256": hashlib.sha256(
                 cr.tobytes() + np.ascontiguousarray(s.mat_albedo).tobytes()
                 + np.ascontiguousarray(s.fuzz_ri).tobytes()).hexdigest()},
             "hash_only": True}
    if args.out:
        Path(args.out).parent.mkdir(parents=True, exist_ok=True)
        Path(args.out).write_text(json.dumps({args.key: entry}, indent=1))
    m = json.loads(MANIFEST.read_text())
    if args.verify:
        old = m["trees"][args.key]
        ok = all(old[k] == entry[k] for k in ("nodes", "indices", "sha256"))
        print(args.key, "matches the manifest" if ok else "DIFFERS from the manifest", entry["sha256"])
        raise SystemExit(0 if ok else 1)
    m["trees"][args.key] = entry
    if not args.no_manifest:
        MANIFEST.write_text(json.dumps(m, indent=1))
    print(args.key, json.dumps(entry))


if __name__ == "__main__":
    main()
