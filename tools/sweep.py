#!/usr/bin/env python3
"""Experiment sweep over the reference's parameter grids, on runtime knobs.

The reference sweeps configurations by regex-editing `src/config.h`, recompiling and running
the GL binary once per point (`analysis/runner.py:16-97`, grids at `:99-192`;
`runner_maxspheres0.py:99-160`); each run appends one `saveStats` row
(`src/raytracer.cpp:441-446`) to the CSV named by OUTPUTFILE.  Here every point is one run of
`build/ort_main` (the reference's `main()` flow on libort.so, `examples/main.cpp`) with the
knobs as flags -- nothing is rebuilt -- and `--stats-ext` appends the five throughput columns
(`Raytracer::statsRow`, octreeraytracer_amd/csrc/raytracer.h) to the reference's fifteen.

    python tools/sweep.py --grid runner --out stats.csv            # analysis/runner.py's 120 points
    python tools/sweep.py --grid maxspheres0 --out stats_ms0.csv   # runner_maxspheres0.py's 72 points
    python tools/sweep.py --grid bench --devices 0,1,2,3,4,5,6,7    # C1-C5 (BASELINE.json), 8 GPUs
    python tools/sweep.py --grid runner --dry-run                  # list the commands only

`parse_stats(path)` reads such a CSV (either width, with or without the reference's header
line, also the reference's older 13-column files) into dicts keyed by column name.
"""
from __future__ import annotations

import argparse
import subprocess
import sys
import time
from itertools import product
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "build" / "ort_main"

# column names of the reference's CSV header (analysis/stats_maxspheres0.csv, 15 columns),
# then the extended columns (SURVEY.md 5 "Metrics")
REF_COLUMNS = ["Uses Octree", "Spheres", "Max Octree Depth", "Min Spheres Per Node", "Num Samples",
               "Max Rays Depth", "Screen Width", "Screen Height", "Min", "Max", "Avg", "Min FPS", "Max FPS",
               "Avg FPS", "Octree Build Time"]
# the reference's older files (analysis/stats.csv, stats_2.csv): no per-node count, no build time
REF_COLUMNS_13 = [c for c in REF_COLUMNS if c not in ("Min Spheres Per Node", "Octree Build Time")]
EXT_COLUMNS = ["mrays_per_s", "bytes_per_ray", "ref_layout_bytes_frac", "gpus", "host_cores"]
INT_COLUMNS = {"Uses Octree", "Spheres", "Max Octree Depth", "Min Spheres Per Node", "Num Samples", "Max Rays Depth",
               "Screen Width", "Screen Height", "gpus", "host_cores"}

# config.h parameter -> ort_main flag (booleans: flag present when the value is 0 / 1)
FLAGS = {"NUMSPHERES": "--spheres", "MAXDEPTH": "--depth", "MAXSPHERESPERNODE": "--per-node",
         "NUMSAMPLES": "--samples", "MAXRAYSDEPTH": "--bounces", "SCR_WIDTH": "--width", "SCR_HEIGHT": "--height"}


def grid_runner() -> list[dict]:
    """analysis/runner.py:99-169: brute force and octree depths 1/5/10 over spheres x quality x resolution."""
    base = {"COLLECTSTATS": 1, "DEBUG": 0, "USEPREBUILT": 0, "MAXSPHERESPERNODE": 1}
    resolutions = [{"SCR_WIDTH": 800, "SCR_HEIGHT": 600}, {"SCR_WIDTH": 1920, "SCR_HEIGHT": 1080}]
    spheres = [10, 100, 250, 500, 1000]
    quality = [{"NUMSAMPLES": 4, "MAXRAYSDEPTH": 4}, {"NUMSAMPLES": 16, "MAXRAYSDEPTH": 8},
               {"NUMSAMPLES": 32, "MAXRAYSDEPTH": 16}]
    out = []
    for n, q, r in product(spheres, quality, resolutions):
        out.append({**base, "USEOCTREE": 0, "NUMSPHERES": n, "MAXDEPTH": -1, **r, **q})
    for n, q, r in product(spheres, quality, resolutions):
        for d in (1, 5, 10):
            out.append({**base, "USEOCTREE": 1, "NUMSPHERES": n, "MAXDEPTH": d, **r, **q})
    return out


def grid_maxspheres0() -> list[dict]:
    """runner_maxspheres0.py:99-150: octree depth 0-5 x maxSpheresPerNode 0/1, 800x600, 4 spp, 4 bounces."""
    base = {"COLLECTSTATS": 1, "DEBUG": 0, "USEPREBUILT": 0, "SCR_WIDTH": 800, "SCR_HEIGHT": 600,
            "NUMSAMPLES": 4, "MAXRAYSDEPTH": 4}
    return [{**base, "USEOCTREE": 1, "NUMSPHERES": n, "MAXDEPTH": d, "MAXSPHERESPERNODE": m}
            for n in (10, 50, 250, 500, 1000, 2000) for d, m in product(range(6), (0, 1))]


def grid_bench() -> list[dict]:
    """BASELINE.json configs C1-C5 (C4 = C3 on several GPUs: pass --devices)."""
    base = {"COLLECTSTATS": 1, "DEBUG": 0, "USEPREBUILT": 0, "USEOCTREE": 1}
    return [{**base, "NUMSPHERES": n, "MAXDEPTH": d, "MAXSPHERESPERNODE": m, "SCR_WIDTH": w, "SCR_HEIGHT": h,
             "NUMSAMPLES": 1, "MAXRAYSDEPTH": b}
            for n, d, m, w, h, b in ((100, 4, 0, 256, 256, 1), (10_000, 6, 0, 1920, 1080, 1),
                                     (100_000, 8, 0, 3840, 2160, 1), (1_000_000, 10, 1, 7680, 4320, 4))]


GRIDS = {"runner": grid_runner, "maxspheres0": grid_maxspheres0, "bench": grid_bench}


def command(exp: dict, out: str, frames: int, warmup: int, gpu_build: bool, devices: str, extended: bool,
            exe: Path = EXE, readback: bool = False) -> list[str]:
    """The ort_main command line of one experiment (the config.h edit + rebuild of runner.py:16-72)."""
    cmd = [str(exe)]
    for k, flag in FLAGS.items():
        if k in exp:
            cmd += [flag, str(exp[k])]
    if not exp.get("USEOCTREE", 1):
        cmd.append("--no-octree")
    if exp.get("USEPREBUILT", 0):
        cmd.append("--prebuilt")
    if exp.get("DEBUG", 0):
        cmd.append("--debug")
    cmd += ["--frames", str(frames), "--warmup", str(warmup)]
    if exp.get("COLLECTSTATS", 1):
        cmd += ["--stats", out] + (["--stats-ext"] if extended else [])
    if gpu_build:
        cmd.append("--gpu-build")
    if devices:
        cmd += ["--devices", devices]
    if readback:
        cmd.append("--readback")
    return cmd


def run_experiment(cmd: list[str], timeout: float) -> bool:
    """runner.py:74-97: run with a timeout, report failure and go on."""
    try:
        r = subprocess.run(cmd, timeout=timeout)
    except subprocess.TimeoutExpired:
        print(f"Execution timed out after {timeout} seconds", flush=True)
        return False
    if r.returncode != 0:
        print(f"Experiment failed (exit {r.returncode})", flush=True)
    return r.returncode == 0


def _num(col: str, v: str):
    v = v.strip()
    return int(v) if col in INT_COLUMNS else float(v)


def parse_row(line: str) -> dict:
    """One ';' row of 13 (older reference files), 15 (saveStats) or 20 (--stats-ext) columns."""
    fields = [f for f in line.strip().split(";")]
    names = {13: REF_COLUMNS_13, 15: REF_COLUMNS, 20: REF_COLUMNS + EXT_COLUMNS}.get(len(fields))
    if names is None:
        raise ValueError(f"stats row has {len(fields)} columns (expected 13, 15 or 20): {line!r}")
    return {c: _num(c, v) for c, v in zip(names, fields)}


def parse_stats(path) -> list[dict]:
    rows = []
    for line in Path(path).read_text().splitlines():
        if not line.strip() or line.startswith("Uses Octree"):  # blank or the reference's header line
            continue
        rows.append(parse_row(line))
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--grid", default="runner", choices=sorted(GRIDS))
    ap.add_argument("--out", default="stats.csv", help="the CSV every run appends its row to (OUTPUTFILE)")
    ap.add_argument("--frames", type=int, default=50, help="timed frames per run (the reference: 50)")
    ap.add_argument("--warmup", type=int, default=15, help="warm-up frames per run (src/raytracer.cpp:455)")
    ap.add_argument("--timeout", type=float, default=500, help="seconds per run (runner.py:184)")
    ap.add_argument("--gpu-build", action="store_true", help="build each octree with ort_build_scene")
    ap.add_argument("--devices", default="", help="e.g. 0,1,2,3,4,5,6,7: render every point on an ort_group")
    ap.add_argument("--readback", action="store_true",
                    help="time every frame with its copy to host memory (default: frames stay on the device, "
                         "as the reference's stay in its GL framebuffer)")
    ap.add_argument("--reference-columns", action="store_true", help="write the reference's 15 columns only")
    ap.add_argument("--dry-run", action="store_true", help="print the commands, run nothing")
    ap.add_argument("--limit", type=int, default=0, help="run only the first N points")
    args = ap.parse_args(argv)
    exps = GRIDS[args.grid]()
    if args.limit:
        exps = exps[:args.limit]
    print(f"Running {len(exps)} parameter combinations", flush=True)
    failed = 0
    for i, exp in enumerate(exps):
        cmd = command(exp, args.out, args.frames, args.warmup, args.gpu_build, args.devices,
                      not args.reference_columns, readback=args.readback)
        print(f"Experiment {i + 1}/{len(exps)}: {' '.join(cmd[1:])}", flush=True)
        if args.dry_run:
            continue
        if not EXE.exists():
            sys.exit(f"{EXE} is missing: make examples")
        t0 = time.time()
        ok = run_experiment(cmd, args.timeout)
        failed += not ok
        print(f"  {'ok' if ok else 'FAILED'} in {time.time() - t0:.1f} s", flush=True)
    if not args.dry_run and Path(args.out).exists():
        rows = parse_stats(args.out)
        print(f"{args.out}: {len(rows)} rows", flush=True)
    return 1 if failed else 0


if __name__ == "__main__":
    sys.exit(main())
