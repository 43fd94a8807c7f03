"""Our saveStats rows (tools/sweep.py on MI355X) beside the reference's published rows for the
same configuration (analysis/stats.csv -- runner.py's grid -- and analysis/stats_maxspheres0.csv).

The reference's rows are wall-clock frame times of its GL window loop (src/raytracer.cpp:476-519)
on the authors' GPU, synchronised to the display: frames at 6.9 ms are its 144 Hz vsync cap, not
the shader's cost.  Ours are Raytracer::run's wall time per frame (one frame in flight, the
frame left in a device buffer as the reference's is left in its framebuffer; `tools/sweep.py
--readback` times each frame with its copy to host memory as well: profiles/r06/*_readback*).

usage: python tools/sweep_compare.py OURS.csv REFERENCE.csv > table.md
"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))
import sweep  # noqa: E402

KEY = ("Uses Octree", "Spheres", "Max Octree Depth", "Num Samples", "Max Rays Depth", "Screen Width", "Screen Height")
VSYNC_MS = 7.0  # the reference's rows at or under this are display-capped (144 Hz)


def main():
    ours = sweep.parse_stats(sys.argv[1])
    ref = sweep.parse_stats(sys.argv[2])
    has_m = any("Min Spheres Per Node" in r for r in ref)
    key = (lambda r: tuple(r[k] for k in KEY) + ((r["Min Spheres Per Node"],) if has_m else ()))
    refd = {key(r): r for r in ref}
    print("| octree | spheres | depth | M | spp | bounces | W x H | ours ms | ours Mrays/s | reference ms | speed-up |")
    print("|---|---|---|---|---|---|---|---|---|---|---|")
    ratios, capped = [], 0
    for r in ours:
        x = refd.get(key(r))
        ref_ms = x["Avg"] * 1e3 if x else None
        sp = ref_ms / (r["Avg"] * 1e3) if x else None
        if x:
            ratios.append(sp)
            capped += ref_ms <= VSYNC_MS
        flag = " (vsync)" if x and ref_ms <= VSYNC_MS else ""
        print(f"| {r['Uses Octree']} | {r['Spheres']} | {r['Max Octree Depth']} | {r['Min Spheres Per Node']} | "
              f"{r['Num Samples']} | {r['Max Rays Depth']} | {r['Screen Width']}x{r['Screen Height']} | "
              f"{r['Avg'] * 1e3:.3f} | {r.get('mrays_per_s', float('nan')):.1f} | "
              f"{'-' if not x else f'{ref_ms:.2f}{flag}'} | {'-' if not x else f'{sp:.1f}x'} |")
    if ratios:
        import math
        g = math.exp(sum(math.log(v) for v in ratios) / len(ratios))
        print(f"\n{len(ratios)} rows matched: speed-up min {min(ratios):.2f}x, geometric mean {g:.1f}x, "
              f"max {max(ratios):.1f}x; {capped} reference rows at the display cap (<= {VSYNC_MS} ms)")


if __name__ == "__main__":
    main()
