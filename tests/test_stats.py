"""(f)4: the saveStats CSV row (src/raytracer.cpp:359-449) with the extended throughput columns
(Raytracer::statsRow, via the no-GPU driver build/stats_row) and the sweep harness that mirrors
analysis/runner.py:99-192 (tools/sweep.py)."""
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "tools"))
import sweep  # noqa: E402

EXE = ROOT / "build" / "stats_row"


def stats_row(trav, nbytes, gpus, cores, times):
    r = subprocess.run([str(EXE), str(trav), repr(float(nbytes)), str(gpus), str(cores)] + [repr(t) for t in times],
                       capture_output=True, text=True, timeout=60, check=True)
    return r.stdout.strip().splitlines()[-1]  # earlier lines: the reference's outlier report


def zfilter(times):
    t = np.asarray(times)
    sd = t.std()
    keep = t[np.abs(t - t.mean()) / sd <= 2.5] if sd > 0 else t
    return keep if keep.size else t


TIMES = [0.0019, 0.0020, 0.0021, 0.0019, 0.0020, 0.0019, 0.0020, 0.0020, 0.0019, 0.0020, 0.0050]


def test_reference_columns_and_zscore_filter():
    row = sweep.parse_row(stats_row(0, 0, 1, 1, TIMES))
    assert list(row) == sweep.REF_COLUMNS
    assert [row[c] for c in sweep.REF_COLUMNS[:8]] == [1, 100000, 8, 0, 1, 1, 3840, 2160]
    clean = zfilter(TIMES)
    assert clean.size == len(TIMES) - 1  # the 5 ms frame is the outlier
    assert row["Min"] == pytest.approx(clean.min(), rel=1e-5) and row["Max"] == pytest.approx(clean.max(), rel=1e-5)
    assert row["Avg"] == pytest.approx(clean.mean(), rel=1e-5)
    assert row["Min FPS"] == pytest.approx(1 / clean.max(), rel=1e-5)
    assert row["Avg FPS"] == pytest.approx(np.mean(1 / clean), rel=1e-5)
    assert row["Octree Build Time"] == 0.25


def test_all_equal_times_fall_back_to_unfiltered():
    # stdDev 0 makes every z-score NaN: the reference then keeps every sample (:422-434)
    row = sweep.parse_row(stats_row(0, 0, 1, 1, [0.1, 0.1, 0.1]))
    assert row["Min"] == row["Max"] == row["Avg"] == 0.1 and row["Avg FPS"] == pytest.approx(10)


def test_extended_columns():
    trav, nbytes = 3840 * 2160, 162.3e9
    row = sweep.parse_row(stats_row(trav, nbytes, 8, 16, TIMES))
    assert list(row) == sweep.REF_COLUMNS + sweep.EXT_COLUMNS
    avg = zfilter(TIMES).mean()
    assert row["mrays_per_s"] == pytest.approx(trav / avg / 1e6, rel=1e-5)
    assert row["bytes_per_ray"] == pytest.approx(nbytes / trav, rel=1e-5)
    # the reference layout's byte rate against 8 TB/s (named so: it is no roofline and exceeds 1)
    assert row["ref_layout_bytes_frac"] == pytest.approx(row["mrays_per_s"] * 1e6 * row["bytes_per_ray"] / 8e12, rel=1e-4)
    assert "roofline_fraction" not in row
    assert row["gpus"] == 8 and row["host_cores"] == 16


def test_parse_reference_csv():
    rows = sweep.parse_stats(ROOT / "tests" / "golden" / "ref_stats_rows.csv")  # reference's own rows
    assert len(rows) == 3
    assert rows[0]["Uses Octree"] == 1 and rows[0]["Spheres"] == 10 and rows[0]["Octree Build Time"] == 3.1e-06
    assert list(rows[2]) == sweep.REF_COLUMNS_13 and rows[2]["Max Octree Depth"] == -1
    with pytest.raises(ValueError):
        sweep.parse_row("1;2;3")


def test_sweep_grids_match_the_reference_runners():
    g = sweep.grid_runner()
    assert len(g) == 30 + 90  # 5 sphere counts x 3 qualities x 2 resolutions, brute force + 3 depths
    assert sum(e["USEOCTREE"] == 0 for e in g) == 30 and {e["MAXDEPTH"] for e in g} == {-1, 1, 5, 10}
    assert len(sweep.grid_maxspheres0()) == 6 * 12
    cmd = sweep.command(g[0], "s.csv", 50, 15, False, "", True)
    assert cmd[1:] == ["--spheres", "10", "--depth", "-1", "--per-node", "1", "--samples", "4", "--bounces", "4",
                       "--width", "800", "--height", "600", "--no-octree", "--frames", "50", "--warmup", "15",
                       "--stats", "s.csv", "--stats-ext"]
    c5 = sweep.command(sweep.grid_bench()[-1], "s.csv", 5, 2, True, "0,1,2,3,4,5,6,7", False)
    assert "--gpu-build" in c5 and c5[-2:] == ["--devices", "0,1,2,3,4,5,6,7"] and "--stats-ext" not in c5


def test_sweep_dry_run(capsys):
    assert sweep.main(["--grid", "maxspheres0", "--dry-run"]) == 0
    out = capsys.readouterr().out
    assert "Running 72 parameter combinations" in out and out.count("Experiment ") == 72
