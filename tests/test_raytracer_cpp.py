"""The C++ Raytracer drop-in (octreeraytracer_amd/csrc/raytracer.{h,cpp}) through the
example entry point build/ort_main (the reference's src/main.cpp flow)."""
import subprocess
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
EXE = ROOT / "build" / "ort_main"


def read_ppm(path):
    data = Path(path).read_bytes()
    parts = data.split(b"\n", 3)
    w, h = map(int, parts[1].split())
    return np.frombuffer(parts[3], np.uint8).reshape(h, w, 3)


def test_example_binary_built():
    assert EXE.exists(), "make examples"


@pytest.mark.gpu
@pytest.mark.parametrize("gpu_build,readback", [(False, False), (True, False), (False, True)])
def test_main_renders_and_writes_stats(ort, oracle, tmp_path, gpu_build, readback):
    """run()'s timed frames into a device frame (default: the reference's frames stay in its GL
    framebuffer) or copied to the host (--readback); then the --ppm frame against the oracle."""
    csv, ppm = tmp_path / "stats.csv", tmp_path / "frame.ppm"
    cmd = [str(EXE), "--spheres", "100", "--depth", "4", "--samples", "1", "--bounces", "1", "--width", "64",
           "--height", "48", "--frames", "3", "--warmup", "1", "--stats", str(csv), "--ppm", str(ppm)]
    cmd += ["--gpu-build"] if gpu_build else []
    cmd += ["--readback"] if readback else []
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    row = csv.read_text().strip().split(";")
    assert len(row) == 15 and row[:8] == ["1", "100", "4", "0", "1", "1", "64", "48"]  # saveStats schema
    s = ort.random_spheres(100, 42)
    t = ort.build_octree(s, 4, 0)
    ref = oracle.render(s, t, ort.FrameParams.default_camera(64, 48))
    from octreeraytracer_amd.image import to_srgb8
    assert np.array_equal(read_ppm(ppm), to_srgb8(ref)[::-1])


@pytest.mark.gpu
def test_main_device_group(ort, oracle, tmp_path):
    """Raytracer over an ort_group (cfg.devices): the frame is banded over the group's contexts
    and gathered to devices[0]; on a one-GPU box device 0 is listed three times (the group then
    gathers by device copies -- RCCL needs distinct devices)."""
    ppm = tmp_path / "frame.ppm"
    cmd = [str(EXE), "--spheres", "1000", "--depth", "5", "--per-node", "1", "--samples", "2", "--bounces", "3",
           "--width", "160", "--height", "100", "--frames", "2", "--warmup", "1", "--devices", "0,0,0", "--ppm", str(ppm)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    s = ort.random_spheres(1000, 42)
    t = ort.build_octree(s, 5, 1)
    ref = oracle.render(s, t, ort.FrameParams.default_camera(160, 100, num_samples=2, max_depth=3))
    from octreeraytracer_amd.image import to_srgb8
    assert np.array_equal(read_ppm(ppm), to_srgb8(ref)[::-1])


@pytest.mark.gpu
def test_sweep_extended_rows(tmp_path):
    """tools/sweep.py drives ort_main over grid points; each run appends a 20-column row."""
    import sys
    sys.path.insert(0, str(ROOT / "tools"))
    import sweep
    csv = tmp_path / "stats.csv"
    for grid in ("bench", "runner"):  # C1 (octree) and the runner's first point (brute force, 4 spp x 4 bounces)
        rc = sweep.main(["--grid", grid, "--limit", "1", "--frames", "4", "--warmup", "1", "--out", str(csv),
                         "--timeout", "120"])
        assert rc == 0
    rows = sweep.parse_stats(csv)
    assert len(rows) == 2 and all(len(r) == 20 for r in rows)
    c1, bf = rows
    assert (c1["Uses Octree"], c1["Spheres"], c1["Screen Width"]) == (1, 100, 256)
    assert c1["mrays_per_s"] * 1e6 * c1["Avg"] == pytest.approx(256 * 256, rel=1e-3)  # one traversal per pixel
    assert c1["bytes_per_ray"] > 12 and c1["gpus"] == 1 and c1["host_cores"] >= 1
    assert (bf["Uses Octree"], bf["Max Octree Depth"], bf["Num Samples"]) == (0, -1, 4)
    assert bf["mrays_per_s"] > 0
