"""bench.py's record-keeping helpers (CPU only).

* device_sha: the hash a PMC record is keyed by covers the gfx950 code objects' instructions
  and kernel descriptors only, so the same sources built in another directory (where the
  compilation-unit id, derived from the source path, changes the code objects' symbol strings)
  hash alike, while any change of device code does not.
* sample_rows: the CPU baseline's row sample spans the whole frame height for every sample
  size (an integer stride collapsed to 1 beyond half the height and sampled the first rows only).
"""
import hashlib
import shutil
import subprocess
from pathlib import Path

import pytest

import bench

ROOT = Path(__file__).resolve().parents[1]
HIPCC = "/opt/rocm/bin/hipcc"
FLAGS = ["-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-w"]


def _fatbin_sha(path):
    return hashlib.sha256(bench._elf_sections(Path(path).read_bytes())[".hip_fatbin"]).hexdigest()[:16]


@pytest.mark.skipif(not Path(HIPCC).exists(), reason="hipcc not installed")
def test_device_sha_is_build_path_independent(tmp_path):
    # the smallest HIP translation unit of the library, compiled once by a relative path from a
    # copy of the tree and once by an absolute path from another directory
    src = ROOT / "octreeraytracer_amd" / "csrc"
    a, b = tmp_path / "a", tmp_path / "b" / "deeper"
    for d in (a, b):
        shutil.copytree(src, d / "pkg" / "csrc")  # (the sources include ../../include/ort.h)
        shutil.copytree(ROOT / "include", d / "include")
    libs = []
    for d, srcpath in ((a, "pkg/csrc/group.hip"), (b, str(b / "pkg" / "csrc" / "group.hip"))):
        obj = d / "group.o"
        subprocess.run([HIPCC, *FLAGS, "-c", srcpath, "-o", str(obj)], cwd=d, check=True)
        lib = d / "libg.so"
        subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(lib), str(obj), "-ldl"],
                       cwd=d, check=True)
        libs.append(lib)
    assert len(bench.gfx950_code_objects(libs[0].read_bytes())) == 1
    # the whole fatbin differs (compilation-unit id), the device code does not
    assert _fatbin_sha(libs[0]) != _fatbin_sha(libs[1])
    assert bench.device_sha(libs[0]) == bench.device_sha(libs[1]) != ""
    # ... and a change of device code changes it
    (b / "pkg" / "csrc" / "group.hip").write_text((b / "pkg" / "csrc" / "group.hip").read_text().replace(
        "d[i] = s[i];", "d[i] = s[i] + 0.0f * (float)y;"))
    subprocess.run([HIPCC, *FLAGS, "-c", "pkg/csrc/group.hip", "-o", "group2.o"], cwd=b, check=True)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", "libg2.so", "group2.o", "-ldl"],
                   cwd=b, check=True)
    assert bench.device_sha(b / "libg2.so") != bench.device_sha(libs[0])


def test_device_sha_of_the_shipped_library_matches_its_code_objects():
    lib = ROOT / "octreeraytracer_amd" / "lib" / "libort.so"
    if not lib.exists():
        pytest.skip("libort.so not built")
    cos = bench.gfx950_code_objects(lib.read_bytes())
    assert len(cos) == 3  # ort_kernel.hip, gpu_build.hip, group.hip
    assert all(bench._elf_sections(co)[".text"] for co in cos)
    assert len(bench.device_sha()) == 16


@pytest.mark.parametrize("height", [7, 100, 1080, 2160, 4320])
def test_sample_rows_spans_the_frame(height):
    for n in sorted({1, 2, 3, height // 3, height // 2, height // 2 + 1, (2 * height) // 3, height - 1, height,
                     height + 5}):
        y0, rows, bh, bs = bench.sample_rows(height, n)
        ys = [y0 + (j // bh) * bs + j % bh for j in range(rows)]
        assert len(set(ys)) == rows and min(ys) >= 0 and max(ys) < height, (height, n)
        want = max(1, min(n, height))
        assert abs(rows - want) <= max(2, want // 10), (height, n, rows)  # about the asked size
        if want >= 4:  # evenly spread: rows in both the bottom and the top eighth of the frame
            assert min(ys) < height / 8 + bs and max(ys) >= height * 7 / 8 - bs, (height, n, ys[:3], ys[-3:])


@pytest.mark.parametrize("pixels,split_ok,pairs,split", [
    (3840 * 2160, True, True, False),   # full C3 frame: tile pairs
    (3840 * 1080, True, True, False),   # 1/2 band (> 2^21 px)
    (3840 * 544, True, False, True),    # 1/4 band: split walks at one frame in flight
    (3840 * 272, True, False, True),    # 1/8 band
    (3840 * 272, False, True, False),   # frames in flight: split walks off, pairs
])
def test_trace_kernel_names_follow_the_tile_rules(pixels, split_ok, pairs, split):
    """The roofline's kernel list names what render_impl launches by default (tile pairs above
    2^21 px or with split walks off, split walks at or below it)."""
    names = bench.trace_kernel_names("c3", {"tree_depth": 8, "n_nodes": 10_953_681}, 1, 1, pixels, split_ok=split_ok)
    assert names[0].startswith("ort_trace_pair<" if pairs else "ort_trace_compact<")
    assert any(n.startswith("ort_trace_split<false, 1>") for n in names) == split
    deep = bench.trace_kernel_names("c5", {"tree_depth": 10, "n_nodes": 239_220_401}, 4, 1, 7680 * 4320)
    assert deep[0].startswith("ort_trace_pair_deep<false, 2>") and deep[-1].startswith("ort_trace_persistent<false, true>")
    # the reference's default config (a 585-node tree, 16 x 8): whole-pixel paths, one kernel
    small = bench.trace_kernel_names("ref_default", {"tree_depth": 3, "n_nodes": 585}, 8, 16, 800 * 600)
    assert len(small) == 3 and small[0].startswith("ort_pixel_paths<0, false, ..., 1>")  # samples in parallel
    assert small[1].startswith("ort_sample_resolve") and small[2].startswith("ort_pixel_paths<0, false, ..., 2>")
    one = bench.trace_kernel_names("c2", {"tree_depth": 6, "n_nodes": 209_000}, 4, 1, 1920 * 1080)
    assert one == [one[0]] and one[0].startswith("ort_pixel_paths<0, false>")  # one sample: whole pixels
