"""The C-ABI library loads and exports every symbol include/ort.h declares (no GPU needed)."""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_symbols():
    text = (ROOT / "include" / "ort.h").read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(ort_[a-z0-9_]+)\s*\(", text)))


def test_header_lists_expected_entry_points():
    names = declared_symbols()
    for must in ("ort_create", "ort_destroy", "ort_upload_scene", "ort_render", "ort_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol(ort):
    lib = ort.lib()
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing
    from octreeraytracer_amd import _lib
    assert sorted(_lib.EXPORTED_SYMBOLS) == declared_symbols()


def test_version_and_thread_error(ort):
    lib = ort.lib()
    assert b"gfx950" in lib.ort_version()
    assert lib.ort_last_error(None) is not None


def test_octree_build_errors_cross_the_abi_as_codes(ort):
    import numpy as np
    s = ort.SphereSet.empty(0)
    with pytest.raises(ort.OrtError) as e:
        ort.build_octree(s, 3, 0)
    assert e.value.code == 1 and "Sphere list is empty" in str(e.value)  # src/octree.cpp:50-52


def test_render_without_gpu_context_fails_loudly(ort):
    """ort_create must fail with an error code (not fall back to a CPU path) when no device exists."""
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    with pytest.raises(ort.OrtError):
        ort.Renderer(0)


def test_struct_layouts_match_header(ort):
    from octreeraytracer_amd import _lib
    assert ctypes.sizeof(_lib.OrtParams) == 4 * (5 + 16 + 3 + 1)
    assert ctypes.sizeof(_lib.OrtTile) == 24


@pytest.mark.parametrize("bad", ["float16", "strided", "short"])
def test_render_rejects_a_bad_numpy_out_before_the_abi(ort, bad):
    """Renderer.render checks a numpy `out` with ValueError (not assert: it must hold under
    python -O), before anything reaches ort_render -- a wrong buffer would be overrun."""
    import numpy as np
    r = object.__new__(ort.Renderer)  # no GPU context needed: the check comes first
    r._ctx = ctypes.c_void_p()
    r._lib = None
    r.device = 0
    p = ort.FrameParams.default_camera(32, 16)
    out = {"float16": np.empty((16, 32, 3), np.float16),
           "strided": np.empty((16, 64, 3), np.float32)[:, ::2],
           "short": np.empty((15, 32, 3), np.float32)}[bad]
    with pytest.raises(ValueError):
        r.render(p, out=out)


def test_header_constants_match_the_bindings():
    """Every #define ORT_OPT_* / ORT_ERR_* / ORT_LAYOUT_* / ORT_COUNT_* in include/ort.h has the same
    value in octreeraytracer_amd/_lib.py (the options the Renderer setters pass through)."""
    from octreeraytracer_amd import _lib
    text = (ROOT / "include" / "ort.h").read_text()
    defs = dict(re.findall(r"#define\s+(ORT_(?:OPT|ERR|LAYOUT|COUNT)_[A-Z0-9_]+)\s+(-?\d+)\b", text))
    assert "ORT_OPT_COST_ORDER" in defs and "ORT_OPT_HEAVY_FIRST" in defs
    missing = [k for k in defs if not hasattr(_lib, k)]
    wrong = {k: (int(v), getattr(_lib, k)) for k, v in defs.items() if hasattr(_lib, k) and getattr(_lib, k) != int(v)}
    assert not wrong, wrong
    # every option has a binding constant (the setters use them)
    assert not [k for k in missing if k.startswith("ORT_OPT_")], missing


def test_product_library_has_no_analysis_surface(ort):
    """libort.so exports include/ort.h and nothing of the test/analysis surface: the ort_debug_*
    hooks (host emulation, walk statistics) live in libort_analysis.so (Makefile `analysis`,
    -DORT_ANALYSIS=1), which the CPU suite loads."""
    import subprocess
    from octreeraytracer_amd import _lib
    out = subprocess.run(["nm", "-D", "--defined-only", str(_lib.LIB_PATH)], capture_output=True, text=True,
                         check=True).stdout
    exported = sorted({l.split()[-1] for l in out.splitlines() if l.split()[-1].startswith("ort_")})
    assert exported == declared_symbols(), sorted(set(exported) ^ set(declared_symbols()))
    alib = _lib.analysis_lib()
    for name in ("ort_debug_emulate_render", "ort_debug_group_emulate", "ort_debug_trace_rays", "ort_debug_split_rays",
                 "ort_debug_fast_order", "ort_debug_walk_steps", "ort_debug_bounce_walks", "ort_debug_wave_stats",
                 "ort_debug_wave_clock"):
        assert hasattr(alib, name), name
        assert not hasattr(ort.lib(), name), name
