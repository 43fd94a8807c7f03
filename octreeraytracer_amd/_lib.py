"""ctypes binding of libort.so (include/ort.h).

The library is built in-tree (``make lib`` / ``__graft_entry__.build()``) at
``octreeraytracer_amd/lib/libort.so``.  There is no Python or CPU fallback for the render
path: if the library (or a GPU) is missing, the calls raise.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

LIB_PATH = Path(__file__).resolve().parent / "lib" / "libort.so"
# the analysis library (Makefile `analysis`): the same kernels plus the ort_debug_* entry points
# (host emulation of the kernel's per-pixel code, walk statistics) the CPU suite and tools/ use
ANALYSIS_LIB_PATH = Path(__file__).resolve().parent / "lib" / "libort_analysis.so"

ORT_OK = 0
ORT_ERR_INVALID_ARG = 1
ORT_ERR_HIP = 2
ORT_ERR_NO_SCENE = 3
ORT_ERR_OUT_OF_MEMORY = 4
ORT_ERR_UNSUPPORTED = 5
ORT_ERR_INTERNAL = 6
ORT_ERR_TIMEOUT = 7

ORT_LAYOUT_COMPACT = 0
ORT_LAYOUT_EXPLICIT = 1
ORT_OPT_FORCE_LAYOUT = 1
ORT_OPT_EXACT_TRAVERSAL = 2
ORT_OPT_REFILL = 3
ORT_OPT_PERSISTENT = 4
ORT_OPT_SORT_PATHS = 6
ORT_OPT_XCD_SWIZZLE = 8
ORT_OPT_KID_SKIP = 9
ORT_OPT_SORT_BOUND = 10
ORT_OPT_COST_ORDER = 11
ORT_OPT_HEAVY_FIRST = 12
ORT_OPT_HEAVY_PRIO = 13
ORT_OPT_SPLIT_HEAVY = 14
ORT_OPT_SPLIT_LEVEL = 15
ORT_OPT_TILE_PAIRS = 16
ORT_OPT_DEBUG_FLAGS = 18  # analysis library only
ORT_OPT_LAUNCH_TIMES = 19
ORT_OPT_PIXEL_PATHS = 20
ORT_OPT_PIXEL_LDS_SCENE = 21
ORT_OPT_PIXEL_HEAVY_FIRST = 22
ORT_OPT_PIXEL_SPECULATE = 23
ORT_OPT_RETIRED = (5, 7, 17)  # include/ort.h ORT_OPT_IS_RETIRED: ORT_ERR_UNSUPPORTED
ORT_LAYOUT_COMPACT_EXACT_EMULATION = 2
ORT_COUNT_N = 6
COUNT_NAMES = ("nodes_popped", "child_records", "leaf_objects", "accepted_hits", "pixels", "traversals")

# Every symbol include/ort.h declares (checked by tests/test_abi.py).
EXPORTED_SYMBOLS = (
    "ort_create", "ort_destroy", "ort_last_error", "ort_set_option", "ort_upload_scene",
    "ort_upload_octree_nodes", "ort_scene_get_info", "ort_render", "ort_last_kernel_ms", "ort_last_trace_ms",
    "ort_trace_times_ms", "ort_frame_trace_times_ms", "ort_build_scene", "ort_scene_export_octree", "ort_last_build_ms", "ort_get_stream",
    "ort_count_traffic", "ort_scene_random", "ort_scene_prebuilt", "ort_scene_debug",
    "ort_octree_build", "ort_octree_sizes", "ort_octree_export", "ort_octree_nodes",
    "ort_octree_indices", "ort_octree_free", "ort_camera_view", "ort_version",
    "ort_group_create", "ort_group_destroy", "ort_group_last_error", "ort_group_size", "ort_group_context",
    "ort_group_set_option", "ort_group_upload_scene", "ort_group_build_scene", "ort_group_render",
    "ort_group_last_frame_ms", "ort_group_create_pipelined", "ort_group_frames_in_flight", "ort_group_submit",
    "ort_group_wait", "ort_group_set_timeout",
)
ORT_GROUP_TRANSPORT_RCCL = 0
ORT_GROUP_TRANSPORT_COPY = 1


class OrtParams(C.Structure):
    _fields_ = [
        ("width", C.c_int32), ("height", C.c_int32), ("num_samples", C.c_int32),
        ("max_depth", C.c_int32), ("use_octree", C.c_int32), ("view", C.c_float * 16),
        ("camera_position", C.c_float * 3), ("camera_zoom", C.c_float),
    ]


class OrtTile(C.Structure):
    _fields_ = [
        ("x0", C.c_int32), ("width", C.c_int32), ("y0", C.c_int32), ("rows", C.c_int32),
        ("band_height", C.c_int32), ("band_stride", C.c_int32),
    ]


class OrtSceneInfo(C.Structure):
    _fields_ = [
        ("n_spheres", C.c_int32), ("n_nodes", C.c_int32), ("n_indices", C.c_int64),
        ("layout", C.c_int32), ("tree_depth", C.c_int32), ("device_bytes", C.c_int64),
    ]


class OrtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"ort error {code}: {msg}")
        self.code = code


_lib = None

_fp = C.POINTER(C.c_float)
_ip = C.POINTER(C.c_int32)
_u64p = C.POINTER(C.c_uint64)
_vp = C.c_void_p


def _declare(lib, debug: str = "none"):
    """Set restype/argtypes of every include/ort.h entry point (a missing one raises), and of
    the analysis-only ort_debug_* hooks: debug "none" skips them (libort.so has none), "all"
    requires them (libort_analysis.so), "present" declares those the library has (an ORT_LIB
    override: tools/ab_stream.py loads earlier or variant builds)."""
    sig = {
        "ort_create": (C.c_int, [C.c_int, C.POINTER(_vp)]),
        "ort_destroy": (C.c_int, [_vp]),
        "ort_last_error": (C.c_char_p, [_vp]),
        "ort_set_option": (C.c_int, [_vp, C.c_int, C.c_int]),
        "ort_upload_scene": (C.c_int, [_vp, _fp, _fp, _fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip, C.c_int64]),
        "ort_upload_octree_nodes": (C.c_int, [_vp, _fp, _fp, _fp, C.c_int32, _vp, C.c_int32, _ip, C.c_int64]),
        "ort_scene_get_info": (C.c_int, [_vp, C.POINTER(OrtSceneInfo)]),
        "ort_build_scene": (C.c_int, [_vp, _fp, _fp, _fp, C.c_int32, C.c_int32, C.c_int32, C.c_int32]),
        "ort_scene_export_octree": (C.c_int, [_vp, _fp, _fp, _ip, _ip, _ip, _ip]),
        "ort_last_build_ms": (C.c_int, [_vp, _fp]),
        "ort_get_stream": (C.c_int, [_vp, C.POINTER(C.c_void_p)]),
        "ort_render": (C.c_int, [_vp, C.POINTER(OrtParams), C.POINTER(OrtTile), _vp, C.c_int, _vp]),
        "ort_last_kernel_ms": (C.c_int, [_vp, _fp]),
        "ort_last_trace_ms": (C.c_int, [_vp, _fp]),
        "ort_trace_times_ms": (C.c_int, [_vp, C.c_int, _fp]),
        "ort_frame_trace_times_ms": (C.c_int, [_vp, C.c_int, _fp, _ip]),
        "ort_count_traffic": (C.c_int, [_vp, C.POINTER(OrtParams), C.POINTER(OrtTile), _u64p]),
        "ort_scene_random": (C.c_int, [C.c_int32, C.c_uint32, _fp, _fp, _fp]),
        "ort_scene_prebuilt": (C.c_int, [_fp, _fp, _fp, _ip]),
        "ort_scene_debug": (C.c_int, [_fp, _fp, _fp, _ip]),
        "ort_octree_build": (C.c_int, [_fp, C.c_int32, C.c_int32, C.c_int32, C.POINTER(_vp)]),
        "ort_octree_sizes": (C.c_int, [_vp, C.POINTER(C.c_int64), C.POINTER(C.c_int64), C.POINTER(C.c_double)]),
        "ort_octree_export": (C.c_int, [_vp, _fp, _fp, _ip, _ip, _ip, _ip]),
        "ort_octree_nodes": (_vp, [_vp]),
        "ort_octree_indices": (_ip, [_vp]),
        "ort_octree_free": (None, [_vp]),
        "ort_camera_view": (C.c_int, [_fp, _fp, C.c_float, C.c_float, _fp]),
        "ort_version": (C.c_char_p, []),
        "ort_group_create": (C.c_int, [_ip, C.c_int32, C.c_int32, C.POINTER(_vp)]),
        "ort_group_destroy": (C.c_int, [_vp]),
        "ort_group_last_error": (C.c_char_p, [_vp]),
        "ort_group_size": (C.c_int, [_vp]),
        "ort_group_context": (C.c_int, [_vp, C.c_int32, C.POINTER(_vp)]),
        "ort_group_set_option": (C.c_int, [_vp, C.c_int, C.c_int]),
        "ort_group_upload_scene": (C.c_int, [_vp, _fp, _fp, _fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip,
                                             C.c_int64]),
        "ort_group_build_scene": (C.c_int, [_vp, _fp, _fp, _fp, C.c_int32, C.c_int32, C.c_int32]),
        "ort_group_render": (C.c_int, [_vp, C.POINTER(OrtParams), _vp, C.c_int32]),
        "ort_group_last_frame_ms": (C.c_int, [_vp, _fp]),
        "ort_group_create_pipelined": (C.c_int, [_ip, C.c_int32, C.c_int32, C.c_int32, C.POINTER(_vp)]),
        "ort_group_frames_in_flight": (C.c_int, [_vp]),
        "ort_group_submit": (C.c_int, [_vp, C.POINTER(OrtParams), _vp, C.c_int32, C.POINTER(C.c_int64)]),
        "ort_group_wait": (C.c_int, [_vp, C.c_int64]),
        "ort_group_set_timeout": (C.c_int, [_vp, C.c_int64]),
        "ort_debug_group_emulate": (C.c_int, [_fp, _fp, _fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip, C.c_int64,
                                              C.c_int32, C.POINTER(OrtParams), _fp]),
        "ort_debug_fast_order": (C.c_int, [C.c_int32, _ip, C.POINTER(C.c_uint8)]),
        "ort_debug_trace_rays": (C.c_int, [_fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip, C.c_int64, _fp,
                                           C.c_int32, C.c_int32, _ip]),
        "ort_debug_split_rays": (C.c_int, [_fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip, C.c_int64, _fp,
                                           C.c_int32, C.c_int32, C.c_int32, _ip]),
        "ort_debug_emulate_render": (C.c_int, [_fp, _fp, _fp, C.c_int32, _fp, _fp, _ip, _ip, _ip, C.c_int32, _ip,
                                               C.c_int64, C.c_int32, C.POINTER(OrtParams), C.POINTER(OrtTile),
                                               _fp, _u64p]),
    }
    for name, (res, args) in sig.items():
        if name.startswith("ort_debug_") and (debug == "none" or (debug == "present" and not hasattr(lib, name))):
            continue
        f = getattr(lib, name)
        f.restype = res
        f.argtypes = args
    if debug != "none":  # the analysis hooks ctypes callers declare themselves (tools/)
        for name in ("ort_debug_wave_stats", "ort_debug_bounce_walks", "ort_debug_walk_steps", "ort_debug_wave_clock"):
            if debug == "all":
                getattr(lib, name)


_alib = None


def lib():
    """Load libort.so (raises if it has not been built).  ORT_LIB overrides the path (A/B builds)."""
    global _lib
    if _lib is None:
        path = os.environ.get("ORT_LIB", str(LIB_PATH))
        if not Path(path).exists():
            raise OSError(f"libort.so not found at {path}: run `make lib` or __graft_entry__.build()")
        l = C.CDLL(path, mode=C.RTLD_GLOBAL)
        _declare(l, debug="present" if "ORT_LIB" in os.environ else "none")
        _lib = l
    return _lib


def analysis_lib():
    """Load libort_analysis.so, the test/analysis library (ort_debug_*: the kernel's per-pixel code
    emulated on the host, walk statistics; never on the render path).  Loaded RTLD_LOCAL beside
    libort.so; CPU processes only -- both carry the same kernel names, so a GPU process must not
    launch through both."""
    global _alib
    if _alib is None:
        if "ORT_LIB" in os.environ and hasattr(lib(), "ort_debug_emulate_render"):
            _alib = lib()  # an analysis variant given by ORT_LIB (tools/ab_stream.py, tools/*_clock.py)
            return _alib
        if not ANALYSIS_LIB_PATH.exists():
            raise OSError(f"libort_analysis.so not found at {ANALYSIS_LIB_PATH}: run `make analysis` or "
                          "__graft_entry__.build()")
        l = C.CDLL(str(ANALYSIS_LIB_PATH), mode=C.RTLD_LOCAL)
        _declare(l, debug="all")
        _alib = l
    return _alib


def check(rc: int, ctx=None):
    if rc != ORT_OK:
        msg = lib().ort_last_error(ctx)
        raise OrtError(rc, msg.decode() if msg else "")


def acheck(rc: int):
    """check() for a call into the analysis library (its own thread-error slot)."""
    if rc != ORT_OK:
        msg = analysis_lib().ort_last_error(None)
        raise OrtError(rc, msg.decode() if msg else "")


def fptr(a):
    return a.ctypes.data_as(_fp) if a is not None else None


def iptr(a):
    return a.ctypes.data_as(_ip) if a is not None else None
