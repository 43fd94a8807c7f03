"""TEST INFRASTRUCTURE ONLY: ctypes wrapper of liboracle.so (CPU restatement of the
reference's fragment shader, see ort_oracle.c) and of _ref/ref_octree (the reference's own
src/octree.cpp).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may use it, as the checker or the timed CPU baseline -- never as the product."""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import tempfile
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
LIB = HERE / "liboracle.so"
REF_OCTREE = HERE / "_ref" / "ref_octree"

COUNT_NAMES = ("nodes_popped", "child_records", "leaf_objects", "accepted_hits", "pixels", "traversals")


class OracleScene(C.Structure):
    _fields_ = [
        ("sphere_center_radius", C.POINTER(C.c_float)), ("sphere_mat_albedo", C.POINTER(C.c_float)),
        ("sphere_fuzz_ri", C.POINTER(C.c_float)), ("n_spheres", C.c_int),
        ("node_min", C.POINTER(C.c_float)), ("node_max", C.POINTER(C.c_float)),
        ("children_offset", C.POINTER(C.c_int)), ("objects_offset", C.POINTER(C.c_int)),
        ("object_count", C.POINTER(C.c_int)), ("n_nodes", C.c_int),
        ("object_indices", C.POINTER(C.c_int)), ("n_indices", C.c_longlong),
    ]


class OracleParams(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("num_samples", C.c_int), ("max_depth", C.c_int),
        ("use_octree", C.c_int), ("view", C.c_float * 16), ("camera_position", C.c_float * 3),
        ("camera_zoom", C.c_float),
    ]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            raise OSError(f"{LIB} not built: run `make -C oracle`")
        l = C.CDLL(str(LIB))
        l.oracle_render.restype = C.c_int
        l.oracle_render.argtypes = [C.POINTER(OracleScene), C.POINTER(OracleParams), C.c_int, C.c_int, C.c_int,
                                    C.c_int, C.c_int, C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_uint64), C.c_int]
        for n in ("oracle_sin", "oracle_cos", "oracle_tan"):
            getattr(l, n).restype = C.c_float
            getattr(l, n).argtypes = [C.c_float]
        l.oracle_pow.restype = C.c_float
        l.oracle_pow.argtypes = [C.c_float, C.c_float]
        l.oracle_rand_sequence.restype = None
        l.oracle_rand_sequence.argtypes = [C.c_float, C.c_float, C.c_int, C.POINTER(C.c_float)]
        l.oracle_trace_rays.restype = None
        l.oracle_trace_rays.argtypes = [C.POINTER(OracleScene), C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_int)]
        l.oracle_traversal_order.restype = None
        l.oracle_traversal_order.argtypes = [C.c_float, C.c_float, C.c_float, C.POINTER(C.c_int)]
        l.oracle_camera.restype = C.c_int
        l.oracle_camera.argtypes = [C.POINTER(OracleParams), C.POINTER(C.c_float)]
        _lib = l
    return _lib


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float)) if a is not None else None


def _ip(a):
    return a.ctypes.data_as(C.POINTER(C.c_int)) if a is not None else None


def make_params(p) -> OracleParams:
    """From any object with the FrameParams fields."""
    o = OracleParams()
    o.width, o.height, o.num_samples, o.max_depth, o.use_octree = (int(p.width), int(p.height), int(p.num_samples),
                                                                  int(p.max_depth), int(p.use_octree))
    v = np.asarray(p.view, np.float32).reshape(16)
    for i in range(16):
        o.view[i] = float(v[i])
    for i in range(3):
        o.camera_position[i] = float(p.camera_position[i])
    o.camera_zoom = float(p.camera_zoom)
    return o


def render(spheres, tree, params, x0=0, y0=0, width=None, rows=None, band_height=0, band_stride=0,
           counts=False, threads=0):
    """Render with the oracle.  spheres: SphereSet-like (center_radius/mat_albedo/fuzz_ri);
    tree: FlatOctree-like or None.  Returns (rows, width, 3) float32 [, counts dict]."""
    width = params.width if width is None else width
    rows = params.height if rows is None else rows
    keep = [np.ascontiguousarray(spheres.center_radius, np.float32),
            np.ascontiguousarray(spheres.mat_albedo, np.float32),
            np.ascontiguousarray(spheres.fuzz_ri, np.float32)]
    sc = OracleScene()
    sc.sphere_center_radius, sc.sphere_mat_albedo, sc.sphere_fuzz_ri = _fp(keep[0]), _fp(keep[1]), _fp(keep[2])
    sc.n_spheres = keep[0].shape[0]
    if tree is not None:
        t = [np.ascontiguousarray(tree.node_min, np.float32), np.ascontiguousarray(tree.node_max, np.float32),
             np.ascontiguousarray(tree.children_offset, np.int32), np.ascontiguousarray(tree.objects_offset, np.int32),
             np.ascontiguousarray(tree.object_count, np.int32), np.ascontiguousarray(tree.object_indices, np.int32)]
        keep += t
        sc.node_min, sc.node_max = _fp(t[0]), _fp(t[1])
        sc.children_offset, sc.objects_offset, sc.object_count = _ip(t[2]), _ip(t[3]), _ip(t[4])
        sc.n_nodes = t[2].shape[0]
        sc.object_indices = _ip(t[5])
        sc.n_indices = t[5].shape[0]
    out = np.empty((rows, width, 3), np.float32)
    cnt = (C.c_uint64 * 6)() if counts else None
    pr = make_params(params)
    rc = lib().oracle_render(C.byref(sc), C.byref(pr), x0, y0, width, rows, band_height, band_stride, _fp(out),
                             cnt, threads)
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    if counts:
        return out, dict(zip(COUNT_NAMES, [int(v) for v in cnt]))
    return out


def trace_rays(spheres, tree, rays) -> np.ndarray:
    """intersectScene(ray, 0.001, MAXFLOAT) per ray (rays: (n, 6) origin, direction): (n, 2)
    int32 {hit, bits of t}."""
    keep = [np.ascontiguousarray(spheres.center_radius, np.float32),
            np.ascontiguousarray(spheres.mat_albedo, np.float32),
            np.ascontiguousarray(spheres.fuzz_ri, np.float32),
            np.ascontiguousarray(tree.node_min, np.float32), np.ascontiguousarray(tree.node_max, np.float32),
            np.ascontiguousarray(tree.children_offset, np.int32), np.ascontiguousarray(tree.objects_offset, np.int32),
            np.ascontiguousarray(tree.object_count, np.int32), np.ascontiguousarray(tree.object_indices, np.int32)]
    sc = OracleScene()
    sc.sphere_center_radius, sc.sphere_mat_albedo, sc.sphere_fuzz_ri = _fp(keep[0]), _fp(keep[1]), _fp(keep[2])
    sc.n_spheres = keep[0].shape[0]
    sc.node_min, sc.node_max = _fp(keep[3]), _fp(keep[4])
    sc.children_offset, sc.objects_offset, sc.object_count = _ip(keep[5]), _ip(keep[6]), _ip(keep[7])
    sc.n_nodes = keep[5].shape[0]
    sc.object_indices = _ip(keep[8])
    sc.n_indices = keep[8].shape[0]
    r = np.ascontiguousarray(rays, np.float32)
    out = np.zeros((len(r), 2), np.int32)
    lib().oracle_trace_rays(C.byref(sc), _fp(r), len(r), _ip(out))
    return out


def rand_sequence(sx: float, sy: float, n: int) -> np.ndarray:
    out = np.empty(n, np.float32)
    lib().oracle_rand_sequence(sx, sy, n, _fp(out))
    return out


def traversal_order(d) -> list:
    o = (C.c_int * 8)()
    lib().oracle_traversal_order(float(d[0]), float(d[1]), float(d[2]), o)
    return list(o)


def camera(params) -> np.ndarray:
    out = np.empty(22, np.float32)
    pr = make_params(params)
    lib().oracle_camera(C.byref(pr), _fp(out))
    return out


def ref_octree_available() -> bool:
    return REF_OCTREE.exists()


def ref_build_octree(center_radius: np.ndarray, max_depth: int, max_per_node: int):
    """Build with the REFERENCE's own src/octree.cpp (oracle/_ref/ref_octree).
    Returns (records (m, 9) int32, indices (k,) int32, build_seconds)."""
    if not REF_OCTREE.exists():
        raise OSError("oracle/_ref/ref_octree not built (needs /root/reference at build time)")
    cr = np.ascontiguousarray(center_radius, np.float32)
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            np.array([cr.shape[0], max_depth, max_per_node], np.int32).tofile(f)
            cr.tofile(f)
        subprocess.run([str(REF_OCTREE), fin, fout], check=True, stdout=subprocess.DEVNULL)
        with open(fout, "rb") as f:
            nn, ni = np.fromfile(f, np.int64, 2)
            secs = float(np.fromfile(f, np.float64, 1)[0])
            rec = np.fromfile(f, np.int32, int(nn) * 9).reshape(-1, 9)
            idx = np.fromfile(f, np.int32, int(ni))
    return rec, idx, secs
