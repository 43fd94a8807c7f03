"""Host scene-build stage (kept reference API) through libort.so.

Mirrors the reference's CPU side:
  * ``random_spheres``   -- Raytracer::generateRandomSpheres (src/raytracer.cpp:254-337),
                            seeded std::mt19937 instead of std::random_device.
  * ``prebuilt_spheres`` -- Raytracer::generatePreBuiltSpheres (src/raytracer.cpp:164-252).
  * ``debug_spheres``    -- the DEBUG scene (src/raytracer.cpp:342-347).
  * ``build_octree``     -- Octree(maxDepth, maxSpheresPerNode).build (src/octree.cpp:47-95),
                            returned in the flattened BFS layout (setGPUData, :268-312).
  * ``camera_view``      -- Camera::GetViewMatrix (src/opengl/camera.h:64-67, 115-126).
All arrays are numpy; the arithmetic runs in the C++ library.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib as L

# Camera pose of the reference's main() (src/main.cpp:34-39): position, yaw, pitch, zoom.
DEFAULT_CAMERA_POSITION = (0.0, 2.5, -10.0)
DEFAULT_YAW = -90.0
DEFAULT_PITCH = 0.0
DEFAULT_ZOOM = 45.0
WORLD_UP = (0.0, 1.0, 0.0)

LAMBERT, METAL, DIELECTRIC = 0, 1, 2


@dataclass
class SphereSet:
    """SoA packing of setupBuffers (src/raytracer.cpp:87-91): three (n, 4) float32 arrays."""

    center_radius: np.ndarray
    mat_albedo: np.ndarray
    fuzz_ri: np.ndarray

    @property
    def n(self) -> int:
        return int(self.center_radius.shape[0])

    @staticmethod
    def empty(n: int) -> "SphereSet":
        return SphereSet(np.zeros((n, 4), np.float32), np.zeros((n, 4), np.float32), np.zeros((n, 4), np.float32))

    @staticmethod
    def from_arrays(centers, radii, materials, albedo, fuzz, refraction_index) -> "SphereSet":
        n = len(radii)
        s = SphereSet.empty(n)
        s.center_radius[:, :3] = np.asarray(centers, np.float32).reshape(n, 3)
        s.center_radius[:, 3] = np.asarray(radii, np.float32)
        s.mat_albedo[:, 0] = np.asarray(materials, np.float32)
        s.mat_albedo[:, 1:] = np.asarray(albedo, np.float32).reshape(n, 3)
        s.fuzz_ri[:, 0] = np.asarray(fuzz, np.float32)
        s.fuzz_ri[:, 1] = np.asarray(refraction_index, np.float32)
        return s


def random_spheres(n: int, seed: int = 42) -> SphereSet:
    s = SphereSet.empty(n)
    L.check(L.lib().ort_scene_random(n, seed & 0xFFFFFFFF, L.fptr(s.center_radius), L.fptr(s.mat_albedo),
                                     L.fptr(s.fuzz_ri)))
    return s


def _fixed(fn) -> SphereSet:
    n = C.c_int32(0)
    L.check(fn(None, None, None, C.byref(n)))
    s = SphereSet.empty(n.value)
    L.check(fn(L.fptr(s.center_radius), L.fptr(s.mat_albedo), L.fptr(s.fuzz_ri), C.byref(n)))
    return s


def prebuilt_spheres() -> SphereSet:
    return _fixed(L.lib().ort_scene_prebuilt)


def debug_spheres() -> SphereSet:
    return _fixed(L.lib().ort_scene_debug)


@dataclass
class FlatOctree:
    """Octree::flattenedTree + objectIndices in SoA form (int32 offsets)."""

    node_min: np.ndarray         # (m, 3) float32
    node_max: np.ndarray         # (m, 3) float32
    children_offset: np.ndarray  # (m,) int32, -1 for leaves
    objects_offset: np.ndarray   # (m,) int32, -1 for empty leaves / internal nodes
    object_count: np.ndarray     # (m,) int32
    object_indices: np.ndarray   # (k,) int32
    build_seconds: float = 0.0
    max_depth: int = 0
    max_spheres_per_node: int = 0

    @property
    def n_nodes(self) -> int:
        return int(self.children_offset.shape[0])

    @property
    def n_indices(self) -> int:
        return int(self.object_indices.shape[0])

    def gpu_records(self) -> np.ndarray:
        """The 36-byte GPUOctreeNode AoS records (src/octree.h:24-30) as an (m, 9) int32 view."""
        rec = np.empty((self.n_nodes, 9), np.int32)
        rec[:, 0:3] = self.node_min.view(np.int32)
        rec[:, 3:6] = self.node_max.view(np.int32)
        rec[:, 6] = self.children_offset
        rec[:, 7] = self.objects_offset
        rec[:, 8] = self.object_count
        return rec

    @staticmethod
    def from_gpu_records(rec: np.ndarray, indices: np.ndarray) -> "FlatOctree":
        rec = np.ascontiguousarray(rec, np.int32).reshape(-1, 9)
        return FlatOctree(rec[:, 0:3].copy().view(np.float32), rec[:, 3:6].copy().view(np.float32),
                          rec[:, 6].copy(), rec[:, 7].copy(), rec[:, 8].copy(),
                          np.ascontiguousarray(indices, np.int32))


def build_octree(spheres: SphereSet, max_depth: int, max_spheres_per_node: int = 0) -> FlatOctree:
    lib = L.lib()
    h = C.c_void_p()
    cr = np.ascontiguousarray(spheres.center_radius, np.float32)
    L.check(lib.ort_octree_build(L.fptr(cr), spheres.n, max_depth, max_spheres_per_node, C.byref(h)))
    try:
        nn, ni, secs = C.c_int64(), C.c_int64(), C.c_double()
        L.check(lib.ort_octree_sizes(h, C.byref(nn), C.byref(ni), C.byref(secs)))
        m, k = nn.value, ni.value
        t = FlatOctree(np.empty((m, 3), np.float32), np.empty((m, 3), np.float32), np.empty(m, np.int32),
                       np.empty(m, np.int32), np.empty(m, np.int32), np.empty(k, np.int32), secs.value,
                       max_depth, max_spheres_per_node)
        L.check(lib.ort_octree_export(h, L.fptr(t.node_min), L.fptr(t.node_max), L.iptr(t.children_offset),
                                      L.iptr(t.objects_offset), L.iptr(t.object_count), L.iptr(t.object_indices)))
        return t
    finally:
        lib.ort_octree_free(h)


def camera_view(position=DEFAULT_CAMERA_POSITION, yaw: float = DEFAULT_YAW, pitch: float = DEFAULT_PITCH,
                world_up=WORLD_UP) -> np.ndarray:
    pos = np.asarray(position, np.float32)
    up = np.asarray(world_up, np.float32)
    out = np.empty(16, np.float32)
    L.check(L.lib().ort_camera_view(L.fptr(pos), L.fptr(up), yaw, pitch, L.fptr(out)))
    return out
