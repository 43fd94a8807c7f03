"""octreeraytracer_amd -- MI355X-native octree sphere ray tracer (gfx950).

A drop-in for the GPU path of Tiago27Cruz/OctreeRayTracer: the reference's scene-build
API (Sphere / Octree / GPUOctreeNode, BFS layout) is kept, and its OpenGL fragment-shader
tracer (shaders/octree_fragment_shader.glsl) is replaced by a hand-written HIP kernel
behind the C ABI of include/ort.h (libort.so).
"""
from ._lib import ORT_ERR_TIMEOUT, OrtError, lib
from .renderer import FrameParams, Renderer, Tile, algorithmic_bytes
from .scene import (FlatOctree, SphereSet, build_octree, camera_view, debug_spheres, prebuilt_spheres,
                    random_spheres)

__all__ = ["ORT_ERR_TIMEOUT", "OrtError", "lib", "FrameParams", "Renderer", "Tile", "algorithmic_bytes", "FlatOctree", "SphereSet",
           "build_octree", "camera_view", "debug_spheres", "prebuilt_spheres", "random_spheres"]
__version__ = "0.1.0"
