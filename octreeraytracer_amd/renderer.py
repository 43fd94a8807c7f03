"""Device renderer: the GL path of the reference replaced by the gfx950 kernel (libort.so).

``Renderer`` owns one ort_ctx (one GPU).  ``upload`` = setupBuffers (src/raytracer.cpp:74-152),
``render`` = the per-frame uniforms + glDrawArrays (src/raytracer.cpp:491-499) followed by a
read of the frame (the reference never reads pixels back; this returns them).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

import numpy as np

from . import _lib as L
from .scene import (DEFAULT_CAMERA_POSITION, DEFAULT_PITCH, DEFAULT_YAW, DEFAULT_ZOOM, FlatOctree, SphereSet,
                    camera_view)


@dataclass
class FrameParams:
    """The shader uniforms (glsl:13-18, 48-53)."""

    width: int
    height: int
    num_samples: int = 1
    max_depth: int = 1
    use_octree: int = 1
    view: np.ndarray = field(default_factory=lambda: camera_view())
    camera_position: tuple = DEFAULT_CAMERA_POSITION
    camera_zoom: float = DEFAULT_ZOOM

    def to_c(self) -> L.OrtParams:
        p = L.OrtParams()
        p.width, p.height = int(self.width), int(self.height)
        p.num_samples, p.max_depth, p.use_octree = int(self.num_samples), int(self.max_depth), int(self.use_octree)
        v = np.asarray(self.view, np.float32).reshape(16)
        for i in range(16):
            p.view[i] = float(v[i])
        for i in range(3):
            p.camera_position[i] = float(self.camera_position[i])
        p.camera_zoom = float(self.camera_zoom)
        return p

    @staticmethod
    def default_camera(width, height, num_samples=1, max_depth=1, use_octree=1, position=DEFAULT_CAMERA_POSITION,
                       yaw=DEFAULT_YAW, pitch=DEFAULT_PITCH, zoom=DEFAULT_ZOOM) -> "FrameParams":
        return FrameParams(width, height, num_samples, max_depth, use_octree, camera_view(position, yaw, pitch),
                           tuple(position), zoom)


@dataclass
class Tile:
    """Rows/columns to render; see ort_tile in include/ort.h.  Output row j is pixel row
    y0 + (j // band_height) * band_stride + j % band_height (GL rows: y = 0 at the bottom)."""

    x0: int
    width: int
    y0: int
    rows: int
    band_height: int = 0
    band_stride: int = 0

    @staticmethod
    def full(p: FrameParams) -> "Tile":
        return Tile(0, p.width, 0, p.height)

    def to_c(self) -> L.OrtTile:
        t = L.OrtTile()
        t.x0, t.width, t.y0, t.rows = int(self.x0), int(self.width), int(self.y0), int(self.rows)
        t.band_height, t.band_stride = int(self.band_height), int(self.band_stride)
        return t

    def pixel_rows(self, height: int) -> np.ndarray:
        j = np.arange(self.rows)
        y = self.y0 + (j // self.band_height) * self.band_stride + j % self.band_height if self.band_height > 0 \
            else self.y0 + j
        return y


class Renderer:
    def __init__(self, device: int = 0):
        self._lib = L.lib()
        self._ctx = C.c_void_p()
        L.check(self._lib.ort_create(device, C.byref(self._ctx)))
        self.device = device

    # -- lifecycle -------------------------------------------------------------------
    def close(self):
        if self._ctx:
            self._lib.ort_destroy(self._ctx)
            self._ctx = C.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        L.check(rc, self._ctx)

    # -- scene -----------------------------------------------------------------------
    def set_layout(self, layout: int):
        """Force ORT_LAYOUT_COMPACT / ORT_LAYOUT_EXPLICIT (-1 = auto) for the next upload."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_FORCE_LAYOUT, int(layout)))

    def set_exact_traversal(self, on: bool):
        """Disable (True) / enable the sign-specialised fast walk; pixels are identical either way."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_EXACT_TRAVERSAL, int(bool(on))))

    def set_launch_times(self, on: int):
        """ORT_OPT_LAUNCH_TIMES: 1 (default) times every trace launch (last_trace_ms, trace_times_ms);
        0 times only the frame (last_kernel_ms) -- fewer event packets per frame; same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_LAUNCH_TIMES, int(on)))

    def set_pixel_paths(self, mode: int):
        """ORT_OPT_PIXEL_PATHS: -1 (default) auto, 0 the per-bounce pipeline, 1 whole-pixel paths in one
        launch wherever they apply (same pixels)."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_PIXEL_PATHS, int(mode)))

    def set_pixel_lds_scene(self, on: int):
        """ORT_OPT_PIXEL_LDS_SCENE: 1 (default) small scenes walked from LDS copies in whole-pixel paths."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_PIXEL_LDS_SCENE, int(on)))

    def set_pixel_speculate(self, mode: int):
        """ORT_OPT_PIXEL_SPECULATE: whole-pixel paths trace a pixel's samples in parallel from last
        frame's per-sample RNG end states (checked, re-traced where they moved); -1 (default) / 1
        on, 0 off."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_PIXEL_SPECULATE, int(mode)))

    def set_pixel_heavy_first(self, mode: int):
        """ORT_OPT_PIXEL_HEAVY_FIRST: whole-pixel paths take the previous frame's heaviest 8x8
        blocks first; -1 (default) for frames of 2+ samples, 0 off, 1 on."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_PIXEL_HEAVY_FIRST, int(mode)))

    def set_xcd_swizzle(self, mode: int):
        """Workgroup -> tile order (ORT_OPT_XCD_SWIZZLE): 2 runs of raster tiles per XCD, 1
        128x128-pixel super-tiles per XCD, 0 raster, -1 (default) raster on small one-tile-workgroup
        tiles and runs otherwise; same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_XCD_SWIZZLE, int(mode)))

    def set_sort_paths(self, mode: int):
        """Order of the alive paths between bounces (same pixels): 0 slot order, 1 radix sort of
        every slot by coherence key, 2 (default) full-key radix sort of the appended alive list,
        sized by the same bounce's list length in the previous frame of this shape (+1/64 + 1024;
        a longer list goes on unsorted) -- no host wait (include/ort.h ORT_OPT_SORT_PATHS)."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_SORT_PATHS, int(mode)))

    def set_persistent(self, on):
        """Persistent trace kernel with lane refill for the bounce >= 1 traces: 2 (default) on, 0 off
        (same pixels).  1 (every trace persistent) was removed: OrtError."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_PERSISTENT, int(on)))

    def set_kid_skip(self, mode: int):
        """Rejected-sphere skip of one-sphere leaf children (kid_table.h); same pixels.  0 off,
        1 on (node records and kid entries from the interleaved copy), 2 on with the two
        separate arrays (testing)."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_KID_SKIP, int(mode)))

    def set_sort_bound(self, bound: int):
        """Testing (ORT_OPT_SORT_BOUND): force the list sort's size; 0 = the previous-frame hint."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_SORT_BOUND, int(bound)))

    def set_heavy_first(self, steps: int):
        """ORT_OPT_HEAVY_FIRST: bounce lists ordered by last frame's walk steps in classes >= 4T, >= 2T,
        >= T (T = steps, default 64), the rest last; 0 off (coherence order only).  Same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_HEAVY_FIRST, int(steps)))

    def set_heavy_prio(self, steps: int):
        """ORT_OPT_HEAVY_PRIO: camera-ray waves holding a walk of >= steps (last frame) run at raised
        issue priority; 0 off (default 150).  Same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_HEAVY_PRIO, int(steps)))

    def set_split_heavy(self, steps: int):
        """ORT_OPT_SPLIT_HEAVY: camera rays whose walk took >= steps (last frame) are walked by 8 lanes
        each, their subtrees dealt round robin, beside the per-tile kernel; 0 off; -1 (default) 200 on
        tiles of at most 2^21 pixels, off on larger ones.  Same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_SPLIT_HEAVY, int(steps)))

    def set_split_level(self, level: int):
        """ORT_OPT_SPLIT_LEVEL: the level of the subtrees a split walk deals (0: depth - 5)."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_SPLIT_LEVEL, int(level)))

    def set_tile_pairs(self, on: int):
        """ORT_OPT_TILE_PAIRS: camera-ray workgroups of two tiles, each wave a heavy and a light 64-pixel
        block by last frame's walk steps; 0 a tile per workgroup; -1 (default) pairs on tiles of more
        than 2^21 pixels.  Same pixels."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_TILE_PAIRS, int(on)))

    def set_debug_flags(self, flags: int):
        """ORT_OPT_DEBUG_FLAGS (analysis, A/B only): 1 no trace-timing events, 2 no queued heavy scan."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_DEBUG_FLAGS, int(flags)))

    def set_cost_order(self, on: int):
        """ORT_OPT_COST_ORDER: 1 (default) camera rays dealt to waves by last frame's walk cost; 0 fixed blocks."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_COST_ORDER, int(on)))

    def set_refill(self, lanes: int):
        """Persistent trace: refill a wave once at least `lanes` of its 64 lanes are idle."""
        self._check(self._lib.ort_set_option(self._ctx, L.ORT_OPT_REFILL, int(lanes)))

    def upload(self, spheres: SphereSet, tree: FlatOctree | None):
        cr = np.ascontiguousarray(spheres.center_radius, np.float32)
        ma = np.ascontiguousarray(spheres.mat_albedo, np.float32)
        fr = np.ascontiguousarray(spheres.fuzz_ri, np.float32)
        if tree is None:
            self._check(self._lib.ort_upload_scene(self._ctx, L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n,
                                                   None, None, None, None, None, 0, None, 0))
            return
        nmin = np.ascontiguousarray(tree.node_min, np.float32)
        nmax = np.ascontiguousarray(tree.node_max, np.float32)
        co = np.ascontiguousarray(tree.children_offset, np.int32)
        oo = np.ascontiguousarray(tree.objects_offset, np.int32)
        cnt = np.ascontiguousarray(tree.object_count, np.int32)
        idx = np.ascontiguousarray(tree.object_indices, np.int32)
        self._check(self._lib.ort_upload_scene(self._ctx, L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n,
                                               L.fptr(nmin), L.fptr(nmax), L.iptr(co), L.iptr(oo), L.iptr(cnt),
                                               tree.n_nodes, L.iptr(idx), tree.n_indices))

    def build_scene(self, spheres: SphereSet, max_depth: int, max_spheres_per_node: int, keep_tree: bool = False):
        """Build the octree on the GPU (ort_build_scene: the reference builder's exact output)
        and make it this renderer's scene.  keep_tree: keep the reference-layout tree on the
        device for export_octree()."""
        cr = np.ascontiguousarray(spheres.center_radius, np.float32)
        ma = np.ascontiguousarray(spheres.mat_albedo, np.float32)
        fr = np.ascontiguousarray(spheres.fuzz_ri, np.float32)
        self._check(self._lib.ort_build_scene(self._ctx, L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n,
                                              int(max_depth), int(max_spheres_per_node), int(bool(keep_tree))))

    def export_octree(self) -> FlatOctree:
        """The kept GPU-built tree (build_scene(keep_tree=True)) as a host FlatOctree."""
        i = self.info()
        n, k = i["n_nodes"], i["n_indices"]
        nmin = np.empty((n, 3), np.float32)
        nmax = np.empty((n, 3), np.float32)
        co = np.empty(n, np.int32)
        oo = np.empty(n, np.int32)
        cnt = np.empty(n, np.int32)
        idx = np.empty(max(k, 1), np.int32)
        self._check(self._lib.ort_scene_export_octree(self._ctx, L.fptr(nmin), L.fptr(nmax), L.iptr(co), L.iptr(oo),
                                                      L.iptr(cnt), L.iptr(idx)))
        return FlatOctree(nmin, nmax, co, oo, cnt, idx[:k])

    def stream_handle(self) -> int:
        """The context's own (non-blocking) HIP stream, e.g. for torch.cuda.ExternalStream."""
        h = C.c_void_p()
        self._check(self._lib.ort_get_stream(self._ctx, C.byref(h)))
        return h.value or 0

    def last_build_ms(self) -> float:
        ms = C.c_float()
        self._check(self._lib.ort_last_build_ms(self._ctx, C.byref(ms)))
        return ms.value

    def info(self) -> dict:
        i = L.OrtSceneInfo()
        self._check(self._lib.ort_scene_get_info(self._ctx, C.byref(i)))
        return {"n_spheres": i.n_spheres, "n_nodes": i.n_nodes, "n_indices": i.n_indices,
                "layout": "compact" if i.layout == L.ORT_LAYOUT_COMPACT else "explicit",
                "tree_depth": i.tree_depth, "device_bytes": i.device_bytes}

    # -- frames ----------------------------------------------------------------------
    def render(self, params: FrameParams, tile: Tile | None = None, out=None, stream=None):
        """Render a tile.  out: None (returns a new (rows, width, 3) float32 numpy array),
        a numpy array, or a device pointer (int) / torch CUDA tensor on this device.
        stream: None (synchronous) or a hipStream_t handle (int), e.g.
        torch.cuda.Stream().cuda_stream.  The null stream (handle 0, torch's default
        stream) cannot be told apart from "no stream": it renders synchronously."""
        tile = tile or Tile.full(params)
        p, t = params.to_c(), tile.to_c()
        s = C.c_void_p(int(stream)) if stream else None
        if out is None:
            out = np.empty((tile.rows, tile.width, 3), np.float32)
        if isinstance(out, np.ndarray):
            if out.dtype != np.float32 or not out.flags.c_contiguous or out.size < tile.rows * tile.width * 3:
                raise ValueError(f"render: out must be a C-contiguous float32 array of >= {tile.rows * tile.width * 3} "
                                 f"elements (got {out.dtype}, {out.size}, contiguous={out.flags.c_contiguous})")
            self._check(self._lib.ort_render(self._ctx, C.byref(p), C.byref(t), out.ctypes.data_as(C.c_void_p), 0, s))
            return out
        ptr = out.data_ptr() if hasattr(out, "data_ptr") else int(out)
        if hasattr(out, "numel"):  # a torch tensor: float32, contiguous, on this context's GPU
            import torch
            if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < tile.rows * tile.width * 3:
                raise ValueError(f"render: out must be a contiguous float32 tensor of >= {tile.rows * tile.width * 3} "
                                 f"elements (got {out.dtype}, {out.numel()}, contiguous={out.is_contiguous()})")
            if out.device.type != "cuda" or out.device.index != self.device:
                raise ValueError(f"render: out is on {out.device}, the context renders on cuda:{self.device}")
        self._check(self._lib.ort_render(self._ctx, C.byref(p), C.byref(t), C.c_void_p(ptr), 1, s))
        return out

    def last_kernel_ms(self) -> float:
        ms = C.c_float()
        self._check(self._lib.ort_last_kernel_ms(self._ctx, C.byref(ms)))
        return ms.value

    def last_trace_ms(self) -> float:
        """First trace kernel of the last frame (camera rays + octree walk; the dominant kernel)."""
        ms = C.c_float()
        self._check(self._lib.ort_last_trace_ms(self._ctx, C.byref(ms)))
        return ms.value

    def trace_times_ms(self, n: int) -> list:
        """Trace-kernel durations (ms) of the last n frames (n <= 64), oldest first."""
        buf = (C.c_float * max(1, n))()
        k = self._lib.ort_trace_times_ms(self._ctx, int(n), buf)
        if k < 0:
            L.check(-k, self._ctx)
        return [buf[i] for i in range(k)]

    def frame_trace_times_ms(self, n: int):
        """Per frame (last n <= 64, oldest first): (summed ms of all its trace kernels, launches)."""
        buf = (C.c_float * max(1, n))()
        nl = (C.c_int32 * max(1, n))()
        k = self._lib.ort_frame_trace_times_ms(self._ctx, int(n), buf, nl)
        if k < 0:
            L.check(-k, self._ctx)
        return [(buf[i], nl[i]) for i in range(k)]

    def count_traffic(self, params: FrameParams, tile: Tile | None = None) -> dict:
        tile = tile or Tile.full(params)
        p, t = params.to_c(), tile.to_c()
        counts = (C.c_uint64 * L.ORT_COUNT_N)()
        self._check(self._lib.ort_count_traffic(self._ctx, C.byref(p), C.byref(t), counts))
        return dict(zip(L.COUNT_NAMES, [int(v) for v in counts]))


# Reference-layout record bytes touched, SURVEY.md 8(d): the algorithmic traffic model.
BYTES_PER = {"nodes_popped": 36, "child_records": 32, "leaf_objects": 20, "accepted_hits": 32, "pixels": 12}


def algorithmic_bytes(counts: dict) -> int:
    return sum(BYTES_PER[k] * int(counts[k]) for k in BYTES_PER)


def emulate_render_host(spheres: SphereSet, tree: FlatOctree | None, params: FrameParams, tile: Tile | None = None,
                        layout: int = L.ORT_LAYOUT_COMPACT):
    """TEST-ONLY: run the kernel's per-pixel code (render_core.h) on the host CPU.
    Used by the CPU test suite to validate the kernel's traversal logic against the
    independent oracle without a GPU.  ``Renderer.render`` never calls this."""
    lib = L.analysis_lib()
    tile = tile or Tile.full(params)
    out = np.empty((tile.rows, tile.width, 3), np.float32)
    counts = (C.c_uint64 * L.ORT_COUNT_N)()
    p, t = params.to_c(), tile.to_c()
    cr = np.ascontiguousarray(spheres.center_radius, np.float32)
    ma = np.ascontiguousarray(spheres.mat_albedo, np.float32)
    fr = np.ascontiguousarray(spheres.fuzz_ri, np.float32)
    if tree is None:
        keep = ()
        args = (None, None, None, None, None, 0, None, 0)
    else:
        keep = tuple(np.ascontiguousarray(a, t) for a, t in (
            (tree.node_min, np.float32), (tree.node_max, np.float32), (tree.children_offset, np.int32),
            (tree.objects_offset, np.int32), (tree.object_count, np.int32), (tree.object_indices, np.int32)))
        args = (L.fptr(keep[0]), L.fptr(keep[1]), L.iptr(keep[2]), L.iptr(keep[3]), L.iptr(keep[4]),
                tree.n_nodes, L.iptr(keep[5]), tree.n_indices)
    L.acheck(lib.ort_debug_emulate_render(L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n, *args, layout,
                                         C.byref(p), C.byref(t), L.fptr(out), counts))
    del keep
    return out, dict(zip(L.COUNT_NAMES, [int(v) for v in counts]))
