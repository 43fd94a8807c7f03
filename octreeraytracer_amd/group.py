"""Several GPUs in one process behind the C ABI (include/ort.h ort_group_*): one context per
device, the frame cut into 16-row bands dealt round-robin, ONE exchange -- the bands gathered
to devices[0] over RCCL (or device copies) -- and a de-interleave kernel there (SURVEY.md
8(e)).  The one-process-per-GPU path of bench.py (torch.distributed) partitions the frame
identically (octreeraytracer_amd/distributed.py)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L
from .renderer import FrameParams
from .scene import FlatOctree, SphereSet

TRANSPORT_RCCL = L.ORT_GROUP_TRANSPORT_RCCL
TRANSPORT_COPY = L.ORT_GROUP_TRANSPORT_COPY


class RenderGroup:
    def __init__(self, devices, transport: int = TRANSPORT_RCCL, inflight: int = 1):
        """inflight: frame slots (ort_group_create_pipelined): submit() returns at once and
        frame k+1 renders while frame k's last blocks finish."""
        self._lib = L.lib()
        self._g = C.c_void_p()
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        rc = self._lib.ort_group_create_pipelined(devs, len(devices), int(transport), int(inflight),
                                                  C.byref(self._g))
        if rc != L.ORT_OK:
            raise L.OrtError(rc, self._lib.ort_group_last_error(None).decode())
        self.devices = list(devices)
        self.inflight = int(inflight)
        # outputs of submitted frames, kept alive until their frame is known complete (the ABI
        # writes them asynchronously; a dropped torch tensor could otherwise be reallocated
        # while the de-interleave kernel still writes it)
        self._pending = {}

    def _check(self, rc):
        if rc != L.ORT_OK:
            raise L.OrtError(rc, self._lib.ort_group_last_error(self._g).decode())

    def close(self):
        if self._g:
            self._lib.ort_group_destroy(self._g)  # synchronizes every stream first
            self._g = C.c_void_p()
        self._pending = {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_timeout(self, ms: int):
        """Bound of every wait on a frame (ort_group_set_timeout; 0 = poll once): an expired wait
        raises OrtError(ORT_ERR_TIMEOUT) naming the frame, its slot and the pending ranks."""
        self._check(self._lib.ort_group_set_timeout(self._g, int(ms)))

    def set_option(self, option: int, value: int):
        self._check(self._lib.ort_group_set_option(self._g, int(option), int(value)))

    def build_scene(self, spheres: SphereSet, max_depth: int, max_spheres_per_node: int):
        cr, ma, fr = (np.ascontiguousarray(a, np.float32) for a in (spheres.center_radius, spheres.mat_albedo,
                                                                      spheres.fuzz_ri))
        self._check(self._lib.ort_group_build_scene(self._g, L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n,
                                                    int(max_depth), int(max_spheres_per_node)))

    def upload(self, spheres: SphereSet, tree: FlatOctree):
        cr, ma, fr = (np.ascontiguousarray(a, np.float32) for a in (spheres.center_radius, spheres.mat_albedo,
                                                                      spheres.fuzz_ri))
        t = [np.ascontiguousarray(a, d) for a, d in (
            (tree.node_min, np.float32), (tree.node_max, np.float32), (tree.children_offset, np.int32),
            (tree.objects_offset, np.int32), (tree.object_count, np.int32), (tree.object_indices, np.int32))]
        self._check(self._lib.ort_group_upload_scene(self._g, L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n,
                                                     L.fptr(t[0]), L.fptr(t[1]), L.iptr(t[2]), L.iptr(t[3]),
                                                     L.iptr(t[4]), tree.n_nodes, L.iptr(t[5]), tree.n_indices))

    def _out(self, params: FrameParams, out):
        n = params.height * params.width * 3
        if out is None:
            out = np.empty((params.height, params.width, 3), np.float32)
        if isinstance(out, np.ndarray):
            if out.dtype != np.float32 or not out.flags.c_contiguous or out.size < n:
                raise ValueError("render: out must be a contiguous float32 array of H*W*3 elements")
            return out, out.ctypes.data_as(C.c_void_p), 0
        import torch
        if out.dtype != torch.float32 or not out.is_contiguous() or out.numel() < n:
            raise ValueError("render: out must be a contiguous float32 tensor of H*W*3 elements")
        if out.device.type != "cuda" or out.device.index != self.devices[0]:
            raise ValueError(f"render: out is on {out.device}, the group assembles on cuda:{self.devices[0]}")
        return out, C.c_void_p(out.data_ptr()), 1

    def render(self, params: FrameParams, out=None):
        """Full frame: a new (H, W, 3) float32 numpy array, a numpy array, or a float32 torch
        tensor on devices[0] (device output).  Synchronous."""
        p = params.to_c()
        out, ptr, dev = self._out(params, out)
        self._check(self._lib.ort_group_render(self._g, C.byref(p), ptr, dev))
        return out

    def submit(self, params: FrameParams, out) -> int:
        """Enqueue a frame into `out` -- a numpy array or a float32 torch tensor on devices[0],
        required: the frame is written asynchronously -- and return its ticket at once
        (ort_group_submit).  Keep `out` untouched until wait(ticket); the group holds a
        reference to it until then."""
        if out is None:
            raise ValueError("submit: out is required (the frame is written after submit returns; read it "
                             "after wait(ticket))")
        p = params.to_c()
        out, ptr, dev = self._out(params, out)
        tk = C.c_int64(-1)
        self._check(self._lib.ort_group_submit(self._g, C.byref(p), ptr, dev, C.byref(tk)))
        self._pending[tk.value] = out
        # submitting frame k waited for the frame that last used its slot (k - inflight) and
        # every frame before it on that slot: those outputs are complete
        for t in [t for t in self._pending if t <= tk.value - self.inflight]:
            del self._pending[t]
        return tk.value

    def wait(self, ticket: int):
        """Block until frame `ticket` is complete in its output (ort_group_wait)."""
        self._check(self._lib.ort_group_wait(self._g, C.c_int64(int(ticket))))
        self._pending.pop(int(ticket), None)

    def context(self, rank: int):
        """Rank `rank`'s context of frame slot 0 (owned by the group)."""
        c = C.c_void_p()
        self._check(self._lib.ort_group_context(self._g, int(rank), C.byref(c)))
        return c

    def count_traffic(self, params: FrameParams, rank: int) -> dict:
        """Reference-layout work counters (ort_count_traffic) of rank `rank`'s band tile."""
        from .distributed import rank_tile
        c = self.context(rank)
        p, t = params.to_c(), rank_tile(params.width, params.height, rank, len(self.devices)).to_c()
        counts = (C.c_uint64 * L.ORT_COUNT_N)()
        rc = self._lib.ort_count_traffic(c, C.byref(p), C.byref(t), counts)
        if rc != L.ORT_OK:
            raise L.OrtError(rc, self._lib.ort_last_error(c).decode())
        return dict(zip(L.COUNT_NAMES, [int(v) for v in counts]))

    def frame_trace_times_ms(self, rank: int, n: int):
        """Per frame of rank `rank`'s slot-0 context (last n <= 64): (summed trace-kernel ms, launches)."""
        c = self.context(rank)
        buf = (C.c_float * max(1, n))()
        nl = (C.c_int32 * max(1, n))()
        k = self._lib.ort_frame_trace_times_ms(c, int(n), buf, nl)
        if k < 0:
            raise L.OrtError(-k, self._lib.ort_last_error(c).decode())
        return [(buf[i], nl[i]) for i in range(k)]

    def last_frame_ms(self) -> float:
        """Latency (device time on devices[0]) of the last frame seen complete."""
        ms = C.c_float()
        self._check(self._lib.ort_group_last_frame_ms(self._g, C.byref(ms)))
        return ms.value


def emulate_group_host(spheres: SphereSet, tree: FlatOctree, params: FrameParams, world: int) -> np.ndarray:
    """TEST-ONLY (no GPU): the group's partition and row map with an in-memory transport, each
    band tile rendered by the host emulation of the kernel (ort_debug_group_emulate)."""
    lib = L.analysis_lib()
    out = np.empty((params.height, params.width, 3), np.float32)
    cr, ma, fr = (np.ascontiguousarray(a, np.float32) for a in (spheres.center_radius, spheres.mat_albedo,
                                                                  spheres.fuzz_ri))
    t = [np.ascontiguousarray(a, d) for a, d in (
        (tree.node_min, np.float32), (tree.node_max, np.float32), (tree.children_offset, np.int32),
        (tree.objects_offset, np.int32), (tree.object_count, np.int32), (tree.object_indices, np.int32))]
    p = params.to_c()
    L.acheck(lib.ort_debug_group_emulate(L.fptr(cr), L.fptr(ma), L.fptr(fr), spheres.n, L.fptr(t[0]), L.fptr(t[1]),
                                        L.iptr(t[2]), L.iptr(t[3]), L.iptr(t[4]), tree.n_nodes, L.iptr(t[5]),
                                        tree.n_indices, int(world), C.byref(p), L.fptr(out)))
    return out
