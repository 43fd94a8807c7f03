"""Lane overlap of 8x8 primary-ray blocks (one wave each), computed on the host with the
kernel's own fast walk (ort_debug_wave_stats, analysis-only): how many nodes the union of a
wave's rays visits versus the rays individually, and how the per-lane lockstep loop spends
its iterations.  Used to price wave-level (packet) traversal; see DESIGN.md.
usage: python tools/wave_stats.py [config] [block_step]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 37
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
lib = L.analysis_lib()
f = lib.ort_debug_wave_stats
f.restype = C.c_int
st = np.zeros(18, np.float64)
fp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
arr = [np.ascontiguousarray(x) for x in (s.center_radius, s.mat_albedo, s.fuzz_ri)]
tt = [np.ascontiguousarray(x) for x in (t.node_min, t.node_max, t.children_offset, t.objects_offset,
                                         t.object_count, t.object_indices)]
rc = f(fp(arr[0]), fp(arr[1]), fp(arr[2]), C.c_int32(s.n), fp(tt[0]), fp(tt[1]), fp(tt[2]), fp(tt[3]),
       fp(tt[4]), C.c_int32(len(t.children_offset)), fp(tt[5]), C.c_int64(len(t.object_indices)),
       C.byref(p.to_c()), C.c_int32(step), fp(st), C.c_int32(18))
L.check(rc)
waves, mixed, lanes, iI, iL, iS, uI, uL, uS, it, itI, itL, trips, laneit, maxlen = st[:15]
print(f"{cfg}: {int(waves)} sampled waves (every {step}th 8x8 block), {int(mixed)} mixed-order, "
      f"{lanes / waves:.1f} fast lanes/wave")
print(f"per wave: individual visits internal {iI / waves:.0f} leaf {iL / waves:.0f} spheres {iS / waves:.0f}"
      f" | union internal {uI / waves:.1f} leaf {uL / waves:.1f} spheres {uS / waves:.1f}"
      f" | per-ray internal {iI / lanes:.1f} leaf {iL / lanes:.1f}")
print(f"union / mean-ray: internal {uI / (iI / lanes * waves):.2f}x leaf {uL / (iL / lanes * waves):.2f}x; "
      f"packet lane utilisation internal {iI / (uI * 64):.2f} leaf {iL / (uL * 64):.2f}")
print(f"lockstep loop per wave: {it / waves:.1f} iterations ({itI / waves:.1f} with internal block, "
      f"{itL / waves:.1f} with leaf block, {trips / waves:.1f} sphere trips), "
      f"lane occupancy {laneit / (it * 64):.2f}")
print(f"wave-uniform iterations (every walking lane pops the same node): leading {st[15] / waves:.1f}, "
      f"all {st[16] / waves:.1f} of {it / waves:.1f}")
