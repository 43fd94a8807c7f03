"""Per-pixel walk steps of the C3 frame for tools/order_model.py (analysis only): the host
restatement of the kernel walk (ort_debug_walk_steps, every 8x8 block) for the default camera
and cameras turned by 0.5-2.5 degrees; saved as /tmp/sim/steps_<tag>.npy."""
import os
os.makedirs("/tmp/sim", exist_ok=True)
import ctypes as C, sys, time, numpy as np
sys.path.insert(0, '/root/repo')
import bench, octreeraytracer_amd as ort
from octreeraytracer_amd import _lib as L
from octreeraytracer_amd.scene import DEFAULT_YAW
W, H, N, D, M, NS, MD = bench.CONFIGS['c3']
s = ort.random_spheres(N, 42); t = ort.build_octree(s, D, M)
lib = L.analysis_lib(); f = lib.ort_debug_walk_steps; f.restype = C.c_int64
fp = lambda a: a.ctypes.data_as(C.c_void_p)
arr = [np.ascontiguousarray(x) for x in (s.center_radius, s.mat_albedo, s.fuzz_ri)]
tt = [np.ascontiguousarray(x) for x in (t.node_min, t.node_max, t.children_offset, t.objects_offset, t.object_count, t.object_indices)]
bw, bh = (W + 7) // 8, (H + 7) // 8
for tag, yaw in (('static', DEFAULT_YAW), ('yaw05', DEFAULT_YAW + 0.5), ('yaw1', DEFAULT_YAW + 1.0), ('yaw15', DEFAULT_YAW + 1.5), ('yaw2', DEFAULT_YAW + 2.0), ('yaw25', DEFAULT_YAW + 2.5)):
    p = ort.FrameParams.default_camera(W, H, yaw=yaw)
    lens = np.zeros(bw * bh * 64, np.int32); cap = bw * bh * 64 * 120
    steps = np.zeros(cap, np.uint16)
    t0 = time.time()
    n = f(fp(arr[0]), fp(arr[1]), fp(arr[2]), C.c_int32(s.n), fp(tt[0]), fp(tt[1]), fp(tt[2]), fp(tt[3]), fp(tt[4]),
          C.c_int32(len(t.children_offset)), fp(tt[5]), C.c_int64(len(t.object_indices)), C.byref(p.to_c()),
          C.c_int32(1), fp(lens), C.c_int64(len(lens)), fp(steps), C.c_int64(cap))
    assert n >= 0, n
    img = lens.reshape(bh, bw, 8, 8).transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)[:H, :W]
    np.save(f'/tmp/sim/steps_{tag}.npy', img.astype(np.int32))
    print(tag, 'mean steps', img.mean(), f'{time.time()-t0:.0f}s', flush=True)
