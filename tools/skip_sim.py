"""Analysis only: pops per ray of the reference walk with the rejected-sphere skip at push
time (tools/skip_sim.cpp skip_sim_push: the GPU's kid entries, 2 spheres per node, the last
rejected sphere per lane), for one-sphere LEAF children only (the current kid table) and for
children whose whole SUBTREE holds one sphere.  Camera rays of sampled 8x8 blocks and one
diffuse bounce off their hits, as tools/prune_sim.py.
usage: python tools/skip_sim.py [config] [block_step]"""
import ctypes as C
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402

so = ROOT / "tools" / "libskip_sim.so"
subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "skip_sim.cpp")], check=True)
lib = C.CDLL(str(so))
fp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731

cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 997
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t0 = time.time()
t = ort.build_octree(s, D, M)
print(f"{cfg}: tree {len(t.children_offset)} nodes in {time.time() - t0:.1f} s", flush=True)
sph = np.ascontiguousarray(s.center_radius, np.float32)
co, oo, cnt, idx = (np.ascontiguousarray(x, np.int32) for x in (t.children_offset, t.objects_offset, t.object_count,
                                                                   t.object_indices))
nmin, nmax = (np.ascontiguousarray(x, np.float32) for x in (t.node_min, t.node_max))
del t
n = len(co)
sum_ids = np.zeros(n, np.int32)
sum_n = np.zeros(n, np.int8)
lib.skip_sim_summaries(fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), C.c_int(1), fp(sum_ids), fp(sum_n))
internal = co != -1
print(f"internal nodes whose subtree holds one sphere: {np.mean(sum_n[internal] == 1):.3f}", flush=True)

p = ort.FrameParams.default_camera(W, H)
V = np.asarray(p.view, np.float32).reshape(4, 4).T
R = V[:3, :3]
eye = np.asarray(p.camera_position, np.float32)
th = np.tan(np.radians(p.camera_zoom) / 2)
bx, by = (W + 7) // 8, (H + 7) // 8
blocks = np.arange(0, bx * by, step)
lx, ly = np.meshgrid(np.arange(8), np.arange(8))
px = ((blocks % bx)[:, None] * 8 + lx.ravel()[None, :]).ravel()
py = ((blocks // bx)[:, None] * 8 + ly.ravel()[None, :]).ravel()
cam = np.stack([(2 * (px + 0.5) / W - 1) * th * W / H, (2 * (py + 0.5) / H - 1) * th, -np.ones_like(px, float)], 1)
d = cam @ R
d /= np.linalg.norm(d, axis=1, keepdims=True)
rays = np.concatenate([np.broadcast_to(eye, d.shape), d], 1).astype(np.float32)


def run(rr, label, cache=1):
    for mode in (0,) if cache != 1 else (0, 1):
        lib.skip_sim_push_subtree(fp(sum_ids) if mode else None, fp(sum_n) if mode else None, C.c_int(1))
        st = np.zeros(8, np.int64)
        per = np.zeros(2 * len(rr), np.int32)
        t0 = time.time()
        lib.skip_sim_push(fp(nmin), fp(nmax), fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), C.c_int(cache),
                          C.c_int(2), fp(np.ascontiguousarray(rr)), C.c_int64(len(rr)), fp(st), fp(per))
        per = per.reshape(-1, 2)
        w = per[: len(per) // 64 * 64].reshape(-1, 64, 2)
        print(f"{label} {'subtree' if mode else 'leaf   '} cache={cache}: pops/ray {st[1] / st[0]:.1f} -> {st[2] / st[0]:.1f} "
              f"({st[2] / st[1] - 1:+.1%}); wave max-lane {w[:, :, 0].max(1).mean():.1f} -> {w[:, :, 1].max(1).mean():.1f}; "
              f"children skipped/ray {st[3] / st[0]:.1f}; mismatches {st[5]}; {time.time() - t0:.1f} s", flush=True)


run(rays, "camera")
# one diffuse bounce off the camera hits (hit points from tools/prune_sim.cpp's reference walk)
pso = ROOT / "tools" / "libprune_sim.so"
subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", str(pso), str(ROOT / "tools" / "prune_sim.cpp")], check=True)
pl = C.CDLL(str(pso))
pl.prune_sim_run.restype = C.c_int64
bounds = np.zeros(6 * n, np.float32)
pl.prune_sim_bounds(fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), C.c_float(1e-3), fp(bounds))
nr = len(rays)
per = np.zeros(8 * nr, np.int32)
ht = np.zeros(nr, np.float32)
hs = np.zeros(nr, np.int32)
pl.prune_sim_run(fp(nmin), fp(nmax), fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), fp(bounds), C.c_int(0),
                 C.c_int(0), fp(np.ascontiguousarray(rays)), C.c_int64(nr), fp(per), fp(ht), fp(hs))
rng = np.random.default_rng(1)
h = ht > 0
o = rays[h, :3] + ht[h, None] * rays[h, 3:]
nrm = (o - sph.reshape(-1, 4)[hs[h], :3]) / sph.reshape(-1, 4)[hs[h], 3:4]
v = rng.normal(size=o.shape)
v /= np.linalg.norm(v, axis=1, keepdims=True)
dd = nrm + v
dd /= np.linalg.norm(dd, axis=1, keepdims=True)
b = np.concatenate([o, dd], 1).astype(np.float32)
run(b[: len(b) // 64 * 64], "bounce")
run(rays, "camera", 2)
run(b[: len(b) // 64 * 64], "bounce", 2)


# pop-time bound (skip_sim_run): a popped subtree whose <= K spheres are all in the lane's
# last-`cache` rejection cache (each with e <= the subtree's pushed tmin) is skipped whole
def run_pop(rr, label, K, cache):
    si = np.zeros(n * K, np.int32)
    sn = np.zeros(n, np.int8)
    lib.skip_sim_summaries(fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), C.c_int(K), fp(si), fp(sn))
    st = np.zeros(16, np.int64)
    lib.skip_sim_run(fp(nmin), fp(nmax), fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), fp(si), fp(sn),
                     C.c_int(K), C.c_int(cache), fp(np.ascontiguousarray(rr)), C.c_int64(len(rr)), fp(st), None)
    print(f"{label} pop-time K={K} cache={cache}: pops/ray {st[1] / st[0]:.1f} -> {st[9] / st[0]:.1f} "
          f"({st[9] / st[1] - 1:+.1%}); sphere tests/ray {st[4] / st[0]:.1f} -> {st[7] / st[0]:.1f}; mismatches {st[10]}",
          flush=True)


for K, cache in ((1, 1), (2, 2)):
    run_pop(rays, "camera", K, cache)
    run_pop(b[: len(b) // 64 * 64], "bounce", K, cache)
