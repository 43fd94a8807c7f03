"""Analysis only: how much of the reference walk a per-node sphere-union bound would prune
(tools/prune_sim.cpp), for sampled 8x8 camera-ray blocks and for one diffuse bounce off
their hits.  Lockstep proxy: per 64-ray wave, the max over its lanes of node pops.
usage: python tools/prune_sim.py [config] [block_step] [margin]"""
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

so = ROOT / "tools" / "libprune_sim.so"
subprocess.run(["g++", "-O2", "-shared", "-fPIC", "-o", str(so), str(ROOT / "tools" / "prune_sim.cpp")], check=True)
lib = C.CDLL(str(so))
lib.prune_sim_run.restype = C.c_int64
fp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 97
margin = float(sys.argv[3]) if len(sys.argv) > 3 else 1e-3
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t0 = time.time()
t = ort.build_octree(s, D, M)
print(f"{cfg}: tree {len(t.children_offset)} nodes in {time.time() - t0:.1f} s", flush=True)
sph = np.ascontiguousarray(s.center_radius, np.float32)
co, oo, cnt, idx = (np.ascontiguousarray(x, np.int32) for x in (t.children_offset, t.objects_offset, t.object_count,
                                                                   t.object_indices))
nmin, nmax = (np.ascontiguousarray(x, np.float32) for x in (t.node_min, t.node_max))
n = len(co)
bounds = np.zeros(6 * n, np.float32)
lib.prune_sim_bounds(fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), C.c_float(margin), fp(bounds))

# camera rays (pinhole through pixel centres of sampled 8x8 blocks; the kernel's jitter is
# sub-pixel and does not matter for these statistics)
p = ort.FrameParams.default_camera(W, H)
V = np.asarray(p.view, np.float32).reshape(4, 4).T  # column-major -> rows
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


def run(rays, prune_from, label, mode=0):
    nr = len(rays)
    per = np.zeros(8 * nr, np.int32)
    ht = np.zeros(nr, np.float32)
    hs = np.zeros(nr, np.int32)
    t0 = time.time()
    bad = lib.prune_sim_run(fp(nmin), fp(nmax), fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), fp(bounds),
                            C.c_int(prune_from), C.c_int(mode), fp(np.ascontiguousarray(rays)), C.c_int64(nr), fp(per), fp(ht), fp(hs))
    per = per.reshape(nr, 8)
    w = per.reshape(-1, 64, 8)
    base, pruned = w[:, :, 0].max(1).sum(), w[:, :, 2].max(1).sum()
    push = (w[:, :, 2] - w[:, :, 3]).max(1).sum()  # pruned at the parent: a pruned child costs no pop
    ipops = w[:, :, 1].max(1).sum()
    ipush = w[:, :, 4].max(1).sum()
    print(f"{label} mode={mode} prune_from={prune_from}: pops/ray {per[:, 0].mean():.1f} -> {per[:, 2].mean():.1f} "
          f"(pruned {per[:, 3].mean():.1f}); wave max-lane pops {base / len(w):.1f} -> {pruned / len(w):.1f} "
          f"({pruned / max(base, 1) - 1:+.1%}); at push {push / len(w):.1f} ({push / max(base, 1) - 1:+.1%}); "
          f"internal {ipops / len(w):.1f} -> {ipush / len(w):.1f} ({ipush / max(ipops, 1) - 1:+.1%}); "
          f"sphere tests/ray {per[:, 5].mean():.1f} -> {per[:, 6].mean():.1f}; pruned internal/ray {per[:, 7].mean():.1f}; hits {np.mean(ht > 0):.2f}; mismatches {bad}; {time.time() - t0:.1f} s",
          flush=True)
    return ht, hs


ht, hs = run(rays, 0, "camera")
# one bounce: cosine-ish diffuse directions around the normal at each camera hit (order kept: waves
# of 64 consecutive hits approximate the sorted bounce list's coherence only loosely)
rng = np.random.default_rng(1)
h = ht > 0
o = rays[h, :3] + ht[h, None] * rays[h, 3:]
nrm = (o - sph.reshape(-1, 4)[hs[h], :3]) / sph.reshape(-1, 4)[hs[h], 3:4]
v = rng.normal(size=o.shape)
v /= np.linalg.norm(v, axis=1, keepdims=True)
dd = nrm + v
dd /= np.linalg.norm(dd, axis=1, keepdims=True)
b = np.concatenate([o, dd], 1).astype(np.float32)
b = b[: len(b) // 64 * 64]
run(b, 0, "bounce")

# lockstep cost model (kernel loop shape), quantized per-node bounds tested at the pop
q = np.zeros(6 * n, np.int8)
lib.prune_sim_quantize(fp(nmin), fp(nmax), fp(co), C.c_int32(n), fp(bounds), fp(q))
qq = q.reshape(n, 6)[co != -1]
print("quantized faces: unbounded %.2f, shrunk %.2f (x lo/hi, y, z): %s" % (
    np.mean(qq == 127), np.mean((qq < 0)), [round(float(np.mean(qq[:, k] == 127)), 2) for k in range(6)]))
costs = np.array([45, 63, 15, 45, float(sys.argv[4]) if len(sys.argv) > 4 else 25], np.float32)
for label, rr in (("camera", rays), ("bounce", b)):
    nwv = len(rr) // 64
    for inl in (0, 1, 2):
        res = []
        for pr in ((0, 1, 2) if inl == 0 else (0,)):
            o2 = np.zeros(2 * nwv, np.float64)
            lib.prune_sim_lockstep(fp(nmin), fp(nmax), fp(co), fp(oo), fp(cnt), fp(idx), C.c_int32(n), fp(sph), fp(q),
                                   C.c_int(pr), C.c_int(inl), fp(costs), fp(np.ascontiguousarray(rr)), C.c_int64(nwv),
                                   fp(o2))
            res.append(o2.reshape(-1, 2).sum(0) / nwv)
        if inl:
            print(f"lockstep {label} inline_leaves={inl}: VALU/wave {res[0][0]:.0f}, iterations {res[0][1]:.1f}", flush=True)
            continue
        print(f"lockstep {label} inline_leaves={inl}: VALU/wave {res[0][0]:.0f} -> at pop {res[1][0]:.0f} "
              f"({res[1][0] / res[0][0] - 1:+.1%}), at push (T per internal node) {res[2][0]:.0f} "
              f"({res[2][0] / res[0][0] - 1:+.1%}); iterations {res[0][1]:.1f} -> {res[1][1]:.1f} / {res[2][1]:.1f}",
              flush=True)
