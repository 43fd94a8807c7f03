"""Do bounce walks that exit the root box soon take longer? (analysis only): the host restatement's
bounce-b walks of a 512x256 window (ort_debug_bounce_walks) against each ray's root-box exit
distance -- a history-free heavy-path class for moving cameras.  usage: python tools/bounce_texit.py [config] [bounce]"""
import ctypes as C, sys, numpy as np
import ctypes as C, sys, numpy as np
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tools')
import bench, octreeraytracer_amd as ort
from octreeraytracer_amd import _lib as L
cfg = sys.argv[1] if len(sys.argv) > 1 else 'c3'
bounce = int(sys.argv[2]) if len(sys.argv) > 2 else 1
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42); t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=max(MD, 4))
lib = L.analysis_lib(); f = lib.ort_debug_bounce_walks; f.restype = C.c_int
f.argtypes = [L._fp, L._fp, L._fp, C.c_int32, L._fp, L._fp, L._ip, L._ip, L._ip, C.c_int32, L._ip, C.c_int64,
              C.POINTER(L.OrtParams), C.POINTER(L.OrtTile), C.c_int32, L._fp, L._ip, C.c_int64, C.POINTER(C.c_int64)]
arr = [np.ascontiguousarray(a, dt) for a, dt in ((s.center_radius, np.float32), (s.mat_albedo, np.float32), (s.fuzz_ri, np.float32),
       (t.node_min, np.float32), (t.node_max, np.float32), (t.children_offset, np.int32), (t.objects_offset, np.int32), (t.object_count, np.int32), (t.object_indices, np.int32))]
x0, y0, ww, hh = W // 2 - 256, H // 2 - 128, 512, 256
tile = ort.Tile(x0, ww, y0, hh)
rays = np.zeros((ww * hh, 8), np.float32); cap = ww * hh * 400
walks = np.zeros((cap, 3), np.int32); n_out = C.c_int64()
L.acheck(f(L.fptr(arr[0]), L.fptr(arr[1]), L.fptr(arr[2]), s.n, L.fptr(arr[3]), L.fptr(arr[4]), L.iptr(arr[5]), L.iptr(arr[6]), L.iptr(arr[7]), t.n_nodes,
           L.iptr(arr[8]), t.n_indices, C.byref(p.to_c()), C.byref(tile.to_c()), bounce, L.fptr(rays), walks.ctypes.data_as(L._ip), cap, C.byref(n_out)))
alive = (rays[:, 6] == 1) & (rays[:, 7] > 0)
o, d, st = rays[alive, 0:3].astype(np.float64), rays[alive, 3:6].astype(np.float64), rays[alive, 7].astype(np.float64)
lo, hi = t.node_min[0].astype(np.float64), t.node_max[0].astype(np.float64)
with np.errstate(divide='ignore', invalid='ignore'):
    inv = 1.0 / d
    t0 = (lo - o) * inv; t1 = (hi - o) * inv
    texit = np.minimum(t0, t1).max(1) * 0 + np.maximum(t0, t1).min(1)
size = (hi - lo).max()
print(cfg, 'bounce', bounce, 'rays', alive.sum(), 'steps mean %.1f' % st.mean())
print(' corr(steps, t_exit) %.3f  spearman %.3f' % (np.corrcoef(st, texit)[0, 1], np.corrcoef(np.argsort(np.argsort(st)), np.argsort(np.argsort(texit)))[0, 1]))
q = np.quantile(texit, [0.25, 0.5, 0.75, 0.9])
for a, b in zip([-1] + list(q), list(q) + [1e30]):
    m = (texit > a) & (texit <= b)
    print('  t_exit in (%.3g, %.3g]: steps mean %.1f  share >= 256: %.3f' % (a, b, st[m].mean(), np.mean(st[m] >= 256)))
ext = hi - lo
F = (np.abs(d) * texit[:, None] / ext).sum(1)
G = (np.abs(d) * np.minimum(texit, 1e9)[:, None] / ext)
def sp(a, b):
    return np.corrcoef(np.argsort(np.argsort(a)), np.argsort(np.argsort(b)))[0, 1]
print(' spearman: t_exit %.3f  F=sum|d_a| t_exit/ext_a %.3f  |d.y| %.3f  Fy %.3f  Fxz %.3f' % (sp(st, texit), sp(st, F), sp(st, np.abs(d[:, 1])), sp(st, G[:, 1]), sp(st, G[:, 0] + G[:, 2])))
q = np.quantile(F, [0.5, 0.75, 0.9])
for a_, b_ in zip([-1] + list(q), list(q) + [1e30]):
    m = (F > a_) & (F <= b_)
    print('  F in (%.3g, %.3g]: steps mean %.1f  share >= 256: %.3f  share of rays %.2f' % (a_, b_, st[m].mean(), np.mean(st[m] >= 256), m.mean()))
rate = (np.abs(d) / ext).sum(1)   # cell crossings per unit length (x 2^D)
mext = ext.min()
for lam in (0.25, 0.5, 1.0, 2.0, 4.0, 1e9):
    Hf = np.minimum(texit, lam * mext) * rate
    print('  lambda %.2g x min extent: spearman %.3f' % (lam, sp(st, Hf)))
print('  rate alone: %.3f' % sp(st, rate))
Hf = np.minimum(texit, mext) * rate
qs = np.quantile(Hf, [0.25, 0.5, 0.75, 0.9])
print('  H quantiles 25/50/75/90%:', ' '.join('%.4f' % v for v in qs))
for a_, b_ in zip([-1] + list(qs), list(qs) + [1e30]):
    m = (Hf > a_) & (Hf <= b_)
    print('  H in (%.4g, %.4g]: steps mean %.1f  share >= 256: %.3f  >= 128: %.3f  rays %.2f' % (a_, b_, st[m].mean(), np.mean(st[m] >= 256), np.mean(st[m] >= 128), m.mean()))
