"""A learned heavy-first class for moved frames? (analysis only): the host restatement's bounce-b walks
(ort_debug_bounce_walks) of a 512x256 window A, binned by the top bits of the path key (octant,
the O most significant origin-code bits, the 6 direction bits), predict the steps of the walks of
window B -- the same camera, window shifted by DX pixels: the scene points a 0.5 deg turn brings
under a pixel, with that pixel's own random numbers.  Spearman of the steps with the bin's mean
(bins A holds; a bin A lacks falls back to the exit distance) against the exit distance alone --
and what a class order does to a persistent trace's tail: window B's walks, in class order,
list-scheduled on P workers (a lane pulls the next walk when its last ends; P ~ the window's
share of the GPU's lanes), makespan over the perfect balance, for the exact per-slot classes,
the exit-distance classes and the bins' means (thresholds 256/128/64 as the exact classes', or
quantiles matching the exit-distance classes' shares).
usage: python tools/bounce_bins.py [config] [bounce] [dx]"""
import ctypes as C
import sys

import numpy as np

sys.path.insert(0, '/root/repo')
import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else 'c5'
bounce = int(sys.argv[2]) if len(sys.argv) > 2 else 1
DX = int(sys.argv[3]) if len(sys.argv) > 3 else 26
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=max(MD, 4))
lib = L.analysis_lib()
f = lib.ort_debug_bounce_walks
f.restype = C.c_int
f.argtypes = [L._fp, L._fp, L._fp, C.c_int32, L._fp, L._fp, L._ip, L._ip, L._ip, C.c_int32, L._ip, C.c_int64,
              C.POINTER(L.OrtParams), C.POINTER(L.OrtTile), C.c_int32, L._fp, L._ip, C.c_int64, C.POINTER(C.c_int64)]
arr = [np.ascontiguousarray(a, dt) for a, dt in (
    (s.center_radius, np.float32), (s.mat_albedo, np.float32), (s.fuzz_ri, np.float32),
    (t.node_min, np.float32), (t.node_max, np.float32), (t.children_offset, np.int32),
    (t.objects_offset, np.int32), (t.object_count, np.int32), (t.object_indices, np.int32))]
lo, hi = t.node_min[0].astype(np.float64), t.node_max[0].astype(np.float64)


def walks(x0, y0, ww=512, hh=256):
    rays = np.zeros((ww * hh, 8), np.float32)
    cap = ww * hh * 400
    wk = np.zeros((cap, 3), np.int32)
    n_out = C.c_int64()
    L.acheck(f(L.fptr(arr[0]), L.fptr(arr[1]), L.fptr(arr[2]), s.n, L.fptr(arr[3]), L.fptr(arr[4]), L.iptr(arr[5]),
               L.iptr(arr[6]), L.iptr(arr[7]), t.n_nodes, L.iptr(arr[8]), t.n_indices, C.byref(p.to_c()),
               C.byref(ort.Tile(x0, ww, y0, hh).to_c()), bounce, L.fptr(rays), wk.ctypes.data_as(L._ip), cap,
               C.byref(n_out)))
    alive = (rays[:, 6] == 1) & (rays[:, 7] > 0)
    return rays[alive, 0:3].astype(np.float64), rays[alive, 3:6].astype(np.float64), rays[alive, 7].astype(np.float64)


def origin_top(o, O, bits=21):
    """The O most significant bits of path_key.h's origin code (splits dealt to the longest cell)."""
    cell = (hi - lo).copy()
    axes = []
    nb = [0, 0, 0]
    for _ in range(bits):
        a = int(np.argmax(cell))
        cell[a] *= 0.5
        nb[a] += 1
        axes.append(a)
    q = [np.clip(((o[:, a] - lo[a]) * ((1 << nb[a]) / (hi[a] - lo[a]))).astype(np.int64), 0, (1 << nb[a]) - 1)
         for a in range(3)]
    rem = list(nb)
    code = np.zeros(len(o), np.int64)
    for i in range(O):
        a = axes[i]
        rem[a] -= 1
        code = (code << 1) | ((q[a] >> rem[a]) & 1)
    return code


def bins(o, d, O):
    m = ((d[:, 2] < 0) << 2) | ((d[:, 0] < 0) << 1) | (d[:, 1] < 0)
    ad = np.abs(d)
    inv = (4 - 0.001) / np.maximum(ad.max(1), 1e-30)
    dq = ((ad[:, 0] * inv).astype(np.int64) << 4) | ((ad[:, 1] * inv).astype(np.int64) << 2) | (ad[:, 2] * inv).astype(np.int64)
    return (m.astype(np.int64) << (6 + O)) | (origin_top(o, O) << 6) | dq


def texit(o, d):
    with np.errstate(divide='ignore', invalid='ignore'):
        inv = 1.0 / d
        t0, t1 = (lo - o) * inv, (hi - o) * inv
    return np.maximum(t0, t1).min(1)


def sp(a, b):
    return np.corrcoef(np.argsort(np.argsort(a)), np.argsort(np.argsort(b)))[0, 1]


x0, y0 = W // 2 - 256, H // 2 - 128
oA, dA, sA = walks(x0, y0)
oB, dB, sB = walks(x0 + DX, y0)
tB = texit(oB, dB)
print(f'{cfg} bounce {bounce}: A {len(sA)} walks, B {len(sB)} (shift {DX} px); steps mean {sB.mean():.1f}')
print(f'  exit distance: spearman {sp(sB, -tB):.3f}')
for O in (4, 6, 8, 10, 12, 14):
    bA, bB = bins(oA, dA, O), bins(oB, dB, O)
    nbin = 1 << (9 + O)
    sm = np.bincount(bA, sA, nbin)
    cn = np.bincount(bA, None, nbin)
    have = cn[bB] >= 2
    pred = np.where(have, sm[bB] / np.maximum(cn[bB], 1), np.nan)
    # fallback: the exit distance mapped to the steps' scale by rank (only the order matters)
    fb = np.interp(-tB, np.sort(-tB), np.sort(sB))
    pred = np.where(have, pred, fb)
    print(f'  bins O={O:2d}: {np.count_nonzero(cn)} bins used, B covered {have.mean():.3f}, spearman {sp(sB, pred):.3f}')


# --- the tail: list scheduling of window B in class order
import heapq  # noqa: E402

mext = (hi - lo).min()


def classes(v, thr):
    return np.where(v >= thr[0], 0, np.where(v >= thr[1], 1, np.where(v >= thr[2], 2, 3)))


def makespan(order, P):
    h = [0.0] * P
    for c in sB[order]:
        heapq.heappush(h, heapq.heappop(h) + c)
    return max(h)


perm = np.random.default_rng(0).permutation(len(sB))  # the order within a class (a stand-in for the key's)
geo = np.where(tB <= 1.2 * mext, 0, np.where(tB <= 2.7 * mext, 1, np.where(tB <= 6.8 * mext, 2, 3)))
bA, bB = bins(oA, dA, 12), bins(oB, dB, 12)
sm, cn = np.bincount(bA, sA, 1 << 21), np.bincount(bA, None, 1 << 21)
have = cn[bB] >= 2
mean = np.where(have, sm[bB] / np.maximum(cn[bB], 1), 0.0)
shares = [np.mean(geo <= k) for k in range(3)]
orders = {'none': np.zeros(len(sB), int), 'exit distance': geo, 'exact': classes(sB, [256, 128, 64]),
          'bins 256/128/64': np.where(have, classes(mean, [256, 128, 64]), geo),
          'bins by quantile': np.where(have, classes(mean, list(np.quantile(mean[have], [1 - q for q in shares]))), geo)}
for P in (230, 460, 920):
    bound = sB.sum() / P
    print(f'  P={P}: makespan / balance: ' + '  '.join(
        f'{k} {makespan(perm[np.argsort(c[perm], kind="stable")], P) / bound:.4f}' for k, c in orders.items()))
