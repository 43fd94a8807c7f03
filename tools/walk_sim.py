"""Lockstep cost model of the fast walk's schedule (analysis only): replays the per-lane step
records of sampled 8x8 primary-ray waves (ort_debug_walk_steps: the kernel's own fast_step)
under (A) the current per-iteration schedule -- pop + internal-node block every iteration, the
leaf-children loop whenever any lane's node has surviving leaf children -- and (B) leaf
postponement (Aila-Laine speculative while-while): a lane that reaches leaf work parks it and
keeps traversing; the leaf loop runs once every walking lane has parked work (a lane that
reaches a second one waits).  Costs in VALU instructions per wave (model constants below).
usage: python tools/walk_sim.py [config] [block_step] [park_share]"""
import ctypes as C
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

POP, INTERNAL, KID, OBJ, RECOMPUTE = 45, 63, 15, 45, 25
THRESH = float(sys.argv[3]) if len(sys.argv) > 3 else 1.0  # (B) leaf loop once this share of walking lanes parked

cfg = sys.argv[1] if len(sys.argv) > 1 else "c3"
step = int(sys.argv[2]) if len(sys.argv) > 2 else 37
W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
s = ort.random_spheres(N, 42)
t = ort.build_octree(s, D, M)
p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
lib = L.analysis_lib()
f = lib.ort_debug_walk_steps
f.restype = C.c_int64
fp = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
arr = [np.ascontiguousarray(x) for x in (s.center_radius, s.mat_albedo, s.fuzz_ri)]
tt = [np.ascontiguousarray(x) for x in (t.node_min, t.node_max, t.children_offset, t.objects_offset,
                                         t.object_count, t.object_indices)]
nw = ((W + 7) // 8 * ((H + 7) // 8) + step - 1) // step
lens = np.zeros(nw * 64, np.int32)
cap = nw * 64 * 200
steps = np.zeros(cap, np.uint16)
n = f(fp(arr[0]), fp(arr[1]), fp(arr[2]), C.c_int32(s.n), fp(tt[0]), fp(tt[1]), fp(tt[2]), fp(tt[3]), fp(tt[4]),
      C.c_int32(len(t.children_offset)), fp(tt[5]), C.c_int64(len(t.object_indices)), C.byref(p.to_c()),
      C.c_int32(step), fp(lens), C.c_int64(len(lens)), fp(steps), C.c_int64(cap))
assert n >= 0, n
offs = np.concatenate([[0], np.cumsum(lens)])
objs_all = (steps[:n] & 0xff).astype(np.int64)
kids_all = ((steps[:n] >> 8) & 0xf).astype(np.int64)

totA = totB = 0
itA = leafA = itB = leafB = 0
for w in range(nw):
    seqs = []
    for l in range(64):
        a, b = offs[64 * w + l], offs[64 * w + l + 1]
        if b > a:
            seqs.append((objs_all[a:b], kids_all[a:b]))
    if not seqs:
        continue
    # (A) lockstep: iteration k runs pop+internal, and the leaf loop if any lane has leaf work
    mx = max(len(o) for o, _ in seqs)
    for k in range(mx):
        mo = mk = 0
        for o, kd in seqs:
            if k < len(o):
                mo, mk = max(mo, o[k]), max(mk, kd[k])
        totA += POP + INTERNAL
        itA += 1
        if mk:
            totA += KID * mk + OBJ * mo
            leafA += 1
    # (B) postponement
    pos = [0] * len(seqs)
    pend = [None] * len(seqs)
    while True:
        walking = [i for i, (o, _) in enumerate(seqs) if pos[i] < len(o)]
        parked = [i for i in range(len(seqs)) if pend[i] is not None]
        if not walking and not parked:
            break
        movers = [i for i in walking if pend[i] is None or seqs[i][1][pos[i]] == 0]
        if movers and sum(pend[i] is not None for i in walking) < THRESH * len(walking):
            totB += POP + INTERNAL
            itB += 1
            for i in movers:
                o, kd = seqs[i]
                if kd[pos[i]]:
                    pend[i] = (o[pos[i]], kd[pos[i]])
                pos[i] += 1
            continue
        # every walking lane has parked work (or nobody walks): run the leaf loop
        mo = max(pend[i][0] for i in parked)
        mk = max(pend[i][1] for i in parked)
        totB += RECOMPUTE + KID * mk + OBJ * mo
        leafB += 1
        for i in parked:
            pend[i] = None
# (C) fold the leaf-children (LK) nodes into their parent's step: a run of LK steps after a
# step belongs to that step (the parent's surviving children, popped consecutively)
FOLD = 55  # per folded child: its box by selects from the parent's slabs, mid planes, 8 tests
totC = itC = 0
lkall = (steps[:n] & 0x8000) != 0
for w in range(nw):
    macro = []
    for l in range(64):
        a, b = offs[64 * w + l], offs[64 * w + l + 1]
        if b <= a:
            continue
        ms = []
        for i in range(a, b):
            if lkall[i] and ms:
                ms[-1][1].append((objs_all[i], kids_all[i]))
            else:
                ms.append(((objs_all[i], kids_all[i]), []))
        macro.append(ms)
    if not macro:
        continue
    mx = max(len(m) for m in macro)
    for k in range(mx):
        here = [m[k] for m in macro if k < len(m)]
        totC += POP + INTERNAL
        itC += 1
        mo = max(h[0][0] for h in here)
        mk = max(h[0][1] for h in here)
        if mk:
            totC += KID * mk + OBJ * mo
        nch = max(len(h[1]) for h in here)
        for j in range(nch):
            ch = [h[1][j] for h in here if j < len(h[1])]
            totC += FOLD
            mo = max(c[0] for c in ch)
            mk = max(c[1] for c in ch)
            if mk:
                totC += KID * mk + OBJ * mo
print(f"(C) fold leaf-children nodes into the parent step: {totC / nw:.0f} VALU/wave ({itC / nw:.1f} iterations), "
      f"C/A {totC / totA:.3f}")
print(f"{cfg}: {nw} sampled waves; model VALU/wave: A {totA / nw:.0f} ({itA / nw:.1f} iterations, "
      f"{leafA / nw:.1f} leaf loops)  B {totB / nw:.0f} ({itB / nw:.1f} iterations, {leafB / nw:.1f} leaf loops)  "
      f"B/A {totB / totA:.3f}")
print(f"steps/lane {np.mean(lens[lens > 0]):.1f}, leaf-work steps/lane {np.count_nonzero(kids_all) / np.count_nonzero(lens):.1f}, "
      f"objects/leaf-work step {objs_all[kids_all > 0].mean():.2f}")
