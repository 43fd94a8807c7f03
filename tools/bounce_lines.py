"""How many distinct cache lines a wave's lanes load per load instruction in the bounce walks,
under different orders of the bounce list (analysis only, CPU).  The rays of bounce B of a
window of a config's frame come from the host restatement of the path
(`ort_debug_bounce_walks`), each with the node records (16-byte interleaved records: 8 per
128-byte line) and leaf objects (16-byte records) its bounce walk loads, step by step.  The
list is ordered by a key, dealt to waves as the persistent kernel deals it (64-item chunks
from one global cursor, idle lanes refilled once `refill` are idle), and each wave's lanes
step in lockstep; per load instruction the distinct lines among the lanes that load are
counted (the quantity `TCP_TOTAL_CACHE_ACCESSES / SQ_INSTS_VMEM_RD` measures on the GPU,
`tools/pmc_mem.sh`).
usage: python tools/bounce_lines.py [config] [bounce] [x0 y0 w h] ..."""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402

MORTON = 21


def morton_plan(lo, hi, bits):
    cell = np.where((hi - lo) > 0, hi - lo, 0.0).astype(np.float64)
    nb = [0, 0, 0]
    axes = []
    for _ in range(bits):
        a = int(np.argmax(cell))  # first longest (as mortonPlan: strictly longer wins)
        cell[a] *= 0.5
        nb[a] += 1
        axes.append(a)
    return axes, nb


def origin_code(o, lo, hi, bits):
    """path_key.h's origin code: bits dealt to the longest cell axis, MSB first (float32 math)."""
    axes, nb = morton_plan(lo, hi, bits)
    q = []
    for a in range(3):
        ext = np.float32(hi[a] - lo[a])
        scale = np.float32((1 << nb[a]) / ext) if ext > 0 else np.float32(0)
        x = (o[:, a].astype(np.float32) - np.float32(lo[a])) * scale
        top = np.float32((1 << nb[a]) - 1)
        qa = np.where(x <= 0, 0, np.where(x >= top, top, np.floor(x))).astype(np.uint64)
        q.append(qa)
    rem = list(nb)
    code = np.zeros(len(o), np.uint64)
    for i, a in enumerate(axes):
        rem[a] -= 1
        code |= ((q[a] >> np.uint64(rem[a])) & np.uint64(1)) << np.uint64(bits - 1 - i)
    return code


def dir_code(d, bits):
    ax, ay, az = np.abs(d[:, 0]), np.abs(d[:, 1]), np.abs(d[:, 2])
    inv = np.float32((1 << bits) - 0.001) / np.maximum(np.maximum(ax, ay), np.maximum(az, np.float32(1e-30)))
    f = lambda v: (v * inv).astype(np.uint64)  # noqa: E731
    return (f(ax) << np.uint64(2 * bits)) | (f(ay) << np.uint64(bits)) | f(az)


def octant(d):
    return ((d[:, 2] < 0).astype(np.uint64) << np.uint64(2)) | ((d[:, 0] < 0).astype(np.uint64) << np.uint64(1)) | \
        (d[:, 1] < 0).astype(np.uint64)


def keys(name, o, d, lo, hi):
    """Sort keys (uint64) of the list orders compared."""
    U = np.uint64
    if name == "slot":
        return np.arange(len(o), dtype=np.uint64)
    if name == "random":
        return np.random.default_rng(0).permutation(len(o)).astype(np.uint64)
    m = octant(d)
    if name == "cur":  # octant | 21-bit origin | 2 direction bits per axis (path_key.h)
        return (m << U(27)) | (origin_code(o, lo, hi, 21) << U(6)) | dir_code(d, 2)
    if name.startswith("hi"):  # octant | origin high bits | direction | origin low bits
        h = int(name[2:])
        c = origin_code(o, lo, hi, 21)
        lo_bits = 21 - h
        return (m << U(27)) | ((c >> U(lo_bits)) << U(6 + lo_bits)) | (dir_code(d, 2) << U(lo_bits)) | \
            (c & U((1 << lo_bits) - 1))
    if name.startswith("w"):  # wide (64-bit) keys: octant | origin bits | direction bits per axis
        ob, db = (int(x) for x in name[1:].split("d"))
        return (m << U(ob + 3 * db)) | (origin_code(o, lo, hi, ob) << U(3 * db)) | dir_code(d, db)
    if name.startswith("s"):  # octant | origin high | dir bits per axis | origin low (64-bit)
        h, db = (int(x) for x in name[1:].split("d"))
        c = origin_code(o, lo, hi, 24)
        lo_bits = 24 - h
        return (m << U(24 + 3 * db)) | ((c >> U(lo_bits)) << U(3 * db + lo_bits)) | (dir_code(d, db) << U(lo_bits)) | \
            (c & U((1 << lo_bits) - 1))
    raise ValueError(name)


def simulate(order, starts, lens, walks, n_waves=128, chunk=64, refill=16):
    """The persistent kernel's schedule over the ordered list: returns (node-load instructions,
    node lines, object-load instructions, object lines, lane-steps, wave iterations)."""
    n = len(order)
    n_chunks = (n + chunk - 1) // chunk
    cursor = 0
    res = np.zeros(6, np.int64)
    # waves take chunks from one cursor in turn (round robin stands in for "whoever asks")
    waves = [dict(items=[], ray=[-1] * 64, pos=[0] * 64) for _ in range(n_waves)]
    active = list(range(n_waves))
    while active:
        still = []
        for w in active:
            W = waves[w]
            idle = [l for l in range(64) if W["ray"][l] < 0]
            if len(idle) >= refill and (W["items"] or cursor < n_chunks):
                if not W["items"] and cursor < n_chunks:
                    W["items"] = list(order[cursor * chunk:min(n, (cursor + 1) * chunk)])
                    cursor += 1
                for l in idle:
                    if not W["items"]:
                        break
                    r = W["items"].pop(0)
                    W["ray"][l] = r
                    W["pos"][l] = 0
                res[5] += 1
                still.append(w)
                continue
            lanes = [l for l in range(64) if W["ray"][l] >= 0]
            if not lanes:
                if W["items"] or cursor < n_chunks:
                    still.append(w)
                continue
            # one step: every walking lane loads its node's record; leaf lanes load objects
            nodes, objs = [], []
            for l in lanes:
                r = W["ray"][l]
                s = starts[r] + W["pos"][l]
                nodes.append(walks[s, 0] >> 3)
                if walks[s, 1] >= 0:
                    objs.append((walks[s, 1], walks[s, 2]))
                W["pos"][l] += 1
                if W["pos"][l] >= lens[r]:
                    W["ray"][l] = -1
            res[0] += 1
            res[1] += len(set(nodes))
            if objs:
                kmax = max(c for _, c in objs)
                for i in range(kmax):
                    ln = {(e + i) >> 3 for e, c in objs if c > i}
                    res[2] += 1
                    res[3] += len(ln)
            res[4] += len(lanes)
            res[5] += 1
            still.append(w)
        active = still
    return res


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    bounce = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
    wins = [int(x) for x in sys.argv[3:]] or [W // 2 - 160, H // 2 - 160, 320, 320]
    t0 = time.time()
    s = ort.random_spheres(N, 42)
    t = ort.build_octree(s, D, M)
    print(f"{cfg}: tree {t.n_nodes} nodes built in {time.time() - t0:.0f} s", flush=True)
    lo, hi = t.node_min[0].astype(np.float64), t.node_max[0].astype(np.float64)
    p = ort.FrameParams.default_camera(W, H, num_samples=1, max_depth=MD)
    lib = L.analysis_lib()
    f = lib.ort_debug_bounce_walks
    f.restype = C.c_int
    f.argtypes = [L._fp, L._fp, L._fp, C.c_int32, L._fp, L._fp, L._ip, L._ip, L._ip, C.c_int32, L._ip, C.c_int64,
                  C.POINTER(L.OrtParams), C.POINTER(L.OrtTile), C.c_int32, L._fp, L._ip, C.c_int64,
                  C.POINTER(C.c_int64)]
    arr = [np.ascontiguousarray(a, dt) for a, dt in (
        (s.center_radius, np.float32), (s.mat_albedo, np.float32), (s.fuzz_ri, np.float32),
        (t.node_min, np.float32), (t.node_max, np.float32), (t.children_offset, np.int32),
        (t.objects_offset, np.int32), (t.object_count, np.int32), (t.object_indices, np.int32))]
    for wi in range(0, len(wins), 4):
        x0, y0, ww, hh = wins[wi:wi + 4]
        tile = ort.Tile(x0, ww, y0, hh)
        rays = np.zeros((ww * hh, 8), np.float32)
        cap = ww * hh * 400
        walks = np.zeros((cap, 3), np.int32)
        n_out = C.c_int64()
        t1 = time.time()
        L.check(f(L.fptr(arr[0]), L.fptr(arr[1]), L.fptr(arr[2]), s.n, L.fptr(arr[3]), L.fptr(arr[4]), L.iptr(arr[5]),
                  L.iptr(arr[6]), L.iptr(arr[7]), t.n_nodes, L.iptr(arr[8]), t.n_indices, C.byref(p.to_c()),
                  C.byref(tile.to_c()), bounce, L.fptr(rays), walks.ctypes.data_as(L._ip), cap, C.byref(n_out)))
        if n_out.value > cap:
            raise SystemExit("walk record cap exceeded")
        alive = (rays[:, 6] == 1) & (rays[:, 7] > 0)
        lens = rays[:, 7].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(lens)])[:-1]
        idx = np.nonzero(alive)[0]
        print(f"window {x0},{y0} {ww}x{hh}, bounce {bounce}: {len(idx)} walking rays of {ww * hh} pixels, "
              f"{lens[idx].mean():.1f} steps/ray ({time.time() - t1:.0f} s)", flush=True)
        o, d = rays[idx, 0:3], rays[idx, 3:6]
        U = np.uint64
        ln = lens[idx].astype(np.float64)
        # heavy first's classes (ORT_OPT_HEAVY_FIRST 64; a static camera's last-frame steps = these)
        hf = np.where(ln >= 256, 0, np.where(ln >= 128, 1, np.where(ln >= 64, 2, 3))).astype(U)
        kc = keys("cur", o, d, lo, hi)
        m = octant(d)

        def node_at(j):
            return np.array([walks[starts[i] + min(j, lens[i] - 1), 0] for i in idx], U)

        fl = np.zeros(len(idx), U)
        for q, i in enumerate(idx):
            seg = walks[starts[i]:starts[i] + lens[i]]
            lf = np.nonzero(seg[:, 1] >= 0)[0]
            fl[q] = seg[lf[0], 0] if len(lf) else (1 << 31)
        runs = [("slot order", keys("slot", o, d, lo, hi), 16), ("random order", keys("random", o, d, lo, hi), 16),
                ("key (no classes)", kc, 16), ("key + heavy first", (hf << U(40)) | kc, 16)]
        runs += [(f"key + heavy first, refill {rf}", (hf << U(40)) | kc, rf) for rf in (8, 24, 32, 48, 64)]
        runs += [("key + log2(steps) class", ((U(99) - np.floor(np.log2(np.maximum(ln, 1))).astype(U)) << U(40)) | kc, 16)]
        for name in ("hi15", "hi9", "w24d3", "s15d3"):
            runs.append((f"key variant {name} + heavy first", (hf << U(60)) | keys(name, o, d, lo, hi), 16))
        for j in (6, 20):  # oracle orders: what the walk itself will load (not computable before it)
            runs.append((f"ORACLE node at step {j}", (hf << U(60)) | (m << U(56)) | (node_at(j) << U(24)) |
                         (kc & U((1 << 24) - 1)), 16))
        runs.append(("ORACLE first leaf", (hf << U(60)) | (m << U(56)) | (fl << U(24)), 16))
        for name, k, rf in runs:
            order = idx[np.argsort(k, kind="stable")]
            r = simulate(order, starts, lens, walks, refill=rf)
            print(f"  {name:34s}: node lines/load {r[1] / r[0]:5.2f}, object lines/load {r[3] / max(1, r[2]):5.2f}, "
                  f"all {(r[1] + r[3]) / (r[0] + r[2]):5.2f}; lane use {r[4] / (64 * r[0]):.3f}; node loads {r[0]}, "
                  f"lines {r[1] + r[3]}", flush=True)


if __name__ == "__main__":
    main()
