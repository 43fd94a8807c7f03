"""Would a denser or treelet node layout put a wave's lanes on fewer cache lines per load in the
bounce walks?  (Analysis only, CPU)

The persistent bounce kernel is bound by its vector-memory path: ~32 L1 tag lookups per wave
load instruction, one 128-byte line per lane that loads.  A layout can only lower
that count by putting the records that the lanes of ONE load instruction need into fewer lines;
a lane's own next record sharing its current line does not help there (at 24 waves per CU a
line is evicted from the 32 KiB L1 long before the same wave's next step: 256 lines, ~32 new
lines per wave step), and L2 already serves 88 % of the requests.  So this model replays the
bounce walks of a window of the frame under the persistent kernel's schedule
(tools/bounce_lines.py: sorted list, 64-item chunks, refill at 16 idle lanes, lockstep) and
counts distinct lines per node-record load for record layouts:

  nk16      16-byte {record, kid entry} (today: a sibling group = one line), BFS order
  rec8      8-byte records (kid entries elsewhere: a second load per step not counted), BFS
  rec8-dfs  8-byte records, sibling groups in depth-first order (a group and its DFS successor
            -- its first child's group -- share a line)
  rec4      4-byte records, BFS;   rec4-dfs: 4 groups per line, depth-first

usage: python tools/treelet_lines.py [config] [bounce] [x0 y0 w h]
"""
import ctypes as C
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import bench  # noqa: E402
import bounce_lines as BL  # noqa: E402
import octreeraytracer_amd as ort  # noqa: E402
from octreeraytracer_amd import _lib as L  # noqa: E402


def simulate_lines(order, starts, lens, line_of, n_waves=128, chunk=64, refill=16):
    """bounce_lines.simulate with a per-walk-record line id: (node loads, node lines, lane-steps)."""
    n = len(order)
    n_chunks = (n + chunk - 1) // chunk
    cursor = 0
    loads = lines = lane_steps = 0
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
                    W["ray"][l] = W["items"].pop(0)
                    W["pos"][l] = 0
                still.append(w)
                continue
            lanes = [l for l in range(64) if W["ray"][l] >= 0]
            if not lanes:
                if W["items"] or cursor < n_chunks:
                    still.append(w)
                continue
            seen = set()
            for l in lanes:
                r = W["ray"][l]
                seen.add(line_of[starts[r] + W["pos"][l]])
                W["pos"][l] += 1
                if W["pos"][l] >= lens[r]:
                    W["ray"][l] = -1
            loads += 1
            lines += len(seen)
            lane_steps += len(lanes)
            still.append(w)
        active = still
    return loads, lines, lane_steps


def dfs_group_rank(co):
    """Rank of each sibling group (children of one node, 8 consecutive records starting at
    childrenOffset) in depth-first pre-order of the groups; group id = (childrenOffset - 1) / 8
    (the breadth-first builder puts the root alone at 0 and every group at 1 + 8 j)."""
    n_groups = (len(co) - 1) // 8
    rank = np.full(n_groups, -1, np.int64)
    nxt = 0
    stack = [0]  # nodes whose children group is next to rank
    while stack:
        v = stack.pop()
        c = int(co[v])
        if c < 0:
            continue
        g = (c - 1) >> 3
        rank[g] = nxt
        nxt += 1
        for o in range(7, -1, -1):  # child 0's group first
            stack.append(c + o)
    return rank


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "c5"
    bounce = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    W, H, N, D, M, NS, MD = bench.CONFIGS[cfg]
    win = [int(x) for x in sys.argv[3:7]] or [W // 2 - 128, H // 2 - 128, 256, 256]
    t0 = time.time()
    s = ort.random_spheres(N, 42)
    t = ort.build_octree(s, D, M)
    print(f"{cfg}: tree {t.n_nodes} nodes built in {time.time() - t0:.0f} s", flush=True)
    co = np.ascontiguousarray(t.children_offset, np.int32)
    assert co[0] == 1 and ((co[co >= 0] - 1) % 8 == 0).all()  # BFS sibling groups at 1 + 8 j
    t0 = time.time()
    grank = dfs_group_rank(co)
    print(f"depth-first group order in {time.time() - t0:.0f} s", flush=True)
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
    x0, y0, ww, hh = win
    tile = ort.Tile(x0, ww, y0, hh)
    rays = np.zeros((ww * hh, 8), np.float32)
    cap = ww * hh * 400
    walks = np.zeros((cap, 3), np.int32)
    n_out = C.c_int64()
    L.acheck(f(L.fptr(arr[0]), L.fptr(arr[1]), L.fptr(arr[2]), s.n, L.fptr(arr[3]), L.fptr(arr[4]), L.iptr(arr[5]),
               L.iptr(arr[6]), L.iptr(arr[7]), t.n_nodes, L.iptr(arr[8]), t.n_indices, C.byref(p.to_c()),
               C.byref(tile.to_c()), bounce, L.fptr(rays), walks.ctypes.data_as(L._ip), cap, C.byref(n_out)))
    if n_out.value > cap:
        raise SystemExit("walk record cap exceeded")
    alive = (rays[:, 6] == 1) & (rays[:, 7] > 0)
    lens = rays[:, 7].astype(np.int64)
    starts = np.concatenate([[0], np.cumsum(lens)])[:-1]
    idx = np.nonzero(alive)[0]
    print(f"window {x0},{y0} {ww}x{hh}, bounce {bounce}: {len(idx)} walking rays, {lens[idx].mean():.1f} steps/ray",
          flush=True)
    o, d = rays[idx, 0:3], rays[idx, 3:6]
    lo, hi = t.node_min[0].astype(np.float64), t.node_max[0].astype(np.float64)
    ln = lens[idx].astype(np.float64)
    U = np.uint64
    hf = np.where(ln >= 256, 0, np.where(ln >= 128, 1, np.where(ln >= 64, 2, 3))).astype(U)
    order = idx[np.argsort((hf << U(40)) | BL.keys("cur", o, d, lo, hi), kind="stable")]
    node = walks[:n_out.value, 0].astype(np.int64)
    grp = np.where(node > 0, (node - 1) >> 3, -1)
    slot = np.where(node > 0, (node - 1) & 7, 0)
    dpos = np.where(node > 0, grank[np.maximum(grp, 0)] * 8 + slot + 1, 0)  # node's place, groups depth-first
    layouts = {"nk16 (today)": node >> 3, "rec8": node >> 4, "rec8-dfs": dpos >> 4, "rec4": node >> 5,
               "rec4-dfs": dpos >> 5}
    base = None
    for name, line_of in layouts.items():
        ld, lines, lanes = simulate_lines(order, starts, lens, line_of)
        per = lines / ld
        base = base or per
        print(f"  {name:14s}: node lines / load {per:6.2f} ({per / base - 1:+.1%}); lanes per load {lanes / ld:5.1f}",
              flush=True)


if __name__ == "__main__":
    main()
