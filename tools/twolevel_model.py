"""Would a two-level node record cut the C5 bounce walks' DEPENDENT loads?  (Analysis only, CPU;
VERDICT r05 item 3.)

The proposal: with breadth-first numbering a node's grandchildren are derivable without loading
its children -- for an internal child c of N, c's children start at childrenOffset(N's first
internal child) + 8 * rank(c among N's internal children) -- so a record R(N) holding N's
internal-child mask, a 64-bit grandchild-occupancy mask and the grandchild base lets the walk
test a node's children and enter a child without first loading that child's record.  R(X) is
still loaded for every internal node X the walk visits (its children need it), and every leaf's
record still is (its object list), so the number of record loads per walk is unchanged; what
changes is how soon a load is needed after it is issued:

  today (16-byte {record, kid entry}): every visited node's record is needed by the step that
  visits it (distance 0: issued by the pop, waited on after the pop's plane reads);
  two-level: a visited leaf's record likewise (distance 0); an internal node X needs R(parent X)
  -- issued one step earlier if the walk descended from its parent (distance 1), two or more
  steps earlier after a backtrack.

This replays the restatement's own bounce walks (ort_debug_bounce_walks: the rays of bounce 1 of
a window of the C5 frame, every node each walk visits, in order) and counts, per walk, the
visits by that distance, and the 128-byte lines per load of the persistent kernel's schedule for
the 16-byte record and for a 32-byte two-level record (tools/treelet_lines.py's model).

usage: python tools/twolevel_model.py [config] [bounce] [x0 y0 w h]
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
from treelet_lines import simulate_lines  # noqa: E402


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
    # parent of every sibling group (children of one node at 1 + 8 g)
    n_groups = (t.n_nodes - 1) // 8
    parent_of_group = np.full(n_groups, -1, np.int64)
    internal = np.nonzero(co >= 0)[0]
    parent_of_group[(co[internal].astype(np.int64) - 1) >> 3] = internal
    del internal
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
    rec = walks[:n_out.value]
    node = rec[:, 0].astype(np.int64)
    leaf = rec[:, 1] >= 0
    par = np.where(node > 0, parent_of_group[np.maximum((node - 1) >> 3, 0)], -1)
    prev = np.concatenate([[-2], node[:-1]])
    first = np.zeros(len(node), bool)
    first[starts[idx]] = True  # a walk's first visit (the root): no earlier step
    descent = (~leaf) & (~first) & (par == prev)
    backtrack = (~leaf) & (~first) & (par != prev)
    n_vis = len(node) - int(first.sum())
    n_leaf = int((leaf & ~first).sum())
    n_desc, n_back = int(descent.sum()), int(backtrack.sum())
    walks_n = len(idx)
    print(f"  visits per walk {n_vis / walks_n:.1f} (the root's excluded): leaves {n_leaf / walks_n:.1f}, "
          f"internal after a descent {n_desc / walks_n:.1f}, internal after a backtrack {n_back / walks_n:.1f}")
    print(f"  record loads per walk: today {n_vis / walks_n:.1f}, two-level {n_vis / walks_n:.1f} (unchanged)")
    print(f"  loads needed by the step that issues them (distance 0): today {n_vis / walks_n:.1f}, two-level "
          f"{n_leaf / walks_n:.1f} ({n_leaf / n_vis - 1:+.1%}); needed one step later (distance 1): two-level "
          f"{n_desc / walks_n:.1f}; two or more: {n_back / walks_n:.1f}")
    # lines per load under the persistent kernel's schedule: 16-byte records (8 per line) vs a
    # 32-byte two-level record (record + kid entry + 64-bit grandchild mask + base: 4 per line)
    lo, hi = t.node_min[0].astype(np.float64), t.node_max[0].astype(np.float64)
    o, d = rays[idx, 0:3], rays[idx, 3:6]
    ln = lens[idx].astype(np.float64)
    U = np.uint64
    hf = np.where(ln >= 256, 0, np.where(ln >= 128, 1, np.where(ln >= 64, 2, 3))).astype(U)
    order = idx[np.argsort((hf << U(40)) | BL.keys("cur", o, d, lo, hi), kind="stable")]
    base = None
    for name, line_of in (("nk16 (today)", node >> 3), ("two-level 32 B", node >> 2)):
        ld, lines, lanes = simulate_lines(order, starts, lens, line_of)
        per = lines / ld
        base = base or per
        print(f"  {name:16s}: node lines / load {per:6.2f} ({per / base - 1:+.1%}); lanes per load {lanes / ld:5.1f}",
              flush=True)


if __name__ == "__main__":
    main()
