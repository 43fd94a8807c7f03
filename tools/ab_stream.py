"""Interleaved A/B timing of libort.so builds in bench.py's steady state: scene built on the
GPU, device output, each build's frames back to back on its own stream (no host sync per
frame), builds alternating in blocks of --block frames in ABBA order so clock and thermal
drift hit every build alike.  Also checks that every build writes bit-identical frames.
usage: python tools/ab_stream.py LIB_A LIB_B [...] [--config c3] [--rounds 12] [--block 10]
       [--world N] [--max-depth D] [--samples S] [--spheres N] [--tree-depth D] [--yaw-step DEG]
A build may carry options: path@option=value,... with option one of the Renderer setters
(e.g. build/ab/libA.so@xcd_swizzle=0).

Each build runs in a worker process of its own (all resident on the GPU, one rendering at a
time): two builds loaded into ONE process share kernel names, and the HIP runtime then
launched one build's kernels with the other's argument layout -- wrong frames, bogus times."""
import argparse
import hashlib
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import numpy as np  # noqa: E402


def morton_order(s):
    """The sphere set with its spheres (ids) in Morton order of their centres (10 bits per axis)."""
    from octreeraytracer_amd.scene import SphereSet
    c = s.center_radius[:, :3].astype(np.float64)
    lo, hi = c.min(0), c.max(0)
    q = np.clip(((c - lo) / np.maximum(hi - lo, 1e-30) * 1023).astype(np.int64), 0, 1023)
    code = np.zeros(len(c), np.int64)
    for b in range(10):
        for a in range(3):
            code |= ((q[:, a] >> b) & 1) << (3 * b + a)
    o = np.argsort(code, kind="stable")
    return SphereSet(s.center_radius[o].copy(), s.mat_albedo[o].copy(), s.fuzz_ri[o].copy())


def config_shape(args):
    """The config's (W, H, N, D, M, NS, MD) with the command line's overrides."""
    import bench
    W, H, N, D, M, NS, MD = bench.CONFIGS[args.config]
    return (W, H, args.spheres or N, args.tree_depth or D, M, args.samples or NS, args.max_depth or MD)


def worker(spec, shape, block, world=1, yaw_step=0.0):
    import ctypes as C

    import torch

    import bench
    import octreeraytracer_amd as ort
    from octreeraytracer_amd import _lib as L

    W, H, N, D, M, NS, MD = shape
    path, _, opts = spec.partition("@")
    lib = C.CDLL(str(Path(path).resolve()), mode=C.RTLD_LOCAL)
    L._declare(lib, debug="present")
    L._lib = lib
    r = ort.Renderer(0)
    spheres = ort.random_spheres(N, 42)
    for o in filter(None, opts.split(",")):
        name, val = o.split("=")
        if name == "morton":  # scene experiment: sphere ids renumbered in Morton order (other pixels)
            if int(val):
                spheres = morton_order(spheres)
            continue
        getattr(r, "set_" + name)(int(val))
    r.build_scene(spheres, D, M)
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD)
    from octreeraytracer_amd.scene import DEFAULT_YAW
    moving = [ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MD, yaw=DEFAULT_YAW + yaw_step * j)
              for j in range(64)] if yaw_step else [p]
    frame = 0
    from octreeraytracer_amd.distributed import rank_tile
    tile = rank_tile(W, H, 0, world)  # world > 1: rank 0's band tile of an N-GPU frame
    out = torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda")
    st = torch.cuda.ExternalStream(r.stream_handle())
    print("ready", flush=True)
    for line in sys.stdin:
        if line.strip() == "hash":
            print(hashlib.md5(out.cpu().numpy().tobytes()).hexdigest(), flush=True)
            continue
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(block):  # a moving camera (--yaw-step) turns back and forth over 64 frames
            j = frame % (2 * len(moving))
            r.render(moving[min(j, 2 * len(moving) - 1 - j)], tile, out=out, stream=st.cuda_stream)
            frame += 1
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / block * 1e3
        print(dt, float(np.median(r.trace_times_ms(block))), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--config", default="c3")
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--block", type=int, default=10)
    ap.add_argument("--max-depth", type=int, default=0, help="override the config's ray bounce depth")
    ap.add_argument("--samples", type=int, default=0, help="override the config's samples per pixel")
    ap.add_argument("--spheres", type=int, default=0, help="override the config's sphere count")
    ap.add_argument("--tree-depth", type=int, default=0, help="override the config's octree depth")
    ap.add_argument("--world", type=int, default=1, help="time rank 0's band tile of this many GPUs")
    ap.add_argument("--yaw-step", type=float, default=0.0, help="moving camera: degrees of yaw per frame")
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        return worker(args.libs[0], config_shape(args), args.block, args.world, args.yaw_step)
    W, H, N, D, M, NS, MD = config_shape(args)
    procs = []
    for spec in args.libs:
        procs.append(subprocess.Popen([sys.executable, "-u", __file__, spec, "--worker", "--config", args.config,
                                       "--block", str(args.block), "--max-depth", str(args.max_depth),
                                       "--samples", str(args.samples), "--spheres", str(args.spheres),
                                       "--tree-depth", str(args.tree_depth),
                                       "--world", str(args.world), "--yaw-step", str(args.yaw_step)], stdin=subprocess.PIPE, stdout=subprocess.PIPE,
                                      text=True, cwd=str(ROOT)))
        while procs[-1].stdout.readline().strip() != "ready":
            if procs[-1].poll() is not None:
                raise SystemExit(f"worker for {spec} died")
    n = len(procs)
    per_frame = [[] for _ in range(n)]
    trace = [[] for _ in range(n)]

    def ask(i, cmd):
        procs[i].stdin.write(cmd + "\n")
        procs[i].stdin.flush()
        ans = procs[i].stdout.readline()
        if not ans:
            raise SystemExit(f"worker {args.libs[i]} died")
        return ans.split()

    for i in range(n):
        ask(i, "block")  # warm-up
    for k in range(args.rounds):
        for i in (range(n) if k % 2 == 0 else reversed(range(n))):
            f, tr = ask(i, "block")
            per_frame[i].append(float(f))
            trace[i].append(float(tr))
    hashes = [ask(i, "hash")[0] for i in range(n)]
    for p in procs:
        p.stdin.close()
        p.wait()
    for i in range(1, n):
        if hashes[i] != hashes[0]:
            print(f"WARNING: build {args.libs[i]} writes a different frame than {args.libs[0]}")
    base = np.median(per_frame[0])
    for i, spec in enumerate(args.libs):
        f, tr = np.median(per_frame[i]), np.median(trace[i])
        print(f"{args.config} {spec.split('/')[-1]:24s} frame {f:.4f} ms (min {np.min(per_frame[i]):.4f})  "
              f"trace {tr:.4f} ms  -> {W * H * NS / args.world / f / 1e3:.1f} M camera rays/s  "
              f"({base / f:.3f}x of {args.libs[0].split('/')[-1]})")


if __name__ == "__main__":
    main()
