#!/usr/bin/env python3
"""Headline benchmark: Mrays/s at 3840x2160, 100k spheres, octree depth 8 (BASELINE.json).

One step = one frame of primary rays (numSamples=1, maxDepth=1 -> one traversal per pixel)
over the seeded synthetic sphere cloud, rendered by the gfx950 kernel with the scene
already resident in HBM (octree built on the GPU by ort_build_scene, byte-identical to the
reference builder; --host-build uses the host builder + upload instead).  `value` counts
traced rays (octree traversals) per second, which for primary-only configs is W*H/s.  With N GPUs (one process per GPU, torchrun) the frame is
partitioned into 16-row bands dealt round-robin to the ranks; each rank renders its bands
into device memory and the bands are gathered to rank 0 over RCCL and de-interleaved into
the final frame -- the gather is inside the timed region.  Total work per step is one
frame whatever N is ("scaling": "strong").

Prints ONE JSON line on rank 0 (contract in the task description).  Extra keys:
  roofline      -- dominant kernel (ort_trace_kernel) against the HBM roof, algorithmic
                   bytes = reference-layout record bytes per SURVEY.md 8(d), counted on the
                   GPU by the kernel's counting variant, / HIP-event kernel time.
  cpu_baseline  -- the CPU oracle (line-by-line restatement of the reference shader; the
                   reference itself has no CPU path) on a bounded row sample, rank 0, N=1.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

CONFIGS = {
    # name: (width, height, spheres, depth, max_spheres_per_node, num_samples, bounce depth)
    "c1": (256, 256, 100, 4, 0, 1, 1),
    "c2": (1920, 1080, 10_000, 6, 0, 1, 1),
    "c3": (3840, 2160, 100_000, 8, 0, 1, 1),
    "c5": (7680, 4320, 1_000_000, 10, 1, 1, 4),
}
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-build", action="store_true", help="build the octree on the host and upload it "
                    "(default: ort_build_scene, the GPU builder)")
    ap.add_argument("--traffic-json", default=str(ROOT / "profiles" / "pmc_traffic.json"),
                    help="PMC-measured HBM bytes per launch (written by tools/pmc_traffic.py)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight, each on its own context and stream (0 = auto: 1 on one GPU, "
                    "2 with N>1, where a band tile's tail would otherwise idle the GPU)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="testing only: every rank on GPU 0 with the gloo backend (exercises the N>1 code "
                    "path on a one-GPU box; not a measurement)")
    ap.add_argument("--save", default="", help="rank 0: save the assembled frame (.pfm/.png)")
    return ap.parse_args()


def main():
    args = parse()
    W, H, NSPH, DEPTH, MPN, NS, MAXD = CONFIGS[args.config]
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    inflight = args.inflight or (1 if world == 1 else 2)
    if inflight > 1:
        # frames in flight only overlap when their streams sit on different hardware queues;
        # with HIP's default 4 queues per process, RCCL's and torch's streams share them
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, 4 * inflight)))

    import torch
    import torch.distributed as dist

    import octreeraytracer_amd as ort

    torch.cuda.set_device(local)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    spheres = ort.random_spheres(NSPH, args.seed)
    rs = [ort.Renderer(local) for _ in range(inflight)]  # one context (scene copy + stream) per frame in flight
    r = rs[0]
    setup = {}
    tree = None
    if args.host_build:  # the reference's CPU builder (restated) + upload
        t0 = time.time()
        tree = ort.build_octree(spheres, DEPTH, MPN)
        setup["host_octree_build_s"] = round(time.time() - t0, 3)
        t0 = time.time()
        for x in rs:
            x.upload(spheres, tree)
        setup["upload_s"] = round((time.time() - t0) / inflight, 3)
    else:  # GPU octree builder, same tree byte for byte (tests/test_gpu_build.py)
        t0 = time.time()
        for x in rs:
            x.build_scene(spheres, DEPTH, MPN)
        setup["gpu_octree_build_ms"] = round(r.last_build_ms(), 2)
        setup["build_scene_wall_s"] = round((time.time() - t0) / inflight, 3)
    info = r.info()
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MAXD)

    # partition: 16-row bands dealt round-robin; every rank renders the same number of rows
    from octreeraytracer_amd.distributed import FrameGather, rank_tile
    tile = rank_tile(W, H, rank, world)
    # inflight+1 band tiles per rank: frame k's gather/assembly overlaps the next frames'
    # renders, and frame k+1 (next context, next stream) fills the tail of frame k
    nslot = inflight + 1
    outs = [torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nslot)]
    out = outs[0]
    gather = FrameGather(dist, W, H, world, rank, "cuda", depth=nslot)
    # each context's own stream (never the HIP null stream, handle 0, which the C ABI reads
    # as "no stream" and renders synchronously)
    streams = [torch.cuda.ExternalStream(x.stream_handle()) for x in rs]
    stream = streams[0]
    gstream = torch.cuda.Stream()
    torch.cuda.set_stream(stream)

    pending = []

    def drain(keep):
        # finish() (RCCL wait + rank-0 assembly into the one frame buffer) on its own stream,
        # so assemblies never overlap each other and never queue behind a render
        frame = None
        with torch.cuda.stream(gstream):
            while len(pending) > keep:
                frame = gather.finish(pending.pop(0))
        return frame

    def step(k, ev=None):
        slot, j = k % nslot, k % inflight
        st = streams[j]
        drain(nslot - 1)  # the previous use of this slot's tile has been gathered
        if world > 1:
            st.wait_stream(gstream)  # ... as far as this frame's stream knows
        torch.cuda.set_stream(st)  # frame k's gather (submit) waits on this stream
        if ev is not None:
            ev[0].record(st)
        rs[j].render(p, tile, out=outs[slot], stream=st.cuda_stream)
        if ev is not None:
            ev[1].record(st)
        pending.append(gather.submit(outs[slot], slot))

    for k in range(args.warmup):
        step(k)
    drain(0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k])
    frame = drain(0)  # every frame gathered and assembled inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]          # whole per-frame pipeline (trace+shade)
    trace_ms = r.trace_times_ms(min(-(-args.steps // inflight), 64))  # dominant kernel, context 0's timed frames
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # algorithmic traffic of this rank's launch (counting variant, untimed); the traced rays
    # of a step = traversals summed over the ranks (W*H*spp for primary-only configs)
    counts = r.count_traffic(p, tile)
    alg_bytes = ort.algorithmic_bytes(counts)
    kern_avg_ms = float(np.mean(kern_ms))
    trace_avg_ms = float(np.mean(trace_ms))
    trav = torch.tensor([counts["traversals"]], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(trav)
    rays_per_frame = int(trav.item())

    result = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_per_frame * args.steps / elapsed / 1e6
        achieved = alg_bytes / (trace_avg_ms * 1e-3) / 1e9
        traffic = None
        tj = Path(args.traffic_json)
        if tj.exists():
            try:
                tr = json.loads(tj.read_text())
                if tr.get("config") == args.config and tr.get("tile_rows") == tile.rows:
                    traffic = int(tr.get("hbm_bytes_per_launch"))
            except Exception:
                traffic = None
        result = {
            "metric": "Mrays/sec at 3840x2160, 100k spheres, depth 8; 1/2/4/8-GPU scaling",
            "value": round(value, 2),
            "unit": "Mrays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded generateRandomSpheres restatement, mt19937 seed %d)" % args.seed,
            "config": {
                "workload": f"{args.config}: {W}x{H} camera rays (spp={NS}, bounces={MAXD}), {NSPH} spheres, "
                            f"octree depth {DEPTH}, maxSpheresPerNode {MPN}",
                "width": W, "height": H, "spheres": NSPH, "octree_depth": DEPTH, "max_spheres_per_node": MPN,
                "num_samples": NS, "max_bounces": MAXD, "nodes": info["n_nodes"], "indices": info["n_indices"],
                "layout": info["layout"], "partition": "16-row bands round-robin + RCCL gather (async, "
                "overlapping the next frame's render)" if world > 1
                else "full frame", "frames_in_flight": inflight, "rays_per_step": rays_per_frame, "rays": "traced rays (octree traversals), "
                "all bounces and ranks",
            },
            "frame_gpu_ms_avg": round(kern_avg_ms, 4),
            "trace_kernel_ms_avg": round(trace_avg_ms, 4),
            "trace_kernel_ms_min": round(float(np.min(trace_ms)), 4),
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": int(alg_bytes),
                "bytes_per_ray": round(alg_bytes / max(1, counts["pixels"]), 1),
                "counts": counts,
                "kernel": "ort_trace_compact<false,true,true> (camera rays + octree walk + shading)",
                "note": "achieved = reference-layout record bytes (SURVEY.md 8(d)) the reference walk reads per "
                        "frame / trace-kernel time; this kernel reads far fewer bytes (compact layout, L2/MALL "
                        "residency) and is instruction-issue bound -- see traffic and DESIGN.md",
            },
            "setup": setup,
        }
        if world == 1 and not args.no_cpu_baseline:
            if tree is None:
                t0 = time.time()
                tree = ort.build_octree(spheres, DEPTH, MPN)  # the oracle walks the host tree
                setup["host_octree_build_s"] = round(time.time() - t0, 3)
            result["cpu_baseline"] = cpu_baseline(spheres, tree, p, args.cpu_seconds)
        if args.save:
            img = frame.cpu().numpy()
            from octreeraytracer_amd import image
            (image.write_png if args.save.endswith(".png") else image.write_pfm)(args.save, img)
    for x in rs:
        x.close()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def cpu_baseline(spheres, tree, p, budget_s):
    """Oracle on the host cores over evenly spaced full rows, sized to ~budget_s of wall time."""
    from oracle import oracle
    threads = min(16, os.cpu_count() or 1)

    def run(n):
        stride = max(1, p.height // n)
        t0 = time.perf_counter()
        oracle.render(spheres, tree, p, 0, stride // 2, p.width, n, band_height=1, band_stride=stride, threads=threads)
        return time.perf_counter() - t0, stride

    n = 2 * threads
    dt, _ = run(n)  # calibration sample
    n = int(max(n, min(p.height, n * budget_s / max(dt, 1e-3))))
    dt, stride = run(n)
    rays = n * p.width * p.num_samples
    # one core (report all cores and 1 core), a smaller row sample
    n1 = max(2, min(p.height, int(n * 0.25 * budget_s / max(dt * threads, 1e-3))))
    stride1 = max(1, p.height // n1)
    t0 = time.perf_counter()
    oracle.render(spheres, tree, p, 0, stride1 // 2, p.width, n1, band_height=1, band_stride=stride1, threads=1)
    dt1 = time.perf_counter() - t0
    rays1 = n1 * p.width * p.num_samples
    return {"value": round(rays / dt / 1e6, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"{n} of {p.height} rows (every {stride}th), {rays} camera rays, {dt:.1f} s wall; "
                      f"oracle/ort_oracle.c -O3, OpenMP dynamic over rows",
            "value_1core": round(rays1 / dt1 / 1e6, 3),
            "sample_1core": f"{n1} rows (every {stride1}th), {rays1} camera rays, {dt1:.1f} s wall, 1 thread"}


if __name__ == "__main__":
    main()
