#!/usr/bin/env python3
"""Headline benchmark: Mrays/s at 3840x2160, 100k spheres, octree depth 8 (BASELINE.json).

One step = one frame of primary rays (numSamples=1, maxDepth=1 -> one traversal per pixel)
over the seeded synthetic sphere cloud, rendered by the gfx950 kernel with the scene
already resident in HBM (octree built on the GPU by ort_build_scene, byte-identical to the
reference builder; --host-build uses the host builder + upload instead).  `value` counts
traced rays (octree traversals, every bounce) per second, which for primary-only configs is
W*H/s.  With N GPUs (one process per GPU) the frame is partitioned into 16-row bands dealt
round-robin to the ranks; each rank renders its bands into device memory and the bands are
gathered to rank 0 over RCCL and de-interleaved into the final frame -- the gather is inside
the timed region.  Total work per step is one frame whatever N is ("scaling": "strong").

`python bench.py --gpus N` (N > 1) without a launcher starts its own N ranks: it runs
`torch.distributed.run` as a child process before anything touches a GPU and passes rank 0's
line through.

Prints ONE JSON line on rank 0 (contract in the task description).  Extra keys:
  roofline      -- the frame's trace kernels (all bounces) against the VALU issue roof: the
                   kernel is instruction-issue bound.  achieved = VALU
                   wave-instructions per frame (rocprofv3 PMC SQ_INSTS_VALU, committed under
                   profiles/pmc_<config>.json) / the trace kernels' summed HIP-event time
                   measured live in this run; peak = 1024 SIMDs x 2.4 GHz / 2 cycles per
                   wave64 VALU instruction (MI355X_MICROARCH.md).  hbm_frac and the
                   reference-layout byte rate are reported beside it.
  cpu_baseline  -- the CPU oracle (line-by-line restatement of the reference shader; the
                   reference itself has no CPU path) on a bounded row sample, rank 0, N=1.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
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
    # the reference's own workloads: src/config.h:10-28's default build (16 samples x 8 bounces)
    # and analysis/stats.csv:114's sweep row -- whole-pixel paths (ORT_OPT_PIXEL_PATHS auto)
    "ref_default": (800, 600, 100, 3, 0, 16, 8),
    "ref_stats114": (1920, 1080, 1000, 5, 1, 16, 8),
}
def pixel_paths_auto(n_nodes, ns, maxd):
    """ort_kernel.hip use_pixel_paths' auto rule on a tree (kPixelPathsAutoNodes, ...5, ...8)."""
    if maxd < 1 or (ns == 1 and maxd == 1):
        return False
    return n_nodes <= (1 << 24 if maxd >= 8 else 1 << 23 if maxd >= 5 else 1 << 19)


def reference_frame_check(config: str, frame, host=None):
    """SHA-256 of the bench's assembled static frame (float32 RGB, GL rows) against the frame the
    reference's own shaders give for the same scene and camera -- run on Mesa llvmpipe with the
    canonical builtins and pixel centre, tests/golden/glsl/canonical.json (tests/test_glsl_parity.py).  None when
    no such hash exists for the config (C5: its tree is too large for llvmpipe) or no frame."""
    cases = {"c1": "c1", "c2": "c2_full", "c3": "c3_full", "ref_default": "config_default", "ref_stats114": "stats114"}
    path = Path(__file__).resolve().parent / "tests" / "golden" / "glsl" / "canonical.json"
    if (frame is None and host is None) or config not in cases or not path.exists():
        return None
    ref = json.loads(path.read_text())["cases"][cases[config]]
    W, H, N, D, M, NS, MD = CONFIGS[config]
    assert (ref["W"], ref["H"], ref["n"], ref["depth"], ref["m"], ref["spp"], ref["md"]) == (W, H, N, D, M, NS, MD)
    img = host if host is not None else (frame.cpu().numpy() if hasattr(frame, "cpu") else np.asarray(frame))
    got = hashlib.sha256(np.ascontiguousarray(img, np.float32).tobytes()).hexdigest()
    return {"frame_sha256": got, "reference_shader_frame_sha256": ref["sha256"], "bit_identical": got == ref["sha256"],
            "reference": "the reference's shaders/octree_fragment_shader.glsl on Mesa llvmpipe with canonical "
                         "builtins and pixel centre, same scene and camera (tests/golden/glsl/canonical.json, "
                         "case %s)" % cases[config]}


def default_inflight(config: str, world: int) -> int:
    """Frames in flight by default: 2 when a GPU's share of a frame is at most 40 M pixel-bounces,
    where the longest walks' drain at the end of every launch would otherwise idle much of the
    GPU (a second frame's launches fill it); 1 for larger shares, where two frames' working
    sets only compete for the caches.  Measured (tools/host_overhead.py, rank 0's band tile,
    profiles/r03_host_overhead_d.log; bench.py N=1): C3 full frame 1.753 -> 1.672 ms/frame,
    C3 1/2, 1/4, 1/8 bands 0.944 -> 0.843, 0.660 -> 0.433, 0.481 -> 0.251; C5 1/4, 1/8 bands
    11.91 -> 11.57, 7.18 -> 6.09; but C5 full frame 42.26 -> 46.30 and C5 1/2 band 21.78 ->
    22.93 ms/frame."""
    W, H, _, _, _, NS, MAXD = CONFIGS[config]
    share = W * H / max(1, world) * max(1, NS) * max(1, MAXD)
    if share > 40e6:
        return 1
    # a 1/4 or 1/8 band: a third frame fills more of each frame's tail (C3 1/8 0.252 -> 0.231,
    # 1/4 0.433 -> 0.426 ms/frame, C5 1/8 6.09 -> 5.83; a fourth was slower; at N = 1 and 2 a
    # third changes nothing: profiles/r03_host_overhead_e.log, _f.log)
    return 3 if world >= 4 else 2


BASELINE_METRIC = "Mrays/sec at 3840x2160, 100k spheres, depth 8; 1/2/4/8-GPU scaling"
HBM_PEAK_GBS = 8000.0       # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SIMDS = 1024                # 256 CUs x 4 SIMDs
CLOCK_GHZ = 2.4             # max engine clock (MI355X_MICROARCH.md)
VALU_CYCLES_PER_INST = 2    # a wave64 VALU instruction issues over 2 cycles (MI355X_MICROARCH.md)
VALU_PEAK_GINST = SIMDS * CLOCK_GHZ / VALU_CYCLES_PER_INST  # 1228.8 G wave-instructions/s


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # untimed warm-up frames: a C3 frame keeps getting faster over the first ~15 frames of a
    # process (the clocks ramping up, profiles/r05_c3_warm3.md): 20 by default measures the steady
    # state (C3 +2.3 % over 5: profiles/r05_warmup_c3.log); 20 C5 frames take ~0.8 s
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--seed", type=int, default=42)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0 = the CPUs this job may use: its cgroup CPU quota when it has "
                    "one, else every CPU of os.sched_getaffinity)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-build", action="store_true", help="build the octree on the host and upload it "
                    "(default: ort_build_scene, the GPU builder)")
    ap.add_argument("--pmc-json", default="",
                    help="PMC record of the trace kernels (default profiles/pmc_<config>.json, written by "
                    "tools/summarize_profile.py)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="frames in flight, each on its own context and stream (0 = auto, default_inflight: 2 "
                    "when a GPU's share of the frame is small enough that its walks' tail would idle it)")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="testing only: every rank on GPU 0 with the gloo backend (exercises the N>1 code "
                    "path on a one-GPU box; not a measurement)")
    ap.add_argument("--emulate", action="store_true",
                    help="testing only, no GPU: every rank renders its tile with the host build of the kernel's "
                    "per-pixel code and the bands are gathered with gloo (exercises the launcher, partition and "
                    "gather on CPU; never a measurement)")
    ap.add_argument("--moving-steps", type=int, default=20,
                    help="also time this many frames with the camera turning --yaw-step degrees per frame (reported "
                    "as moving_camera, after the main timed region; 0 = skip)")
    ap.add_argument("--yaw-step", type=float, default=0.5, help="moving_camera: degrees of yaw per frame")
    ap.add_argument("--moving-control", type=int, default=4,
                    help="moving_camera: also render this many poses of the turn statically (the main loop's way, "
                    "after warm-up frames of the pose: exact hints), reported as static_same_poses (0 = skip)")
    ap.add_argument("--control-steps", type=int, default=8, help="static_same_poses: timed frames per pose")
    ap.add_argument("--single-steps", type=int, default=10,
                    help="N > 1 with frames in flight: also time this many frames with one frame in flight "
                    "(reported as single_frame, after the main timed region; 0 = skip)")
    ap.add_argument("--opt", "--group-opt", dest="group_opt", action="append", default=[], metavar="NAME=VALUE",
                    help="ort_set_option(ORT_OPT_<NAME>, VALUE) on every context, after bench.py's own settings "
                    "(A/B; recorded in the line's config)")
    ap.add_argument("--group", action="store_true",
                    help="one process drives all N GPUs through the C-ABI group (ort_group_*: a context per device, "
                    "RCCL ncclSend/ncclRecv gather over xGMI); with --rehearse-one-gpu every rank is GPU 0 and the "
                    "gather uses device copies")
    ap.add_argument("--gather-timeout", type=float, default=120.0,
                    help="seconds any wait on a frame's gather may take before the run exits non-zero naming the "
                    "rank and the frame slot (process group timeout; gloo: each gather; --group: every frame wait)")
    ap.add_argument("--save", default="", help="rank 0: save the assembled frame (.pfm/.png)")
    return ap.parse_args(argv)


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def self_launch(args) -> int:
    """`bench.py --gpus N` without a launcher: start N ranks with torch.distributed.run as a
    CHILD process (nothing here has touched a GPU) and pass its output and exit code on."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", str(Path(__file__).resolve())] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def metric_name(cfg: str) -> str:
    W, H, NSPH, DEPTH, MPN, NS, MAXD = CONFIGS[cfg]
    if cfg == "c3":
        return BASELINE_METRIC
    sph = f"{NSPH // 1_000_000}M" if NSPH % 1_000_000 == 0 else (f"{NSPH // 1000}k" if NSPH >= 1000 else str(NSPH))
    extra = f", bounce depth {MAXD}" if MAXD > 1 else ""
    return f"Mrays/sec at {W}x{H}, {sph} spheres, depth {DEPTH}{extra}; 1/2/4/8-GPU scaling"


def cpu_info() -> dict:
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count() or 1
    quota = None
    try:  # cgroup v2 CPU quota, if any
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    return {"model": model, "nproc": os.cpu_count() or 1, "affinity": aff, "cgroup_cpu_quota": quota}


def lib_sha() -> str:
    p = ROOT / "octreeraytracer_amd" / "lib" / "libort.so"
    return hashlib.sha256(p.read_bytes()).hexdigest()[:16] if p.exists() else ""


def _elf_sections(b: bytes) -> dict:
    """{name: bytes} of an ELF64 image (SHT_NOBITS sections empty)."""
    import struct
    shoff = struct.unpack_from("<Q", b, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", b, 0x3A)
    hdr = [struct.unpack_from("<IIQQQQIIQQ", b, shoff + i * shentsize) for i in range(shnum)]
    names = hdr[shstrndx][4]
    out = {}
    for h in hdr:
        name = b[names + h[0]:b.index(b"\0", names + h[0])].decode()
        out[name] = b"" if h[1] == 8 else b[h[4]:h[4] + h[5]]
    return out


def gfx950_code_objects(b: bytes) -> list:
    """The gfx950 code objects of a host ELF's .hip_fatbin: one clang offload bundle per HIP
    translation unit, in link order."""
    import struct
    sec = _elf_sections(b).get(".hip_fatbin", b"")
    out, i = [], 0
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    while (j := sec.find(magic, i)) >= 0:
        n = struct.unpack_from("<Q", sec, j + len(magic))[0]
        q = j + len(magic) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", sec, q)
            triple = sec[q + 24:q + 24 + tl]
            q += 24 + tl
            if triple.endswith(b"gfx950"):
                out.append(sec[j + off:j + off + size])
        i = j + len(magic)
    return out


def device_sha(path=None) -> str:
    """SHA-256 (16 hex) of the device code of libort.so: per gfx950 code object (link order) its
    .text (the instructions) and .rodata (the kernel descriptors: registers, LDS, scratch).  A
    PMC record therefore stays valid across host-only rebuilds and rebuilds in another directory
    (the compilation-unit id, derived from the source path, only reaches the code objects'
    symbol strings), and goes stale with any kernel change."""
    p = Path(path) if path else ROOT / "octreeraytracer_amd" / "lib" / "libort.so"
    if not p.exists():
        return ""
    h = hashlib.sha256()
    cos = gfx950_code_objects(p.read_bytes())
    for co in cos:
        sec = _elf_sections(co)
        for name in (".text", ".rodata"):
            h.update(name.encode() + len(sec.get(name, b"")).to_bytes(8, "little") + sec.get(name, b""))
    return h.hexdigest()[:16] if cos else ""


def load_pmc(args, tile_rows) -> dict | None:
    path = Path(args.pmc_json) if args.pmc_json else ROOT / "profiles" / f"pmc_{args.config}.json"
    if not path.exists():
        return None
    try:
        rec = json.loads(path.read_text())
    except (OSError, ValueError):
        return None
    if rec.get("config") != args.config:
        return None
    rec["_path"] = str(path.relative_to(ROOT)) if path.is_relative_to(ROOT) else str(path)
    return rec


def roofline(pmc, counts, full_traversals, alg_bytes, trace_ms_avg, kernels_ran):
    """The trace kernels of one frame against the VALU issue roof (see the module docstring)."""
    t = trace_ms_avg * 1e-3
    r = {"bound": "valu", "achieved": None, "peak": round(VALU_PEAK_GINST, 1), "unit": "Gwave-inst/s (VALU issue)",
         "frac": None, "traffic": None, "kernels": kernels_ran, "trace_ms_per_frame": round(trace_ms_avg, 4)}
    r["ref_layout_equiv_GBs"] = round(alg_bytes / t / 1e9, 1)
    r["algorithmic_bytes_per_frame"] = int(alg_bytes)
    r["ref_layout_bytes_per_ray"] = round(alg_bytes / max(1, counts["traversals"]), 1)
    r["counts"] = counts
    if pmc is None:
        r["note"] = "no PMC record for this config (profiles/pmc_<config>.json): issue rate unmeasured"
        return r
    tr = pmc["trace"]
    # the record must come from the kernels that ran: its device-code hash (or, for records
    # without one, the whole library's) against this build's
    if pmc.get("device_sha"):
        r["pmc_device_sha"] = pmc["device_sha"]
        r["pmc_matches_build"] = pmc["device_sha"] == device_sha()
    else:
        r["pmc_build_sha"] = pmc.get("lib_sha", "")
        r["pmc_matches_build"] = pmc.get("lib_sha", "") == lib_sha()
    r["pmc_source"] = pmc["_path"]
    if not r["pmc_matches_build"]:
        r["note"] = ("the PMC record was taken with other kernels (device code hash differs): issue rate not "
                     "reported; re-run tools/profile_box.sh + tools/summarize_profile.py for this build")
        return r
    # per-rank share of the full-frame counters (N > 1: the rank's traversals / the frame's)
    share = counts["traversals"] / max(1, full_traversals) if full_traversals else 1.0
    insts = tr["valu_insts_per_frame"] * share
    achieved = insts / t / 1e9
    r["achieved"] = round(achieved, 1)
    r["frac"] = round(achieved / VALU_PEAK_GINST, 4)
    r["valu_lane_utilization"] = round(tr["valu_lane_utilization"], 4)
    r["useful_lane_frac"] = round(r["frac"] * tr["valu_lane_utilization"], 4)
    r["valu_insts_per_wave"] = round(tr["valu_insts_per_wave"], 1)
    r["salu_insts_per_wave"] = round(tr["salu_insts_per_wave"], 1)
    if tr.get("hbm_bytes_per_frame") is not None:
        traffic = tr["hbm_bytes_per_frame"] * share
        r["traffic"] = int(traffic)
        r["hbm_GBs"] = round(traffic / t / 1e9, 1)
        r["hbm_frac"] = round(traffic / t / 1e9 / HBM_PEAK_GBS, 5)
    r["pmc_trace_ms_per_frame"] = round(tr["trace_ms_per_frame"], 4)
    # the same VALU over the profile run's own trace time (its kernel-trace summary's timed window,
    # profiles/<name>.md): reproducible from profiles/ alone; frac above uses this run's live time
    if tr.get("trace_ms_per_frame"):
        r["frac_at_profile_trace_time"] = round(insts / (tr["trace_ms_per_frame"] * share * 1e-3) / 1e9
                                                / VALU_PEAK_GINST, 4)
    if share != 1.0:
        r["pmc_scaled_by_traversal_share"] = round(share, 5)
    return r


def main():
    from octreeraytracer_amd.distributed import GatherTimeout
    try:
        return _main()
    except GatherTimeout as e:  # exits non-zero naming the rank and the pending slot
        print(f"bench.py: {e}", file=sys.stderr, flush=True)
        sys.exit(3)


def _main():
    args = parse()
    W, H, NSPH, DEPTH, MPN, NS, MAXD = CONFIGS[args.config]
    if args.group:
        return group_bench(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(self_launch(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.emulate:
        return emulate(args, world, rank)
    local = 0 if args.rehearse_one_gpu else int(os.environ.get("LOCAL_RANK", "0"))
    inflight = args.inflight or default_inflight(args.config, world)
    if inflight > 1:
        # frames in flight only overlap when their streams sit on different hardware queues;
        # with HIP's default 4 queues per process, RCCL's and torch's streams share them
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, 4 * inflight)))

    import torch
    import torch.distributed as dist

    import octreeraytracer_amd as ort

    torch.cuda.set_device(local)
    from datetime import timedelta
    pg_timeout = timedelta(seconds=args.gather_timeout)  # bounds every collective (RCCL: the watchdog aborts)
    if world > 1:
        if args.rehearse_one_gpu:
            dist.init_process_group("gloo", timeout=pg_timeout)
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=pg_timeout)

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
    if inflight > 1:
        # frames in flight fill each frame's tail themselves: split walks of the heaviest camera
        # rays (ORT_OPT_SPLIT_HEAVY, on by default for tiles <= 2^21 px) only add launches then --
        # C3 1/8 band at 3 in flight 0.266 -> 0.227 ms/frame without them, 1/4 band 0.458 -> 0.423
        # (profiles/r04_host_overhead_inflight_o.log); the single-frame phase below turns them on
        for x in rs:
            x.set_split_heavy(0)

    from octreeraytracer_amd import _lib as L
    for o in args.group_opt:  # A/B options, after the settings above
        name, val = o.split("=")
        for x in rs:
            x._check(x._lib.ort_set_option(x._ctx, getattr(L, "ORT_OPT_" + name.upper()), int(val)))

    # partition: 16-row bands dealt round-robin; every rank renders the same number of rows
    from octreeraytracer_amd.distributed import FrameGather, rank_tile
    tile = rank_tile(W, H, rank, world)
    # inflight+1 band tiles per rank: frame k's gather/assembly overlaps the next frames'
    # renders, and frame k+1 (next context, next stream) fills the tail of frame k
    nslot = inflight + 1
    outs = [torch.empty((tile.rows, W, 3), dtype=torch.float32, device="cuda") for _ in range(nslot)]
    # gloo: each gather's wait bounded on the host; nccl: a wait with a bound would block the host
    # every frame, so the process group's timeout (above) bounds a stalled gather instead
    gather = FrameGather(dist, W, H, world, rank, "cuda", depth=nslot,
                         timeout_s=args.gather_timeout if args.rehearse_one_gpu and world > 1 else None)
    # each context's own stream (never the HIP null stream, handle 0, which the C ABI reads
    # as "no stream" and renders synchronously)
    streams = [torch.cuda.ExternalStream(x.stream_handle()) for x in rs]
    gstream = torch.cuda.Stream()
    torch.cuda.set_stream(streams[0])

    pending = []

    def drain(keep):
        # finish() (RCCL wait + rank-0 assembly into the one frame buffer) on its own stream,
        # so assemblies never overlap each other and never queue behind a render
        frame = None
        with torch.cuda.stream(gstream):
            while len(pending) > keep:
                handle, fin = pending.pop(0)
                frame = gather.finish(handle)
                if fin is not None:
                    fin.record(gstream)  # the frame is assembled (rank 0) / its tile sent
        return frame

    def step(k, ev=None, params=None):
        slot, j = k % nslot, k % inflight
        st = streams[j]
        drain(nslot - 1)  # the previous use of this slot's tile has been gathered
        if world > 1:
            st.wait_stream(gstream)  # ... as far as this frame's stream knows
        torch.cuda.set_stream(st)  # frame k's gather (submit) waits on this stream
        if ev is not None:
            ev[0].record(st)
        rs[j].render(params or p, tile, out=outs[slot], stream=st.cuda_stream)
        if ev is not None:
            ev[1].record(st)
            if world == 1:  # no gather: the frame is complete when its render is
                ev[2].record(st)
        pending.append((gather.submit(outs[slot], slot), ev[2] if ev is not None and world > 1 else None))

    for k in range(args.warmup):
        step(k)
    drain(0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(k, evs[k])
    frame = drain(0)  # every frame gathered and assembled inside the timed region
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # the static camera's frame (the later phases reuse the frame buffer)
    saved = frame.cpu().numpy() if (args.save and rank == 0 and frame is not None) else None
    # the assembled static frame, kept on the device for the check against the reference's own
    # shaders at the end (hashing it here would pause the host long enough for the clocks to drop
    # before the single-frame phase)
    parity_frame = frame.clone() if (rank == 0 and frame is not None and args.config in ("c1", "c2", "c3", "ref_default", "ref_stats114")) else None
    kern_ms = [a.elapsed_time(b) for a, b, _ in evs]       # whole per-frame pipeline (trace+shade+sort)
    latency_ms = [a.elapsed_time(c) for a, _, c in evs]    # render start -> frame gathered and assembled
    nframes0 = min(-(-args.steps // inflight), 64)          # context 0's timed frames
    first_trace_ms = r.trace_times_ms(nframes0)             # bounce-0 trace kernel of each frame
    ftrace = r.frame_trace_times_ms(nframes0)               # every trace kernel of each frame, summed
    trace_ms = [m for m, _ in ftrace]
    launches = sorted({n for _, n in ftrace})
    t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    # with frames in flight: also time one frame in flight, so that lines of different frame
    # counts can be compared at equal settings; per frame render + gather + assembly, the next
    # frame's render queued behind them on the GPU (no host wait; after the main timed region,
    # not part of `value`)
    single = None
    trace_ms_in_flight = None
    if inflight > 1 and args.single_steps > 0:
        rs[0].set_split_heavy(-1)  # one frame in flight: the default (split walks on small tiles)
        sev = [tuple(torch.cuda.Event(enable_timing=True) for _ in range(3)) for _ in range(args.single_steps)]
        # untimed warm-up frames of this setting: the first split frame of a context creates its
        # second stream and allocates the heavy-ray lists (hipMalloc: synchronous, milliseconds),
        # the second is the first with a queued heavy list -- at 10 timed frames the first one's
        # setup alone had put a C2 frame at 0.85 ms for a 0.27 ms trace kernel (round 5)
        for _ in range(3):
            st = streams[0]
            if world > 1:
                st.wait_stream(gstream)
            torch.cuda.set_stream(st)
            rs[0].render(p, tile, out=outs[0], stream=st.cuda_stream)
            pending.append((gather.submit(outs[0], 0), None))
            drain(0)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for k in range(args.single_steps):
            st = streams[0]
            if world > 1:
                st.wait_stream(gstream)
            torch.cuda.set_stream(st)
            sev[k][0].record(st)
            rs[0].render(p, tile, out=outs[0], stream=st.cuda_stream)
            sev[k][1].record(st)
            if world == 1:
                sev[k][2].record(st)  # no gather: the frame is complete when its render is
            pending.append((gather.submit(outs[0], 0), sev[k][2] if world > 1 else None))
            drain(0)  # the next render waits (on the GPU) for this frame's gather and assembly
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_single = torch.tensor([time.perf_counter() - t1], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t_single, op=dist.ReduceOp.MAX)
        single = (float(t_single.item()), [a.elapsed_time(c) for a, _, c in sev])
        # the trace kernels of these frames ran alone on the GPU: the roofline's kernel times
        # (with frames in flight, two frames' kernels overlap and each launch lasts longer)
        n_single = min(args.single_steps, 64)
        first_trace_ms = r.trace_times_ms(n_single)
        ftrace_iso = r.frame_trace_times_ms(n_single)
        trace_ms_in_flight, trace_ms = trace_ms, [m for m, _ in ftrace_iso]
        rs[0].set_split_heavy(0)  # back to the pipelined setting of every context (main loop)

    # the split-walk setting every context runs the moving-camera phase with: the main loop's
    split_moving = 0 if inflight > 1 else -1

    # moving camera: the cost order and heavy-first lists deal work by the previous frame's walk
    # steps, which a static camera makes exact; an interactive caller turns the camera
    # (src/main.cpp:120-163).  The same pipeline, the camera turning yaw_step degrees per frame
    # from the static pose, so every frame's hints are stale (by frames_in_flight frames: each
    # context renders every frames_in_flight-th frame; after the main timed
    # region, not part of `value`)
    moving = None
    if args.moving_steps > 0:
        from octreeraytracer_amd.scene import DEFAULT_YAW
        poses = [ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MAXD,
                                                yaw=DEFAULT_YAW + args.yaw_step * (k + 1))
                 for k in range(args.moving_steps)]
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        for k in range(args.moving_steps):
            step(args.warmup + args.steps + k, params=poses[k])
        drain(0)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t_mov = torch.tensor([time.perf_counter() - t2], dtype=torch.float64, device="cuda")
        if world > 1:
            dist.all_reduce(t_mov, op=dist.ReduceOp.MAX)
        # traced rays of those frames: W*H*spp per frame for primary rays, else counted per pose
        # (the counting kernels, untimed)
        if NS * MAXD == 1:
            mov_rays = None
        else:
            mov_rays = torch.tensor([sum(r.count_traffic(q, tile)["traversals"] for q in poses)],
                                    dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(mov_rays)
        moving = (float(t_mov.item()), None if mov_rays is None else float(mov_rays.item()))
        # the control: poses of the turn rendered statically, each the way the main loop renders
        # (frames in flight, a warm-up frame of the pose first: exact hints) -- moving / control
        # isolates what stale hints cost from what the turned view itself costs (other
        # geometry in view)
        ctrl = None
        if args.moving_control > 0:
            sel = sorted({round(i * (args.moving_steps - 1) / max(1, args.moving_control - 1))
                          for i in range(args.moving_control)})
            ctrl_t, ctrl_rays, kk = 0.0, 0.0, args.warmup + args.steps + args.moving_steps
            for i in sel:
                for _ in range(2):  # warm-up frames of the pose (the cost hints become exact)
                    step(kk, params=poses[i])
                    kk += 1
                drain(0)
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                t3 = time.perf_counter()
                for _ in range(args.control_steps):
                    step(kk, params=poses[i])
                    kk += 1
                drain(0)
                torch.cuda.synchronize()
                if world > 1:
                    dist.barrier()
                torch.cuda.synchronize()
                ctrl_t += time.perf_counter() - t3
                if NS * MAXD != 1:
                    ctrl_rays += args.control_steps * r.count_traffic(poses[i], tile)["traversals"]
            tc = torch.tensor([ctrl_t, ctrl_rays], dtype=torch.float64, device="cuda")
            if world > 1:
                dist.all_reduce(tc[:1], op=dist.ReduceOp.MAX)
                dist.all_reduce(tc[1:])
            ctrl = (float(tc[0].item()), float(tc[1].item()) if NS * MAXD != 1 else None, len(sel))
        moving = moving + (ctrl,)

    # algorithmic traffic of this rank's launch (counting variant, untimed); the traced rays
    # of a step = traversals summed over the ranks (W*H*spp for primary-only configs)
    counts = r.count_traffic(p, tile)
    alg_bytes = ort.algorithmic_bytes(counts)
    trav = torch.tensor([counts["traversals"]], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(trav)
    rays_per_frame = int(trav.item())

    result = None
    if rank == 0:
        ms_per_step = elapsed / args.steps * 1e3
        value = rays_per_frame * args.steps / elapsed / 1e6
        pmc = load_pmc(args, tile.rows)
        kernels = trace_kernel_names(args.config, info, MAXD, NS, tile.rows * W)
        result = {
            "metric": metric_name(args.config),
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
                "layout": info["layout"], "options": args.group_opt or None,
                "partition": "16-row bands round-robin + RCCL gather (async, "
                "overlapping the next frame's render)" if world > 1
                else "full frame", "frames_in_flight": inflight, "rays_per_step": rays_per_frame, "rays": "traced rays (octree traversals), "
                "all bounces and ranks",
            },
            "frame_gpu_ms_avg": round(float(np.mean(kern_ms)), 4),
            # per frame on rank 0: its render's start to the assembled frame (gather included);
            # with frames in flight a frame's latency exceeds ms_per_step (its share of throughput)
            "frame_latency_ms_avg": round(float(np.mean(latency_ms)), 4),
            "frame_latency_ms_max": round(float(np.max(latency_ms)), 4),
            "single_frame": None if single is None else {
                "frames_in_flight": 1, "steps": args.single_steps,
                "value": round(rays_per_frame * args.single_steps / single[0] / 1e6, 2),
                "ms_per_step": round(single[0] / args.single_steps * 1e3, 4),
                "frame_latency_ms_avg": round(float(np.mean(single[1])), 4),
                "note": "one frame in flight (render, gather, assembly, then the next); `value` above keeps "
                        "frames_in_flight frames in flight"},
            "moving_camera": None if moving is None else {
                "value": round((moving[1] if moving[1] is not None else rays_per_frame * args.moving_steps)
                               / moving[0] / 1e6, 2),
                "yaw_step_deg": args.yaw_step, "steps": args.moving_steps,
                "ms_per_step": round(moving[0] / args.moving_steps * 1e3, 4),
                "frames_in_flight": inflight, "split_heavy": split_moving,
                "static_same_poses": None if not moving[2] else {
                    "value": round((moving[2][1] if moving[2][1] is not None
                                    else rays_per_frame * args.control_steps * moving[2][2]) / moving[2][0] / 1e6, 2),
                    "poses": moving[2][2], "steps_per_pose": args.control_steps,
                    "ms_per_step": round(moving[2][0] / (args.control_steps * moving[2][2]) * 1e3, 4),
                    "note": "poses of the turn, each rendered statically like the main loop (frames in flight, "
                            "after warm-up frames of the pose: exact hints); moving value / this = the price of "
                            "stale hints alone"},
                "note": "the camera turns yaw_step_deg per frame (the interactive case): the per-slot walk-cost "
                        "hints that order work are frames_in_flight frames stale (each context renders every "
                        "frames_in_flight-th frame); `value` above is the static camera of the "
                        "reference's saveStats runs"},
            "trace_kernels_ms_avg": round(float(np.mean(trace_ms)), 4),
            # with frames in flight: trace_kernels_ms_avg and the first-trace figures are taken over
            # the one-frame-in-flight phase (kernels alone on the GPU); this is the main loop's
            "trace_kernels_ms_avg_in_flight": None if trace_ms_in_flight is None
            else round(float(np.mean(trace_ms_in_flight)), 4),
            "trace_launches_per_frame": launches,
            "first_trace_kernel_ms_avg": round(float(np.mean(first_trace_ms)), 4),
            "first_trace_kernel_ms_min": round(float(np.min(first_trace_ms)), 4),
            "roofline": roofline(pmc, counts, (pmc or {}).get("traversals_per_frame"), alg_bytes,
                                 float(np.mean(trace_ms)), kernels),
            "setup": setup,
            "parity": reference_frame_check(args.config, parity_frame, saved),
            "build_sha": lib_sha(),
            "device_sha": device_sha(),
        }
        if world == 1 and not args.no_cpu_baseline:
            if tree is None:
                t0 = time.time()
                tree = ort.build_octree(spheres, DEPTH, MPN)  # the oracle walks the host tree
                setup["host_octree_build_s"] = round(time.time() - t0, 3)
            result["cpu_baseline"] = cpu_baseline(spheres, tree, p, args.cpu_seconds, args.cpu_threads)
        if args.save:
            img = saved
            from octreeraytracer_amd import image
            (image.write_png if args.save.endswith(".png") else image.write_pfm)(args.save, img)
    for x in rs:
        x.close()
    if world > 1:
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps(result), flush=True)


def group_bench(args):
    import octreeraytracer_amd as ort
    try:
        return _group_bench(args)
    except ort.OrtError as e:
        if e.code == ort.ORT_ERR_TIMEOUT:  # the message names the frame, its slot and the pending ranks
            print(f"bench.py --group: {e}", file=sys.stderr, flush=True)
            sys.exit(3)
        raise


def _group_bench(args):
    """--group: ONE process drives N GPUs through the C-ABI group (include/ort.h ort_group_*),
    the path a caller of Raytracer::render() uses: a context per device per frame slot, the
    same 16-row band partition, the bands gathered to devices[0] by RCCL ncclSend/ncclRecv
    (grouped) and de-interleaved there -- inside the timed region.  With --rehearse-one-gpu
    every rank is GPU 0 and the gather uses device copies (a control-path check on a one-GPU
    box, not a scaling measurement).  The line carries a frame check: the last frame against
    a single-context ort_render of the same scene, bit for bit."""
    W, H, NSPH, DEPTH, MPN, NS, MAXD = CONFIGS[args.config]
    N = args.gpus
    # frame slots: the RCCL transport with several slots (their communicators' gathers running
    # concurrently) has not run between distinct devices yet, so it is opt-in (--inflight);
    # the copy-transport rehearsal takes the per-config default
    inflight = args.inflight or (default_inflight(args.config, N) if args.rehearse_one_gpu or N == 1 else 1)
    if inflight > 1:  # as main(): frame slots overlap only on distinct hardware queues -- one per
        # stream: every rank's render stream on its device (all of them on GPU 0 in the rehearsal)
        # plus devices[0]'s gather stream, per frame slot (a shared queue serialises a gather
        # behind another slot's render: +10 % single-frame latency in the rehearsal)
        need = inflight * (N + 1) if args.rehearse_one_gpu else 4 * inflight
        os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, max(8, need)))
    import torch

    import octreeraytracer_amd as ort
    from octreeraytracer_amd.group import TRANSPORT_COPY, TRANSPORT_RCCL, RenderGroup
    devices = [0] * N if args.rehearse_one_gpu else list(range(N))
    transport = TRANSPORT_COPY if args.rehearse_one_gpu else TRANSPORT_RCCL
    spheres = ort.random_spheres(NSPH, args.seed)
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MAXD)
    g = RenderGroup(devices, transport, inflight=inflight)
    g.set_timeout(int(args.gather_timeout * 1000))  # a stalled frame: OrtError(ORT_ERR_TIMEOUT) names slot + ranks
    from octreeraytracer_amd import _lib as L
    for o in args.group_opt:
        name, val = o.split("=")
        g.set_option(getattr(L, "ORT_OPT_" + name.upper()), int(val))
    t0 = time.time()
    g.build_scene(spheres, DEPTH, MPN)
    setup = {"group_build_scene_wall_s": round(time.time() - t0, 3)}
    dev0 = torch.device("cuda", devices[0])
    nslot = inflight + 1  # frame k writes outs[k % nslot]; submit(k) has waited for frame k - inflight
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device=dev0) for _ in range(nslot)]

    def sync_all():
        for d in sorted(set(devices)):
            torch.cuda.synchronize(d)

    tickets = [g.submit(p, outs[k % nslot]) for k in range(args.warmup)]
    for tk in tickets:
        g.wait(tk)
    sync_all()
    t0 = time.perf_counter()
    tickets = [g.submit(p, outs[k % nslot]) for k in range(args.steps)]
    for tk in tickets:
        g.wait(tk)
    sync_all()
    elapsed = time.perf_counter() - t0
    latency = g.last_frame_ms()  # the last frame: submission on devices[0] -> assembled
    last = outs[(args.steps - 1) % nslot]
    frame = last.cpu().numpy()
    # single-frame phase: one frame in flight at a time (render() = submit + wait), latency
    single = []
    for _ in range(max(3, min(args.steps, 10))):
        t1 = time.perf_counter()
        g.render(p, out=outs[0])
        single.append((time.perf_counter() - t1) * 1e3)
    single_lat = g.last_frame_ms()
    counts = [g.count_traffic(p, r) for r in range(N)]
    rays_per_frame = sum(c["traversals"] for c in counts)
    nframes0 = min(-(-args.steps // inflight), 64)
    ftrace = g.frame_trace_times_ms(0, nframes0)
    trace_ms = [m for m, _ in ftrace]
    info = None
    with ort.Renderer(devices[0]) as ref:  # the frame check: one context, the whole frame
        ref.build_scene(spheres, DEPTH, MPN)
        info = ref.info()
        want = ref.render(p)
    same = bool(np.array_equal(frame.view(np.uint32), want.view(np.uint32)))
    pmc = load_pmc(args, 0)
    alg_bytes = ort.algorithmic_bytes(counts[0])
    value = rays_per_frame * args.steps / elapsed / 1e6
    result = {
        "metric": metric_name(args.config),
        "value": round(value, 2),
        "unit": "Mrays/s",
        "n_gpus": N,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
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
            "layout": info["layout"], "driver": "C-ABI group (ort_group_submit/ort_group_wait), one process",
            "devices": devices,
            "partition": "16-row bands round-robin + " + ("device-copy gather (rehearsal on one GPU: NOT a "
                                                          "scaling measurement)" if args.rehearse_one_gpu
                                                          else "RCCL ncclSend/ncclRecv gather to devices[0]"),
            "frames_in_flight": inflight, "rays_per_step": rays_per_frame,
            "rays": "traced rays (octree traversals), all bounces and ranks",
        },
        "frame_latency_ms": round(latency, 4),
        "single_frame": {"frames_in_flight": 1, "ms_per_frame_wall": round(float(np.median(single)), 4),
                         "value": round(rays_per_frame / float(np.median(single)) / 1e3, 2),
                         "frame_latency_ms": round(single_lat, 4)},
        "trace_kernels_ms_avg_rank0": round(float(np.mean(trace_ms)), 4),
        "roofline": roofline(pmc, counts[0], (pmc or {}).get("traversals_per_frame"), alg_bytes,
                             float(np.mean(trace_ms)),
                             trace_kernel_names(args.config, info, MAXD, NS, W * -(-H // (16 * N)) * 16,
                                                split_ok=inflight == 1 and not args.rehearse_one_gpu)),
        "frame_check": ("bit-identical to a single-context ort_render of the same scene" if same
                        else "MISMATCH against a single-context ort_render"),
        "parity": reference_frame_check(args.config, None, np.asarray(frame)),
        "setup": setup,
        "build_sha": lib_sha(),
        "device_sha": device_sha(),
    }
    g.close()
    print(json.dumps(result), flush=True)
    if not same:
        raise SystemExit("group frame differs from the single-context render")


SPLIT_AUTO_PIXELS = 1 << 21  # ort_kernel.hip kSplitAutoPixels: split walks at or below, tile pairs above


def trace_kernel_names(cfg, info, maxd, ns, pixels, split_ok=True):
    """The trace kernels a frame of this config launches (ort_kernel.hip render_impl, default
    options: tile pairs on tiles above 2^21 pixels, split walks of the heaviest camera rays at or
    below it, 1 sample; split_ok False: the caller turned the split walks off, tile pairs)."""
    deep = info["tree_depth"] > 8
    if pixel_paths_auto(info["n_nodes"], ns, maxd):
        if ns > 4:  # the steady state: samples in parallel (ORT_OPT_PIXEL_SPECULATE: 2+ chunks of 4+), resolve, fixup list
            return ["ort_pixel_paths<0, %s, ..., 1> (whole-pixel paths, every (pixel, sample) in parallel from last "
                    "frame's per-sample RNG end states)" % str(deep).lower(),
                    "ort_sample_resolve (each pixel's samples summed in order; pixels whose states moved listed)",
                    "ort_pixel_paths<0, %s, ..., 2> (the listed pixels' remaining samples from their true state)"
                    % str(deep).lower()]
        return ["ort_pixel_paths<0, %s> (whole-pixel paths: every sample and bounce of the frame in one launch)"
                % str(deep).lower()]
    pairs = pixels > SPLIT_AUTO_PIXELS or not split_ok
    tile = ("ort_trace_pair%s<false, %d> (two tiles per workgroup: camera rays + walk + %s)" if pairs else
            "ort_trace_compact%s<false, true, %d> (camera rays + walk + %s)")
    split = [] if pairs or ns != 1 else ["ort_trace_split<%s, %d> (the heaviest camera rays, 8 lanes each, second "
                                         "stream)" % (str(deep).lower(), 1 if maxd == 1 else 2)]
    if maxd == 1 and ns == 1:
        return [tile % ("_deep" if deep else "", 1, "shading into the frame")] + split
    return [tile % ("_deep" if deep else "", 2, "bounce-0 shading, cost order")] + split + \
        ["ort_trace_persistent<false, %s> (bounces >= 1, sorted alive paths heavy first, lane refill%s)"
         % (str(deep).lower(), ", leaf hold" if deep else "")]


def emulate(args, world, rank):
    """--emulate: the N>1 control path on CPU (gloo), tiles rendered by the host build of the
    kernel's per-pixel code.  Prints a JSON line marked as emulation; never a measurement."""
    import torch
    import torch.distributed as dist

    import octreeraytracer_amd as ort
    from octreeraytracer_amd.distributed import FrameGather, rank_tile
    from octreeraytracer_amd.renderer import emulate_render_host
    W, H, NSPH, DEPTH, MPN, NS, MAXD = CONFIGS[args.config]
    if world > 1:
        dist.init_process_group("gloo")
    spheres = ort.random_spheres(NSPH, args.seed)
    tree = ort.build_octree(spheres, DEPTH, MPN)
    p = ort.FrameParams.default_camera(W, H, num_samples=NS, max_depth=MAXD)
    tile = rank_tile(W, H, rank, world)
    gather = FrameGather(dist, W, H, world, rank, "cpu")
    t0 = time.perf_counter()
    frame = None
    trav = 0
    for _ in range(args.steps):
        local, counts = emulate_render_host(spheres, tree, p, tile)
        trav = counts["traversals"]
        frame = gather(torch.from_numpy(local))
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed, float(trav)], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(t[1:], op=dist.ReduceOp.SUM)
        dist.all_reduce(t[:1], op=dist.ReduceOp.MAX)
    if rank == 0:
        digest = hashlib.sha256(np.ascontiguousarray(frame.numpy()).tobytes()).hexdigest()
        print(json.dumps({"metric": metric_name(args.config), "value": round(float(t[1]) * args.steps / float(t[0]) / 1e6, 4),
                          "unit": "Mrays/s", "n_gpus": world, "steps": args.steps, "warmup": 0,
                          "ms_per_step": round(float(t[0]) / args.steps * 1e3, 3), "higher_is_better": True,
                          "scaling": "strong", "vs_baseline": None, "dtype": "f32",
                          "data": "EMULATION (host build of the kernel code, gloo): a control-path test, not a "
                                  "measurement", "config": {"workload": args.config, "width": W, "height": H},
                          "frame_sha256": digest, "parity": reference_frame_check(args.config, frame)}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def sample_rows(height: int, n: int):
    """A row sample of about n rows spread evenly over the whole frame height, as the oracle's
    band arguments: (y0, rows, band_height, band_stride) -- tile row j is frame row
    y0 + (j // band_height) * band_stride + j % band_height.  Up to half the height: single rows
    every height // n rows.  Beyond: bands of bh rows every bs rows (bs <= 16) with bh / bs
    closest to n / height, across the whole height (an integer stride would collapse to 1 there
    and sample the first n rows only)."""
    n = max(1, min(int(n), height))
    if 2 * n <= height:
        stride = height // n
        return stride // 2, n, 1, stride
    if n == height:
        return 0, height, 1, 1
    best = None
    for bs in range(2, 17):
        for bh in range(1, bs):
            err = abs(bh / bs - n / height)
            if best is None or err < best[0] - 1e-12:
                best = (err, bh, bs)
    _, bh, bs = best
    rows = bh * (height // bs) + min(bh, height % bs)
    return 0, rows, bh, bs


def cpu_baseline(spheres, tree, p, budget_s, threads=0):
    """Oracle on the host cores over a row sample spread evenly over the frame (sample_rows),
    sized to ~budget_s of wall time.  `value` counts traced rays (octree traversals, every
    bounce, from the oracle's own counters) per second, the unit of the GPU line's `value`;
    camera rays per second are reported beside it."""
    from oracle import oracle
    ci = cpu_info()
    # the job's CPU share: a cgroup quota (the GPU box grants 16 CPUs of a 256-thread host) caps
    # throughput, and more threads than the quota only get throttled (measured: 256 threads
    # on a 16-CPU quota ran the oracle 2.3x slower than 16)
    threads = threads or (max(1, int(ci["cgroup_cpu_quota"])) if ci["cgroup_cpu_quota"] else ci["affinity"])

    def run(n, nthreads):
        y0, rows, bh, bs = sample_rows(p.height, n)
        t0 = time.perf_counter()
        _, c = oracle.render(spheres, tree, p, 0, y0, p.width, rows, band_height=bh, band_stride=bs, counts=True,
                             threads=nthreads)
        return time.perf_counter() - t0, rows, (y0, bh, bs), c

    def where(rows, geo):
        y0, bh, bs = geo
        last = y0 + ((rows - 1) // bh) * bs + (rows - 1) % bh
        return (f"{rows} of {p.height} rows (row stride {bs} from row {y0})" if bh == 1 else
                f"{rows} of {p.height} rows ({bh} of every {bs}, rows {y0}..{last})")

    n = 2 * threads
    dt, _, _, _ = run(min(n, p.height), threads)  # calibration sample
    n = int(max(min(n, p.height), min(p.height, n * budget_s / max(dt, 1e-3))))
    dt, rows, geo, c = run(n, threads)
    cam = rows * p.width * p.num_samples
    # one core (report all cores and 1 core), a smaller row sample
    n1 = max(2, min(p.height, int(rows * 0.25 * budget_s / max(dt * threads, 1e-3))))
    dt1, rows1, geo1, c1 = run(n1, 1)
    return {"value": round(c["traversals"] / dt / 1e6, 3), "unit": "Mrays/s (traced rays: octree traversals, every bounce)",
            "cores": threads, "kind": "port",
            "sample": f"{where(rows, geo)}, {c['traversals']} traversals of {cam} camera rays, {dt:.1f} s wall; "
                      f"oracle/ort_oracle.c -O3, OpenMP dynamic over rows, {threads} threads",
            "camera_rays_per_s_M": round(cam / dt / 1e6, 3),
            "cpu_model": ci["model"], "nproc": ci["nproc"], "affinity_cpus": ci["affinity"],
            "cgroup_cpu_quota": ci["cgroup_cpu_quota"],
            "value_1core": round(c1["traversals"] / dt1 / 1e6, 3),
            "sample_1core": f"{where(rows1, geo1)}, {c1['traversals']} traversals, {dt1:.1f} s wall, 1 thread"}


if __name__ == "__main__":
    main()
