"""Summarise a tools/profile_box.sh output directory into profiles/<name>.json + .md and the
PMC record bench.py reads (profiles/pmc_<config>.json).

usage: python tools/summarize_profile.py gpurun_out/<tag> profiles/<name> <config> [--no-record]

Trace kernels = the production (COUNT=false) instances of the walk kernels that
ort_frame_trace_times_ms times: ort_trace_compact[_deep], ort_trace_persistent,
ort_trace_kernel.  Per-frame figures = the sum over a frame's launches."""
import csv
import json
import re
import sys
from collections import defaultdict
from pathlib import Path

args = [a for a in sys.argv[1:] if not a.startswith("--")]
src, dst, cfg = Path(args[0]), Path(args[1]), args[2]
record = "--no-record" not in sys.argv
# the production trace kernels (COUNT false): per-tile camera kernels (one or two tiles per
# workgroup), the persistent bounce kernel, the split walks (no COUNT variant)
TRACE_RE = re.compile(r"ort_trace_((compact_deep|compact|pair_deep|pair|persistent|kernel)<(false|0)|split<)|ort_pixel_paths<|"
                      r"ort_sample_resolve")


def short(name):
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return n.split("(")[0]


def is_trace(name):
    return bool(TRACE_RE.search(short(name)))


meta = json.loads((src / "meta.json").read_text())
bargs = json.loads((src / "bench_args.json").read_text()) if (src / "bench_args.json").exists() else {}
bench_frames = bargs.get("steps", 10) + bargs.get("warmup", 3)

# kernel trace of bench.py: per-kernel stats and per-frame trace-kernel time
stats = {}
ks = next(src.glob("trace/**/*kernel_stats.csv"), None)
if ks:
    for r in csv.DictReader(open(ks)):
        stats[r["Name"]] = {k: r[k] for k in ("Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
trace_ns_total = 0.0
trace_launches = 0
kt = next(src.glob("trace/**/*kernel_trace.csv"), None)
timed_stats = {}  # per kernel over bench.py's timed window only (its warm-up frames left out)
if kt:  # the timed steps only (bench.py's warm-up frames include the cost order's first frame)
    allk = [(float(r["Start_Timestamp"]), float(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(kt))]
    durs = sorted((t0, t1 - t0) for t0, t1, n in allk if is_trace(n))
    warm_b = bargs.get("warmup", 3)
    durs = durs[warm_b * len(durs) // bench_frames:]
    bench_frames -= warm_b
    trace_ns_total = sum(d for _, d in durs)
    trace_launches = len(durs)
    if durs:  # the window: first timed trace launch .. end of the last trace launch
        w0, w1 = durs[0][0], max(t0 + d for t0, d in durs)
        per = defaultdict(list)
        for t0, t1, n in allk:
            if w0 <= t0 and t1 <= w1:
                per[n].append(t1 - t0)
        tot = sum(sum(v) for v in per.values()) or 1.0
        timed_stats = {n: {"Calls": len(v), "AverageNs": sum(v) / len(v), "MinNs": min(v), "MaxNs": max(v),
                           "Percentage": 100.0 * sum(v) / tot} for n, v in per.items()}
else:  # from the stats: production trace kernels' total time
    for n, st in stats.items():
        if is_trace(n):
            trace_ns_total += float(st["AverageNs"]) * int(st["Calls"])
            trace_launches += int(st["Calls"])

# PMC passes over tools/prof_frame.py (meta["frames"] production frames + one counting pass)
# (trace kernels: the first warm_frames frames' launches are left out -- the cost order's first
# frame walks in tile order)
per_kernel = defaultdict(lambda: defaultdict(float))
launches = defaultdict(lambda: defaultdict(int))
frames = meta["frames"]
warm = meta.get("warm_frames", 0)
for f in src.glob("pmc_*/**/pmc_counter_collection.csv"):
    rows = defaultdict(list)  # (kernel, counter) -> values in dispatch order
    for r in sorted(csv.DictReader(open(f)), key=lambda r: int(r.get("Dispatch_Id") or 0)):
        rows[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (n, c), vals in rows.items():
        if is_trace(n) and warm:
            vals = vals[warm * len(vals) // (frames + warm):]
        per_kernel[n][c] += sum(vals)
        launches[n][c] += len(vals)
kernels = {}
for n, cs in per_kernel.items():
    k = {"trace": is_trace(n)}
    for c, v in cs.items():
        k[c + "_per_frame"] = v / frames
    k["launches_per_frame"] = max(launches[n].values()) / frames
    kernels[n] = k


def tsum(counter):
    return sum(k.get(counter + "_per_frame", 0.0) for k in kernels.values() if k["trace"])


trace = {
    "kernels": sorted(n for n, k in kernels.items() if k["trace"]),
    "valu_insts_per_frame": tsum("SQ_INSTS_VALU"),
    "salu_insts_per_frame": tsum("SQ_INSTS_SALU"),
    "waves_per_frame": tsum("SQ_WAVES"),
    "trace_ms_per_frame": trace_ns_total / bench_frames / 1e6 if trace_ns_total else None,
    "trace_launches_per_frame": trace_launches / bench_frames,
}
w = max(1.0, trace["waves_per_frame"])
trace["valu_insts_per_wave"] = trace["valu_insts_per_frame"] / w
trace["salu_insts_per_wave"] = trace["salu_insts_per_frame"] / w
act = tsum("SQ_ACTIVE_INST_VALU")
trace["valu_lane_utilization"] = tsum("SQ_THREAD_CYCLES_VALU") / max(1.0, 64 * act)
if any("FETCH_SIZE_per_frame" in k for k in kernels.values()):
    # MI355X_MICROARCH.md HBM: FETCH_SIZE (KB) reads 1/2 of wide streaming reads on gfx950 -> x2
    trace["hbm_bytes_per_frame"] = tsum("FETCH_SIZE") * 1024 * 2 + tsum("WRITE_SIZE") * 1024
wc = tsum("SQ_WAVE_CYCLES")
if wc:
    trace["wait_any_frac"] = tsum("SQ_WAIT_ANY") / wc
    trace["wait_inst_frac"] = tsum("SQ_WAIT_INST_ANY") / wc
    trace["active_inst_frac"] = tsum("SQ_ACTIVE_INST_ANY") / wc
h, m = tsum("TCC_HIT_sum"), tsum("TCC_MISS_sum")
if h + m:
    trace["l2_hit_rate"] = h / (h + m)
if trace["trace_ms_per_frame"]:
    t = trace["trace_ms_per_frame"] * 1e-3
    peak = 1024 * 2.4e9 / 2  # VALU wave-instruction issue peak (bench.py)
    trace["valu_issue_frac"] = trace["valu_insts_per_frame"] / t / peak
    trace["useful_lane_frac"] = trace["valu_issue_frac"] * trace["valu_lane_utilization"]
    if "hbm_bytes_per_frame" in trace:
        trace["hbm_GBs"] = trace["hbm_bytes_per_frame"] / t / 1e9
        trace["hbm_frac"] = trace["hbm_GBs"] / 8000.0
    g = tsum("GRBM_GUI_ACTIVE")
    if g:
        # GRBM_GUI_ACTIVE: summed over the 8 XCDs (MI355X_MICROARCH.md DVFS); PMC-run clock
        trace["grbm_clock_GHz_vs_trace_time"] = g / 8 / (trace["trace_ms_per_frame"] * 1e6)

res = {"config": cfg, "source": str(src), "lib_sha": meta.get("lib_sha", ""), "device_sha": meta.get("device_sha", ""), "frames_profiled": frames,
       "warm_frames_excluded": warm,
       "bench_frames": bench_frames, "traversals_per_frame": meta["traversals_per_frame"], "tile_rows": meta["tile_rows"],
       "trace": trace, "kernels": kernels, "kernel_stats": stats, "kernel_stats_timed": timed_stats}
dst.parent.mkdir(parents=True, exist_ok=True)
Path(str(dst) + ".json").write_text(json.dumps(res, indent=1))
if record:
    (dst.parent / f"pmc_{cfg}.json").write_text(json.dumps({
        "config": cfg, "tile_rows": meta["tile_rows"], "lib_sha": meta.get("lib_sha", ""), "device_sha": meta.get("device_sha", ""),
        "traversals_per_frame": meta["traversals_per_frame"], "trace": trace,
        "method": "rocprofv3 separate --pmc passes over tools/prof_frame.py (production kernels only), summed over "
                  "each frame's trace-kernel launches; FETCH_SIZE*1024*2 (gfx950: FETCH_SIZE reads 1/2 of the "
                  "bytes, MI355X_MICROARCH.md HBM) + WRITE_SIZE*1024; trace time from the kernel trace of bench.py",
        "summary": str(dst) + ".md"}, indent=1))

lines = [f"# rocprofv3 summary: {src.name} ({cfg})", "",
         f"build {meta.get('lib_sha', '')}; kernel trace of `bench.py --config {cfg}` ({bench_frames} frames) and "
         f"PMC passes of `tools/prof_frame.py` ({frames} frames).", "",
         "## trace kernels per frame (the roofline's kernels)", "", "| quantity | value |", "|---|---|"]
lines += [f"| {k} | {v:.6g} |" if isinstance(v, float) else f"| {k} | {v} |" for k, v in trace.items()]
if timed_stats:
    lines += ["", f"## kernel stats over the timed window ({bench_frames} frames of bench.py, warm-up frames left out)",
              "", "The window the roofline's kernel time comes from: `trace_ms_per_frame` above is the sum of these "
              "trace kernels' averages x launches per frame.", "",
              "| kernel | calls | avg ns | min ns | max ns | % |", "|---|---|---|---|---|---|"]
    for n, st in sorted(timed_stats.items(), key=lambda kv: -kv[1]["Percentage"]):
        lines.append(f"| `{short(n)[:90]}` | {st['Calls']} | {st['AverageNs']:.0f} | {st['MinNs']:.0f} | "
                     f"{st['MaxNs']:.0f} | {st['Percentage']:.2f} |")
lines += ["", "## kernel stats over the whole run (rocprofv3 --stats: warm-up frames, the counting pass included)", "",
          "| kernel | calls | avg ns | min ns | max ns | % |", "|---|---|---|---|---|---|"]
for n, st in sorted(stats.items(), key=lambda kv: -float(kv[1]["Percentage"])):
    lines.append(f"| `{short(n)[:90]}` | {st['Calls']} | {float(st['AverageNs']):.0f} | {st['MinNs']} | {st['MaxNs']} | "
                 f"{float(st['Percentage']):.2f} |")
lines += ["", "## PMC per frame, per kernel (tools/prof_frame.py, separate passes)", ""]
cols = sorted({c for k in kernels.values() for c in k if c.endswith("_per_frame")})
lines += ["| kernel | " + " | ".join(c.replace("_per_frame", "") for c in cols) + " |",
          "|---|" + "---|" * len(cols)]
for n, k in sorted(kernels.items(), key=lambda kv: -kv[1].get("SQ_INSTS_VALU_per_frame", 0)):
    if k.get("SQ_INSTS_VALU_per_frame", 0) < 1e5 and not k["trace"]:
        continue
    lines.append(f"| `{n[:70]}` | " + " | ".join(f"{k.get(c, 0):.4g}" for c in cols) + " |")
Path(str(dst) + ".md").write_text("\n".join(lines) + "\n")
print("\n".join(lines[:40]))
