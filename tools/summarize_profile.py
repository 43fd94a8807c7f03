"""Summarise a tools/profile_box.sh output directory into profiles/<tag>.json + .md.
usage: python tools/summarize_profile.py gpurun_out/<tag> profiles/<name>"""
import csv
import json
import sys
from collections import defaultdict
from pathlib import Path

src, dst = Path(sys.argv[1]), Path(sys.argv[2])
KERNEL = sys.argv[3] if len(sys.argv) > 3 else "ort_trace_compact<false, true, true>"

stats = {}
ks = next(src.glob("trace/*kernel_stats.csv"), None)
if ks:
    for r in csv.DictReader(open(ks)):
        stats[r["Name"]] = {k: r[k] for k in ("Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}

pmc = defaultdict(list)
for f in src.glob("pmc_*/pmc_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if KERNEL in r["Kernel_Name"]:
            pmc[r["Counter_Name"]].append(float(r["Counter_Value"]))
per_launch = {k: sum(v) / len(v) for k, v in pmc.items()}

res = {"kernel": KERNEL, "kernel_stats": stats, "pmc_per_launch": per_launch}
avg_ns = None
for name, st in stats.items():
    if KERNEL in name:
        avg_ns = float(st["AverageNs"])
res["avg_ns"] = avg_ns
d = {}
if "FETCH_SIZE" in per_launch and "WRITE_SIZE" in per_launch:
    # MI355X_MICROARCH.md HBM: FETCH_SIZE (KB) reads 1/2 of wide streaming reads on gfx950 -> x2
    d["hbm_bytes_per_launch"] = per_launch["FETCH_SIZE"] * 1024 * 2 + per_launch["WRITE_SIZE"] * 1024
    d["fetch_bytes_raw"] = per_launch["FETCH_SIZE"] * 1024
    d["write_bytes"] = per_launch["WRITE_SIZE"] * 1024
    if avg_ns:
        d["hbm_GBs"] = d["hbm_bytes_per_launch"] / avg_ns
if "TCC_HIT_sum" in per_launch:
    h, m = per_launch["TCC_HIT_sum"], per_launch["TCC_MISS_sum"]
    d["l2_hit_rate"] = h / max(1.0, h + m)
if "TCC_EA0_RDREQ_DRAM_sum" in per_launch:
    d["dram_read_frac_of_ea_reads"] = per_launch["TCC_EA0_RDREQ_DRAM_sum"] / max(1.0, per_launch["TCC_EA0_RDREQ_sum"])
if "SQ_THREAD_CYCLES_VALU" in per_launch:
    d["valu_lane_utilization"] = per_launch["SQ_THREAD_CYCLES_VALU"] / max(1.0, 64 * per_launch["SQ_ACTIVE_INST_VALU"])
if "SQ_INSTS_VALU" in per_launch:
    w = per_launch.get("SQ_WAVES", 1.0)
    d["valu_insts_per_wave"] = per_launch["SQ_INSTS_VALU"] / w
    d["lds_insts_per_wave"] = per_launch.get("SQ_INSTS_LDS", 0) / w
    d["vmem_rd_insts_per_wave"] = per_launch.get("SQ_INSTS_VMEM_RD", 0) / w
    d["salu_insts_per_wave"] = per_launch.get("SQ_INSTS_SALU", 0) / w
if "SQ_WAVE_CYCLES" in per_launch and "SQ_WAIT_ANY" in per_launch:
    wc = per_launch["SQ_WAVE_CYCLES"]
    d["wait_any_frac"] = per_launch["SQ_WAIT_ANY"] / wc
    d["wait_inst_frac"] = per_launch["SQ_WAIT_INST_ANY"] / wc
    d["active_inst_frac"] = per_launch["SQ_ACTIVE_INST_ANY"] / wc
if "GRBM_GUI_ACTIVE" in per_launch and avg_ns:
    d["effective_clock_GHz"] = per_launch["GRBM_GUI_ACTIVE"] / 8 / avg_ns
res["derived"] = d
dst.parent.mkdir(parents=True, exist_ok=True)
# traffic record consumed by bench.py (roofline.traffic) for the bench config
if len(sys.argv) > 4 and "hbm_bytes_per_launch" in d:
    cfg, rows = sys.argv[4].split(":")
    (dst.parent / "pmc_traffic.json").write_text(json.dumps({
        "config": cfg, "tile_rows": int(rows), "kernel": KERNEL,
        "hbm_bytes_per_launch": d["hbm_bytes_per_launch"],
        "method": "rocprofv3 separate --pmc passes: FETCH_SIZE*1024*2 (gfx950: FETCH_SIZE reads 1/2 of the "
                  "bytes, MI355X_MICROARCH.md HBM) + WRITE_SIZE*1024, averaged over launches",
        "source": str(src)}, indent=1))
Path(str(dst) + ".json").write_text(json.dumps(res, indent=1))
lines = [f"# rocprofv3 summary: {src.name}", "", "## kernel stats (kernel trace of bench.py)", "",
         "| kernel | calls | avg ns | min ns | max ns | % |", "|---|---|---|---|---|---|"]
for n, st in stats.items():
    lines.append(f"| `{n[:90]}` | {st['Calls']} | {float(st['AverageNs']):.0f} | {st['MinNs']} | {st['MaxNs']} | "
                 f"{float(st['Percentage']):.2f} |")
lines += ["", f"## PMC per launch of `{KERNEL}` (tools/prof_frame.py, separate passes)", "",
          "| counter | value |", "|---|---|"]
lines += [f"| {k} | {v:.6g} |" for k, v in sorted(per_launch.items())]
lines += ["", "## derived", "", "| quantity | value |", "|---|---|"]
lines += [f"| {k} | {v:.6g} |" for k, v in d.items()]
Path(str(dst) + ".md").write_text("\n".join(lines) + "\n")
print("\n".join(lines))
