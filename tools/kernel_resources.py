"""Per-kernel VGPR / spill / occupancy table of ort_kernel.hip from the compiler's
kernel-resource-usage remarks (no GPU needed).
usage: python tools/kernel_resources.py [filter-substring] [-- extra hipcc flags]"""
import re
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
args = sys.argv[1:]
extra = []
if "--" in args:
    i = args.index("--")
    args, extra = args[:i], args[i + 1:]
flt = args[0] if args else ""
cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off", "-fno-fast-math",
       "-fno-slp-vectorize", "-fPIC", "-Wno-unused-parameter", "-c", str(ROOT / "octreeraytracer_amd/csrc/ort_kernel.hip"),
       "-o", "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"] + extra
err = subprocess.run(cmd, capture_output=True, text=True).stderr
rows, cur = [], None
for line in err.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"remark:\s+(VGPRs|AGPRs|SGPRs|VGPRs Spill|SGPRs Spill|Occupancy \[waves/SIMD\]|ScratchSize \[bytes/lane\]):"
                  r" (\d+)", line)
    if m and cur is not None:
        cur[m.group(1)] = int(m.group(2))


def demangle(n):
    try:
        return subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    except OSError:
        return n


print(f"{'kernel':70s} {'VGPR':>5s} {'SGPR':>5s} {'vspill':>6s} {'sspill':>6s} {'occ':>4s}")
for r in rows:
    d = demangle(r["name"]).replace("(anonymous namespace)::", "").split("(")[0]
    if flt and flt not in d:
        continue
    print(f"{d[:70]:70s} {r.get('VGPRs', -1):5d} {r.get('SGPRs', -1):5d} {r.get('VGPRs Spill', 0):6d} "
          f"{r.get('SGPRs Spill', 0):6d} {r.get('Occupancy [waves/SIMD]', -1):4d}")
