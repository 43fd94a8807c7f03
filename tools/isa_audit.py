"""ISA audit of a trace kernel's walk loop (analysis only): compiles
ort_kernel.hip for gfx950 to assembly (--cuda-device-only -S, the product flags), takes one
kernel's code, and classifies every instruction of the blocks the compiler marks as inside a
loop, by loop (header label, depth):
  slab   f32 arithmetic, min/max/min3/max3/med3, f32 compares, v_alignbit of the child tests
  int    integer / bit work: u32/i32/b32/b64 arithmetic and logic, bfe/bfi/bitop3, shifts,
         ffbh (clz), mbcnt, address adds
  move   v_mov / v_cndmask (selects)
  lds    ds_* ; vmem: buffer_/global_ loads and stores ; salu: s_* except branches/waits ;
  ctrl   branches and s_waitcnt / s_nop
Depth-1 blocks of the walk loop hold the internal-node visit, the push and the pop; deeper
loops are the inline leaf children and their sphere tests.
usage: python tools/isa_audit.py [kernel-substring] (default: ort_trace_pairILb0ELi1E, the C3 kernel)"""
import re
import subprocess
import sys
from collections import defaultdict
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
want = sys.argv[1] if len(sys.argv) > 1 else "ort_trace_pairILb0ELi1E"
asm = "/tmp/_ort_isa_audit.s"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-ffp-contract=off",
                "-fno-fast-math", "-fno-slp-vectorize", "-fPIC", "-Wno-unused-parameter", "--cuda-device-only", "-S",
                str(ROOT / "octreeraytracer_amd/csrc/ort_kernel.hip"), "-o", asm], check=True, capture_output=True)
text = open(asm).read()
names = [n for n in re.findall(r"^(_Z\S+):", text, re.M) if want in n]
if not names:
    raise SystemExit(f"no kernel matching {want}")
name = names[0]
body = text[text.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]

SLAB = re.compile(r"^v_(add|sub|subrev|mul|fma|fmac|min|max|min3|max3|med3|cmp_\w+_f32|cmpx_\w+_f32|div_\w+|rcp|sqrt|"
                  r"alignbit)\w*")
INT = re.compile(r"^v_(\w+_(u32|i32|b32|b64|u16|u64|i64)|bfe|bfi|bitop3|lshl|lshr|ashr|ffbh|ffbl|mbcnt|xad|and_or|"
                  r"or3|add3|lshl_add|lshl_or|add_lshl|xor3|cvt)\w*")
blocks = []
cur = None
for line in body.splitlines():
    m = re.match(r"^(\.LBB\S+):\s*(;.*)?$", line)
    if m:
        ann = m.group(2) or ""
        lm = re.search(r"Header=(\S+) Depth=(\d+)", ann)
        hm = re.search(r"Loop Header: Depth=(\d+)", ann)
        loop = (lm.group(1), int(lm.group(2))) if lm else ((m.group(1).replace(".LBB", "BB"), int(hm.group(1))) if hm else None)
        cur = {"label": m.group(1), "loop": loop, "ins": []}
        blocks.append(cur)
        continue
    t = line.strip()
    if cur is None or not t or t.startswith((";", ".")):
        continue
    cur["ins"].append(t.split()[0])


def classify(op):
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("buffer_", "global_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith(("s_cbranch", "s_branch", "s_waitcnt", "s_nop", "s_endpgm", "s_setprio")):
        return "ctrl"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("v_mov", "v_cndmask")):
        return "move"
    if INT.match(op) and not op.endswith("_f32"):
        return "int"
    if SLAB.match(op):
        return "slab"
    if op.startswith("v_"):
        return "int"
    return "other"


KINDS = ["slab", "int", "move", "lds", "vmem", "salu", "ctrl"]
per_loop = defaultdict(lambda: defaultdict(int))
print(f"kernel {name}")
print(f"{'block':12s} {'loop (header, depth)':28s} " + " ".join(f"{k:>5s}" for k in KINDS))
for b in blocks:
    if not b["loop"]:
        continue
    c = defaultdict(int)
    for op in b["ins"]:
        c[classify(op)] += 1
    for k in KINDS:
        per_loop[b["loop"]][k] += c[k]
    if sum(c.values()):
        print(f"{b['label']:12s} {str(b['loop']):28s} " + " ".join(f"{c[k]:5d}" for k in KINDS))
print("\nper loop (all blocks of each loop body at that depth; a block runs only when its branch is taken):")
for loop, c in sorted(per_loop.items(), key=lambda kv: (kv[0][1], kv[0][0])):
    v = c["slab"] + c["int"] + c["move"]
    print(f"  {str(loop):28s} VALU {v:4d} (slab {c['slab']}, int {c['int']}, move {c['move']})  lds {c['lds']}  "
          f"vmem {c['vmem']}  salu {c['salu']}  ctrl {c['ctrl']}")
