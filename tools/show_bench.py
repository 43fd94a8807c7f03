"""One summary line per bench.py JSON line: value, ms/step, roofline frac, PMC match, single-frame
value, CPU baseline.  usage: python tools/show_bench.py BENCH.json [...]"""
import json
import sys

for p in sys.argv[1:]:
    d = json.loads(open(p).read().strip().splitlines()[-1])
    r = d.get("roofline") or {}
    sf = d.get("single_frame") or {}
    cb = d.get("cpu_baseline") or {}
    print(f"{p}: {d['value']} {d['unit']}  {d['ms_per_step']} ms/step  frac {r.get('frac')}  "
          f"pmc_matches {r.get('pmc_matches_build')}  single-frame {sf.get('value')}  cpu {cb.get('value')}")
