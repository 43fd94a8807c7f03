"""The reference shaders on Mesa llvmpipe against the CPU oracle over one whole frame, with both
timed on this machine's CPUs (analysis only; profiles/r05_glsl_c3_full.log).
usage: LP_NUM_THREADS=8 python tools/glsl_vs_oracle.py"""
import sys, time, os, numpy as np
from pathlib import Path
ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT)); sys.path.insert(0, str(ROOT / 'tools'))
import make_glsl_golden as M
from oracle import oracle as O
c = dict(M.CASES['c3_full_rows']); s, t, p = M.case_inputs(c)
tm = {}
img, r = M.run_glsl(s, t, p, tm)
print('reference shader on llvmpipe, 8 threads: C3 frame draw %.0f ms -> %.3f Mrays/s' % (tm['draw_ms'], p.width * p.height / tm['draw_ms'] / 1e3))
t0 = time.time(); o = O.render(s, t, p, threads=8); dt = time.time() - t0
print('oracle, 8 threads: C3 frame %.0f ms -> %.3f Mrays/s' % (dt * 1e3, p.width * p.height / dt / 1e6))
d = np.abs(img.astype(np.float64) - o).max(-1)
print('full C3 frame: px %d, within 1e-6 %.6f, within 1e-5 %.6f, > 1e-3: %d' % (d.size, np.mean(d <= 1e-6), np.mean(d <= 1e-5), int((d > 1e-3).sum())))
