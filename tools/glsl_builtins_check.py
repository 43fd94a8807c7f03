"""How much of the GLSL-vs-oracle difference is GLSL's builtins? (analysis only)

Runs the reference's shaders on Mesa llvmpipe (oracle/_ref/glsl_run) twice per case of
tools/make_glsl_golden.py: as they are, and with a PRELUDE inserted after the fragment shader's
#version line (in memory; the reference's file is never touched) that substitutes the oracle's
canonical builtins (include/ort_math.h: double-precision sin/cos/pow with fma, the glm forms of
normalize/dot/length/cross/reflect, min/max in the GLSL spec's (y < x) ? y : x form) for llvmpipe's, via function-like macros -- and compares both
frames with the CPU oracle.  (What a prelude cannot reach is llvmpipe's own arithmetic in the
shader's expressions; measured, it changes nothing there: with the prelude every frame of
tests/golden/glsl/canonical.json is bit-identical to the oracle's.)
The prelude also reads the pixel centre from gl_FragCoord instead of the interpolated FragCoord
varying (FRAGCOORD_REPLACE below).
usage: LP_NUM_THREADS=8 python tools/glsl_builtins_check.py [case ...]"""
import re
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import make_glsl_golden as M  # noqa: E402
from oracle import oracle as O  # noqa: E402


def consts():
    """The constants and tables of include/ort_math.h as GLSL double literals (exact decimal)."""
    text = (ROOT / "include" / "ort_math.h").read_text()
    c = {}
    for name, val in re.findall(r"#define (ORT_\w+) (-?0x[0-9a-fA-F.]+p[+-]?\d+)", text):
        c[name] = float.fromhex(val)
    for tab in ("ORT_LOG2_TAB_VALUES", "ORT_EXP2_TAB_VALUES"):
        body = text[text.index(f"#define {tab}"):]
        body = body[body.index("{") + 1:body.index("}")]
        c[tab] = [float.fromhex(v) for v in re.findall(r"-?0x[0-9a-fA-F.]+p[+-]?\d+", body)]
    return c


def lit(x):
    return repr(float(x)) + "LF"


# The pixel centre: the reference's fragment shader reads the FragCoord varying its vertex shader
# sets to (clip xy + 1) / 2 * iResolution at the quad's corners (vertex_shader.glsl:15), i.e. the
# exact pixel centre (x + 0.5, y + 0.5) wherever interpolation is exact -- but the precision of
# varying interpolation is implementation-defined, and llvmpipe's plane equations miss it by an ulp
# at some frame sizes (e.g. 344x180 or 333x177: 39-44 % of the pixels then differ, since the pixel's
# RNG is seeded from FragCoord, octree_fragment_shader.glsl:640).  The canonical frame reads the
# centre from gl_FragCoord, which the rasterizer gives exactly (glsl_run's //@replace line).
FRAGCOORD_REPLACE = "//@replace in vec2 FragCoord;\t#define FragCoord gl_FragCoord\n"


def prelude():
    c = consts()
    tab = lambda k: "double[{}]({})".format(len(c[k]), ", ".join(lit(v) for v in c[k]))  # noqa: E731
    return FRAGCOORD_REPLACE + f"""
// ---- analysis prelude: the canonical builtins of include/ort_math.h (and the exact pixel centre) ----
const double ORT_LOG2_TAB[32] = {tab("ORT_LOG2_TAB_VALUES")};
const double ORT_EXP2_TAB[32] = {tab("ORT_EXP2_TAB_VALUES")};
const double ORT_RNE = 6755399441055744.0LF;
float ort_nan() {{ return uintBitsToFloat(0x7fc00000u); }}
float ort_inf() {{ return uintBitsToFloat(0x7f800000u); }}
float ort_dot(vec3 a, vec3 b) {{ precise float r = (a.x * b.x + a.y * b.y) + a.z * b.z; return r; }}
float ort_dot(vec2 a, vec2 b) {{ precise float r = a.x * b.x + a.y * b.y; return r; }}
vec3 ort_normalize(vec3 v) {{ precise float s = 1.0 / sqrt(ort_dot(v, v)); precise vec3 r = v * s; return r; }}
vec3 ort_cross(vec3 x, vec3 y) {{
    precise vec3 r = vec3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); return r; }}
vec3 ort_reflect(vec3 i, vec3 n) {{ precise float k = 2.0 * ort_dot(n, i); precise vec3 r = i - k * n; return r; }}
void ort_sincos(float xf, out float sn, out float cs) {{
    if (isnan(xf) || isinf(xf)) {{ sn = ort_nan(); cs = ort_nan(); return; }}
    precise double x = double(xf);
    precise double kd = (x * {lit(c["ORT_2_PI_D"])} + ORT_RNE) - ORT_RNE;
    precise double r = fma(-kd, {lit(c["ORT_PIO2_LO_D"])}, fma(-kd, {lit(c["ORT_PIO2_HI_D"])}, x));
    precise double z = r * r;
    precise double sp = fma(r * z, fma(z, fma(z, fma(z, {lit(c["ORT_SIN_P3"])}, {lit(c["ORT_SIN_P2"])}),
                                         {lit(c["ORT_SIN_P1"])}), {lit(c["ORT_SIN_P0"])}), r);
    precise double cp = fma(z, fma(z, fma(z, fma(z, {lit(c["ORT_COS_P3"])}, {lit(c["ORT_COS_P2"])}),
                                   {lit(c["ORT_COS_P1"])}), {lit(c["ORT_COS_P0"])}), 1.0LF);
    int q = int(kd) & 3;
    double sv = (q & 1) != 0 ? cp : sp, cv = (q & 1) != 0 ? sp : cp;
    sn = float((q & 2) != 0 ? -sv : sv);
    cs = float(((q + 1) & 2) != 0 ? -cv : cv);
}}
float ort_sin(float x) {{ float s, c; ort_sincos(x, s, c); return s; }}
float ort_cos(float x) {{ float s, c; ort_sincos(x, s, c); return c; }}
float ort_tan(float x) {{ float s, c; ort_sincos(x, s, c); return float(double(s) / double(c)); }}
double ort_log2_d(float xf) {{
    uint ix = floatBitsToUint(xf);
    int ks = 0;
    if (ix < 0x00800000u) {{ float xs = xf * 8388608.0; ix = floatBitsToUint(xs); ks = -23; }}
    uint tmp = ix - 0x3f330000u;
    int i = int((tmp >> 19) & 15u);
    uint iz = ix - (tmp & 0xff800000u);
    int k = (int(tmp) >> 23) + ks;
    float zf = uintBitsToFloat(iz);
    precise double r = fma(double(zf), ORT_LOG2_TAB[2 * i], -1.0LF);
    precise double p = r * fma(r, fma(r, fma(r, fma(r, {lit(c["ORT_LOG2_P4"])}, {lit(c["ORT_LOG2_P3"])}),
                                         {lit(c["ORT_LOG2_P2"])}), {lit(c["ORT_LOG2_P1"])}), {lit(c["ORT_LOG2_P0"])});
    precise double res = (double(k) + ORT_LOG2_TAB[2 * i + 1]) + p;
    return res;
}}
float ort_exp2_f(double t) {{
    precise double kd = (t * 32.0LF + ORT_RNE) - ORT_RNE;
    precise double r = fma(kd, -0.03125LF, t);
    int ki = int(kd);
    precise double p = fma(r, fma(r, fma(r, {lit(c["ORT_EXP2_P2"])}, {lit(c["ORT_EXP2_P1"])}), {lit(c["ORT_EXP2_P0"])}), 1.0LF);
    uvec2 w = unpackDouble2x32(ORT_EXP2_TAB[ki & 31]);
    w.y += uint((ki >> 5) << 20);
    precise double res = packDouble2x32(w) * p;
    return float(res);
}}
float ort_pow(float x, float y) {{
    if (isnan(x) || isnan(y)) return ort_nan();
    if (x < 0.0) return ort_nan();
    if (y == 0.0) return 1.0;
    if (x == 0.0) return (y > 0.0) ? 0.0 : ort_inf();
    if (isinf(x)) return (y > 0.0) ? ort_inf() : 0.0;
    if (x == 1.0) return 1.0;
    precise double t = double(y) * ort_log2_d(x);
    if (t >= 128.0LF) return ort_inf();
    if (t <= -150.0LF) return 0.0;
    return ort_exp2_f(t);
}}
vec3 ort_pow(vec3 x, vec3 y) {{ return vec3(ort_pow(x.x, y.x), ort_pow(x.y, y.y), ort_pow(x.z, y.z)); }}
float ort_min(float x, float y) {{ return (y < x) ? y : x; }}
float ort_max(float x, float y) {{ return (x < y) ? y : x; }}
vec3 ort_min(vec3 x, vec3 y) {{ return vec3(ort_min(x.x, y.x), ort_min(x.y, y.y), ort_min(x.z, y.z)); }}
vec3 ort_max(vec3 x, vec3 y) {{ return vec3(ort_max(x.x, y.x), ort_max(x.y, y.y), ort_max(x.z, y.z)); }}
#define sin(x) ort_sin(x)
#define cos(x) ort_cos(x)
#define tan(x) ort_tan(x)
#define pow(x, y) ort_pow(x, y)
#define normalize(v) ort_normalize(v)
#define dot(a, b) ort_dot(a, b)
#define length(v) sqrt(ort_dot(v, v))
#define cross(a, b) ort_cross(a, b)
#define reflect(i, n) ort_reflect(i, n)
#define min(x, y) ort_min(x, y)
#define max(x, y) ort_max(x, y)
// ---- end of prelude ----
"""


def run(s, t, p, pre=None):
    """The GLSL frame, with the prelude text pre inserted (or as is)."""
    if pre is None:
        return M.run_glsl(s, t, p)[0]
    with tempfile.TemporaryDirectory() as d:
        Path(f"{d}/pre.glsl").write_text(pre)
        return M.run_glsl(s, t, p, prelude=f"{d}/pre.glsl")[0]


def stats(img, o):
    d = np.abs(img.astype(np.float64) - o.astype(np.float64)).max(-1)
    bits = (img.view(np.uint32) == o.view(np.uint32)).all(-1)
    return (f"bit-equal {bits.mean():.4f}  <=1e-6 {np.mean(d <= 1e-6):.5f}  <=1e-4 {np.mean(d <= 1e-4):.5f}  "
            f">1e-3 {int((d > 1e-3).sum())}")


def main():
    pre = prelude()
    names = sys.argv[1:] or [n for n in M.CASES if n != "c3_full_rows"]
    for name in names:
        c = M.CASES[name]
        s, t, p = M.case_inputs(c)
        o = O.render(s, t if p.use_octree else None, p)
        print(f"{name:18s} as is:          {stats(run(s, t, p), o)}", flush=True)
        print(f"{'':18s} canonical builtins: {stats(run(s, t, p, pre), o)}", flush=True)


if __name__ == "__main__":
    main()
