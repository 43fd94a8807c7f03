"""Known-answer tests of the canonical builtins (include/ort_math.h) and shader tables."""
import json
import sys
import math
from pathlib import Path

import numpy as np
import pytest

G = Path(__file__).resolve().parent / "golden"


def f32(x):
    return float(np.float32(x))


def ulp_diff(a, b):
    ia = np.array([a], np.float32).view(np.int32)[0]
    ib = np.array([b], np.float32).view(np.int32)[0]
    return abs(int(ia) - int(ib))


def test_sin_cos_within_one_ulp(oracle):
    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-7, 7, 4000), rng.uniform(-100, 100, 500), [0.0, 1e-30, 1e-8]]).astype(np.float32)
    lib = oracle.lib()
    for x in xs:
        assert ulp_diff(lib.oracle_sin(float(x)), f32(math.sin(float(x)))) <= 1, x
        assert ulp_diff(lib.oracle_cos(float(x)), f32(math.cos(float(x)))) <= 1, x


def test_pow_within_one_ulp(oracle):
    rng = np.random.default_rng(1)
    lib = oracle.lib()
    for y in (1.0 / 3.0, 5.0, 1.0 / 2.2):
        yf = f32(y)
        for x in rng.uniform(0, 1, 3000).astype(np.float32):
            want = f32(float(x) ** float(yf))
            assert ulp_diff(lib.oracle_pow(float(x), yf), want) <= 1, (x, yf)
    assert lib.oracle_pow(0.0, 0.45) == 0.0
    assert lib.oracle_pow(1.0, 0.45) == 1.0
    assert math.isnan(lib.oracle_pow(-0.5, 5.0))  # GLSL: undefined for x < 0 -> NaN here
    assert lib.oracle_pow(2.0, 0.0) == 1.0


def test_math_known_answers(oracle):
    m = json.loads((G / "manifest.json").read_text())["math"]
    lib = oracle.lib()
    for x, s, c, g in zip(m["x"], m["sin"], m["cos"], m["pow_gamma"]):
        assert lib.oracle_sin(x) == s and lib.oracle_cos(x) == c
        assert lib.oracle_pow(abs(np.float32(x)) / 7.0, 1.0 / 2.2) == g


def test_rand2D_sequences(oracle):
    m = json.loads((G / "manifest.json").read_text())["rand2D"]
    for k, seq in m.items():
        sx, sy = map(float, k.split(","))
        got = oracle.rand_sequence(sx, sy, len(seq))
        assert got.tolist() == seq
        assert (got >= 0).all() and (got < 1).all()


def test_rand2D_first_value_by_hand(oracle):
    """glsl:89-101 restated in numpy: float products, uint hash, fract."""
    sx, sy = np.float32(0.25), np.float32(0.75)
    s = np.uint32(np.float32(sx * np.float32(1664525.0)) + np.float32(sy * np.float32(1013904223.0)))
    s = np.uint32(s + np.uint32(1013904223))
    s ^= s >> np.uint32(16)
    s = np.uint32((int(s) * 0x85EBCA6B) & 0xFFFFFFFF)
    s ^= s >> np.uint32(13)
    s = np.uint32((int(s) * 0xC2B2AE35) & 0xFFFFFFFF)
    s ^= s >> np.uint32(16)
    v = np.float32(np.float32(s) / np.float32(4294967296.0))
    v = np.float32(v - np.floor(v))
    assert oracle.rand_sequence(0.25, 0.75, 1)[0] == v


# traversal orders of glsl:352-447 for every non-zero sign vector, derived from the shader file
# itself by tools/extract_orders.py (not hand-typed)
GOLDEN_ORDERS = Path(__file__).resolve().parent / "golden" / "traversal_orders.json"


def _clauses():
    return json.loads(GOLDEN_ORDERS.read_text())["clauses"]


def test_traversal_order_table_covers_26_sign_vectors(oracle):
    """The oracle's table (oracle/ort_oracle.c traversal_order) equals the shader's, clause by
    clause, for all 26 non-zero sign vectors."""
    seen = set()
    for c in _clauses():
        for v in c["sign_vectors"]:
            assert oracle.traversal_order(tuple(0.3 * x for x in v)) == c["order"], (c["name"], v)
            seen.add(tuple(v))
    assert len(seen) == 26 and (0, 0, 0) not in seen
    # SURVEY.md 8(c) examples (shader table, not test.py's formula)
    assert oracle.traversal_order((-1, 0, 0)) == [3, 1, 2, 0, 7, 5, 6, 4]
    assert oracle.traversal_order((-1, -1, -1)) == [7, 5, 6, 4, 3, 1, 2, 0]
    assert oracle.traversal_order((0, 1, 0)) == [2, 0, 3, 1, 6, 4, 7, 5]


def test_kernel_closed_form_orders_match_shader_tables(ort):
    """The kernel's fast walk uses order[r] = perm(r) ^ m (render_core.h rank_perm) for rays
    with no zero direction component, and a rank LUT built from it; both against the shader's
    tables for the 8 all-non-zero sign vectors."""
    import ctypes as C

    from octreeraytracer_amd import _lib as L
    lib = L.analysis_lib()
    by_vec = {tuple(v): c["order"] for c in _clauses() for v in c["sign_vectors"]}
    for sx in (-1, 1):
        for sy in (-1, 1):
            for sz in (-1, 1):
                m = (int(sz < 0) << 2) | (int(sx < 0) << 1) | int(sy < 0)
                order = (C.c_int32 * 8)()
                lut = (C.c_uint8 * 256)()
                L.acheck(lib.ort_debug_fast_order(m, order, lut))
                want = by_vec[(sx, sy, sz)]
                assert list(order) == want, (sx, sy, sz)
                # LUT row: child mask (octant space) -> reversed rank bits (rank r = bit 7 - r)
                for cmask in range(256):
                    bits = sum(0x80 >> r for r in range(8) if (cmask >> want[r]) & 1)
                    assert lut[cmask] == bits, (m, cmask)


def test_rank_lut_is_a_bit_permutation(ort):
    """fast_step folds the rejected-sphere skip into the child mask before its one rank-LUT read
    (render_core.h, ORT_KID_SKIP_FOLD): lut[c & ~s] == lut[c] & ~lut[s] for every child mask c
    and skip mask s, which holds because each LUT row maps octant bits to rank bits one for one."""
    import ctypes as C

    from octreeraytracer_amd import _lib as L
    lib = L.analysis_lib()
    c = np.arange(256)[:, None]
    s = np.arange(256)[None, :]
    for m in range(8):
        order = (C.c_int32 * 8)()
        lut = (C.c_uint8 * 256)()
        L.acheck(lib.ort_debug_fast_order(m, order, lut))
        t = np.frombuffer(bytes(lut), np.uint8).astype(np.int64)
        assert sorted(int(t[1 << k]) for k in range(8)) == [1 << r for r in range(8)], m  # one rank bit each
        assert (t[c & ~s] == (t[c] & ~t[s] & 0xFF)).all(), m


def test_order_fixture_is_current():
    """tests/golden/traversal_orders.json was generated from the reference shader (checked
    against the file when the reference is present, i.e. in the build container)."""
    import hashlib
    rec = json.loads(GOLDEN_ORDERS.read_text())
    shader = Path("/root/reference/shaders/octree_fragment_shader.glsl")
    assert rec["generator"] == "tools/extract_orders.py" and len(rec["clauses"]) == 8
    if shader.exists():
        assert hashlib.sha256(shader.read_bytes()).hexdigest() == rec["source_sha256"]
        sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "tools"))
        import extract_orders
        assert extract_orders.extract(shader.read_text()) == rec["clauses"]


def test_canonical_builtins_sweep(tmp_path):
    """tools/math_check.c: sin/cos over |x| <= 8 and pow(x, y) over x in (0, 4] for the shader's
    exponents (1/2.2, 1/3, 5) and two others, against libm rounded to float -- every result
    within 1 ulp.  Strided here (seconds); the every-float sweep (stride 1) is recorded in
    profiles/r03_math_check_exhaustive.log."""
    import subprocess
    root = Path(__file__).resolve().parents[1]
    exe = tmp_path / "math_check"
    subprocess.run(["gcc", "-O2", "-std=c99", "-ffp-contract=off", "-I", str(root / "include"),
                    str(root / "tools" / "math_check.c"), "-lm", "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "4099"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK: every result within 1 ulp" in r.stdout
