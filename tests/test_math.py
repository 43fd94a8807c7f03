"""Known-answer tests of the canonical builtins (include/ort_math.h) and shader tables."""
import json
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


# traversal orders of glsl:352-447 for every non-zero sign vector
GLSL_ORDERS = {
    "cyan": ([0, 1, 2, 3, 4, 5, 6, 7], [(1, 1, 1)]),
    "yellow": ([2, 0, 3, 1, 6, 4, 7, 5], [(-1, 1, 1), (-1, 1, 0), (0, 1, 0), (0, 1, 1)]),
    "red": ([3, 1, 2, 0, 7, 5, 6, 4], [(-1, -1, 1), (-1, 0, 1), (0, 0, 1), (0, -1, 1), (-1, -1, 0), (0, -1, 0),
                                        (-1, 0, 0)]),
    "dark purple": ([1, 0, 3, 2, 5, 4, 7, 6], [(1, -1, 1), (1, 0, 1), (1, -1, 0), (1, 0, 0)]),
    "blue": ([4, 5, 6, 7, 0, 1, 2, 3], [(1, 1, -1), (1, 0, -1), (0, 1, -1), (1, 1, 0)]),
    "purple": ([6, 4, 7, 5, 2, 0, 3, 1], [(-1, 1, -1)]),
    "green": ([7, 5, 6, 4, 3, 1, 2, 0], [(-1, -1, -1), (-1, 0, -1), (0, -1, -1), (0, 0, -1)]),
    "black": ([5, 4, 7, 6, 1, 0, 3, 2], [(1, -1, -1)]),
}


def test_traversal_order_table_covers_26_sign_vectors(oracle):
    seen = set()
    for order, vecs in GLSL_ORDERS.values():
        for v in vecs:
            assert oracle.traversal_order(tuple(0.3 * c for c in v)) == order, v
            seen.add(v)
    assert len(seen) == 26
    # SURVEY.md 8(c) examples (shader table, not test.py's formula)
    assert oracle.traversal_order((-1, 0, 0)) == [3, 1, 2, 0, 7, 5, 6, 4]
    assert oracle.traversal_order((-1, -1, -1)) == [7, 5, 6, 4, 3, 1, 2, 0]
    assert oracle.traversal_order((0, 1, 0)) == [2, 0, 3, 1, 6, 4, 7, 5]
