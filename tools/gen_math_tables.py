"""Generates the constants of the canonical transcendentals in include/ort_math.h (round 3):
table-driven log2/exp2 for pow, and the sin/cos kernels, all evaluated in double with fma.

Everything is computed with mpmath at 60 digits and rounded to double once:
  * log2: 16 sub-intervals of z in [0.69921875, 1.3984375) (float bit ranges, see
    ort__log2_d); per interval invc = double(1 / centre) (1.0 for the one holding 1.0) and
    logc = double(-log2(invc)) -- so log2(z) = logc + log2(1 + r) with r = z * invc - 1 holds
    for ANY invc; the polynomial fits log2(1 + r) / r over the largest |r| of the tables;
  * exp2: T[j] = double(2^(j/32)); the polynomial fits 2^r over |r| <= 1/64;
  * sin/cos: polynomials over |r| <= pi/4 + 2^-10 (the reduction may land slightly past pi/4).
Polynomials are least-squares fits at Chebyshev nodes (near-minimax; the error budget, a few
2^-33 relative, is far below a float ulp), then checked here against mpmath.
usage: python tools/gen_math_tables.py   (prints the C fragment)"""
import mpmath as mp

mp.mp.dps = 60


def d(x) -> float:
    return float(mp.mpf(x))  # rounds to nearest double


def hexd(x: float) -> str:
    return float.hex(x)


def fit(func, lo, hi, powers, n=400, weight=None):
    """least squares for func(t) ~ sum c_k * t^p_k at Chebyshev nodes in [lo, hi]"""
    xs = [lo + (hi - lo) * (1 - mp.cos(mp.pi * (i + 0.5) / n)) / 2 for i in range(n)]
    A = mp.matrix(n, len(powers))
    b = mp.matrix(n, 1)
    for i, x in enumerate(xs):
        w = weight(x) if weight else 1
        for j, p in enumerate(powers):
            A[i, j] = x ** p * w
        b[i] = func(x) * w
    c = mp.lu_solve(A.T * A, A.T * b)
    return [d(c[j]) for j in range(len(powers))]


def float_bits(u: int) -> mp.mpf:
    import struct
    return mp.mpf(struct.unpack("<f", struct.pack("<I", u))[0])


def main():
    out = []
    # ---- log2 tables ---------------------------------------------------------------
    OFF = 0x3F330000
    rmax = mp.mpf(0)
    tab = []
    for i in range(16):
        lo = float_bits(OFF + (i << 19))
        hi = float_bits(OFF + ((i + 1) << 19))
        if lo <= 1 < hi:
            invc = 1.0
        else:
            invc = d(2 / (lo + hi))
        logc = d(-mp.log(mp.mpf(invc), 2))
        tab.append((invc, logc))
        for z in (lo, hi):
            rmax = max(rmax, abs(z * mp.mpf(invc) - 1))
    out.append("/* log2 table (tools/gen_math_tables.py): {invc, logc} per sub-interval, |r| <= %.6f */" % float(rmax))
    out.append("#define ORT_LOG2_TAB_VALUES { \\")
    for invc, logc in tab:
        out.append("    %s, %s, \\" % (hexd(invc), hexd(logc)))
    out.append("}")
    R = rmax * mp.mpf("1.001")
    lc = fit(lambda r: mp.log(1 + r, 2) / r if r != 0 else 1 / mp.log(2), -R, R, [0, 1, 2, 3, 4])
    err = max(abs((sum(c * r ** k for k, c in enumerate(lc)) * r - mp.log(1 + r, 2)))
              for r in mp.linspace(-R, R, 2001))
    out.append("/* log2(1 + r) = r * (A0 + A1 r + ... + A4 r^4), max abs error %.3g (2^%.1f) */" %
               (float(err), float(mp.log(err, 2))))
    out += ["#define ORT_LOG2_P%d %s" % (k, hexd(c)) for k, c in enumerate(lc)]
    # ---- exp2 table ----------------------------------------------------------------
    out.append("/* exp2 table: 2^(j/32), j = 0..31 */")
    out.append("#define ORT_EXP2_TAB_VALUES { \\")
    for j in range(0, 32, 4):
        out.append("    " + ", ".join(hexd(d(mp.mpf(2) ** (mp.mpf(jj) / 32))) for jj in range(j, j + 4)) + ", \\")
    out.append("}")
    Re = mp.mpf(1) / 64 * mp.mpf("1.0001")
    ec = fit(lambda r: (mp.mpf(2) ** r - 1) / r if r != 0 else mp.log(2), -Re, Re, [0, 1, 2])
    err = max(abs((1 + r * sum(c * r ** k for k, c in enumerate(ec))) / mp.mpf(2) ** r - 1)
              for r in mp.linspace(-Re, Re, 2001))
    out.append("/* 2^r = 1 + r * (C0 + C1 r + C2 r^2), |r| <= 1/64, max rel error %.3g (2^%.1f) */" %
               (float(err), float(mp.log(err, 2))))
    out += ["#define ORT_EXP2_P%d %s" % (k, hexd(c)) for k, c in enumerate(ec)]
    # ---- sin / cos -----------------------------------------------------------------
    Rs = mp.pi / 4 + mp.mpf(2) ** -10
    Z = Rs * Rs
    sc = fit(lambda z: (mp.sin(mp.sqrt(z)) / mp.sqrt(z) - 1) / z if z != 0 else mp.mpf(-1) / 6, mp.mpf(0), Z,
             [0, 1, 2, 3], weight=None)
    err = max(abs((r + r ** 3 * sum(c * (r * r) ** k for k, c in enumerate(sc))) / mp.sin(r) - 1)
              for r in mp.linspace(mp.mpf(2) ** -20, Rs, 2001))
    out.append("/* sin(r) = r + r^3 (S0 + S1 z + S2 z^2 + S3 z^3), z = r^2, |r| <= pi/4 + 2^-10: rel error %.3g (2^%.1f) */"
               % (float(err), float(mp.log(err, 2))))
    out += ["#define ORT_SIN_P%d %s" % (k, hexd(c)) for k, c in enumerate(sc)]
    cc = fit(lambda z: (mp.cos(mp.sqrt(z)) - 1) / z if z != 0 else mp.mpf(-1) / 2, mp.mpf(0), Z, [0, 1, 2, 3])
    err = max(abs((1 + r * r * sum(c * (r * r) ** k for k, c in enumerate(cc))) / mp.cos(r) - 1)
              for r in mp.linspace(0, Rs, 2001))
    out.append("/* cos(r) = 1 + z (C0 + C1 z + C2 z^2 + C3 z^3): rel error %.3g (2^%.1f) */" %
               (float(err), float(mp.log(err, 2))))
    out += ["#define ORT_COS_P%d %s" % (k, hexd(c)) for k, c in enumerate(cc)]
    pio2 = mp.pi / 2
    hi = d(pio2)
    out.append("/* pi/2 = PIO2_HI + PIO2_LO (double + double), 2/pi */")
    out.append("#define ORT_PIO2_HI_D %s" % hexd(hi))
    out.append("#define ORT_PIO2_LO_D %s" % hexd(d(pio2 - mp.mpf(hi))))
    out.append("#define ORT_2_PI_D %s" % hexd(d(2 / mp.pi)))
    print("\n".join(out))


if __name__ == "__main__":
    main()
