/*
 * ort_math.h -- canonical GLSL builtins shared by the HIP kernel and the CPU oracle.
 *
 * The reference evaluates these builtins inside a vendor GL driver
 * (shaders/octree_fragment_shader.glsl uses normalize/sqrt/fract/min/max/sin/cos/pow;
 * e.g. :146, :152-156, :168-170, :522, :661).  Their exact results are driver-defined,
 * so this project pins ONE canonical form and compiles the SAME
 * source on the host (gcc -ffp-contract=off) and on gfx950 (hipcc -ffp-contract=off):
 *
 *   normalize(v)  = v * (1.0f / sqrtf(dot(v,v)))     glm form, include/glm/detail/func_geometric.inl:82-90
 *   dot(a,b)      = (a.x*b.x + a.y*b.y) + a.z*b.z   glm compute_dot, func_geometric.inl:48-55
 *   min(x,y)      = (y < x) ? y : x                  GLSL spec form (NaN behaviour fixed)
 *   max(x,y)      = (x < y) ? y : x
 *   fract(x)      = x - floorf(x)
 *   sin/cos/pow   = float(double-precision kernel)   identical IEEE op sequence on both sides
 *
 * Only IEEE-exact primitives are used (+ - * / sqrt floor, int<->float conversions,
 * bit casts), so host and device produce bit-identical results.  This header is C99 so
 * the plain-C oracle can include it; under hipcc every function is __host__ __device__.
 */
#ifndef ORT_MATH_H
#define ORT_MATH_H

#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define ORT_HD __host__ __device__ static inline __attribute__((always_inline))
#else
#define ORT_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

/* ---- scalar helpers ---------------------------------------------------- */
ORT_HD float ort_minf(float x, float y) { return (y < x) ? y : x; }
ORT_HD float ort_maxf(float x, float y) { return (x < y) ? y : x; }
ORT_HD float ort_fract(float x) { return x - floorf(x); }

ORT_HD double ort__bits_to_d(uint64_t u) { double d; __builtin_memcpy(&d, &u, 8); return d; }
ORT_HD uint64_t ort__d_to_bits(double d) { uint64_t u; __builtin_memcpy(&u, &d, 8); return u; }
ORT_HD float ort__nanf(void) { uint32_t u = 0x7fc00000u; float f; __builtin_memcpy(&f, &u, 4); return f; }
ORT_HD float ort__inff(void) { uint32_t u = 0x7f800000u; float f; __builtin_memcpy(&f, &u, 4); return f; }

/* ---- canonical sin / cos / pow (round 3) -------------------------------- */
/* All three are evaluated in double with explicit fma() -- an IEEE-exact, correctly rounded
 * primitive on both sides (glibc fma / v_fma_f64), so host and device stay bit-identical --
 * and rounded to float once.  Constants, tables and polynomial fits come from
 * tools/gen_math_tables.py (mpmath); every fit's error is below 2^-31 relative, so results
 * are within 1 float ulp of the correctly rounded value (most are correctly rounded;
 * tools/math_check.c samples the whole range against libm).  Round 2 used fdlibm-style
 * kernels without fma (sin/cos ~2x the double ops; pow an 11-term log series with a double
 * division plus a 14-term exp series) -- 5.5 % of a C3 frame (tools/ab_stream.py against the
 * hardware v_sin/v_log/v_exp, ORT_MEASURE_NATIVE_MATH). */
/* log2 table (tools/gen_math_tables.py): {invc, logc} per sub-interval, |r| <= 0.029630 */
#define ORT_LOG2_TAB_VALUES { \
    0x1.661ec6a5122f9p+0, -0x1.efec61b011f85p-2, \
    0x1.571ed3c506b3ap+0, -0x1.b0b67f4f46812p-2, \
    0x1.49539e3b2d067p+0, -0x1.7418acebbf18fp-2, \
    0x1.3c995a47babe7p+0, -0x1.39de8e1559f6ep-2, \
    0x1.30d190130d190p+0, -0x1.01d9bbcfa61d4p-2, \
    0x1.25e22708092f1p+0, -0x1.97c1cb13c7ec0p-3, \
    0x1.1bb4a4046ed29p+0, -0x1.2f9e32d5bfdd1p-3, \
    0x1.12358e75d3033p+0, -0x1.960caf9abb7c1p-4, \
    0x1.0953f39010954p+0, -0x1.a6f9c377dd31dp-5, \
    0x1.0000000000000p+0, 0x0.0p+0, \
    0x1.e573ac901e574p-1, 0x1.3aa2fdd27f1bfp-4, \
    0x1.ca4b3055ee191p-1, 0x1.476a9f983f74dp-3, \
    0x1.b2036406c80d9p-1, 0x1.e840be74e6a4dp-3, \
    0x1.9c2d14ee4a102p-1, 0x1.406463b1b0448p-2, \
    0x1.886e5f0abb04ap-1, 0x1.88e9c72e0b224p-2, \
    0x1.767dce434a9b1p-1, 0x1.ce0a4923a587dp-2, \
}
/* log2(1 + r) = r * (A0 + A1 r + ... + A4 r^4), max abs error 1.04e-11 (2^-36.5) */
#define ORT_LOG2_P0 0x1.71547652bd036p+0
#define ORT_LOG2_P1 -0x1.7154745ecb27fp-1
#define ORT_LOG2_P2 0x1.ec7097bcc7ca0p-2
#define ORT_LOG2_P3 -0x1.7199d1e6054f7p-2
#define ORT_LOG2_P4 0x1.27be1ddd081fep-2
/* exp2 table: 2^(j/32), j = 0..31 */
#define ORT_EXP2_TAB_VALUES { \
    0x1.0000000000000p+0, 0x1.059b0d3158574p+0, 0x1.0b5586cf9890fp+0, 0x1.11301d0125b51p+0, \
    0x1.172b83c7d517bp+0, 0x1.1d4873168b9aap+0, 0x1.2387a6e756238p+0, 0x1.29e9df51fdee1p+0, \
    0x1.306fe0a31b715p+0, 0x1.371a7373aa9cbp+0, 0x1.3dea64c123422p+0, 0x1.44e086061892dp+0, \
    0x1.4bfdad5362a27p+0, 0x1.5342b569d4f82p+0, 0x1.5ab07dd485429p+0, 0x1.6247eb03a5585p+0, \
    0x1.6a09e667f3bcdp+0, 0x1.71f75e8ec5f74p+0, 0x1.7a11473eb0187p+0, 0x1.82589994cce13p+0, \
    0x1.8ace5422aa0dbp+0, 0x1.93737b0cdc5e5p+0, 0x1.9c49182a3f090p+0, 0x1.a5503b23e255dp+0, \
    0x1.ae89f995ad3adp+0, 0x1.b7f76f2fb5e47p+0, 0x1.c199bdd85529cp+0, 0x1.cb720dcef9069p+0, \
    0x1.d5818dcfba487p+0, 0x1.dfc97337b9b5fp+0, 0x1.ea4afa2a490dap+0, 0x1.f50765b6e4540p+0, \
}
/* 2^r = 1 + r * (C0 + C1 r + C2 r^2), |r| <= 1/64, max rel error 1.45e-10 (2^-32.7) */
#define ORT_EXP2_P0 0x1.62e42fef8dc43p-1
#define ORT_EXP2_P1 0x1.ebfccc6482734p-3
#define ORT_EXP2_P2 0x1.c6b13c3d5a15cp-5
/* sin(r) = r + r^3 (S0 + S1 z + S2 z^2 + S3 z^3), z = r^2, |r| <= pi/4 + 2^-10: rel error 1.94e-11 (2^-35.6) */
#define ORT_SIN_P0 -0x1.555555545bd2ep-3
#define ORT_SIN_P1 0x1.11110de9a5104p-7
#define ORT_SIN_P2 -0x1.a0139ffd174f6p-13
#define ORT_SIN_P3 0x1.6dbb8c887bacbp-19
/* cos(r) = 1 + z (C0 + C1 z + C2 z^2 + C3 z^3): rel error 2.72e-10 (2^-31.8) */
#define ORT_COS_P0 -0x1.fffffffaa5ec3p-2
#define ORT_COS_P1 0x1.55554cac4c412p-5
#define ORT_COS_P2 -0x1.6c0dfe3485608p-10
#define ORT_COS_P3 0x1.9a6bcbbb1ebeep-16
/* pi/2 = PIO2_HI + PIO2_LO (double + double), 2/pi */
#define ORT_PIO2_HI_D 0x1.921fb54442d18p+0
#define ORT_PIO2_LO_D 0x1.1a62633145c07p-54
#define ORT_2_PI_D 0x1.45f306dc9c883p-1

#if defined(__HIPCC__)
#define ORT_TAB_DECL static constexpr
#else
#define ORT_TAB_DECL static const
#endif

/* round-to-nearest-even of a double with |v| < 2^51, as (v + 1.5*2^52) - 1.5*2^52 */
#define ORT_RNE_SHIFT 0x1.8p52

/* sin and cos of the same float argument (each equals what it would be on its own).
 * Reduction by pi/2 in double with a two-part constant and fma: r = x - k*pi/2 to ~2^-100
 * absolute for |x| < 2^24 (beyond that the results stay deterministic, not accurate). */
ORT_HD void ort_sincosf(float xf, float* sn, float* cs) {
#if ORT_NATIVE_TRIG && defined(__HIP_DEVICE_COMPILE__)
    *sn = __builtin_amdgcn_sinf(xf * 0.15915494309189535f);
    *cs = __builtin_amdgcn_cosf(xf * 0.15915494309189535f);
    return;
#endif
    if (!(xf == xf) || xf == ort__inff() || xf == -ort__inff()) {
        *sn = ort__nanf();
        *cs = ort__nanf();
        return;
    }
    const double x = (double)xf;
    const double kd = (x * ORT_2_PI_D + ORT_RNE_SHIFT) - ORT_RNE_SHIFT;
    const double r = fma(-kd, ORT_PIO2_LO_D, fma(-kd, ORT_PIO2_HI_D, x));
    const double z = r * r;
    const double s0 = ORT_SIN_P0, s1 = ORT_SIN_P1, s2 = ORT_SIN_P2, s3 = ORT_SIN_P3;
    const double c0 = ORT_COS_P0, c1 = ORT_COS_P1, c2 = ORT_COS_P2, c3 = ORT_COS_P3;
    const double sp = fma(r * z, fma(z, fma(z, fma(z, s3, s2), s1), s0), r);
    const double cp = fma(z, fma(z, fma(z, fma(z, c3, c2), c1), c0), 1.0);
    const int q = (int)((int64_t)kd & 3);
    const double sv = (q & 1) ? cp : sp, cv = (q & 1) ? sp : cp;
    *sn = (float)((q & 2) ? -sv : sv);
    *cs = (float)(((q + 1) & 2) ? -cv : cv);
}
ORT_HD float ort_sinf(float xf) {
#if ORT_NATIVE_TRIG && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sinf(xf * 0.15915494309189535f);
#endif
    float s, c;
    ort_sincosf(xf, &s, &c);
    return s;
}
ORT_HD float ort_cosf(float xf) {
#if ORT_NATIVE_TRIG && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_cosf(xf * 0.15915494309189535f);
#endif
    float s, c;
    ort_sincosf(xf, &s, &c);
    return c;
}
/* tan is only used on the host for the camera frustum (glsl:192). */
ORT_HD float ort_tanf(float xf) {
    float s, c;
    ort_sincosf(xf, &s, &c);
    return (float)((double)s / (double)c);
}

/* log2 of a positive finite float, in double: x = 2^k z with z in [0.69921875, 1.3984375)
 * (16 sub-intervals by the float's bits), log2 z = logc + log2(1 + r), r = z * invc - 1. */
ORT_HD double ort__log2_d(float xf) {
    ORT_TAB_DECL double tab[32] = ORT_LOG2_TAB_VALUES;
    uint32_t ix;
    __builtin_memcpy(&ix, &xf, 4);
    int ks = 0;
    if (ix < 0x00800000u) { /* subnormal: scale by 2^23 (exact) */
        const float xs = xf * 8388608.0f;
        __builtin_memcpy(&ix, &xs, 4);
        ks = -23;
    }
    const uint32_t tmp = ix - 0x3f330000u;
    const int i = (int)((tmp >> 19) & 15u);
    const uint32_t iz = ix - (tmp & 0xff800000u);
    const int k = (int)((int32_t)tmp >> 23) + ks;
    float zf;
    __builtin_memcpy(&zf, &iz, 4);
    const double r = fma((double)zf, tab[2 * i], -1.0);
    const double a0 = ORT_LOG2_P0, a1 = ORT_LOG2_P1, a2 = ORT_LOG2_P2, a3 = ORT_LOG2_P3, a4 = ORT_LOG2_P4;
    const double p = r * fma(r, fma(r, fma(r, fma(r, a4, a3), a2), a1), a0);
    return ((double)k + tab[2 * i + 1]) + p;
}
/* 2^t as a float, t finite in (-150, 128): 2^(m/32) from the table, 2^r by a polynomial */
ORT_HD float ort__exp2_f(double t) {
    ORT_TAB_DECL double tab[32] = ORT_EXP2_TAB_VALUES;
    const double kd = (t * 32.0 + ORT_RNE_SHIFT) - ORT_RNE_SHIFT;
    const double r = fma(kd, -0.03125, t); /* exact: kd / 32 is exact */
    const int64_t ki = (int64_t)kd;
    const double c0 = ORT_EXP2_P0, c1 = ORT_EXP2_P1, c2 = ORT_EXP2_P2;
    const double p = fma(r, fma(r, fma(r, c2, c1), c0), 1.0);
    const uint64_t sb = ort__d_to_bits(tab[ki & 31]) + ((uint64_t)(ki >> 5) << 52);
    return (float)(ort__bits_to_d(sb) * p);
}
/* GLSL pow(x, y): undefined for x < 0 (we return NaN, as exp2(y*log2(x)) would). */
ORT_HD float ort_powf(float x, float y) {
#if ORT_NATIVE_POW && defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#endif
    if (!(x == x) || !(y == y)) return ort__nanf();
    if (x < 0.0f) return ort__nanf();
    if (y == 0.0f) return 1.0f;
    if (x == 0.0f) return (y > 0.0f) ? 0.0f : ort__inff();
    if (x == ort__inff()) return (y > 0.0f) ? ort__inff() : 0.0f;
    if (x == 1.0f) return 1.0f;
    const double t = (double)y * ort__log2_d(x);
    if (t >= 128.0) return ort__inff();
    if (t <= -150.0) return 0.0f;
    return ort__exp2_f(t);
}

/* ---- the random generator of glsl:89-101 --------------------------------- */
/* state = uint(x*1664525.0 + y*1013904223.0) + 1013904223u ; the GLSL float*uint
 * promotes the uint literal to float (1013904223 -> 1013904192.0f). */
typedef struct ort_rng { float x, y; } ort_rng;
ORT_HD float ort_rand2D(ort_rng* st) {
    const float p0 = st->x * 1664525.0f;
    const float p1 = st->y * 1013904192.0f;
    const float sum = p0 + p1;
    uint32_t s = (uint32_t)sum + 1013904223u;
    s = s ^ (s >> 16);
    s *= 0x85ebca6bu;
    s = s ^ (s >> 13);
    s *= 0xc2b2ae35u;
    s = s ^ (s >> 16);
    st->x = ort_fract(st->y * 1664525.0f);
    st->y = ort_fract((float)s / 4294967296.0f);
    return st->y;
}

#endif /* ORT_MATH_H */
