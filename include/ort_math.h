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

/* ---- sin / cos --------------------------------------------------------- */
/* Cody-Waite reduction by pi/2 in three parts (fdlibm split), then the fdlibm
 * minimax kernels for |r| <= pi/4, all in double.  Accurate to < 1 double ulp for
 * |x| < 2^19; the float result is (almost always) the correctly rounded value.       */
#define ORT_INVPIO2 6.36619772367581382433e-01
#define ORT_PIO2_1  1.57079632673412561417e+00
#define ORT_PIO2_2  6.07710050630396597660e-11
#define ORT_PIO2_3  2.02226624871116645580e-21

ORT_HD double ort__ksin(double r) {
    const double z = r * r;
    const double p = -1.66666666666666324348e-01 + z * (8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 +
                     z * (2.75573137070700676789e-06 + z * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10))));
    return r + (r * z) * p;
}
ORT_HD double ort__kcos(double r) {
    const double z = r * r;
    const double p = 4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * (2.48015872894767294178e-05 +
                     z * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11))));
    return (1.0 - 0.5 * z) + (z * z) * p;
}
/* returns quadrant k (mod 4) and reduced argument r */
ORT_HD int ort__rem_pio2(double x, double* r) {
    const double kd = floor(x * ORT_INVPIO2 + 0.5);
    *r = ((x - kd * ORT_PIO2_1) - kd * ORT_PIO2_2) - kd * ORT_PIO2_3;
    const int64_t k = (int64_t)kd;
    return (int)(k & 3);
}
#if defined(ORT_MEASURE_NATIVE_MATH) && defined(__HIP_DEVICE_COMPILE__)
/* MEASUREMENT ONLY (tools/build_variant.sh ... -DORT_MEASURE_NATIVE_MATH): the hardware
 * v_sin/v_cos/v_log/v_exp in place of the canonical kernels, to price them in A/B.  Changes
 * pixels; never in a product build. */
#define ORT_NATIVE_MATH 1
#endif
ORT_HD float ort_sinf(float xf) {
#ifdef ORT_NATIVE_MATH
    return __builtin_amdgcn_sinf(xf * 0.15915494309189535f);
#endif
    if (!(xf == xf) || xf == ort__inff() || xf == -ort__inff()) return ort__nanf();
    double r; const int q = ort__rem_pio2((double)xf, &r);
    double v;
    switch (q) {
        case 0: v = ort__ksin(r); break;
        case 1: v = ort__kcos(r); break;
        case 2: v = -ort__ksin(r); break;
        default: v = -ort__kcos(r); break;
    }
    return (float)v;
}
ORT_HD float ort_cosf(float xf) {
#ifdef ORT_NATIVE_MATH
    return __builtin_amdgcn_cosf(xf * 0.15915494309189535f);
#endif
    if (!(xf == xf) || xf == ort__inff() || xf == -ort__inff()) return ort__nanf();
    double r; const int q = ort__rem_pio2((double)xf, &r);
    double v;
    switch (q) {
        case 0: v = ort__kcos(r); break;
        case 1: v = -ort__ksin(r); break;
        case 2: v = -ort__kcos(r); break;
        default: v = ort__ksin(r); break;
    }
    return (float)v;
}
/* tan is only used on the host for the camera frustum (glsl:192); same kernels. */
ORT_HD float ort_tanf(float xf) {
    double r; const int q = ort__rem_pio2((double)xf, &r);
    const double s = ort__ksin(r), c = ort__kcos(r);
    return (float)((q & 1) ? (-c / s) : (s / c));
}

/* ---- pow ---------------------------------------------------------------- */
#define ORT_LN2_HI 6.93147180369123816490e-01
#define ORT_LN2_LO 1.90821492927058770002e-10
#define ORT_INVLN2 1.44269504088896338700e+00

/* natural log of a positive, finite, normal-or-subnormal double */
ORT_HD double ort__log_d(double x) {
    uint64_t u = ort__d_to_bits(x);
    int e = (int)((u >> 52) & 0x7ff);
    if (e == 0) { /* subnormal: scale up by 2^54 */
        x = x * 18014398509481984.0;
        u = ort__d_to_bits(x);
        e = (int)((u >> 52) & 0x7ff) - 54;
    }
    e -= 1023;
    double m = ort__bits_to_d((u & 0x000fffffffffffffull) | 0x3ff0000000000000ull); /* [1,2) */
    if (m > 1.41421356237309504880) { m = m * 0.5; e += 1; }
    const double s = (m - 1.0) / (m + 1.0);
    const double z = s * s;
    const double series = 1.0 + z * (1.0 / 3 + z * (1.0 / 5 + z * (1.0 / 7 + z * (1.0 / 9 + z * (1.0 / 11 +
                          z * (1.0 / 13 + z * (1.0 / 15 + z * (1.0 / 17 + z * (1.0 / 19 + z * (1.0 / 21))))))))));
    const double lm = 2.0 * s * series;
    const double ed = (double)e;
    return ed * ORT_LN2_HI + (ed * ORT_LN2_LO + lm);
}
/* e^z for |z| <= 200 (result is then converted to float by the caller) */
ORT_HD double ort__exp_d(double z) {
    const double kd = floor(z * ORT_INVLN2 + 0.5);
    const double r = (z - kd * ORT_LN2_HI) - kd * ORT_LN2_LO;
    const double p = 1.0 + r * (1.0 + r * (1.0 / 2 + r * (1.0 / 6 + r * (1.0 / 24 + r * (1.0 / 120 + r * (1.0 / 720 +
                     r * (1.0 / 5040 + r * (1.0 / 40320 + r * (1.0 / 362880 + r * (1.0 / 3628800 + r * (1.0 / 39916800 +
                     r * (1.0 / 479001600 + r * (1.0 / 6227020800.0)))))))))))));
    const int64_t k = (int64_t)kd;
    /* 2^k as two factors so that k in [-300, 300] never overflows the exponent field */
    const int64_t k1 = k / 2, k2 = k - k1;
    const double s1 = ort__bits_to_d((uint64_t)(k1 + 1023) << 52);
    const double s2 = ort__bits_to_d((uint64_t)(k2 + 1023) << 52);
    return (p * s1) * s2;
}
/* GLSL pow(x, y): undefined for x < 0 (we return NaN, as exp2(y*log2(x)) would). */
ORT_HD float ort_powf(float x, float y) {
#ifdef ORT_NATIVE_MATH
    return __builtin_amdgcn_exp2f(y * __builtin_amdgcn_logf(x));
#endif
    if (!(x == x) || !(y == y)) return ort__nanf();
    if (x < 0.0f) return ort__nanf();
    if (y == 0.0f) return 1.0f;
    if (x == 0.0f) return (y > 0.0f) ? 0.0f : ort__inff();
    if (x == ort__inff()) return (y > 0.0f) ? ort__inff() : 0.0f;
    if (x == 1.0f) return 1.0f;
    const double z = (double)y * ort__log_d((double)x);
    if (z > 89.0) return ort__inff();
    if (z < -110.0) return 0.0f;
    return (float)ort__exp_d(z);
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
