/* math_check.c -- accuracy of the canonical builtins of include/ort_math.h against libm
 * (double sin/cos/pow rounded to float: the correctly rounded float except where the exact
 * value is within a double ulp of a float midpoint).  Sweeps every float of the ranges the
 * shader feeds them (sin/cos: |x| <= 8; pow: x in (0, 4] with y = 1/2.2, 1/3, 5) plus strided
 * samples of the whole finite range, and reports the largest ulp difference and how many
 * results differ from the rounded libm value at all.
 *   gcc -O2 -std=c99 -ffp-contract=off -Iinclude tools/math_check.c -lm -o /tmp/math_check
 *   /tmp/math_check [stride]   (stride 1 = every float in the dense ranges; default 1) */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ort_math.h"

static int64_t ulps(float a, float b) {
    int32_t ia, ib;
    memcpy(&ia, &a, 4);
    memcpy(&ib, &b, 4);
    if (ia < 0) ia = (int32_t)0x80000000 - ia;
    if (ib < 0) ib = (int32_t)0x80000000 - ib;
    return llabs((long long)ia - (long long)ib);
}

typedef struct {
    int64_t n, diff, worst;
    float worst_x;
} Stat;

static void acc(Stat* s, float x, float got, float want) {
    if (isnan(got) && isnan(want)) return;
    const int64_t u = ulps(got, want);
    s->n++;
    if (u) s->diff++;
    if (u > s->worst) {
        s->worst = u;
        s->worst_x = x;
    }
}

static float from_bits(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)atoi(argv[1]) : 1u;
    Stat ss = {0}, sc = {0};
    /* sin/cos: every float in [0, 8] (and the negatives by symmetry of the sweep) */
    for (uint32_t u = 0; u <= 0x41000000u; u += stride) {
        for (int sg = 0; sg < 2; ++sg) {
            const float x = from_bits(u | (sg ? 0x80000000u : 0u));
            float s, c;
            ort_sincosf(x, &s, &c);
            acc(&ss, x, s, (float)sin((double)x));
            acc(&sc, x, c, (float)cos((double)x));
        }
    }
    /* and a strided sample up to 2^24 */
    for (uint32_t u = 0x41000000u; u <= 0x4b800000u; u += 4099u) {
        const float x = from_bits(u);
        float s, c;
        ort_sincosf(x, &s, &c);
        acc(&ss, x, s, (float)sin((double)x));
        acc(&sc, x, c, (float)cos((double)x));
    }
    printf("sin: %lld args, %lld differ from rounded libm, worst %lld ulp at %a\n", (long long)ss.n,
           (long long)ss.diff, (long long)ss.worst, ss.worst_x);
    printf("cos: %lld args, %lld differ from rounded libm, worst %lld ulp at %a\n", (long long)sc.n,
           (long long)sc.diff, (long long)sc.worst, sc.worst_x);
    const float ys[] = {1.0f / 2.2f, 1.0f / 3.0f, 5.0f, 2.5f, -0.75f};
    int bad = ss.worst > 1 || sc.worst > 1;
    for (int j = 0; j < 5; ++j) {
        Stat sp = {0};
        const float y = ys[j];
        /* every float in (0, 4] (subnormals included), and strided beyond */
        for (uint32_t u = 1; u <= 0x40800000u; u += stride) {
            const float x = from_bits(u);
            acc(&sp, x, ort_powf(x, y), (float)pow((double)x, (double)y));
        }
        for (uint32_t u = 0x40800000u; u < 0x7f800000u; u += 8191u) {
            const float x = from_bits(u);
            acc(&sp, x, ort_powf(x, y), (float)pow((double)x, (double)y));
        }
        printf("pow(x, %a): %lld args, %lld differ from rounded libm, worst %lld ulp at x=%a\n", y, (long long)sp.n,
               (long long)sp.diff, (long long)sp.worst, sp.worst_x);
        bad |= sp.worst > 1;
    }
    printf(bad ? "FAIL: some result is more than 1 ulp off\n" : "OK: every result within 1 ulp\n");
    return bad;
}
