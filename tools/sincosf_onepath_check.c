// Host-side check that glibc_sincosf (csrc/common.hpp) in its one-path form equals the
// two-branch form it replaced, for every float |y| < 120:  gcc -O2 -fopenmp -ffp-contract=off
// tools/sincosf_onepath_check.c -o /tmp/chk && /tmp/chk  (test infrastructure only)
#include <stdio.h>
#include <stdint.h>
#include <string.h>
#include <math.h>
static inline uint32_t fu(float f){uint32_t u;memcpy(&u,&f,4);return u;}
static inline float uf(uint32_t u){float f;memcpy(&f,&u,4);return f;}
static float poly(double x, double x2, int cos_branch, int neg_cos) {
    if (!cos_branch) {
        const double x3 = x * x2;
        const double s1 = 0x1.1107605230bc4p-7 + x2 * -0x1.994eb3774cf24p-13;
        const double x7 = x3 * x2;
        const double s = x + x3 * -0x1.555545995a603p-3;
        return (float)(s + x7 * s1);
    }
    const double g = neg_cos ? -1.0 : 1.0;
    const double x4 = x2 * x2;
    const double c2 = g * -0x1.6c087e89a359dp-10 + x2 * (g * 0x1.99343027bf8c3p-16);
    const double c1 = g * 0x1p0 + x2 * (g * -0x1.ffffffd0c621cp-2);
    const double x6 = x4 * x2;
    const double c = c1 + x4 * (g * 0x1.55553e1068f19p-5);
    return (float)(c + x6 * c2);
}
static void old_sc(float y, float *sv, float *cv) {
    const uint32_t top = (fu(y) >> 20) & 0x7ffu;
    double x = y;
    if (top < ((fu((float)0x1.921FB54442D18p-1) >> 20) & 0x7ffu)) {
        if (top < ((fu(0x1p-12f) >> 20) & 0x7ffu)) { *sv = y; *cv = 1.0f; return; }
        const double x2 = x * x;
        *sv = poly(x, x2, 0, 0); *cv = poly(x, x2, 1, 0); return;
    }
    const double r = x * 0x1.45F306DC9C883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * 0x1.921FB54442D18p0;
    const double s = ((n + 1) & 2) ? -1.0 : 1.0;
    const int neg = (n & 2) != 0;
    const double xs = x * s, x2 = x * x;
    *sv = poly(xs, x2, (n & 1) != 0, neg);
    *cv = poly(xs, x2, (n & 1) == 0, neg);
}
static void new_sc(float y, float *sv, float *cv) {
    const uint32_t top = (fu(y) >> 20) & 0x7ffu;
    double x = y;
    if (top < ((fu(0x1p-12f) >> 20) & 0x7ffu)) { *sv = y; *cv = 1.0f; return; }
    const double r = x * 0x1.45F306DC9C883p+23;
    const int n = ((int32_t)r + 0x800000) >> 24;
    x = x - n * 0x1.921FB54442D18p0;
    const double x2 = x * x;
    const float sp = poly(x, x2, 0, 0), cp = poly(x, x2, 1, 0);
    const float ss = ((n + 1) & 2) ? -sp : sp;
    const float cs = (n & 2) ? -cp : cp;
    *sv = (n & 1) ? cs : ss;
    *cv = (n & 1) ? ss : cs;
}
int main(void) {
    const uint32_t hi = fu(120.0f);
    long bad = 0;
    #pragma omp parallel for reduction(+:bad) schedule(static)
    for (long i = 0; i < (long)hi; i++) {
        for (int sg = 0; sg < 2; sg++) {
            float y = uf((uint32_t)i | (sg ? 0x80000000u : 0u)), s0, c0, s1, c1;
            old_sc(y, &s0, &c0); new_sc(y, &s1, &c1);
            if (fu(s0) != fu(s1) || fu(c0) != fu(c1)) { if (bad < 5) printf("diff %a: %a %a vs %a %a\n", y, s0, c0, s1, c1); bad++; }
        }
    }
    printf("checked all |y| < 120: %ld differences\n", bad);
    return bad != 0;
}
