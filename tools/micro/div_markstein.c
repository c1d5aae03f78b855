/* x / b through b's reciprocal (Markstein's sequence, as the ARAP energy's adiv in csrc/kernels.hip):
 *   y = RN(1/b), q0 = RN(x y), res = x - q0 b (exact by FMA), q = res == 0 ? q0 : RN(q0 + res y)
 * against IEEE division on random operands (random exponents within +-100, random mantissas, a
 * quarter of the divisors near the ARAP pair areas, some with an all-ones mantissa) and on the
 * signed-zero / exact-quotient cases.  Prints "bad <mismatches> of <trials>".
 * build: gcc -O2 -ffp-contract=off div_markstein.c -lm; run: ./a.out <divisors> */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double rnd(void) {
    const uint64_t m = xr() & ((1ull << 52) - 1);
    const int e = (int)(xr() % 200) - 100 + 1023;
    const uint64_t b = ((xr() & 1) << 63) | ((uint64_t)e << 52) | m;
    double d;
    memcpy(&d, &b, 8);
    return d;
}
static double adiv(double x, double b, double y) {
    const double q0 = x * y;
    const double res = fma(-q0, b, x);
    return res == 0.0 ? q0 : fma(res, y, q0);
}
static int same(double a, double b) { return memcmp(&a, &b, 8) == 0; }

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000;
    long bad = 0, trials = 0;
    for (long i = 0; i < n; i++) {
        double b = (i % 4 == 0) ? 0.5 * (1.0 + (double)(xr() % 1000000) / 1e6) : rnd();
        if (i % 1000 == 1) { uint64_t bb; memcpy(&bb, &b, 8); bb |= (1ull << 52) - 1; memcpy(&b, &bb, 8); }
        const double y = 1.0 / b;
        double xs[12];
        for (int k = 0; k < 8; k++) xs[k] = rnd();
        xs[8] = 0.0; xs[9] = -0.0; xs[10] = 3.0 * b; xs[11] = -0.5 * b;   /* zeros, exact quotients */
        for (int k = 0; k < 12; k++) {
            trials++;
            if (!same(adiv(xs[k], b, y), xs[k] / b)) {
                if (bad < 10) printf("mismatch x=%a b=%a\n", xs[k], b);
                bad++;
            }
        }
    }
    printf("bad %ld of %ld\n", bad, trials);
    return bad != 0;
}
