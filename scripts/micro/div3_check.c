/* Host check of the division-free mean used by the V-cycle kernels (pamg_device.h div3):
 *   q0 = RN(x * t), t = RN(1/3); r = fma(-3, q0, x) (exact); q = fma(r, t, q0)
 * equals RN(x / 3) (Markstein's theorem: q0 within 1 ulp of x/3, t the correctly rounded
 * reciprocal, no under/overflow) -- the kernels take it for 2^-1000 <= |x| <= 2^1000 and
 * divide otherwise (zeros, subnormals, huge values, inf, NaN). This program compares the two
 * bit for bit on random doubles of every exponent in that range and on structured values.
 * Build: gcc -O2 -mfma -ffp-contract=off -fopenmp div3_check.c -lm -o div3_check */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

static double div3_fast(double x) {
    const double t = 1.0 / 3.0;
    const double q0 = x * t;
    const double r = fma(-3.0, q0, x);
    return fma(r, t, q0);
}

static uint64_t bits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

int main(int argc, char **argv) {
    const long n = argc > 1 ? atol(argv[1]) : 1000000000L;
    long bad = 0, tested = 0;
#pragma omp parallel for reduction(+ : bad, tested) schedule(static)
    for (long k = 0; k < n; ++k) {
        uint64_t z = (uint64_t)k * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull;   /* splitmix64 */
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        z ^= z >> 31;
        /* exponent uniform in [-1000, 1000], random mantissa and sign */
        const int e = (int)((z >> 52) % 2001) - 1000;
        const uint64_t u = (z & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(e + 1023) << 52);
        double x;
        memcpy(&x, &u, 8);
        ++tested;
        if (bits(div3_fast(x)) != bits(x / 3.0)) {
            ++bad;
            if (bad < 5) printf("mismatch x=%a fast=%a div=%a\n", x, div3_fast(x), x / 3.0);
        }
    }
    /* structured: multiples of 3 and their neighbours, powers of two and their neighbours */
    for (long m = 1; m < 20000000; ++m) {
        const double xs[4] = {3.0 * (double)m, nextafter(3.0 * (double)m, 0.0), nextafter(3.0 * (double)m, INFINITY),
                              ldexp(1.0, (int)(m % 2000) - 1000)};
        for (int i = 0; i < 4; ++i)
            for (int sgn = 0; sgn < 2; ++sgn) {
                const double x = sgn ? -xs[i] : xs[i];
                ++tested;
                if (bits(div3_fast(x)) != bits(x / 3.0)) {
                    ++bad;
                    if (bad < 10) printf("mismatch x=%a fast=%a div=%a\n", x, div3_fast(x), x / 3.0);
                }
            }
    }
    printf("div3: %ld values, %ld mismatches\n", tested, bad);
    return bad != 0;
}
