/* Exactness check of the fp64 NTT arithmetic (fhe-sorting_amd/csrc/device/
 * ntt.hip: fp_mulmod, fp_reduce, fp_in, fp_out) on the host, IEEE binary64
 * with round-to-nearest-even and a correctly rounded fma() -- the same
 * operations v_mul_f64 / v_fma_f64 / v_rndne_f64 / v_add_f64 perform.
 * For primes q < 2^41 and integer operands |y| <= 2^50 (the bounds DESIGN.md
 * §5 derives for the FP passes) it checks, against exact 128-bit integers:
 *   fp_mulmod(y, w) == y w - h q  for the h the code computes, r == y w mod q,
 *   and |r| <= (1/2 + 3 |y| 2^-53) q + 1;
 *   fp_reduce(v) likewise for |v| <= 2^51;
 *   fp_out(fp_in(x, c), c) == x for x < 2^52.
 * usage: fp_mulmod_check <trials> <seed>; prints "ok <n>" or the first failure. */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef unsigned long long u64;
typedef __int128 i128;

static u64 rng_state;
static u64 rnd(void) { /* splitmix64 */
    u64 z = (rng_state += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static int is_prime(u64 n) {
    if (n < 2) return 0;
    for (u64 p = 2; p < 64; ++p)
        if (n % p == 0) return n == p;
    u64 d = n - 1;
    int s = 0;
    while (!(d & 1)) d >>= 1, ++s;
    static const u64 bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    for (int i = 0; i < 12; ++i) {
        u64 a = bases[i] % n, x = 1, b = a, e = d;
        while (e) {
            if (e & 1) x = (u64)((unsigned __int128)x * b % n);
            b = (u64)((unsigned __int128)b * b % n);
            e >>= 1;
        }
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (int r = 1; r < s && comp; ++r) {
            x = (u64)((unsigned __int128)x * x % n);
            if (x == n - 1) comp = 0;
        }
        if (comp) return 0;
    }
    return 1;
}
static double dbits(u64 x) { double d; memcpy(&d, &x, 8); return d; }
static u64 ubits(double d) { u64 x; memcpy(&x, &d, 8); return x; }
static const double TWO52 = 4503599627370496.0;
static const u64 MAGIC = 0x4330000000000000ull;
static double fp_in(u64 x, double c) { return dbits(x | MAGIC) - c; }
static u64 fp_out(double v, double c) { return ubits(v + c) ^ MAGIC; }
/* returns r and the quotient used */
static double fp_mulmod(double y, double w, double q, double qi, double *hq) {
    const double b = y * w;
    const double e = fma(y, w, -b);
    const double h = rint(b * qi);
    *hq = h;
    return fma(-h, q, b) + e;
}
static double fp_reduce(double v, double q, double qi, double *hq) {
    const double h = rint(v * qi);
    *hq = h;
    return fma(-h, q, v);
}
static i128 imod(i128 a, i128 m) { a %= m; return a < 0 ? a + m : a; }

int main(int argc, char **argv) {
    const long trials = argc > 1 ? atol(argv[1]) : 1000000;
    rng_state = argc > 2 ? strtoull(argv[2], 0, 10) : 1;
    long n = 0;
    for (int pi = 0; pi < 24; ++pi) {
        /* primes just below 2^41, near 2^40 (the scaling primes), and smaller */
        const int bits = pi < 8 ? 41 : pi < 16 ? 40 : 30 + pi % 8;
        u64 q = ((1ull << bits) - 1 - (rnd() % (1ull << (bits - 6)))) | 1;
        while (!is_prime(q)) q -= 2;
        const double qd = (double)q, qi = 1.0 / qd;
        for (long t = 0; t < trials / 24; ++t, ++n) {
            /* y: signed integers up to 2^50 in magnitude, with the extremes */
            const int sh = (int)(rnd() % 51);
            i128 y = (i128)(rnd() >> (64 - sh - 1));
            if (t % 7 == 0) y = ((i128)1 << 50) - (i128)(rnd() % 4);
            if (rnd() & 1) y = -y;
            u64 w = rnd() % q;
            if (t % 11 == 0) w = q - 1 - rnd() % 3;
            double h;
            const double r = fp_mulmod((double)y, (double)w, qd, qi, &h);
            const i128 exact = y * (i128)w - (i128)h * (i128)q;
            const double ay = fabs((double)y);
            const double bound = (0.5 + 3.0 * ay * 0x1p-53) * qd + 1.0;
            if ((double)exact != r || (i128)r != exact || fabs(r) > bound || imod((i128)r - y * (i128)w, q) != 0) {
                printf("mulmod FAIL q=%llu y=%lld w=%llu r=%.17g exact=%lld\n", q, (long long)y, w, r, (long long)exact);
                return 1;
            }
            /* reduction of |v| <= 2^51 */
            i128 v = (i128)(rnd() >> 13);
            if (rnd() & 1) v = -v;
            const double rr = fp_reduce((double)v, qd, qi, &h);
            const i128 ex2 = v - (i128)h * (i128)q;
            if ((i128)rr != ex2 || fabs(rr) > (0.5 + 3.0 * fabs((double)v) * 0x1p-53) * qd + 1.0) {
                printf("reduce FAIL q=%llu v=%lld r=%.17g\n", q, (long long)v, rr);
                return 1;
            }
            /* conversions: x < 2^52 through an offset c = 2^52 + k q */
            const u64 x = rnd() >> 12;
            const double c = TWO52 + (double)(rnd() % 10) * qd;
            if (x + (u64)(c - TWO52) < (1ull << 52) && fp_out(fp_in(x, c), c) != x) {
                printf("convert FAIL x=%llu\n", x);
                return 1;
            }
        }
    }
    printf("ok %ld\n", n);
    return 0;
}
