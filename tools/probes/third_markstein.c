/* Validation of the cube's division by 3 (test tool, not product code).
 *
 * The cube needs f32(RN64(s / 3)) for finite s >= 0 (epipolar_matching.py:81,
 * :96).  The kernels compute q0 = RN(s * y), y = RN(1/3), and one Markstein
 * correction r = fma(-q0, 3, s) (exact), q1 = fma(r, y, q0).  Markstein's
 * theorem (y the correctly rounded reciprocal, q0 within one ulp of s/3) makes
 * q1 = RN(s / 3).  This program checks it against the IEEE division on
 * random doubles over the whole positive range, on every binade's edges, and
 * on adversarial inputs whose quotient lies next to a rounding midpoint.
 *
 *   gcc -O2 -mfma -ffp-contract=off -o /tmp/third_markstein tools/probes/third_markstein.c -lm
 *   /tmp/third_markstein 200000000
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t bits(double x) { uint64_t u; memcpy(&u, &x, 8); return u; }
static double from(uint64_t u) { double x; memcpy(&x, &u, 8); return x; }

static uint64_t rng_state = 0x9E3779B97F4A7C15ull;
static uint64_t next_u64(void) {   /* splitmix64 */
    uint64_t z = (rng_state += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static const double kThird = 1.0 / 3.0;
static long long checked = 0, bad = 0, corrected = 0;   /* corrected: q0 != RN(s/3) */

static void check(double s) {
    if (!(s >= 0.0) || isinf(s)) return;
    const double ref = s / 3.0;
    const double q0 = s * kThird;
    const double r = fma(-q0, 3.0, s);
    const double q1 = fma(r, kThird, q0);
    ++checked;
    corrected += bits(q0) != bits(ref);
    if (bits(q1) != bits(ref) || bits((double)(float)q1) != bits((double)(float)ref)) {
        if (bad < 10) printf("MISMATCH s=%a ref=%a q1=%a\n", s, ref, q1);
        ++bad;
    }
}

int main(int argc, char **argv) {
    const long long n = argc > 1 ? atoll(argv[1]) : 100000000LL;
    /* 1. uniformly random bit patterns (every binade, subnormals included) */
    for (long long i = 0; i < n; ++i) check(from(next_u64() >> 1));
    /* 2. random values in the residual range [0, 2^16) */
    for (long long i = 0; i < n; ++i) check(ldexp((double)(next_u64() >> 11), -53 + (int)(next_u64() % 70) - 50));
    /* 3. binade edges and small integers */
    for (int e = -1074; e <= 1023; ++e)
        for (int d = -8; d <= 8; ++d) check(from(bits(ldexp(1.0, e)) + (uint64_t)(int64_t)d));
    for (int k = 0; k < 1 << 20; ++k) { check((double)k); check(k * 0.5); check(k * 0.25); }
    /* 4. adversarial: s next to 3 * (midpoint of two consecutive doubles q, q+ulp) */
    for (long long i = 0; i < n; ++i) {
        const int e = (int)(next_u64() % 2000) - 1000;
        const uint64_t k = (1ull << 52) | (next_u64() & ((1ull << 52) - 1));
        const double q = ldexp((double)k, e - 52);
        const double mid = q + ldexp(0.5, e - 52);     /* not representable: q and mid ~ 2^-53 */
        /* s = the doubles around 3 * mid (rounded), +-4 ulps */
        const double s0 = 3.0 * q + ldexp(1.5, e - 52);
        for (int d = -4; d <= 4; ++d) check(from(bits(s0) + (uint64_t)(int64_t)d));
        (void)mid;
    }
    printf("checked %lld values (%lld where q0 != RN(s/3)), %lld mismatches\n", checked, corrected, bad);
    return bad != 0;
}
