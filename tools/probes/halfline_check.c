/* Would pre-scaling the lines by 0.5 reproduce the pairwise kernel's float32
 * residuals?  (Test tool for a proposed change, not product code.)
 *
 * Kernel today:  d1 = |fma(c1, ry, c0*rx) + c2|, d2 = |fma(r1, cy, r0*cx) + r2|,
 *                v = f32(half(d1 + d2)) with half = exponent decrement (exact
 *                after the f32 cast, tests/test_host_logic.py).
 * Proposal:      the same with every line component multiplied by 0.5 first,
 *                v' = f32(d1' + d2').  Variant B halves the column's line and
 *                point and only the row line's constant term.
 * Inputs: normalised lines (random angles, some near an axis so one component
 * is tiny or subnormal), l2 and points over many magnitudes within the fast
 * path's tame bounds (|x|,|y| <= 2^40, |l2| <= 2^60), zeros.
 *
 *   gcc -O2 -ffp-contract=off -o /tmp/halfline tools/probes/halfline_check.c -lm && /tmp/halfline 20000000
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s_ = 0x853C49E6748FEA9Bull;
static uint64_t nx(void) {
    uint64_t z = (s_ += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double u01(void) { return (double)(nx() >> 11) * 0x1p-53; }

static double half_bits(double s) {   /* the kernel's half_for_f32 */
    uint64_t b; memcpy(&b, &s, 8);
    uint32_t hi = (uint32_t)(b >> 32);
    hi = hi >= 0x00100000u ? hi - 0x00100000u : 0u;
    b = ((uint64_t)hi << 32) | (uint32_t)b;
    double r; memcpy(&r, &b, 8); return r;
}

static double coord(void) {
    switch (nx() % 6) {
    case 0: return 0.0;
    case 1: return floor(u01() * 8000.0) * 0.5;                       /* detector half-integers */
    case 2: return ldexp(u01(), (int)(nx() % 40));                    /* up to 2^40 */
    case 3: return ldexp(u01(), -(int)(nx() % 1074));                 /* tiny, subnormal */
    case 4: return -ldexp(u01(), (int)(nx() % 40));
    default: return u01() * 4000.0;
    }
}

static void line(double l[3]) {
    const int mode = (int)(nx() % 4);
    double a;
    if (mode == 0) a = u01() * 6.283185307179586;
    else a = ldexp(u01(), -(int)(nx() % 1100)) * ((nx() & 1) ? 1 : -1);   /* near an axis */
    const double c = cos(a), s = sin(a);
    l[0] = (mode == 2) ? s : c;
    l[1] = (mode == 2) ? c : s;
    switch (nx() % 4) {
    case 0: l[2] = 0.0; break;
    case 1: l[2] = ldexp(u01() - 0.5, (int)(nx() % 60)); break;
    case 2: l[2] = ldexp(u01() - 0.5, -(int)(nx() % 1074)); break;
    default: l[2] = (u01() - 0.5) * 8000.0;
    }
}

int main(int argc, char **argv) {
    const long long n = argc > 1 ? atoll(argv[1]) : 10000000LL;
    long long bad = 0, badb = 0;
    for (long long i = 0; i < n; ++i) {
        double c[3], r[3];
        line(c);
        line(r);
        const double rx = coord(), ry = coord(), cx = coord(), cy = coord();
        const double d1 = fabs(fma(c[1], ry, c[0] * rx) + c[2]);
        const double d2 = fabs(fma(r[1], cy, r[0] * cx) + r[2]);
        const float v = (float)half_bits(d1 + d2);
        double hc[3], hr[3];
        for (int k = 0; k < 3; ++k) { hc[k] = 0.5 * c[k]; hr[k] = 0.5 * r[k]; }
        const double e1 = fabs(fma(hc[1], ry, hc[0] * rx) + hc[2]);
        const double e2 = fabs(fma(hr[1], cy, hr[0] * cx) + hr[2]);
        const float w = (float)(e1 + e2);
        /* variant B: halve the column's line AND point, and the row line's l2 only */
        const double hcx = 0.5 * cx, hcy = 0.5 * cy, hr2 = 0.5 * r[2];
        const double g1 = fabs(fma(hc[1], ry, hc[0] * rx) + hc[2]);
        const double g2 = fabs(fma(r[1], hcy, r[0] * hcx) + hr2);
        const float wb = (float)(g1 + g2);
        uint32_t a, b, bb; memcpy(&a, &v, 4); memcpy(&b, &w, 4); memcpy(&bb, &wb, 4);
        if (a != bb) {
            if (badb < 8) printf("MISMATCH(B) c=(%a,%a,%a) r=(%a,%a,%a) p=(%a,%a) q=(%a,%a): %a vs %a\n",
                                 c[0], c[1], c[2], r[0], r[1], r[2], rx, ry, cx, cy, v, wb);
            ++badb;
        }
        if (a != b) {
            if (bad < 8) printf("MISMATCH c=(%a,%a,%a) r=(%a,%a,%a) p=(%a,%a) q=(%a,%a): %a vs %a\n",
                                c[0], c[1], c[2], r[0], r[1], r[2], rx, ry, cx, cy, v, w);
            ++bad;
        }
    }
    printf("checked %lld pairs, %lld float32 mismatches (half lines), %lld (variant B: half column, half row l2)\n", n, bad, badb);
    return bad != 0 || badb != 0;
}
