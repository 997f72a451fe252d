// Does `v_add_f64 d, |a|, |b| div:2` (VOP3 output modifier) give the float32
// value of 0.5 * (|a| + |b|) on gfx950, with fp64 denormals enabled?  Compares
// float32 bit patterns against the reference expression on random doubles over
// every binade, subnormals and binade edges.  Test tool, not product code.
//
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/probes/omod_half tools/probes/omod_half.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

__global__ void omod_kernel(const double *a, const double *b, unsigned *bad, unsigned *first, size_t n) {
    const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    if (i >= n) return;
    double h;
    asm volatile("v_add_f64 %0, |%1|, |%2| div:2" : "=v"(h) : "v"(a[i]), "v"(b[i]));
    const float got = (float)h;
    const float want = (float)(0.5 * (fabs(a[i]) + fabs(b[i])));
    unsigned g, w;
    memcpy(&g, &got, 4);
    memcpy(&w, &want, 4);
    if (g != w) {
        atomicAdd(bad, 1u);
        atomicMin(first, (unsigned)i);
    }
}

static unsigned long long st = 0x243F6A8885A308D3ull;
static unsigned long long nxt() {
    unsigned long long z = (st += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
static double from(unsigned long long u) { double x; memcpy(&x, &u, 8); return x; }

int main() {
    const size_t n = 1 << 24;
    double *ha = (double *)malloc(n * 8), *hb = (double *)malloc(n * 8);
    size_t k = 0;
    for (int e = -1074; e <= 1023 && k + 64 < n; ++e)   // binade edges, both operands
        for (int d = -4; d <= 4; ++d) {
            ha[k] = ldexp(1.0, e); hb[k++] = from(*(unsigned long long *)&ha[k - 1] + d);
            ha[k] = ldexp(1.0, e) * (d & 1 ? -1 : 1); hb[k++] = 0.0;
        }
    for (; k < n / 2; ++k) {                              // random bit patterns (finite)
        do { ha[k] = from(nxt()); } while (!std::isfinite(ha[k]));
        do { hb[k] = from(nxt()); } while (!std::isfinite(hb[k]));
        if (std::isinf(fabs(ha[k]) + fabs(hb[k]))) { ha[k] = 1.0; hb[k] = 2.0; }
    }
    for (; k < n; ++k) {                                  // the residual range, and tiny ones
        const int e = (int)(nxt() % 1200) - 1100;
        ha[k] = ldexp((double)(nxt() >> 11), e - 53) * ((nxt() & 1) ? 1 : -1);
        hb[k] = ldexp((double)(nxt() >> 11), e - 53 + (int)(nxt() % 8));
    }
    double *da, *db;
    unsigned *dbad, *dfirst, hbad = 0, hfirst = 0xFFFFFFFFu;
    CHECK(hipMalloc(&da, n * 8));
    CHECK(hipMalloc(&db, n * 8));
    CHECK(hipMalloc(&dbad, 4));
    CHECK(hipMalloc(&dfirst, 4));
    CHECK(hipMemcpy(da, ha, n * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(db, hb, n * 8, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dbad, &hbad, 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dfirst, &hfirst, 4, hipMemcpyHostToDevice));
    omod_kernel<<<(unsigned)((n + 255) / 256), 256>>>(da, db, dbad, dfirst, n);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(&hbad, dbad, 4, hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(&hfirst, dfirst, 4, hipMemcpyDeviceToHost));
    printf("checked %zu pairs, %u float32 mismatches", n, hbad);
    if (hbad) printf(" (first at %u: a=%a b=%a)", hfirst, ha[hfirst], hb[hfirst]);
    printf("\n");
    return hbad != 0;
}
