// VALU issue-rate probe for the instructions of the pairwise kernel's inner
// loop (fp64 mul/fma/add, the f64->f32 convert, the 32-bit saturating
// subtract, v_min3_u32).  Each lane runs 8 independent chains of one
// instruction so latency is hidden; the result is cycles per wave-instruction
// per SIMD (4 = a 16-lane SIMD retiring one wave64 op every 4 clocks).
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/probes/valu_rate tools/probes/valu_rate.hip
//   ./tools/probes/valu_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kIters = 4096;

template <int OP>
__global__ __launch_bounds__(256) void valu_kernel(double *out, double seed) {
    double a[8];
    float f[8];
    uint32_t u[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        a[k] = seed + threadIdx.x + k;
        f[k] = (float)a[k];
        u[k] = threadIdx.x * 7u + k;
    }
    const double b = seed * 0.5, c = seed * 0.25;
    for (int it = 0; it < kIters; ++it) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if constexpr (OP == 0) asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(a[k]) : "v"(b), "v"(c));
            if constexpr (OP == 1) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 2) asm volatile("v_mul_f64 %0, %0, %1" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 3) asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[k]) : "v"(a[k]));
            if constexpr (OP == 4) asm volatile("v_sub_u32_e64 %0, %0, %1 clamp" : "+v"(u[k]) : "s"(0x100000u));
            if constexpr (OP == 5) asm volatile("v_min3_u32 %0, %0, %1, %2" : "+v"(u[k]) : "v"(u[(k + 1) & 7]), "v"(u[(k + 2) & 7]));
            if constexpr (OP == 6) asm volatile("v_add_f64 %0, |%0|, |%1|" : "+v"(a[k]) : "v"(b));
            if constexpr (OP == 7) asm volatile("v_add_f32 %0, %0, %1" : "+v"(f[k]) : "v"((float)b));
        }
    }
    double s = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) s += a[k] + f[k] + u[k];
    if (s == 12345.678) out[threadIdx.x] = s;   // keep the chains live
}

template <int OP>
float time_op(double *d, int blocks) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    valu_kernel<OP><<<blocks, 256>>>(d, 1.0001);
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0));
    for (int r = 0; r < 5; ++r) valu_kernel<OP><<<blocks, 256>>>(d, 1.0001);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms / 5;
}

int main() {
    hipDeviceProp_t prop;
    CHECK(hipGetDeviceProperties(&prop, 0));
    const int cus = prop.multiProcessorCount;
    const double clk_hz = prop.clockRate * 1e3;   // kHz -> Hz (peak)
    double *d;
    CHECK(hipMalloc(&d, 4096 * sizeof(double)));
    const int blocks = cus * 8;   // 8 workgroups x 4 waves per CU = 8 waves per SIMD
    const char *names[] = {"v_fma_f64", "v_add_f64", "v_mul_f64", "v_cvt_f32_f64",
                           "v_sub_u32 clamp", "v_min3_u32", "v_add_f64 |a|+|b|", "v_add_f32"};
    float ms[8];
    ms[0] = time_op<0>(d, blocks);
    ms[1] = time_op<1>(d, blocks);
    ms[2] = time_op<2>(d, blocks);
    ms[3] = time_op<3>(d, blocks);
    ms[4] = time_op<4>(d, blocks);
    ms[5] = time_op<5>(d, blocks);
    ms[6] = time_op<6>(d, blocks);
    ms[7] = time_op<7>(d, blocks);
    printf("CUs %d, peak clock %.0f MHz, %d workgroups x 256 threads, %d x 8 ops per lane\n", cus,
           clk_hz / 1e6, blocks, kIters);
    const double wave_instr_per_simd = (double)blocks * 4 / (cus * 4) * kIters * 8;
    for (int k = 0; k < 8; ++k) {
        const double cyc = ms[k] * 1e-3 * clk_hz / wave_instr_per_simd;
        printf("%-20s %8.3f ms  %5.2f clocks per wave64 instruction per SIMD (at peak clock)\n",
               names[k], ms[k], cyc);
    }
    CHECK(hipFree(d));
    return 0;
}
