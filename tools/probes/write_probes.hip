// write_probes.hip — the HBM store-stream patterns studied in DESIGN.md §3.5
// (block sizes, cache policies, XCD-sequential order, the pairwise kernel's
// own row order and shape models).  A standalone experiment, not part of
// libmvmatch.so: the library keeps only the fastest pattern (mode 17) as
// mvm_hbm_write_probe.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../include \
//         -I../../bpc_baseline_amd/csrc -o write_probes write_probes.hip
//   ./write_probes mode=17 mib=4096 [grid=N lds=BYTES rpw=16 rg=4 pace=0]
//
// Modes: 0 nt 16 KiB/WG, 1 plain 16 KiB/WG, 2 nt 64 KiB/WG, 3 plain 64 KiB/WG,
// 4 nt grid-stride, 5 plain grid-stride, 6 sc1, 7 sc0 sc1, 8 nt sc1 (16 KiB/WG),
// 9 / 10 the pairwise kernel's row order (chunk-outer / row-major) on 256 KiB
// per WG, 11 XCD-sequential nt 16 KiB, 12 rows order XCD-sequential, 13 plain
// XCD-sequential, 14 XCD-sequential scrambled, 15 / 16 XCD-sequential 32 /
// 64 KiB, 17 XCD-sequential 8 KiB (the library's probe), 18 16-row-unit model
// (lines read from L2), 20 / 21 store-shape models of the pairwise kernel.
#include <hip/hip_runtime.h>

#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "mvm_device.h"

static int g_argc;
static char **g_argv;
static int arg(const char *key, int dflt) {
    const size_t n = strlen(key);
    for (int i = 1; i < g_argc; ++i)
        if (!strncmp(g_argv[i], key, n) && g_argv[i][n] == '=') return atoi(g_argv[i] + n + 1);
    return dflt;
}

namespace {
// ------------------------------------------------------- write probe ----
// Speed-of-light reference for the roofline: every workgroup writes one
// contiguous 16 KiB block with 16-byte nontemporal stores (4 per lane, each
// wave instruction 1 KiB contiguous) -- the store form of the residual kernels.
template <int PER_LANE, bool NT, bool XCD = false, bool SCRAMBLE = false>
__global__ __launch_bounds__(kThreads) void write_probe_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    uint32_t blk = blockIdx.x;
    if (XCD) {                  // each XCD writes a contiguous eighth
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        uint32_t k = blk / 8;
        const uint32_t cnt = q + (x < r ? 1u : 0u);
        if (SCRAMBLE) k = (uint32_t)(((uint64_t)k * 2654435761ull) % cnt);   // odd multiplier:
        blk = x * q + min(x, r) + k;                                         // a permutation when gcd = 1
    }
    const size_t base = (size_t)blk * (PER_LANE * kThreads) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < PER_LANE; ++k) {
        const size_t i = base + (size_t)k * kThreads;
        if (i < n16) {
            if (NT) __builtin_nontemporal_store(v, dst + i);
            else dst[i] = v;
        }
    }
}

// cache-policy variants of the 16 KiB/WG stream (inline asm: the builtins
// expose only nt); POL 1 = sc1, 2 = sc0 sc1, 3 = nt sc1
template <int POL>
__global__ __launch_bounds__(kThreads) void write_probe_pol_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    const size_t base = (size_t)blockIdx.x * (4 * kThreads) + threadIdx.x;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const size_t i = base + (size_t)k * kThreads;
        if (i < n16) {
            const uint64_t ptr = reinterpret_cast<uint64_t>(dst + i);
            if (POL == 1) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(ptr), "v"(v) : "memory");
            if (POL == 2) asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(ptr), "v"(v) : "memory");
            if (POL == 3) asm volatile("global_store_dwordx4 %0, %1, off nt sc1" ::"v"(ptr), "v"(v) : "memory");
        }
    }
}

// the pairwise kernel's store ORDER on a 256 KiB block per workgroup: 64 rows
// of 4 KiB, wave w owns rows 16w..16w+15 and walks chunk-outer / row-inner
// (consecutive stores of a wave are 4 KiB apart); ROWMAJOR = 1 walks each
// row's 4 chunks first (consecutive stores contiguous)
template <bool ROWMAJOR, bool XCD = false>
__global__ __launch_bounds__(kThreads) void write_probe_rows_kernel(f32x4 *dst, size_t n16, float val) {
    const f32x4 v = {val, val, val, val};
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    uint32_t blk = blockIdx.x;
    if (XCD) {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const size_t base = (size_t)blk * (64 * 256);         // 16-byte units: 64 rows x 256
    for (int a = 0; a < 16; ++a) {
        for (int b = 0; b < 4; ++b) {
            const int row = wave * 16 + (ROWMAJOR ? a : (a % 4) * 4 + b) ;
            const int chunk = ROWMAJOR ? b : a / 4;
            const size_t i = base + (size_t)row * 256 + chunk * 64 + lane;
            if (i < n16) __builtin_nontemporal_store(v, dst + i);
        }
    }
}

// store-shape model of a residual kernel: workgroups own `rpw * rg` (OWN 1)
// or `4 * rpw * rg` (OWN 0) rows of 4 KiB, XCD-sequential; OWN 0: wave w owns
// rpw rows of each group and walks chunk-outer / row-inner (the pairwise
// kernel, rpw rows open per wave); OWN 1: wave w owns 1-KiB chunk w of every
// row of the group (the workgroup's 4 waves share rpw open rows)
// `pace` s_sleep(1) (~64 clocks) after each store stands in for the residual
// arithmetic between a real kernel's stores
template <int OWN>
__global__ __launch_bounds__(kThreads) void write_probe_shape_kernel(f32x4 *dst, size_t n16,
                                                                     int rpw, int rg, int pace,
                                                                     float val) {
    const f32x4 v = {val, val, val, val};
    const int wave = threadIdx.x / kWave, lane = threadIdx.x % kWave;
    uint32_t blk = blockIdx.x;
    {
        const uint32_t nb = gridDim.x, q = nb / 8, r = nb % 8, x = blk % 8;
        blk = x * q + min(x, r) + blk / 8;
    }
    const int rows_wg = (OWN == 0 ? 4 : 1) * rpw * rg;
    const size_t base = (size_t)blk * rows_wg * 256;       // 16-byte units, 256 per row
    for (int g = 0; g < rg; ++g) {
        if (OWN == 0) {
            const int r0 = g * 4 * rpw + wave * rpw;
            for (int c = 0; c < 4; ++c)
                for (int r = 0; r < rpw; ++r) {
                    const size_t i = base + (size_t)(r0 + r) * 256 + c * 64 + lane;
                    if (i < n16) __builtin_nontemporal_store(v, dst + i);
                    for (int z = 0; z < pace; ++z) __builtin_amdgcn_s_sleep(1);
                }
        } else {
            const int r0 = g * rpw;
            for (int r = 0; r < rpw; ++r) {
                const size_t i = base + (size_t)(r0 + r) * 256 + wave * 64 + lane;
                if (i < n16) __builtin_nontemporal_store(v, dst + i);
                for (int z = 0; z < pace; ++z) __builtin_amdgcn_s_sleep(1);
            }
        }
    }
}

// model of a "16-row unit" decomposition: a persistent grid, workgroup k of
// XCD x walks units k, k+W, ... of that XCD's eighth; per unit it reads a
// 44 KiB line block (from a 4 MiB L2-resident region) and writes 64 KiB
// (16 rows of 4 KiB, 4 waves x 4 rows)
__global__ __launch_bounds__(kThreads) void write_probe_units_kernel(f32x4 *dst, size_t n16,
                                                                     const f32x4 *lines) {
    const uint32_t W = gridDim.x / 8, x = blockIdx.x % 8, k = blockIdx.x / 8;
    const size_t n_units = n16 / 4096;                        // 64 KiB = 4096 x 16 B
    const size_t u0 = n_units * x / 8, u1 = n_units * (x + 1) / 8;
    const int t = threadIdx.x;
    for (size_t u = u0 + k; u < u1; u += W) {
        const f32x4 *lb = lines + (u % 90) * 2816;            // 44 KiB = 2816 x 16 B
        f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int q = 0; q < 11; ++q) acc += lb[t + 256 * q];
        f32x4 *ob = dst + u * 4096;
#pragma unroll
        for (int q = 0; q < 16; ++q) __builtin_nontemporal_store(acc, ob + t + 256 * q);
    }
}

// grid-stride variant: a fixed grid of `waves per CU` x 256 CUs workgroups
template <bool NT>
__global__ __launch_bounds__(kThreads) void write_probe_stride_kernel(f32x4 *dst, size_t n16,
                                                                      float val) {
    const f32x4 v = {val, val, val, val};
    const size_t step = (size_t)gridDim.x * kThreads * 4;
    for (size_t b = (size_t)blockIdx.x * kThreads * 4 + threadIdx.x; b < n16; b += step) {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const size_t i = b + (size_t)k * kThreads;
            if (i < n16) {
                if (NT) __builtin_nontemporal_store(v, dst + i);
                else dst[i] = v;
            }
        }
    }
}

int launch(int mode, f32x4 *d, size_t n16, hipStream_t s) {
    const int per = (mode == 2 || mode == 3) ? 16 : 4;
    const size_t blocks = (n16 + per * kThreads - 1) / (per * kThreads);
    const unsigned stride_grid = (unsigned)arg("grid", 256 * 8);
    const size_t plds = (size_t)arg("lds", 0);   // unused LDS per WG: caps resident WGs per CU
    switch (mode) {
        case 1: write_probe_kernel<4, false><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 2: write_probe_kernel<16, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 3: write_probe_kernel<16, false><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 4: write_probe_stride_kernel<true><<<stride_grid, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 5: write_probe_stride_kernel<false><<<stride_grid, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 6: write_probe_pol_kernel<1><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 7: write_probe_pol_kernel<2><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 8: write_probe_pol_kernel<3><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 11: write_probe_kernel<4, true, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 12: write_probe_rows_kernel<false, true><<<(unsigned)((n16 + 16383) / 16384), kThreads, plds, s>>>(d, n16, 1.0f); break;
        case 13: write_probe_kernel<4, false, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 14: write_probe_kernel<4, true, true, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 15: write_probe_kernel<8, true, true><<<(unsigned)((n16 + 8 * kThreads - 1) / (8 * kThreads)), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 16: write_probe_kernel<16, true, true><<<(unsigned)((n16 + 16 * kThreads - 1) / (16 * kThreads)), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 17: write_probe_kernel<2, true, true><<<(unsigned)((n16 + 2 * kThreads - 1) / (2 * kThreads)), kThreads, plds, s>>>(d, n16, 1.0f); break;
        case 18: {
            // lines region: the last 4 MiB of the buffer (units stop before it)
            const size_t reserve = (4u << 20) / 16;
            if (n16 <= reserve + 4096) { fprintf(stderr, "buffer too small\n"); return 1; };
            const unsigned grid = (unsigned)arg("grid", 8 * 96);
            write_probe_units_kernel<<<grid, kThreads, 0, s>>>(d, n16 - reserve, d + (n16 - reserve));
            break;
        }
        case 20:
        case 21: {
            const int rpw = arg("rpw", 16), rg = arg("rg", 4);
            const int pace = arg("pace", 0);
            const size_t rows_wg = (size_t)(mode == 20 ? 4 : 1) * rpw * rg;
            const unsigned g = (unsigned)((n16 + rows_wg * 256 - 1) / (rows_wg * 256));
            if (mode == 20) write_probe_shape_kernel<0><<<g, kThreads, plds, s>>>(d, n16, rpw, rg, pace, 1.0f);
            else write_probe_shape_kernel<1><<<g, kThreads, plds, s>>>(d, n16, rpw, rg, pace, 1.0f);
            break;
        }
        case 9: write_probe_rows_kernel<false><<<(unsigned)((n16 + 16383) / 16384), kThreads, 0, s>>>(d, n16, 1.0f); break;
        case 10: write_probe_rows_kernel<true><<<(unsigned)((n16 + 16383) / 16384), kThreads, 0, s>>>(d, n16, 1.0f); break;
        default: write_probe_kernel<4, true><<<(unsigned)blocks, kThreads, 0, s>>>(d, n16, 1.0f); break;
    }
    return hipGetLastError() == hipSuccess ? 0 : 1;
}
}  // namespace

int main(int argc, char **argv) {
    g_argc = argc;
    g_argv = argv;
    const int mode = arg("mode", 17);
    const size_t bytes = (size_t)arg("mib", 4096) << 20;
    f32x4 *d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    if (launch(mode, d, bytes / 16, nullptr)) return 1;   // warm-up
    const int reps = 5;
    (void)hipEventRecord(e0, nullptr);
    for (int r = 0; r < reps; ++r)
        if (launch(mode, d, bytes / 16, nullptr)) return 1;
    (void)hipEventRecord(e1, nullptr);
    (void)hipEventSynchronize(e1);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("mode %d: %.3f ms per %zu MiB = %.0f GB/s\n", mode, ms / reps, bytes >> 20,
           bytes / (ms / reps * 1e-3) / 1e9);
    (void)hipFree(d);
    return 0;
}
