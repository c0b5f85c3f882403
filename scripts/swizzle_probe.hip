// Cross-lane exchange costs on this box (measurement tool, not product code): the quad broadcasts and butterflies
// of the four-lane rollout as DPP (a VALU instruction) against ds_swizzle_b32 (the LDS unit's crossbar, no LDS
// memory), at 1 and 4 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/swizzle_probe scripts/swizzle_probe.hip
// Every block has 256 threads (one wave per SIMD of a CU); the grid is CUs x W blocks.  Each wave runs ITER rounds of
// one form written as inline asm.  Prints one JSON line per (form, W): SIMD cycles per VALU instruction and per
// exchange (wall x clock / (W x ITER x count)).
//   fma8            8 independent v_fma_f32 per round (the plain VALU rate)
//   dpp8            8 independent v_mov_b32_dpp quad_perm per round
//   swz8            8 independent ds_swizzle_b32 quad_perm per round, one lgkmcnt(0) wait per round
//   fma6_dpp2       6 fma + 2 dpp per round
//   fma6_swz2       6 fma + 2 swizzles per round (swizzles waited one round later)
//   swz_chain       one dependent swizzle chain (latency: issue -> data)
//   dpp_chain       one dependent dpp chain
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

enum { FMA8, DPP8, SWZ8, FMA6_DPP2, FMA6_SWZ2, SWZ_CHAIN, DPP_CHAIN, FMA12_SWZ4 };

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, int iters, uint64_t* clk) {
    float a[8], x[4];
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = threadIdx.x * 2e-3f + i;
    const float b = 0.999f, c = 1e-4f;
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            if constexpr (OP == FMA8) {
#pragma unroll
                for (int i = 0; i < 8; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if constexpr (OP == DPP8) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
            }
            if constexpr (OP == SWZ8) {
#pragma unroll
                for (int i = 0; i < 8; ++i)
                    asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(QUAD_PERM,1,0,3,2)" : "+v"(a[i]));
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
            if constexpr (OP == FMA6_DPP2) {
#pragma unroll
                for (int i = 0; i < 6; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
            }
            if constexpr (OP == FMA6_SWZ2) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int i = 0; i < 2; ++i)
                    asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(QUAD_PERM,1,0,3,2)" : "+v"(x[i]));
#pragma unroll
                for (int i = 0; i < 6; ++i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
            }
            if constexpr (OP == FMA12_SWZ4) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
                for (int i = 0; i < 4; ++i)
                    asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(QUAD_PERM,1,0,3,2)" : "+v"(x[i]));
#pragma unroll
                for (int i = 0; i < 12; ++i)
                    asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i & 7]) : "v"(b), "v"(c));
            }
            if constexpr (OP == SWZ_CHAIN) {
                asm volatile("ds_swizzle_b32 %0, %0 offset:swizzle(QUAD_PERM,1,0,3,2)\n\ts_waitcnt lgkmcnt(0)"
                             : "+v"(a[0]));
            }
            if constexpr (OP == DPP_CHAIN) {
                asm volatile("s_nop 1\n\tv_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf"
                             : "+v"(a[0]));
            }
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) s += x[i];
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

// per round: count of the instruction class the figure is quoted per (VALU for the fma mixes, exchanges otherwise)
template <int OP>
void run(const char* name, int per_round, int cus, float* out, uint64_t* clk) {
    const int iters = 400;
    for (int W = 1; W <= 4; W *= 4) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        k<OP><<<cus * W, 256>>>(out, iters, clk);  // warm
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; ++r) k<OP><<<cus * W, 256>>>(out, iters, clk);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        uint64_t h[2];
        (void)hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        const double us = 1e3 * ms / reps;
        const double mhz = h[1] ? 100.0 * (double)h[0] / (double)h[1] : 0.0;
        const double n = (double)W * iters * 8 * per_round;
        printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"us\": %.2f, \"clock_mhz\": %.0f, \"cyc_per_unit_simd\": %.2f, "
               "\"cyc_per_unit_wave_block0\": %.2f}\n",
               name, W, us, mhz, us * mhz / n, (double)h[0] / (iters * 8.0 * per_round));
        (void)hipEventDestroy(e0);
        (void)hipEventDestroy(e1);
    }
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    float* out;
    uint64_t* clk;
    (void)hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    (void)hipMalloc(&clk, 2 * sizeof(uint64_t));
    run<FMA8>("fma8 (per fma)", 8, cus, out, clk);
    run<DPP8>("dpp8 (per dpp)", 8, cus, out, clk);
    run<SWZ8>("swz8 (per swizzle)", 8, cus, out, clk);
    run<FMA6_DPP2>("fma6_dpp2 (per round of 8)", 8, cus, out, clk);
    run<FMA6_SWZ2>("fma6_swz2 (per fma)", 6, cus, out, clk);
    run<FMA12_SWZ4>("fma12_swz4 (per fma)", 12, cus, out, clk);
    run<SWZ_CHAIN>("swz_chain (per swizzle)", 1, cus, out, clk);
    run<DPP_CHAIN>("dpp_chain (per dpp)", 1, cus, out, clk);
    return 0;
}
