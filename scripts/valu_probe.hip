// VALU issue rates on this box (measurement tool, not product code): cycles per wave64 instruction per SIMD
// for instruction forms the rollout kernels use, at 1/2/4/8 waves per SIMD.
// Build: hipcc --offload-arch=gfx950 -O3 -o /tmp/valu_probe scripts/valu_probe.hip
// Every block has 256 threads (one wave per SIMD of a CU); the grid is CUs x W blocks.  Each wave runs
// ITER x 64 instructions of one form (8 independent chains; OP dep: one dependent chain) written as inline
// asm.  Prints one JSON line per (form, W): wall time, in-kernel clock (s_memtime / s_memrealtime), SIMD
// cycles per instruction = wall x clock / (W x ITER x 64).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef float f2 __attribute__((ext_vector_type(2)));
enum { FMA, DEP, DPP, SIN, PK, CND, MOVS, ADD_DPP_QP, ADDS, CNDVCC, MED3S, MULLIT, FMAS, MOVV, RCP, MAD64, MULHI, XOR, CMP, ADDV, CNDVCC_SET, CNDE64VCC, CNDCMP, MIX_FMA_DPP, MIX_FMA_SADD, MIX_FMA_CND32, CNDE64V };

template <int OP>
__global__ void __launch_bounds__(256) k(float* out, int iters, uint64_t* clk) {
    float a[8];
    f2 p[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 0.5f};
    }
    const float b = 0.999f, c = 1e-4f;
    const f2 pb = f2{0.999f, 1.001f};
    const uint64_t m = 0x5555555555555555ull;
    const float sv = 1.25f;
    if constexpr (OP == CNDVCC_SET || OP == CNDE64VCC || OP == MIX_FMA_CND32) asm volatile("s_mov_b64 vcc, 0x5555" ::: "vcc");
    uint64_t mk;  // a lane mask formed by a VALU compare (as the rollout's lane selects are)
    asm volatile("v_cmp_gt_u32_e64 %0, 2, %1" : "=s"(mk) : "v"(threadIdx.x & 3));
    const uint64_t t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                if constexpr (OP == FMA) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                if constexpr (OP == DEP) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
                if constexpr (OP == DPP)
                    asm volatile("v_mov_b32_dpp %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
                if constexpr (OP == ADD_DPP_QP)
                    asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
                if constexpr (OP == SIN) asm volatile("v_sin_f32 %0, %0" : "+v"(a[i]));
                if constexpr (OP == PK) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p[i]) : "v"(pb));
                if constexpr (OP == CND) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(m));
                if constexpr (OP == MOVS) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "s"(sv));
                if constexpr (OP == ADDS) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i]) : "s"(sv));
                if constexpr (OP == ADDV) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == CNDVCC) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == MED3S) asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(sv), "v"(b));
                if constexpr (OP == MULLIT) asm volatile("v_mul_f32 %0, 0x3eaaaaab, %0" : "+v"(a[i]));
                if constexpr (OP == FMAS) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "s"(sv), "v"(c));
                if constexpr (OP == MOVV) asm volatile("v_mov_b32 %0, %1" : "=v"(a[i]) : "v"(a[(i + 1) & 7]));
                if constexpr (OP == RCP) asm volatile("v_rcp_f32 %0, %0" : "+v"(a[i]));
                if constexpr (OP == MAD64) asm volatile("v_mad_u64_u32 %0, vcc, %1, %1, 0" : "=v"(p[i]) : "v"(a[i]));
                if constexpr (OP == MULHI) asm volatile("v_mul_hi_u32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == XOR) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == CNDVCC_SET) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == CNDE64VCC) asm volatile("v_cndmask_b32_e64 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                if constexpr (OP == CNDE64V) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "s"(mk));
                if constexpr (OP == CNDCMP) {
                    if ((i & 3) == 0) asm volatile("v_cmp_lt_f32_e32 vcc, %0, %1" :: "v"(a[i]), "v"(b) : "vcc");
                    asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                }
                if constexpr (OP == MIX_FMA_DPP) {
                    if (i & 1) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf" : "+v"(a[i]));
                    else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                }
                if constexpr (OP == MIX_FMA_SADD) {
                    if (i & 1) asm volatile("v_add_f32 %0, %1, %0" : "+v"(a[i]) : "s"(sv));
                    else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                }
                if constexpr (OP == MIX_FMA_CND32) {
                    if ((i & 3) == 3) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(a[i]) : "v"(b));
                    else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
                }
                if constexpr (OP == CMP) asm volatile("v_cmp_lt_f32_e64 s[4:5], %0, %1" :: "v"(a[i]), "v"(b) : "s4", "s5");
            }
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    float s = 0.0f;
#pragma unroll
    for (int i = 0; i < 8; ++i) s += a[i] + p[i].x + p[i].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = t1 - t0;
        clk[1] = r1 - r0;
    }
}

template <int OP>
void run(const char* name, int cus, float* out, uint64_t* clk) {
    const int iters = 400;
    for (int W = 1; W <= 4; W *= 4) {
        hipEvent_t e0, e1;
        hipEventCreate(&e0);
        hipEventCreate(&e1);
        k<OP><<<cus * W, 256>>>(out, iters, clk);  // warm
        hipDeviceSynchronize();
        hipEventRecord(e0);
        const int reps = 5;
        for (int r = 0; r < reps; ++r) k<OP><<<cus * W, 256>>>(out, iters, clk);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms = 0;
        hipEventElapsedTime(&ms, e0, e1);
        uint64_t h[2];
        hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
        const double us = 1e3 * ms / reps;
        const double mhz = h[1] ? 100.0 * (double)h[0] / (double)h[1] : 0.0;
        const double insts = (double)W * iters * 64;
        printf("{\"form\": \"%s\", \"waves_per_simd\": %d, \"us\": %.2f, \"clock_mhz\": %.0f, \"cyc_per_inst_simd\": %.2f, "
               "\"cyc_per_inst_wave_block0\": %.2f}\n",
               name, W, us, mhz, us * mhz / insts, (double)h[0] / (iters * 64.0));
        hipEventDestroy(e0);
        hipEventDestroy(e1);
    }
}

int main_all() {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    float* out;
    uint64_t* clk;
    hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    hipMalloc(&clk, 2 * sizeof(uint64_t));
    run<FMA>("v_fma_f32 x8 chains", cus, out, clk);
    run<DEP>("v_fma_f32 one dependent chain", cus, out, clk);
    run<DPP>("v_mov_b32_dpp quad_perm x8", cus, out, clk);
    run<ADD_DPP_QP>("v_add_f32_dpp quad_perm x8", cus, out, clk);
    run<SIN>("v_sin_f32 x8", cus, out, clk);
    run<PK>("v_pk_mul_f32 x8", cus, out, clk);
    run<CND>("v_cndmask_b32_e64 sgpr mask x8", cus, out, clk);
    run<MOVS>("v_mov_b32 from sgpr x8", cus, out, clk);
    run<ADDS>("v_add_f32 sgpr+vgpr x8", cus, out, clk);
    run<ADDV>("v_add_f32 vgpr+vgpr (e32) x8", cus, out, clk);
    run<CNDVCC>("v_cndmask_b32_e32 vcc x8", cus, out, clk);
    run<MED3S>("v_med3_f32 with sgpr x8", cus, out, clk);
    run<MULLIT>("v_mul_f32 literal x8", cus, out, clk);
    run<FMAS>("v_fma_f32 with sgpr x8", cus, out, clk);
    run<MOVV>("v_mov_b32 vgpr x8", cus, out, clk);
    run<RCP>("v_rcp_f32 x8", cus, out, clk);
    run<MAD64>("v_mad_u64_u32 x8", cus, out, clk);
    run<MULHI>("v_mul_hi_u32 x8", cus, out, clk);
    run<XOR>("v_xor_b32 x8", cus, out, clk);
    run<CMP>("v_cmp_lt_f32_e64 to sgpr x8", cus, out, clk);
    return 0;
}

int main(int argc, char** argv) {
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    float* out;
    uint64_t* clk;
    hipMalloc(&out, (size_t)cus * 8 * 256 * sizeof(float));
    hipMalloc(&clk, 2 * sizeof(uint64_t));
    if (argc > 1) return main_all();
    run<CNDVCC>("v_cndmask_b32_e32 vcc (unset) x8", cus, out, clk);
    run<CNDVCC_SET>("v_cndmask_b32_e32 vcc (s_mov) x8", cus, out, clk);
    run<CNDE64VCC>("v_cndmask_b32_e64 vcc x8", cus, out, clk);
    run<CNDE64V>("v_cndmask_b32_e64 cmp mask x8", cus, out, clk);
    run<CNDCMP>("v_cmp_e32 vcc + 4 cndmask_e32", cus, out, clk);
    run<MIX_FMA_DPP>("mix fma / add_dpp 1:1", cus, out, clk);
    run<MIX_FMA_SADD>("mix fma / add sgpr 1:1", cus, out, clk);
    run<MIX_FMA_CND32>("mix fma / cndmask_e32 3:1", cus, out, clk);
    run<FMA>("v_fma_f32 x8 chains", cus, out, clk);
    return 0;
}
