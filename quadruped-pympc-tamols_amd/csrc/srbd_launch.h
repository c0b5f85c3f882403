// srbd_launch.h -- internal launchers shared by srbd_kernels.hip, tamols_kernel.hip and srbd_api.hip.
#pragma once

#include "srbd_core.h"

namespace srbd {

bool rollout_specialised(int kind, int H, int S);
void launch_rollout(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                    int rec_stride, int threads, hipStream_t s);
void launch_rng(const ModelConst& mc, const StepInput* in, float* noise, hipStream_t s);
void launch_transpose(const float* src, int n, int P, int ldn, float* dst, hipStream_t s);
size_t merge_smem_bytes(int nrec, int P);
void launch_merge(const ModelConst& mc, const StepInput* in, const float* recs, int nrec, int rec_stride,
                  int rows_in_rec, const float* noise, float* rank_out, StepOutput* out, hipStream_t s);
void launch_advance(const ModelConst& mc, StepInput* in, const StepOutput* out, hipStream_t s);
void launch_div_selftest(const float* a, const float* b, int n, float* o, hipStream_t s);

// TAMOLS (tamols_kernel.hip)
constexpr int TAMOLS_NQ = 19;        // nearest-neighbour queries per candidate
constexpr int TAMOLS_MAXCAND = 320;  // rows * cols (LDS: 23 doubles per candidate)

struct TamolsArgs {
    int rows, cols, ncand;
    int has_vel, has_base, has_feet;
    int contact[4];
    double vel[3], base[3];
    double feet[12], seeds[12], hips[12];
    srbd_tamols_params p;
};

size_t tamols_smem_bytes(int ncand);
void launch_tamols(const TamolsArgs& a, const double* hm, double* scores, double* footholds, double* boxes,
                   int* valid, double* seedh, hipStream_t s);

}  // namespace srbd
