// srbd_api.hip -- C-ABI of libsrbd_hip.so (declared in include/srbd_mpc.h).
//
// A context owns: the per-context constants (ModelConst, kernarg), a pinned StepInput staging
// buffer and its device copy (one H2D per step), the noise matrix in SoA layout [P][ldn]
// (ldn = rows rounded up to 256, padding zero), the per-block partial records, a StepOutput
// (one D2H per step) and, optionally, a captured hipGraph of the whole step.
#include <dlfcn.h>
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>  // types only: RCCL is dlopen'ed (the caller's copy, e.g. torch's)

#include "srbd_jaxrng.h"
#include "srbd_launch.h"

using namespace srbd;

namespace {
thread_local std::string g_last_error;

// The thread form always runs 256 samples (four leaves of the reduction tree) per block: its kernel is compiled for
// that block size (the shapes it is the default for, N > 65 536, used it anyway).
int rollout_threads(int) { return 256; }
// Four lanes per sample unless the samples alone fill the GPU (measured crossover: zero-order
// N ~ 65536, splines beyond 262144; scripts/kernel_sweep.py).  SRBD_ROLLOUT=thread|quad (read at create)
// picks the other of the two forms at a shape (tests: both give the same costs bit for bit; measurement).
int rollout_mode(int kind, int n_local) {
    const char* e = getenv("SRBD_ROLLOUT");
    if (e && !strcmp(e, "thread")) return ROLLOUT_THREAD;
    if (e && !strcmp(e, "quad")) return ROLLOUT_QUAD;
    const int quad_max = kind == SRBD_ZERO_ORDER ? 65536 : 524288;
    return n_local <= quad_max ? ROLLOUT_QUAD : ROLLOUT_THREAD;
}
// Four-lane kernel: 64 samples (4 waves, one per SIMD) per block.  128 samples (2 waves per SIMD)
// halves the block records but measured 15.7 -> 21.3 us for the C2 rollout (the two waves do slow
// each other), and the zero-order kernel's LDS noise stage is sized for 64.
int quad_samples_per_block(int n_local) {
    (void)n_local;
    return 64;
}
constexpr int MAX_RECORDS = 8192;  // merge_kernel holds 8 record minima per thread x 1024 threads
constexpr int TAGGED_OUT = -1;     // enqueue_device_step: the launch writes tagged outputs (wait_tagged), no flag
}  // namespace

struct srbd_ctx {
    srbd_config cfg;
    ModelConst mc;
    // rollout blocks, leaf records per block (the reduction tree's leaves, srbd_core.h) and this rank's leaves;
    // wrec_stride: floats per leaf / level-1 record; rrec_stride: floats of one rank buffer (its exchange-level
    // node records, t_xmax of them)
    int mode = 0, threads = 64, nblocks = 0, lpb = 1, nleaf = 0, wrec_stride = 0, rrec_stride = 0;
    hipStream_t stream = nullptr;
    bool own_stream = true;
    StepInput* d_in = nullptr;
    StepInput* h_in = nullptr;
    StepInput* d_in_host = nullptr;  // device alias of the mapped pinned h_in (upload_input)
    StepOutput* d_out = nullptr;
    // Host-driven steps: the merge writes StepOutput straight into mapped pinned host memory (h_out,
    // device alias d_out_host) and then publishes a sequence number in h_flag; the host spins on it.
    // (Measured on MI355X: launch + spin on a mapped flag 5.8 us vs launch + hipStreamSynchronize 11.3;
    // a 2-kernel graph + sync 19.4: hipGraphs cost more than they save at this size.)
    StepOutput* h_out = nullptr;
    StepOutput* d_out_host = nullptr;
    uint32_t* h_flag = nullptr;
    uint32_t* d_flag = nullptr;
    uint32_t seq = 0;
    // Sharded transport owned by the library: an RCCL communicator (srbd_comm_init) and the rank
    // record / gathered records it exchanges with ncclAllGather on the context stream.
    ncclComm_t comm = nullptr;
    int comm_world = 0;
    float* d_myrec = nullptr;
    float* d_gath = nullptr;
    // xGMI exchange (merge_xchg_kernel): this rank's mailbox (uncached device memory, IPC-exported),
    // the peer table handed to the kernel, a device word pair {error, epoch counter}, the cached stage
    // the second merge pass reads, and the two-step / one-step graphs of the device-resident chain.
    float* xg_base = nullptr;
    std::vector<void*> xg_opened;
    XchgArgs xa{};
    XchgArgs* d_xa = nullptr;  // device copy (the rollout launch's in-launch exchange, GroupArgs::xa)
    int xg_world = 0;
    int* xg_err = nullptr;
    float* xg_stage = nullptr;
    hipGraphExec_t g_xg2 = nullptr, g_xg1 = nullptr;
    // Noise matrices, double buffered: the rollout launch of a step reading d_noise[cur] also draws the
    // predicted next step's noise (counter + 1) into the other buffer (MPPI / random sampling; CEM's
    // draws depend on the sigma the step produces).
    float* d_noise[2] = {nullptr, nullptr};
    int cur = 0;
    bool pref_valid = false;
    int pref_buf = 0;
    uint64_t pref_seed = 0, pref_ctr = 0;
    bool chain_started = false;  // sharded device-resident chain
    float* d_noise_rm = nullptr;
    size_t noise_rm_cap = 0;
    float* d_costs = nullptr;
    float* d_wrec = nullptr;
    // in-launch level-1 fold of the leaf records (GroupArgs): gsize = TREE_FAN leaves per node, ngroups
    // level-1 records the merge reads; gsize 1: the merge reads the nleaf leaf records
    int gsize = 1, ngroups = 0;
    float* d_grec = nullptr;
    uint32_t* d_gcnt = nullptr;
    // in-launch final merge (final_merge_ok): the rollout's last group writes the host step's outputs
    bool final_merge = false;
    uint32_t* d_gdone = nullptr;
    // fast_tail (fast_tail_ok, SRBD_FAST_TAIL=0 turns it off): the node records the folders hand over, tagged words
    bool fast_tail = false;
    bool gen_env = true;  // SRBD_GEN != "0" at create (gen_now)
    int gen_rg = GEN_REGEN_QUADS;  // quads the epilogue regenerates (SRBD_GEN_RG at create), the rest stored and read
    int gen_quad_min = 0;  // four-lane form: rows from which the launch makes its draws (gen_now); 0 off
    uint64_t* d_gtag = nullptr;
    // its host-step outputs as tagged words (GroupArgs::outt, tagged_outputs), host-mapped
    uint64_t* h_outt = nullptr;
    uint64_t* d_outt = nullptr;
    // host steps pass the step input to the rollout as a kernel argument (ks_ok): no upload kernel
    bool ks = false;
    hipGraphExec_t g_dev2 = nullptr, g_dev1 = nullptr;
    float* d_ga_freq = nullptr;  // injected per-row step frequencies (gait-adaptive parity mode), ldn floats
    bool input_ready = false;
    // Armed host steps (srbd_set_armed): during a step the next one's copy, rollout and merge are queued
    // behind it, the copy kernel spinning on the host-mapped word h_go; the next srbd_step writes its
    // input and stores the go word instead of launching.  The armed run writes its costs into
    // d_costs_arm (swapped in when it fires), so a cancelled run (which recomputes the previous input)
    // leaves every buffer a later call reads unchanged.
    int arm_mode = 0;
    uint64_t arm_deadline_us = 50000;
    uint32_t* h_go = nullptr;
    uint32_t* d_go = nullptr;
    uint32_t* d_fired = nullptr;  // arm_copy_kernel's verdict for the chain behind it (Publish::gate)
    int64_t arm_refired = 0;      // claimed chains whose copy had already given up: re-run unarmed
    uint32_t arm_test_delay_us = 0;  // srbd_debug_arm_delay: host sleep between claim and go (tests only)
    float* d_costs_arm = nullptr;
    bool armed = false;
    uint32_t arm_seq = 0;
    int arm_buf = 0, arm_nflags = 1;
    bool arm_fused = true;  // the chain's draws were made ahead (fused); else its RNG kernel draws them
    uint64_t arm_seed = 0, arm_ctr = 0;
    std::chrono::steady_clock::time_point arm_t0;
    int64_t arm_served = 0, arm_cancelled = 0;
    int64_t foothold_chained = 0;  // srbd_foothold_mpc_step calls run chained (srbd_foothold_chain)
    std::string err;
};

// At most one armed context per process: an armed copy kernel holds its hardware queue until it fires,
// is cancelled or reaches its deadline, and other streams may share that queue.  So every entry point
// cancels the armed context's pending step (g_arm_mu guards g_armed and the contexts' armed flags).
static std::mutex g_arm_mu;
static srbd_ctx* g_armed = nullptr;
static void arm_cancel_locked(srbd_ctx* c) {
    if (!c || !c->armed) return;
    __atomic_store_n(c->h_go, c->arm_seq | ARM_CANCEL, __ATOMIC_RELEASE);
    c->armed = false;
    ++c->arm_cancelled;
    if (g_armed == c) g_armed = nullptr;
}
// Cancel the process's armed step unless it belongs to `keep`.
static void arm_cancel_others(const srbd_ctx* keep = nullptr) {
    std::lock_guard<std::mutex> lk(g_arm_mu);
    if (g_armed && g_armed != keep) arm_cancel_locked(g_armed);
}
static void arm_cancel(srbd_ctx* c) {
    std::lock_guard<std::mutex> lk(g_arm_mu);
    arm_cancel_locked(c);
    if (g_armed) arm_cancel_locked(g_armed);
}

#define HIP_TRY(ctx, expr)                                                                          \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);                        \
            return SRBD_E_HIP;                                                                      \
        }                                                                                           \
    } while (0)

static int fail(srbd_ctx* c, int code, const std::string& m) {
    if (c) c->err = m;
    else g_last_error = m;
    return code;
}

// ------------------------------------------------------------------ configuration
static int params_leg(const srbd_config* c) {
    if (c->parametrization == SRBD_LINEAR_SPLINE) return (c->num_splines + 1) * 3;
    if (c->parametrization == SRBD_CUBIC_SPLINE) return 12 * c->num_splines;
    return 3 * c->horizon;
}

extern "C" int srbd_num_params(const srbd_config* cfg) {
    if (!cfg || cfg->horizon < 1 || cfg->horizon > SRBD_MAX_HORIZON) return SRBD_E_INVALID;
    if (cfg->parametrization < 0 || cfg->parametrization > 2) return SRBD_E_INVALID;
    if (cfg->parametrization != SRBD_ZERO_ORDER && cfg->num_splines < 1) return SRBD_E_INVALID;
    const int P = 4 * params_leg(cfg);
    return P > SRBD_MAX_PARAMS ? SRBD_E_INVALID : P;
}

extern "C" int srbd_abi_version(void) { return SRBD_ABI_VERSION; }

extern "C" int srbd_device_count(int32_t* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (count) *count = (e == hipSuccess) ? n : 0;
    return e == hipSuccess ? SRBD_OK : SRBD_E_NODEVICE;
}

// Spline coefficients at `step` (NMPC:181-257): idx from the f32 linspace comparison, q = step /
// f32(horizon_leg / S) - idx, and the Hermite weights in the reference's f32 order.
static void spline_coef(const srbd_config* c, float step, int horizon_leg, int* idx, float* q, float* omq, float* a,
                        float* b, float* cc, float* d) {
    *idx = 0;
    *q = *omq = *a = *b = *cc = *d = 0.0f;
    if (c->parametrization == SRBD_ZERO_ORDER) {
        *idx = (int)(int16_t)step;
        return;
    }
    const int S = c->num_splines;
    int ix = 0;
    for (int i = 0; i <= S; ++i) {
        const float cb = (float)((double)c->horizon * (double)i / (double)S);
        if (step >= cb) ix = i;
    }
    float tau = step / (float)((double)horizon_leg / (double)S);
    tau = tau - (float)ix;
    const float qq = tau / 1.0f;
    *idx = ix;
    *q = qq;
    *omq = 1.0f - qq;
    *a = 2.0f * qq * qq * qq - 3.0f * qq * qq + 1.0f;
    *b = (qq * qq * qq - 2.0f * qq * qq + qq) * 1.0f;
    *cc = -2.0f * qq * qq * qq + 3.0f * qq * qq;
    *d = (qq * qq * qq - qq * qq) * 1.0f;
}

static int build_model(const srbd_config* cfg, ModelConst* mc, std::string* why) {
    const int P = srbd_num_params(cfg);
    if (P < 0) {
        *why = "unsupported horizon/parametrization/num_splines";
        return SRBD_E_INVALID;
    }
    if (cfg->num_samples < 1) {
        *why = "num_samples must be >= 1";
        return SRBD_E_INVALID;
    }
    if (cfg->method < 0 || cfg->method > 2) {
        *why = "unknown sampling method";
        return SRBD_E_INVALID;
    }
    const int world = cfg->world_size < 1 ? 1 : cfg->world_size;
    if (cfg->rank < 0 || cfg->rank >= world || cfg->num_samples < world) {
        *why = "bad rank/world_size";
        return SRBD_E_INVALID;
    }
    const TreeShape ts = tree_shape(cfg->num_samples, world, cfg->rank);
    if (!ts.ok) {
        *why = "too few rows for world_size ranks: every rank needs at least one 64-row leaf";
        return SRBD_E_INVALID;
    }
    if (cfg->parametrization == SRBD_CUBIC_SPLINE && 10 * (cfg->num_splines - 1) + 11 >= params_leg(cfg)) {
        *why = "cubic spline needs num_splines >= 1";
        return SRBD_E_INVALID;
    }
    memset(mc, 0, sizeof(*mc));
    mc->H = cfg->horizon;
    mc->P = P;
    mc->PL = P / 4;
    mc->kind = cfg->parametrization;
    mc->S = cfg->num_splines;
    mc->method = cfg->method;
    const int ne = cfg->num_elite > 0 ? cfg->num_elite : 10;
    mc->K = num_elite(cfg->method, ne);
    if (mc->K > MAXK || (cfg->method == SRBD_CEM_MPPI && mc->K < 2)) {
        *why = "num_elite must be in [2, SRBD_MAX_ELITE] (sample variance over the elite set)";
        return SRBD_E_INVALID;
    }
    mc->N = cfg->num_samples;
    // rows of this rank: whole nodes of the reduction tree's exchange level (srbd_core.h tree_shape)
    mc->row0 = (int)ts.row0;
    mc->n_local = (int)ts.nrows;
    mc->ldn = (mc->n_local + 255) / 256 * 256;
    mc->t_leaves = ts.leaves;
    mc->t_depth = ts.depth;
    mc->t_xlevel = ts.xlevel;
    mc->t_xnodes = ts.xnodes;
    mc->t_xmax = ts.xmax;
    mc->t_world = world;
    mc->leaf0 = mc->row0 / LEAF_ROWS;
    mc->nleaf = (mc->n_local + LEAF_ROWS - 1) / LEAF_ROWS;
    mc->inv_m = 1.0f / cfg->mass;
    mc->mg = cfg->mg;
    if (!(cfg->grf_min >= 0.0f && cfg->grf_max >= cfg->grf_min && cfg->mu >= 0.0f)) {
        *why = "need 0 <= grf_min <= grf_max and mu >= 0";
        return SRBD_E_INVALID;
    }
    mc->grf_min = cfg->grf_min;
    mc->grf_max = cfg->grf_max;
    mc->mu = cfg->mu;
    mc->neg_mu = -cfg->mu;
    memcpy(mc->inertia, cfg->inertia, sizeof(mc->inertia));
    inv3(cfg->inertia, mc->Iinv);
    for (int i = 0; i < 12; ++i) mc->Q[i] = cfg->q_diag[i];
    for (int n = 0; n < MAXH; ++n) mc->dts[n] = n < cfg->horizon ? cfg->dts[n] : 0.0f;
    for (int n = 0; n < cfg->horizon; ++n)
        spline_coef(cfg, (float)n, cfg->horizon, &mc->sidx[n], &mc->sq[n], &mc->somq[n], &mc->sa[n], &mc->sb[n],
                    &mc->sc[n], &mc->sd[n]);
    spline_coef(cfg, 0.0f, 1, &mc->fidx, &mc->fq, &mc->fomq, &mc->fa, &mc->fb, &mc->fc, &mc->fd);
    mc->sigma_mppi = cfg->sigma_mppi;
    for (int i = 0; i < 3; ++i) mc->sigma_rs[i] = cfg->sigma_random_sampling[i];
    mc->ga = 0;
    mc->ga_freq = nullptr;
    for (int i = 0; i < 5; ++i) mc->fz_ns[i] = mc->mg / (float)i;  // the division fill_input makes per step
    // the parameter columns final_grf_pred's decode reads (the column-split merge's tail block)
    mc->ntail = 0;
    for (int leg = 0; leg < 4; ++leg) {
        auto rec = [&](int j) {
            const int col = leg * mc->PL + j;
            if (!is_tail_col(*mc, col)) {
                mc->tailmask[col >> 5] |= 1u << (col & 31);
                mc->tailc[mc->ntail++] = (short)col;
            }
            return 0.0f;
        };
        float fx, fy, fz;
        decode_leg(mc->kind, mc->H, mc->S, mc->fidx, mc->fq, mc->fomq, mc->fa, mc->fb, mc->fc, mc->fd, 0, rec, fx, fy,
                   fz);
    }
    return SRBD_OK;
}

// Host part of the per-step input (StepInput) -- identical on every rank.
static int fill_input(const srbd_config* cfg, const ModelConst& mc, StepInput* in, const float* state,
                      const float* ref, const float* contact, int stride, const float* best, const float* sigma,
                      uint64_t seed, uint64_t counter) {
    if (!state || !ref || !contact || !best || stride < mc.H) return SRBD_E_INVALID;
    if (mc.method == SRBD_CEM_MPPI && !sigma) return SRBD_E_INVALID;
    memcpy(in->state, state, sizeof(in->state));
    memcpy(in->ref, ref, sizeof(in->ref));
    memset(in->contact, 0, sizeof(in->contact));
    for (int l = 0; l < 4; ++l)
        for (int n = 0; n < mc.H; ++n) in->contact[l][n] = contact[(size_t)l * stride + n];
    for (int n = 0; n < mc.H; ++n) {
        const float ns = in->contact[0][n] + in->contact[1][n] + in->contact[2][n] + in->contact[3][n];
        in->fzref[n] = mc.mg / ns;  // inf when no leg is in stance: neutralised by the clip (App. A.3)
    }
    float cf = 0.0f;
    for (int i = 12; i < 24; ++i) {
        const float e = state[i] - ref[i];
        cf = cf + (e * cfg->q_diag[i]) * e;
    }
    in->cost_feet = cf;
    in->seed_lo = (uint32_t)seed;
    in->seed_hi = (uint32_t)(seed >> 32);
    in->ctr_lo = (uint32_t)counter;
    in->ctr_hi = (uint32_t)(counter >> 32);
    memcpy(in->best, best, sizeof(float) * mc.P);
    if (sigma) memcpy(in->sigma, sigma, sizeof(float) * mc.P);
    else memset(in->sigma, 0, sizeof(in->sigma));
    return SRBD_OK;
}

// ------------------------------------------------------------------ lifetime
extern "C" int srbd_create(const srbd_config* cfg, srbd_ctx** out) {
    if (!cfg || !out) return fail(nullptr, SRBD_E_INVALID, "null argument");
    *out = nullptr;
    ModelConst mc;
    std::string why;
    int rc = build_model(cfg, &mc, &why);
    if (rc) return fail(nullptr, rc, why);
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0)
        return fail(nullptr, SRBD_E_NODEVICE, "no HIP device visible (this library has no CPU fallback)");
    if (cfg->device_id < 0 || cfg->device_id >= ndev) return fail(nullptr, SRBD_E_NODEVICE, "bad device_id");
    srbd_ctx* c = new srbd_ctx();
    c->cfg = *cfg;
    c->mc = mc;
    c->mode = rollout_mode(mc.kind, mc.n_local);
    // the four-lane kernel addresses noise through a buffer descriptor (31-bit byte offsets)
    if ((long long)mc.P * mc.ldn * 4 >= (1LL << 31)) c->mode = ROLLOUT_THREAD;
    c->threads = c->mode == ROLLOUT_QUAD ? 4 * quad_samples_per_block(mc.n_local) : rollout_threads(mc.n_local);
    {  // srbd_step, and the xGMI sharded step (xg_step); SRBD_KS=0 at create: the upload kernel instead (A/B)
        const char* e = getenv("SRBD_KS");
        c->ks = ks_ok(mc, c->mode) && !(e && e[0] == '0');
    }
    const int spb = rollout_spb(c->mode, c->threads);  // samples per rollout block
    c->nblocks = (mc.n_local + spb - 1) / spb;
    c->lpb = spb / LEAF_ROWS;
    c->nleaf = mc.nleaf;
    // the merge reads the level-1 records (the launch folds the leaves) or the leaf records
    if (c->nblocks > MAX_RECORDS ||
        (group_size(mc) > 1 ? (mc.nleaf + TREE_FAN - 1) / TREE_FAN : mc.nleaf) > MAX_RECORDS) {
        delete c;
        return fail(nullptr, SRBD_E_INVALID, "too many samples per rank");
    }
    c->wrec_stride = rec_floats_wave(mc.P, mc.K);
    c->rrec_stride = mc.t_xmax * rec_floats_rank(mc.P, mc.K);
    auto cleanup_fail = [&](const char* what, hipError_t e) {
        std::string m = std::string(what) + ": " + hipGetErrorString(e);
        srbd_destroy(c);
        return fail(nullptr, SRBD_E_HIP, m);
    };
    hipError_t e;
    if ((e = hipSetDevice(cfg->device_id)) != hipSuccess) return cleanup_fail("hipSetDevice", e);
    if ((e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking)) != hipSuccess)
        return cleanup_fail("hipStreamCreate", e);
    merge_prepare();
    if ((e = hipHostMalloc((void**)&c->h_in, sizeof(StepInput), hipHostMallocMapped)) != hipSuccess)
        return cleanup_fail("hipHostMalloc", e);
    if ((e = hipHostGetDevicePointer((void**)&c->d_in_host, c->h_in, 0)) != hipSuccess)
        return cleanup_fail("hipHostGetDevicePointer", e);
    if ((e = hipHostMalloc((void**)&c->h_out, sizeof(StepOutput), hipHostMallocMapped | hipHostMallocCoherent)) !=
        hipSuccess)
        return cleanup_fail("hipHostMalloc", e);
    if ((e = hipHostGetDevicePointer((void**)&c->d_out_host, c->h_out, 0)) != hipSuccess)
        return cleanup_fail("hipHostGetDevicePointer", e);
    if ((e = hipHostMalloc((void**)&c->h_flag, sizeof(uint32_t) * MERGE_MAX_BLOCKS, hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
        return cleanup_fail("hipHostMalloc", e);
    if ((e = hipHostGetDevicePointer((void**)&c->d_flag, c->h_flag, 0)) != hipSuccess)
        return cleanup_fail("hipHostGetDevicePointer", e);
    for (int i = 0; i < MERGE_MAX_BLOCKS; ++i) __atomic_store_n(c->h_flag + i, 0u, __ATOMIC_RELEASE);
    memset(c->h_in, 0, sizeof(StepInput));
    memset(c->h_out, 0, sizeof(StepOutput));
    const size_t noise_bytes = sizeof(float) * (size_t)mc.P * mc.ldn;
    if ((e = hipMalloc((void**)&c->d_in, STEP_INPUT_ALLOC)) != hipSuccess) return cleanup_fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&c->d_out, sizeof(StepOutput))) != hipSuccess) return cleanup_fail("hipMalloc", e);
    // a column-split merge only ORs late bits into status, so the device output starts zeroed (srbd_sync_result)
    if ((e = hipMemset(c->d_out, 0, sizeof(StepOutput))) != hipSuccess) return cleanup_fail("hipMemset", e);
    for (int b = 0; b < 2; ++b)
        if ((e = hipMalloc((void**)&c->d_noise[b], noise_bytes)) != hipSuccess) return cleanup_fail("hipMalloc", e);
    if ((e = hipMalloc((void**)&c->d_costs, sizeof(float) * mc.ldn)) != hipSuccess)
        return cleanup_fail("hipMalloc", e);
    // every block writes lpb leaf records (the last block's past nleaf are never read)
    if ((e = hipMalloc((void**)&c->d_wrec, sizeof(float) * (size_t)c->nblocks * c->lpb * c->wrec_stride)) != hipSuccess)
        return cleanup_fail("hipMalloc", e);
    const char* ge = getenv("SRBD_GEN");
    c->gen_env = !(ge && !strcmp(ge, "0"));
    if (const char* gr = getenv("SRBD_GEN_RG")) c->gen_rg = std::max(0, std::min(mc.P / 4, atoi(gr)));
    if (const char* gq = getenv("SRBD_GEN_QUAD_MIN")) c->gen_quad_min = atoi(gq);
    c->gsize = group_size(mc);
    c->ngroups = (c->nleaf + TREE_FAN - 1) / TREE_FAN;
    if (c->gsize > 1) {
        if ((e = hipMalloc((void**)&c->d_grec, sizeof(float) * (size_t)c->ngroups * c->wrec_stride)) != hipSuccess)
            return cleanup_fail("hipMalloc", e);
        if ((e = hipMalloc((void**)&c->d_gcnt, sizeof(uint32_t) * (size_t)c->ngroups)) != hipSuccess)
            return cleanup_fail("hipMalloc", e);
        c->final_merge = final_merge_ok(mc, c->mode, c->ngroups, c->wrec_stride);
        if ((e = hipMalloc((void**)&c->d_gdone, sizeof(uint32_t))) != hipSuccess ||
            (e = hipMemsetAsync(c->d_gdone, 0, sizeof(uint32_t), c->stream)) != hipSuccess)
            c->final_merge = false;
        const char* ft = getenv("SRBD_FAST_TAIL");
        if (c->final_merge && fast_tail_ok(mc, c->mode, c->ngroups, c->wrec_stride) && !(ft && !strcmp(ft, "0"))) {
            const size_t tb = sizeof(uint64_t) * (size_t)FT_GTAG_WORDS(mc.P);
            const size_t ob = sizeof(uint64_t) * (size_t)(mc.P + TAGGED_OUT_EXTRA);
            c->fast_tail = hipMalloc((void**)&c->d_gtag, tb) == hipSuccess &&
                           hipMemsetAsync(c->d_gtag, 0, tb, c->stream) == hipSuccess &&
                           hipHostMalloc((void**)&c->h_outt, ob, hipHostMallocMapped | hipHostMallocCoherent) ==
                               hipSuccess &&
                           hipHostGetDevicePointer((void**)&c->d_outt, c->h_outt, 0) == hipSuccess;
            if (c->h_outt) memset(c->h_outt, 0, ob);
        }
        if ((e = hipMemsetAsync(c->d_gcnt, 0, sizeof(uint32_t) * (size_t)c->ngroups, c->stream)) != hipSuccess)
            return cleanup_fail("hipMemset", e);
    }
    for (int b = 0; b < 2; ++b)
        if ((e = hipMemsetAsync(c->d_noise[b], 0, noise_bytes, c->stream)) != hipSuccess)
            return cleanup_fail("hipMemset", e);
    if ((e = hipMemsetAsync(c->d_in, 0, STEP_INPUT_ALLOC, c->stream)) != hipSuccess)
        return cleanup_fail("hipMemset", e);
    if ((e = hipStreamSynchronize(c->stream)) != hipSuccess) return cleanup_fail("hipStreamSynchronize", e);
    *out = c;
    return SRBD_OK;
}

static void comm_release(srbd_ctx* c);
static uint64_t next_seed(const srbd_ctx* c, uint64_t seed);
static void xg_drop_graphs(srbd_ctx* c);

extern "C" void srbd_destroy(srbd_ctx* c) {
    if (!c) return;
    arm_cancel(c);
    (void)hipSetDevice(c->cfg.device_id);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    comm_release(c);
    if (c->g_dev2) (void)hipGraphExecDestroy(c->g_dev2);
    if (c->g_dev1) (void)hipGraphExecDestroy(c->g_dev1);
    for (int b = 0; b < 2; ++b) (void)hipFree(c->d_noise[b]);
    (void)hipFree(c->d_in);
    (void)hipFree(c->d_out);
    (void)hipFree(c->d_noise_rm);
    (void)hipFree(c->d_costs);
    (void)hipFree(c->d_costs_arm);
    (void)hipFree(c->d_fired);
    if (c->h_go) (void)hipHostFree(c->h_go);
    (void)hipFree(c->d_wrec);
    (void)hipFree(c->d_grec);
    (void)hipFree(c->d_gcnt);
    (void)hipFree(c->d_gdone);
    (void)hipFree(c->d_gtag);
    if (c->h_outt) (void)hipHostFree(c->h_outt);
    (void)hipFree(c->d_ga_freq);
    if (c->h_in) (void)hipHostFree(c->h_in);
    if (c->h_out) (void)hipHostFree(c->h_out);
    if (c->h_flag) (void)hipHostFree(c->h_flag);
    if (c->stream && c->own_stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

extern "C" const char* srbd_last_error(const srbd_ctx* c) { return c ? c->err.c_str() : g_last_error.c_str(); }

extern "C" int srbd_set_stream(srbd_ctx* c, void* s) {
    if (!c) return SRBD_E_INVALID;
    arm_cancel(c);
    (void)hipSetDevice(c->cfg.device_id);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->own_stream) HIP_TRY(c, hipStreamDestroy(c->stream));
    if (c->g_dev2) (void)hipGraphExecDestroy(c->g_dev2);
    if (c->g_dev1) (void)hipGraphExecDestroy(c->g_dev1);
    c->g_dev2 = c->g_dev1 = nullptr;
    xg_drop_graphs(c);
    if (s) {
        c->stream = (hipStream_t)s;
        c->own_stream = false;
    } else {
        HIP_TRY(c, hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
        c->own_stream = true;
    }
    return SRBD_OK;
}

// ------------------------------------------------------------------ step
// Draw the next step's noise inside the rollout launch (extra blocks beside the rollout).  The draws
// never depend on the step (CEM stores unscaled normals, scaled by sigma on read).  Measured per
// step: N = 65 536 MPPI 64.2 -> 53.9 us, CEM cubic H16 98.4 -> 89.9 us, CEM N = 10 000 52.4 ->
// 48.3 us.  Above 65 536 rows the rollout fills every CU and the fused draws slow it.
constexpr int FUSE_MAX_ROWS = 65536;
static bool fusable(const srbd_ctx* c) { return c->mc.n_local <= FUSE_MAX_ROWS; }

// The step's draws made inside the rollout launch (gen_ok; SRBD_GEN=0 turns it off): host steps (the input by value)
// at shapes whose draws do not fuse into the previous launch, device Philox stream.  The caller also checks that no
// noise is injected.
// The four-lane form (GEN: rollout_quad_kernel) is opt-in (SRBD_GEN_QUAD_MIN=rows at create; measured slower at the
// north-star shape: step launch 33.1 vs 30.3 us -- the same VALU work moved onto the rollout waves),
// with the in-launch final merge and unarmed (armed chains carry the next step's draws).
static bool gen_now(const srbd_ctx* c) {
    if (!c->gen_env || !c->ks || !gen_ok(c->mc, c->mode)) return false;
    if (c->mode == ROLLOUT_QUAD)
        return c->gen_quad_min > 0 && !c->arm_mode && c->final_merge && c->mc.n_local >= c->gen_quad_min;
    return !fusable(c);
}

// Device-chain steps draw on the device: CEM draws are then unscaled (StepInput::noise_scaled = 0)
// whatever the last host step injected.
static int reset_noise_scaled(srbd_ctx* c) {
    HIP_TRY(c, hipMemsetAsync(&c->d_in->noise_scaled, 0, sizeof(int32_t), c->stream));
    return SRBD_OK;
}

static int upload_noise(srbd_ctx* c, const float* noise, int buf) {
    const ModelConst& mc = c->mc;
    const size_t bytes = sizeof(float) * (size_t)mc.n_local * mc.P;
    if (c->noise_rm_cap < bytes) {
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        (void)hipFree(c->d_noise_rm);
        c->d_noise_rm = nullptr;
        HIP_TRY(c, hipMalloc((void**)&c->d_noise_rm, bytes));
        c->noise_rm_cap = bytes;
    }
    HIP_TRY(c, hipMemcpyAsync(c->d_noise_rm, noise, bytes, hipMemcpyHostToDevice, c->stream));
    launch_transpose(c->d_noise_rm, mc.n_local, mc.P, mc.ldn, c->d_noise[buf], c->stream);
    return SRBD_OK;
}

// Noise of a step: injected (noise != NULL), the draws the previous step's rollout launch made when
// (seed, counter) match its prediction, else device draws generated now on the step's stream.
// Returns in *buf the buffer holding them.  Everything is ordered on one stream.
// gen: the rollout launch makes the step's draws itself (gen_now): nothing to draw here.
static int acquire_noise(srbd_ctx* c, const float* noise, uint64_t seed, uint64_t ctr, int* buf, bool gen = false) {
    int rc = SRBD_OK;
    if (gen && !noise) {
        *buf = c->cur;
    } else if (!noise && c->pref_valid && c->pref_seed == seed && c->pref_ctr == ctr) {
        *buf = c->pref_buf;
    } else {
        *buf = c->cur;
        if (noise) rc = upload_noise(c, noise, *buf);
        else launch_rng(c->mc, c->d_in, seed, ctr, 0, 0, c->d_noise[*buf], c->stream);
    }
    c->pref_valid = false;
    c->cur = *buf;
    return rc;
}

// rollout (+ next draws, counter + 1 from the device StepInput) -> merge on noise buffer `buf`
// The step's StepInput into device memory: a one-block copy kernel pulling it from the mapped pinned
// staging (host step p50 36.4 -> 35.1 us, p99 51.8 -> 44.0 at C2, against an async H2D copy): the header
// and best[P] (+ sigma[P] for CEM), the bytes the step reads.
static int upload_input(srbd_ctx* c) {
    const size_t P4 = sizeof(float) * (size_t)c->mc.P;
    const size_t sig = offsetof(StepInput, sigma);
    launch_copy16(c->d_in_host, c->d_in, offsetof(StepInput, best) + P4, sig, c->mc.method == SRBD_CEM_MPPI ? P4 : 0,
                  c->stream);
    return SRBD_OK;
}

// The step input as the rollout's kernel argument: StepInput's prefix and best[P] from the staging, the
// unused tail of best zeroed (the whole struct is the argument, and block 0 copies all of it to d_in).
static void fill_ksi(const srbd_ctx* c, StepInputK* k) {
    const size_t used = offsetof(StepInput, best) + sizeof(float) * (size_t)c->mc.P;
    memcpy(k, c->h_in, used);
    memset(reinterpret_cast<unsigned char*>(k) + used, 0, sizeof(StepInputK) - used);
}

// The records the merge reads: the group records when the rollout launch reduces its blocks in groups.
static GroupArgs grp_of(const srbd_ctx* c) { return GroupArgs{c->d_grec, c->d_gcnt, c->gsize}; }
static const float* merge_src(const srbd_ctx* c) { return c->gsize > 1 ? c->d_grec : c->d_wrec; }
static int merge_nrec(const srbd_ctx* c) { return c->gsize > 1 ? c->ngroups : c->nleaf; }
// tree levels a rank record folds up from the merge's input records (leaves or level-1 nodes) to the exchange level
static int levels_up(const srbd_ctx* c) { return c->mc.t_xlevel - (c->gsize > 1 ? 1 : 0); }

// Returns the number of merge blocks that publish (wait_published).
static int enqueue_device_step(srbd_ctx* c, int buf, float* rank_out, StepOutput* out, int chain = 0,
                               int ctr_inc = 1, bool fuse_next = false, Publish pub = {nullptr, 0},
                               float* costs = nullptr, const void* ksi = nullptr, bool gen = false) {
    const ModelConst& mc = c->mc;
    const RngJob next{c->d_noise[1 - buf], 0, 0, 1, 1, pub.gate};
    GroupArgs grp = grp_of(c);
    grp.gate = pub.gate;
    grp.ksi = ksi;
    grp.gen = gen && !fuse_next ? 1 + c->gen_rg : 0;
    // the rollout launch merges and publishes (not for the gait-adaptive rollout or the cost terms, which
    // srbd_set_gait / srbd_set_cost_terms can switch on after create: other kernels)
    if (c->final_merge && !mc.ga && !mc.cost_on && out && !rank_out && !chain && pub.flag) {
        grp.out = out;
        grp.flag = pub.flag;
        grp.seq = pub.seq;
        grp.gdone = c->d_gdone;
        grp.ngroups = c->ngroups;
        grp.fence_sys = merge_fence_sys();
        if (c->fast_tail) {
            grp.fast = 1;
            grp.gtag = c->d_gtag;
            if (!pub.gate) grp.outt = c->d_outt;  // armed chains keep the flag (their cancel token travels in it)
        }
        launch_rollout(mc, c->d_in, c->d_noise[buf], costs ? costs : c->d_costs, c->d_wrec, c->wrec_stride, c->mode,
                       c->threads, c->stream, fuse_next ? &next : nullptr, grp);
        return grp.outt ? TAGGED_OUT : 1;
    }
    launch_rollout(mc, c->d_in, c->d_noise[buf], costs ? costs : c->d_costs, c->d_wrec, c->wrec_stride, c->mode,
                   c->threads, c->stream, fuse_next ? &next : nullptr, grp);
    return launch_merge(mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, 0, c->d_noise[buf], rank_out, out, chain,
                        c->stream, nullptr, ctr_inc, pub, rank_out ? levels_up(c) : 0);
}

// Wait for the merge to publish `seq`.  Polls the stream now and then so a device fault or a launch
// failure surfaces as an error instead of a hang.
// `nflags` merge blocks publish, each into its own word.
static bool published(const srbd_ctx* c, uint32_t seq, int nflags) {
    for (int i = 0; i < nflags; ++i)
        if (__atomic_load_n(c->h_flag + i, __ATOMIC_ACQUIRE) != seq) return false;
    return true;
}

// cancelled != NULL (an armed chain): also accepts the chain's cancel token seq | ARM_CANCEL (it did not
// fire, Publish::gate) and reports it there.
static int wait_published(srbd_ctx* c, uint32_t seq, int nflags = 1, int* cancelled = nullptr) {
    auto token = [&]() {
        return cancelled && __atomic_load_n(c->h_flag, __ATOMIC_ACQUIRE) == (seq | ARM_CANCEL);
    };
    if (cancelled) *cancelled = 0;
    for (uint64_t it = 1;; ++it) {
        if (published(c, seq, nflags)) return SRBD_OK;
        if (token()) {
            *cancelled = 1;
            return SRBD_OK;
        }
        if ((it & 4095) == 0) {
            const hipError_t e = hipStreamQuery(c->stream);
            if (e == hipSuccess) {  // drained: the flag stores have completed
                if (published(c, seq, nflags)) return SRBD_OK;
                if (token()) {
                    *cancelled = 1;
                    return SRBD_OK;
                }
                // a launch that stopped part-way can leave group / final-merge arrival counts behind: clear them
                // so the next step starts from zero (they are zero between completed launches)
                if (c->d_gcnt) (void)hipMemsetAsync(c->d_gcnt, 0, sizeof(uint32_t) * (size_t)c->ngroups, c->stream);
                if (c->d_gdone) (void)hipMemsetAsync(c->d_gdone, 0, sizeof(uint32_t), c->stream);
                return fail(c, SRBD_E_HIP, "step completed without publishing its outputs");
            }
            if (e != hipErrorNotReady) HIP_TRY(c, e);
        }
        __builtin_ia32_pause();
    }
}

// A step whose merge reported a timed-out in-launch hand-off (StepOutput::status != 0: fast_tail -1, the column
// split's tail block / a slice 1 / 2): drain the stream, so no block of that launch is still writing, reset the
// hand-off state (the split's epoch and tagged words -- zeroed, so the next launch cannot accept a late word of
// the timed-out one --, the arrival counts, the device output's status) and fail the call.  Every path that
// launches a merge zeroes the status it reads before the launch (the column split only ORs its late bits in):
// srbd_step and srbd_step_finish the host-mapped one; device chains the device one, zeroed at create and here.
// An armed chain queued behind the timed-out step is cancelled first, so the drain does not wait out its copy
// kernel's deadline and the next call does not claim a chain that has given up.
static int check_handoff(srbd_ctx* c, int st = 0) {
    if (!st) st = __atomic_load_n(&c->h_out->status, __ATOMIC_ACQUIRE);
    if (st == 0) return SRBD_OK;
    arm_cancel(c);
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemset(reinterpret_cast<char*>(c->d_in) + sizeof(StepInput), 0, sizeof(SplitXchg)));
    if (c->d_gcnt) HIP_TRY(c, hipMemset(c->d_gcnt, 0, sizeof(uint32_t) * (size_t)c->ngroups));
    if (c->d_gdone) HIP_TRY(c, hipMemset(c->d_gdone, 0, sizeof(uint32_t)));
    HIP_TRY(c, hipMemset(&c->d_out->status, 0, sizeof(int32_t)));
    c->h_out->status = 0;
    return fail(c, SRBD_E_HIP, "merge hand-off timed out (status " + std::to_string(st) + ")");
}

// A fast_tail host step wrote its outputs as tagged words (GroupArgs::outt): wait until every word carries `seq`
// (word by word from the last, so a spin reads one word), then unpack them into h_out for copy_out.  The GPU's
// stores reach host memory in any order; a word is whole (one 8-byte store), so a tagged word is that step's value.
static int wait_tagged(srbd_ctx* c, uint32_t seq) {
    const int P = c->mc.P, n = P + TAGGED_OUT_EXTRA;
    const uint64_t* w = c->h_outt;
    auto tag_ok = [&](int i) { return (uint32_t)(__atomic_load_n(w + i, __ATOMIC_ACQUIRE) >> 32) == seq; };
    int i = n - 1;
    for (uint64_t it = 1; i >= 0; ++it) {
        if (tag_ok(i)) {
            --i;
            continue;
        }
        if ((it & 4095) == 0) {
            const hipError_t e = hipStreamQuery(c->stream);
            if (e == hipSuccess) {  // drained: every store of the launch has landed
                while (i >= 0 && tag_ok(i)) --i;
                if (i < 0) break;
                if (c->d_gcnt) (void)hipMemsetAsync(c->d_gcnt, 0, sizeof(uint32_t) * (size_t)c->ngroups, c->stream);
                if (c->d_gdone) (void)hipMemsetAsync(c->d_gdone, 0, sizeof(uint32_t), c->stream);
                return fail(c, SRBD_E_HIP, "step completed without publishing its outputs");
            }
            if (e != hipErrorNotReady) HIP_TRY(c, e);
        }
        __builtin_ia32_pause();
    }
    StepOutput& o = *c->h_out;
    auto val = [&](int k) { return (uint32_t)__atomic_load_n(w + k, __ATOMIC_RELAXED); };
    for (int j = 0; j < P; ++j) o.best[j] = u2f(val(j));
    for (int k = 0; k < 12; ++k) o.grf[k] = u2f(val(P + k));
    for (int k = 0; k < 24; ++k) o.pred[k] = u2f(val(P + 12 + k));
    o.best_cost = u2f(val(P + 36));
    o.best_index = (int32_t)val(P + 37);
    o.best_freq = u2f(val(P + 38));
    o.status = (int32_t)val(P + 39);
    return SRBD_OK;
}

static int copy_out(srbd_ctx* c, float* best, float* sigma, srbd_result* out) {
    const StepOutput& o = *c->h_out;
    memcpy(best, o.best, sizeof(float) * c->mc.P);
    if (sigma && c->mc.method == SRBD_CEM_MPPI) memcpy(sigma, o.sigma, sizeof(float) * c->mc.P);
    if (out) {
        memcpy(out->grf, o.grf, sizeof(out->grf));
        memcpy(out->predicted_state, o.pred, sizeof(out->predicted_state));
        out->best_cost = o.best_cost;
        out->best_index = o.best_index;
        out->best_freq = o.best_freq;
        out->status = o.status;
    }
    return SRBD_OK;
}

// Queue the next host step behind the work on the stream, its copy kernel spinning on h_go
// (srbd_set_armed).  fused: the draws for (seed, ctr) are already in noise buffer `buf` (made by this
// step's rollout launch), so only that call can be served; else the chain's RNG kernel draws into `buf`
// keyed by the copied input's (seed, counter), so any device-draw call can be.
static void arm_next(srbd_ctx* c, uint64_t seed, uint64_t ctr, int buf, bool fused = true) {
    std::lock_guard<std::mutex> lk(g_arm_mu);
    if (g_armed && g_armed != c) arm_cancel_locked(g_armed);
    uint32_t s = (c->seq + 1) & ~ARM_CANCEL;  // the cancel token is seq | ARM_CANCEL
    if (s == 0) s = 1;
    c->seq = s;
    const size_t P4 = sizeof(float) * (size_t)c->mc.P;
    // the age a claim checks runs from before the copy kernel can start waiting (its deadline counts from
    // its own start, which is later), so a claim never sees a younger chain than the kernel does
    c->arm_t0 = std::chrono::steady_clock::now();
    launch_arm_copy(c->d_go, s, c->arm_deadline_us * 100ull, c->d_in_host, c->d_in, offsetof(StepInput, best) + P4,
                    offsetof(StepInput, sigma), c->mc.method == SRBD_CEM_MPPI ? P4 : 0, c->d_fired, c->stream);
    if (!fused) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[buf], c->stream, c->d_fired);
    c->arm_nflags = enqueue_device_step(c, buf, nullptr, c->d_out_host, 0, 0, fused, Publish{c->d_flag, s, c->d_fired},
                                        c->d_costs_arm);
    c->arm_fused = fused;
    c->armed = true;
    c->arm_seq = s;
    c->arm_buf = buf;
    c->arm_seed = seed;
    c->arm_ctr = ctr;
    g_armed = c;
}

// The armed chain can serve this call: device draws, the predicted (seed, counter), and well inside the
// copy kernel's deadline (the host never fires a chain that may have timed out).
static bool arm_claim(srbd_ctx* c, const float* noise, uint64_t seed, uint64_t counter) {
    std::lock_guard<std::mutex> lk(g_arm_mu);
    if (g_armed && g_armed != c) arm_cancel_locked(g_armed);
    if (!c->armed) return false;
    const double age_us =
        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - c->arm_t0).count();
    if (!noise && (!c->arm_fused || (seed == c->arm_seed && counter == c->arm_ctr)) &&
        age_us < 0.5 * (double)c->arm_deadline_us) {
        c->armed = false;  // claimed: nobody cancels it now
        ++c->arm_served;
        if (g_armed == c) g_armed = nullptr;
        return true;
    }
    arm_cancel_locked(c);
    return false;
}

extern "C" int srbd_step(srbd_ctx* c, const float* state, const float* ref, const float* contact,
                         int32_t contact_stride, float* best, float* sigma, const float* noise, uint64_t seed,
                         uint64_t counter, srbd_result* out, float* out_costs) {
    if (!c) return SRBD_E_INVALID;
    if (c->cfg.world_size > 1) return fail(c, SRBD_E_STATE, "sharded context: use srbd_step_local/finish");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    // the armed chain's copy kernel reads h_in only after the go word, so it can be rewritten now
    const bool fire = c->arm_mode && arm_claim(c, noise, seed, counter);
    int rc = fill_input(&c->cfg, c->mc, c->h_in, state, ref, contact, contact_stride, best, sigma, seed, counter);
    if (rc) {
        if (fire) __atomic_store_n(c->h_go, c->arm_seq | ARM_CANCEL, __ATOMIC_RELEASE);
        return fail(c, rc, "invalid step arguments");
    }
    c->h_in->noise_scaled = noise ? 1 : 0;
    c->h_out->status = 0;  // check_handoff
    const bool want_arm = c->arm_mode && !noise;
    int nflags = 1;
    uint32_t seq = 0;
    // the unarmed launch of this call (also the fallback of a claimed chain that had already given up)
    auto launch_unarmed = [&]() -> int {
        int r;
        // the step input as the rollout's kernel argument (its block 0 writes the device copy), or uploaded
        StepInputK ksi;
        const bool ks = c->ks && !c->mc.ga && !c->mc.cost_on;
        if (ks)
            fill_ksi(c, &ksi);
        else if ((r = upload_input(c)))
            return r;
        int buf = 0;
        const bool gen = !noise && gen_now(c);
        if ((r = acquire_noise(c, noise, seed, counter, &buf, gen))) return r;
        const bool fuse = !noise && !gen && fusable(c);
        const Publish pub{c->d_flag, ++c->seq, nullptr};
        seq = pub.seq;
        nflags = enqueue_device_step(c, buf, nullptr, c->d_out_host, 0, 0, fuse, pub, nullptr, ks ? &ksi : nullptr,
                                     gen);
        HIP_TRY(c, hipGetLastError());
        if (fuse) {
            c->pref_valid = true;
            c->pref_buf = 1 - buf;
            c->pref_seed = next_seed(c, seed);
            c->pref_ctr = counter + 1;
        }
        return SRBD_OK;
    };
    // arm the next step behind this one (its launches overlap this step's GPU time); with costs wanted
    // the copy-back goes first (it would queue behind the armed copy kernel)
    // fused: the next step's draws are in pref_buf; unfused: the chain redraws into this step's buffer
    auto arm = [&]() {
        if (c->pref_valid) arm_next(c, next_seed(c, seed), counter + 1, c->pref_buf, true);
        else if (!fusable(c)) arm_next(c, next_seed(c, seed), counter + 1, c->cur, false);
    };
    const int claimed_buf = c->arm_buf;
    const bool claimed_fused = c->arm_fused;
    if (fire) {
        if (c->arm_test_delay_us) std::this_thread::sleep_for(std::chrono::microseconds(c->arm_test_delay_us));
        __atomic_store_n(c->h_go, c->arm_seq, __ATOMIC_RELEASE);
        seq = c->arm_seq;
        nflags = c->arm_nflags;
        std::swap(c->d_costs, c->d_costs_arm);  // the fired run's costs
        c->cur = c->arm_buf;
        c->pref_valid = c->arm_fused;
        if (c->arm_fused) {
            c->pref_buf = 1 - c->arm_buf;
            c->pref_seed = next_seed(c, seed);
            c->pref_ctr = counter + 1;
        }
    } else if ((rc = launch_unarmed())) {
        return rc;
    }
    if (want_arm && !out_costs) arm();
    int cancelled = 0;
    if ((rc = nflags == TAGGED_OUT ? wait_tagged(c, seq) : wait_published(c, seq, nflags, fire ? &cancelled : nullptr)))
        return rc;
    if (cancelled) {
        // The claimed chain had already given up (its copy kernel's deadline passed before the go word, e.g.
        // this thread was preempted between the claim and the go store): it computed nothing and published
        // its cancel token.  Undo the claim, cancel the chain just armed behind it, run the call unarmed --
        // never the previous input's outputs (round-2 advisor finding).
        std::swap(c->d_costs, c->d_costs_arm);
        arm_cancel(c);
        {
            std::lock_guard<std::mutex> lk(g_arm_mu);  // srbd_armed_stats reads them under the lock
            ++c->arm_refired;
            --c->arm_served;  // counted as served at the claim
            ++c->arm_cancelled;
        }
        c->pref_valid = claimed_fused;  // this call's draws are in the claimed chain's buffer
        c->pref_buf = claimed_buf;
        c->pref_seed = seed;
        c->pref_ctr = counter;
        if ((rc = launch_unarmed())) return rc;
        if (want_arm && !out_costs) arm();
        if ((rc = nflags == TAGGED_OUT ? wait_tagged(c, seq) : wait_published(c, seq, nflags))) return rc;
    }
    if (out_costs) {
        HIP_TRY(c, hipMemcpyAsync(out_costs, c->d_costs, sizeof(float) * c->mc.n_local, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        if (want_arm) arm();
    }
    if ((rc = check_handoff(c))) return rc;
    c->input_ready = true;
    return copy_out(c, best, sigma, out);
}

// Armed host steps (see srbd_ctx): enable != 0 queues each following srbd_step's successor ahead of its
// input; deadline_us bounds the copy kernel's wait (0: 50 ms).  Disabling cancels a pending step.
extern "C" int srbd_set_armed(srbd_ctx* c, int32_t enable, uint64_t deadline_us) {
    if (!c) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    if (enable && c->cfg.world_size > 1) return fail(c, SRBD_E_STATE, "armed steps are for srbd_step (unsharded)");
    if (enable && !c->h_go) {
        HIP_TRY(c, hipHostMalloc((void**)&c->h_go, 64, hipHostMallocMapped | hipHostMallocCoherent));
        HIP_TRY(c, hipHostGetDevicePointer((void**)&c->d_go, c->h_go, 0));
        __atomic_store_n(c->h_go, 0u, __ATOMIC_RELEASE);
    }
    if (enable && !c->d_costs_arm) HIP_TRY(c, hipMalloc((void**)&c->d_costs_arm, sizeof(float) * c->mc.ldn));
    if (enable && !c->d_fired) {
        HIP_TRY(c, hipMalloc((void**)&c->d_fired, sizeof(uint32_t)));
        HIP_TRY(c, hipMemset(c->d_fired, 0, sizeof(uint32_t)));
    }
    c->arm_mode = enable ? 1 : 0;
    c->arm_deadline_us = deadline_us ? deadline_us : 50000;
    return SRBD_OK;
}

extern "C" int srbd_armed_refired(const srbd_ctx* c, int64_t* refired) {
    if (!c || !refired) return SRBD_E_INVALID;
    std::lock_guard<std::mutex> lk(g_arm_mu);
    *refired = c->arm_refired;
    return SRBD_OK;
}

extern "C" int srbd_debug_arm_delay(srbd_ctx* c, uint32_t delay_us) {
    if (!c) return SRBD_E_INVALID;
    c->arm_test_delay_us = delay_us;
    return SRBD_OK;
}

extern "C" int srbd_foothold_chained(const srbd_ctx* c, int64_t* n) {
    if (!c || !n) return SRBD_E_INVALID;
    *n = c->foothold_chained;
    return SRBD_OK;
}

extern "C" int srbd_debug_split_drop(srbd_ctx* c) {
    if (!c) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    const uint32_t one = 1;
    HIP_TRY(c, hipMemcpyAsync(reinterpret_cast<char*>(c->d_in) + sizeof(StepInput) + offsetof(SplitXchg, drop), &one,
                              sizeof(one), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return SRBD_OK;
}

extern "C" int srbd_armed_stats(const srbd_ctx* c, int64_t* served, int64_t* cancelled) {
    if (!c) return SRBD_E_INVALID;
    std::lock_guard<std::mutex> lk(g_arm_mu);
    if (served) *served = c->arm_served;
    if (cancelled) *cancelled = c->arm_cancelled;
    return SRBD_OK;
}

// ------------------------------------------------------------------ sharded step
extern "C" int srbd_record_floats(const srbd_ctx* c) { return c ? c->rrec_stride : SRBD_E_INVALID; }

extern "C" int srbd_step_local(srbd_ctx* c, const float* state, const float* ref, const float* contact,
                               int32_t contact_stride, const float* best, const float* sigma, const float* noise_local,
                               uint64_t seed, uint64_t counter, void* d_record) {
    if (!c || !d_record) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    // the pinned staging buffer may still feed an in-flight H2D of the previous call
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    int rc = fill_input(&c->cfg, c->mc, c->h_in, state, ref, contact, contact_stride, best, sigma, seed, counter);
    if (rc) return fail(c, rc, "invalid step arguments");
    c->h_in->noise_scaled = noise_local ? 1 : 0;
    if ((rc = upload_input(c))) return rc;
    int buf = 0;
    if ((rc = acquire_noise(c, noise_local, seed, counter, &buf))) return rc;
    const bool fuse = !noise_local && fusable(c);
    enqueue_device_step(c, buf, (float*)d_record, nullptr, 0, 0, fuse);
    if (fuse) {
        c->pref_valid = true;
        c->pref_buf = 1 - buf;
        c->pref_seed = next_seed(c, seed);
        c->pref_ctr = counter + 1;
    }
    c->chain_started = false;
    HIP_TRY(c, hipGetLastError());
    c->input_ready = true;
    return SRBD_OK;
}

extern "C" int srbd_step_finish(srbd_ctx* c, const void* d_records, int32_t nrec, float* best, float* sigma,
                                srbd_result* out, float* out_costs_local) {
    if (!c || !d_records || nrec < 1 || !best) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "srbd_step_finish before srbd_step_local");
    if (nrec != c->mc.t_world) return fail(c, SRBD_E_INVALID, "srbd_step_finish takes world_size rank records");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    const Publish pub{c->d_flag, ++c->seq};
    c->h_out->status = 0;  // check_handoff (a column split ORs late bits in)
    // the gathered rank buffers are the exchange level's node list in order (ceil partition, tree_shape)
    const int nflags = launch_merge(c->mc, c->d_in, (const float*)d_records, c->mc.t_xnodes,
                                    rec_floats_rank(c->mc.P, c->mc.K), 1, nullptr, nullptr, c->d_out_host, 0,
                                    c->stream, nullptr, 1, pub);
    HIP_TRY(c, hipGetLastError());
    int rc = wait_published(c, pub.seq, nflags);
    if (rc) return rc;
    if ((rc = check_handoff(c))) return rc;
    if (out_costs_local) {
        HIP_TRY(c, hipMemcpyAsync(out_costs_local, c->d_costs, sizeof(float) * c->mc.n_local, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return copy_out(c, best, sigma, out);
}

// Device-resident sharded chain: draws keyed by the device counter, which srbd_device_step_finish
// advances after the merge.
extern "C" int srbd_device_step_local(srbd_ctx* c, void* d_record) {
    if (!c || !d_record) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step_local once first");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    const bool fuse = fusable(c);
    if (!c->chain_started) {
        const int rc = reset_noise_scaled(c);
        if (rc) return rc;
    }
    if (!c->chain_started || !fuse) {  // draws of this step (device counter); later ones come fused
        c->cur = 0;
        launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);
    }
    c->pref_valid = false;
    enqueue_device_step(c, c->cur, (float*)d_record, nullptr, 0, 0, fuse);
    if (fuse) c->cur = 1 - c->cur;
    c->chain_started = true;
    HIP_TRY(c, hipGetLastError());
    return SRBD_OK;
}

extern "C" int srbd_device_step_finish(srbd_ctx* c, const void* d_records, int32_t nrec) {
    if (!c || !d_records || nrec < 1) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step_local once first");
    if (nrec != c->mc.t_world) return fail(c, SRBD_E_INVALID, "srbd_device_step_finish takes world_size rank records");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    launch_merge(c->mc, c->d_in, (const float*)d_records, c->mc.t_xnodes, rec_floats_rank(c->mc.P, c->mc.K), 1,
                 nullptr, nullptr, c->d_out, 1, c->stream, nullptr, 1);
    HIP_TRY(c, hipGetLastError());
    return SRBD_OK;
}

extern "C" int srbd_sync_result(srbd_ctx* c, float* best, float* sigma, srbd_result* out) {
    if (!c || !best) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipMemcpyAsync(c->h_out, c->d_out, sizeof(StepOutput), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    // a device chain's merges OR a timed-out hand-off into d_out's status (sticky over the chain): report it
    // and reset the hand-off state, as a host step does
    const int st = c->h_out->status;
    int rc;
    if (st && (rc = check_handoff(c, st))) return rc;
    return copy_out(c, best, sigma, out);
}

// The device draws of a step keyed by (seed, counter): this shard's additional_random_parameters rows,
// row-major n_local x P (CEM: the unscaled standard normals; the step multiplies them by sigma).
extern "C" int srbd_draw_noise(srbd_ctx* c, uint64_t seed, uint64_t counter, float* out) {
    if (!c || !out) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    const ModelConst& mc = c->mc;
    c->pref_valid = false;  // the buffer the prefetched draws were in is overwritten
    c->cur = 0;
    launch_rng(mc, c->d_in, seed, counter, 0, 0, c->d_noise[0], c->stream);
    HIP_TRY(c, hipGetLastError());
    std::vector<float> soa((size_t)mc.P * mc.n_local);
    HIP_TRY(c, hipMemcpy2DAsync(soa.data(), sizeof(float) * mc.n_local, c->d_noise[0], sizeof(float) * mc.ldn,
                                sizeof(float) * mc.n_local, mc.P, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (int j = 0; j < mc.P; ++j)
        for (int k = 0; k < mc.n_local; ++k) out[(size_t)k * mc.P + j] = soa[(size_t)j * mc.n_local + k];
    return SRBD_OK;
}

extern "C" int srbd_copy_costs(srbd_ctx* c, float* out_costs) {
    if (!c || !out_costs) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipMemcpyAsync(out_costs, c->d_costs, sizeof(float) * c->mc.n_local, hipMemcpyDeviceToHost,
                              c->stream));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    return SRBD_OK;
}

// ------------------------------------------------------------------ gait-adaptive sampling
static void drop_graphs(srbd_ctx* c) {
    if (c->g_dev2) (void)hipGraphExecDestroy(c->g_dev2);
    if (c->g_dev1) (void)hipGraphExecDestroy(c->g_dev1);
    c->g_dev2 = c->g_dev1 = nullptr;
    xg_drop_graphs(c);
}

extern "C" int srbd_set_gait(srbd_ctx* c, const float* timing, float pgg_dt, float duty_factor, const float* freq_set,
                             int32_t n_freq, const float* freq_local) {
    if (!c || !timing || !freq_set || n_freq < 1 || n_freq > SRBD_MAX_FREQS) return SRBD_E_INVALID;
    arm_cancel(c);
    if (c->mc.method == SRBD_CEM_MPPI)
        return fail(c, SRBD_E_INVALID,
                    "gait-adaptive CEM is not provided (the reference's branch is broken as wired, SURVEY App. B #2)");
    if (c->mc.kind != SRBD_ZERO_ORDER && c->mc.S + 1 > GA_MAXCB) return fail(c, SRBD_E_INVALID, "num_splines > 32");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));  // no step in flight reads the staging or d_ga_freq
    StepInput* in = c->h_in;
    for (int l = 0; l < 4; ++l) in->ga_timing[l] = timing[l];
    in->ga_dt = pgg_dt;
    in->ga_duty = duty_factor;
    in->ga_nfreq = n_freq;
    for (int i = 0; i < SRBD_MAX_FREQS; ++i) in->ga_freqs[i] = i < n_freq ? freq_set[i] : 0.0f;
    // chunk boundaries float32(linspace(0, H, S+1)) as spline_coef forms them; integer steps compare
    // >= a boundary exactly when they are >= its ceiling
    for (int i = 0; i < GA_MAXCB; ++i) {
        const int S = c->mc.S > 0 ? c->mc.S : 1;
        const float cb = (float)((double)c->mc.H * (double)i / (double)S);
        in->ga_cb[i] = i <= S ? (int)ceilf(cb) : 1 << 30;
    }
    in->ga_explicit = freq_local ? 1 : 0;
    if (freq_local) {
        if (!c->d_ga_freq) {
            HIP_TRY(c, hipMalloc((void**)&c->d_ga_freq, sizeof(float) * (size_t)c->mc.ldn));
            HIP_TRY(c, hipMemset(c->d_ga_freq, 0, sizeof(float) * (size_t)c->mc.ldn));
        }
        HIP_TRY(c, hipMemcpy(c->d_ga_freq, freq_local, sizeof(float) * (size_t)c->mc.n_local, hipMemcpyHostToDevice));
    }
    if (!c->mc.ga || c->mc.ga_freq != c->d_ga_freq) {  // kernels take ModelConst by value: recapture graphs
        c->mc.ga = 1;
        c->mc.ga_freq = c->d_ga_freq;
        drop_graphs(c);
    }
    return SRBD_OK;
}

extern "C" int srbd_clear_gait(srbd_ctx* c) {
    if (!c) return SRBD_E_INVALID;
    arm_cancel(c);
    if (c->mc.ga) {
        HIP_TRY(c, hipSetDevice(c->cfg.device_id));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        c->mc.ga = 0;
        drop_graphs(c);
    }
    return SRBD_OK;
}

extern "C" int srbd_set_cost_terms(srbd_ctx* c, const float* r_force, float w_smooth, float w_cone) {
    if (!c || !r_force) return SRBD_E_INVALID;
    arm_cancel(c);
    const float w[5] = {r_force[0], r_force[1], r_force[2], w_smooth, w_cone};
    for (float x : w)
        if (!(x >= 0.0f && x < INFINITY)) return fail(c, SRBD_E_INVALID, "cost weights must be finite and >= 0");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    ModelConst& mc = c->mc;
    const int on = (w[0] != 0.0f || w[1] != 0.0f || w[2] != 0.0f || w_smooth != 0.0f || w_cone != 0.0f) ? 1 : 0;
    if (on != mc.cost_on || memcmp(mc.cost_r, r_force, sizeof(mc.cost_r)) || mc.cost_smooth != w_smooth ||
        mc.cost_cone != w_cone) {
        mc.cost_on = on;
        memcpy(mc.cost_r, r_force, sizeof(mc.cost_r));
        mc.cost_smooth = w_smooth;
        mc.cost_cone = w_cone;
        drop_graphs(c);  // kernels take ModelConst by value: recapture
    }
    return SRBD_OK;
}

// Device noise stream: Philox (seed, counter) or the reference's jax.random stream (srbd_jaxrng.h).
extern "C" int srbd_set_rng(srbd_ctx* c, int32_t kind) {
    if (!c) return SRBD_E_INVALID;
    if (kind != SRBD_RNG_PHILOX && kind != SRBD_RNG_JAX && kind != SRBD_RNG_JAX_LEGACY)
        return fail(c, SRBD_E_INVALID, "unknown RNG kind");
    if (kind != SRBD_RNG_PHILOX && (uint64_t)(c->mc.N - 1) * (uint64_t)c->mc.P >= (1ull << 32))
        return fail(c, SRBD_E_INVALID, "the jax.random stream counts draws in 32 bits: (N - 1) * P must be < 2^32");
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    if (c->mc.rng != kind) {
        c->mc.rng = kind;
        c->pref_valid = false;  // prefetched draws belong to the other stream
        drop_graphs(c);          // kernels take ModelConst by value: recapture
    }
    return SRBD_OK;
}

extern "C" int srbd_get_rng(const srbd_ctx* c) { return c ? c->mc.rng : SRBD_E_INVALID; }

// The key of the step after one keyed `seed`: the same seed for Philox (the counter advances), with_newkey
// (split(key)[0]) for the JAX stream.
static uint64_t next_seed(const srbd_ctx* c, uint64_t seed) {
    return c->mc.rng == SRBD_RNG_PHILOX ? seed : jax_next_key(seed, c->mc.rng == SRBD_RNG_JAX);
}

// ------------------------------------------------------------------ host merge (no device)
// The same reduction tree as the device (srbd_core.h): 64-row leaves summed in the balanced pairwise tree,
// TREE_FAN children per node folded in order, node key = the children's minimum, child sums rescaled by
// expf(-1 * (m_child - m_node)).  Host and device differ only by their expf; the host merge is W-invariant, as
// the device's is.
namespace {
struct HostNode {
    uint64_t key = ~0ull;
    float s = 0.0f;
    std::vector<float> v;
    std::vector<uint64_t> top;  // the K smallest keys under the node, ascending
};

HostNode host_fold(const HostNode* ch, int n, int P, int K, bool sums) {
    HostNode o;
    for (int c = 0; c < n; ++c) o.key = std::min(o.key, ch[c].key);
    const float m = u2f((uint32_t)(o.key >> 32));
    o.v.assign(P, 0.0f);
    if (sums)
        for (int c = 0; c < n; ++c) {
            const float sc = expf(-1.0f * (u2f((uint32_t)(ch[c].key >> 32)) - m));
            o.s = o.s + sc * ch[c].s;
            for (int j = 0; j < P; ++j) o.v[j] = o.v[j] + sc * ch[c].v[j];
        }
    for (int c = 0; c < n; ++c) o.top.insert(o.top.end(), ch[c].top.begin(), ch[c].top.end());
    std::sort(o.top.begin(), o.top.end());
    if ((int)o.top.size() > K) o.top.resize(K);
    return o;
}

// The leaf sum: the balanced pairwise tree over 64 values in row order (wave_sum_f32's lane-63 chain)
float pairwise64(float* v) {
    for (int n = 32; n >= 1; n >>= 1)
        for (int i = 0; i < n; ++i) v[i] = v[2 * i] + v[2 * i + 1];
    return v[0];
}

std::vector<HostNode> host_fold_level(const std::vector<HostNode>& lv, int P, int K, bool sums) {
    std::vector<HostNode> up;
    for (size_t g = 0; g < lv.size(); g += TREE_FAN)
        up.push_back(host_fold(lv.data() + g, (int)std::min<size_t>(TREE_FAN, lv.size() - g), P, K, sums));
    return up;
}
}  // namespace

static uint64_t host_rec_key(const float* R, int P, int q) {
    return ((uint64_t)f2u(R[REC_HDR + P + 2 * q + 1]) << 32) | (uint64_t)f2u(R[REC_HDR + P + 2 * q]);
}

extern "C" int srbd_shard_rows(int64_t num_samples, int32_t rank, int32_t world, int64_t* row0, int64_t* rows) {
    if (num_samples < 1 || world < 1 || rank < 0 || rank >= world || !row0 || !rows) return SRBD_E_INVALID;
    const TreeShape t = tree_shape(num_samples, world, rank);
    if (!t.ok) return fail(nullptr, SRBD_E_INVALID, "too few rows for world_size ranks");
    *row0 = t.row0;
    *rows = t.nrows;
    return SRBD_OK;
}

extern "C" int srbd_record_floats_host(const srbd_config* cfg) {
    if (!cfg) return SRBD_E_INVALID;
    ModelConst mc;
    std::string why;
    const int rc = build_model(cfg, &mc, &why);
    if (rc) return fail(nullptr, rc, why);
    return mc.t_xmax * rec_floats_rank(mc.P, mc.K);
}

extern "C" int srbd_make_record_host(const srbd_config* cfg, int32_t rank, int32_t world, const float* costs,
                                     const float* noise_rows, float* rec) {
    srbd_config cc = *cfg;
    cc.rank = rank;
    cc.world_size = world;
    ModelConst mc;
    std::string why;
    int rc = build_model(&cc, &mc, &why);
    if (rc) return fail(nullptr, rc, why);
    const int P = mc.P, K = mc.K, n = mc.n_local, rf = rec_floats_rank(P, K);
    const bool sums = mc.method != SRBD_RANDOM_SAMPLING;
    std::vector<HostNode> lv;
    for (int l = 0; l < mc.nleaf; ++l) {  // leaves: 64 consecutive rows
        HostNode o;
        const int r0 = l * LEAF_ROWS, r1 = std::min(n, r0 + LEAF_ROWS);
        for (int k = r0; k < r1; ++k) {
            const uint64_t kk = cost_key(costs[k], (uint32_t)(mc.row0 + k));
            o.key = std::min(o.key, kk);
            o.top.push_back(kk);
        }
        std::sort(o.top.begin(), o.top.end());
        if ((int)o.top.size() > K) o.top.resize(K);
        o.v.assign(P, 0.0f);
        if (sums) {  // rows past the shard's end are empty leaf slots: e = 0
            const float m = u2f((uint32_t)(o.key >> 32));
            float e[LEAF_ROWS], t[LEAF_ROWS];
            for (int k = 0; k < LEAF_ROWS; ++k) e[k] = r0 + k < r1 ? expf(-1.0f * (costs[r0 + k] - m)) : 0.0f;
            for (int k = 0; k < LEAF_ROWS; ++k) t[k] = e[k];
            o.s = pairwise64(t);
            for (int j = 0; j < P; ++j) {
                for (int k = 0; k < LEAF_ROWS; ++k) t[k] = r0 + k < r1 ? e[k] * noise_rows[(size_t)(r0 + k) * P + j] : 0.0f;
                o.v[j] = pairwise64(t);
            }
        }
        lv.push_back(std::move(o));
    }
    for (int L = 0; L < mc.t_xlevel; ++L) lv = host_fold_level(lv, P, K, sums);
    memset(rec, 0, sizeof(float) * (size_t)mc.t_xmax * rf);
    for (size_t g = 0; g < lv.size(); ++g) {  // this rank's exchange-level nodes
        const HostNode& o = lv[g];
        float* R = rec + g * rf;
        R[0] = u2f((uint32_t)(o.key >> 32));
        R[1] = sums ? o.s : 1.0f;
        R[2] = u2f((uint32_t)o.key);
        for (int j = 0; j < P; ++j) R[REC_HDR + j] = o.v[j];
        for (int e = 0; e < K; ++e) {
            const uint64_t kk = e < (int)o.top.size() ? o.top[e] : ~0ull;
            R[REC_HDR + P + 2 * e] = u2f((uint32_t)kk);
            R[REC_HDR + P + 2 * e + 1] = u2f((uint32_t)(kk >> 32));
            for (int j = 0; j < P; ++j)
                R[REC_HDR + P + 2 * K + e * P + j] =
                    kk == ~0ull ? 0.0f : noise_rows[(size_t)((uint32_t)kk - mc.row0) * P + j];
        }
    }
    return SRBD_OK;
}

extern "C" int srbd_finish_host(const srbd_config* cfg, const float* recs, int32_t nrec, const float* state,
                                const float* contact, int32_t stride, float* best, float* sigma, srbd_result* out) {
    if (!cfg || !recs || nrec < 1) return SRBD_E_INVALID;
    srbd_config cc = *cfg;
    cc.rank = 0;
    cc.world_size = nrec;  // one rank buffer per rank
    ModelConst mc;
    std::string why;
    int rc = build_model(&cc, &mc, &why);
    if (rc) return fail(nullptr, rc, why);
    const int P = mc.P, K = mc.K, stridef = rec_floats_rank(P, K);
    StepInput* in = new StepInput();
    rc = fill_input(&cc, mc, in, state, state, contact, stride, best, sigma, 0, 0);  // ref unused here
    if (rc) {
        delete in;
        return fail(nullptr, rc, "invalid arguments");
    }
    // the gathered buffers are the exchange level's node list: fold it to the root
    const bool sums = mc.method != SRBD_RANDOM_SAMPLING;
    std::vector<HostNode> lv(mc.t_xnodes);
    float btag = 0.0f;
    uint64_t bk = ~0ull;
    for (int r = 0; r < mc.t_xnodes; ++r) {
        const float* R = recs + (size_t)r * stridef;
        HostNode& o = lv[r];
        o.key = ((uint64_t)f2u(R[0]) << 32) | f2u(R[2]);
        btag = o.key < bk ? R[3] : btag;
        bk = std::min(bk, o.key);
        o.s = R[1];
        o.v.assign(R + REC_HDR, R + REC_HDR + P);
    }
    while (lv.size() > 1) lv = host_fold_level(lv, P, K, sums);
    const float beta = u2f((uint32_t)(bk >> 32));
    std::vector<float> V(P + 1, 0.0f);
    if (sums) {
        for (int j = 0; j < P; ++j) V[j] = lv[0].v[j];
        V[P] = lv[0].s;
    }
    nrec = mc.t_xnodes;
    // global top-K keys with their rows
    std::vector<std::pair<uint64_t, const float*>> cand;
    for (int r = 0; r < nrec; ++r)
        for (int q = 0; q < K; ++q) {
            const float* R = recs + (size_t)r * stridef;
            const uint64_t kk = host_rec_key(R, P, q);
            if (kk != ~0ull) cand.push_back({kk, R + REC_HDR + P + 2 * K + (size_t)q * P});
        }
    std::sort(cand.begin(), cand.end(), [](auto& a, auto& b) { return a.first < b.first; });
    const int Kv = std::min<int>(K, (int)cand.size());
    std::vector<float> nb(P);
    for (int j = 0; j < P; ++j) {
        nb[j] = mc.method == SRBD_RANDOM_SAMPLING ? in->best[j] + cand[0].second[j] : in->best[j] + V[j] / V[P];
        if (mc.method == SRBD_CEM_MPPI && sigma) {
            float s = 0.0f;
            for (int e = 0; e < Kv; ++e) s = s + cand[e].second[j];
            const float mean = s / (float)Kv;
            float var = 0.0f;
            for (int e = 0; e < Kv; ++e) {
                const float d = cand[e].second[j] - mean;
                var = var + d * d;
            }
            var = var / (float)(Kv - 1);
            float sg = sqrtf(var + 1e-8f);
            sg = sg > 5.0f ? 5.0f : sg;
            sg = sg < 0.2f ? 0.2f : sg;
            sigma[j] = sg;
        }
    }
    float grf[12], pred[24];
    final_grf_pred(mc, *in, nb.data(), grf, pred);
    memcpy(best, nb.data(), sizeof(float) * P);
    if (out) {
        memcpy(out->grf, grf, sizeof(grf));
        memcpy(out->predicted_state, pred, sizeof(pred));
        out->best_cost = beta;
        out->best_index = (int32_t)(uint32_t)bk;
        out->best_freq = btag;
        out->status = 0;
    }
    delete in;
    return SRBD_OK;
}

// ------------------------------------------------------------------ sharded transport (RCCL)
// One process per GPU; torch.distributed (or any launcher) only carries rank 0's ncclUniqueId.
// Every step then runs from C++: rollout -> rank record -> ncclAllGather over xGMI -> merge, all on
// the context stream, so a Python loop never sits between the kernels and the collective.
namespace {
struct RcclApi {
    void* h = nullptr;
    ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    const char* (*error_string)(ncclResult_t) = nullptr;
};
RcclApi g_rccl;
std::string g_rccl_err;

// Resolve RCCL from `path` (the copy the process already uses, e.g. torch/lib/librccl.so), else the
// system one.  dlopen of an already loaded path returns that same object.
bool rccl_load(const char* path) {
    if (g_rccl.h) return true;
    const char* cands[3] = {path, "/opt/rocm/lib/librccl.so.1", "librccl.so.1"};
    for (const char* p : cands) {
        if (!p || !*p) continue;
        void* h = dlopen(p, RTLD_NOW | RTLD_LOCAL);
        if (!h) continue;
        RcclApi a;
        a.h = h;
        a.get_unique_id = (decltype(a.get_unique_id))dlsym(h, "ncclGetUniqueId");
        a.comm_init_rank = (decltype(a.comm_init_rank))dlsym(h, "ncclCommInitRank");
        a.comm_destroy = (decltype(a.comm_destroy))dlsym(h, "ncclCommDestroy");
        a.all_gather = (decltype(a.all_gather))dlsym(h, "ncclAllGather");
        a.error_string = (decltype(a.error_string))dlsym(h, "ncclGetErrorString");
        if (a.get_unique_id && a.comm_init_rank && a.comm_destroy && a.all_gather && a.error_string) {
            g_rccl = a;
            return true;
        }
        dlclose(h);
    }
    g_rccl_err = "RCCL not found (tried the given path and /opt/rocm/lib/librccl.so.1)";
    return false;
}
}  // namespace

#define RCCL_TRY(ctx, expr)                                                                   \
    do {                                                                                      \
        const ncclResult_t r_ = (expr);                                                       \
        if (r_ != ncclSuccess) return fail((ctx), SRBD_E_HIP, std::string(#expr ": ") + g_rccl.error_string(r_)); \
    } while (0)

static void xg_drop_graphs(srbd_ctx* c) {
    if (c->g_xg2) (void)hipGraphExecDestroy(c->g_xg2);
    if (c->g_xg1) (void)hipGraphExecDestroy(c->g_xg1);
    c->g_xg2 = c->g_xg1 = nullptr;
}

static void comm_release(srbd_ctx* c) {
    if (c->comm && g_rccl.comm_destroy) (void)g_rccl.comm_destroy(c->comm);
    c->comm = nullptr;
    (void)hipFree(c->d_myrec);
    (void)hipFree(c->d_gath);
    c->d_myrec = c->d_gath = nullptr;
    for (void* p : c->xg_opened) (void)hipIpcCloseMemHandle(p);
    c->xg_opened.clear();
    (void)hipFree(c->xg_base);
    (void)hipFree(c->xg_err);
    (void)hipFree(c->xg_stage);
    (void)hipFree(c->d_xa);
    c->xg_stage = nullptr;
    c->d_xa = nullptr;
    xg_drop_graphs(c);
    c->xg_base = nullptr;
    c->xg_err = nullptr;
    c->xg_world = 0;
}

extern "C" int srbd_comm_get_unique_id(const char* rccl_path, uint8_t* id_out) {
    if (!id_out) return SRBD_E_INVALID;
    if (!rccl_load(rccl_path)) return fail(nullptr, SRBD_E_STATE, g_rccl_err);
    ncclUniqueId id;
    const ncclResult_t r = g_rccl.get_unique_id(&id);
    if (r != ncclSuccess) return fail(nullptr, SRBD_E_HIP, std::string("ncclGetUniqueId: ") + g_rccl.error_string(r));
    memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
    return SRBD_OK;
}

extern "C" int srbd_comm_init(srbd_ctx* c, const char* rccl_path, const uint8_t* id_in) {
    if (!c || !id_in) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!rccl_load(rccl_path)) return fail(c, SRBD_E_STATE, g_rccl_err);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    comm_release(c);
    ncclUniqueId id;
    memcpy(id.internal, id_in, NCCL_UNIQUE_ID_BYTES);
    const int world = c->cfg.world_size > 0 ? c->cfg.world_size : 1;
    RCCL_TRY(c, g_rccl.comm_init_rank(&c->comm, world, id, c->cfg.rank));
    c->comm_world = world;
    HIP_TRY(c, hipMalloc((void**)&c->d_myrec, sizeof(float) * c->rrec_stride));
    HIP_TRY(c, hipMalloc((void**)&c->d_gath, sizeof(float) * (size_t)c->rrec_stride * world));
    return SRBD_OK;
}

static int gather_records(srbd_ctx* c) {
    if (!c->comm) return fail(c, SRBD_E_STATE, "srbd_comm_init first");
    RCCL_TRY(c, g_rccl.all_gather(c->d_myrec, c->d_gath, (size_t)c->rrec_stride, ncclFloat32, c->comm, c->stream));
    return SRBD_OK;
}

// ---- xGMI exchange: rank records stored straight into every rank's mailbox by the merge kernel
static size_t xg_bytes(const srbd_ctx* c, int world) {
    // two slots per rank (exchange parity, merge_xchg_kernel) + one flag word per rank
    return ((sizeof(float) * 2 * (size_t)world * c->rrec_stride + sizeof(uint32_t) * world) + 255) / 256 * 256;
}

extern "C" int srbd_xgmi_export(srbd_ctx* c, uint8_t* handle_out) {
    if (!c || !handle_out) return SRBD_E_INVALID;
    arm_cancel(c);
    const int world = c->cfg.world_size > 0 ? c->cfg.world_size : 1;
    if (world > XCHG_MAX_WORLD) return fail(c, SRBD_E_INVALID, "xGMI exchange: world_size > 16");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    if (!c->xg_base) {
        const size_t bytes = xg_bytes(c, world);
        HIP_TRY(c, hipExtMallocWithFlags((void**)&c->xg_base, bytes, hipDeviceMallocUncached));
        HIP_TRY(c, hipMemset(c->xg_base, 0, bytes));
        HIP_TRY(c, hipMalloc((void**)&c->xg_err, 2 * sizeof(int)));
        HIP_TRY(c, hipMemset(c->xg_err, 0, 2 * sizeof(int)));
        HIP_TRY(c, hipMalloc((void**)&c->xg_stage, sizeof(float) * (size_t)world * c->rrec_stride));
        HIP_TRY(c, hipMalloc((void**)&c->d_xa, sizeof(XchgArgs)));
    }
    hipIpcMemHandle_t h;
    HIP_TRY(c, hipIpcGetMemHandle(&h, c->xg_base));
    memcpy(handle_out, &h, sizeof(h));
    return SRBD_OK;
}

// Peer table + fresh epochs: the flags and the epoch counter restart at 0 on every rank (connect runs on
// all ranks before any exchange kernel, so no peer is writing these words yet).
static int xg_table(srbd_ctx* c, int world, float* const* bases) {
    const size_t flag_off = 2 * (size_t)world * c->rrec_stride;
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    HIP_TRY(c, hipMemset(c->xg_base + flag_off, 0, sizeof(uint32_t) * world));
    HIP_TRY(c, hipMemset(c->xg_err, 0, 2 * sizeof(int)));
    HIP_TRY(c, hipDeviceSynchronize());
    xg_drop_graphs(c);
    c->xa = XchgArgs{};
    c->xa.mailbox = c->xg_base;
    c->xa.flags = reinterpret_cast<uint32_t*>(c->xg_base + flag_off);
    for (int r = 0; r < world; ++r) {
        c->xa.peer_mailbox[r] = bases[r];
        c->xa.peer_flags[r] = reinterpret_cast<uint32_t*>(bases[r] + flag_off);
    }
    c->xa.err = c->xg_err;
    c->xa.epoch = reinterpret_cast<uint32_t*>(c->xg_err + 1);
    c->xa.stage = c->xg_stage;
    c->xa.rank = c->cfg.rank;
    c->xa.world = world;
    c->xa.stride = c->rrec_stride;
    HIP_TRY(c, hipMemcpy(c->d_xa, &c->xa, sizeof(XchgArgs), hipMemcpyHostToDevice));
    c->xg_world = world;
    return SRBD_OK;
}

// handles: world x 64 bytes in rank order (each rank's srbd_xgmi_export).
extern "C" int srbd_xgmi_connect(srbd_ctx* c, const uint8_t* handles) {
    if (!c || !handles) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->xg_base) return fail(c, SRBD_E_STATE, "srbd_xgmi_export first");
    const int world = c->cfg.world_size > 0 ? c->cfg.world_size : 1;
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    float* bases[XCHG_MAX_WORLD] = {};
    for (int r = 0; r < world; ++r) {
        if (r == c->cfg.rank) {
            bases[r] = c->xg_base;
            continue;
        }
        hipIpcMemHandle_t h;
        memcpy(&h, handles + 64 * r, sizeof(h));
        void* p = nullptr;
        HIP_TRY(c, hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
        c->xg_opened.push_back(p);
        bases[r] = static_cast<float*>(p);
    }
    return xg_table(c, world, bases);
}

// All ranks' contexts live in this process (tests, or one process driving several GPUs).
extern "C" int srbd_xgmi_connect_local(srbd_ctx* const* ctxs, int32_t world) {
    if (!ctxs || world < 1 || world > XCHG_MAX_WORLD) return SRBD_E_INVALID;
    arm_cancel_others();
    float* bases[XCHG_MAX_WORLD] = {};
    for (int r = 0; r < world; ++r) {
        if (!ctxs[r] || !ctxs[r]->xg_base || ctxs[r]->cfg.rank != r || ctxs[r]->cfg.world_size != world)
            return fail(nullptr, SRBD_E_STATE, "every context must be srbd_xgmi_export'ed, rank r at index r");
        bases[r] = ctxs[r]->xg_base;
    }
    for (int r = 0; r < world; ++r)
        if (int rc = xg_table(ctxs[r], world, bases)) return rc;
    return SRBD_OK;
}

// Exercise the mailboxes once (every rank must call it; bounded wait).  *ok = 1 when every peer's
// word arrived.  The caller agrees across ranks and falls back to RCCL if any rank failed.
extern "C" int srbd_xgmi_probe(srbd_ctx* c, int32_t* ok) {
    if (!c || !ok) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->xg_world) return fail(c, SRBD_E_STATE, "srbd_xgmi_connect first");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    int* d_ok = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d_ok, sizeof(int)));
    launch_xchg_probe(c->xa, d_ok, c->stream);
    int h = 0;
    hipError_t e = hipMemcpyAsync(&h, d_ok, sizeof(int), hipMemcpyDeviceToHost, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d_ok);
    HIP_TRY(c, e);
    *ok = h;
    return SRBD_OK;
}

extern "C" int srbd_xgmi_disconnect(srbd_ctx* c) {
    if (!c) return SRBD_E_INVALID;
    arm_cancel(c);
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    for (void* p : c->xg_opened) (void)hipIpcCloseMemHandle(p);
    c->xg_opened.clear();
    c->xg_world = 0;
    xg_drop_graphs(c);
    return SRBD_OK;
}

// rollout (+ next draws) -> merge_xchg (rank record out to every mailbox, wait, merge the W records)
static void enqueue_xchg_step(srbd_ctx* c, int buf, StepOutput* out, int chain, bool fuse_next, Publish pub,
                              const void* ksi = nullptr) {
    const ModelConst& mc = c->mc;
    const RngJob next{c->d_noise[1 - buf], 0, 0, 1, 1};
    GroupArgs grp = grp_of(c);
    grp.ksi = ksi;  // the step input as the rollout's kernel argument (its block 0 writes the device copy)
    if (c->final_merge && !mc.ga && !mc.cost_on && out && !chain && pub.flag) {
        // host step: the rollout launch's final merger folds this rank's buffer, exchanges and merges (one launch)
        grp.out = out;
        grp.flag = pub.flag;
        grp.seq = pub.seq;
        grp.gdone = c->d_gdone;
        grp.ngroups = c->ngroups;
        grp.fence_sys = merge_fence_sys();
        grp.xa = c->d_xa;
        grp.levels_up = levels_up(c);
        launch_rollout(mc, c->d_in, c->d_noise[buf], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                       c->stream, fuse_next ? &next : nullptr, grp);
        return;
    }
    launch_rollout(mc, c->d_in, c->d_noise[buf], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                   c->stream, fuse_next ? &next : nullptr, grp);
    launch_merge_xchg(mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, c->d_noise[buf], c->xa, out, chain,
                      c->stream, 1, pub, levels_up(c));
}

// Device-resident exchange chain as replayed graphs (the epoch lives on the device, so a replay is a
// valid next exchange): two steps per graph alternating the noise buffers when the next draws fuse
// into the rollout launch, one-step graph for an odd count.
static int xg_capture(srbd_ctx* c) {
    const bool fuse = fusable(c);
    hipGraph_t g;
    HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    for (int half = 0; half < 2; ++half) {
        if (!fuse) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);
        enqueue_xchg_step(c, fuse ? half : 0, c->d_out, 1, fuse, Publish{nullptr, 0});
    }
    HIP_TRY(c, hipStreamEndCapture(c->stream, &g));
    hipError_t e = hipGraphInstantiate(&c->g_xg2, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_TRY(c, e);
    HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    if (!fuse) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);
    enqueue_xchg_step(c, 0, c->d_out, 1, fuse, Publish{nullptr, 0});
    HIP_TRY(c, hipStreamEndCapture(c->stream, &g));
    e = hipGraphInstantiate(&c->g_xg1, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_TRY(c, e);
    return SRBD_OK;
}

static int xg_device_steps(srbd_ctx* c, int steps) {
    int rc;
    if (!c->g_xg2 && (rc = xg_capture(c))) return rc;
    c->pref_valid = false;
    if ((rc = reset_noise_scaled(c))) return rc;
    if (fusable(c)) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);  // first step's draws
    for (int i = 0; i < steps / 2; ++i) HIP_TRY(c, hipGraphLaunch(c->g_xg2, c->stream));
    if (steps & 1) HIP_TRY(c, hipGraphLaunch(c->g_xg1, c->stream));
    c->cur = 0;
    return SRBD_OK;
}

static int xg_check_err(srbd_ctx* c) {
    int e = 0;
    HIP_TRY(c, hipMemcpy(&e, c->xg_err, sizeof(int), hipMemcpyDeviceToHost));
    return e ? fail(c, SRBD_E_HIP, "xGMI exchange timed out waiting for a peer's record") : SRBD_OK;
}

static int xg_step(srbd_ctx* c, const float* state, const float* ref, const float* contact, int32_t contact_stride,
                   float* best, float* sigma, const float* noise_local, uint64_t seed, uint64_t counter,
                   srbd_result* out, float* out_costs_local) {
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    int rc = fill_input(&c->cfg, c->mc, c->h_in, state, ref, contact, contact_stride, best, sigma, seed, counter);
    if (rc) return fail(c, rc, "invalid step arguments");
    c->h_in->noise_scaled = noise_local ? 1 : 0;
    StepInputK ksi;  // as srbd_step: the rollout's kernel argument, or the upload kernel
    const bool ks = c->ks && !c->mc.ga && !c->mc.cost_on;
    if (ks)
        fill_ksi(c, &ksi);
    else if ((rc = upload_input(c)))
        return rc;
    int buf = 0;
    if ((rc = acquire_noise(c, noise_local, seed, counter, &buf))) return rc;
    const bool fuse = !noise_local && fusable(c);
    const Publish pub{c->d_flag, ++c->seq};
    c->h_out->status = 0;  // check_handoff / the exchange's -1
    enqueue_xchg_step(c, buf, c->d_out_host, 0, fuse, pub, ks ? &ksi : nullptr);
    HIP_TRY(c, hipGetLastError());
    if (fuse) {
        c->pref_valid = true;
        c->pref_buf = 1 - buf;
        c->pref_seed = next_seed(c, seed);
        c->pref_ctr = counter + 1;
    }
    c->chain_started = false;
    c->input_ready = true;
    if ((rc = wait_published(c, pub.seq))) return rc;
    if (c->h_out->status != 0) return xg_check_err(c) ? SRBD_E_HIP : check_handoff(c);
    if (out_costs_local) {
        HIP_TRY(c, hipMemcpyAsync(out_costs_local, c->d_costs, sizeof(float) * c->mc.n_local, hipMemcpyDeviceToHost,
                                  c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
    }
    return copy_out(c, best, sigma, out);
}

// One host-driven sharded step (Sampling_MPC call) with the exchange inside: the rank's rows, the
// rank records exchanged (xGMI mailboxes when connected, else ncclAllGather), the merge; outputs
// identical on every rank.
extern "C" int srbd_step_sharded(srbd_ctx* c, const float* state, const float* ref, const float* contact,
                                 int32_t contact_stride, float* best, float* sigma, const float* noise_local,
                                 uint64_t seed, uint64_t counter, srbd_result* out, float* out_costs_local) {
    if (!c || !best) return SRBD_E_INVALID;
    arm_cancel(c);
    if (c->xg_world)
        return xg_step(c, state, ref, contact, contact_stride, best, sigma, noise_local, seed, counter, out,
                       out_costs_local);
    if (!c->comm) return fail(c, SRBD_E_STATE, "srbd_comm_init or srbd_xgmi_connect first");
    int rc = srbd_step_local(c, state, ref, contact, contact_stride, best, sigma, noise_local, seed, counter,
                             c->d_myrec);
    if (rc) return rc;
    if ((rc = gather_records(c))) return rc;
    return srbd_step_finish(c, c->d_gath, c->comm_world, best, sigma, out, out_costs_local);
}

// `steps` device-resident sharded steps (warm start kept on the device), elapsed ms by hipEvents.
extern "C" int srbd_sharded_device_steps(srbd_ctx* c, int32_t steps, float* elapsed_ms) {
    if (!c || steps < 1) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->xg_world && !c->comm) return fail(c, SRBD_E_STATE, "srbd_comm_init or srbd_xgmi_connect first");
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run a host step first");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    hipEvent_t e0, e1;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    HIP_TRY(c, hipEventRecord(e0, c->stream));
    int rc = SRBD_OK;
    if (c->xg_world) {
        rc = xg_device_steps(c, steps);
    } else {
        for (int i = 0; i < steps && !rc; ++i) {
            rc = srbd_device_step_local(c, c->d_myrec);
            if (!rc) rc = gather_records(c);
            if (!rc) rc = srbd_device_step_finish(c, c->d_gath, c->comm_world);
        }
    }
    HIP_TRY(c, hipEventRecord(e1, c->stream));
    HIP_TRY(c, hipEventSynchronize(e1));
    float ms = 0.0f;
    HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (elapsed_ms) *elapsed_ms = ms;
    if (!rc && c->xg_world) rc = xg_check_err(c);
    return rc;
}

// ------------------------------------------------------------------ checkpoint
// The evolving state of a context is what its device-resident steps start from: the device copy of
// the warm start (best[P]), sigma[P] (CEM) and the RNG key (seed, counter) in StepInput.  Host steps
// take all of it as arguments (the Python Sampling_MPC keeps it: best_control_parameters,
// sigma_cem_mppi, master_key), so a checkpoint of a host-driven controller is those arguments; this
// pair covers the device-resident chains (srbd_bench_device_steps, srbd_sharded_device_steps,
// srbd_device_step_local), whose warm start never leaves the device.
extern "C" int srbd_get_state(srbd_ctx* c, float* best, float* sigma, uint64_t* seed, uint64_t* counter) {
    if (!c || !best) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "no state yet: run srbd_step (or srbd_set_state) first");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    StepInput* h = c->h_in;  // staging: overwritten by the next host step anyway
    HIP_TRY(c, hipMemcpy(h, c->d_in, sizeof(StepInput), hipMemcpyDeviceToHost));
    memcpy(best, h->best, sizeof(float) * c->mc.P);
    if (sigma && c->mc.method == SRBD_CEM_MPPI) memcpy(sigma, h->sigma, sizeof(float) * c->mc.P);
    if (seed) *seed = ((uint64_t)h->seed_hi << 32) | h->seed_lo;
    if (counter) *counter = ((uint64_t)h->ctr_hi << 32) | h->ctr_lo;
    return SRBD_OK;
}

extern "C" int srbd_set_state(srbd_ctx* c, const float* best, const float* sigma, uint64_t seed, uint64_t counter) {
    if (!c || !best) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step once first (it sets the state/reference inputs)");
    if (c->mc.method == SRBD_CEM_MPPI && !sigma) return fail(c, SRBD_E_INVALID, "CEM: sigma is part of the state");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    HIP_TRY(c, hipStreamSynchronize(c->stream));
    StepInput* h = c->h_in;
    HIP_TRY(c, hipMemcpy(h, c->d_in, sizeof(StepInput), hipMemcpyDeviceToHost));
    memcpy(h->best, best, sizeof(float) * c->mc.P);
    if (c->mc.method == SRBD_CEM_MPPI) memcpy(h->sigma, sigma, sizeof(float) * c->mc.P);
    h->seed_lo = (uint32_t)seed;
    h->seed_hi = (uint32_t)(seed >> 32);
    h->ctr_lo = (uint32_t)counter;
    h->ctr_hi = (uint32_t)(counter >> 32);
    h->noise_scaled = 0;  // device-resident steps draw on the device
    HIP_TRY(c, hipMemcpy(c->d_in, h, sizeof(StepInput), hipMemcpyHostToDevice));
    c->pref_valid = false;  // no prefetched draws belong to the restored key
    return SRBD_OK;
}

// ------------------------------------------------------------------ measurement
// Device-resident chain (benchmark): two steps per graph, each step's rollout launch also drawing
// the next step's noise into the other buffer (device counter + 1), each merge writing the warm
// start back and advancing the counter.  CEM (draws depend on the new sigma): draws inline.
static int capture_dev_graphs(srbd_ctx* c) {
    hipGraph_t g;
    const bool fuse = fusable(c);
    HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    for (int half = 0; half < 2; ++half) {
        const int buf = fuse ? half : 0;
        if (!fuse) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);
        enqueue_device_step(c, buf, nullptr, c->d_out, /*chain=*/1, /*ctr_inc=*/1, fuse);
    }
    HIP_TRY(c, hipStreamEndCapture(c->stream, &g));
    hipError_t e = hipGraphInstantiate(&c->g_dev2, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_TRY(c, e);
    HIP_TRY(c, hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    if (!fuse) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);
    enqueue_device_step(c, 0, nullptr, c->d_out, 1, 1, fuse);
    HIP_TRY(c, hipStreamEndCapture(c->stream, &g));
    e = hipGraphInstantiate(&c->g_dev1, g, nullptr, nullptr, 0);
    (void)hipGraphDestroy(g);
    HIP_TRY(c, e);
    return SRBD_OK;
}

extern "C" int srbd_bench_device_steps(srbd_ctx* c, int32_t steps, float* ms) {
    if (!c || steps < 1 || !ms) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step once before benchmarking");
    if (c->cfg.world_size > 1 || !c->own_stream) return fail(c, SRBD_E_STATE, "needs an unsharded, own-stream context");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    c->pref_valid = false;
    int rc;
    if (!c->g_dev2 && (rc = capture_dev_graphs(c))) return rc;
    if ((rc = reset_noise_scaled(c))) return rc;
    hipEvent_t e0, e1;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    HIP_TRY(c, hipEventRecord(e0, c->stream));
    if (fusable(c)) launch_rng(c->mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream);  // first step's draws
    for (int i = 0; i < steps / 2; ++i) HIP_TRY(c, hipGraphLaunch(c->g_dev2, c->stream));
    if (steps & 1) HIP_TRY(c, hipGraphLaunch(c->g_dev1, c->stream));
    HIP_TRY(c, hipEventRecord(e1, c->stream));
    HIP_TRY(c, hipEventSynchronize(e1));
    HIP_TRY(c, hipEventElapsedTime(ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    c->cur = 0;
    return SRBD_OK;
}

// Host-to-host srbd_step latency at the C-ABI boundary: `steps` calls cycling through n_in input sets
// (state / ref 24 floats, contact 4 x stride each), the warm start fed back, counters consecutive from
// counter0 and (JAX stream) each key with_newkey of the last (so the fused next-step draws are used, as a
// controller at 100 Hz does); each call timed with the steady clock.  lat_us: `steps` floats.  sigma: CEM
// in/out or NULL.
extern "C" int srbd_bench_host_steps(srbd_ctx* c, const float* state, const float* ref, const float* contact,
                                     int32_t contact_stride, int32_t n_in, float* best, float* sigma, uint64_t seed,
                                     uint64_t counter0, int32_t steps, float* lat_us) {
    if (!c || !state || !ref || !contact || !best || !lat_us || n_in < 1 || steps < 1) return SRBD_E_INVALID;
    srbd_result res;
    for (int32_t i = 0; i < steps; ++i, seed = next_seed(c, seed)) {
        const int k = i % n_in;
        const auto t0 = std::chrono::steady_clock::now();
        const float* st = state + 24 * k;
        const float* rf = ref + 24 * k;
        const float* ct = contact + (size_t)4 * contact_stride * k;
        const uint64_t ctr = counter0 + (uint64_t)i;
        const int rc = c->cfg.world_size > 1  // the library-owned exchange (xGMI mailboxes or RCCL)
                           ? srbd_step_sharded(c, st, rf, ct, contact_stride, best, sigma, nullptr, seed, ctr, &res,
                                               nullptr)
                           : srbd_step(c, st, rf, ct, contact_stride, best, sigma, nullptr, seed, ctr, &res, nullptr);
        const auto t1 = std::chrono::steady_clock::now();
        if (rc) return rc;
        lat_us[i] = std::chrono::duration<float, std::micro>(t1 - t0).count();
    }
    return SRBD_OK;
}

extern "C" int srbd_time_kernels(srbd_ctx* c, int32_t iters, float* rollout_us, float* rng_us, float* reduce_us,
                                 float* fused_us, float* floor_us) {
    arm_cancel(c);
    // Average duration of each kernel of the step from ONE event pair around `iters` back-to-back
    // launches of it on the context stream: the per-launch figure then carries no event/dispatch
    // overhead of its own (an event pair around a single launch adds ~6 us at this size) and agrees
    // with rocprofv3's kernel-trace average (profiles/).  The empty-kernel row (floor) is the same
    // measurement of a kernel that does nothing: launch-to-launch spacing only.
    if (!c || iters < 1) return SRBD_E_INVALID;
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step once before timing");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    c->pref_valid = false;
    c->cur = 0;
    if (int rc = reset_noise_scaled(c)) return rc;
    const ModelConst& mc = c->mc;
    hipEvent_t e0, e1;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    auto timed = [&](auto&& launch, float* us) -> int {
        launch();  // warm: first-launch code object / kernarg setup stays outside
        HIP_TRY(c, hipEventRecord(e0, c->stream));
        for (int i = 0; i < iters; ++i) launch();
        HIP_TRY(c, hipEventRecord(e1, c->stream));
        HIP_TRY(c, hipEventSynchronize(e1));
        float ms = 0.0f;
        HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
        if (us) *us = ms * 1000.0f / (float)iters;
        return SRBD_OK;
    };
    int rc = SRBD_OK;
    if (!rc) rc = timed([&] { launch_rng(mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream); }, rng_us);
    if (!rc)
        rc = timed([&] {
            launch_rollout(mc, c->d_in, c->d_noise[0], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                           c->stream, nullptr, grp_of(c));
        }, rollout_us);
    if (!rc)
        rc = timed([&] {
            launch_merge(mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, 0, c->d_noise[0], nullptr, c->d_out,
                         0, c->stream);
        }, reduce_us);
    // the launch the step actually runs when fusion applies: rollout + the next step's draws
    if (fused_us) *fused_us = 0.0f;
    if (!rc && fusable(c)) {
        const RngJob next{c->d_noise[1], 0, 0, 1, 1};
        rc = timed([&] {
            launch_rollout(mc, c->d_in, c->d_noise[0], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                           c->stream, &next, grp_of(c));
        }, fused_us);
    }
    if (!rc) rc = timed([&] { launch_empty(c->stream); }, floor_us);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (!rc) HIP_TRY(c, hipGetLastError());
    return rc;
}

// Average duration of ONE kind of launch, `iters` back to back between one hipEvent pair (as srbd_time_kernels),
// so a rocprofv3 pass over this call sees only that launch (a PMC A/B of two launches of one kernel name).
//   SRBD_TL_STEP_ROLLOUT: the rollout launch exactly as srbd_step issues it -- the step input by value (KS), the
//     in-launch final merge (FM, publishing into the host-mapped outputs) and the next step's draws (fused) where
//     they apply; *form = 1 fused | 2 KS | 4 FM | 8 thread-per-sample rollout (else four lanes per sample) |
//     16 fast_tail | 32 the step's draws made in the launch (gen_now: srbd_step issues no RNG launch).
//   SRBD_TL_STEP_MERGE: the merge launch srbd_step issues after it (0 us when the rollout launch merges).
extern "C" int srbd_time_launch(srbd_ctx* c, int32_t which, int32_t iters, float* us, int32_t* form) {
    if (!c || iters < 1 || !us) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step once before timing");
    if (c->cfg.world_size > 1) return fail(c, SRBD_E_STATE, "needs an unsharded context");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    c->pref_valid = false;
    c->cur = 0;
    if (int rc = reset_noise_scaled(c)) return rc;
    const ModelConst& mc = c->mc;
    const bool ks = c->ks && !mc.ga && !mc.cost_on;
    const bool fm = c->final_merge && !mc.ga && !mc.cost_on;
    const bool gen = gen_now(c) && ks;
    const bool fuse = fusable(c) && !gen;
    StepInputK ksi;
    if (ks) fill_ksi(c, &ksi);
    if (form)
        *form = (which == SRBD_TL_STEP_ROLLOUT)
                    ? ((fuse ? 1 : 0) | (ks ? 2 : 0) | (fm ? 4 : 0) | (c->mode == ROLLOUT_THREAD ? 8 : 0) |
                       (fm && c->fast_tail ? 16 : 0) | (gen ? 32 : 0))
                    : 0;
    const RngJob next{c->d_noise[1], 0, 0, 1, 1, nullptr};
    int nflags = 0;  // publish flags of the last launch (0: it publishes nothing)
    auto launch = [&]() {
        switch (which) {
            case SRBD_TL_RNG: launch_rng(mc, c->d_in, 0, 0, 1, 0, c->d_noise[0], c->stream); break;
            case SRBD_TL_ROLLOUT:
            case SRBD_TL_ROLLOUT_FUSED:
                launch_rollout(mc, c->d_in, c->d_noise[0], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                               c->stream, which == SRBD_TL_ROLLOUT_FUSED && fuse ? &next : nullptr, grp_of(c));
                break;
            case SRBD_TL_STEP_ROLLOUT: {
                GroupArgs grp = grp_of(c);
                grp.ksi = ks ? &ksi : nullptr;
                grp.gen = gen ? 1 + c->gen_rg : 0;
                if (fm) {
                    grp.out = c->d_out_host;
                    grp.flag = c->d_flag;
                    grp.seq = ++c->seq;
                    grp.gdone = c->d_gdone;
                    grp.ngroups = c->ngroups;
                    grp.fence_sys = merge_fence_sys();
                    if (c->fast_tail) {
                        grp.fast = 1;
                        grp.gtag = c->d_gtag;
                    }
                }
                launch_rollout(mc, c->d_in, c->d_noise[0], c->d_costs, c->d_wrec, c->wrec_stride, c->mode, c->threads,
                               c->stream, fuse ? &next : nullptr, grp);
                nflags = fm ? 1 : 0;
                break;
            }
            case SRBD_TL_STEP_MERGE:
                nflags = launch_merge(mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, 0, c->d_noise[0],
                                      nullptr, c->d_out_host, 0, c->stream, nullptr, 0,
                                      Publish{c->d_flag, ++c->seq, nullptr});
                break;
            default: launch_empty(c->stream); break;
        }
    };
    if (which < SRBD_TL_RNG || which > SRBD_TL_EMPTY) return fail(c, SRBD_E_INVALID, "unknown launch");
    if (which == SRBD_TL_STEP_MERGE && fm) {
        *us = 0.0f;
        return SRBD_OK;
    }
    hipEvent_t e0, e1;
    HIP_TRY(c, hipEventCreate(&e0));
    HIP_TRY(c, hipEventCreate(&e1));
    launch();  // warm
    HIP_TRY(c, hipEventRecord(e0, c->stream));
    for (int i = 0; i < iters; ++i) launch();
    HIP_TRY(c, hipEventRecord(e1, c->stream));
    HIP_TRY(c, hipEventSynchronize(e1));
    float ms = 0.0f;
    HIP_TRY(c, hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    HIP_TRY(c, hipGetLastError());
    *us = ms * 1000.0f / (float)iters;
    if (nflags > 0) return wait_published(c, c->seq, nflags);  // the launches published into h_flag
    return SRBD_OK;
}

// Diagnostic: average duration (us) of the merge kernel's phases from s_memrealtime stamps (100 MHz):
// [min key, weighted sums, elite, outputs, tail].
extern "C" int srbd_debug_merge_phases(srbd_ctx* c, int32_t iters, float* out_us) {
    if (!c || iters < 1 || !out_us) return SRBD_E_INVALID;
    arm_cancel(c);
    if (!c->input_ready) return fail(c, SRBD_E_STATE, "run srbd_step once first");
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    uint64_t* d = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d, 64 * sizeof(uint64_t)));
    HIP_TRY(c, hipMemsetAsync(d, 0, 64 * sizeof(uint64_t), c->stream));
    double acc[48] = {};
    for (int i = 0; i < iters; ++i) {
        launch_merge(c->mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, 0, c->d_noise[c->cur], nullptr,
                     c->d_out, 0, c->stream, d);
        uint64_t hh[64];
        HIP_TRY(c, hipMemcpyAsync(hh, d, sizeof(hh), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(c, hipStreamSynchronize(c->stream));
        for (int b = 0; b < 2; ++b) {  // block 0, block 1 (a column-split merge's first slice block)
            const uint64_t* h = hh + 32 * b;
            double* a = acc + 24 * b;
            if (!h[0]) continue;
            for (int k = 0; k < 5; ++k) a[k] += (double)(h[k + 1] - h[k]) * 0.01;  // 100 MHz ticks -> us
            // staged merge: records in LDS, tail lanes' force-independent step done (from the start)
            for (int k = 5; k < 7; ++k) a[k] += h[k + 1] > h[0] ? (double)(h[k + 1] - h[0]) * 0.01 : 0.0;
            // shader clock (MHz): s_memtime ticks over the same span as the 100 MHz s_memrealtime stamps
            a[7] += h[5] > h[0] ? (double)(h[9] - h[8]) / ((double)(h[5] - h[0]) * 0.01) : 0.0;
            for (int k = 0; k < 16; ++k) a[8 + k] += h[16 + k] > h[0] ? (double)(h[16 + k] - h[0]) * 0.01 : 0.0;
        }
        HIP_TRY(c, hipMemsetAsync(d, 0, 64 * sizeof(uint64_t), c->stream));
    }
    (void)hipFree(d);
    for (int k = 0; k < 48; ++k) out_us[k] = (float)(acc[k] / iters);
    return SRBD_OK;
}

extern "C" int srbd_selftest_div(const float* a, const float* b, int32_t n, float* out_host, float* out_dev) {
    if (!a || !b || n < 0) return SRBD_E_INVALID;
    if (out_host)
        for (int i = 0; i < n; ++i) out_host[i] = b[i] == 3.0f ? div3(a[i]) : div_by(a[i], b[i], 1.0f / b[i]);
    if (out_dev) {
        float *da = nullptr, *db = nullptr, *dout = nullptr;
        const size_t bytes = sizeof(float) * (size_t)(n > 0 ? n : 1);
        if (hipMalloc((void**)&da, bytes) != hipSuccess || hipMalloc((void**)&db, bytes) != hipSuccess ||
            hipMalloc((void**)&dout, bytes) != hipSuccess)
            return fail(nullptr, SRBD_E_NODEVICE, "device unavailable");
        (void)hipMemcpy(da, a, bytes, hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b, bytes, hipMemcpyHostToDevice);
        launch_div_selftest(da, db, n, dout, nullptr);
        hipError_t e = hipMemcpy(out_dev, dout, bytes, hipMemcpyDeviceToHost);
        (void)hipFree(da);
        (void)hipFree(db);
        (void)hipFree(dout);
        if (e != hipSuccess) return fail(nullptr, SRBD_E_HIP, hipGetErrorString(e));
    }
    return SRBD_OK;
}

// The JAX normal's log1p (srbd_jaxrng.h log1p_fast) on the host and / or the device; *nfallback (host) counts the
// arguments the float64 log1p decided.
extern "C" int srbd_selftest_log1p(const float* t, int32_t n, float* out_host, float* out_dev, int64_t* nfallback) {
    if (!t || n < 0) return SRBD_E_INVALID;
    if (out_host) {
        int64_t fb = 0;
        for (int i = 0; i < n; ++i) {
            float f;
            if (!log1p_try(t[i], &f)) {
                f = log1p_cr(t[i]);
                ++fb;
            }
            out_host[i] = f;
        }
        if (nfallback) *nfallback = fb;
    }
    if (out_dev) {
        float *dt = nullptr, *dout = nullptr;
        const size_t bytes = sizeof(float) * (size_t)(n > 0 ? n : 1);
        if (hipMalloc((void**)&dt, bytes) != hipSuccess || hipMalloc((void**)&dout, bytes) != hipSuccess)
            return fail(nullptr, SRBD_E_NODEVICE, "device unavailable");
        (void)hipMemcpy(dt, t, bytes, hipMemcpyHostToDevice);
        launch_log1p_selftest(dt, n, dout, nullptr);
        hipError_t e = hipMemcpy(out_dev, dout, bytes, hipMemcpyDeviceToHost);
        (void)hipFree(dt);
        (void)hipFree(dout);
        if (e != hipSuccess) return fail(nullptr, SRBD_E_HIP, hipGetErrorString(e));
    }
    return SRBD_OK;
}

// ------------------------------------------------------------------ TAMOLS
// One call = one launch (tamols_fused_kernel): the patches are raycast (or read from host-mapped
// staging), scored and reduced on the device; the outputs land in host-mapped memory and the call
// spins on a host-mapped sequence word, so there is no copy command and no stream synchronise.
struct srbd_tamols_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // host-mapped output block [scores 4 nc | footholds 12 | boxes 24 | seed heights 4 | valid 4 x int32]
    double* h_out = nullptr;
    double* d_out_host = nullptr;
    double* h_hm = nullptr;  // host-mapped heightmaps: in (srbd_tamols_run) or out (run_terrain)
    double* d_hm_host = nullptr;
    double* d_part = nullptr;  // per-block partials
    unsigned* d_cnt = nullptr;  // block / leg counters, [4] the feed's leg arrivals (zero between calls)
    double* d_feed = nullptr;   // the feed's footholds (srbd_foothold_mpc_step's chained form)
    uint64_t* h_outt = nullptr;  // host-mapped tagged outputs, 4 x TAMOLS_OUT_WORDS (tamols_leg_out)
    uint64_t* d_outt = nullptr;
    uint32_t seq = 0;
    size_t cap_cand = 0;
    uint64_t* d_dbg = nullptr;  // srbd_tamols_phases: stamps of the last call
    std::string err;
};

extern "C" int srbd_tamols_create(int32_t device_id, srbd_tamols_ctx** out) {
    if (!out) return SRBD_E_INVALID;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0 || device_id < 0 || device_id >= ndev)
        return fail(nullptr, SRBD_E_NODEVICE, "no HIP device visible (this library has no CPU fallback)");
    srbd_tamols_ctx* t = new srbd_tamols_ctx();
    t->device = device_id;
    bool ok = hipSetDevice(device_id) == hipSuccess &&
              hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) == hipSuccess &&
              hipHostMalloc((void**)&t->h_outt, sizeof(uint64_t) * 4 * TAMOLS_OUT_WORDS,
                            hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess &&
              hipHostGetDevicePointer((void**)&t->d_outt, t->h_outt, 0) == hipSuccess &&
              hipMalloc((void**)&t->d_part, sizeof(double) * 4 * TAMOLS_BPL * 4) == hipSuccess &&
              hipMalloc((void**)&t->d_cnt, sizeof(unsigned) * 8) == hipSuccess &&
              hipMemset(t->d_cnt, 0, sizeof(unsigned) * 8) == hipSuccess &&
              hipMalloc((void**)&t->d_feed, sizeof(double) * 12) == hipSuccess && tamols_prepare() == 0 &&
              hipDeviceSynchronize() == hipSuccess;
    if (!ok) {
        srbd_tamols_destroy(t);
        return fail(nullptr, SRBD_E_HIP, "TAMOLS context allocation failed");
    }
    for (int w = 0; w < 4 * TAMOLS_OUT_WORDS; ++w) __atomic_store_n(t->h_outt + w, (uint64_t)0, __ATOMIC_RELEASE);
    *out = t;
    return SRBD_OK;
}

extern "C" void srbd_tamols_destroy(srbd_tamols_ctx* t) {
    if (!t) return;
    arm_cancel_others();
    (void)hipSetDevice(t->device);
    if (t->stream) (void)hipStreamSynchronize(t->stream);
    (void)hipFree(t->d_part);
    (void)hipFree(t->d_cnt);
    (void)hipFree(t->d_feed);
    (void)hipFree(t->d_dbg);
    if (t->h_out) (void)hipHostFree(t->h_out);
    if (t->h_hm) (void)hipHostFree(t->h_hm);
    if (t->h_outt) (void)hipHostFree(t->h_outt);
    if (t->stream) (void)hipStreamDestroy(t->stream);
    delete t;
}

extern "C" const char* srbd_tamols_last_error(const srbd_tamols_ctx* t) {
    return t ? t->err.c_str() : g_last_error.c_str();
}

#define TAM_TRY(t, expr)                                                                            \
    do {                                                                                            \
        hipError_t _e = (expr);                                                                     \
        if (_e != hipSuccess) {                                                                     \
            (t)->err = std::string(#expr) + ": " + hipGetErrorString(_e);                          \
            return SRBD_E_HIP;                                                                      \
        }                                                                                           \
    } while (0)

static int tamols_reserve(srbd_tamols_ctx* t, int nc) {
    if (t->cap_cand < (size_t)nc) {
        TAM_TRY(t, hipStreamSynchronize(t->stream));
        if (t->h_out) (void)hipHostFree(t->h_out);
        if (t->h_hm) (void)hipHostFree(t->h_hm);
        t->h_out = t->h_hm = t->d_out_host = t->d_hm_host = nullptr;
        t->cap_cand = 0;
        const size_t out_doubles = 4 * (size_t)nc + 12 + 24 + 4 + 2;
        const unsigned fl = hipHostMallocMapped | hipHostMallocCoherent;
        TAM_TRY(t, hipHostMalloc((void**)&t->h_out, sizeof(double) * out_doubles, fl));
        TAM_TRY(t, hipHostGetDevicePointer((void**)&t->d_out_host, t->h_out, 0));
        TAM_TRY(t, hipHostMalloc((void**)&t->h_hm, sizeof(double) * 4 * 3 * nc, fl));
        TAM_TRY(t, hipHostGetDevicePointer((void**)&t->d_hm_host, t->h_hm, 0));
        t->cap_cand = nc;
    }
    return SRBD_OK;
}

// One call's arguments, output pointers and sequence number.
static void tamols_job_fill(srbd_tamols_ctx* t, TamolsJob& j, const double* seeds, const double* hips,
                            const double* vel, const double* base, const int32_t* contact, const double* feet,
                            const srbd_tamols_params* p, int rows, int cols, bool scores) {
    const int nc = rows * cols;
    TamolsArgs& a = j.a;
    memset(&a, 0, sizeof(a));
    a.rows = rows;
    a.cols = cols;
    a.ncand = nc;
    a.has_vel = vel != nullptr;
    a.has_base = base != nullptr;
    a.has_feet = feet != nullptr;
    for (int i = 0; i < 4; ++i) a.contact[i] = contact ? contact[i] : 0;
    for (int i = 0; i < 3; ++i) {
        a.vel[i] = vel ? vel[i] : 0.0;
        a.base[i] = base ? base[i] : 0.0;
    }
    for (int i = 0; i < 12; ++i) {
        a.feet[i] = feet ? feet[i] : 0.0;
        a.seeds[i] = seeds[i];
        a.hips[i] = hips[i];
    }
    a.p = *p;
    j.rows = rows;
    j.cols = cols;
    j.scores = scores ? t->d_out_host : nullptr;
    j.outt = t->d_outt;
    j.part = t->d_part;
    j.cnt = t->d_cnt;
    j.seq = ++t->seq;
    j.dbg = t->d_dbg;
}

// Every leg's output words carry the call's number (a word is one 8-byte store: a tagged word holds that call's value;
// checked from each leg's last word, the one the leg stores last in lane order).
static bool tamols_published(const srbd_tamols_ctx* t, uint32_t seq) {
    for (int l = 0; l < 4; ++l)
        for (int w = TAMOLS_OUT_USED - 1; w >= 0; --w)
            if ((uint32_t)(__atomic_load_n(t->h_outt + l * TAMOLS_OUT_WORDS + w, __ATOMIC_ACQUIRE) >> 32) != seq)
                return false;
    return true;
}

// The outputs of a published call (host-mapped) into the caller's arrays.
static void tamols_outputs(const srbd_tamols_ctx* t, int nc, double* out_fh, double* out_box, int32_t* out_valid,
                           double* out_scores, double* out_seedh) {
    for (int l = 0; l < 4; ++l) {
        const uint64_t* w = t->h_outt + l * TAMOLS_OUT_WORDS;
        const auto dbl = [&](int k) {  // double k of the leg's words (low half first)
            const uint64_t b = (w[2 * k] & 0xFFFFFFFFull) | (w[2 * k + 1] << 32);
            double d;
            memcpy(&d, &b, sizeof(d));
            return d;
        };
        for (int k = 0; k < 3; ++k) out_fh[3 * l + k] = dbl(k);
        for (int k = 0; k < 6; ++k) out_box[6 * l + k] = dbl(3 + k);
        if (out_seedh) out_seedh[l] = dbl(9);
        out_valid[l] = (int32_t)(uint32_t)w[20];
    }
    if (out_scores) memcpy(out_scores, t->h_out, sizeof(double) * 4 * nc);
}

// Launch one call and wait for its published sequence number (bounded: the stream is polled now and
// then, so a fault or a launch failure surfaces as an error instead of a hang).
static int tamols_launch_wait(srbd_tamols_ctx* t, TamolsJob& j, const double* seeds, const double* hips,
                              const double* vel, const double* base, const int32_t* contact, const double* feet,
                              const srbd_tamols_params* p, int rows, int cols, double* out_fh, double* out_box,
                              int32_t* out_valid, double* out_scores, double* out_seedh) {
    tamols_job_fill(t, j, seeds, hips, vel, base, contact, feet, p, rows, cols, out_scores != nullptr);
    launch_tamols_fused(j, t->stream);
    TAM_TRY(t, hipGetLastError());
    for (uint64_t it = 1;; ++it) {
        if (tamols_published(t, j.seq)) break;
        if ((it & 4095) == 0) {
            const hipError_t e = hipStreamQuery(t->stream);
            if (e == hipSuccess) {
                if (tamols_published(t, j.seq)) break;
                t->err = "TAMOLS launch completed without publishing its outputs";
                return SRBD_E_HIP;
            }
            if (e != hipErrorNotReady) TAM_TRY(t, e);
        }
        __builtin_ia32_pause();
    }
    tamols_outputs(t, rows * cols, out_fh, out_box, out_valid, out_scores, out_seedh);
    return SRBD_OK;
}

// The raycast patches' part of a terrain job: centres = the seeds, one yaw.
static void tamols_terrain_job(TamolsJob& j, const srbd_terrain* ter, double yaw, double dist_x, double dist_y,
                               double ray_z) {
    j.use_terrain = 1;
    j.t = ter->dev;
    j.yaw_c = cos(yaw);  // the same host cos / sin terrain_enqueue forms for a patch's yaw
    j.yaw_s = sin(yaw);
    j.dist_x = dist_x;
    j.dist_y = dist_y;
    j.inv_dx = 1.0 / dist_x;
    j.inv_dy = 1.0 / dist_y;
    j.ray_z = ray_z;
    // the raycast patch is ray_xy's lattice: four points per nearest-neighbour query, one block per leg
    // (SRBD_TAMOLS_LATTICE=0: every point scanned, 16 blocks per leg -- the same results)
    const char* le = getenv("SRBD_TAMOLS_LATTICE");
    const bool lattice_env = !(le && le[0] == '0');
    j.lattice = lattice_env && std::isfinite(dist_x) && std::isfinite(dist_y) && dist_x > 0.0 && dist_y > 0.0 &&
                std::isfinite(j.yaw_c) && std::isfinite(j.yaw_s);
}

extern "C" int srbd_tamols_run(srbd_tamols_ctx* t, const double* hm, int32_t rows, int32_t cols, const double* seeds,
                               const double* hips, const double* vel, const double* base, const int32_t* contact,
                               const double* feet, const srbd_tamols_params* p, double* out_fh, double* out_box,
                               int32_t* out_valid, double* out_scores, double* out_seedh) {
    if (!t || !hm || !seeds || !hips || !p || !out_fh || !out_box || !out_valid) return SRBD_E_INVALID;
    arm_cancel_others();
    const int nc = rows * cols;
    if (rows < 1 || cols < 1 || nc > TAMOLS_MAXCAND) {
        t->err = "patch must have 1..320 points";
        return SRBD_E_INVALID;
    }
    TAM_TRY(t, hipSetDevice(t->device));
    if (int rc = tamols_reserve(t, nc)) return rc;
    memcpy(t->h_hm, hm, sizeof(double) * 12 * nc);  // the previous call has completed (it was waited for)
    TamolsJob j;
    memset(&j, 0, sizeof(j));
    j.use_terrain = 0;
    j.hm = t->d_hm_host;
    return tamols_launch_wait(t, j, seeds, hips, vel, base, contact, feet, p, rows, cols, out_fh, out_box, out_valid,
                              out_scores, out_seedh);
}

// TAMOLS on patches raycast from a device terrain in the same launch (centres = the seeds).
extern "C" int srbd_tamols_run_terrain(srbd_tamols_ctx* t, srbd_terrain* ter, double yaw, int32_t rows, int32_t cols,
                                       double dist_x, double dist_y, double ray_z, const double* seeds,
                                       const double* hips, const double* vel, const double* base,
                                       const int32_t* contact, const double* feet, const srbd_tamols_params* p,
                                       double* out_fh, double* out_box, int32_t* out_valid, double* out_scores,
                                       double* out_seedh, double* out_hm) {
    if (!t || !ter || !seeds || !hips || !p || !out_fh || !out_box || !out_valid) return SRBD_E_INVALID;
    arm_cancel_others();
    const int nc = rows * cols;
    if (rows < 1 || cols < 1 || nc > TAMOLS_MAXCAND) {
        t->err = "patch must have 1..320 points";
        return SRBD_E_INVALID;
    }
    if (ter->device != t->device) {
        t->err = "terrain and TAMOLS contexts are on different devices";
        return SRBD_E_INVALID;
    }
    TAM_TRY(t, hipSetDevice(t->device));
    if (int rc = tamols_reserve(t, nc)) return rc;
    TamolsJob j;
    memset(&j, 0, sizeof(j));
    tamols_terrain_job(j, ter, yaw, dist_x, dist_y, ray_z);
    j.hm_out = out_hm ? t->d_hm_host : nullptr;
    const int rc = tamols_launch_wait(t, j, seeds, hips, vel, base, contact, feet, p, rows, cols, out_fh, out_box,
                                      out_valid, out_scores, out_seedh);
    if (!rc && out_hm) memcpy(out_hm, t->h_hm, sizeof(double) * 12 * nc);
    return rc;
}

// srbd_foothold_mpc_step chained on the device (srbd_host.cpp calls this first; 1 = not taken, the caller runs the
// sequential chain).  The TAMOLS launch and the MPC step's rollout launch go onto the MPC context's stream back to
// back: the TAMOLS launch also writes the step's device StepInput (TamolsJob::Feed -- the reference's feet = the
// footholds, swing feet = the footholds, cost_feet), so the host waits once, for the step, instead of for TAMOLS,
// then staging the step, then for the step.  The inputs are the ones the sequential chain stages (fill_input over
// prepare_state's outputs rounded to float), so the results are the same bits (tests/test_gpu_foothold_step.py).
// Taken for unsharded, unarmed MPPI / random-sampling contexts without the gait-adaptive rollout or cost terms, the
// step input fitting the kernel argument (P <= KSI_MAXP); SRBD_FOOTHOLD_CHAIN=0 turns it off.
extern "C" int srbd_foothold_chain(srbd_tamols_ctx* t, srbd_terrain* ter, const srbd_tamols_params* p, srbd_ctx* c,
                                   srbd_foothold_io* io, const float* contact, int32_t stride, float* best,
                                   int32_t ppl, uint64_t seed, uint64_t counter, srbd_result* out) {
    constexpr int DECLINED = 1;
    const ModelConst& mc = c->mc;
    const char* env = getenv("SRBD_FOOTHOLD_CHAIN");
    if ((env && env[0] == '0') || c->cfg.world_size > 1 || c->arm_mode || mc.method == SRBD_CEM_MPPI || mc.ga ||
        mc.cost_on || mc.P > KSI_MAXP || t->device != c->cfg.device_id || ter->device != t->device)
        return DECLINED;
    const int rows = io->rows, cols = io->cols, nc = rows * cols;
    const int nwords = (int)((offsetof(StepInput, best) + sizeof(float) * (size_t)mc.P) / 16);
    if (rows < 1 || cols < 1 || nc > TAMOLS_MAXCAND || nwords > TAMOLS_THREADS || stride < mc.H) return DECLINED;
    for (int l = 0; l < 4; ++l)  // prepare_state's lift-off zeroing would index past best[P]
        if ((l + 1) * (size_t)ppl > (size_t)mc.P) return DECLINED;
    arm_cancel_others();
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    if (int rc = tamols_reserve(t, nc)) return fail(c, rc, t->err);
    // prepare_state's warm-start zeroing (NMPC:563-627) reads only the contacts; the feet it substitutes are the
    // footholds, written on the device by the feed
    for (int l = 0; l < 4; ++l)
        if (io->previous_contact[l] == 1.0 && io->current_contact[l] == 0.0)
            for (int k = 0; k < ppl; ++k) best[l * ppl + k] = 0.0f;
    float st[24], rf[24];
    for (int i = 0; i < 24; ++i) st[i] = (float)io->state_in[i];
    for (int i = 0; i < 12; ++i) {
        rf[i] = (float)io->ref_base[i];
        rf[12 + i] = 0.0f;  // the feed's
    }
    int rc = fill_input(&c->cfg, mc, c->h_in, st, rf, contact, stride, best, nullptr, seed, counter);
    if (rc) return fail(c, rc, "invalid step arguments");
    c->h_in->noise_scaled = 0;
    c->h_out->status = 0;  // check_handoff
    StepInputK ksi;
    fill_ksi(c, &ksi);
    int32_t cint[4];
    for (int l = 0; l < 4; ++l) cint[l] = (int32_t)io->current_contact[l];
    TamolsJob j;
    memset(&j, 0, sizeof(j));
    tamols_terrain_job(j, ter, io->yaw, io->dist_x, io->dist_y, io->ray_z);
    j.hm_out = io->heightmaps ? t->d_hm_host : nullptr;
    tamols_job_fill(t, j, io->seeds, io->hips, io->forward_vel, io->state_in, cint, io->state_in + 12, p, rows, cols,
                    io->scores != nullptr);
    j.feed.in = c->d_in;
    j.feed.fh = t->d_feed;
    j.feed.cnt = t->d_cnt + 4;
    j.feed.nwords = nwords;
    for (int l = 0; l < 4; ++l) j.feed.swing[l] = io->current_contact[l] == 0.0;
    for (int i = 0; i < 12; ++i) j.feed.q[i] = c->cfg.q_diag[12 + i];
    // cost_feet = sum (e q) e over the feet: with zero feet weights it is +0 whenever every e is finite -- the case
    // when the seeds, the state's feet, the patch geometry and the scene are bounded (the footholds, candidates or
    // seeds at raycast heights, then round to finite floats) -- so the host's value stands and each leg writes its
    // own feet; else the last leg sums it on the device
    {
        const auto ok = [](double v) { return std::isfinite(v) && fabs(v) < 1e30; };
        // a ray misses (miss_z) unless the ground plane lies at or below its start
        const bool hits = ter->dev.has_ground && ter->dev.ground_z <= io->ray_z;
        bool known = ter->bounded && ok(io->ray_z) && ok(io->dist_x * rows) && ok(io->dist_y * cols) &&
                     (hits || ok(ter->dev.miss_z));
        for (int i = 0; i < 12 && known; ++i)
            known = j.feed.q[i] == 0.0f && ok(io->seeds[i]) && ok(io->state_in[12 + i]);
        j.feed.cf_known = known;
        if (known) {  // fill_input's sum over the staged (finite) feet is +0 already; stated here
            const float z = 0.0f;
            c->h_in->cost_feet = z;
            memcpy(ksi.head + offsetof(StepInput, cost_feet), &z, sizeof(z));
        }
    }
    // the step's draws: the previous step's prefetch, else drawn now -- queued ahead of TAMOLS (they do not read it)
    int buf = 0;
    if ((rc = acquire_noise(c, nullptr, seed, counter, &buf))) return rc;
    launch_tamols_fused(j, c->stream, &ksi);
    HIP_TRY(c, hipGetLastError());
    const bool fuse = fusable(c);
    const Publish pub{c->d_flag, ++c->seq, nullptr};
    const int nflags = enqueue_device_step(c, buf, nullptr, c->d_out_host, 0, 0, fuse, pub);
    HIP_TRY(c, hipGetLastError());
    if (fuse) {
        c->pref_valid = true;
        c->pref_buf = 1 - buf;
        c->pref_seed = next_seed(c, seed);
        c->pref_ctr = counter + 1;
    }
    // a launch that stopped part-way can leave the feed's arrival count behind: cleared on every failure from here
    const auto failed = [&](int r) {
        (void)hipStreamSynchronize(c->stream);
        (void)hipMemset(t->d_cnt + 4, 0, sizeof(unsigned));
        return r;
    };
    if ((rc = nflags == TAGGED_OUT ? wait_tagged(c, pub.seq) : wait_published(c, pub.seq, nflags))) return failed(rc);
    if (!tamols_published(t, j.seq)) {  // stream order: TAMOLS completed before the step began
        (void)hipStreamSynchronize(c->stream);
        if (!tamols_published(t, j.seq))
            return failed(fail(c, SRBD_E_HIP, "TAMOLS launch completed without publishing its outputs"));
    }
    tamols_outputs(t, nc, io->footholds, io->boxes, io->valid, io->scores, io->seed_heights);
    if (io->heightmaps) memcpy(io->heightmaps, t->h_hm, sizeof(double) * 12 * nc);
    io->stage = 1;
    // prepare_state's outputs as the sequential chain reports them (the step used their float roundings)
    memcpy(io->ref_out, io->ref_base, sizeof(double) * 12);
    memcpy(io->ref_out + 12, io->footholds, sizeof(double) * 12);
    memcpy(io->state_out, io->state_in, sizeof(double) * 24);
    for (int l = 0; l < 4; ++l)
        if (io->current_contact[l] == 0.0) memcpy(io->state_out + 12 + 3 * l, io->footholds + 3 * l, sizeof(double) * 3);
    io->stage = 2;
    if ((rc = check_handoff(c))) return failed(rc);
    c->input_ready = true;
    copy_out(c, best, nullptr, out);
    io->stage = 3;
    ++c->foothold_chained;
    return SRBD_OK;
}

// Diagnostic: stamp the phases of the following calls (enable != 0), or read the last call's stamps:
// out_us[5] = the mean over blocks of (patch, queries, scores, count) durations and the span from the
// first block's start to the last leg's end (us, 100 MHz s_memrealtime).
extern "C" int srbd_tamols_phases(srbd_tamols_ctx* t, int32_t enable, float* out_us) {
    if (!t) return SRBD_E_INVALID;
    arm_cancel_others();
    TAM_TRY(t, hipSetDevice(t->device));
    const size_t n = 4 * TAMOLS_BPL * 8;
    if (enable && !t->d_dbg) {
        TAM_TRY(t, hipMalloc((void**)&t->d_dbg, sizeof(uint64_t) * n));
        TAM_TRY(t, hipMemset(t->d_dbg, 0, sizeof(uint64_t) * n));
    }
    if (out_us && t->d_dbg) {
        std::vector<uint64_t> h(n);
        TAM_TRY(t, hipMemcpy(h.data(), t->d_dbg, sizeof(uint64_t) * n, hipMemcpyDeviceToHost));
        double acc[4] = {0, 0, 0, 0};
        uint64_t lo = ~0ull, hi = 0;
        int nb = 0;
        for (size_t blk = 0; blk < 4 * TAMOLS_BPL; ++blk) {
            const uint64_t* s = h.data() + blk * 8;
            if (!s[0]) continue;
            ++nb;
            for (int k = 0; k < 4; ++k) acc[k] += (double)(s[k + 1] - s[k]);
            lo = std::min(lo, s[0]);
            if (s[5]) hi = std::max(hi, s[5]);
        }
        for (int k = 0; k < 4; ++k) out_us[k] = nb ? (float)(acc[k] / nb * 0.01) : 0.0f;
        out_us[4] = hi > lo ? (float)((double)(hi - lo) * 0.01) : 0.0f;
    }
    if (!enable && t->d_dbg) {
        (void)hipFree(t->d_dbg);
        t->d_dbg = nullptr;
    }
    return SRBD_OK;
}

// Diagnostic: the raw stamps of the last call (4 x TAMOLS_BPL x 8 uint64, 100 MHz ticks).
extern "C" int srbd_tamols_phases_raw(srbd_tamols_ctx* t, uint64_t* out) {
    if (!t || !out || !t->d_dbg) return SRBD_E_INVALID;
    arm_cancel_others();
    TAM_TRY(t, hipSetDevice(t->device));
    TAM_TRY(t, hipMemcpy(out, t->d_dbg, sizeof(uint64_t) * 4 * TAMOLS_BPL * 8, hipMemcpyDeviceToHost));
    return SRBD_OK;
}

#ifdef SRBD_ROLLOUT_STAMPS
// Probe build only: one merge launch of the context's last rollout records with the phase stamps on (merge_body's
// MERGE_STAMP / MERGE_MARK: 32 words per block for blocks 0 and 1, s_memrealtime ticks of 10 ns).
extern "C" int srbd_probe_merge_phases(srbd_ctx* c, uint64_t* host64) {
    if (!c || !host64) return SRBD_E_INVALID;
    HIP_TRY(c, hipSetDevice(c->cfg.device_id));
    uint64_t* d = nullptr;
    HIP_TRY(c, hipMalloc((void**)&d, sizeof(uint64_t) * 64));
    hipError_t e = hipMemsetAsync(d, 0, sizeof(uint64_t) * 64, c->stream);
    if (e == hipSuccess) {
        launch_merge(c->mc, c->d_in, merge_src(c), merge_nrec(c), c->wrec_stride, 0, c->d_noise[c->cur], nullptr,
                     c->d_out, 0, c->stream, d);
        e = hipMemcpyAsync(host64, d, sizeof(uint64_t) * 64, hipMemcpyDeviceToHost, c->stream);
    }
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    (void)hipFree(d);
    HIP_TRY(c, e);
    return SRBD_OK;
}
#endif
