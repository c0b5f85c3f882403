/*
 * srbd_mpc.h -- C-ABI of the MI355X-native sampling SRBD MPC (libsrbd_hip.so).
 *
 * This is the drop-in boundary for the reference's sampling controller hot path.
 * Each entry point names the reference interface it replaces (paths relative to
 * the reference repository root Magicyw/Quadruped-PyMPC-TAMOLS):
 *
 *   srbd_create            <- Sampling_MPC.__init__            centroidal_nmpc_jax.py:23-178
 *   srbd_step              <- Sampling_MPC.jitted_compute_control, i.e.
 *                             compute_control_random_sampling   centroidal_nmpc_jax.py:629-787
 *                             compute_control_mppi              centroidal_nmpc_jax.py:789-932
 *                             compute_control_cem_mppi          centroidal_nmpc_jax.py:934-1094
 *                             (called from srbd_controller_interface.py:140,159)
 *   srbd_step_local /
 *   srbd_step_finish       <- the same call, split around the one cross-GPU exchange
 *                             (row-sharded rollouts)
 *   srbd_tamols_run        <- VisualFootholdAdaptation.compute_adaptation, strategy 'tamols'
 *                             visual_foothold_adaptation.py:153-231 (+ helpers :261-714)
 *   srbd_terrain_patches   <- gym_quadruped HeightMap.update_height_map (wb_interface.py:233-234)
 *
 * Conventions: plain pointers and sizes, caller owns every host array, nothing is
 * retained past a call, 0 = success and negative SRBD_E* codes on failure (message
 * via srbd_last_error), nothing throws across the ABI.  One context per thread or
 * process; a context creates its HIP state lazily in srbd_create (never at load).
 * Results are bitwise reproducible for identical inputs (fixed reduction order).
 */
#ifndef SRBD_MPC_H
#define SRBD_MPC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SRBD_ABI_VERSION 1
#define SRBD_MAX_HORIZON 32
#define SRBD_MAX_PARAMS 384
#define SRBD_MAX_ELITE 16
#define SRBD_MAX_FREQS 8 /* candidate step frequencies of the gait-adaptive sampler */

enum {
    SRBD_OK = 0,
    SRBD_E_INVALID = -1,  /* bad argument / unsupported configuration */
    SRBD_E_HIP = -2,      /* HIP runtime error */
    SRBD_E_NODEVICE = -3, /* no HIP device visible: there is no CPU fallback */
    SRBD_E_STATE = -4,    /* call out of order */
    SRBD_E_NOMEM = -5
};

/* mpc_params['sampling_method'] (config.py:181) */
enum { SRBD_RANDOM_SAMPLING = 0, SRBD_MPPI = 1, SRBD_CEM_MPPI = 2 };
/* mpc_params['control_parametrization'] (config.py:182) */
enum { SRBD_ZERO_ORDER = 0, SRBD_LINEAR_SPLINE = 1, SRBD_CUBIC_SPLINE = 2 };

typedef struct srbd_config {
    int32_t num_samples;     /* N = num_parallel_computations (global, all ranks) */
    int32_t horizon;         /* H (<= SRBD_MAX_HORIZON) */
    int32_t method;          /* SRBD_RANDOM_SAMPLING | SRBD_MPPI | SRBD_CEM_MPPI */
    int32_t parametrization; /* SRBD_ZERO_ORDER | SRBD_LINEAR_SPLINE | SRBD_CUBIC_SPLINE */
    int32_t num_splines;     /* S (linear / cubic) */
    int32_t num_elite;       /* CEM elite count; reference: 10 (centroidal_nmpc_jax.py:1075) */
    int32_t device_id;       /* HIP ordinal */
    int32_t rank;            /* shard index: rows srbd_shard_rows(num_samples, rank, world_size) */
    int32_t world_size;      /* 1 for single GPU */
    int32_t use_graph;       /* 1: replay srbd_step as one hipGraph */
    float mass;              /* config.mass */
    float mg;                /* float32(mass * 9.81), rounded once from double as the reference does */
    float grf_min, grf_max, mu;
    float inertia[9];        /* config.inertia, row-major, float32 */
    float dts[SRBD_MAX_HORIZON]; /* Centroidal_Model_JAX.dts (centroidal_model_jax.py:42-53) */
    float q_diag[24];        /* diag(Q), centroidal_nmpc_jax.py:118-130 */
    float sigma_mppi;        /* mpc_params['sigma_mppi'] */
    float sigma_random_sampling[3]; /* mpc_params['sigma_random_sampling'] */
} srbd_config;

typedef struct srbd_result {
    float grf[12];             /* nmpc_GRFs (FL, FR, RL, RR) x (x, y, z) */
    float predicted_state[24]; /* nmpc_predicted_state */
    float best_cost;           /* saturated cost of the best sample */
    int32_t best_index;        /* global row of the best sample (nanargmin, first on ties) */
    int32_t status;
    float best_freq;           /* gait-adaptive: step frequency of the best sample (best_step_frequency,
                                  centroidal_nmpc_jax_gait_adaptive.py:705,861); 0 otherwise */
} srbd_result;

typedef struct srbd_ctx srbd_ctx;

/* Parameter count P for a configuration (centroidal_nmpc_jax.py:52-93), or < 0. */
int srbd_num_params(const srbd_config* cfg);
int srbd_device_count(int32_t* count);
int srbd_abi_version(void);

int srbd_create(const srbd_config* cfg, srbd_ctx** out);
void srbd_destroy(srbd_ctx* ctx);
/* Last error of ctx, or of the calling thread's last failed srbd_create when ctx == NULL. */
const char* srbd_last_error(const srbd_ctx* ctx);
/* Launch on a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); disables graphs. */
int srbd_set_stream(srbd_ctx* ctx, void* hip_stream);

/*
 * One sampling iteration (one jitted_compute_control call).
 *   state, ref        : 24 floats each (prepare_state_and_reference output, cast to f32)
 *   contact           : 4 rows x contact_stride floats, row-major; the first H columns are used
 *   best_params       : P floats, in: previous best, out: updated best (reassigned by the interface)
 *   sigma             : P floats (CEM only, in/out; NULL otherwise)
 *   noise             : NULL -> device RNG: Philox4x32-10 keyed by (seed, counter), or the reference's
 *                       jax.random stream keyed by seed (srbd_set_rng);
 *                       else N x P row-major additional_random_parameters (row 0 must be zero)
 *   out_costs         : N floats (saturated) or NULL
 */
int srbd_step(srbd_ctx* ctx, const float* state, const float* ref, const float* contact, int32_t contact_stride,
              float* best_params, float* sigma, const float* noise, uint64_t seed, uint64_t counter,
              srbd_result* out, float* out_costs);

/* Armed host steps: the same srbd_step calls with the launch latency taken off the call.  Each
 * srbd_step with device draws (noise == NULL) queues its successor -- copy, rollout and merge for
 * (seed, counter + 1) -- behind itself; that chain's copy kernel waits (bounded by deadline_us, 0: 50 ms)
 * on a host-mapped word, and the next srbd_step stores its inputs and that word instead of launching.  A
 * call the chain cannot serve (injected noise, another counter or seed, past half the deadline) and every
 * other entry point cancel it: the cancelled chain computes nothing (its copy kernel writes its verdict
 * to a device word every kernel of the chain checks first) and nothing a caller reads changes.  A claimed
 * chain whose copy kernel had already given up (deadline passed before the go word) publishes a cancel
 * token instead of outputs, and the call re-runs unarmed.  Outputs are bit-identical to unarmed steps.  One context per process
 * is armed at a time.  While armed, the copy kernel occupies its hardware queue (other streams of the
 * process that share that queue wait behind it, up to the deadline), hence opt-in: for a process whose
 * controller owns the GPU queue (the reference's 100 Hz MPC loop).  No reference counterpart (launch
 * latency has none in JAX's dispatch model); replaces nothing in SCI:140-159's call.  enable = 0 cancels. */
int srbd_set_armed(srbd_ctx* ctx, int32_t enable, uint64_t deadline_us);
/* Armed steps served (fired) and cancelled since the context was created. */
int srbd_armed_stats(const srbd_ctx* ctx, int64_t* served, int64_t* cancelled);
/* Claimed chains that had already given up and were re-run unarmed (counted as cancelled above). */
int srbd_armed_refired(const srbd_ctx* ctx, int64_t* refired);
/* Test hook: the host sleeps delay_us between claiming an armed chain and storing its go word. */
int srbd_debug_arm_delay(srbd_ctx* ctx, uint32_t delay_us);
/* Test hook: the next column-split merge (CEM, or > 256 records) has one slice withhold its hand-off word, so
 * the tail block's bounded wait (2 s) times out and the step fails with SRBD_E_HIP; the call resets the
 * hand-off state, and the following step is exact again. */
int srbd_debug_split_drop(srbd_ctx* ctx);
/* srbd_foothold_mpc_step calls on this context that ran chained on the device (TAMOLS writing the step's input;
 * one host wait), since the context was created. */
int srbd_foothold_chained(const srbd_ctx* ctx, int64_t* n);

/*
 * Gait-adaptive sampling (centroidal_nmpc_jax_gait_adaptive.py; replaces
 * compute_rollout :326-501 and the step-frequency draws :687-692 (random sampling), :834-838
 * (MPPI)).  After this call every step of the context (srbd_step, the sharded and device-resident
 * forms) samples one step frequency per sample and rolls out with that sample's own contact
 * sequence: PeriodicGaitGeneratorJax (periodic_gait_generator_jax.py:68-151) advanced from
 * `timing` with pgg_dt * f per step and contact = t < duty_factor; the per-leg decode index counts
 * the leg's stance steps (GA:353-379) and the cost gains (f - 1.3) * 100 * (f - 1.3) (GA:500).
 * The caller's contact sequence of srbd_step is still the one the final GRFs use (GA:720-796).
 *   timing      : 4 floats, the periodic gait generator phase of each leg (pgg_phase_signal)
 *   pgg_dt      : mpc_params['dt'] (GA:179);  duty_factor: 0.65 in the reference (GA:179)
 *   freq_set    : n_freq (1..SRBD_MAX_FREQS) candidate frequencies, drawn uniformly per sample
 *                 (jax.random.choice); the caller forms the set per method and call:
 *                 RS: optimize_swing ? step_freq_available : n x nominal; MPPI: step_freq_available
 *   freq_local  : NULL -> device draw (Philox, keyed by seed/counter and global row); else the
 *                 frequency of each of this shard's rows (parity / injection mode, like `noise`)
 * Call again before each step to change any of these; srbd_clear_gait returns to the plain path.
 * CEM is not supported (the reference's gait-adaptive CEM is broken as wired):
 * SRBD_E_INVALID.
 */
int srbd_set_gait(srbd_ctx* ctx, const float* timing, float pgg_dt, float duty_factor, const float* freq_set,
                  int32_t n_freq, const float* freq_local);
int srbd_clear_gait(srbd_ctx* ctx);

/*
 * Opt-in per-sample cost terms (the north star's "friction-cone + GRF-smoothing terms").  The
 * reference's sampling cost has none of them (its R input cost is commented out, NMPC:132-157 and
 * :453-484; the cone is enforced by projection), so all weights default to 0 and
 * then the cost is exactly the reference's.  Per horizon step and leg, with f the clipped, masked
 * force and fref the step's gravity share:
 *   r_force[q] * u_q^2         u = (fx, fy, fz - fref if the leg is in stance else fz)
 *                              (the reference's R; its values were 0.1, 0.1, 0.001)
 *   w_smooth * |f_n - f_{n-1}|^2            steps n >= 1 (GRF smoothing)
 *   w_cone * (max(0, |fx'| - mu fz)^2 + max(0, |fy'| - mu fz)^2)   fx', fy' before the cone clip
 * Weights must be finite and >= 0.  Applies to every following step of the context (all methods,
 * parametrizations and rollout forms, gait-adaptive included).
 */
int srbd_set_cost_terms(srbd_ctx* ctx, const float r_force[3], float w_smooth, float w_cone);

/*
 * Device noise stream of every following step of the context (default SRBD_RNG_PHILOX):
 *   SRBD_RNG_PHILOX     : Philox4x32-10 + Box-Muller keyed by (seed, counter) (this library's own stream)
 *   SRBD_RNG_JAX        : the reference's jax.random stream (centroidal_nmpc_jax.py:654-676, 811, 957;
 *                         gait-adaptive choice :692, 836), jax_threefry_partitionable = True (JAX >= 0.5)
 *   SRBD_RNG_JAX_LEGACY : the same with jax_threefry_partitionable = False (earlier JAX)
 * In the JAX modes the `seed` of srbd_step is the step's key (uint32[2] packed key[0] << 32 | key[1], the
 * key the reference's interface passes: master_key after with_newkey, srbd_controller_interface.py:126-164);
 * `counter` only numbers the steps.  The draws made ahead (fused next-step draws, device-resident chains,
 * armed steps) assume the next key is with_newkey's split(key)[0] (srbd_jax_split, include/srbd_host.h).
 */
enum { SRBD_RNG_PHILOX = 0, SRBD_RNG_JAX = 1, SRBD_RNG_JAX_LEGACY = 2 };
int srbd_set_rng(srbd_ctx* ctx, int32_t kind);
int srbd_get_rng(const srbd_ctx* ctx);

/* Sharded form.  The rows of a rank are whole nodes of one level of the fixed reduction tree every merge
 * folds (64-row leaves, 32 children per node; the exchange level is the highest one that gives every rank a
 * node), so the merged result is the same bits for every world_size.  A rank's record ("rank buffer") holds
 * its nodes of that level, ceil(nodes / world_size) record slots; gathered in rank order the buffers are the
 * level's node list.  Size in floats (identical on every rank). */
int srbd_record_floats(const srbd_ctx* ctx);
/* Host-only: srbd_record_floats of a context of this configuration (rank / world_size as given). */
int srbd_record_floats_host(const srbd_config* cfg);
/* Host-only: the first global row and row count of `rank` of `world` ranks over num_samples rows
 * (SRBD_E_INVALID when some rank would get no node). */
int srbd_shard_rows(int64_t num_samples, int32_t rank, int32_t world, int64_t* row0, int64_t* rows);
/* Rows of this rank only; writes this rank's partial record to d_record (device pointer).
 * noise_local: NULL or (rows of this shard) x P row-major.  Asynchronous on the context stream. */
int srbd_step_local(srbd_ctx* ctx, const float* state, const float* ref, const float* contact, int32_t contact_stride,
                    const float* best_params, const float* sigma, const float* noise_local, uint64_t seed,
                    uint64_t counter, void* d_record);
/* Merge the gathered rank buffers (device pointer, rank order; num_records == world_size) and finish the step. */
int srbd_step_finish(srbd_ctx* ctx, const void* d_records, int32_t num_records, float* best_params, float* sigma,
                     srbd_result* out, float* out_costs_local);
/* Host-only merge of rank records (same math; no device needed). */
int srbd_finish_host(const srbd_config* cfg, const float* records, int32_t num_records, const float* state,
                     const float* contact, int32_t contact_stride, float* best_params, float* sigma,
                     srbd_result* out);
/* Host-only: build one rank record from a shard's saturated costs and noise rows (shard x P row-major). */
int srbd_make_record_host(const srbd_config* cfg, int32_t rank, int32_t world_size, const float* costs,
                          const float* noise_rows, float* record);

/*
 * Checkpoint / restore (exact golden replays of device-resident chains).  The state is what the next
 * device-resident step starts from: the warm start best_params (P floats), sigma (P floats, CEM
 * only; may be NULL otherwise) and the device RNG key (seed, counter).  After a host srbd_step it is
 * that step's inputs; every device-resident step (srbd_bench_device_steps, srbd_sharded_device_steps,
 * srbd_device_step_local/finish) advances it on the device.  Host steps are stateless here: their
 * state is their arguments (Sampling_MPC.get_state in the Python mirror).  Both calls block until the
 * context stream is idle and need one srbd_step first (it sets the state / reference inputs).
 */
int srbd_get_state(srbd_ctx* ctx, float* best_params, float* sigma, uint64_t* seed, uint64_t* counter);
int srbd_set_state(srbd_ctx* ctx, const float* best_params, const float* sigma, uint64_t seed, uint64_t counter);

/* Measurement: replay `steps` device-resident steps (RNG -> rollout -> reduction -> warm start
 * written back on device) back to back; returns elapsed ms (hipEvents on the context stream). */
int srbd_bench_device_steps(srbd_ctx* ctx, int32_t steps, float* elapsed_ms);
/* Measurement: `steps` srbd_step calls from C (srbd_step_sharded on a sharded context with a connected
 * xGMI / RCCL exchange), cycling through n_in input sets (state / ref: n_in x 24 floats, contact:
 * n_in x 4 x contact_stride), best (and sigma, CEM) fed back, counters counter0, counter0 + 1, ...;
 * lat_us[i] = wall time of call i (host-to-host at the C-ABI boundary, us). */
int srbd_bench_host_steps(srbd_ctx* ctx, const float* state, const float* ref, const float* contact,
                          int32_t contact_stride, int32_t n_in, float* best_params, float* sigma, uint64_t seed,
                          uint64_t counter0, int32_t steps, float* lat_us);
/* Average per-launch duration (us) of each kernel of one step: one hipEvent pair on the context
 * stream around `iters` back-to-back launches of that kernel (agrees with rocprofv3's kernel-trace
 * average).  fused_rollout_us: the rollout launch that also draws the next step's noise (the form
 * the step runs when fusion applies; 0 otherwise).  event_floor_us: the same measurement of an
 * empty kernel (launch-to-launch spacing).  Any out pointer may be NULL. */
int srbd_time_kernels(srbd_ctx* ctx, int32_t iters, float* rollout_us, float* rng_us, float* reduce_us,
                      float* fused_rollout_us, float* event_floor_us);

/* Measurement: average duration (us) of one kind of launch, `iters` back to back (one hipEvent pair), alone, so
 * a rocprofv3 pass over the call sees only it.  SRBD_TL_STEP_ROLLOUT is the rollout launch exactly as srbd_step
 * issues it (*form: 1 fused next-step draws | 2 step input by value | 4 in-launch final merge | 8 thread-per-sample
 * rollout kernel, else four lanes per sample | 16 fast_tail | 32 the launch makes the step's
 * draws itself: srbd_step then issues no RNG launch); SRBD_TL_STEP_MERGE
 * the merge launch srbd_step issues after it (0 when the rollout launch merges).  form may be NULL. */
enum { SRBD_TL_RNG = 0, SRBD_TL_ROLLOUT = 1, SRBD_TL_ROLLOUT_FUSED = 2, SRBD_TL_STEP_ROLLOUT = 3,
       SRBD_TL_STEP_MERGE = 4, SRBD_TL_EMPTY = 5 };
int srbd_time_launch(srbd_ctx* ctx, int32_t which, int32_t iters, float* us, int32_t* form);

/* Device-resident sharded chain (benchmark / pipelined callers): reuses the inputs of the last
 * srbd_step_local on the device.  srbd_device_step_local: RNG -> rollout -> rank record into d_record;
 * srbd_device_step_finish: merge -> outputs -> warm start (best/sigma/counter) written back on
 * device.  Both are asynchronous on the context stream. */
int srbd_device_step_local(srbd_ctx* ctx, void* d_record);
int srbd_device_step_finish(srbd_ctx* ctx, const void* d_records, int32_t num_records);
/* Block until the context stream is idle and copy the last step's outputs. */
int srbd_sync_result(srbd_ctx* ctx, float* best_params, float* sigma, srbd_result* out);
/* Test / diagnostic: the device draws a step keyed by (seed, counter) uses (the context's stream,
 * srbd_set_rng): this shard's rows of additional_random_parameters, n_local x P row-major (row 0 of the
 * problem is zero; CEM: the unscaled standard normals the step multiplies by sigma).  Blocks. */
int srbd_draw_noise(srbd_ctx* ctx, uint64_t seed, uint64_t counter, float* out_rows);
/* Saturated costs of this rank's rows from the last step (lazy materialisation). */
int srbd_copy_costs(srbd_ctx* ctx, float* out_costs);

/*
 * Sharded transport owned by the library (one process per GPU).  RCCL is loaded at run time from
 * `rccl_path` (the copy the process already uses, e.g. torch/lib/librccl.so) or /opt/rocm/lib.
 *   srbd_comm_get_unique_id : rank 0 makes the id (128 bytes); the caller broadcasts it
 *   srbd_comm_init          : every rank joins (rank / world_size from the context's config)
 *   srbd_step_sharded       : srbd_step_local + ncclAllGather of the rank records + srbd_step_finish
 *   srbd_sharded_device_steps: `steps` device-resident sharded steps, elapsed ms (hipEvents)
 */
int srbd_comm_get_unique_id(const char* rccl_path, uint8_t* id_out);
int srbd_comm_init(srbd_ctx* ctx, const char* rccl_path, const uint8_t* id_in);
int srbd_step_sharded(srbd_ctx* ctx, const float* state, const float* ref, const float* contact,
                      int32_t contact_stride, float* best_params, float* sigma, const float* noise_local,
                      uint64_t seed, uint64_t counter, srbd_result* out, float* out_costs_local);
int srbd_sharded_device_steps(srbd_ctx* ctx, int32_t steps, float* elapsed_ms);

/*
 * xGMI exchange (no collective launch): the merge kernel stores its rank record straight into
 * every rank's mailbox (uncached device memory, IPC-mapped over xGMI), sets per-rank epoch flags,
 * waits (bounded, 2 s) for the W records in its own mailbox and merges them in the same launch.
 * Once connected, srbd_step_sharded / srbd_sharded_device_steps use it instead of RCCL.
 *   srbd_xgmi_export        : allocate this rank's mailbox, 64-byte IPC handle out
 *   srbd_xgmi_connect       : world x 64 handle bytes in rank order (the caller all-gathers them)
 *   srbd_xgmi_connect_local : every rank's context in this process (index r = rank r)
 *   srbd_xgmi_probe         : one bounded round trip through the mailboxes (*ok = 1 on success)
 *   srbd_xgmi_disconnect    : back to RCCL (srbd_comm_init) for later steps
 */
int srbd_xgmi_export(srbd_ctx* ctx, uint8_t* handle_out);
int srbd_xgmi_connect(srbd_ctx* ctx, const uint8_t* handles);
int srbd_xgmi_connect_local(srbd_ctx* const* ctxs, int32_t world);
int srbd_xgmi_probe(srbd_ctx* ctx, int32_t* ok);
int srbd_xgmi_disconnect(srbd_ctx* ctx);

/* Diagnostic: mean duration (us) of the merge kernel's 5 phases (s_memrealtime stamps), then (staged merge)
 * the times from its start at which the records were in LDS and the tail prep was done, then the
 * shader clock in MHz over the kernel, then 16 finer marks (us from the start; 0 = unset): 24 floats for
 * block 0, then the same 24 for block 1 of a column-split merge (a slice block; zeros when unsplit): 48. */
int srbd_debug_merge_phases(srbd_ctx* ctx, int32_t iters, float* out_us);

/* Self-test of the correctly rounded division used in the rollout (a/b; b == 3 uses the constant
 * path).  Host results always; device results when out_dev != NULL (needs a GPU). */
int srbd_selftest_div(const float* a, const float* b, int32_t n, float* out_host, float* out_dev);
/* Self-test of the reference noise stream's log1p (jax.random.normal's erf_inv argument, NMPC:654/811/957): the
 * float of log1p(t) evaluated as float64 (t in (-1, 0]), on the host (out_host, with *nfallback = the arguments the
 * float64 log1p itself decided) and / or the device (out_dev).  Either output may be NULL. */
int srbd_selftest_log1p(const float* t, int32_t n, float* out_host, float* out_dev, int64_t* nfallback);

/* ------------------------------------------------------------------ TAMOLS */
typedef struct srbd_tamols_params {
    double gradient_delta;    /* 0.04 */
    double slope_threshold;   /* 0.7 */
    double w_edge, w_rough, w_dev, w_nominal, w_tracking, w_stability;
    double stability_margin;  /* 0.06 */
    double swing_time;        /* estimated_swing_time 0.25 */
    double h_des;             /* hip height */
    double l_min, l_max;      /* per-robot reach */
    double box_dx, box_dy;    /* constraint box */
    double stance_duration;   /* 0.3 (visual_foothold_adaptation.py:387) */
    double alphas[5];         /* np.linspace(0.2, 0.8, 5) (visual_foothold_adaptation.py:402) */
} srbd_tamols_params;

typedef struct srbd_tamols_ctx srbd_tamols_ctx;

int srbd_tamols_create(int32_t device_id, srbd_tamols_ctx** out);
void srbd_tamols_destroy(srbd_tamols_ctx* ctx);
const char* srbd_tamols_last_error(const srbd_tamols_ctx* ctx);
/*
 * heightmaps : 4 legs x rows x cols x 3 (x, y, z) doubles (HeightMap.data[:, :, 0, :])
 * seeds, hips: 4 x 3;  forward_vel: 3 or NULL;  base_pos: 3 or NULL;
 * contact    : 4 (1 stance, 0 swing) or NULL (-> all swing);  feet: 4 x 3 or NULL
 * outputs    : footholds 4x3, boxes 4x2x3, valid 4, scores 4 x rows*cols (or NULL),
 *              seed_heights 4 (nearest height + 0.02 at the seed, or NULL)
 */
int srbd_tamols_run(srbd_tamols_ctx* ctx, const double* heightmaps, int32_t rows, int32_t cols, const double* seeds,
                    const double* hips, const double* forward_vel, const double* base_pos, const int32_t* contact,
                    const double* feet, const srbd_tamols_params* params, double* out_footholds, double* out_boxes,
                    int32_t* out_valid, double* out_scores, double* out_seed_heights);

/* ------------------------------------------------------------------ terrain heightmap patches
 * GPU producer of the per-leg heightmap patches TAMOLS consumes: replaces
 * gym_quadruped's HeightMap.update_height_map (a MuJoCo mj_ray per patch point on the CPU; called at
 * quadruped_pympc/interfaces/wb_interface.py:233-234 with HeightMap(13, 7, 0.04, 0.04), simulation.py
 * :490-511).  The scene is uploaded once; every patch point casts a vertical ray down from ray_z and
 * takes the highest surface at or below ray_z: the ground plane, the top face of a box (yawed about
 * z) or of an upright cylinder, or a height field (cells split along the (i, j)-(i+1, j+1) diagonal).
 * A ray that hits nothing reports miss_z.  Patch point (i, j) of a patch centred at c with yaw psi:
 *   dx = (i - (rows - 1) / 2) * dist_x,  dy = (j - (cols - 1) / 2) * dist_y,
 *   x = c.x + cos(psi) dx - sin(psi) dy,  y = c.y + sin(psi) dx + cos(psi) dy   (float64).
 * gym_quadruped is absent here, so this layout is the one our PatchHeightMap uses (parity unpinned
 * against the real sensor; pinned against oracle/terrain_oracle.py bit for bit). */
enum { SRBD_PRIM_BOX = 0, SRBD_PRIM_CYLINDER = 1 };
typedef struct srbd_terrain_prim {
    int32_t type, pad;
    double cx, cy, cz; /* centre */
    double a, b, c;    /* box: half sizes x, y, z;  cylinder: radius, unused, half height */
    double yaw;        /* box rotation about z (radians) */
} srbd_terrain_prim;

typedef struct srbd_terrain srbd_terrain;

/* hfield: hf_nx x hf_ny heights, row-major [ix][iy], point (ix, iy) at (hf_x0 + ix hf_dx, hf_y0 + iy hf_dy);
 * NULL for none.  has_ground: a plane at ground_z. */
int srbd_terrain_create(int32_t device_id, const srbd_terrain_prim* prims, int32_t nprims, int32_t has_ground,
                        double ground_z, const double* hfield, int32_t hf_nx, int32_t hf_ny, double hf_x0,
                        double hf_y0, double hf_dx, double hf_dy, double miss_z, srbd_terrain** out);
void srbd_terrain_destroy(srbd_terrain* terrain);
const char* srbd_terrain_last_error(const srbd_terrain* terrain);
/* npatch patches (centres npatch x 3, yaws npatch) -> out npatch x rows x cols x 3 (x, y, z). */
int srbd_terrain_patches(srbd_terrain* terrain, const double* centers, const double* yaws, int32_t npatch,
                         int32_t rows, int32_t cols, double dist_x, double dist_y, double ray_z, double* out);
/* srbd_tamols_run with the four patches raycast on the device from `terrain` (centres = the seeds,
 * one yaw) in the same launch (the heightmap sensor fused into the search): no host round trip of the
 * patch.  out_heightmaps (4 x rows x cols x 3) and out_scores may be NULL (then only the footholds,
 * boxes, validity and seed heights cross PCIe). */
int srbd_tamols_run_terrain(srbd_tamols_ctx* ctx, srbd_terrain* terrain, double yaw, int32_t rows, int32_t cols,
                            double dist_x, double dist_y, double ray_z, const double* seeds, const double* hips,
                            const double* forward_vel, const double* base_pos, const int32_t* contact,
                            const double* feet, const srbd_tamols_params* params, double* out_footholds,
                            double* out_boxes, int32_t* out_valid, double* out_scores, double* out_seed_heights,
                            double* out_heightmaps);
/* ------------------------------------------------------------------ one C4 MPC step in one call
 * The per-MPC-step chain of helpers/foothold_pipeline.py TamolsMpcStep.step (wb_interface.py:230-291 +
 * srbd_controller_interface.py:113-180, MPPI / random sampling, one sampling iteration) behind one host call:
 * srbd_tamols_run_terrain on the patches around the seeds -> the adapted footholds (an infeasible leg: the seed at
 * its terrain height, VFA:223-228) as ref_foot_* after ref_base -> srbd_prepare_state -> srbd_step (device draws).
 * The same calls in the same order as the Python chain, so the same results bit for bit; the host work between
 * them is C instead of ~60 us of Python. */
typedef struct srbd_foothold_io {
    /* inputs */
    double state_in[24];        /* position, linear_velocity, orientation, angular_velocity, foot_FL..RR */
    double ref_base[12];        /* ref_position, ref_linear_velocity, ref_orientation, ref_angular_velocity */
    double seeds[12], hips[12]; /* reference footholds and hips, legs FL FR RL RR */
    double forward_vel[3];      /* TAMOLS forward velocity (the base linear velocity) */
    double current_contact[4], previous_contact[4];
    double yaw, dist_x, dist_y, ray_z;
    int32_t rows, cols;
    /* outputs */
    double footholds[12];       /* adapted ref_foot_* */
    double boxes[24];           /* constraint boxes (valid legs) */
    double seed_heights[4];
    int32_t valid[4];
    double state_out[24], ref_out[24]; /* prepare_state_and_reference's outputs */
    double* scores;             /* 4 x rows*cols, or NULL */
    double* heightmaps;         /* 4 x rows x cols x 3, or NULL */
    int32_t stage;              /* out: the calls that completed (0 none, 1 TAMOLS, 2 + prepare_state, 3 + step),
                                   so a caller can leave its objects as the chain would on an error */
    int32_t pad;
} srbd_foothold_io;

/* best_params (in/out, 4 x params_per_leg floats): the warm start; lift-off legs are zeroed before the step and the
 * step's result replaces it.  contact: 4 x contact_stride floats (the first `horizon` columns are used). */
int srbd_foothold_mpc_step(srbd_tamols_ctx* tamols, srbd_terrain* terrain, const srbd_tamols_params* params,
                           srbd_ctx* ctx, srbd_foothold_io* io, const float* contact, int32_t contact_stride,
                           float* best_params, int32_t params_per_leg, uint64_t seed, uint64_t counter,
                           srbd_result* out);

/* ------------------------------------------------------------------ one plugin-API MPC step in one call
 * SRBDControllerInterface.compute_control's sampling branch (srbd_controller_interface.py:113-180) over the plain
 * Sampling_MPC, behind one host call: prepare_state_and_reference (centroidal_nmpc_jax.py:563-627, no solution
 * shift: the caller keeps that case) -> per sampling iteration: with_newkey (:498-501) -> CEM's
 * with_newsigma(sigma_cem_mppi) at iteration 0 -> jitted_compute_control (srbd_step on device draws) -> the GRFs
 * times current_contact (SCI:175-178).  The same calls in the same order as the Python chain, so the same bits.
 * Key (in/out, advanced once per iteration as with_newkey + the step's key arguments do):
 *   SRBD_RNG_PHILOX   : key = (seed, counter); with_newkey: counter + 1; the step runs (seed, counter)
 *   SRBD_RNG_JAX[_LEGACY]: key[0] = the packed JAX key (key[0] << 32 | key[1]), key[1] = the controller's call
 *                       count; with_newkey: key = split(key)[0]; the step runs (packed key, call count + 1). */
typedef struct srbd_interface_io {
    /* inputs */
    double state_in[24];        /* position, linear_velocity, orientation, angular_velocity, foot_FL..RR */
    double ref_in[24];          /* ref_position .. ref_angular_velocity, ref_foot_FL..RR */
    double current_contact[4];  /* contact_sequence[:, 0] */
    double previous_contact[4]; /* the interface's previous_contact_mpc */
    double sigma_reset;         /* CEM: mpc_params['sigma_cem_mppi'] */
    uint64_t key[2];            /* in/out, see above */
    int32_t horizon, iterations, rng, cem; /* H, num_sampling_iterations, SRBD_RNG_*, method == CEM */
    /* outputs */
    double state_out[24], ref_out[24]; /* prepare_state_and_reference's outputs */
    double grf[12];             /* the last iteration's GRFs times current_contact (float64) */
    int32_t stage;              /* the calls that completed: 0 none, 1 prepare_state, 2 + i: iteration i's step */
    int32_t pad;
} srbd_interface_io;

/* contact / contact64: 4 x contact_stride float32 or float64 values (exactly one non-NULL; the first `horizon`
 * columns are used, float64 rounded to float32 as the step stages them).  best_params (in/out, 4 x params_per_leg):
 * the warm start (lift-off legs zeroed, then each iteration's result); sigma (in/out, CEM only, P floats).  `out`:
 * the last iteration's srbd_result. */
int srbd_interface_step(srbd_ctx* ctx, srbd_interface_io* io, const float* contact, const double* contact64,
                        int32_t contact_stride, float* best_params, int32_t params_per_leg, float* sigma,
                        srbd_result* out);

/* Diagnostic: enable != 0 stamps the phases of the following TAMOLS calls; out_us[5] (may be NULL)
 * receives the last call's mean per-block durations of (patch, queries, scores, slice argmin + count)
 * and the span from the first block's start to the last leg's end, in us.  enable == 0 turns it off. */
int srbd_tamols_phases(srbd_tamols_ctx* ctx, int32_t enable, float* out_us);
/* Diagnostic: the last call's raw stamps, 4 legs x 16 blocks x 8 uint64 (100 MHz). */
int srbd_tamols_phases_raw(srbd_tamols_ctx* ctx, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* SRBD_MPC_H */
