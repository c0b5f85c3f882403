// srbd_launch.h -- internal launchers shared by srbd_kernels.hip, tamols_kernel.hip and srbd_api.hip.
#pragma once

#include <string>
#include <vector>

#include "srbd_core.h"

namespace srbd {

// One batch of noise draws: into `noise` (SoA), keyed by (seed, ctr) or, when dev_ctr != 0, by the
// device StepInput's seed and counter + ctr_offset (device-resident chains).
struct RngJob {
    float* noise;
    uint64_t seed, ctr;
    int dev_ctr, ctr_offset;
    const uint32_t* gate;  // armed chain: skip the draws when *gate holds the cancel bit (ARM_CANCEL)
};
int rng_grid(const ModelConst& mc);

// In-launch level-1 fold of the reduction tree (srbd_core.h): the leaf records of TREE_FAN consecutive leaves (a
// level-1 node) are folded by the node's last arriving block into grecs[node], a record of the same format, so
// the merge reads ceil(nleaf / TREE_FAN) records instead of nleaf.  gsize == TREE_FAN when on, 1 when off.
struct XchgArgs;
constexpr int GROUP_LDS_FLOATS = 6144;  // the last arriver stages its node's records in LDS (24 KB)
constexpr int GROUP_MIN_LEAVES = 128;   // the merge reads the leaf records up to this many
struct GroupArgs {
    float* grecs;   // ngroups x rec_stride (level-1 node records)
    uint32_t* cnt;  // ngroups arrival counters, zero between launches (each node's last arriver resets its own)
    int gsize;      // TREE_FAN (the fold runs) or 1
    const uint32_t* gate;  // armed chain (Publish::gate): every block exits at once when the chain did not fire
    // Final merge in the rollout launch (zero-order four-lane kernel, host steps): the last group arriver to
    // finish counts itself in *gdone; the block that completes the count merges the ngroups group records
    // into the step outputs `out` and publishes `seq` in `flag`, as merge_kernel would (launch_rollout_final).
    StepOutput* out = nullptr;
    uint32_t* flag = nullptr;
    uint32_t seq = 0;
    uint32_t* gdone = nullptr;  // zero between launches (the final merger resets it)
    int ngroups = 0;
    int fence_sys = 1;
    // host steps: the step input by value (host memory, read by the launcher): the rollout takes it as a
    // kernel argument and writes the device StepInput itself (ks_ok), no upload kernel
    const void* ksi = nullptr;  // a StepInputK
    // sharded host steps over xGMI: the final merger folds the rank's buffer (`levels_up` levels above the
    // level-1 records), exchanges it with the peers and merges the gathered buffers, as merge_xchg_kernel does
    // (device copy of the context's XchgArgs)
    const XchgArgs* xa = nullptr;
    int levels_up = 0;
    // unsharded host steps with 2..TREE_FAN level-1 nodes (fast_tail_ok): the node folders count in *gdone before
    // they fold, the last to count folds the root itself; the others hand their node records over as 8-byte words
    // tagged with `seq` in gtag (ngroups x (REC_HDR + P) words), polled word by word (fast_tail)
    int fast = 0;
    uint64_t* gtag = nullptr;
    // fast_tail's outputs as tagged words (host-mapped, P + 40 of them: best[P] | grf 12 | pred 24 | best_cost,
    // best_index, best_freq, status, each (seq << 32 | bits)) instead of StepOutput + flag (tagged_outputs)
    uint64_t* outt = nullptr;
    // the step's draws made inside the rollout launch (gen_ok: thread form, zero-order H 12, MPPI, device Philox
    // stream): the horizon generates each step's values and stores the quads the epilogue does not regenerate; no
    // RNG launch
    int gen = 0;  // 0 off, else 1 + the quads the epilogue regenerates (the horizon stores the others)
};
// C5 host p50 (us) at 0 / 4 / 6 / 8 / 10 / 12 / 16 / 24 / 36 regenerated quads: 167.9 / 156.5 / 150.9 / 150.9 /
// 149.4 / 152.6 / 153.7 / 156.5 / 164.7 (the RNG launch + read: 188.0)
constexpr int GEN_REGEN_QUADS = 8;
constexpr int TAGGED_OUT_EXTRA = 40;
bool gen_ok(const ModelConst& mc, int mode);
// words of the gtag buffer: header words [64][4] (a lane per node), then column words [64][P + 1] -- 64 node slots,
// so every address fast_tail's unconditional loads form (nodes < TREE_FAN, columns < 256) lies in the allocation
#define FT_GTAG_WORDS(P) (256 + 64 * ((P) + 1) + 256)
bool ks_ok(const ModelConst& mc, int mode);
bool fast_tail_ok(const ModelConst& mc, int mode, int ngroups, int rec_stride);
// LDS the in-launch final merge needs (merge_body<256> of ngroups records) and whether the launch can do it
size_t final_merge_lds(const ModelConst& mc, int ngroups, int rec_stride);
bool final_merge_ok(const ModelConst& mc, int mode, int ngroups, int rec_stride);
int merge_fence_sys();
// TREE_FAN when the rollout launch folds level 1 of the tree, else 1 (group_size)
int group_size(const ModelConst& mc);

// rollout forms: one thread per sample (block = `threads` samples) or four lanes per sample (block = 256
// threads = 64 samples)
enum { ROLLOUT_THREAD = 0, ROLLOUT_QUAD = 1 };
// samples per rollout block of a mode's `threads`
inline int rollout_spb(int mode, int threads) { return mode == ROLLOUT_QUAD ? threads / 4 : threads; }
bool rollout_specialised(int kind, int H, int S);
// next != NULL: extra blocks of the same launch generate the next step's draws (RngJob) beside the
// rollout, on the CUs it leaves idle.
void launch_rollout(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                    int rec_stride, int mode, int threads, hipStream_t s, const RngJob* next = nullptr,
                    const GroupArgs& grp = GroupArgs{nullptr, nullptr, 1, nullptr});
// the thread-per-sample forms (srbd_rollout_thread.hip): plain and gait-adaptive
void launch_rollout_thread(const ModelConst& mc, const StepInput* in, const float* noise, float* costs, float* recs,
                           int rec_stride, int threads, hipStream_t s, const RngJob* next, const GroupArgs& grp);
void launch_rollout_ga_thread(const ModelConst& mc, const StepInput* in, const float* noise, float* costs,
                              float* recs, int rec_stride, int spb, hipStream_t s, const RngJob* next,
                              const GroupArgs& grp);
// Counter: `ctr` (host-known), or in->ctr + ctr_offset when dev_ctr != 0 (device-resident chain).
void launch_rng(const ModelConst& mc, const StepInput* in, uint64_t seed, uint64_t ctr, int dev_ctr, int ctr_offset,
                float* noise, hipStream_t s, const uint32_t* gate = nullptr);
void launch_transpose(const float* src, int n, int P, int ldn, float* dst, hipStream_t s);
size_t merge_smem_bytes(int nrec, int P, int K, int cols = 0);  // cols: a column-split block's columns + 1
// Completion published to the host: after every output write is visible system-wide, the merge
// stores `seq` into `flag` (host-mapped pinned memory); the host spins on it instead of a stream sync.
struct Publish {
    uint32_t* flag;
    uint32_t seq;
    // armed chain: the word arm_copy_kernel writes (seq when it fired, seq | ARM_CANCEL when not); a chain
    // that did not fire computes nothing and publishes seq | ARM_CANCEL, so the host never takes the
    // previous input's outputs for the current call (it re-runs the step unarmed)
    const uint32_t* gate;
};
// chain != 0: also write the new parameters / sigma / RNG counter back into `in` (device warm start).
// With step outputs and no rank record the merge is column-split over merge_blocks(mc) blocks, each
// publishing flag[block]; returns the number of blocks that publish.
#ifndef SRBD_MERGE_SPLIT_COLS
#define SRBD_MERGE_SPLIT_COLS 4
#endif
constexpr int MERGE_SPLIT_COLS = SRBD_MERGE_SPLIT_COLS;  // parameter columns per slice block (-D overrides)
constexpr int MERGE_MAX_BLOCKS = 64;  // publish flags the host context holds
constexpr int MERGE_SPLIT_MIN_RECS = 256;
int merge_split_cols(const ModelConst& mc);
void merge_prepare();  // once per context: the LDS-staged merge's dynamic LDS limit
int merge_blocks(const ModelConst& mc);
// The tree's levels above the `nrec` input records (leaves or level-1 nodes, in global order): to the root and the
// step outputs, or (rank_out) `levels_up` levels up to this rank's exchange-level nodes, one rank record each.
int launch_merge(const ModelConst& mc, StepInput* in, const float* recs, int nrec, int rec_stride,
                  int rows_in_rec, const float* noise, float* rank_out, StepOutput* out, int chain, hipStream_t s,
                  uint64_t* dbg = nullptr, int ctr_inc = 1, Publish pub = {nullptr, 0, nullptr}, int levels_up = 0);
// xGMI exchange of rank records (merge_xchg_kernel).  mailbox: this rank's 2 x W slots of one rank
// buffer each (its exchange-level node records; half epoch & 1, slot r of a half written by rank r); flags: W epochs (word r written
// by rank r; waits accept >= epoch); peer_*: every rank's mailbox / flags as
// this GPU addresses them (IPC-mapped; entry `rank` is the local one).  epoch: this rank's exchange
// counter in device memory, advanced by every exchange kernel (so the chain can be a replayed graph).
constexpr int XCHG_MAX_WORLD = 16;
constexpr uint64_t XCHG_TIMEOUT_TICKS = 200000000ull;  // 2 s at the 100 MHz s_memrealtime clock
struct XchgArgs {
    float* mailbox;
    uint32_t* flags;
    float* peer_mailbox[XCHG_MAX_WORLD];
    uint32_t* peer_flags[XCHG_MAX_WORLD];
    float* stage;  // cached world x stride copy the second merge pass reads (mailbox is uncached)
    int* err;
    uint32_t* epoch;
    int rank, world, stride;  // stride: floats per mailbox slot (one rank record)
};
void launch_xchg_probe(const XchgArgs& x, int* ok, hipStream_t s);
void launch_merge_xchg(const ModelConst& mc, StepInput* in, const float* recs, int nrec, int rec_stride,
                       const float* noise, const XchgArgs& x, StepOutput* out, int chain, hipStream_t s, int ctr_inc,
                       Publish pub, int levels_up);
void launch_advance(const ModelConst& mc, StepInput* in, const StepOutput* out, hipStream_t s);
void launch_empty(hipStream_t s);  // measurement: the event floor
// src -> dst bytes [0, bytes0) and [off1, off1 + bytes1); all multiples of 16
void launch_copy16(const void* src, void* dst, size_t bytes0, size_t off1, size_t bytes1, hipStream_t s);
// Armed step: the copy kernel launched ahead of its input.  Lane 0 spins (s_sleep, bounded by
// `deadline_ticks` of the 100 MHz clock) on the host-mapped word `go` until it reads `seq` (fire: copy as
// launch_copy16 does, source read with system-scope loads) or `seq | ARM_CANCEL` / the deadline (no
// copy: the chain behind it recomputes the previous input and the host discards that run).
constexpr uint32_t ARM_CANCEL = 0x80000000u;
void launch_arm_copy(const uint32_t* go, uint32_t seq, uint64_t deadline_ticks, const void* src, void* dst,
                     size_t bytes0, size_t off1, size_t bytes1, uint32_t* fired, hipStream_t s);
void launch_div_selftest(const float* a, const float* b, int n, float* o, hipStream_t s);
void launch_log1p_selftest(const float* t, int n, float* o, hipStream_t s);

// TAMOLS (tamols_kernel.hip)
constexpr int TAMOLS_NQ = 19;        // nearest-neighbour queries per candidate
constexpr int TAMOLS_MAXCAND = 320;  // rows * cols

struct TamolsArgs {
    int rows, cols, ncand;
    int has_vel, has_base, has_feet;
    int contact[4];
    double vel[3], base[3];
    double feet[12], seeds[12], hips[12];
    srbd_tamols_params p;
};

// Terrain raycast (terrain_kernel.hip).  Device scene: primitives with the box yaw's cos / sin
// precomputed on the host (prim.pad unused).
struct TerrainDev {
    const srbd_terrain_prim* prims;
    const double* cs;  // nprims x (cos yaw, sin yaw)
    int nprims;
    int has_ground;
    double ground_z, miss_z;
    const double* hf;
    int hf_nx, hf_ny;
    double hf_x0, hf_y0, hf_dx, hf_dy;
};
// Patch p: centre centers[3p..], yaw cos / sin in cs_yaw[2p..] (device arrays).
struct PatchJob {
    const double* centers;
    const double* cs_yaw;
    int npatch, rows, cols;
    double dist_x, dist_y, ray_z;
    double* out;  // npatch x rows x cols x 3
};
void launch_terrain_patches(const TerrainDev& t, const PatchJob& j, hipStream_t s);

}  // namespace srbd

// Device-resident terrain scene (opaque in the C-ABI).
struct srbd_terrain {
    int device = 0;
    hipStream_t stream = nullptr;
    srbd_terrain_prim* d_prims = nullptr;
    double* d_cs = nullptr;
    double* d_hf = nullptr;
    double* d_job = nullptr;  // centres | yaw cos, sin
    double* d_out = nullptr;
    size_t cap_job = 0, cap_out = 0;
    double* h_job = nullptr;  // pinned staging of the job inputs
    srbd::TerrainDev dev{};
    // every scene value (primitives, height field, the ground height) finite and below 1e30 in magnitude, so every
    // raycast height that hits is a finite double well inside float's range (srbd_foothold_chain's cost_feet)
    bool bounded = false;
    std::string err;
};

namespace srbd {
// Raycast npatch patches on stream s into the scene's device output buffer (*d_out).
int terrain_enqueue(srbd_terrain* t, const double* centers, const double* yaws, int npatch, int rows, int cols,
                    double dist_x, double dist_y, double ray_z, hipStream_t s, double** d_out);

// One TAMOLS call as one launch (tamols_kernel.hip): TAMOLS_BPL blocks per leg, each raycasting (or
// reading) the leg's patch and scoring its slice of the candidates; the leg's last block merges the
// slices, the last leg publishes `seq` into `flag`.  Outputs are host-mapped pointers.
#ifndef SRBD_TAMOLS_BPL
#define SRBD_TAMOLS_BPL 16  // blocks per leg (a build-time knob for scripts/build_variants.sh sweeps)
#endif
constexpr int TAMOLS_BPL = SRBD_TAMOLS_BPL;
constexpr int TAMOLS_THREADS = 1024;
constexpr int TAMOLS_LDS_PRIMS = 1024;  // scenes up to this many primitives are staged in LDS (80 KB)
// A leg's outputs as 8-byte words (seq << 32 | 32 bits), each stored once, so the host polls the words themselves
// (no fence and flag behind them): the foothold's 3 doubles (words 0-5, low half first), the box's 6 (6-17), the seed
// height (18-19), the validity (20).
constexpr int TAMOLS_OUT_WORDS = 24;
constexpr int TAMOLS_OUT_USED = 21;
struct TamolsJob {
    TamolsArgs a;
    int use_terrain;     // 1: raycast the patches from `t` (centres = the seeds), 0: read `hm`
    int lattice;         // use_terrain with dist_x, dist_y > 0: the patch is a lattice (one block per leg)
    TerrainDev t;
    double yaw_c, yaw_s, dist_x, dist_y, ray_z;
    double inv_dx, inv_dy;  // 1 / dist_x, 1 / dist_y (the lattice queries)
    int rows, cols;
    const double* hm;    // 4 x nc x 3 (device-visible) when !use_terrain
    double* hm_out;      // 4 x nc x 3 raycast patches or NULL
    double* scores;      // 4 x nc or NULL
    uint64_t* outt;      // host-mapped, 4 x TAMOLS_OUT_WORDS tagged words (tamols_leg_out)
    double* part;        // 4 x TAMOLS_BPL x 4 partials (device)
    unsigned* cnt;       // 4 per-leg block counters (device, zero between calls)
    uint32_t seq;
    uint64_t* dbg;       // diagnostic phase stamps (4 x TAMOLS_BPL x 8) or NULL
    // The chained foothold step (srbd_foothold_mpc_step): the launch also writes the MPC step's device StepInput,
    // so the rollout launch queued behind it needs no host round trip.  Block (0, 0) copies the host step input
    // (the kernel argument, launch_tamols_fused's ksi) except the words holding the feet and cost_feet; the last
    // leg to finish writes those: the reference's feet = the footholds, swing feet of the state = the footholds
    // (prepare_state), cost_feet over them as fill_input sums it.
    struct Feed {
        StepInput* in;   // device StepInput of the MPC context (NULL: no feed)
        double* fh;      // 12 doubles of device scratch: the legs' footholds
        unsigned* cnt;   // leg arrival counter (device, zero between calls)
        int nwords;      // 16-byte words of StepInput to copy (the prefix and best[P])
        int swing[4];    // current contact == 0: the state's foot is the foothold
        float q[12];     // q_diag[12..24)
        int cf_known;    // the host's cost_feet stands (zero feet weights, bounded inputs): each leg writes its own
                         // feet, no cross-leg step
    } feed;
};
void launch_tamols_fused(const TamolsJob& j, hipStream_t s, const StepInputK* ksi = nullptr);
int tamols_prepare();  // once per context: the staged scene's dynamic LDS limit (0 on success)

}  // namespace srbd
