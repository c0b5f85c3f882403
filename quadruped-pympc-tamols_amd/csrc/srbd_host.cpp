// srbd_host.cpp -- host producers and transports around the MPC step (include/srbd_host.h).
// Reference paths are relative to the reference repository root:
//   PGG  = quadruped_pympc/helpers/periodic_gait_generator.py
//   NMPC = quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py
//   ROS  = ros2/run_controller.py
// Built with -ffp-contract=off: every float64 operation rounds as NumPy's does.
#include <math.h>
#include <string.h>

#include "../../include/srbd_host.h"
#include "../../include/srbd_mpc.h"
#include "srbd_jaxrng.h"

namespace {

// Python's float `x % 1.0` (result takes the divisor's sign; fmod is exact).
double pymod1(double x) {
    double r = fmod(x, 1.0);
    if (r != 0.0) {
        if (r < 0.0) r += 1.0;
    } else {
        r = copysign(0.0, 1.0);
    }
    return r;
}

void gait_offsets(int32_t gait, double off[4]) {  // PGG:24-41
    static const double tab[7][4] = {{0.5, 1.0, 1.0, 0.5},    {0.8, 0.3, 0.8, 0.3},  {0.5, 0.5, 0.0, 0.0},
                                     {0.0, 0.25, 0.75, 0.5},  {0.0, 0.25, 0.5, 0.75}, {0.0, 0.5, 0.75, 0.25},
                                     {0.5, 1.0, 0.75, 1.25}};
    static const double other[4] = {0.0, 0.5, 0.5, 0.0};
    memcpy(off, (gait >= 0 && gait < 7) ? tab[gait] : other, sizeof(double) * 4);
}

}  // namespace

extern "C" int srbd_pgg_reset(srbd_pgg* g) {
    if (!g) return SRBD_E_INVALID;
    gait_offsets(g->gait_type, g->phase_offset);
    for (int l = 0; l < 4; ++l) {
        g->phase_signal[l] = g->phase_offset[l];
        g->init[l] = 0;
    }
    return SRBD_OK;
}

extern "C" int srbd_pgg_init(srbd_pgg* g, int32_t gait_type, double duty_factor, double step_freq, int32_t horizon) {
    if (!g || horizon < 1) return SRBD_E_INVALID;
    memset(g, 0, sizeof(*g));
    g->duty_factor = duty_factor;
    g->step_freq = step_freq;
    g->horizon = horizon;
    g->gait_type = gait_type;
    g->previous_gait_type = gait_type;
    return srbd_pgg_reset(g);
}

// PGG:48-76, one leg at a time in the reference's order of operations.
extern "C" int srbd_pgg_run(srbd_pgg* g, double dt, double step_freq, double contact_out[4]) {
    if (!g || !contact_out) return SRBD_E_INVALID;
    const double inc = dt * step_freq;
    for (int l = 0; l < 4; ++l) {
        double ph = g->phase_signal[l] + inc;
        ph = pymod1(ph);
        double c;
        if (g->init[l]) {
            if (ph <= g->phase_offset[l]) {
                c = 1.0;
            } else {
                g->init[l] = 0;
                c = 1.0;
                ph = 0.0;
            }
        } else {
            c = ph < g->duty_factor ? 1.0 : 0.0;
        }
        g->phase_signal[l] = ph;
        contact_out[l] = c;
    }
    return SRBD_OK;
}

extern "C" int srbd_pgg_set_phase_signal(srbd_pgg* g, const double phase[4], const int32_t* init) {
    if (!g || !phase) return SRBD_E_INVALID;
    for (int l = 0; l < 4; ++l) {
        g->phase_signal[l] = phase[l];
        g->init[l] = init ? (init[l] != 0) : 0;
    }
    return SRBD_OK;
}

// PGG:93-118.  The generator state is restored afterwards (set_phase_signal(t_init, init_init)).
extern "C" int srbd_pgg_contact_sequence(srbd_pgg* g, const double* dts, const int32_t* lens, int32_t n_dts,
                                         double* out, int32_t out_cap) {
    if (!g || !out || g->horizon < 1) return SRBD_E_INVALID;
    const int H = g->horizon;
    if (g->gait_type == SRBD_GAIT_FULL_STANCE) {
        if (out_cap < 8 * H) return SRBD_E_INVALID;
        for (int i = 0; i < 8 * H; ++i) out[i] = 1.0;
        srbd_pgg_reset(g);
        return 2 * H;
    }
    if (out_cap < 4 * H || (H > 1 && (!dts || !lens || n_dts < 1))) return SRBD_E_INVALID;
    double t_init[4];
    int32_t init_init[4];
    memcpy(t_init, g->phase_signal, sizeof(t_init));
    memcpy(init_init, g->init, sizeof(init_init));
    double c[4];
    srbd_pgg_run(g, 0.0, g->step_freq, c);
    for (int l = 0; l < 4; ++l) out[l * H] = c[l];
    int j = 0;
    for (int i = 1; i < H; ++i) {
        if (i >= lens[j]) ++j;
        if (j >= n_dts) {  // the reference would raise IndexError here
            srbd_pgg_set_phase_signal(g, t_init, init_init);
            return SRBD_E_INVALID;
        }
        srbd_pgg_run(g, dts[j], g->step_freq, c);
        for (int l = 0; l < 4; ++l) out[l * H + i] = c[l];
    }
    srbd_pgg_set_phase_signal(g, t_init, init_init);
    return H;
}

// NMPC:563-627 (shift_solution off, config.py:188).
extern "C" int srbd_prepare_state(const double state_in[24], const double ref_in[24], const double current_contact[4],
                                  const double previous_contact[4], int32_t params_per_leg, float* best_params,
                                  double state_out[24], double ref_out[24]) {
    if (!state_in || !ref_in || !current_contact || !previous_contact || !state_out || !ref_out)
        return SRBD_E_INVALID;
    if (best_params && params_per_leg < 1) return SRBD_E_INVALID;
    double st[24];
    memcpy(st, state_in, sizeof(st));
    for (int l = 0; l < 4; ++l)
        if (current_contact[l] == 0.0) memcpy(st + 12 + 3 * l, ref_in + 12 + 3 * l, sizeof(double) * 3);
    memcpy(ref_out, ref_in, sizeof(double) * 24);
    memcpy(state_out, st, sizeof(st));
    if (best_params)
        for (int l = 0; l < 4; ++l)
            if (previous_contact[l] == 1.0 && current_contact[l] == 0.0)
                for (int j = 0; j < params_per_leg; ++j) best_params[l * params_per_leg + j] = 0.0f;
    return SRBD_OK;
}

// srbd_api.hip: the chained form (TAMOLS writes the step's device input; one host wait), 1 when not taken.
extern "C" int srbd_foothold_chain(srbd_tamols_ctx* t, srbd_terrain* ter, const srbd_tamols_params* p, srbd_ctx* c,
                                   srbd_foothold_io* io, const float* contact, int32_t stride, float* best,
                                   int32_t ppl, uint64_t seed, uint64_t counter, srbd_result* out);

// helpers/foothold_pipeline.py TamolsMpcStep.step in one host call (include/srbd_mpc.h).  The base position and
// the current feet TAMOLS reads are the state's own (state_in[0:3], state_in[12:24]); its contact flags are the
// current contact truncated to int32 (VFA's astype).  Chained on the device where the context allows it, else the
// calls in sequence below; the same results either way.
extern "C" int srbd_foothold_mpc_step(srbd_tamols_ctx* tamols, srbd_terrain* terrain, const srbd_tamols_params* params,
                                      srbd_ctx* ctx, srbd_foothold_io* io, const float* contact,
                                      int32_t contact_stride, float* best_params, int32_t params_per_leg,
                                      uint64_t seed, uint64_t counter, srbd_result* out) {
    if (!tamols || !terrain || !params || !ctx || !io || !contact || !best_params || !out || params_per_leg < 1)
        return SRBD_E_INVALID;
    io->stage = 0;
    const int chained = srbd_foothold_chain(tamols, terrain, params, ctx, io, contact, contact_stride, best_params,
                                            params_per_leg, seed, counter, out);
    if (chained != 1) return chained;
    int32_t cint[4];
    for (int l = 0; l < 4; ++l) cint[l] = (int32_t)io->current_contact[l];
    int rc = srbd_tamols_run_terrain(tamols, terrain, io->yaw, io->rows, io->cols, io->dist_x, io->dist_y, io->ray_z,
                                     io->seeds, io->hips, io->forward_vel, io->state_in, cint, io->state_in + 12,
                                     params, io->footholds, io->boxes, io->valid, io->scores, io->seed_heights,
                                     io->heightmaps);
    if (rc != SRBD_OK) return rc;
    io->stage = 1;
    double ref_in[24];
    memcpy(ref_in, io->ref_base, sizeof(double) * 12);
    memcpy(ref_in + 12, io->footholds, sizeof(double) * 12);  // wb_interface.py:268-285
    rc = srbd_prepare_state(io->state_in, ref_in, io->current_contact, io->previous_contact, params_per_leg,
                            best_params, io->state_out, io->ref_out);
    if (rc != SRBD_OK) return rc;
    io->stage = 2;
    float st[24], rf[24];
    for (int i = 0; i < 24; ++i) {
        st[i] = (float)io->state_out[i];
        rf[i] = (float)io->ref_out[i];
    }
    rc = srbd_step(ctx, st, rf, contact, contact_stride, best_params, nullptr, nullptr, seed, counter, out, nullptr);
    if (rc == SRBD_OK) io->stage = 3;
    return rc;
}

// ROS:343-358.  The payload words are written with relaxed atomic stores between the odd and even
// sequence stores, so a reader that sees the same even sequence before and after its copy holds one
// message (release on the closing store; acquire/fence on the reader side).
extern "C" int srbd_shm_publish(uint64_t* seq, double* payload, const srbd_shm_msg* m) {
    if (!seq || !payload || !m) return SRBD_E_INVALID;
    double buf[SRBD_SHM_DOUBLES];
    memcpy(buf + SRBD_SHM_GRF, m->grf, sizeof(double) * 12);
    memcpy(buf + SRBD_SHM_FOOTHOLDS, m->footholds, sizeof(double) * 12);
    memcpy(buf + SRBD_SHM_JOINTS_POS, m->joints_pos, sizeof(double) * 12);
    memcpy(buf + SRBD_SHM_JOINTS_VEL, m->joints_vel, sizeof(double) * 12);
    memcpy(buf + SRBD_SHM_JOINTS_ACC, m->joints_acc, sizeof(double) * 12);
    memcpy(buf + SRBD_SHM_PRED, m->pred, sizeof(double) * 12);
    buf[SRBD_SHM_BEST_FREQ] = m->best_freq;
    buf[SRBD_SHM_LOOP_TIME] = m->loop_time;
    buf[SRBD_SHM_STAMP] = m->stamp;
    const uint64_t s = __atomic_load_n(seq, __ATOMIC_RELAXED);
    if ((s & 1u) == 0) __atomic_store_n(seq, s + 1, __ATOMIC_RELAXED);  // odd: writing
    __atomic_thread_fence(__ATOMIC_RELEASE);
    uint64_t* w = reinterpret_cast<uint64_t*>(payload);
    const uint64_t* b = reinterpret_cast<const uint64_t*>(buf);
    for (int i = 0; i < SRBD_SHM_DOUBLES; ++i) __atomic_store_n(w + i, b[i], __ATOMIC_RELAXED);
    __atomic_store_n(seq, (s | 1u) + 1, __ATOMIC_RELEASE);  // even: stable
    return SRBD_OK;
}

// ROS:565-580.
extern "C" int srbd_shm_read(const uint64_t* seq, const double* payload, srbd_shm_msg* m, uint64_t* seq_out) {
    if (!seq || !payload || !m) return SRBD_E_INVALID;
    const uint64_t s1 = __atomic_load_n(seq, __ATOMIC_ACQUIRE);
    if (s1 & 1u) return 0;
    uint64_t buf[SRBD_SHM_DOUBLES];
    const uint64_t* r = reinterpret_cast<const uint64_t*>(payload);
    for (int i = 0; i < SRBD_SHM_DOUBLES; ++i) buf[i] = __atomic_load_n(r + i, __ATOMIC_RELAXED);
    __atomic_thread_fence(__ATOMIC_ACQUIRE);
    const uint64_t s2 = __atomic_load_n(seq, __ATOMIC_RELAXED);
    if (s1 != s2) return 0;
    const double* d = reinterpret_cast<const double*>(buf);
    memcpy(m->grf, d + SRBD_SHM_GRF, sizeof(double) * 12);
    memcpy(m->footholds, d + SRBD_SHM_FOOTHOLDS, sizeof(double) * 12);
    memcpy(m->joints_pos, d + SRBD_SHM_JOINTS_POS, sizeof(double) * 12);
    memcpy(m->joints_vel, d + SRBD_SHM_JOINTS_VEL, sizeof(double) * 12);
    memcpy(m->joints_acc, d + SRBD_SHM_JOINTS_ACC, sizeof(double) * 12);
    memcpy(m->pred, d + SRBD_SHM_PRED, sizeof(double) * 12);
    m->best_freq = d[SRBD_SHM_BEST_FREQ];
    m->loop_time = d[SRBD_SHM_LOOP_TIME];
    m->stamp = d[SRBD_SHM_STAMP];
    if (seq_out) *seq_out = s2;
    return 1;
}

// ------------------------------------------------------------------ jax.random keys (srbd_jaxrng.h)
extern "C" int srbd_jax_prng_key(uint64_t seed, uint32_t key_out[2]) {  // threefry_seed
    if (!key_out) return SRBD_E_INVALID;
    key_out[0] = (uint32_t)(seed >> 32);
    key_out[1] = (uint32_t)seed;
    return SRBD_OK;
}

extern "C" int srbd_jax_split(const uint32_t key[2], int32_t num, int32_t partitionable, uint32_t* out) {
    if (!key || !out || num < 1) return SRBD_E_INVALID;
    // partitionable: key i = threefry(key, (0, i)); legacy: the 2 num bits of iota(2 num), reshaped (num, 2)
    for (int32_t i = 0; i < num; ++i) {
        if (partitionable) {
            uint32_t x0 = 0, x1 = (uint32_t)i;
            srbd::threefry2x32_20(key[0], key[1], x0, x1);
            out[2 * i] = x0;
            out[2 * i + 1] = x1;
        } else {
            const uint64_t M = 2 * (uint64_t)num;
            out[2 * i] = srbd::jax_bits(key[0], key[1], 2 * (uint64_t)i, M, false);
            out[2 * i + 1] = srbd::jax_bits(key[0], key[1], 2 * (uint64_t)i + 1, M, false);
        }
    }
    return SRBD_OK;
}

// ------------------------------------------------------------------ one plugin-API MPC step in one call
// SRBDControllerInterface.compute_control's sampling branch (srbd_controller_interface.py:113-180) over the plain
// Sampling_MPC (include/srbd_mpc.h srbd_interface_step): prepare_state_and_reference (NMPC:563-627, no solution
// shift), then per sampling iteration with_newkey (NMPC:498-501), CEM's with_newsigma(sigma_cem_mppi) at iteration 0,
// jitted_compute_control (srbd_step on device draws, NMPC:629-1094), and the GRFs times current_contact (SCI:175-178).
// The same calls in the same order as the Python chain, so the same bits.
extern "C" int srbd_interface_step(srbd_ctx* ctx, srbd_interface_io* io, const float* contact,
                                   const double* contact64, int32_t contact_stride, float* best_params,
                                   int32_t params_per_leg, float* sigma, srbd_result* out) {
    if (!ctx || !io || (!contact == !contact64) || !best_params || !out || params_per_leg < 1 ||
        io->iterations < 1 || contact_stride < io->horizon || io->horizon < 1 || io->horizon > SRBD_MAX_HORIZON)
        return SRBD_E_INVALID;
    if (io->cem && !sigma) return SRBD_E_INVALID;
    io->stage = 0;
    int rc = srbd_prepare_state(io->state_in, io->ref_in, io->current_contact, io->previous_contact, params_per_leg,
                                best_params, io->state_out, io->ref_out);
    if (rc != SRBD_OK) return rc;
    io->stage = 1;
    float st[24], rf[24];
    for (int i = 0; i < 24; ++i) {  // the step's float32 staging (Context._stage: numpy's round-to-nearest cast)
        st[i] = (float)io->state_out[i];
        rf[i] = (float)io->ref_out[i];
    }
    float cf[4 * SRBD_MAX_HORIZON];
    const float* cs = contact;
    int32_t stride = contact_stride;
    if (contact64) {
        const int H = io->horizon;
        for (int l = 0; l < 4; ++l)
            for (int k = 0; k < H; ++k) cf[l * H + k] = (float)contact64[(size_t)l * contact_stride + k];
        cs = cf;
        stride = H;
    }
    const int P = 4 * params_per_leg;
    for (int it = 0; it < io->iterations; ++it) {
        uint64_t seed, counter;
        if (io->rng == SRBD_RNG_PHILOX) {  // master_key = (seed, counter + 1)
            io->key[1] += 1;
            seed = io->key[0];
            counter = io->key[1];
        } else {  // master_key = split(master_key)[0]; the call count numbers the device step
            const uint32_t k[2] = {(uint32_t)(io->key[0] >> 32), (uint32_t)io->key[0]};
            uint32_t o[4];
            if ((rc = srbd_jax_split(k, 2, io->rng == SRBD_RNG_JAX ? 1 : 0, o)) != SRBD_OK) return rc;
            io->key[0] = ((uint64_t)o[0] << 32) | o[1];
            io->key[1] += 1;
            seed = io->key[0];
            counter = io->key[1];
        }
        if (io->cem && it == 0)
            for (int j = 0; j < P; ++j) sigma[j] = (float)io->sigma_reset;
        rc = srbd_step(ctx, st, rf, cs, stride, best_params, io->cem ? sigma : nullptr, nullptr, seed, counter, out,
                       nullptr);
        if (rc != SRBD_OK) return rc;
        io->stage = 2 + it;
    }
    for (int l = 0; l < 4; ++l)
        for (int c = 0; c < 3; ++c) io->grf[3 * l + c] = (double)out->grf[3 * l + c] * io->current_contact[l];
    return SRBD_OK;
}
