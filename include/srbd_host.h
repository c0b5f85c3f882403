/*
 * srbd_host.h -- C-ABI of the host-side producers and transports around the sampling MPC step
 * (libsrbd_hip.so).  Plain C++ on the host: no device work.
 *
 *   srbd_pgg_init / srbd_pgg_reset   <- PeriodicGaitGenerator.__init__ / reset
 *                                       quadruped_pympc/helpers/periodic_gait_generator.py:8-46
 *   srbd_pgg_run                     <- PeriodicGaitGenerator.run               :48-76
 *   srbd_pgg_set_phase_signal        <- PeriodicGaitGenerator.set_phase_signal  :78-87
 *   srbd_pgg_contact_sequence        <- PeriodicGaitGenerator.compute_contact_sequence :93-118
 *   srbd_prepare_state               <- Sampling_MPC.prepare_state_and_reference
 *                                       quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py:563-627
 *   srbd_shm_publish / srbd_shm_read <- the MPC -> WBC shared-memory seqlock of ros2/run_controller.py
 *                                       (payload layout :50-83, writer :343-358, reader :565-580)
 *
 * Same conventions as srbd_mpc.h: caller-owned arrays, 0 / negative SRBD_E* codes, no retained
 * pointers.  Arithmetic is float64 in the reference's order (built with -ffp-contract=off).
 */
#ifndef SRBD_HOST_H
#define SRBD_HOST_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* quadruped_pympc/helpers/quadruped_utils.py GaitType values */
enum {
    SRBD_GAIT_TROT = 0,
    SRBD_GAIT_PACE = 1,
    SRBD_GAIT_BOUNDING = 2,
    SRBD_GAIT_CIRCULARCRAWL = 3,
    SRBD_GAIT_BFDIAGONALCRAWL = 4,
    SRBD_GAIT_BACKDIAGONALCRAWL = 5,
    SRBD_GAIT_FRONTDIAGONALCRAWL = 6,
    SRBD_GAIT_FULL_STANCE = 7
};

/* Gait generator state (plain data: the caller may copy, inspect or persist it). */
typedef struct srbd_pgg {
    double duty_factor, step_freq;
    double phase_signal[4];
    double phase_offset[4];
    int32_t init[4];
    int32_t gait_type, previous_gait_type, horizon;
} srbd_pgg;

int srbd_pgg_init(srbd_pgg* g, int32_t gait_type, double duty_factor, double step_freq, int32_t horizon);
/* offsets and phase from gait_type, init cleared (periodic_gait_generator.py:22-46) */
int srbd_pgg_reset(srbd_pgg* g);
/* advance every leg by dt * step_freq and return its contact flag (1.0 / 0.0) */
int srbd_pgg_run(srbd_pgg* g, double dt, double step_freq, double contact_out[4]);
/* init == NULL clears the start-up hold */
int srbd_pgg_set_phase_signal(srbd_pgg* g, const double phase[4], const int32_t* init);
/*
 * Look-ahead contact sequence, row-major 4 x cols into out (capacity out_cap doubles); returns cols
 * (horizon, or 2 * horizon of ones for FULL_STANCE, which also resets the generator) or a negative
 * code.  dts[j] holds for steps i < lens[j] (nonuniform sampling); the state is restored afterwards.
 */
int srbd_pgg_contact_sequence(srbd_pgg* g, const double* dts, const int32_t* lens, int32_t n_dts, double* out,
                              int32_t out_cap);

/*
 * prepare_state_and_reference: state_in = [position, linear_velocity, orientation, angular_velocity,
 * foot_FL, foot_FR, foot_RL, foot_RR] (24), ref_in = [ref_position, ref_linear_velocity,
 * ref_orientation, ref_angular_velocity, ref_foot_FL..RR] (24).  Swing feet (current_contact == 0)
 * take the reference foot; a leg lifting off (previous 1 -> current 0) zeroes its params_per_leg
 * entries of best_params (in/out, 4 * params_per_leg floats; may be NULL).
 */
int srbd_prepare_state(const double state_in[24], const double ref_in[24], const double current_contact[4],
                       const double previous_contact[4], int32_t params_per_leg, float* best_params,
                       double state_out[24], double ref_out[24]);

/* ---- MPC -> WBC shared-memory seqlock (single writer, any number of readers) ---- */
#define SRBD_SHM_DOUBLES 75
enum {
    SRBD_SHM_GRF = 0,         /* 12: GRFs (contact-masked), legs FL FR RL RR */
    SRBD_SHM_FOOTHOLDS = 12,  /* 12 */
    SRBD_SHM_JOINTS_POS = 24, /* 12 */
    SRBD_SHM_JOINTS_VEL = 36, /* 12 */
    SRBD_SHM_JOINTS_ACC = 48, /* 12 */
    SRBD_SHM_PRED = 60,       /* 12: predicted state [p, v, rpy, omega] */
    SRBD_SHM_BEST_FREQ = 72,
    SRBD_SHM_LOOP_TIME = 73,
    SRBD_SHM_STAMP = 74
};

/* One MPC result as the writer packs it (joints may be NULL -> zeros, as the sampling controller). */
typedef struct srbd_shm_msg {
    double grf[12], footholds[12], joints_pos[12], joints_vel[12], joints_acc[12], pred[12];
    double best_freq, loop_time, stamp;
} srbd_shm_msg;

/* Pack and publish: seq odd while writing, even when stable (run_controller.py:343-358).
 * seq and payload (SRBD_SHM_DOUBLES) live in memory shared with the readers. */
int srbd_shm_publish(uint64_t* seq, double* payload, const srbd_shm_msg* msg);
/* Consistent snapshot: returns 1 and fills msg (and *seq_out) when no write overlapped the copy,
 * 0 when the writer was active (caller keeps its previous values), negative on bad arguments. */
int srbd_shm_read(const uint64_t* seq, const double* payload, srbd_shm_msg* msg, uint64_t* seq_out);

/* jax.random keys of the reference's noise stream (srbd_set_rng SRBD_RNG_JAX / SRBD_RNG_JAX_LEGACY; the
 * draws themselves are made on the device).  partitionable: jax_threefry_partitionable (1 = JAX's default
 * since 0.5.0, 0 = earlier JAX).  A key is uint32[2]; srbd_step's `seed` packs it as key[0] << 32 | key[1].
 *   srbd_jax_prng_key <- jax.random.PRNGKey(seed)   quadruped_pympc/controllers/sampling/centroidal_nmpc_jax.py:167
 *   srbd_jax_split    <- jax.random.split(key, num) (with_newkey = split(key)[0], centroidal_nmpc_jax.py:498-501) */
int srbd_jax_prng_key(uint64_t seed, uint32_t key_out[2]);
int srbd_jax_split(const uint32_t key[2], int32_t num, int32_t partitionable, uint32_t* keys_out /* num x 2 */);

#ifdef __cplusplus
}
#endif
#endif /* SRBD_HOST_H */
