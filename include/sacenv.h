/*
 * sacenv.h — C ABI of the MI355X-native vectorised boat environment engine.
 *
 * Drop-in boundary for the hot path of Nilau1998/SAC-Agent: the Gym env
 * `BoatEnv` (environment/boat_env.py:9-140) and everything its step/reset
 * call (Boat dynamics boat_env.py:143-326, Wind wind.py:5-99, RewardFunction
 * reward_functions.py:9-57, Integrator control_theory/control_blocks.py:5-36).
 * The reference has no FFI; its boundary is the Python Gym surface. This
 * library replaces that surface's compute with gfx950 HIP kernels over N
 * envs held as structure-of-arrays in HBM; the Python package
 * `sac-agent_amd/sacenv` re-exposes the Gym surface on top.
 *
 * Conventions
 *   - Every pointer inside the structs and every array argument is a DEVICE
 *     pointer owned by the caller (torch tensors in the Python host).
 *   - The params / state / out structs themselves are HOST memory; they are
 *     read during the call only (captured by value into the launch).
 *   - `stream` is a hipStream_t (void* here so the header needs no HIP
 *     headers); NULL = the default stream. Every call only enqueues work on
 *     `stream`: no host synchronisation, no allocation, graph-capturable.
 *   - Return value: 0 on success, otherwise an SACENV_E_* code (argument
 *     errors) or a hipError_t from the launch (> 0). No exception crosses
 *     the ABI. sacenv_error_string() names the code.
 *   - Bit-for-bit the reference's float64 arithmetic order; state is f64.
 */
#ifndef SACENV_H
#define SACENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SACENV_ABI_VERSION 1
#define SACENV_OBS_DIM 11      /* Boat.return_state, boat_env.py:308-323 */
#define SACENV_MT_N 624        /* MT19937 words per env (numpy legacy RNG) */
#define SACENV_MAX_KNOTS 16    /* wind.fixed_points upper bound */
#define SACENV_N_COUNTERS 5    /* info-dict termination counters, boat_env.py:24-32 */

/* termination codes; 1..5 follow the info-dict key order boat_env.py:24-32,
 * the chain's priority stays goal > oob > fuel > timeout > rudder (:84-105). */
enum {
  SACENV_TERM_NONE = 0,
  SACENV_TERM_REACHED_GOAL = 1,
  SACENV_TERM_OUT_OF_BOUNDS = 2,
  SACENV_TERM_OUT_OF_FUEL = 3,
  SACENV_TERM_RUDDER_BROKEN = 4,
  SACENV_TERM_TIMEOUT = 5,
  SACENV_TERM_TRUNCATED = 6 /* harness time limit (max_episode_steps); not a reference termination */
};

enum {
  SACENV_OK = 0,
  SACENV_E_NULL = -1,        /* required pointer is NULL */
  SACENV_E_EXPERIMENT = -2,  /* experiment not in 1..6  (wind.py:65-67 ValueError) */
  SACENV_E_KNOTS = -3,       /* fixed_points < 4 or > SACENV_MAX_KNOTS (wind.py:73-75) */
  SACENV_E_SIZE = -4,        /* n_envs / n_ids / wind_len out of range */
  SACENV_E_RANGE = -5        /* start-y half width < 1 (np.random.randint low >= high) */
};

/* Everything the hot path reads from the reference config
 * (configs/original_config.yaml:2-65), plus derived launch constants. */
typedef struct SacenvBoatParams {
  int32_t n_envs;             /* envs held by this state (per GPU / rank) */
  int32_t experiment;         /* base_settings.experiment, 1..6 (wind.py:26-67) */
  int32_t test_mode;          /* base_settings.test_mode; 0 => action drives rudder (boat_env.py:72-73) */
  int32_t wind_len;           /* L = int(t_max/dt) (wind.py:14-15) */
  int32_t n_knots;            /* wind.fixed_points (wind.py:76-78) */
  int32_t fuel0;              /* boat.fuel (boat_env.py:180) */
  int32_t start_y_half;       /* int(0.8*track_width) (boat_env.py:147-150) */
  int32_t max_episode_steps;  /* > 0: truncate (term 6) after this many steps; 0: off */
  int32_t autoreset;          /* 1: envs that end are reset inside step (obs row = reset obs) */
  int32_t reserved0;
  double dt, t_max, goal_line, oob_limit, track_width;  /* oob = width + offset (:200-201) */
  double boat_m, boat_m_x, boat_m_y, boat_I, boat_Iz;
  double propeller_diameter, wake_friction, c_r_front, c_r_side, thrust_deduction, rho;
  double boat_area_front, boat_area_side, boat_l, boat_b, rudder_area;
  double n_rpm;               /* 20, boat_env.py:178 */
  double max_velocity;        /* wind.max_velocity */
  double wind_dir_rad;        /* float(wind.direction) * (pi/180) (wind.py:370) */
  double reward_k;            /* (-y_a / y_b) with y_a=0.03, y_b=3.4 (reward_functions.py:53) */
  double reward_center;       /* track_width * 0.2 */
  double knot_step;           /* (n_knots-1)/(wind_len-1): grid index -> knot coordinate */
  double obs_lo[SACENV_OBS_DIM], obs_hi[SACENV_OBS_DIM]; /* normalize() bounds, :310-321 */
  const double *spline_g;     /* [n_knots*n_knots]: (m/6) = G @ knots, not-a-knot cubic */
  const double *wind_table;   /* NULL, or [2][wind_len] (velocity, angle) shared by all envs */
} SacenvBoatParams;

/* Per-env carried state, SoA, length n_envs unless noted. */
typedef struct SacenvBoatState {
  double *s_x, *s_y, *s_r;    /* position integrator outputs (get_kinematics :297-306) */
  double *v_x, *v_y, *v_r;    /* velocity integrator outputs (run_model_step :205-209) */
  double *rudder;             /* Boat.rudder_angle (f64, pinned-numpy semantics) */
  double *t;                  /* Boat.t, accumulated t += dt (:69) */
  double *ep_reward;          /* info['episode_reward'] (:113, :122) */
  int32_t *index;             /* Boat.index == steps since reset (:155, :211); fuel = fuel0 - index */
  int32_t *start_y;           /* Boat.s_y_start (:147-150) */
  double *wind_y;             /* [2][n_knots][n_envs] folded knot values of the wind curves */
  double *wind_m;             /* [2][n_knots][n_envs] folded second derivatives / 6 */
  double *knots_raw;          /* NULL, or [2][n_knots][n_envs]: the drawn knot values (debug) */
  uint32_t *mt_key;           /* [n_envs][624] per-env MT19937 state (np.random legacy) */
  int32_t *mt_pos;            /* [n_envs] next word index in mt_key, 624 => twist first */
  uint32_t *counters;         /* [5][n_envs] cumulative termination counters (never reset) */
} SacenvBoatState;

/* Step outputs. obs/reward/done/term are required; the rest may be NULL. */
typedef struct SacenvBoatStepOut {
  float *obs;                 /* [n_envs][11] (reset obs for envs auto-reset this step) */
  float *reward;              /* [n_envs] */
  uint8_t *done;              /* [n_envs] 1 if term != 0 */
  uint8_t *term;              /* [n_envs] SACENV_TERM_* */
  float *final_obs;           /* [n_envs][11] terminal obs, written only where done && autoreset */
  double *final_ep_reward;    /* [n_envs] episode reward, written only where done */
  double *accel;              /* [3][n_envs] a_x, a_y, a_r of this step */
  double *reward64;           /* [n_envs] reward in float64 */
} SacenvBoatStepOut;

int sacenv_abi_version(void);
const char *sacenv_error_string(int code);

/* np.random.seed(seeds[e]) for every env: legacy MT19937 init_genrand.
 * Replaces the global-RNG seeding the reference relies on (boat_env.py:147,
 * wind.py:78; numpy RandomState._legacy_seeding). */
int sacenv_boat_seed(const SacenvBoatParams *p, const SacenvBoatState *s,
                     const uint32_t *seeds, void *stream);

/* Boat(config) for envs ids[0..n_ids) (ids == NULL: all n_envs), consuming
 * each env's RNG in the reference's order (randint, then 8 knots per random
 * wind curve), info['episode_reward'] = 0, and writes their obs rows.
 * Replaces BoatEnv.reset (boat_env.py:120-126) / Boat.__init__ (:144-201)
 * and Wind.generate_wind (wind.py:26-99). obs may be NULL. */
int sacenv_boat_reset(const SacenvBoatParams *p, const SacenvBoatState *s,
                      const int32_t *ids, int32_t n_ids, float *obs, void *stream);

/* As sacenv_boat_reset but with the draws supplied by the caller (no RNG):
 * start_y[n_ids], knots[n_ids][2][n_knots] (knots may be NULL for
 * experiments 1-3). For replaying recorded episodes. */
int sacenv_boat_reset_explicit(const SacenvBoatParams *p, const SacenvBoatState *s,
                               const int32_t *ids, int32_t n_ids, const int32_t *start_y,
                               const double *knots, float *obs, void *stream);

/* One BoatEnv.step for every env (boat_env.py:67-115): action[n_envs] f32.
 * With p->autoreset, envs that end are reset in the same launch. */
int sacenv_boat_step(const SacenvBoatParams *p, const SacenvBoatState *s,
                     const float *action, const SacenvBoatStepOut *out, void *stream);

/* Wind.get_wind for n (env, index) pairs (wind.py:20-24); used to expose
 * env.boat.wind.wind_velocity / wind_angle tables (recorder.py:45-56). */
int sacenv_boat_wind_eval(const SacenvBoatParams *p, const SacenvBoatState *s,
                          const int32_t *env_ids, const int32_t *idx, int32_t n,
                          double *out_velocity, double *out_angle, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SACENV_H */
