/*
 * sacenv.h — C ABI of the MI355X-native vectorised boat environment engine.
 *
 * Drop-in boundary for the hot path of Nilau1998/SAC-Agent: the Gym env
 * `BoatEnv` (environment/boat_env.py:9-140) and everything its step/reset
 * call (Boat dynamics boat_env.py:143-326, Wind wind.py:5-99, RewardFunction
 * reward_functions.py:9-57, Integrator control_theory/control_blocks.py:5-36).
 * The reference has no FFI; its boundary is the Python Gym surface. This
 * library runs that surface's compute as gfx950 HIP kernels over N envs held
 * in one caller-owned device ARENA; the Python package `sac-agent_amd/sacenv`
 * re-exposes the Gym surface on top (INTEGRATION.md shows the bindings).
 *
 * Conventions
 *   - The arena is a DEVICE buffer of sacenv_boat_layout()->total_bytes
 *     bytes owned by the caller (a torch uint8 tensor in the Python host),
 *     zero-filled before sacenv_boat_init(). Its fields are SoA arrays whose
 *     byte offsets sacenv_boat_layout() reports, so an FFI user can view them.
 *   - `params` is HOST memory, read during the call (captured by value into
 *     the launch). It must not change after sacenv_boat_init().
 *   - `stream` is a hipStream_t (void* here so the header needs no HIP
 *     headers); NULL = the default stream. Apart from sacenv_boat_init (one
 *     small host->device copy), every call only enqueues kernels on `stream`:
 *     no host synchronisation, no allocation, graph-capturable.
 *   - Return value: 0 on success, otherwise an SACENV_E_* code (argument
 *     errors) or a hipError_t from the launch (> 0). No exception crosses the
 *     ABI; sacenv_error_string() names the code.
 *   - Float64 arithmetic in the reference's expression order; state is f64.
 */
#ifndef SACENV_H
#define SACENV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SACENV_ABI_VERSION 20
#define SACENV_OBS_DIM 11      /* Boat.return_state, boat_env.py:308-323 */
#define SACENV_MT_N 624        /* MT19937 words per env (numpy legacy RNG) */
#define SACENV_MAX_KNOTS 16    /* wind.fixed_points upper bound */
#define SACENV_N_COUNTERS 5    /* info-dict termination counters, boat_env.py:24-32 */
#define SACENV_SLOTS 257       /* episode slots per env in autoreset mode (active + 256 ahead) */
#define SACENV_REFILL_PERIOD 256 /* autoreset: at most this many step launches between refills */
#define SACENV_RECORD_BYTES 50 /* packed per-env step record (see layout.record) */
#define SACENV_TRANS_OBS 11     /* s' entries in the transition row (the whole obs) */
#define SACENV_TRANS_BYTES 53   /* per-env transition row of sacenv_boat_step_pooled */
#define SACENV_TRANS_BYTES_EXP2 57 /* the same in experiment 2 (+ obs3_next) */
#define SACENV_PAIR_STRIDE 16  /* bytes between envs in the paired f64 state fields */

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
  SACENV_E_SIZE = -4,        /* n_envs / n_ids / wind_len / n_helpers out of range */
  SACENV_E_RANGE = -5,       /* start-y half width < 1 (np.random.randint low >= high) */
  SACENV_E_MODE = -6         /* call not valid in this autoreset mode */
};

/* optional outputs (params.out_flags) */
enum {
  SACENV_OUT_ACCEL = 1,      /* layout.accel: a_x, a_y, a_r of the step (f64) */
  SACENV_OUT_REWARD64 = 2,   /* layout.reward64: reward in f64 */
  SACENV_OUT_KNOTS = 4       /* layout.knots_raw: drawn knot values per slot (allocated only then) */
};

/* Everything the hot path reads from the reference config
 * (configs/original_config.yaml:2-65), plus launch constants. Sums and
 * differences the reference forms from config values are passed pre-formed
 * (the same single IEEE operation). */
typedef struct SacenvBoatParams {
  int32_t n_envs;             /* envs in this arena (per GPU / rank) */
  int32_t experiment;         /* base_settings.experiment, 1..6 (wind.py:26-67) */
  int32_t test_mode;          /* 0 => action drives rudder (boat_env.py:72-73) */
  int32_t wind_len;           /* L = int(t_max/dt) (wind.py:14-15) */
  int32_t n_knots;            /* wind.fixed_points (wind.py:76-78) */
  int32_t fuel0;              /* boat.fuel (boat_env.py:180) */
  int32_t start_y_half;       /* int(0.8*track_width) (boat_env.py:147-150) */
  int32_t max_episode_steps;  /* > 0: truncate (term 6) after this many steps; 0: off */
  int32_t autoreset;          /* 1: envs that end start their next episode inside step */
  int32_t n_helpers;          /* autoreset: workgroups of sacenv_boat_refill's draw launch (1..65536) */
  int32_t out_flags;          /* SACENV_OUT_* bitmask */
  int32_t use_wind_table;     /* 1: wind from layout.wind_table [2][L] for every env */
  double dt, t_max, goal_line, oob_limit, track_width;  /* oob = width + offset (:200-201) */
  double c_r_front, c_r_side, rho, boat_area_front, boat_area_side, boat_l, boat_b, rudder_area;
  double m_plus_mx;           /* (boat_m + boat_m_x) :239 */
  double m_plus_my;           /* (boat_m + boat_m_y) :230, :265 */
  double i_plus_iz;           /* (boat_I + boat_Iz)  :281 */
  double one_minus_wf;        /* (1 - wake_friction) :221 */
  double one_minus_td;        /* (1 - thrust_deduction) :227 */
  double n_rpm;               /* self.n = 20 (:178) */
  double n_times_d;           /* self.n * propeller_diameter (:224) */
  double n_squared;           /* np.square(self.n) (:226) */
  double d_pow4;              /* np.power(propeller_diameter, 4) (:226) */
  double max_velocity;        /* wind.max_velocity */
  double wind_dir_rad;        /* float(wind.direction) * (pi/180) (wind.py:370) */
  double reward_k;            /* (-y_a / y_b), y_a=0.03, y_b=3.4 (reward_functions.py:53) */
  double reward_center;       /* track_width * 0.2 (reward_functions.py:53) */
  double knot_step;           /* (n_knots-1)/(wind_len-1): grid index -> knot coordinate */
  double knot_inv;            /* (wind_len-1)/(n_knots-1): knot coordinate -> grid index */
} SacenvBoatParams;

/* Byte offsets of the arena fields. n_pad = n_envs rounded up to 64; per-env
 * arrays have n_pad entries (entries >= n_envs are padding). */
typedef struct SacenvBoatLayout {
  int64_t total_bytes;
  int64_t n_pad;
  /* Paired f64 fields: stored as 16-B pairs per env, [n_pad][2], env e's element at
   * offset + 16 e: (s_x, s_y) (s_r, v_x) (v_y, v_r) (rudder, ep_reward). t is f64 [n_pad]. */
  int64_t s_x, s_y, s_r, v_x, v_y, v_r, rudder, t, ep_reward;
  int64_t wind_coef;          /* f64 pairs [2 curves][(y0, m0), (y1, m1)][n_pad][2]: the active episode's
                                 spline piece of the interval of the next step's wind sample (a copy of
                                 its slot's wind_knots; a new episode starts with y0 = y(0), exact at
                                 t = 0) */
  int64_t wind0_next;         /* f64 [n_pad][2] autoreset: the next episode's curve values at grid
                                 index 0 (copy, refreshed in each episode's first step) */
  int64_t start_y_next;       /* i32 [n_pad] autoreset: Boat.s_y_start of the next episode (same) */
  int64_t index;              /* i32 [n_pad] steps since reset; fuel = fuel0 - index */
  int64_t cons;               /* i32 [n_pad] episodes started (active slot = cons % SLOTS) */
  int64_t fill;               /* i32 [n_pad] episodes drawn (autoreset; cons < fill <= cons + SLOTS) */
  int64_t mt_pos;             /* i32 [n_pad] bits 0..15: next MT word index (624 => twist first; after
                                 a refill's draw launch up to 1 248, past 624 in mt_next); bit 16: mt_next
                                 holds the block after mt_key. A host write stores the index plain. */
  int64_t start_y;            /* i32 [SLOTS][n_pad] Boat.s_y_start per slot */
  int64_t counters;           /* u32 [5][n_pad] cumulative termination counters */
  int64_t refill_list;        /* i32 [3][n_pad] by refill rank: env, first and end episode number drawn
                                 (sacenv_boat_refill's listing launch writes env, fill, cons; its draw
                                 launch the end episode; its fit launch reads them) */
  int64_t wind_knots;         /* f64 [n_pad][SLOTS][2][n_knots][2]: per episode slot and curve, each
                                 knot's folded value and 2nd derivative / 6 (episode-contiguous:
                                 the refill writes whole lines) */
  int64_t knots_raw;          /* f64 [n_pad][SLOTS][2][n_knots] drawn knot values, only with
                                 SACENV_OUT_KNOTS (else -1: no storage; a refill's fit reads the drawn
                                 knots from the slot's own wind_knots y fields) */
  int64_t mt_key;             /* u32 [n_pad][624] per-env MT19937 state (the current block) */
  int64_t record;             /* u8 [50 n_pad]: obs f32 [n_pad][11] | reward f32 [n_pad]
                                 | done u8 [n_pad] | term u8 [n_pad]  (the all-gather payload) */
  int64_t obs, reward, done, term; /* the four parts of `record` */
  int64_t final_obs;          /* f32 [n_pad][11] terminal obs of envs that auto-reset */
  int64_t final_ep_reward;    /* f64 [n_pad] episode reward of envs that ended */
  int64_t accel;              /* f64 [3][n_pad] a_x, a_y, a_r */
  int64_t reward64;           /* f64 [n_pad] */
  int64_t refill_mask;        /* u64 [n_pad/64]: the refill's scratch (look-back words of its
                                 listing launch: (epoch, envs listed) per 1 024 envs) */
  int64_t status;             /* i32 [64] (256 B): [0] refills done, [1] SACENV_STATUS_* bits,
                                 [2] envs listed by the last refill */
  int64_t spline_g;           /* f64 [n_knots][n_knots]: (m/6) = G @ knots (written by init) */
  int64_t wind_table;         /* f64 [2][wind_len] (velocity, angle), if use_wind_table */
  int64_t last_term;          /* i32 [n_pad] info['termination'] as the reference's info dict keeps it:
                                 the env's last termination code 1..5 (0: none yet); every step
                                 updates it, resets never clear it (boat_env.py:24-32,84-105,120-126;
                                 main.py:83 reads it) */
  int64_t mt_next;            /* u32 [n_pad][624] the block after mt_key, twisted ahead by the refill's
                                 fit launch (valid while mt_pos bit 16 is set) */
} SacenvBoatLayout;

/* status bits (layout.status[1]); sticky until the arena is re-initialised */
enum {
  SACENV_STATUS_SLOT_UNDERFLOW = 1, /* an env restarted past its pre-drawn episodes: more than
                                       SACENV_REFILL_PERIOD step launches without a refill */
  SACENV_STATUS_HANDOFF_TIMEOUT = 2, /* sacenv_boat_segment: an action row's flag never came
                                        (~seconds); the launch stopped stepping */
  SACENV_STATUS_LIST_TIMEOUT = 4      /* sacenv_boat_refill: a listing workgroup's look-back word
                                        never came (~seconds); that refill's list is incomplete */
};
/* hand-off flag value of a wave / workgroup that gave up (sacenv_boat_segment) */
#define SACENV_FLAG_ABORT 0xFFFFFFFFu

int sacenv_abi_version(void);
const char *sacenv_error_string(int code);

/* Validate params and compute the arena layout (host only, no device work). */
int sacenv_boat_layout(const SacenvBoatParams *p, SacenvBoatLayout *out);

/* Seed every env's RNG exactly like np.random.seed(seeds[e]) (legacy MT19937
 * init_genrand; numpy RandomState._legacy_seeding), upload the spline
 * constants, and build every env's first Boat — BoatEnv.__init__ constructs
 * one (boat_env.py:15; Boat.__init__ :144-201, Wind wind.py:26-99) — drawing
 * in the reference's order (randint :147, then 8 knot values per random
 * curve wind.py:78). In autoreset mode the next SLOTS-1 episodes are
 * pre-drawn too (same per-env stream, same order). `seeds` is a DEVICE u32 [n_envs];
 * `obs` (nullable) receives the first observations [n_envs][11] f32. */
int sacenv_boat_init(const SacenvBoatParams *p, void *arena, const uint32_t *seeds, void *stream);

/* BoatEnv.reset (boat_env.py:120-126) for envs ids[0..n_ids) (device i32;
 * ids == NULL: all envs): a new Boat, info['episode_reward'] = 0, obs rows
 * written to layout.obs. Draw order per env is the reference's. */
int sacenv_boat_reset(const SacenvBoatParams *p, void *arena, const int32_t *ids, int32_t n_ids,
                      void *stream);

/* Done-mask compaction: ids (device i32[n]) of the nonzero
 * bytes of done[0..n) in ascending order, and their number in *count (device
 * i32). Stream-ordered; nothing is read back to the host. */
int sacenv_compact_done(const uint8_t *done, int32_t n, int32_t *ids, int32_t *count, void *stream);

/* sacenv_boat_reset for the device-resident list ids[0 .. *count) (count is a
 * DEVICE pointer, e.g. from sacenv_compact_done): BoatEnv.reset for exactly
 * the envs that ended, with no host synchronisation (graph-capturable). */
int sacenv_boat_reset_list(const SacenvBoatParams *p, void *arena, const int32_t *ids,
                           const int32_t *count, void *stream);

/* Non-autoreset mode only: reset with caller-supplied draws (no RNG):
 * start_y[n_ids] (device i32), knots[n_ids][2][n_knots] (device f64,
 * nullable for experiments 1-3 or with the wind table). For replaying
 * recorded episodes. */
int sacenv_boat_reset_explicit(const SacenvBoatParams *p, void *arena, const int32_t *ids,
                               int32_t n_ids, const int32_t *start_y, const double *knots,
                               void *stream);

/* One BoatEnv.step for every env (boat_env.py:67-115); action: device f32
 * [n_envs]. Outputs go to the arena's record (+ optional outputs). With
 * autoreset, an env that ends starts its next (pre-drawn) episode in the same
 * launch: its obs row is the new episode's, the terminal obs is in
 * final_obs. The launch only CONSUMES pre-drawn episodes (no RNG or spline
 * work on the step's path); sacenv_boat_refill replaces them. */
int sacenv_boat_step(const SacenvBoatParams *p, void *arena, const float *action, void *stream);

/* sacenv_boat_step that also writes the step's transitions for a pooled
 * replay buffer (main.py:81-88 -> agent/buffer.py:13-22) to
 * the device row `trans` (SACENV_TRANS_BYTES x n_pad bytes, experiment 2:
 * SACENV_TRANS_BYTES_EXP2; 16-B aligned):
 *   s'       f32 [n_pad][11]  the obs after the step, BEFORE any auto-reset
 *                             (the terminal obs of envs that ended)
 *   reward   f32 [n_pad]
 *   action   f32 [n_pad]      the step's action
 *   term     u8  [n_pad]      termination code; done = term != 0
 *   obs3_next f32 [n_pad]     experiment 2 only: envs that auto-reset, obs[3]
 *                             (normalised start s_y) of the new episode's
 *                             first obs (its other entries are fixed by the
 *                             config: a fresh Boat, boat_env.py:152-198)
 * Each env's s is the previous row's s', or the fresh-Boat obs for envs that
 * ended there (sacenv/dist.py TransitionStream; the staged replay sampler).
 * 53 B per env instead of the record + action + terminal obs (98 B), written
 * by the step launch itself. (ABI 15 and before: s' entries 0..8 only, 45 B,
 * rudder and fuel rebuilt on the receiver; a sampler that gathers single rows
 * out of a segment cannot rebuild them.) */
int sacenv_boat_step_pooled(const SacenvBoatParams *p, void *arena, const float *action, void *trans,
                            void *stream);

/* n_steps sacenv_boat_step calls fused into one launch: replaces n_steps
 * calls of BoatEnv.step (environment/boat_env.py:67-115) with known actions,
 * the loop of main.py:70-114 when the actions are known ahead (SURVEY.md
 * §7.6 K-step rollout). actions is device f32
 * [n_steps][n_envs]; step k's record (the layout.record format, 50 n_pad
 * bytes) goes to records + k * 50 n_pad and, when final_obs is not NULL, the
 * terminal obs of the envs that auto-reset in step k to final_obs +
 * k * 11 n_pad. The carried state stays in registers between the steps.
 * Results equal n_steps step calls bit for bit; counts as n_steps step
 * launches for the refill contract (autoreset: n_steps <= SACENV_REFILL_PERIOD,
 * with a refill at most SACENV_REFILL_PERIOD launches before the last step). */
int sacenv_boat_rollout(const SacenvBoatParams *p, void *arena, const float *actions, int32_t n_steps,
                        void *records, float *final_obs, void *stream);

/* n_steps BoatEnv.step calls (boat_env.py:67-115) in ONE persistent launch,
 * closed-loop safe: the step loop of main.py:70-91 with the env kept on the
 * device between steps. Step ks reads its action row actions + ks *
 * action_stride (device f32, n_envs values per row) and writes the arena's
 * record and final_obs exactly as sacenv_boat_step does; results equal n_steps
 * sacenv_boat_step calls bit for bit (the carried state stays in registers).
 *   Action hand-off, per owner wave w (envs 64w .. 64w+63): when act_ready is
 *   not NULL (device u32 [n_pad/64]), the wave steps ks only once act_ready[w]
 *   >= seq0 + ks + 1 -- a producer (a policy on another stream) writes the
 *   wave's 64 actions of row ks, then releases that value; every row already
 *   published (e.g. act_ready[w] = 0x7fffffff) is the open-loop case.
 *   act_ready == NULL: every row is ready. When step_done is not NULL (device
 *   u32 [n_pad/64]), the wave stores step_done[w] = seq0 + ks + 1 once step
 *   ks's record is visible device-wide (release); the record is rewritten by
 *   step ks+1, which cannot start before row ks+1 is published, so a consumer
 *   that reads step ks's record before publishing row ks+1 sees it intact.
 *   Flags are read device-coherently (sc0 sc1); sequence numbers stay below
 *   2^31 (checked whenever act_ready or step_done is given). A flag that never
 *   comes (~seconds of polling) sets SACENV_STATUS_HANDOFF_TIMEOUT and ends the
 *   launch. Abort protocol: once that bit is set, every later hand-off launch
 *   (this one, sacenv_sac_act_handoff) steps / computes nothing; a wave or
 *   workgroup that gives up stores SACENV_FLAG_ABORT into the flag its peer
 *   waits on, and a peer that reads SACENV_FLAG_ABORT gives up too (it never
 *   reads the rows behind it). The host learns of it from the status bit.
 * trans (nullable, 16-B aligned, trans_stride a multiple of 16): step ks's
 * pooled transition row (sacenv_boat_step_pooled's format) at trans + ks *
 * trans_stride. stage (nullable, 16-B aligned, not with trans): the staged
 * replay rows of sacenv_replay_sample_staged -- ENV-MAJOR (ABI 20): env e, step
 * ks at stage + (e * n_steps + ks) * 64: s' f32 [11] (the obs before any
 * auto-reset), reward f32, action f32, u32 term | last_term << 8 (last_term:
 * layout.last_term after the step), obs3_next f32 (experiment 2), 0 -- written
 * only where bit ks % 64 of stage_marks[e * ceil(n_steps / 64) + ks / 64] is set
 * (u64 [n_pad][ceil(n_steps / 64)]; sacenv_replay_stage_mark: the rows
 * a learn will sample; stage_marks == NULL: every row; with stage_marks, n_steps <=
 * SACENV_REFILL_PERIOD in any mode, else SACENV_E_SIZE). The launch CONSUMES the
 * marks: it clears the words it read (steps 0..n_steps-1), so the next draws into
 * the buffer start from zero (round 6; a stale mark would only write one more
 * row). Counts as n_steps step
 * launches for the refill contract (autoreset: n_steps <= SACENV_REFILL_PERIOD). */
int sacenv_boat_segment(const SacenvBoatParams *p, void *arena, const float *actions, int64_t action_stride,
                        int32_t n_steps, const uint32_t *act_ready, uint32_t *step_done, uint32_t seq0,
                        void *trans, int64_t trans_stride, void *stage, uint64_t *stage_marks,
                        void *stream);

/* Co-residency data for the closed loop (main.py:70-91 on the device): the
 * workgroups per CU the segment launch's kernel can keep resident for these
 * params (with or without pooled rows), its grid (n_pad / 64 one-wave
 * workgroups), its VGPRs per lane as allocated and its LDS bytes per workgroup.
 * It describes the kernel sacenv_boat_segment launches for these params: with
 * more owner waves than the device has SIMDs that is the two-waves-per-SIMD
 * instantiation (constants as literals, <= 256 VGPRs), else the one-wave form.
 * The hand-off only makes progress when every owner wave and every policy
 * workgroup it waits on can be resident at once; sacenv.ClosedLoop plans the
 * policy launches by per-SIMD VGPR and per-CU LDS accounting and refuses a
 * configuration that cannot. No reference counterpart (the reference steps one
 * env on the host). */
/* A HIP stream on a hardware queue of its own (hipExtStreamCreateWithCUMask over
 * every CU; streams with a CU mask never share a queue). The closed loop's policy
 * stream must run CONCURRENTLY with the env stream: ordinary streams are spread
 * over GPU_MAX_HW_QUEUES shared hardware queues, and two that land on one queue
 * serialise -- the persistent env launch queued behind a policy launch that waits
 * for it is a deadlock until the hand-off timeout. */
int sacenv_stream_create_exclusive(void **stream);
int sacenv_stream_destroy(void *stream);

/* with_trans: 0 no rows, 1 pooled transition rows, 2 staged replay rows */
int sacenv_boat_segment_occupancy(const SacenvBoatParams *p, int32_t with_trans, int32_t *blocks_per_cu,
                                  int32_t *grid, int32_t *vgprs, int32_t *lds_bytes);

/* Autoreset mode: draw (RNG, Boat.__init__ boat_env.py:144-201 / Wind
 * wind.py:26-99) and spline-fit the replacement episodes of every env that
 * ended since the previous refill, topping its slot ring up to SLOTS
 * episodes, in the env's own draw order. Call it at least once every
 * SACENV_REFILL_PERIOD step launches (sacenv_boat_step / sacenv_mixed_step),
 * counted from init; more often is harmless. Envs that restart more often
 * than that without a refill set SACENV_STATUS_SLOT_UNDERFLOW. */
int sacenv_boat_refill(const SacenvBoatParams *p, void *arena, void *stream);

/* Wind.get_wind(index) (wind.py:20-24) of each env's CURRENT episode for n
 * (env, index) pairs (device i32 arrays) -> device f64 out arrays. Exposes
 * env.boat.wind.wind_velocity / wind_angle (recorder.py:45-56). */
int sacenv_boat_wind_eval(const SacenvBoatParams *p, const void *arena, const int32_t *env_ids,
                          const int32_t *idx, int32_t n, double *out_velocity, double *out_angle,
                          void *stream);

/* ------------------------------------------------------------------------
 * Toy integrator envs: environment/toy_parachute.py:7-41 and
 * environment/toy_car.py:5-33 (both built on control_blocks.py:5-36
 * Integrator). The reference runs each as a script with no Gym surface; the
 * build exposes them as vectorised envs with the same per-iteration update:
 * one step = one loop iteration, obs = the recorded signals (parachute [s, v],
 * car [s_x, s_y]), reward 0, done when the script's loop would stop. */

enum { SACENV_TOY_PARACHUTE = 1, SACENV_TOY_CAR = 2 };

/* toy termination codes (term array; 5/6 as for the boat) */
enum { SACENV_TOY_TERM_GROUND = 1 /* parachute s < 0: the script's break (:29-30) */ };

typedef struct SacenvToyParams {
  int32_t n_envs;
  int32_t kind;               /* SACENV_TOY_PARACHUTE / SACENV_TOY_CAR */
  int32_t autoreset;          /* 1: an env that ends restarts from the initial state in the step */
  int32_t max_episode_steps;  /* > 0: truncate (term 6) after this many steps */
  double dt;                  /* loop time step: 0.01 parachute (:21), 0.1 car (:20) */
  double t_max;               /* loop end `while t <= t_max`: 500 (both) */
  double integ_dt;            /* Integrator.dt (control_blocks.py:7): 0.1 */
  /* parachute (toy_parachute.py:11-19) */
  double h0, h1, area_closed, area_open, mass, c_w, rho, g;
  /* car (toy_car.py:8-9, :13, :24) */
  double car_accel, car_v_max, car_dangle;
} SacenvToyParams;

/* SoA arena of one toy env type (n_pad = n_envs rounded up to 64). */
typedef struct SacenvToyLayout {
  int64_t total_bytes;
  int64_t n_pad;
  int64_t state;      /* f64 [5][n_pad]: parachute (v_out, s_out, total_a, t, -),
                         car (angle, v_out, s_x_out, s_y_out, t) -- the integrators'
                         STORED (clamped) outputs and the loop variables */
  int64_t count;      /* i32 [n_pad] iterations since reset (Integrator.counter) */
  int64_t counters;   /* u32 [3][n_pad] cumulative: ground, timeout, truncated */
  int64_t record;     /* u8 [14 n_pad]: obs f32 [n_pad][2] | reward f32 | done u8 | term u8 */
  int64_t obs, reward, done, term;
  int64_t final_obs;  /* f32 [n_pad][2] obs of the step that ended (auto-reset) */
} SacenvToyLayout;

int sacenv_toy_layout(const SacenvToyParams *p, SacenvToyLayout *out);
/* initial state of every env (the scripts' variables before the loop) + obs */
int sacenv_toy_init(const SacenvToyParams *p, void *arena, void *stream);
/* restart envs ids[0..n_ids) (NULL: all) from the initial state */
int sacenv_toy_reset(const SacenvToyParams *p, void *arena, const int32_t *ids, int32_t n_ids,
                     void *stream);
/* one loop iteration for every env (no action: the toys are open-loop) */
int sacenv_toy_step(const SacenvToyParams *p, void *arena, void *stream);

/* Mixed batch (BASELINE configs[4]): one launch stepping a boat arena and up
 * to two toy arenas (toy_params[n_toys], toy_arenas[n_toys]) with
 * heterogeneous workgroups (boat owners, then each toy's waves). Equivalent to sacenv_boat_step + sacenv_toy_step per toy arena;
 * bp may be NULL for toys only. */
int sacenv_mixed_step(const SacenvBoatParams *bp, void *boat_arena, const float *boat_action,
                      const SacenvToyParams *toy_params, void *const *toy_arenas, int32_t n_toys,
                      void *stream);
/* sacenv_mixed_step whose boat waves also write the boat's transition row
 * (sacenv_boat_step_pooled's format) to trans; bp must not be NULL. */
int sacenv_mixed_step_pooled(const SacenvBoatParams *bp, void *boat_arena, const float *boat_action,
                             const SacenvToyParams *toy_params, void *const *toy_arenas, int32_t n_toys,
                             void *trans, void *stream);
/* The mixed batch as ONE persistent launch of n_steps steps (the boat as
 * sacenv_boat_segment's open loop: action row ks at boat_actions + ks *
 * action_stride, the carried state in registers; each toy wave runs n_steps
 * iterations of toy_parachute.py:23-40 / toy_car.py:22-32 with its state in
 * registers). Results equal n_steps sacenv_mixed_step calls bit for bit (the
 * arenas, each step's record rewritten in place, the terminal obs of the last
 * restart). Counts as n_steps step launches for the boat's refill contract. */
int sacenv_mixed_segment(const SacenvBoatParams *bp, void *boat_arena, const float *boat_actions,
                         int64_t action_stride, int32_t n_steps, const SacenvToyParams *toy_params,
                         void *const *toy_arenas, int32_t n_toys, void *stream);

/* ------------------------------------------------------------------------
 * Device replay buffer: agent/buffer.py:3-35 ReplayBuffer (SURVEY.md §8(f)
 * rank 1), the consumer of the step records. Same ring semantics
 * (index = mem_cntr % mem_size, buffer.py:14-22) and the same sampling
 * stream: np.random.choice(min(mem_cntr, mem_size), batch) (buffer.py:27)
 * = numpy-legacy masked-rejection randint on an MT19937 state held in the
 * arena, so a buffer seeded like np.random.seed(s) draws the reference's
 * batch indices bit for bit. */

typedef struct SacenvReplayParams {
  int64_t mem_size;        /* ReplayBuffer(max_size) (buffer.py:5) */
  int32_t obs_dim;         /* prod(input_shape) */
  int32_t act_dim;         /* n_actions */
  int32_t reward_f32;      /* 1: store() reads f32 rewards (VecBoatEnv), 0: f64 */
  uint32_t terminal_mask;  /* terminal = (terminal_mask >> code) & 1 for the u8 codes store()
                              receives: 2 = "code 1" (env term: reached_goal, main.py:83-88;
                              or a 0/1 done array) */
} SacenvReplayParams;

typedef struct SacenvReplayLayout {
  int64_t total_bytes;
  int64_t state;      /* f32 [mem_size][obs_dim] state_memory (buffer.py:7) */
  int64_t new_state;  /* f32 [mem_size][obs_dim] new_state_memory (:8) */
  int64_t action;     /* f32 [mem_size][act_dim] action_memory (:9) */
  int64_t reward;     /* f64 [mem_size] reward_memory (:10) */
  int64_t terminal;   /* u8 [mem_size] terminal_memory (:11) */
  int64_t mem_cntr;   /* i64 transitions stored (:6) */
  int64_t mt_key;     /* u32 [624] sampling stream state */
  int64_t mt_pos;     /* i32 next word (624: twist first) */
} SacenvReplayLayout;

int sacenv_replay_layout(const SacenvReplayParams *p, SacenvReplayLayout *out);
/* mem_cntr = 0 and the sampling stream = np.random.seed(seed) */
int sacenv_replay_init(const SacenvReplayParams *p, void *arena, uint32_t seed, void *stream);
/* store_transition (buffer.py:13-22) for n transitions in order: row i goes to
 * (mem_cntr + i) % mem_size; new_state of rows whose code is nonzero is taken
 * from final_state when it is non-NULL (auto-reset envs: the terminal obs).
 * All pointers are device pointers; reward is f32 or f64 per params. */
int sacenv_replay_store(const SacenvReplayParams *p, void *arena, int64_t n, const float *state,
                        const float *action, const void *reward, const float *new_state,
                        const float *final_state, const uint8_t *code, void *stream);
/* store_transition for the n envs of one env step (main.py:81-88): as
 * sacenv_replay_store, and last_term[i] (u8, caller-owned device array of n,
 * zero-initialised = info['termination'] == '') carries env i's
 * info['termination'] across steps and resets like the reference's info dict
 * (boat_env.py:24-32,84-105,120-126): codes 1..5 overwrite it, 0 and 6
 * (truncation) keep it, and terminal = (terminal_mask >> last_term[i]) & 1.
 * last_term == NULL is sacenv_replay_store. */
int sacenv_replay_store_env(const SacenvReplayParams *p, void *arena, int64_t n, const float *state,
                            const float *action, const void *reward, const float *new_state,
                            const float *final_state, const uint8_t *code, uint8_t *last_term,
                            void *stream);
/* sacenv_replay_store_env with the buffer's mem_cntr before this call given by
 * the caller (`cntr`, which a host that issues every store knows): ONE launch,
 * which also sets the device count to cntr + n (sacenv_replay_store_env reads
 * the device count and advances it in a second launch, so it can be captured in
 * a graph; this form cannot: cntr is a launch argument). */
int sacenv_replay_store_env_at(const SacenvReplayParams *p, void *arena, int64_t cntr, int64_t n,
                               const float *state, const float *action, const void *reward,
                               const float *new_state, const float *final_state, const uint8_t *code,
                               uint8_t *last_term, void *stream);
/* sample_buffer(batch) (buffer.py:24-35): indices (i64) and the gathered rows.
 * Any output but idx may be NULL. An empty buffer is an error (SACENV_E_SIZE:
 * np.random.choice(0, n) raises) detected on the host from `stored`. */
int sacenv_replay_sample(const SacenvReplayParams *p, void *arena, int32_t batch, int64_t stored,
                         int64_t *idx, float *state, float *action, double *reward,
                         float *new_state, uint8_t *terminal, void *stream);
/* A replay buffer shared by W ranks without moving the transitions (the
 * pooled buffer of main.py:81-88 / agent/buffer.py:3-35):
 * every rank keeps a full-size ring but writes only its own rows. Per env
 * step the pooled buffer appends `period` transitions in global env order;
 * this rank's n of them start at `offset`. store_shard writes them at ring
 * rows (mem_cntr + offset + i) % mem_size and advances mem_cntr by period
 * (offset + n <= period, n <= mem_size). sample_shard draws the batch exactly
 * as sacenv_replay_sample (every rank's sampling stream, seeded alike, draws
 * the same indices) and gathers the rows THIS rank wrote -- row p holds the
 * latest global sequence number s = p (mod mem_size), s < mem_cntr; it is this
 * rank's iff s mod period lies in [offset, offset + n) -- with the other rows'
 * bytes zero, so an integer SUM all-reduce of the gathered bits over the ranks
 * is the pooled buffer's batch, bit for bit: B rows cross the links per
 * learn() instead of every transition per step. */
int sacenv_replay_store_shard(const SacenvReplayParams *p, void *arena, int64_t n, int64_t offset,
                              int64_t period, const float *state, const float *action, const void *reward,
                              const float *new_state, const float *final_state, const uint8_t *code,
                              uint8_t *last_term, void *stream);
int sacenv_replay_sample_shard(const SacenvReplayParams *p, void *arena, int32_t batch, int64_t stored,
                               int64_t offset, int64_t n, int64_t period, int64_t *idx, float *state,
                               float *action, double *reward, float *new_state, uint8_t *terminal,
                               void *stream);

/* The pooled buffer sampled out of STAGED SEGMENTS (the exchange that scales,
 * DESIGN.md §6): main.py:78-90 with every rank's envs storing their transitions
 * into one ReplayBuffer(mem_size) (buffer.py:13-22) each step and one learn() --
 * sample_buffer(batch), buffer.py:24-35 -- after every step, WITHOUT a ring: the
 * index draws are made ahead, the persistent step launch writes the rows they
 * will read (sacenv_boat_segment's stage: 64 B per step and env), and the
 * segment's learns are gathered from them afterwards. The pooled ring appends `period` = world x n rows per step in
 * global env order; with mem_size <= seg x period every row learn k of segment
 * g can reach was written in segment g or g - 1, so those two buffers are the
 * ring. Global step numbers: segment g holds steps g*seg .. g*seg + seg - 1. */
typedef struct SacenvStagedParams {
  int64_t period;        /* pooled rows per step: world x n */
  int64_t offset;        /* this rank's first global env (rank x n) */
  int32_t n;             /* this rank's envs */
  int32_t n_pad;         /* the env arena's n_pad: the rows' field stride */
  int32_t seg;           /* steps (rows) per segment buffer */
  int32_t experiment;    /* 2: the rows carry obs3_next */
  float first_obs[SACENV_OBS_DIM]; /* a fresh Boat's obs (boat_env.py:152-198 -> return_state) */
} SacenvStagedParams;

/* Device scratch of sacenv_replay_stage_draw for this buffer and batch shape. */
int sacenv_replay_stage_scratch_bytes(const SacenvReplayParams *p, int32_t batch, int32_t n_batches,
                                      int64_t *bytes);
/* The index draws of the n_batches learn() calls after steps g*seg ..
 * g*seg + n_batches - 1: batch k = np.random.choice(min(c_k, mem_size), batch)
 * on the arena's sampling stream (seeded like np.random.seed), c_k = (g*seg +
 * k + 1) x period transitions stored; fewer than `batch`: learn() returns
 * before sampling (continuous_agent.py:97-98), idx = -1 and no words drawn.
 * idx: i64 [n_batches][batch]. Call for g = 0, 1, 2, ... in order; the draws
 * depend only on the stream and the counts, so segment g's may be drawn
 * before it steps. Once every learn of the segment samples [0, mem_size),
 * the stream's MT blocks are generated by one wave and the accepted words
 * ranked over the whole stream by many workgroups (scratch: a device buffer of
 * sacenv_replay_stage_scratch_bytes); before that, one workgroup draws them in
 * order. */
int sacenv_replay_stage_draw(const SacenvReplayParams *p, void *arena, const SacenvStagedParams *sp, int64_t g,
                             int32_t batch, int32_t n_batches, int64_t *idx, void *scratch, int64_t scratch_bytes,
                             void *stream);
/* The rows of segment g some learn will read (u64 [n_pad][ceil(seg / 64)], bit
 * j % 64 of env e's word j / 64 for step j, as sacenv_boat_segment reads them;
 * cleared first): every row the draws of segment g (idx_g) and g + 1
 * (idx_next, nullable) sample that lies in segment g on this rank, and the row
 * before it (its s). sacenv_boat_segment writes exactly these (stage_marks). */
int sacenv_replay_stage_mark(const SacenvReplayParams *p, const SacenvStagedParams *sp, int64_t g,
                             const int64_t *idx_g, const int64_t *idx_next, int32_t batch, int32_t n_batches,
                             uint64_t *marks, void *stream);
/* The batches of segment g's learns (idx from sacenv_replay_stage_draw): each
 * sampled ring row resolves to the transition the pooled ring holds there at
 * learn k; this rank's are read from the staged rows of stage_cur (segment g)
 * and stage_prev (segment g - 1; for g = 0 its last row holds the obs every env
 * starts from, term 0): s' = the row's obs, s = the previous step's s' or,
 * where that step ended, the fresh-Boat obs (first_obs; experiment 2 with that
 * row's obs3_next), reward, action, terminal = (terminal_mask >> last_term) & 1
 * (main.py:83-88). Output `words` (u32, n_batches x 26 batch), per batch:
 * reward f64 [batch] (two words each) | state f32 [batch][11] | new_state f32
 * [batch][11] | action f32 [batch] | terminal u32 [batch]; other ranks' rows
 * are zero words, so an integer SUM all-reduce over the ranks is the pooled
 * buffer's batches, bit for bit, on every rank. Needs obs_dim 11, act_dim 1,
 * mem_size <= seg x period. */
int sacenv_replay_sample_staged(const SacenvReplayParams *p, const SacenvStagedParams *sp, int64_t g,
                                const void *stage_cur, const void *stage_prev, const int64_t *idx, int32_t batch,
                                int32_t n_batches, uint32_t *words, void *stream);

/* The rows of a replay arena at given indices (idx: i64 [batch], device): the
 * gather half of sacenv_replay_sample (buffer.py:28-33) without the draw; an
 * index outside [0, mem_size) gives zero bits. Any output may be NULL. */
int sacenv_replay_gather(const SacenvReplayParams *p, void *arena, int32_t batch, const int64_t *idx,
                         float *state, float *action, double *reward, float *new_state, uint8_t *terminal,
                         void *stream);

/* The COUNTER-BASED sampler of the staged replay (round 6): the
 * draws of sacenv_replay_stage_draw with the same distribution per learn --
 * np.random.choice(min(c_k, mem_size), batch): uniform with replacement over
 * the rows stored, learns with c_k < batch skipped (idx -1) -- from
 * Philox4x64-10 (numpy's np.random.Philox generator function) instead of one
 * MT19937 stream: draw i of global learn L = g*seg + k is the first of the
 * four 64-bit words of Philox4x64-10(counter (i, L, j, 0), key (seed, 0)),
 * j = 0, 1, ..., whose bits under numpy's mask (the smallest 2^b - 1 >= range
 * - 1) are <= range - 1. Every draw is independent, so a segment's draws are
 * one parallel launch with no sequential chain, in any order, for any g. The
 * same thread marks the rows it draws on this rank and their predecessors:
 * rows of segment g in marks_cur, of segment g - 1 in marks_prev (u64
 * [n_pad][ceil(seg / 64)] each, nullable, NOT cleared: a segment's marks start from zero --
 * cleared by the caller, or by the sacenv_boat_segment launch that consumed them
 * last). Drawing segments g and g + 1 completes segment g's marks
 * (sacenv_replay_stage_mark's set). tiles (nullable, i32 [ceil(n_batches x
 * batch / 256)]): the records per 256-slot tile this rank's
 * sacenv_replay_stage_pack of segment g will write (pass them there with
 * counted = 1: no count pass). */
int sacenv_replay_stage_draw_ctr(const SacenvReplayParams *p, const SacenvStagedParams *sp, int64_t g,
                                 int32_t batch, int32_t n_batches, uint64_t seed, int64_t *idx,
                                 uint64_t *marks_prev, uint64_t *marks_cur, int32_t *tiles, void *stream);
/* The ALL-GATHER form of the staged exchange. stage_chunk: the record capacity
 * of one rank's chunk (the most records any rank packs in expectation over any
 * segment + 8 standard deviations + 64; every slot at one rank) and the chunk's
 * bytes (a 16-B header, 100 B per record, 256-B multiple). stage_pack: this
 * rank's rows of segment g's learns (as sacenv_replay_sample_staged reads
 * them) as 25-word records -- slot (learn x batch + draw) | terminal << 31,
 * reward f32, state [11], new_state [11], action -- behind the count, in slot
 * order (no atomics: the chunk's bytes are the same run to run); rank 0
 * (offset 0) also packs the skipped learns' all-zero rows; `tiles` is device
 * scratch of ceil(n_batches x batch / 256) i32 (counted = 1: it holds the tile
 * counts sacenv_replay_stage_draw_ctr wrote for segment g). stage_unpack: the
 * world chunks of an all-gather (rank r's at r x chunk_bytes) into
 * sacenv_replay_sample_staged's words, bit for bit; a count above cap sets
 * bit 0 of *status_word (device i32). */
int sacenv_replay_stage_chunk(const SacenvReplayParams *p, const SacenvStagedParams *sp, int32_t batch,
                              int32_t n_batches, int64_t *cap_rows, int64_t *chunk_bytes);
int sacenv_replay_stage_pack(const SacenvReplayParams *p, const SacenvStagedParams *sp, int64_t g,
                             const void *stage_cur, const void *stage_prev, const int64_t *idx, int32_t batch,
                             int32_t n_batches, int64_t cap, void *chunk, int32_t *tiles, int32_t counted,
                             void *stream);
int sacenv_replay_stage_unpack(int32_t world, int64_t chunk_bytes, int64_t cap, int32_t batch, int32_t n_batches,
                               const void *gathered, uint32_t *words, int32_t *status_word, void *stream);
/* One segment's side work of the counter-based, all-gather staged exchange in ONE
 * launch (ABI 20): sacenv_replay_stage_draw_ctr of segment draw_g (draw_g < 0:
 * none), sacenv_replay_stage_pack of segment pack_g with counted tiles (pack_g <
 * 0: none) and sacenv_replay_stage_unpack of `gathered` (NULL: none), each
 * bit-identical to its own entry point. The three run side by side, so their
 * buffers must be disjoint: the pack's idx / tiles are not the draws' (ring them,
 * as sacenv.replay.StagedReplay does: draws of g + 2 beside the pack of g), and
 * the chunk the pack writes is not in the gathered range the unpack reads
 * (SACENV_E_RANGE). cap is the chunk's record capacity (pack and unpack). */
typedef struct SacenvStageSide {
  int64_t draw_g;           /* segment whose learns are drawn; < 0: no draws */
  uint64_t seed;
  int64_t *draw_idx;        /* i64 [n_batches x batch] */
  uint64_t *marks_prev;     /* nullable (draw_g == 0) */
  uint64_t *marks_cur;
  int32_t *draw_tiles;      /* i32 [ceil(n_batches x batch / 256)] */
  int64_t pack_g;           /* segment packed; < 0: no pack */
  const void *stage_cur;
  const void *stage_prev;
  const int64_t *pack_idx;  /* segment pack_g's draws */
  const int32_t *pack_tiles;/* and their tile counts */
  int64_t cap;
  void *chunk;
  const void *gathered;     /* world chunks to unpack; NULL: no unpack */
  int64_t chunk_bytes;
  uint32_t *words;
  int32_t *status_word;
  int32_t world;
  int32_t reserved;
} SacenvStageSide;
int sacenv_replay_stage_side(const SacenvReplayParams *p, const SacenvStagedParams *sp, int32_t batch,
                             int32_t n_batches, const SacenvStageSide *work, void *stream);
/* A collective's kernel stood in for on one GPU (bench.py's N = 1 replay path):
 * `workgroups` workgroups of 256 threads copy `bytes` (16-B multiple, aligned)
 * from src to dst and stay resident until min_us have passed since each
 * started (<= 1e5). No reference counterpart. */
int sacenv_copy_standin(const void *src, void *dst, int64_t bytes, int32_t workgroups, double min_us,
                        void *stream);

/* ------------------------------------------------------------------------
 * SAC agent on the device: the batched
 * policy of ContinuousAgent.choose_action (agent/continuous_agent.py:57-61)
 * and one ContinuousAgent.learn (:96-154) over the five networks of
 * networks/networks.py:14-133 (actor, critic 1, critic 2, value, target
 * value: 256-256 MLPs, f32), as fp32 MFMA kernels (v_mfma_f32_16x16x4_f32).
 *
 * All five networks, the four Adam states and the kernel-side transposes of
 * the 256x256 layers (kernel copies in MFMA fragment order) live in one caller-owned f32 WEIGHTS buffer of
 * sacenv_sac_layout()->total_floats floats. Net n starts at layout.net[n]
 * (0 actor, 1 critic 1, 2 critic 2, 3 value, 4 target value); inside a net
 * the tensors sit at layout.tensor[shape][k] (shape 0 actor, 1 critic,
 * 2 value; k = fc1.weight [256][in], fc1.bias, fc2.weight [256][256],
 * fc2.bias, head-0 weight [256], head-0 bias, head-1 weight, head-1 bias;
 * -1 where absent): the torch layout of nn.Linear, so the host can view each
 * parameter in place. Adam's exp_avg / exp_avg_sq of net n < 4 start at
 * adam_m[n] / adam_v[n] with the same inner offsets. After the host writes
 * weights, sacenv_sac_sync() refreshes the kernel copies; learn keeps them.
 * `scratch` is a device buffer of layout.scratch_bytes (no contents kept
 * between calls). Same conventions as above: device pointers, host params,
 * stream-ordered, graph-capturable, 0 or an SACENV_E_* / hipError_t. */

#define SACENV_SAC_HIDDEN 256   /* layer1_size = layer2_size (original_config.yaml:18-19) */

typedef struct SacenvSacParams {
  int32_t obs_dim;       /* input_dims[0] (11 for the boat), 1..14: the critic's fc1 input
                            is obs_dim + the action + a bias column of ones, in 16 columns */
  int32_t n_actions;     /* 1 (the boat's action_space.shape) */
  int32_t hidden;        /* SACENV_SAC_HIDDEN */
  int32_t batch;         /* learn batch (batch_size), a multiple of 256 */
  /* Python floats of the reference; the kernels cast them to f32 where torch does */
  double max_action;     /* action_space.high[0] (base_agent.py:15-17) */
  double gamma;          /* agent.gamma */
  double tau;            /* agent.tvn_parameter_modulation_tau */
  double reward_scale;   /* agent.reward_scale */
  double lr_actor;       /* agent.learning_rate_alpha */
  double lr_critic;      /* agent.learning_rate_beta (critics, value) */
  double adam_beta1, adam_beta2, adam_eps;  /* torch.optim.Adam defaults 0.9, 0.999, 1e-8 */
} SacenvSacParams;

typedef struct SacenvSacLayout {
  int64_t total_floats;
  int64_t net[5];
  int64_t adam_m[4];
  int64_t adam_v[4];
  int64_t w2f[5];          /* kernel copy of fc2.weight in MFMA fragment order, nets 0..4 */
  int64_t w2tf[4];         /* the same of fc2.weight transposed, nets 0..3 */
  int64_t net_floats[3];   /* floats of one net per shape */
  int64_t tensor[3][8];
  int64_t scratch_bytes;
} SacenvSacLayout;

int sacenv_sac_layout(const SacenvSacParams *p, SacenvSacLayout *out);
/* rebuild the kernel copies of the 256x256 layers from the weights (after the host wrote them) */
int sacenv_sac_sync(const SacenvSacParams *p, float *weights, void *stream);
/* choose_action for n observations [n][obs_dim]: action = tanh(mean + eps*std)
 * * max_action with the given standard normal draws eps [n] (networks.py:47-70,
 * reparameterize=False); log_prob [n] may be NULL. */
int sacenv_sac_act(const SacenvSacParams *p, const float *weights, const float *obs, int32_t n,
                   const float *eps, float *action, float *log_prob, void *stream);
/* sacenv_sac_act as the producer of a closed loop with sacenv_boat_segment
 * (main.py:70-91: choose_action, then env.step, with no launch boundary on the
 * env side): the 64 rows of workgroup b are owner wave b's envs; it reads its
 * obs rows once obs_ready[b] >= obs_want (the segment's step_done flags) and,
 * once its actions are visible device-wide, stores act_ready[b] = act_value
 * (the segment's act_ready flags). Values below 2^31; a flag that never comes
 * (~seconds) sets SACENV_STATUS_HANDOFF_TIMEOUT in *status (nullable). */
/* The hand-off act kernel's resident workgroups per CU, its grid for n rows (64
 * rows per 256-thread workgroup), VGPRs per lane and LDS bytes per workgroup:
 * the policy half of the closed loop's co-residency plan. */
int sacenv_sac_act_occupancy(int32_t n, int32_t *blocks_per_cu, int32_t *grid, int32_t *vgprs,
                             int32_t *lds_bytes);

int sacenv_sac_act_handoff(const SacenvSacParams *p, const float *weights, const float *obs, int32_t n,
                           const float *eps, float *action, const uint32_t *obs_ready, uint32_t obs_want,
                           uint32_t *act_ready, uint32_t act_value, int32_t *status, void *stream);
/* one learn() on a sampled batch (state, new_state f32 [batch][obs_dim],
 * action f32 [batch], reward f64 [batch] as sample_buffer returns it, done u8
 * [batch]) with the policy draws of its sample() (eps1) and rsample() (eps2),
 * f32 [batch]. adam_step = the optimizers' step count after this call (1 on
 * the first; a captured graph replays the step it was captured with, so
 * capture one graph per step value or call eagerly). losses (device f32 [4],
 * may be NULL) <- value, actor, critic 1, critic 2 losses. Calls on one
 * weights/scratch pair must be ordered on one stream. */
int sacenv_sac_learn(const SacenvSacParams *p, float *weights, void *scratch, const float *state,
                     const float *action, const double *reward, const float *new_state,
                     const uint8_t *done, const float *eps1, const float *eps2, int32_t adam_step,
                     float *losses, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* SACENV_H */
