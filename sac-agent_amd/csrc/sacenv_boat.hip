// sacenv_boat.hip — gfx950 kernels + C ABI for the vectorised boat env.
//
// The step launch (k_step) runs owner waves only: one lane per env, 64
// consecutive envs per wave, BoatEnv.step (boat_env.py:67-115) on float64
// SoA state. In autoreset mode an env that ends (terminated or truncated)
// starts its next episode at once from a PRE-DRAWN slot (SLOTS = 257 per env:
// the active episode + 256 ahead), so no RNG or spline work ever sits on the
// step's path, and the step keeps no refill bookkeeping beyond the episode
// counter `cons`.
// The refill launches (at least every 256 steps): k_need_masks marks the envs
// whose ring is short (fill < cons + SLOTS); k_refill ranks them from those
// masks (DPP scans, no atomics) and, one wave per env, draws
// the replacement episodes from the env's own numpy-legacy MT19937 stream
// (Boat.__init__ boat_env.py:144-201: randint, then the wind knots,
// wind.py:69-90), fits the not-a-knot spline, finds its exact grid-sample
// min/max from the critical points (instead of the reference's 10 000-sample
// scan, wind.py:80-89) and k_refill_fit stores the renormalised, scaled curve
// (wind.py:86-99). Kept out of the step launch, this work no longer shares
// SIMDs with the owners (measured: in-step helper waves cost 1.6 us/step).
//
// Floating-point order follows the reference expression by expression
// (left-to-right products, no FMA contraction: -ffp-contract=off); the only
// differences from the CPU step are the libm/ocml transcendentals.

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "sacenv.h"

#pragma clang fp contract(off)

namespace {

constexpr int kWave = 64;
constexpr int kMtN = SACENV_MT_N;
constexpr int kMtM = 397;
constexpr uint32_t kMtUpper = 0x80000000u;
constexpr uint32_t kMtLower = 0x7fffffffu;
constexpr uint32_t kMtMatrixA = 0x9908b0dfu;
constexpr int kMaxK = SACENV_MAX_KNOTS;
constexpr int kSlots = SACENV_SLOTS;
constexpr double kPi = 3.141592653589793;  // np.pi

// ---------------------------------------------------------------- arena
// Per-env byte widths; a field's offset is (sum of widths before it) * n_pad.
// n_pad is a multiple of 64, so every array is 64-byte aligned.
// U_COEF / U_W0N / U_SYN are lane-coalesced copies of slot data the step
// reads every launch (see owner_wave): the active episode's spline piece
// (y0, y1, m0, m1 per curve) of the interval of this step's wind sample, and
// the next episode's curve values at grid index 0 and start y. Slots differ
// from env to env, so reading them from the slot ring itself would scatter
// every wave's loads over up to 33 rows. U_COEF follows the carried state
// directly: fields 0..16 are loaded as one run (owner_load).
constexpr int U_SX = 0, U_SY = 8, U_SR = 16, U_VX = 24, U_VY = 32, U_VR = 40, U_RUD = 48,
              U_EP = 56, U_COEF = 64, U_W0N = 128, U_T = 144, U_IDX = 152,
              U_CONS = 156, U_FILL = 160, U_MTPOS = 164, U_SYN = 168, U_STARTY = 172,
              U_CNT = U_STARTY + 4 * kSlots,
              U_LIST = U_CNT + 4 * SACENV_N_COUNTERS, U_CSNAP = U_LIST + 12, U_LTERM = U_CSNAP + 4,
              U_WIND = U_LTERM + 4;
constexpr int U_MT_BYTES = 4 * kMtN;
// U_MTPOS holds the MT word index (bits 0..15, up to 2 x 624) and kMtNextOk:
// mt_next holds the block after mt_key (twisted ahead by the refill's fit
// launch), so a draw window may run past the block end without a twist; an
// index past 624 then reads mt_next, and the fit launch makes it current.
// Every other writer of the index (the wave-path draws, seeding, the host)
// stores it plain, which withdraws the pre-twisted block.
constexpr int kMtPosMask = 0xFFFF, kMtNextOk = 1 << 16;
// The f64 fields below U_PAIRED are stored as 16-B pairs per env, [n_pad][2]:
// (s_x, s_y) (s_r, v_x) (v_y, v_r) (rudder, ep_reward), the spline piece as
// (y0, m0) (y1, m1) per curve, and the two next-episode y0. A field's pair
// block starts at (u & ~15) * n_pad and it is element (u & 8) / 8 of each
// pair, so the step moves them with 16-B per-lane loads and stores.
constexpr int U_PAIRED = 144;
constexpr int64_t kWindUnits = 16LL * kSlots;  // f64 x 2 curves x slots, per knot

__host__ __device__ inline int64_t pad64(int64_t n) { return (n + 63) / 64 * 64; }
__host__ __device__ inline int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

__host__ __device__ inline void compute_layout(int n, int nk, int L, int use_table, int raw_knots,
                                               SacenvBoatLayout* o) {
  const int64_t np = pad64(n), nw = np / 64;
  o->n_pad = np;
  // paired fields: the offset of env 0's element; consecutive envs are 16 B apart
  auto pair_off = [np](int u) { return (int64_t)(u & ~15) * np + (u & 8); };
  o->s_x = pair_off(U_SX);
  o->s_y = pair_off(U_SY);
  o->s_r = pair_off(U_SR);
  o->v_x = pair_off(U_VX);
  o->v_y = pair_off(U_VY);
  o->v_r = pair_off(U_VR);
  o->rudder = pair_off(U_RUD);
  o->t = U_T * np;
  o->ep_reward = pair_off(U_EP);
  o->wind_coef = U_COEF * np;
  o->wind0_next = U_W0N * np;
  o->start_y_next = U_SYN * np;
  o->index = U_IDX * np;
  o->cons = U_CONS * np;
  o->fill = U_FILL * np;
  o->mt_pos = U_MTPOS * np;
  o->start_y = U_STARTY * np;
  o->counters = U_CNT * np;
  o->refill_list = U_LIST * np;
  // the drawn knots (raw, before the fit) are kept per slot only when asked for
  // (SACENV_OUT_KNOTS); the refill's fit reads them from the slot's own y fields
  const int64_t uw = U_WIND, wk = kWindUnits * nk, rk = raw_knots ? 1 : 0;
  o->wind_knots = uw * np;
  o->knots_raw = raw_knots ? (uw + 2 * wk) * np : -1;
  o->mt_key = (uw + (2 + rk) * wk) * np;
  o->mt_next = o->mt_key + U_MT_BYTES * np;
  const int64_t ur = uw + (2 + rk) * wk + 2 * U_MT_BYTES;
  o->record = ur * np;
  o->obs = ur * np;
  o->reward = (ur + 44) * np;
  o->done = (ur + 48) * np;
  o->term = (ur + 49) * np;
  o->final_obs = (ur + 50) * np;
  o->final_ep_reward = (ur + 94) * np;
  o->accel = (ur + 102) * np;
  o->reward64 = (ur + 126) * np;
  int64_t off = align256((ur + 134) * np);
  o->refill_mask = off;
  off += align256(8 * nw);
  o->status = off;
  off += 256;
  o->spline_g = off;
  off += align256(8LL * kMaxK * kMaxK);
  o->wind_table = off;
  off += use_table ? align256(16LL * L) : 0;
  o->total_bytes = off;
  o->last_term = U_LTERM * np;
}

// Device view: pointers are recomputed from (base, n_pad, n_knots) at use,
// which keeps the kernels' scalar-register footprint small.
struct Arena {
  char* b;
  int64_t np;
  int nk;
  int rk;  // 1: knots_raw is allocated (SACENV_OUT_KNOTS)
  template <class T>
  __device__ __forceinline__ T* at(int64_t units) const { return reinterpret_cast<T*>(b + units * np); }
  __device__ __forceinline__ double* f64(int u) const { return at<double>(u); }
  __device__ __forceinline__ int32_t* i32(int u) const { return at<int32_t>(u); }
  __device__ __forceinline__ int nwaves() const { return (int)(np / 64); }
  __device__ __forceinline__ int64_t wk() const { return kWindUnits * nk; }
  // episode-contiguous slot storage: [env][slot][curve][knot] (+ [y, m] pairs)
  __device__ __forceinline__ double* wind_knots() const { return at<double>(U_WIND); }
  __device__ __forceinline__ double* knots_raw() const { return at<double>(U_WIND + 2 * wk()); }
  __device__ __forceinline__ uint32_t* mt_key() const { return at<uint32_t>(U_WIND + (2 + rk) * wk()); }
  __device__ __forceinline__ uint32_t* mt_next() const { return mt_key() + kMtN * np; }
  __device__ __forceinline__ int64_t ur() const { return U_WIND + (2 + rk) * wk() + 2 * U_MT_BYTES; }
  __device__ __forceinline__ float* obs() const { return at<float>(ur()); }
  __device__ __forceinline__ float* reward() const { return at<float>(ur() + 44); }
  __device__ __forceinline__ uint8_t* done() const { return at<uint8_t>(ur() + 48); }
  __device__ __forceinline__ uint8_t* term() const { return at<uint8_t>(ur() + 49); }
  __device__ __forceinline__ float* final_obs() const { return at<float>(ur() + 50); }
  __device__ __forceinline__ double* final_ep() const { return at<double>(ur() + 94); }
  __device__ __forceinline__ double* accel() const { return at<double>(ur() + 102); }
  __device__ __forceinline__ double* reward64() const { return at<double>(ur() + 126); }
  __device__ __forceinline__ char* tail() const { return b + align256((ur() + 134) * np); }
  // envs of owner wave w that ended since the last refill
  __device__ __forceinline__ unsigned long long* refill_mask() const {
    return reinterpret_cast<unsigned long long*>(tail());
  }

  // per refill rank: the env's MT position as k_need_masks read it (its episode
  // counter goes to refill_list(2)): the refill tops the ring up from these
  // snapshots, so a step launch that runs concurrently with the refill (and
  // rewrites cons) cannot change what it draws
  __device__ __forceinline__ int32_t* cons_snap() const { return i32(U_CSNAP); }
  // [0] refills done, [1] SACENV_STATUS_* bits, [2] envs ranked by the last refill
  __device__ __forceinline__ int32_t* status() const {
    return reinterpret_cast<int32_t*>(tail() + align256(8 * nwaves()));
  }
  // refill rank -> [0] env, [1] first and [2] end episode number drawn
  __device__ __forceinline__ int32_t* refill_list(int k) const { return i32(U_LIST + 4 * k); }
  // element index of (env, slot, curve, knot) in knots_raw; x2 (+1) in wind_knots
  __device__ __forceinline__ int64_t wix(int slot, int c, int k, int e) const {
    return (((int64_t)e * kSlots + slot) * 2 + c) * nk + k;
  }
  // The slot ring of a wave's 64 envs is one contiguous block: its base is
  // uniform (64-bit, scalar registers) and a lane's (y, m) offset inside it
  // stays 32-bit (< 64 x 33 KB), so the step's gathers keep the SGPR-base
  // addressing mode at any env count.
  __device__ __forceinline__ const char* wk_wave(int e0) const {
    return reinterpret_cast<const char*>(wind_knots()) + (int64_t)e0 * (int64_t)kSlots * 32 * nk;
  }
  __device__ __forceinline__ uint32_t wko_l(int slot, int c, int k, int l) const {
    return ((((uint32_t)l * (uint32_t)kSlots + (uint32_t)slot) * 2u + (uint32_t)c) * (uint32_t)nk + (uint32_t)k) * 16u;
  }
  // (y, m) of knot k and k+1 of env e: 32 contiguous bytes
  __device__ __forceinline__ void piece(int slot, int c, int k, int e, double (&q)[4]) const {
    const char* base = wk_wave(e & ~63) + wko_l(slot, c, k, e & 63);
    const double2 a = *reinterpret_cast<const double2*>(base), b = *reinterpret_cast<const double2*>(base + 16);
    q[0] = a.x, q[1] = a.y, q[2] = b.x, q[3] = b.y;  // memory order: y0, m0, y1, m1
  }
  // the 32 bytes at byte offset off of the wave's ring block (piece_if's load)
  __device__ __forceinline__ void piece_at(const char* wbase, uint32_t off, double (&q)[4]) const {
    const char* base = wbase + off;
    const double2 a = *reinterpret_cast<const double2*>(base), b = *reinterpret_cast<const double2*>(base + 16);
    q[0] = a.x, q[1] = a.y, q[2] = b.x, q[3] = b.y;
  }
  // piece() for lane `lane` of the wave whose ring block starts at wbase, for
  // lanes with `use`; the others read the block's first line (a fixed address:
  // one cache line per wave), so the load needs no branch
  __device__ __forceinline__ void piece_if(bool use, const char* wbase, int slot, int c, int k, int lane,
                                           double (&q)[4]) const {
    const char* base = wbase + (use ? wko_l(slot, c, k, lane) : 0u);
    const double2 a = *reinterpret_cast<const double2*>(base), b = *reinterpret_cast<const double2*>(base + 16);
    q[0] = a.x, q[1] = a.y, q[2] = b.x, q[3] = b.y;
  }
  __device__ __forceinline__ const double* wy0p(const char* wbase, int slot, int c, int lane) const {
    return reinterpret_cast<const double*>(wbase + wko_l(slot, c, 0, lane));
  }
  // Per-lane accesses as uniform base + 32-bit byte offset: the compiler then
  // uses the SGPR-base addressing mode (no 64-bit address arithmetic in VALU).
  // Offsets stay below 2^32 for n_envs <= 2^22 (check_params).
  template <class T>
  __device__ __forceinline__ T& at_e(int64_t unit, uint32_t off) const {
    return *reinterpret_cast<T*>(b + unit * np + off);
  }
  // the per-env fields below U_WIND: the whole byte offset in 32 bits (u < 724
  // and n_pad <= 2^22 by check_params), so each access is one VALU add
  // on the lane offset and an SGPR-base load/store
  template <class T>
  __device__ __forceinline__ T& at_s(int u, uint32_t off) const {
    return *reinterpret_cast<T*>(b + ((uint32_t)u * (uint32_t)np + off));
  }
  __device__ __forceinline__ double& f64e(int u, uint32_t eo) const {
    return u < U_PAIRED ? at_s<double>(u & ~15, 2u * eo + (uint32_t)(u & 8)) : at_s<double>(u, eo);
  }
  // the pair whose block starts at unit u (16-aligned, < U_PAIRED)
  __device__ __forceinline__ double2& f64p(int u, uint32_t eo) const { return at_s<double2>(u, 2u * eo); }
  __device__ __forceinline__ int32_t& i32e(int u, uint32_t eo4) const { return at_s<int32_t>(u, eo4); }
};

__host__ inline Arena make_arena(const SacenvBoatParams& p, void* base) {
  return Arena{static_cast<char*>(base), pad64(p.n_envs), p.n_knots, (p.out_flags & SACENV_OUT_KNOTS) ? 1 : 0};
}

// Launch constants built on the host: the small tables whose offsets depend
// on n_helpers / wind_len, and the reciprocals of the config divisors (IEEE
// 1/x on the host is the same double as on the device; computing them here
// keeps eight uniform fp64 divisions out of every lane).
struct Tail {
  const double* g;
  const double* table;
  double r_mx, r_my, r_iz, r_nd, r_w;  // 1/(m+m_x), 1/(m+m_y), 1/(I+I_z), 1/(n D), 1/width
  double r_goal, r_two_w, r_fuel;      // observation spans: 1/goal, 1/(2 width), 1/fuel
  // the force laws' constant factors, folded once per launch (make_tail): each
  // law is then (velocity^2) x one constant instead of a left-to-right chain of
  // four to six products (boat_env.py:213-281); ~30 fewer f64 multiplies a
  // step, rounding within ~2 ulp of the reference's order (state tolerance 1e-5)
  double k_front, k_thrust, k_side, k_rud_front, k_hull, k_rud_moment;
};

// ---------------------------------------------------------------- LDS of a drawing wave

struct RngLds {           // an episode draw (k_refill: 5.3 KB, more waves per CU)
  uint32_t win[kWave];    // MT window (tempered words pos .. pos+63)
  uint32_t blk[2][kMtN];  // current MT block, next (twisted) block
  double y[2][kMaxK];     // knot values per curve (unfolded)
};
struct DrawLds : RngLds {  // draw + wave fit (init / host resets)
  double m[2][kMaxK];     // second derivatives / 6 per curve (unfolded)
  double g[kMaxK * kMaxK];
#ifdef SACENV_STAMPS
  uint64_t stamp[8];
#endif
};

// diagnostic phase clocks (tools/stamps.py; -DSACENV_STAMPS builds only, never
// loaded by the product path)
#if defined(SACENV_STAMPS)
#define DRAW_STAMP(l, i)                                                   \
  do {                                                                     \
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");            \
    (l).stamp[i] = __builtin_amdgcn_s_memrealtime();                       \
  } while (0)
#else
#define DRAW_STAMP(l, i) \
  do {                   \
  } while (0)
#endif

// ---------------------------------------------------------------- MT19937
#include "mt19937.h"

// ---------------------------------------------------------------- wind curve

struct Knot {
  int j;
  double t;
};

__device__ __forceinline__ Knot knot_coord(const SacenvBoatParams& p, int i) {
  const double s = (double)i * p.knot_step;
  int j = (int)s;
  if (j > p.n_knots - 2) j = p.n_knots - 2;
  return Knot{j, s - (double)j};
}

// Not-a-knot cubic on interval [j, j+1] in second-derivative form.
__device__ __forceinline__ double spline_piece(double y0, double y1, double m0, double m1, double t) {
  const double u = 1.0 - t;
  return u * y0 + t * y1 + (u * u * u - u) * m0 + (t * t * t - t) * m1;
}

__device__ __forceinline__ double curve_env(const SacenvBoatParams& p, const Arena& A, int slot, int c,
                                            int e, int i) {
  const Knot k = knot_coord(p, i);
  double q[4];
  A.piece(slot, c, k.j, e, q);
  return spline_piece(q[0], q[2], q[1], q[3], k.t);
}

__host__ __device__ __forceinline__ int n_curves(int experiment) {
  return experiment == 6 ? 2 : (experiment == 4 || experiment == 5) ? 1 : 0;
}

// Wind.get_wind(index) (wind.py:20-24) for the tables of wind.py:26-99.
__device__ __forceinline__ void wind_at(const SacenvBoatParams& p, const Arena& A, const double* table,
                                        int slot, int e, int idx, double& wv, double& wa) {
  if (idx > p.wind_len - 1) idx = p.wind_len - 1;  // reference: IndexError
  if (idx < 0) idx = 0;
  if (p.use_wind_table) {
    wv = table[idx];
    wa = table[p.wind_len + idx];
    return;
  }
  switch (p.experiment) {
    case 3:
      wv = p.max_velocity;
      wa = p.wind_dir_rad;
      return;
    case 4:
      wv = curve_env(p, A, slot, 0, e, idx);
      wa = p.wind_dir_rad;
      return;
    case 5: {
      wv = p.max_velocity;
      const double r = curve_env(p, A, slot, 0, e, idx) <= 0.5 / 2 ? 0.0 : 1.0;  // wind.py:92-99
      wa = (r * kPi) + kPi / 2;
      return;
    }
    case 6:
      wv = curve_env(p, A, slot, 0, e, idx);
      wa = curve_env(p, A, slot, 1, e, idx);
      return;
    default:  // 1, 2: no wind
      wv = 0.0;
      wa = 0.0;
      return;
  }
}

// The polynomial coefficients below as loop-invariant VGPR copies (trig_k(),
// once per launch). Written as plain fma() with literals, the compiler builds
// each 64-bit coefficient with two v_mov_b32 and a v_fmac; read from SGPRs,
// it rebuilt them with two s_mov_b32 per use inside the step loop (the SGPR
// file is full with the loop's addresses): ~60 SALU issue slots per step.
struct TrigK {
  double s[10];  // sine series: 1/21!, -1/19!, 1/17!, ..., -1/3! (sincos_fast uses the last 8)
  double c[7];   // cosine series: 1/16!, -1/14!, ..., 1/4!
  double e[10];  // exp_v's polynomial (ocml's exp coefficients)
  // exp_v's other constants: log2(e), -ln2 high / low, and its overflow / underflow
  // bounds. As literals the loop rebuilt each one with two s_mov_b32 every step (an
  // SALU op between f64 ops costs ~7 cycles of one wave's issue): as VGPR copies the
  // persistent step measured 1.189 -> 1.157 us (round 6, alternating A/B)
  double ec[5];
};
__device__ __forceinline__ double vconst(double x) {
  double r;
  asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "s"(x));
  return r;
}
template <bool kV = true>  // kV: VGPR copies (the multi-step loop); else plain constants
__device__ __forceinline__ TrigK trig_k() {
  constexpr double sn[10] = {1.9572941063391262e-20,  -8.22063524662432950e-18, 2.8114572543455206e-15,
                             -7.647163731819816e-13,  1.6059043836821613e-10,   -2.505210838544172e-08,
                             2.7557319223985893e-06,  -1.984126984126984e-04,   8.333333333333333e-03,
                             -1.6666666666666666e-01};
  constexpr double cs[7] = {4.779477332387385e-14, -1.1470745597729725e-11, 2.08767569878681e-09,
                            -2.755731922398589e-07, 2.48015873015873e-05,   -1.388888888888889e-03,
                            4.1666666666666664e-02};
  TrigK k;
#pragma unroll
  for (int i = 0; i < 10; ++i) k.s[i] = kV ? vconst(sn[i]) : sn[i];
#pragma unroll
  for (int i = 0; i < 7; ++i) k.c[i] = kV ? vconst(cs[i]) : cs[i];
  constexpr double ex[10] = {2.5022322536502990e-08, 2.7630903490112654e-07, 2.755751454582531e-06,
                             2.480149103909504e-05,  1.9841269589115522e-04, 1.3888888945916382e-03,
                             8.333333333455043e-03,  4.1666666666519754e-02, 1.6666666666666477e-01,
                             5.000000000000012e-01};
#pragma unroll
  for (int i = 0; i < 10; ++i) k.e[i] = kV ? vconst(ex[i]) : ex[i];
  constexpr double ec[5] = {1.4426950408889634, -0.69314718055994529, -2.3190468138462996e-17, 1024.0,
                            -1075.0};
#pragma unroll
  for (int i = 0; i < 5; ++i) k.ec[i] = kV ? vconst(ec[i]) : ec[i];
  return k;
}
__device__ __forceinline__ double fma_v(double a, double b, double c) {
  double r;
  asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// exp(x): ocml's __ocml_exp_f64 restated operation for operation (the same
// double for every x, NaN and the range ends included: within 1 ulp of glibc,
// tools/ubench notes), its polynomial read from VGPRs. Inlined from the
// library, the compiler kept the coefficients in VGPRs but fed them to
// v_fmac, copying each one first: 9 v_mov_b64 a step.
__device__ __forceinline__ double exp_v(double x, const TrigK& K) {
  const double n = rint(x * K.ec[0]);
  double r = fma(K.ec[1], n, x);
  r = fma(K.ec[2], n, r);
  double q = fma_v(K.e[0], r, K.e[1]);
#pragma unroll
  for (int i = 2; i < 10; ++i) q = fma_v(r, q, K.e[i]);
  q = fma(r, q, 1.0);
  q = fma(r, q, 1.0);
  double e = ldexp(q, (int)n);
  e = K.ec[3] < x ? __builtin_inf() : e;
  return K.ec[4] > x ? 0.0 : e;
}

// sin(x) for |x| <= kSinBound with no argument reduction: x + x^3 P(x^2), P
// the Taylor series through x^21 (truncation < 1e-20, below half an ulp),
// about 12 FMAs against ocml's reduction + two polynomials + select.
constexpr double kSinBound = 1.25;
__device__ __forceinline__ double sin_taylor(double x, const TrigK& K) {
  const double z = x * x;
  double q = fma_v(z, K.s[0], K.s[1]);
#pragma unroll
  for (int i = 2; i < 10; ++i) q = fma_v(q, z, K.s[i]);
  return fma(x * z, q, x);  // the negated series of before, bit for bit
}

// sin and cos of x for |x| <= kCwBound: k = rint(x 2/pi), r = x - k pi/2 by fma
// in three Cody-Waite terms (each fma rounds once: r within ~1 ulp), Taylor
// polynomials on |r| <= pi/4 (sin through r^17, cos through r^16: truncation
// below 1e-17) and the quadrant swap. Within 1 ulp of glibc's sin/cos up to
// 1e13 (measured, 2e6 samples per decade); the bound keeps (int)k exact.
constexpr double kCwBound = 1.0e5;
__device__ __forceinline__ void sincos_quadrant(double r, double z, double ps, double pc, double k, double* sp,
                                                double* cp);
__device__ __forceinline__ void sincos_fast(double x, double* sp, double* cp, const TrigK& K) {
  const double k = rint(x * 0.6366197723675814);
  double r = fma(-k, 1.5707963267948966, x);
  r = fma(-k, 6.123233995736766e-17, r);
  r = fma(-k, -1.4973849048591698e-33, r);
  const double z = r * r;
  double ps = fma_v(z, K.s[2], K.s[3]);
#pragma unroll
  for (int i = 4; i < 10; ++i) ps = fma_v(ps, z, K.s[i]);
  double pc = fma_v(z, K.c[0], K.c[1]);
#pragma unroll
  for (int i = 2; i < 7; ++i) pc = fma_v(pc, z, K.c[i]);
  sincos_quadrant(r, z, ps, pc, k, sp, cp);
}

// sincos_fast's tail: the series values from the two polynomials, then the
// quadrant of k = rint(x 2/pi) (swap, and the signs as sign-bit xors)
__device__ __forceinline__ void sincos_quadrant(double r, double z, double ps, double pc, double k, double* sp,
                                                double* cp) {
  const double sr = fma(r * z, ps, r);
  const double cr = 1.0 - fma(-(z * z), pc, 0.5 * z);
  const int q = (int)k;
  const double a = (q & 1) ? cr : sr, b = (q & 1) ? sr : cr;  // sin, cos of r + (q&1) pi/2
  // negate by the quadrant as a sign-bit xor on the high word (the same double as
  // -a, signed zeros and NaNs included): q & 2 for sin, (q + 1) & 2 for cos, moved
  // to bit 31 by one shift each -- 5 VALU fewer than two compares and selects
  const uint64_t ms = (uint64_t)(((uint32_t)q << 30) & 0x80000000u) << 32;
  const uint64_t mc = (uint64_t)((((uint32_t)q + 1u) << 30) & 0x80000000u) << 32;
  *sp = __longlong_as_double((long long)((uint64_t)__double_as_longlong(a) ^ ms));
  *cp = __longlong_as_double((long long)((uint64_t)__double_as_longlong(b) ^ mc));
}

// The fast forms for every lane, then ocml's for the lanes outside their
// range (NaN included) behind one wave-uniform branch that is almost never
// taken: a lane's result depends on its own argument only. Each such branch
// ends a scheduling region, so the step evaluates its early transcendentals
// (wind angle, advance ratio, rudder: all known once the action is in) in
// one region (trig3), where the three chains interleave, and keeps the one
// late one (yaw) on its own.
// (ocml's functions stay inline: called out of line, to keep their tables
// and temporaries out of the step loop's registers, the step measured
// 0.12 us slower -- the call's register save and restore conventions)
struct SinCos {
  double s, c;
};
__device__ __forceinline__ double sin_ocml(double x) { return sin(x); }
__device__ __forceinline__ SinCos sincos_ocml(double x) {
  SinCos r;
  sincos(x, &r.s, &r.c);
  return r;
}

__device__ __forceinline__ void sincos_cw(double x, double* sp, double* cp, const TrigK& K) {
  sincos_fast(x, sp, cp, K);
  const bool ok = fabs(x) <= kCwBound;
  if (__ballot(!ok) != 0ull && !ok) {
    const SinCos r = sincos_ocml(x);
    *sp = r.s, *cp = r.c;
  }
}

__device__ __forceinline__ void trig3(double j, double r, double w, double* sj, double* sr, double* sw,
                                      double* cw, const TrigK& K) {
  // the four Horner chains (sin j, sin r, and the sin and cos polynomials of w's
  // reduced argument) issued interleaved, their ends aligned: each FMA's
  // dependent predecessor is three instructions back, so the chains hide each
  // other's latency (written one after the other, the asm FMAs issued as two
  // serial 10-deep chains with a hazard nop between dependent pairs). The same
  // operations as sin_taylor / sincos_fast, so the same doubles.
  const double kw = rint(w * 0.6366197723675814);
  double rw = fma(-kw, 1.5707963267948966, w);
  rw = fma(-kw, 6.123233995736766e-17, rw);
  rw = fma(-kw, -1.4973849048591698e-33, rw);
  const double zj = j * j, zr = r * r, zw = rw * rw;
  double qj = fma_v(zj, K.s[0], K.s[1]);
  double qr = fma_v(zr, K.s[0], K.s[1]);
  double ps = 0.0, pc = 0.0;
#pragma unroll
  for (int i = 2; i < 10; ++i) {
    qj = fma_v(qj, zj, K.s[i]);
    qr = fma_v(qr, zr, K.s[i]);
    if (i == 3) ps = fma_v(zw, K.s[2], K.s[3]);
    if (i >= 4) ps = fma_v(ps, zw, K.s[i]);
    if (i == 4) pc = fma_v(zw, K.c[0], K.c[1]);
    if (i >= 5) pc = fma_v(pc, zw, K.c[i - 3]);
  }
  *sj = fma(j * zj, qj, j);
  *sr = fma(r * zr, qr, r);
  sincos_quadrant(rw, zw, ps, pc, kw, sw, cw);
  const bool okj = fabs(j) <= kSinBound, okr = fabs(r) <= kSinBound, okw = fabs(w) <= kCwBound;
  if (__ballot(!(okj && okr && okw)) != 0ull) {
    if (!okj) *sj = sin_ocml(j);
    if (!okr) *sr = sin_ocml(r);
    if (!okw) {
      const SinCos q = sincos_ocml(w);
      *sw = q.s, *cw = q.c;
    }
  }
}

// x / c for a per-launch constant c, from r = RN(1/c): Markstein's correction
// step returns the correctly rounded quotient, i.e. the same double as IEEE
// division, in 3 dependent FLOPs instead of the ~10 of a full fp64 divide.
__device__ __forceinline__ double div_c(double x, double c, double r) {
  const double q = x * r;
  const double err = fma(-q, c, x);
  return fma(err, r, q);
}

// ---------------------------------------------------------------- observation
// Boat.return_state / normalize (boat_env.py:308-326): (v - lo) / (hi - lo).
// Config-dependent spans divide exactly (div_c); the reference's literal
// spans are applied as reciprocals (the float32 observation is the output).
struct Obs {
  float v[SACENV_OBS_DIM];
};

struct ObsConst {  // per-launch reciprocals of the config-dependent spans
  double goal, two_w, fuel;
  // the literal spans' reciprocals (k[7]: the rudder offset pi/3), as VGPR
  // copies in the step loop (obs_const_v): as literals each use cost two s_mov
  double k[8];
};

__device__ __forceinline__ ObsConst obs_const(const Tail& T) {
  return ObsConst{T.r_goal, T.r_two_w, T.r_fuel,
                  {1.0 / 5.0, 1.0 / 0.025, 1.0 / 0.37, 1.0 / (2 * kPi), 1.0 / 8.5e-3, 1.0 / 1.4e-5,
                   1.0 / (kPi / 3 - (-kPi / 3)), kPi / 3}};
}
__device__ __forceinline__ ObsConst obs_const_v(const Tail& T) {
  ObsConst o = obs_const(T);
#pragma unroll
  for (int i = 0; i < 8; ++i) o.k[i] = vconst(o.k[i]);
  return o;
}

__device__ __forceinline__ Obs make_obs(const SacenvBoatParams& p, const ObsConst& oc, double s_x,
                                        double v_x, double a_x, double s_y, double v_y, double a_y,
                                        double s_r, double v_r, double a_r, double rudder,
                                        double fuel) {
  Obs o;
  o.v[0] = (float)div_c(s_x, p.goal_line, oc.goal);
  o.v[1] = (float)(v_x * oc.k[0]);
  o.v[2] = (float)(a_x * oc.k[1]);
  o.v[3] = (float)div_c(s_y + p.track_width, p.track_width + p.track_width, oc.two_w);
  o.v[4] = (float)(v_y * (1.0 / 2.0));
  o.v[5] = (float)(a_y * oc.k[2]);
  o.v[6] = (float)(s_r * oc.k[3]);
  o.v[7] = (float)(v_r * oc.k[4]);
  o.v[8] = (float)(a_r * oc.k[5]);
  o.v[9] = (float)((rudder + oc.k[7]) * oc.k[6]);
  o.v[10] = (float)div_c(fuel, (double)p.fuel0, oc.fuel);
  return o;
}

typedef float f4v __attribute__((ext_vector_type(4)));

// Cache policy of the step's output stores: write-through (sc1: the line
// leaves the XCD L2 as it issues, so the launch ends with no dirty lines to
// write back at its boundary; measured 0.21 us/step faster than plain stores,
// DESIGN.md §4). Scalars as agent-scope relaxed atomic stores; the 16-B pairs
// and obs rows (no 16-B sc1 atomic form) as write-through buffer stores (aux
// bit 4).
// kWT false: a plain (write-back) store, for the open-loop multi-step launch,
// whose record rows are rewritten every step in place: they stay in the XCD's
// L2 and are written back once, at the launch's end (measured: a write-through
// record made every step wait for the previous step's stores to reach memory,
// as the step's loads count behind them in vmcnt)
template <bool kWT = true, class T>
__device__ __forceinline__ void st_out(T& ref, T v) {
  if (kWT)
    __hip_atomic_store(&ref, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else
    ref = v;
}

// a 16-B pair of the paired state (block unit u), write-through
typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void st_pair(char* base, int u, uint32_t np, uint32_t eo, double a, double b) {
  const uint32_t off = (uint32_t)u * np + 2u * eo;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(base, 0, 0x7fffffff, 0x00020000);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, make_double2(a, b)), r, off, 0, 16);
}

__device__ __forceinline__ void store_obs(float* dst, const Obs& o) {
#pragma unroll
  for (int k = 0; k < SACENV_OBS_DIM; ++k) dst[k] = o.v[k];
}

// ---------------------------------------------------------------- cross-lane helpers

// DPP lane permutes (gfx9 dpp_ctrl): register-to-register, no LDS round trip.
template <int kCtrl>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), kCtrl, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), kCtrl, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double row16_min(double v) {
  v = fmin(v, dpp_f64<0xB1>(v));      // quad_perm [1,0,3,2]
  v = fmin(v, dpp_f64<0x4E>(v));      // quad_perm [2,3,0,1]
  v = fmin(v, dpp_f64<0x141>(v));     // row_half_mirror
  return fmin(v, dpp_f64<0x140>(v));  // row_mirror
}
__device__ __forceinline__ double row16_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  return fmax(v, dpp_f64<0x140>(v));
}
__device__ __forceinline__ double readlane_f64(double v, int src) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), src),
                          __builtin_amdgcn_readlane(__double2loint(v), src));
}
// Wave-wide inclusive prefix sum: row shifts, then row_bcast15/31 carry rows.
__device__ __forceinline__ int wave_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xF, 0xF, true);   // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xF, 0xF, true);   // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xF, 0xF, true);   // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xF, 0xF, true);   // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xA, 0xF, false);  // row_bcast:15
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xC, 0xF, false);  // row_bcast:31
  return x;
}

// ---------------------------------------------------------------- spline extrema

// Grid-sample min/max of one spline interval: the cubic is monotone between
// its critical points, so the extreme grid samples of interval j are its
// first/last grid points and the neighbours of each critical point
// (tests/test_host_cpu.py::test_grid_extrema_rule_is_exact). The ten
// candidates are split over S lanes (lane s evaluates candidates s, s+S, ...);
// critical points need only grid-point accuracy, so approximate rcp/rsq do.
// Interval j's piece is (y0, y1, a, b) = (y[j], y[j+1], m[j], m[j+1]): every
// candidate lies in [lo, hi], whose grid samples all fall in interval j.
// The grid indices [lo, hi] of interval j (a launch constant per interval: the
// fit kernel forms it once per lane, not per fit).
struct IvGrid {
  double jd, lod, hid;
  bool valid;
};
__device__ __forceinline__ IvGrid interval_grid(const SacenvBoatParams& p, int j) {
  const int L = p.wind_len;
  // (inv = RN(1/knot_step) puts ceil(j inv) within one of the first grid index of
  // interval j: start one below and step up, and symmetrically for the last)
  int lo = (int)ceil((double)j * p.knot_inv) - 1;
  if (lo < 0) lo = 0;
  while (lo < L && knot_coord(p, lo).j < j) ++lo;
  int hi = (int)floor((double)(j + 1) * p.knot_inv) + 1;
  if (hi > L - 1) hi = L - 1;
  while (hi >= 0 && knot_coord(p, hi).j > j) --hi;
  return IvGrid{(double)j, (double)lo, (double)hi, lo <= hi};
}

template <int S>
__device__ __forceinline__ void interval_extrema_on(const SacenvBoatParams& p, const IvGrid& gr, int s,
                                                    double y0, double y1, double a, double b, double& mn,
                                                    double& mx) {
  mn = INFINITY;
  mx = -INFINITY;
  if (!gr.valid) return;
  const double inv = p.knot_inv;
  const double qa = 3.0 * (b - a), qb = 6.0 * a, qc = y1 - y0 - 2.0 * a - b;
  // the piece in the power basis, f(t) = y0 + c1 t + c2 t^2 + c3 t^3 (spline_piece
  // expanded: c1 = y1 - y0 - 2 m0 - m1, c2 = 3 m0, c3 = m1 - m0): 3 FMAs per
  // candidate instead of spline_piece's 11 operations. The extreme grid samples
  // agree with spline_piece's evaluation of them to a few ulp (the renormalisation
  // bar is the reference's interp1d samples, 1e-12: test_wind_tables_vs_reference)
  const double c1 = qc, c2 = 3.0 * a, c3 = b - a;
  double r0 = -1.0, r1 = -1.0;  // roots of the derivative in [0,1]; -1 = none
  const double scale = fabs(qa) + fabs(qb) + fabs(qc);
  if (fabs(qa) <= 1e-14 * scale) {
    if (qb != 0.0) r0 = -qc * __builtin_amdgcn_rcp(qb);
  } else {
    const double disc = qb * qb - 4.0 * qa * qc;
    if (disc >= 0.0) {
      const double sq = disc > 0.0 ? disc * __builtin_amdgcn_rsq(disc) : 0.0;
      const double q = -0.5 * (qb + copysign(sq, qb));
      r0 = q * __builtin_amdgcn_rcp(qa);
      if (q != 0.0) r1 = qc * __builtin_amdgcn_rcp(q);
    }
  }
  const bool ok0 = r0 > -0.01 && r0 < 1.01, ok1 = r1 > -0.01 && r1 < 1.01;
  // the candidates as doubles (exact small integers): every one lies in [lo, hi],
  // i.e. in interval j, so its knot coordinate is t = i * knot_step - j, the same
  // double knot_coord forms -- no integer conversions per candidate (v_cvt costs
  // 8 cycles at one wave per SIMD, tools/ubench/valu_mix.hip)
  const double jd = gr.jd, lod = gr.lod, hid = gr.hid;
  const double i0 = ok0 ? floor((jd + r0) * inv) : lod;
  const double i1 = ok1 ? floor((jd + r1) * inv) : lod;
#pragma unroll
  for (int t = 0; t < (10 + S - 1) / S; ++t) {
    const int q = s + S * t;  // candidate number 0..9
    double i;
    if (q == 0) {
      i = lod;
    } else if (q == 1) {
      i = hid;
    } else {
      const bool first = q < 6;
      const double d = (double)((first ? q - 2 : q - 6) - 1);
      const bool ok = first ? ok0 : ok1;
      i = fmin(fmax((first ? i0 : i1) + d, lod), hid);
      i = ok ? i : lod;
    }
    if (q < 10) {
      const double t = i * p.knot_step - jd;
      const double v = fma(fma(fma(c3, t, c2), t, c1), t, y0);
      mn = fmin(mn, v);
      mx = fmax(mx, v);
    }
  }
}
template <int S>
__device__ __forceinline__ void interval_extrema(const SacenvBoatParams& p, int j, int s, double y0,
                                                 double y1, double a, double b, double& mn,
                                                 double& mx) {
  interval_extrema_on<S>(p, interval_grid(p, j), s, y0, y1, a, b, mn, mx);
}

// ---------------------------------------------------------------- spline constants

__device__ __forceinline__ void load_g(const SacenvBoatParams& p, const double* g, DrawLds& l, int lane) {
  for (int i = lane; i < p.n_knots * p.n_knots; i += kWave) l.g[i] = g[i];
  __syncthreads();
}

// ---------------------------------------------------------------- episode draw

// The RNG half of Boat(config) for env `e`, by all 64 lanes (e uniform):
// np.random.randint(-hw, hw) (boat_env.py:147-150), then n knot values per
// random curve (wind.py:78; velocity first in exp 6) into l.y. Explicit
// draws (replays) bypass the RNG. Returns start_y in all lanes.
__device__ int32_t draw_knots_wave(const SacenvBoatParams& p, const Arena& A, RngLds& l, int e,
                                   int lane, const int32_t* ex_start_y, const double* ex_knots,
                                   int pos0 = -1, bool have_w0 = false, uint32_t w0_pre = 0u) {
  const int nk = p.n_knots;
  // draws follow the reference even when a recorded wind table overrides the
  // curves; only the spline fit is skipped then
  const int ndraw = n_curves(p.experiment);
  const int ncurves = p.use_wind_table ? 0 : ndraw;
  if (ex_start_y != nullptr) {
    for (int c = 0; c < ncurves; ++c)
      if (lane < nk) l.y[c][lane] = ex_knots[c * nk + lane];
    return *ex_start_y;
  }
  MtStream st;
  st.gkey = A.mt_key() + (int64_t)e * kMtN;
  st.pos = pos0 >= 0 ? pos0 : A.i32(U_MTPOS)[e] & kMtPosMask;  // pos0: prefetched by the caller
  // (a pos0 past 624 lies in the block after mt_key: mt_fetch twists mt_key to it;
  // mt_finish stores the index plain, withdrawing mt_next)
  st.cur = 0;
  st.loaded = false;
  st.nxt_valid = false;
  st.advanced = false;
  // masked rejection on 32-bit words (numpy random_bounded_uint64_fill ->
  // buffered_bounded_masked_uint32)
  const uint32_t rng = (uint32_t)(2 * p.start_y_half - 1);
  uint32_t mask = rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  uint32_t val = 0;
  const int need = 2 * nk * ndraw;  // words of the knot values after the randint
  // the first window, or the caller's copy of it (raw words pos0 .. pos0+63 of the
  // stored block, loaded ahead when the window does not cross the block end)
  const uint32_t w0 = have_w0 ? mt_temper(w0_pre) : mt_fetch(st, l, lane);
  const unsigned long long acc0 = __ballot(((w0 & mask) <= rng) && lane < kWave - need);
  if (acc0) {
    // fast path: one 64-word window holds the randint draw and every knot
    const int k = __ffsll((long long)acc0) - 1;
    val = (uint32_t)__builtin_amdgcn_readlane((int)w0, k) & mask;
    if (ndraw > 0) {  // window through LDS: per-lane gathers without bpermute
      l.win[lane] = w0;
      __syncthreads();
    }
    for (int c = 0; c < ndraw; ++c) {
      const int src = k + 1 + c * 2 * nk + ((2 * lane) & 31);
      const uint32_t wa = l.win[src & (kWave - 1)];
      const uint32_t wb = l.win[(src + 1) & (kWave - 1)];
      if (lane < nk) {  // np.random.sample: legacy_double = genrand_res53 on two words
        const double a = (double)(wa >> 5), b = (double)(wb >> 6);
        l.y[c][lane] = (a * 67108864.0 + b) / 9007199254740992.0;
      }
    }
    st.pos += k + 1 + need;
  } else {
    // general path: rejection runs past the window, or the knots do
    for (;;) {
      const uint32_t w = mt_fetch(st, l, lane);
      const unsigned long long acc = __ballot((w & mask) <= rng);
      if (acc) {
        const int k = __ffsll((long long)acc) - 1;
        val = (uint32_t)__builtin_amdgcn_readlane((int)w, k) & mask;
        st.pos += k + 1;
        break;
      }
      st.pos += kWave;
    }
    for (int c = 0; c < ndraw; ++c) {
      const uint32_t w = mt_fetch(st, l, lane);
      l.win[lane] = w;
      __syncthreads();
      const uint32_t wa = l.win[(2 * lane) & (kWave - 1)];
      const uint32_t wb = l.win[(2 * lane + 1) & (kWave - 1)];
      if (lane < nk) {
        const double a = (double)(wa >> 5), b = (double)(wb >> 6);
        l.y[c][lane] = (a * 67108864.0 + b) / 9007199254740992.0;
      }
      __syncthreads();
      st.pos += 2 * nk;
    }
  }
  mt_finish(st, l, A.i32(U_MTPOS) + e, lane);
  return -p.start_y_half + (int32_t)val;
}

// wind.py:87-89 min-max renormalisation of one knot's (value, 2nd derivative)
// when the grid samples leave [0, 1], then the table scaling of wind.py:86-89
// (velocity * max_v, angle * pi * 2; exp 5 keeps the unit curve for the
// rectifier, wind.py:92-99)
__device__ __forceinline__ void fold_knot(const SacenvBoatParams& p, int c, double mn, double mx, double& yv,
                                          double& mv) {
  if (mn < 0.0 || mx > 1.0) {
    const double span = mx - mn;
    yv = (yv - mn) / span;
    mv = mv / span;
  }
  if (p.experiment == 4 || (p.experiment == 6 && c == 0)) {
    yv = yv * p.max_velocity;
    mv = mv * p.max_velocity;
  } else if (p.experiment == 6 && c == 1) {
    yv = yv * kPi * 2;
    mv = mv * kPi * 2;
  }
}

// The spline half: from the knot values in l.y (lanes 16c + j hold knot j of
// curve c), second derivatives m = G @ y, exact grid min/max, the min-max
// renormalisation (wind.py:87-89) and the table scaling (wind.py:86-99);
// stores the folded coefficients of `slot`. l.g must be loaded.
__device__ void fit_store_wave(const SacenvBoatParams& p, const Arena& A, DrawLds& l, int e, int slot,
                               int lane) {
  const int nk = p.n_knots;
  const int ncurves = p.use_wind_table ? 0 : n_curves(p.experiment);
  if (ncurves == 0) return;
  __syncthreads();
  const int c = lane >> 4, j = lane & 15;
  const bool knot_lane = c < ncurves && j < nk;
  double yv = 0.0, mv = 0.0;
  if (knot_lane) {
    yv = l.y[c][j];
#pragma unroll
    for (int k = 0; k < kMaxK; ++k)
      if (k < nk) mv += l.g[j * nk + k] * l.y[c][k];
    l.m[c][j] = mv;
  }
  __syncthreads();
  // lanes 32c + u work on curve c: S lanes per interval (4 if <= 8 intervals)
  double mn = INFINITY, mx = -INFINITY;
  {
    const int cc = lane >> 5, u = lane & 31;
    if (nk - 1 <= 8) {
      const int jj = u >> 2;
      if (cc < ncurves && jj < nk - 1)
        interval_extrema<4>(p, jj, u & 3, l.y[cc][jj], l.y[cc][jj + 1], l.m[cc][jj], l.m[cc][jj + 1], mn, mx);
    } else {
      if (cc < ncurves && u < nk - 1)
        interval_extrema<1>(p, u, 0, l.y[cc][u], l.y[cc][u + 1], l.m[cc][u], l.m[cc][u + 1], mn, mx);
    }
  }
  mn = row16_min(mn);
  mx = row16_max(mx);
  // curve c's extremes are the two rows of its half-wave: uniform values
  const double cmn0 = fmin(readlane_f64(mn, 0), readlane_f64(mn, 16));
  const double cmx0 = fmax(readlane_f64(mx, 0), readlane_f64(mx, 16));
  const double cmn1 = fmin(readlane_f64(mn, 32), readlane_f64(mn, 48));
  const double cmx1 = fmax(readlane_f64(mx, 32), readlane_f64(mx, 48));
  mn = c == 0 ? cmn0 : cmn1;
  mx = c == 0 ? cmx0 : cmx1;
  if (knot_lane) {
    fold_knot(p, c, mn, mx, yv, mv);
    *reinterpret_cast<double2*>(A.wind_knots() + 2 * A.wix(slot, c, j, e)) = double2{yv, mv};
  }
  __syncthreads();
}

// start y and (raw, or SACENV_OUT_KNOTS) the raw knot values of a drawn episode
__device__ __forceinline__ void store_draw(const SacenvBoatParams& p, const Arena& A, const RngLds& l,
                                           int e, int slot, int32_t start_y, int lane, bool raw = false) {
  const int nk = p.n_knots;
  const int ncurves = p.use_wind_table ? 0 : n_curves(p.experiment);
  if (lane == 0) A.i32(U_STARTY)[(int64_t)slot * A.np + e] = start_y;
  const int c = lane >> 4, j = lane & 15;
  if (c < ncurves && j < nk) {
    if (raw) A.wind_knots()[2 * A.wix(slot, c, j, e)] = l.y[c][j];  // the fit's input, in the slot's y
    if (A.rk) A.knots_raw()[A.wix(slot, c, j, e)] = l.y[c][j];
  }
}

// Boat(config) in one go (init / host-driven resets): draw + fit into slot.
__device__ int32_t draw_episode_wave(const SacenvBoatParams& p, const Arena& A, DrawLds& l, int e,
                                     int slot, int lane, const int32_t* ex_start_y,
                                     const double* ex_knots) {
  const int32_t start_y = draw_knots_wave(p, A, l, e, lane, ex_start_y, ex_knots);
  __syncthreads();
  store_draw(p, A, l, e, slot, start_y, lane);
  fit_store_wave(p, A, l, e, slot, lane);
  return start_y;
}

// scalar state of a fresh Boat (boat_env.py:152-198) and its observation;
// the wind piece copy of the episode in `slot` starts at its first interval
__device__ __forceinline__ Obs fresh_state(const SacenvBoatParams& p, const Arena& A, const Tail& T, int e,
                                           int32_t start_y, int slot) {
  const double s_y = p.experiment == 2 ? (double)start_y : 0.0;  // :166-169
  const int nc = p.use_wind_table ? 0 : n_curves(p.experiment);
  const uint32_t eo = (uint32_t)e * 8u;
  for (int c = 0; c < nc; ++c) {
    double q[4];
    A.piece(slot, c, 0, e, q);
    for (int k = 0; k < 4; ++k) A.f64e(U_COEF + 32 * c + 8 * k, eo) = q[k];
  }
  A.f64e(U_SX, eo) = 0.0;
  A.f64e(U_SY, eo) = s_y;
  A.f64e(U_SR, eo) = 0.0;
  A.f64e(U_VX, eo) = 0.0;
  A.f64e(U_VY, eo) = 0.0;
  A.f64e(U_VR, eo) = 0.0;
  A.f64e(U_RUD, eo) = 0.0;
  A.f64e(U_T, eo) = 0.0;
  A.f64e(U_EP, eo) = 0.0;  // :122
  A.i32(U_IDX)[e] = 0;
  if (p.out_flags & SACENV_OUT_ACCEL) {  // a fresh Boat's a_x, a_y, a_r are 0 (:182-196)
    A.at_e<double>(A.ur() + 102, eo) = 0.0;
    A.at_e<double>(A.ur() + 110, eo) = 0.0;
    A.at_e<double>(A.ur() + 118, eo) = 0.0;
  }
  return make_obs(p, obs_const(T), 0.0, 0.0, 0.0, s_y, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, (double)p.fuel0);
}

// ---------------------------------------------------------------- kernels

__global__ void k_spline_g(SacenvBoatParams p, double* __restrict__ g) {
  // (m/6) = G @ y for the not-a-knot cubic on uniform knots (knot coordinate):
  // rows 1..n-2: m[j-1] + 4 m[j] + m[j+1] = 6 (y[j-1] - 2 y[j] + y[j+1]);
  // rows 0, n-1: m[0] - 2 m[1] + m[2] = 0, m[n-3] - 2 m[n-2] + m[n-1] = 0.
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  const int n = p.n_knots;
  double a[kMaxK][kMaxK], r[kMaxK][kMaxK];
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) a[i][j] = r[i][j] = 0.0;
  a[0][0] = 1.0, a[0][1] = -2.0, a[0][2] = 1.0;
  a[n - 1][n - 3] = 1.0, a[n - 1][n - 2] = -2.0, a[n - 1][n - 1] = 1.0;
  for (int j = 1; j < n - 1; ++j) {
    a[j][j - 1] = 1.0, a[j][j] = 4.0, a[j][j + 1] = 1.0;
    r[j][j - 1] = 1.0, r[j][j] = -2.0, r[j][j + 1] = 1.0;  // (6 * rhs) / 6
  }
  for (int c = 0; c < n; ++c) {  // Gauss-Jordan, partial pivoting
    int piv = c;
    for (int i = c + 1; i < n; ++i)
      if (fabs(a[i][c]) > fabs(a[piv][c])) piv = i;
    for (int j = 0; j < n; ++j) {
      double t = a[c][j]; a[c][j] = a[piv][j]; a[piv][j] = t;
      t = r[c][j]; r[c][j] = r[piv][j]; r[piv][j] = t;
    }
    const double d = a[c][c];
    for (int j = 0; j < n; ++j) a[c][j] /= d, r[c][j] /= d;
    for (int i = 0; i < n; ++i) {
      if (i == c) continue;
      const double f = a[i][c];
      if (f == 0.0) continue;
      for (int j = 0; j < n; ++j) a[i][j] -= f * a[c][j], r[i][j] -= f * r[c][j];
    }
  }
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) g[i * n + j] = r[i][j];
}

constexpr int kMaskThreads = 1024;
constexpr uint32_t kSpinLimit = 1u << 22;  // ~seconds of polling: then a launch gives up

__global__ void __launch_bounds__(kWave) k_seed(SacenvBoatParams p, Arena A, const uint32_t* __restrict__ seeds) {
  const int e = blockIdx.x * kWave + threadIdx.x;
  // k_need_masks' look-back words (refill_mask): no stale epoch may match (the
  // caller's arena need not be zeroed; k_need_masks' workgroups <= owner waves <= envs)
  if (e < A.nwaves()) A.refill_mask()[e] = 0ull;
  if (e >= p.n_envs) return;
  // mt19937_seed (init_genrand), numpy RandomState._legacy_seeding(int)
  uint32_t x = seeds[e];
  uint32_t* key = A.mt_key() + (int64_t)e * kMtN;
  for (int i = 0; i < kMtN; ++i) {
    key[i] = x;
    x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
  }
  A.i32(U_MTPOS)[e] = kMtN;  // (plain: mt_next not twisted yet)
  A.i32(U_CONS)[e] = 0;
  A.i32(U_FILL)[e] = 0;
}

// mode 0: first Boat (init). autoreset: slots 0..SLOTS-1 <- episodes 0..SLOTS-1.
// mode 1: reset listed envs. non-autoreset: slot 0 <- a new draw;
//         autoreset: start the next pre-drawn slot, then refill the freed one.
// mode 2: explicit draws (non-autoreset), slot 0.
// One Boat per listed env. ids == NULL: env = block index. dev_count != NULL:
// the list length is read on the device (ids[0 .. *dev_count), grid-stride),
// so a reset of the envs sacenv_compact_done found needs no host round trip.
__global__ void __launch_bounds__(kWave) k_draw(SacenvBoatParams p, Arena A, Tail T, int mode,
                                                const int32_t* __restrict__ ids,
                                                const int32_t* __restrict__ ex_start_y,
                                                const double* __restrict__ ex_knots,
                                                const int32_t* __restrict__ dev_count) {
  __shared__ DrawLds lds;
  const int lane = threadIdx.x;
  const int nq = dev_count != nullptr ? *dev_count : (int)gridDim.x;
  if ((int)blockIdx.x >= nq) return;
  load_g(p, T.g, lds, lane);
  for (int q = blockIdx.x; q < nq; q += gridDim.x) {
    const int e = ids != nullptr ? ids[q] : q;
    if (e < 0 || e >= p.n_envs) continue;  // uniform per block
    int32_t start_y;
    int slot = 0;
    if (mode == 2) {
      start_y = draw_episode_wave(p, A, lds, e, 0, lane, ex_start_y + q,
                                  ex_knots != nullptr ? ex_knots + (int64_t)q * 2 * p.n_knots : nullptr);
    } else if (!p.autoreset) {
      start_y = draw_episode_wave(p, A, lds, e, 0, lane, nullptr, nullptr);
    } else if (mode == 0) {
      // the first episode here; sacenv_boat_init's refill draws the next SLOTS-1 in
      // the env's order (all envs in parallel, the fits spread over lane groups:
      // seconds faster at 65 536 envs than SLOTS serial draw-and-fits per wave)
      start_y = draw_episode_wave(p, A, lds, e, 0, lane, nullptr, nullptr);
      if (lane == 0) {
        A.i32(U_CONS)[e] = 0;
        A.i32(U_FILL)[e] = 1;
      }
    } else {
      // start the next pre-drawn episode and draw one more behind the last
      // (per-env draw order: the refill continues from fill)
      const int c = A.i32(U_CONS)[e] + 1;
      const int f = A.i32(U_FILL)[e];
      if (c >= f && lane == 0) atomicOr(&A.status()[1], SACENV_STATUS_SLOT_UNDERFLOW);
      slot = c % kSlots;
      start_y = A.i32(U_STARTY)[(int64_t)slot * A.np + e];
      if (lane == 0) A.i32(U_CONS)[e] = c;
      draw_episode_wave(p, A, lds, e, f % kSlots, lane, nullptr, nullptr);
      if (lane == 0) A.i32(U_FILL)[e] = f + 1;
    }
    if (lane == 0) {
      const Obs o = fresh_state(p, A, T, e, start_y, slot);
      store_obs(A.obs() + (int64_t)e * SACENV_OBS_DIM, o);
    }
    __syncthreads();
  }
}

// Done-mask compaction (the reset list of BoatEnv.reset for the envs that
// ended): ids of the nonzero bytes of done[0..n), ascending,
// and their count. One workgroup of 1024 lanes, 64 bytes per lane per pass:
// per-lane counts -> DPP wave scan -> LDS scan of the 16 wave totals.
__global__ void __launch_bounds__(1024) k_compact(const uint8_t* __restrict__ done, int n, int aligned,
                                                  int32_t* __restrict__ ids, int32_t* __restrict__ count) {
  __shared__ int wsum[16];
  __shared__ int base_s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) base_s = 0;
  __syncthreads();
  for (int64_t c0 = 0; c0 < n; c0 += 1024 * 64) {
    const int64_t e0 = c0 + (int64_t)t * 64;
    uint64_t bits = 0;  // bit j: done[e0 + j] != 0
    if (aligned && e0 + 64 <= n) {
      const uint4* v = reinterpret_cast<const uint4*>(done + e0);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint4 x = v[k];
        const uint32_t wds[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
        for (int d = 0; d < 4; ++d)
#pragma unroll
          for (int by = 0; by < 4; ++by)
            if ((wds[d] >> (8 * by)) & 0xffu) bits |= 1ull << (16 * k + 4 * d + by);
      }
    } else {
      for (int j = 0; j < 64 && e0 + j < n; ++j)
        if (done[e0 + j]) bits |= 1ull << j;
    }
    const int cnt = __popcll(bits);
    const int incl = wave_incl_scan(cnt);
    if (lane == 63) wsum[w] = incl;
    __syncthreads();
    int wbase = 0;
    for (int k = 0; k < w; ++k) wbase += wsum[k];
    int pos = base_s + wbase + incl - cnt;
    while (bits) {
      const int j = __ffsll((long long)bits) - 1;
      bits &= bits - 1ull;
      ids[pos++] = (int32_t)(e0 + j);
    }
    __syncthreads();
    if (t == 1023) base_s += wbase + incl;
    __syncthreads();
  }
  if (t == 0) *count = base_s;
}

// Non-serialising phase clocks of the refill (tools/refill_stamps.py; -DSACENV_STAMPS
// builds only): a stamp is taken once the value(s) it names are in registers
// (the empty asm consumes them), no other wait is added.
#ifdef SACENV_STAMPS
#define REFILL_STAMP(slot, ...)                                     \
  do {                                                              \
    asm volatile("" ::__VA_ARGS__);                                 \
    (slot) = __builtin_amdgcn_s_memrealtime();                      \
  } while (0)
constexpr int kRefillStamps = 24;  // per refill wave: start, total read, fast path done, 19 wave draws, end, draws
#else
#define REFILL_STAMP(slot, ...) \
  do {                          \
  } while (0)
#endif

// sacenv_boat_refill, launch 1: every listed env gets its slot ring topped up
// to SLOTS episodes (fill = cons + SLOTS), drawn in the env's order (start y
// and raw knots). A wave takes four consecutive ranks, one 16-lane group each.
// Fast path, one episode per group: the group loads the 16 + 2*nk*curves words
// at the env's MT position (when they lie inside the current 624-word block),
// tempers them, takes the first accepted randint word among the first 16
// (masked rejection, numpy legacy) and turns the following word pairs into the
// knots (genrand_res53), lane = (curve, knot): one wave instruction serves four
// envs, where the wave-per-env draw spent ~330 wave instructions on each (the
// refill was VALU-bound). A window that crosses the block end reads on in
// mt_next when the last fit launch twisted it ahead (kMtNextOk). The rest --
// a crossing without mt_next (a second one since the last refill), a randint
// rejected 16 times, more than 8 knots -- goes through the wave-per-env draw
// (draw_knots_wave), env by env. Block 0 counts the refill.
constexpr int kGroupLanes = 16;
constexpr int kGroups = kWave / kGroupLanes;
__global__ void __launch_bounds__(kWave) k_refill(SacenvBoatParams p, Arena A) {
  __shared__ RngLds lds;
  const int lane = threadIdx.x;
#ifdef SACENV_STAMPS
  uint64_t stm[kRefillStamps] = {};
  int n_st = 0;
#endif
  REFILL_STAMP(stm[0], "s"(lane));
  const int total = __builtin_amdgcn_readfirstlane(A.status()[2]);  // listed by k_need_masks
  REFILL_STAMP(stm[1], "s"(total));
  if (blockIdx.x == 0 && lane == 0) A.status()[0] += 1;
  const int G = (int)gridDim.x;
  const int g = lane / kGroupLanes, gl = lane % kGroupLanes;
  const int nk = p.n_knots;
  const int ndraw = n_curves(p.experiment);  // draws follow the reference even with a wind table
  const int ncurves = p.use_wind_table ? 0 : ndraw;
  const int need = 2 * nk * ndraw;           // knot words after the randint word
  const int nwords = kGroupLanes + need;     // <= 48 on the fast path
  const bool grp_ok = nk <= 8;               // 16 lanes = 2 curves x 8 knots
  const uint32_t rng = (uint32_t)(2 * p.start_y_half - 1);
  uint32_t mask = rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  // rank r's env, fill, cons snapshot and MT position (k_need_masks), loaded
  // with the count and not behind it: list rows below n_pad are always memory
  const int np_ = (int)A.np;
  int r0 = blockIdx.x * kGroups;
  int rq = r0 + g < np_ ? r0 + g : 0;
  int e_n = A.refill_list(0)[rq], f_n = A.refill_list(1)[rq], c_n = A.refill_list(2)[rq], p_n = A.cons_snap()[rq];
  for (; r0 < total; r0 += kGroups * G) {
    const int rr = r0 + g;
    const bool ok = rr < total;
    const int e = ok ? e_n : 0;
    const int c = ok ? c_n : 0;
    const int f0 = ok ? f_n : 0;
    const int pos = ok ? (p_n & kMtPosMask) : kMtN;
    const bool nx = ok && (p_n & kMtNextOk) != 0;  // mt_next holds the next block
    if (r0 + kGroups * G < total) {  // the next iteration's rank, in flight with this one
      rq = rr + kGroups * G < np_ ? rr + kGroups * G : 0;
      e_n = A.refill_list(0)[rq], f_n = A.refill_list(1)[rq], c_n = A.refill_list(2)[rq], p_n = A.cons_snap()[rq];
    }
    if (ok && c >= f0 && gl == 0) atomicOr(&A.status()[1], SACENV_STATUS_SLOT_UNDERFLOW);
    const int f_end = ok && f0 < c + kSlots ? c + kSlots : f0;
    // The group's episodes f0, f0+1, ... on the fast path, one per pass, while
    // each next window lies inside the current MT block (round 4: an env that
    // consumed several episodes drew only its first here, the rest wave by wave
    // at ~4 us each -- about half of a refill's draws)
    int f_next = f0, pos_next = pos;  // the next episode to draw and its MT position
    bool live = ok && f0 < f_end && grp_ok;
    uint32_t* const gw = lds.blk[0] + g * 3 * kGroupLanes;
#pragma unroll 1
    while (__ballot(live) != 0ull) {  // uniform: until every group left the fast path
      // (with the next block pre-twisted, a window may cross the block end)
      bool fast = live && pos_next + nwords <= (nx ? 2 * kMtN : kMtN);
      // the group's words pos_next .. pos_next + nwords - 1 (raw, key order), tempered;
      // index 624 on from mt_next
      const int64_t eo = (int64_t)e * kMtN;
      uint32_t w[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int i = pos_next + gl + kGroupLanes * q;
        const uint32_t* src = i < kMtN ? A.mt_key() + eo + i : A.mt_next() + eo + (i - kMtN);
        w[q] = fast && gl + kGroupLanes * q < nwords ? mt_temper(*src) : 0u;
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the last pass's reads of gw are done
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int q = 0; q < 3; ++q) gw[gl + kGroupLanes * q] = w[q];
      // np.random.randint (boat_env.py:147-150): the first accepted of the first 16 words
      const unsigned long long acc = __ballot(fast && (w[0] & mask) <= rng);
      const uint32_t gacc = (uint32_t)(acc >> (kGroupLanes * g)) & 0xFFFFu;
      fast = fast && gacc != 0u;
      const int k = fast ? __builtin_ctz(gacc) : 0;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // the group's words, then reads
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      REFILL_STAMP(stm[2], "v"(k));
      if (fast) {
        const int slot = f_next % kSlots;
        const int cc = gl / 8, jj = gl % 8;  // knot jj of curve cc (wind.py:78; velocity first)
        if (cc < ncurves && jj < nk) {
          const int src = k + 1 + cc * 2 * nk + 2 * jj;  // np.random.sample: res53 of two words
          const double a = (double)(gw[src] >> 5), bb = (double)(gw[src + 1] >> 6);
          const double kv = (a * 67108864.0 + bb) / 9007199254740992.0;
          A.wind_knots()[2 * A.wix(slot, cc, jj, e)] = kv;  // k_refill_fit's input, in the slot's y
          if (A.rk) A.knots_raw()[A.wix(slot, cc, jj, e)] = kv;
        }
        if (gl == 0) {
          A.i32(U_STARTY)[(int64_t)slot * A.np + e] = -p.start_y_half + (int32_t)(gw[k] & mask);
          A.i32(U_MTPOS)[e] = (pos_next + k + 1 + need) | (nx ? kMtNextOk : 0);
        }
        f_next = f_next + 1;
        pos_next = pos_next + k + 1 + need;
      }
      live = fast && f_next < f_end;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");  // LDS free for the wave draws
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // the rest, env by env, by the whole wave
#pragma unroll 1
    for (int j = 0; j < kGroups; ++j) {
      const int src = j * kGroupLanes;
      if (__builtin_amdgcn_readlane((int)ok, src) == 0) break;  // uniform; later groups too
      const int ej = __builtin_amdgcn_readlane(e, src);
      const int fe = __builtin_amdgcn_readlane(f_end, src);
      int f = __builtin_amdgcn_readlane(f_next, src);
      const int pj = __builtin_amdgcn_readlane(pos_next, src);
      bool first = true;
      for (; f < fe; ++f) {
        const int32_t start_y = draw_knots_wave(p, A, lds, ej, lane, nullptr, nullptr, first ? pj : -1);
#ifdef SACENV_STAMPS
        const int sb = 3 + (n_st < 18 ? n_st : 18);  // the end of each wave draw (first 19)
        ++n_st;
#endif
        REFILL_STAMP(stm[sb], "v"(start_y));
        first = false;
        __syncthreads();
        store_draw(p, A, lds, ej, f % kSlots, start_y, lane, true);
        __syncthreads();
      }
      if (lane == 0) {
        A.i32(U_FILL)[ej] = fe;
        A.refill_list(1)[r0 + j] = __builtin_amdgcn_readlane(f0, src);
        A.refill_list(2)[r0 + j] = fe;
      }
    }
  }
#ifdef SACENV_STAMPS
  stm[22] = __builtin_amdgcn_s_memrealtime();
  stm[23] = (uint64_t)n_st;
  if (lane == 0 && (int64_t)(blockIdx.x + 1) * kRefillStamps * 8 <= 24 * A.np) {
    uint64_t* d = reinterpret_cast<uint64_t*>(A.accel()) + (int64_t)blockIdx.x * kRefillStamps;
    for (int i = 0; i < kRefillStamps; ++i) d[i] = stm[i];
  }
#endif
}

// sacenv_boat_refill, launch 2: the spline fits of the episodes launch 1
// drew. A group of GS lanes (8, or 16 for more than 8 knots) fits one
// (env, curve): lane j forms m[j] = (G @ y)[j] and the grid extrema of
// interval j, the group reduces min/max by shuffles, and lane j folds and
// stores knot j (the operations of fit_store_wave in the same order:
// bit-identical coefficients). Grid-stride over the groups.
//
// Per lane, what depends only on j (a lane constant: the group's lanes are the
// knots) is formed once per launch: G's row jj in registers (zero past nk) and
// interval j's grid range. kFull (nk == GS) drops every per-knot bound check.
// The group's shuffles are DPP moves inside a 16-lane row (no LDS round trip).
template <int GS>
__device__ __forceinline__ double group_min(double v) {
  v = fmin(v, dpp_f64<0xB1>(v));  // quad_perm [1,0,3,2]
  v = fmin(v, dpp_f64<0x4E>(v));  // quad_perm [2,3,0,1]
  v = fmin(v, dpp_f64<0x141>(v));  // row_half_mirror: the other quad of the 8
  if (GS == 16) v = fmin(v, dpp_f64<0x140>(v));  // row_mirror: the other 8 of the row
  return v;
}
template <int GS>
__device__ __forceinline__ double group_max(double v) {
  v = fmax(v, dpp_f64<0xB1>(v));
  v = fmax(v, dpp_f64<0x4E>(v));
  v = fmax(v, dpp_f64<0x141>(v));
  if (GS == 16) v = fmax(v, dpp_f64<0x140>(v));
  return v;
}
// lane i + 1's value (row_shl:1; the row's last lane keeps its own, unused)
__device__ __forceinline__ double next_lane_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(__double2loint(v), __double2loint(v), 0x101, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(__double2hiint(v), __double2hiint(v), 0x101, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

template <int GS, bool kFull>
__device__ __forceinline__ void fit_group(const SacenvBoatParams& p, const Arena& A, const double (&gr)[GS],
                                          const IvGrid& ig, int item, int j, int jj, int j1, int nc) {
  const int nk = kFull ? GS : p.n_knots;
  const int rr = item / nc, c = item - rr * nc;
  const int e = A.refill_list(0)[rr], f0 = A.refill_list(1)[rr], f1 = A.refill_list(2)[rr];
  for (int f = f0; f < f1; ++f) {  // uniform across the group
    const int slot = f % kSlots;
    // the curve's nk drawn knots, in the slot's y fields (k_refill put them there);
    // every lane of the group reads them all before any lane writes the fitted pairs
    const double* kr = A.wind_knots() + 2 * A.wix(slot, c, 0, e);
    double yk[GS];
#pragma unroll
    for (int k = 0; k < GS; ++k) yk[k] = kr[2 * (kFull || k < nk ? k : nk - 1)];
    double yv = kr[2 * jj];
    const double y1 = kr[2 * j1];
    // m = G @ y in the reference's order (terms past nk: none when kFull; else a
    // select, so no +0.0 term can turn a -0.0 sum into +0.0)
    double mv = 0.0;
#pragma unroll
    for (int k = 0; k < GS; ++k) {
      const double s = mv + gr[k] * yk[k];
      mv = kFull || k < nk ? s : mv;
    }
    const double m1 = next_lane_f64(mv);
    double mn, mx;
    interval_extrema_on<1>(p, ig, 0, yv, y1, mv, m1, mn, mx);  // (ig invalid: +-inf)
    mn = group_min<GS>(mn);
    mx = group_max<GS>(mx);
    if (kFull || j < nk) {
      fold_knot(p, c, mn, mx, yv, mv);
      *reinterpret_cast<double2*>(A.wind_knots() + 2 * A.wix(slot, c, j, e)) = double2{yv, mv};
    }
  }
}

constexpr int kAheadEnvs = 8;  // envs per twist-ahead workgroup of the fit launch (mt_ahead)
// mt19937_gen of one block by one wave, from memory and in registers: word i
// needs old[i], old[i+1] and old[i+397] (i < 227) or new[i-227], so lane l
// forms the chains c, c+227, c+454 for c = l, l+64, l+128, l+192 (< 227) and
// every dependency but word 623's (new[0], new[396]: two readlanes) stays in
// the lane -- no LDS, no barriers. All loads complete before the first store,
// so o may be n (the block made current is twisted in place); with `cur`, the
// old block is also copied there.
__device__ __forceinline__ void mt_twist_regs(const uint32_t* o, uint32_t* n, uint32_t* cur, int lane) {
  constexpr int kD = kMtN - kMtM;  // 227
  uint32_t a0[4], a1[4], a2[4], b0[4], b1[4], c0[4], c1[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = lane + kWave * k;
    const bool ok = c < kD, okc = c < kMtN - 1 - 2 * kD;  // (c + 454 < 623)
    a0[k] = ok ? o[c] : 0u;
    a1[k] = ok ? o[c + 1] : 0u;
    a2[k] = ok ? o[c + kMtM] : 0u;
    b0[k] = ok ? o[c + kD] : 0u;
    b1[k] = ok ? o[c + kD + 1] : 0u;
    c0[k] = okc ? o[c + 2 * kD] : 0u;
    c1[k] = okc ? o[c + 2 * kD + 1] : 0u;
  }
  const uint32_t last = o[kMtN - 1];
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  uint32_t nb2 = 0u, na0 = 0u;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int c = lane + kWave * k;
    if (c < kD) {
      const uint32_t na = mt_mix(a0[k], a1[k], a2[k]);
      const uint32_t nb = mt_mix(b0[k], b1[k], na);
      n[c] = na;
      n[c + kD] = nb;
      if (cur) cur[c] = a0[k], cur[c + kD] = b0[k];
      if (c < kMtN - 1 - 2 * kD) {
        n[c + 2 * kD] = mt_mix(c0[k], c1[k], nb);
        if (cur) cur[c + 2 * kD] = c0[k];
      }
      if (k == 0) na0 = na;
      if (k == 2) nb2 = nb;
    }
  }
  // word 623: mix(old[623], new[0], new[396]); new[396] = chain 169 = lane 41, k = 2
  const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)na0, 0);
  const uint32_t n396 = (uint32_t)__builtin_amdgcn_readlane((int)nb2, kMtM - 1 - kD - 2 * kWave);
  if (lane == 0) {
    n[kMtN - 1] = mt_mix(last, n0, n396);
    if (cur) cur[kMtN - 1] = last;
  }
}

// The fit launch's first np/kAheadEnvs workgroups twist each env's next MT
// block ahead (mt_next, flagged kMtNextOk in U_MTPOS), so k_refill's 16-lane
// groups draw windows that cross a block end from memory instead of leaving
// the fast path for a wave-per-env draw with its twist (one in ~13 episodes).
// An env whose draws ran into mt_next (index past 624) first gets it as its
// current block. Needed by the envs that crossed or went through a wave draw
// since the last refill (all of them after seeding); the rest are skipped.
__device__ __forceinline__ void mt_ahead(const SacenvBoatParams& p, const Arena& A, int b, int lane) {
  const int e0 = b * kAheadEnvs;
  int v = 0;
  bool need = false;
  // (past 8 knots every draw is a wave draw, which withdraws mt_next: nothing to gain)
  if (lane < kAheadEnvs && e0 + lane < p.n_envs && p.n_knots <= 8) {
    v = A.i32(U_MTPOS)[e0 + lane];
    need = (v & kMtNextOk) == 0 || (v & kMtPosMask) > kMtN;
  }
  unsigned long long m = __ballot(need);
#pragma unroll 1
  while (m != 0ull) {  // uniform
    const int j = __ffsll((long long)m) - 1;
    m &= m - 1ull;
    const int e = e0 + j;
    const int vj = __builtin_amdgcn_readlane(v, j);
    const bool adv = (vj & kMtNextOk) != 0 && (vj & kMtPosMask) > kMtN;
    uint32_t* const key = A.mt_key() + (int64_t)e * kMtN;
    uint32_t* const nxt = A.mt_next() + (int64_t)e * kMtN;
    mt_twist_regs(adv ? nxt : key, nxt, adv ? key : nullptr, lane);
    if (lane == 0) A.i32(U_MTPOS)[e] = ((vj & kMtPosMask) - (adv ? kMtN : 0)) | kMtNextOk;
  }
}

// GS lanes per (env, curve): 8 for up to 8 knots, else 16; one instantiation
// per width, so the 8-knot launch carries no 16-knot registers
template <int GS, bool kFull>
__global__ void __launch_bounds__(kWave) k_refill_fit(SacenvBoatParams p, Arena A, Tail T) {
  const int lane = threadIdx.x;
  const int ahead = (int)(A.np / kAheadEnvs);
  if ((int)blockIdx.x < ahead) {
    mt_ahead(p, A, (int)blockIdx.x, lane);
    return;
  }
  const int fb = (int)blockIdx.x - ahead, fgrid = (int)gridDim.x - ahead;
  const int nc = p.use_wind_table ? 0 : n_curves(p.experiment);
  const int nk = kFull ? GS : p.n_knots;
  const int items = A.status()[2] * nc;  // (env, curve) groups
#ifdef SACENV_STAMPS
  const uint64_t st0 = __builtin_amdgcn_s_memrealtime();
  uint64_t* const fst = reinterpret_cast<uint64_t*>(A.reward64()) + 2 * (int64_t)blockIdx.x;
  const bool fst_ok = lane == 0 && (int64_t)(blockIdx.x + 1) * 16 <= 8 * A.np;
  if (fst_ok) fst[0] = st0, fst[1] = 0;
#endif
  if (items == 0 || fb * (kWave / GS) >= items) return;  // uniform
  const int j = lane & (GS - 1);
  const int jj = j < nk ? j : nk - 1, j1 = jj + 1 < nk ? jj + 1 : jj;
  double gr[GS];
#pragma unroll
  for (int k = 0; k < GS; ++k) gr[k] = kFull || k < nk ? T.g[jj * nk + k] : 0.0;
  IvGrid ig = interval_grid(p, j < nk - 1 ? j : 0);
  ig.valid = ig.valid && j < nk - 1;
  const int per = kWave / GS;
  for (int base = fb * per; base < items; base += fgrid * per) {
    const int item = base + lane / GS;
    if (item >= items) break;
    fit_group<GS, kFull>(p, A, gr, ig, item, j, jj, j1, nc);
  }
#ifdef SACENV_STAMPS
  __syncthreads();
  if (fst_ok) fst[1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// sacenv_boat_refill, launch 0: which envs consumed pre-drawn episodes since
// their ring was last topped up (fill < cons + SLOTS), listed for launch 1 in
// env order. Derived from the episode counters, so the step launch keeps no
// flags of its own (measured: owner-side flag words cost 0.25-0.4 us/step).
// 16 owner waves' envs per workgroup (one wave each). A workgroup counts its
// flagged envs (ballots, a scan of the 16 popcounts), publishes the count as
// its look-back word (refill_mask[b] = (epoch, count); epoch = refills done + 1,
// so no word of an earlier refill matches and nothing is reset), sums the words
// of workgroups 0..b-1 -- one vector load of up to 64 words per pass, polled
// until every one carries this epoch -- and stores each flagged env's id at its
// rank in refill_list(0), one coalesced store per wave; the last workgroup
// stores the total in status[2]. k_refill then finds its envs with one load
// each. The ranks are those of a serial scan over the envs (the lists, and so
// the arenas, are the same at every run). Round 2's design had the last
// workgroup to take a ticket rank all 1 024 masks: 14.7 us a refill.
__device__ __forceinline__ unsigned long long lookback_load(const unsigned long long* w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__global__ void __launch_bounds__(kMaskThreads) k_need_masks(SacenvBoatParams p, Arena A) {
  __shared__ int wcnt[kMaskThreads / kWave];
  const int t = threadIdx.x, lane = t & (kWave - 1), wv = t >> 6;
  const int nw = A.nwaves(), b = (int)blockIdx.x;
  const int w = b * (kMaskThreads / kWave) + wv, e = w * kWave + lane;
  const uint32_t epoch = (uint32_t)A.status()[0] + 1u;
  bool need = false;
  int c = 0, fl = 0, mp = 0;
  if (w < nw && e < p.n_envs) {
    c = A.i32(U_CONS)[e];
    fl = A.i32(U_FILL)[e];
    mp = A.i32(U_MTPOS)[e];
    need = fl < c + kSlots;
  }
  const unsigned long long m = __ballot(need);
  if (lane == 0) wcnt[wv] = __popcll(m);
  __syncthreads();
  if (t < kWave) {  // wave 0: the workgroup's count, its look-back, each wave's base
    unsigned long long* const look = A.refill_mask();
    const int cnt = t < kMaskThreads / kWave ? wcnt[t] : 0;
    const int incl = wave_incl_scan(cnt);
    const int total = __builtin_amdgcn_readlane(incl, kMaskThreads / kWave - 1);
    if (t == 0)
      __hip_atomic_store(look + b, ((unsigned long long)epoch << 32) | (uint32_t)total, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    int before = 0;
    for (int q0 = 0; q0 < b; q0 += kWave) {
      const int q = q0 + t;
      unsigned long long x = q < b ? lookback_load(look + q) : ((unsigned long long)epoch << 32);
      for (uint32_t it = 0; __ballot((uint32_t)(x >> 32) != epoch) != 0ull; ++it) {
        if (it >= kSpinLimit) {  // a predecessor that never publishes: flag it, rank as if it listed none
          if (t == 0) atomicOr(&A.status()[1], SACENV_STATUS_LIST_TIMEOUT);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
        if ((uint32_t)(x >> 32) != epoch) x = lookback_load(look + q);
      }
      int v = (uint32_t)(x >> 32) == epoch ? (int)(uint32_t)x : 0;
      v += __shfl_xor(v, 32);
      v += __shfl_xor(v, 16);
      v += __shfl_xor(v, 8);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 1);
      before += v;
    }
    if (t < kMaskThreads / kWave) wcnt[t] = before + incl - cnt;
    if (t == 0 && b == (int)gridDim.x - 1) A.status()[2] = before + total;
  }
  __syncthreads();
  if (need) {  // rank r: the env and its counters as of now, one load each for k_refill
    const int r = wcnt[wv] + __popcll(m & ((1ull << lane) - 1ull));
    A.refill_list(0)[r] = e;
    A.refill_list(1)[r] = fl;
    A.refill_list(2)[r] = c;  // the cons snapshot (k_refill then stores the end episode here)
    A.cons_snap()[r] = mp;
  }
}

// Uniform fp64 constants as VGPR copies: the step reads ~40 config doubles,
// more than the SGPR file holds next to the addresses, and SGPR spills
// (v_writelane/v_readlane pairs) cost more than VGPR operands; the owner
// wave has VGPRs to spare (LDS, not registers, bounds occupancy).
__device__ __forceinline__ double vreg(double x) {
  double r;
  asm volatile("v_mov_b64 %0, %1" : "=v"(r) : "s"(x));
  return r;
}
__device__ __forceinline__ SacenvBoatParams vreg_params(SacenvBoatParams q) {
  // (the force laws' factors are Tail's folded constants: not copied)
  q.dt = vreg(q.dt), q.t_max = vreg(q.t_max), q.goal_line = vreg(q.goal_line);
  q.oob_limit = vreg(q.oob_limit), q.track_width = vreg(q.track_width);
  q.m_plus_mx = vreg(q.m_plus_mx), q.m_plus_my = vreg(q.m_plus_my), q.i_plus_iz = vreg(q.i_plus_iz);
  q.one_minus_wf = vreg(q.one_minus_wf);
  q.n_times_d = vreg(q.n_times_d);
  q.reward_k = vreg(q.reward_k), q.reward_center = vreg(q.reward_center);
  q.knot_step = vreg(q.knot_step);
  return q;
}
__device__ __forceinline__ Tail vreg_tail(Tail t) {
  t.r_mx = vreg(t.r_mx), t.r_my = vreg(t.r_my), t.r_iz = vreg(t.r_iz), t.r_nd = vreg(t.r_nd);
  t.r_w = vreg(t.r_w), t.r_goal = vreg(t.r_goal), t.r_two_w = vreg(t.r_two_w), t.r_fuel = vreg(t.r_fuel);
  t.k_front = vreg(t.k_front), t.k_thrust = vreg(t.k_thrust), t.k_side = vreg(t.k_side);
  t.k_rud_front = vreg(t.k_rud_front), t.k_hull = vreg(t.k_hull), t.k_rud_moment = vreg(t.k_rud_moment);
  return t;
}

// ---------------------------------------------------------------- toy envs
// environment/toy_parachute.py:7-41 and environment/toy_car.py:5-33, one
// env per lane, as vectorised envs: one step = one iteration of the
// script's loop, obs = the signals the script records. The integrators
// (control_blocks.py:5-36) keep their STORED output (clamped to the limits,
// :27-32) but return the unclamped value (:36); the first call returns the
// initial value (:21-22).

constexpr int UT_CNT = 40, UT_CTR = 44, UT_OBS = 56, UT_REW = 64, UT_DONE = 68, UT_TERM = 69,
              UT_FOBS = 70, UT_TOTAL = 78;  // per-env bytes after the 5 f64 state fields

__host__ __device__ inline void toy_layout(int n, SacenvToyLayout* o) {
  const int64_t np = pad64(n);
  o->n_pad = np;
  o->state = 0;
  o->count = UT_CNT * np;
  o->counters = UT_CTR * np;
  o->record = UT_OBS * np;
  o->obs = UT_OBS * np;
  o->reward = UT_REW * np;
  o->done = UT_DONE * np;
  o->term = UT_TERM * np;
  o->final_obs = UT_FOBS * np;
  o->total_bytes = align256(UT_TOTAL * np);
}

struct ToyArena {
  char* b;
  int64_t np;
  __device__ __forceinline__ double* f(int k) const { return reinterpret_cast<double*>(b + 8LL * k * np); }
  __device__ __forceinline__ int32_t* count() const { return reinterpret_cast<int32_t*>(b + UT_CNT * np); }
  __device__ __forceinline__ uint32_t* ctr(int k) const {
    return reinterpret_cast<uint32_t*>(b + UT_CTR * np) + (int64_t)k * np;
  }
  __device__ __forceinline__ float* obs() const { return reinterpret_cast<float*>(b + UT_OBS * np); }
  __device__ __forceinline__ float* reward() const { return reinterpret_cast<float*>(b + UT_REW * np); }
  __device__ __forceinline__ uint8_t* done() const { return reinterpret_cast<uint8_t*>(b + UT_DONE * np); }
  __device__ __forceinline__ uint8_t* term() const { return reinterpret_cast<uint8_t*>(b + UT_TERM * np); }
  __device__ __forceinline__ float* final_obs() const { return reinterpret_cast<float*>(b + UT_FOBS * np); }
};

// the scripts' variables before the loop, and the signals they stand for
__device__ __forceinline__ void toy_initial(const SacenvToyParams& p, double f[5], float obs[2]) {
  for (int k = 0; k < 5; ++k) f[k] = 0.0;
  if (p.kind == SACENV_TOY_PARACHUTE) {
    f[1] = p.h0;  // v_integrator = Integrator(initial_value=h_0) (:21)
    obs[0] = (float)p.h0;
    obs[1] = 0.0f;
  } else {
    obs[0] = 0.0f;
    obs[1] = 0.0f;
  }
}

// one loop iteration; returns the termination code (0: the loop goes on)
__device__ __forceinline__ uint8_t toy_advance(const SacenvToyParams& p, double f[5], int& count,
                                               float obs[2]) {
  const bool first = count == 0;
  uint8_t term = SACENV_TERM_NONE;
  ++count;
  if (p.kind == SACENV_TOY_PARACHUTE) {
    // f = (a_integrator stored output = v, v_integrator stored output = s, total_a, t)
    double total_a = f[2] - p.g;                               // :24
    const double v = first ? 0.0 : total_a * p.integ_dt + f[0];  // :25
    const double s = first ? p.h0 : v * p.integ_dt + f[1];       // :26
    f[0] = v;
    f[1] = s;
    obs[0] = (float)s;
    obs[1] = (float)v;
    if (s < 0.0) {  // :29-30 ground reached: the script breaks
      term = SACENV_TOY_TERM_GROUND;
    } else {
      const double area = s < p.h1 ? p.area_open : p.area_closed;  // :33-36
      const double F_w = v * v * 0.5 * p.rho * p.c_w * area;
      total_a = F_w / p.mass;  // :38
      f[3] = f[3] + p.dt;      // :40
      if (!(f[3] <= p.t_max)) term = SACENV_TERM_TIMEOUT;  // :23
    }
    f[2] = total_a;
  } else {
    // f = (car_angle, a_integrator stored output, v_x / v_y integrator stored outputs, t)
    const double angle = f[0] + p.car_dangle;                          // :24
    const double v = first ? 0.0 : p.car_accel * p.integ_dt + f[1];   // :25
    const double vx = v * cos(angle), vy = v * sin(angle);            // :27-28
    const double sx = first ? 0.0 : vx * p.integ_dt + f[2];           // :30
    const double sy = first ? 0.0 : vy * p.integ_dt + f[3];           // :31
    f[0] = angle;
    f[1] = v >= p.car_v_max ? p.car_v_max : v;  // stored clamp (upper_limit=10, :12)
    f[2] = sx;
    f[3] = sy;
    f[4] = f[4] + p.dt;  // :33
    obs[0] = (float)sx;
    obs[1] = (float)sy;
    if (!(f[4] <= p.t_max)) term = SACENV_TERM_TIMEOUT;  // :22
  }
  return term;
}

// one toy wave: 64 envs, one per lane
__device__ __forceinline__ void toy_wave(const SacenvToyParams& p, const ToyArena& T, int ob, int lane) {
  const int e = ob * kWave + lane;
  if (e >= p.n_envs) return;
  double f[5];
  for (int k = 0; k < 5; ++k) f[k] = T.f(k)[e];
  int count = T.count()[e];
  float obs[2];
  uint8_t term = toy_advance(p, f, count, obs);
  if (term == SACENV_TERM_NONE && p.max_episode_steps > 0 && count >= p.max_episode_steps)
    term = SACENV_TERM_TRUNCATED;
  if (term != SACENV_TERM_NONE) {
    const int c = term == SACENV_TOY_TERM_GROUND ? 0 : term == SACENV_TERM_TIMEOUT ? 1 : 2;
    T.ctr(c)[e] += 1u;
    if (p.autoreset) {
      T.final_obs()[2 * e] = obs[0];
      T.final_obs()[2 * e + 1] = obs[1];
      toy_initial(p, f, obs);
      count = 0;
    }
  }
  for (int k = 0; k < 5; ++k) T.f(k)[e] = f[k];
  T.count()[e] = count;
  reinterpret_cast<float2*>(T.obs())[e] = make_float2(obs[0], obs[1]);
  T.reward()[e] = 0.0f;
  T.done()[e] = term != SACENV_TERM_NONE ? 1 : 0;
  T.term()[e] = term;
}

// n_steps iterations of one toy wave in a persistent launch (sacenv_mixed_segment):
// the state and the iteration count in registers, each step's record (obs,
// reward, done, term) and a restarting lane's terminal obs stored as
// toy_wave stores them, the counters added once at the end. Results equal
// n_steps toy_wave launches bit for bit (the same toy_advance arithmetic).
__device__ __forceinline__ void toy_roll_wave(const SacenvToyParams& p, const ToyArena& T, int ob, int lane,
                                              int n_steps) {
  const int e = ob * kWave + lane;
  if (e >= p.n_envs) return;
  double f[5];
  for (int k = 0; k < 5; ++k) f[k] = T.f(k)[e];
  int count = T.count()[e];
  uint32_t ends[3] = {0u, 0u, 0u};
  for (int ks = 0; ks < n_steps; ++ks) {
    float obs[2];
    uint8_t term = toy_advance(p, f, count, obs);
    if (term == SACENV_TERM_NONE && p.max_episode_steps > 0 && count >= p.max_episode_steps)
      term = SACENV_TERM_TRUNCATED;
    if (term != SACENV_TERM_NONE) {
      ++ends[term == SACENV_TOY_TERM_GROUND ? 0 : term == SACENV_TERM_TIMEOUT ? 1 : 2];
      if (p.autoreset) {
        reinterpret_cast<float2*>(T.final_obs())[e] = make_float2(obs[0], obs[1]);
        toy_initial(p, f, obs);
        count = 0;
      }
    }
    reinterpret_cast<float2*>(T.obs())[e] = make_float2(obs[0], obs[1]);
    T.reward()[e] = 0.0f;
    T.done()[e] = term != SACENV_TERM_NONE ? 1 : 0;
    T.term()[e] = term;
  }
  for (int k = 0; k < 5; ++k) T.f(k)[e] = f[k];
  T.count()[e] = count;
  for (int c = 0; c < 3; ++c)
    if (ends[c] != 0u) T.ctr(c)[e] += ends[c];
}

// toy arenas stepped inside a mixed launch
struct MixedToys {
  SacenvToyParams p[2];
  ToyArena a[2];
  int nb[2];
  int n;
};

// ---------------------------------------------------------------- owner wave

// The owner wave's SoA state is loaded 16 B per lane and redistributed through
// LDS: lanes 0-31 read 512 contiguous bytes of one field, lanes 32-63 of the
// next (6 load instructions instead of 13). Outputs are stored per lane as
// soon as they are final (EARLY_STORE); the obs rows go out through LDS as
// float4 (64 rows x 44 B = 176 float4).
constexpr int kCoef = 8;  // wind_coef fields: 2 curves x (y0, y1, m0, m1)
constexpr int kMkWords = SACENV_REFILL_PERIOD / 32;  // 32-bit mark words per env (one bit per step)
struct OwnerLds {
  float obs[kWave * SACENV_OBS_DIM];  // the wave's obs rows, stored as float4
  // staged replay rows: bit (ks % 32) of mk[ks / 32][lane] marks lane's row of step ks
  // (word-major: the 64 lanes of one read hit 64 consecutive words, no bank conflict)
  uint32_t mk[kMkWords][kWave];
};

// t += dt (boat_env.py:69) accumulates exactly when dt = m * 2^e with m < 2^22:
// every partial sum k*dt (k <= 2^31) is then a double, so t == index * dt
// bit for bit and t need not be carried in HBM (8 B read + 8 B write per
// env-step for the default dt = 0.25).
__host__ __device__ inline bool t_from_index(double dt) {
  uint64_t bits;
  memcpy(&bits, &dt, sizeof bits);
  return (bits & ((1ull << 30) - 1ull)) == 0ull;
}

// Each dynamics field is stored as soon as it is final, so the write traffic
// drains while the wave still computes (measured: -0.15 us/step against
// staging every output for 16-B stores at the end).
#define EARLY_STORE(u, v)                      \
  do {                                         \
    if (!kRoll) st_out(A.f64e(u, eo), (v));    \
  } while (0)
#define EARLY_STORE2(u, v0, v1)                                     \
  do {                                                              \
    if (!kRoll) st_pair(A.b, (u), (uint32_t)A.np, eo, (v0), (v1));  \
  } while (0)

// (store_row with non-temporal stores: rows written once and not read back by the launch)
template <int ROW>
__device__ __forceinline__ void store_row_nt(float* row, const float* w) {
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
#pragma unroll
  for (int i = 0; i + 4 <= ROW; i += 4)
    __builtin_nontemporal_store(f4u{w[i], w[i + 1], w[i + 2], w[i + 3]}, reinterpret_cast<f4u*>(row + i));
  constexpr int t = ROW & ~3;
  static_assert(ROW - t == 3, "an obs row: 11 floats");
  __builtin_nontemporal_store(f3u{w[t], w[t + 1], w[t + 2]}, reinterpret_cast<f3u*>(row + t));
}

// one env's row of ROW floats (4-B aligned) from registers: dwordx4 stores,
// then the 1..3-float tail as one store
template <int ROW>
__device__ __forceinline__ void store_row(float* row, const float* w) {
  typedef float f4u __attribute__((ext_vector_type(4), aligned(4)));
  typedef float f3u __attribute__((ext_vector_type(3), aligned(4)));
  typedef float f2u __attribute__((ext_vector_type(2), aligned(4)));
#pragma unroll
  for (int i = 0; i + 4 <= ROW; i += 4) *reinterpret_cast<f4u*>(row + i) = f4u{w[i], w[i + 1], w[i + 2], w[i + 3]};
  constexpr int t = ROW & ~3;
  if (ROW - t == 3) *reinterpret_cast<f3u*>(row + t) = f3u{w[t], w[t + 1], w[t + 2]};
  if (ROW - t == 2) *reinterpret_cast<f2u*>(row + t) = f2u{w[t], w[t + 1]};
  if (ROW - t == 1) row[t] = w[t];
}

// 64 obs rows (2816 B) from LDS to a 16-B aligned row block: 3 float4 stores
template <int ROW = SACENV_OBS_DIM, bool kWT = true>  // floats per env row (11: obs; 9: the pooled row's s')
__device__ __forceinline__ void store_obs_block(const float* lds_rows, float* dst_rows, int lane) {
  const f4v* src = reinterpret_cast<const f4v*>(lds_rows);
  // write-through 16-B buffer stores (sc1, aux bit 4): 0.13 us/step faster than
  // nontemporal ones, which leave the rows dirty in L2 for the boundary
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(dst_rows, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int i = 0; i < (ROW * 16 + kWave - 1) / kWave; ++i) {
    const uint32_t q = (uint32_t)lane + kWave * i;
    if (q < kWave * ROW / 4)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, src[q]), r, q * 16u, 0, kWT ? 16 : 0);
  }
}

// Where a multi-step launch (kRoll: sacenv_boat_rollout, sacenv_boat_segment)
// puts step ks's outputs, and how it receives step ks's action.
struct RollArgs {
  char* rec;              // the 50-B/env record of step ks at rec + ks * rec_stride
  int64_t rec_stride;     // bytes; 0: every step into the same record (the arena's)
  float* fin;             // terminal obs of restarting envs at fin + ks * fin_stride (or null)
  int64_t fin_stride;     // floats
  char* trans;            // pooled transition row of step ks at trans + ks * trans_stride (or null)
  int64_t trans_stride;   // bytes
  // staged replay rows (kRows == 2): env e's 64-B row of step ks at stage + (e * K + ks) * 64
  // (K = n_steps: env-major, an env's rows of consecutive steps adjacent), written where bit
  // (ks % 64) of marks[e * ceil(K / 64) + ks / 64] is set (marks == null: every row)
  char* stage;
  unsigned long long* marks;  // (consumed: the launch clears the words it read)
  int64_t act_stride;     // floats between consecutive action rows
  // Action hand-off (sacenv_boat_segment): owner wave w steps ks only once
  // ready[w] >= seq0 + ks + 1, and publishes done[w] = seq0 + ks + 1 once step
  // ks's outputs are visible device-wide. ready == null: every row is ready.
  const uint32_t* ready;
  uint32_t* done;
  uint32_t seq0;
  int32_t* status;        // SACENV_STATUS_HANDOFF_TIMEOUT on a hand-off that never came
};

// A hand-off flag, read device-coherently (sc0 sc1: past the XCD's
// non-coherent L2) with a vector load. flag_issue returns the loaded VGPR
// without waiting for it; flag_value makes it uniform (and waits).
__device__ __forceinline__ uint32_t flag_issue(const uint32_t* f) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(f), 0, 4, 0x00020000);
  return __builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 17);
}
__device__ __forceinline__ uint32_t flag_value(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)v);
}
__device__ __forceinline__ uint32_t flag_load(const uint32_t* f) { return flag_value(flag_issue(f)); }
// an action value of an explicitly handed-off row: device-coherent like the flag
__device__ __forceinline__ float act_load(const char* row, uint32_t off) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(row), 0, 0x7fffffff,
                                                                     0x00020000);
  return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 17));
}
// Spin until the flag reaches `want` (sequence numbers stay below 2^31). Returns
// the last value seen; on timeout flags the status and returns 0.
__device__ uint32_t wait_flag(const uint32_t* f, uint32_t want, uint32_t seen, int32_t* status, int lane) {
  for (uint32_t it = 0; seen < want; ++it) {
    if (it >= kSpinLimit) {
      if (lane == 0) atomicOr(status, SACENV_STATUS_HANDOFF_TIMEOUT);
      return 0u;
    }
    __builtin_amdgcn_s_sleep(2);
    seen = flag_load(f);
  }
  return seen;
}

// One owner wave: BoatEnv.step for 64 consecutive envs, one per lane.
// kRoll: n_steps steps in one launch (sacenv_boat_rollout, sacenv_boat_segment)
// with the state in registers, step ks's outputs where RollArgs says; the
// state is loaded once and stored once.
// kNc: spline curves of the wind (0: constants or the shared table; 1: exp
// 4/5; 2: exp 6); kTIdx: t derived from the index (t_from_index). Both are
// launch constants; as template arguments the step carries no code (and no
// loads whose pending registers the waitcnt pass must respect) of the other
// wind kinds.
// kHand (kRoll only): rows published step by step and/or done flags (the
// closed loop); without it the loop carries no flag code at all (the launch
// checked that every row was already published).
template <bool kRoll, int kNc, bool kTIdx, bool kHand = false, int kRows = 1, bool kVc = kRoll>
__device__ __forceinline__ void owner_wave(const SacenvBoatParams& pin, const Arena& A, const Tail& Tin,
                                           const float* __restrict__ action, OwnerLds& l, int ob,
                                           int lane, int n_steps = 1, const RollArgs* ra = nullptr,
                                           char* trans1 = nullptr, uint32_t seen0 = 0u) {
#ifdef SACENV_STAMPS
  const uint64_t st_real0 = __builtin_amdgcn_s_memrealtime();
  uint64_t st_loaded = 0, st_computed = 0;
#define OWNER_STAMP(v)                                            \
  do {                                                            \
    if (!kRoll) { /* (multi-step launches: the PHASE clocks) */   \
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory"); \
      v = __builtin_amdgcn_s_memrealtime();                       \
    }                                                             \
  } while (0)
#else
#define OWNER_STAMP(v) \
  do {                 \
  } while (0)
#endif
  const int e = ob * kWave + lane;
  const uint32_t eo = (uint32_t)e * 8u, eo4 = (uint32_t)e * 4u;  // per-lane byte offsets
  const char* const wbase = A.wk_wave(ob * kWave);  // the wave's slot-ring block (uniform)
  const bool active = e < pin.n_envs;
  // the (first) action, in flight with the state loads. A handed-off row
  // (sacenv_boat_segment) is read only after its flag says it is ready.
  // Padding lanes (e >= n_envs) read their wave's first env -- memory their own
  // wave's hand-off flag covers -- and step with action 0, so padding state
  // never depends on another wave's row.
  const char* const abase = reinterpret_cast<const char*>(action) + (active ? eo4 : (uint32_t)ob * 256u);
  // info['termination'] as the reference's info dict keeps it (main.py:83): the last
  // termination code 1..5, carried across steps and auto-resets
  uint32_t lt = (uint32_t)A.i32e(U_LTERM, eo4);
  const uint32_t* const rdy = kHand ? (ra->ready != nullptr ? ra->ready + ob : nullptr) : nullptr;
  const int64_t arow = kRoll ? ra->act_stride * 4 : 0;  // bytes between action rows
  // kHand: the latest value of this wave's ready flag (the launch waited for row 0)
  uint32_t seen = seen0;
  bool failed = false;      // a hand-off timed out: the launch stops stepping
  const bool per_step = kHand && rdy != nullptr && seen < ra->seq0 + (uint32_t)n_steps;
  float act_cur = *reinterpret_cast<const float*>(abase);
  constexpr bool t_idx = kTIdx;
  constexpr int nc = kNc;  // spline curves of the wind
  // per-lane 8-B loads straight into registers, coalesced over the wave's
  // 512-B rows; the wind piece and index first, as the wind is evaluated
  // first (measured 0.16 us/step faster than 16-B loads staged through LDS)
  int32_t index = A.i32e(U_IDX, eo4);
  int cons = pin.autoreset ? A.i32e(U_CONS, eo4) : 0;  // (early: the refresh gathers' slot)
  double cf[kCoef];
#pragma unroll
  for (int k = 0; k < kCoef; ++k) cf[k] = 0.0;
  if (nc > 0) {  // two uniform branches, not one per field; 16-B pairs (y0, m0), (y1, m1)
#pragma unroll
    for (int k = 0; k < 4; k += 2) {
      const double2 q = A.f64p(U_COEF + 8 * k, eo);
      cf[k] = q.x, cf[k + 1] = q.y;
    }
    if (nc > 1) {
#pragma unroll
      for (int k = 4; k < 8; k += 2) {
        const double2 q = A.f64p(U_COEF + 8 * k, eo);
        cf[k] = q.x, cf[k + 1] = q.y;
      }
    }
  }
  const double2 p_sxy = A.f64p(U_SX, eo), p_srvx = A.f64p(U_SR, eo), p_vyvr = A.f64p(U_VY, eo);
  const double2 p_rudep = A.f64p(U_RUD, eo);
  double s_x = p_sxy.x, s_y = p_sxy.y, s_r = p_srvx.x;
  double v_x = p_srvx.y, v_y = p_vyvr.x, v_r = p_vyvr.y;
  double rudder = p_rudep.x, t = t_idx ? 0.0 : A.f64e(U_T, eo), ep = p_rudep.y;
  // keep the whole load burst ahead of the first computation: the scheduler
  // would otherwise hoist the refresh-address math (index, cons) above the
  // state loads and wait for those two first
  __builtin_amdgcn_sched_barrier(0);
  // (the caller moved the fp64 constants to VGPRs ahead of the load burst:
  // measured 0.09 us/step faster than doing it here, behind the burst)
  const SacenvBoatParams& p = pin;
  const Tail& T = Tin;
  constexpr bool kWT = !kRoll || kHand;  // write-through outputs (st_out)
  // one-step launch: plain constants (the compiler places them; the VGPR copies
  // cost their moves in every launch: k_step 5.02 -> 5.36 us measured), the
  // multi-step loop: VGPR copies, moved once per launch
  const TrigK K = trig_k<kVc>();
  const ObsConst oc = kVc ? obs_const_v(T) : obs_const(T);
  // Wind.get_wind(index) (wind.py:20-24, IndexError guard) of this step. Curves:
  // from the lane's copy of its spline piece (wind_coef, loaded with the
  // state). The copy is refreshed from the active slot at the end of a step
  // whose successor enters the next knot interval, and in an episode's first
  // step (a new episode starts with y0 = y(0) in the piece, exact at t = 0
  // whatever the other fields hold): the few lanes that refresh issue their scattered slot
  // loads here and store the piece at the end.
  // rollout: the next pre-drawn episode's y(0) and start y, carried in registers
  double y0c[2] = {0.0, 0.0};
  int32_t syc = 0;
  if (kRoll && p.autoreset) {
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (c < nc) y0c[c] = A.f64e(U_W0N + 8 * c, eo);
    if (p.experiment == 2) syc = A.i32e(U_SYN, eo4);
  }
#ifdef SACENV_STAMPS
  // per-phase shader-clock sums over a launch's steps (tools/phase_stamps.py):
  // issue-progress clocks, no waits added; sched barriers pin the phase edges
  uint64_t ph[4] = {0, 0, 0, 0}, ph_t = 0;
#define PHASE(i)                                         \
  do {                                                   \
    __builtin_amdgcn_sched_barrier(0);                   \
    const uint64_t ph_now = __builtin_amdgcn_s_memtime(); \
    if ((i) > 0) ph[(i) - 1] += ph_now - ph_t;           \
    ph_t = ph_now;                                       \
    __builtin_amdgcn_sched_barrier(0);                   \
  } while (0)
#else
#define PHASE(i) \
  do {           \
  } while (0)
#endif
  // carried between the steps of a multi-step launch (updated at each step's
  // end, not recomputed): the knot coordinate of this step's grid index, and
  // the lane's ring byte offsets of its current and next episode slots
  // (wko_l(slot, 0, 0, lane)): ~25 integer VALU a step less
  Knot kcur = knot_coord(p, index > p.wind_len - 1 ? p.wind_len - 1 : index);
  const uint32_t slot_bytes = 2u * 16u * (uint32_t)A.nk, lane_ring = A.wko_l(0, 0, 0, lane);
  const int slot0 = cons % kSlots;
  int nslot = slot0 + 1 == kSlots ? 0 : slot0 + 1;
  uint32_t so = lane_ring + (uint32_t)slot0 * slot_bytes, sno = lane_ring + (uint32_t)nslot * slot_bytes;
  // staged replay rows: each lane's mark bits of every step of the launch (its env's
  // ceil(n_steps / 64) words, env-major), staged in LDS once (a per-step global load
  // would sit in the loop's vmcnt accounting, and the step's first full wait would
  // expose its ~1-us latency every step)
  if (kRoll && kRows == 2) {
    // the launch consumes its marks: each env's words are read by its lane alone and
    // cleared, so the staged replay's next draws into this buffer start from zero (no
    // fill kernel). No marks: every row, all bits set (the loop reads mk[(ks / 32) % 8]
    // with no per-step branch on the pointer)
    static_assert((kMkWords & (kMkWords - 1)) == 0, "l.mk is indexed (ks / 32) % kMkWords");
    if (ra->marks != nullptr) {
      const int W = (n_steps + 63) / 64;  // (n_steps <= 256 with marks: sacenv_boat_segment)
      unsigned long long* const w = ra->marks + (int64_t)e * W;
      for (int q = 0; q < W; ++q) {
        const unsigned long long m = w[q];
        w[q] = 0ull;
        l.mk[2 * q][lane] = (uint32_t)m;
        l.mk[2 * q + 1][lane] = (uint32_t)(m >> 32);
      }
    } else {
#pragma unroll
      for (int q = 0; q < kMkWords; ++q) l.mk[q][lane] = ~0u;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // the staged rows: the wave's rows through one buffer resource (env-major: lane's row
  // of step ks at s_lane + ks * 64 from the wave's first env's), the step's offset in
  // the scalar offset
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      (kRoll && kRows == 2) ? ra->stage + (int64_t)ob * kWave * n_steps * 64 : nullptr, 0, 0x7fffffff, 0x00020000);
  const uint32_t s_lane = (kRoll && kRows == 2) ? (uint32_t)lane * (uint32_t)n_steps * 64u : 0u;
  uint32_t mkw = 0u;
  // every load of the launch's prologue has landed before the step loop: the waitcnt
  // pass then sees no load pending at the loop's entry, and the loop keeps no wait
  // for them -- such a wait, on later steps, also waits for the previous step's
  // stores (vmcnt counts both on gfx950)
  if (kRoll) __builtin_amdgcn_s_waitcnt(0);
  for (int ks = 0; ks < (kRoll ? n_steps : 1) && (!kHand || !failed); ++ks) {
  PHASE(0);
  const float act = active ? act_cur : 0.0f;
  // the next step's action, a step ahead: open-loop rows at once; a handed-off
  // row if its flag already said so, else after this step's outputs (below)
  bool act_next = false;
  uint32_t flag_now = 0u;
  if (kRoll && ks + 1 < n_steps) {
    if (!kHand || !per_step) {  // open loop, or every row of the launch already published
      act_cur = *reinterpret_cast<const float*>(abase + (int64_t)(ks + 1) * arow);
      act_next = true;
    } else {
      if (seen >= ra->seq0 + (uint32_t)ks + 2u) {
        act_cur = act_load(abase, (uint32_t)((ks + 1) * arow));
        act_next = true;
      }
      flag_now = flag_issue(rdy);  // in flight during the step, read at its end
    }
  }
  const int wi = index > p.wind_len - 1 ? p.wind_len - 1 : index;
  Knot knext = kcur;
  double wv = 0.0, wa = 0.0;
  bool refresh = false;
  int jn = 0;
  double rq[kCoef];  // refreshed piece (refresh lanes), stored at the end
  if (nc == 0) {
    wind_at(p, A, T.table, 0, e, wi, wv, wa);  // constants or the shared table
  } else {
    const double tt = kcur.t;  // = knot_coord(p, wi).t
    const double c0 = spline_piece(cf[0], cf[2], cf[1], cf[3], tt);  // cf: y0 m0 y1 m1
    if (nc == 2) {  // exp 6 (the only two-curve experiment)
      wv = c0;
      wa = spline_piece(cf[4], cf[6], cf[5], cf[7], tt);
    } else if (p.experiment == 4) {
      wv = c0;
      wa = p.wind_dir_rad;
    } else {  // 5: rectified angle (wind.py:92-99)
      wv = p.max_velocity;
      wa = ((c0 <= 0.5 / 2 ? 0.0 : 1.0) * kPi) + kPi / 2;
    }
    const int wn = index + 1 > p.wind_len - 1 ? p.wind_len - 1 : index + 1;
    knext = knot_coord(p, wn);
    jn = knext.j;
    refresh = index == 0 || jn != kcur.j;
    // (one wave-uniform branch: in ~3 of 4 steps no lane of the wave refreshes)
    if (__ballot(refresh) != 0ull) {  // the piece of the next step's interval for refreshing lanes, stored at
      // the end (own registers, read only there). Unconditional loads, the
      // other lanes reading one fixed line: with no branch around them the
      // waitcnt pass can count the loads in flight (a load under a divergent
      // branch made the first use of every earlier load wait for all of them)
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (c < nc) {
          double q[4];
          A.piece_at(wbase, refresh ? so + (uint32_t)(c * A.nk + jn) * 16u : 0u, q);
          rq[4 * c] = q[0], rq[4 * c + 1] = q[1], rq[4 * c + 2] = q[2], rq[4 * c + 3] = q[3];
        }
    }
  }
  // autoreset: the next pre-drawn episode's curve values at grid index 0 and
  // start y. Lanes in an episode's first step gather them from the slot ring
  // and refresh their lane-coalesced copies; the others read the copies. One
  // unconditional load per value from a per-lane address (no branch: see the
  // refresh loads above; no select between two loaded registers either).
  double y0n[2];
  int32_t syn = 0;
  const bool hdr_refresh = p.autoreset && index == 0;
  {
    const int ns = nslot;  // (cons + 1) % kSlots
#pragma unroll
    for (int c = 0; c < 2; ++c)
      if (c < nc) {
        // (rollout: the copy is in registers; other lanes read the ring's first line)
        const double v = *(hdr_refresh ? reinterpret_cast<const double*>(wbase + sno + (uint32_t)(c * A.nk) * 16u)
                                       : (kRoll ? A.wind_knots() : &A.f64e(U_W0N + 8 * c, eo)));
        y0n[c] = kRoll && !hdr_refresh ? y0c[c] : v;
      }
    if (nc == 0 && p.experiment == 2) {
      const int32_t v = *(hdr_refresh ? &A.i32e(U_STARTY + 4 * ns, eo4) : &A.i32e(U_SYN, eo4));
      syn = kRoll && !hdr_refresh ? syc : v;
    }
  }
  OWNER_STAMP(st_loaded);
  const double r_mx = T.r_mx, r_my = T.r_my, r_iz = T.r_iz, r_nd = T.r_nd, r_w = T.r_w;

  // BoatEnv.step :69-73
  t = t_idx ? (double)(index + 1) * p.dt : t + p.dt;  // boat_env.py:69
  const int32_t fuel = p.fuel0 - (index + 1);
  if (p.test_mode == 0) rudder = rudder + div_c((double)act, 10.0, 0.1);  // action / 10
  if (!t_idx) EARLY_STORE(U_T, t);
  const bool first = index == 0;  // integrator counter == 0 (control_blocks.py:21-22)
  const double v_x_w = v_x * p.one_minus_wf;
  const double J = p.n_rpm != 0.0 ? div_c(v_x_w, p.n_times_d, r_nd) : 0.0;  // :222-224
  double sin_J, sin_rud, swa, cwa;
  trig3(J, rudder, wa, &sin_J, &sin_rud, &swa, &cwa, K);
  PHASE(1);

  // eom_longitudinal :213-239
  const double F_R = (v_x * v_x) * T.k_front;
  const double F_T = sin_J * T.k_thrust;
  const double F_C = v_y * p.m_plus_my * v_r;
  // v^2 sign(v) as v |v| (|.| is a free operand modifier): one multiply instead
  // of a square, two compares, a convert and a multiply; the same double for
  // every v != 0 (multiplying by +-1 is exact, in any position)
  const double w2s = wv * fabs(wv);
  const double F_W = (w2s * T.k_front) * cwa;
  const double a_x = div_c(-F_R + F_T + F_C + F_W, p.m_plus_mx, r_mx);
  v_x = first ? 3.0 : a_x * p.dt + v_x;

  // eom_transverse :241-265 (new v_x)
  const double F_R2 = (v_y * fabs(v_y)) * T.k_side;
  const double vx2 = v_x * v_x;  // (the new v_x)
  const double F_RU = sin_rud * (vx2 * T.k_rud_front);
  const double F_C2 = v_x * p.m_plus_mx * v_r;
  const double F_W2 = (w2s * T.k_side) * swa;
  const double a_y = div_c(-F_R2 + F_RU + F_C2 + F_W2, p.m_plus_my, r_my);
  v_y = first ? 0.0 : a_y * p.dt + v_y;

  // eom_yawning :267-281
  const double M_hull = (v_r * fabs(v_r)) * T.k_hull;
  const double M_rud = ((v_x * fabs(v_x)) * T.k_rud_moment) * sin_rud;
  const double a_r = div_c(-M_hull + M_rud, p.i_plus_iz, r_iz);
  v_r = first ? 0.0 : a_r * p.dt + v_r;
  EARLY_STORE2(U_VY, v_y, v_r);

  // get_kinematics :283-306
  // drift = atan2(v_x, v_y) has sin = v_x / v, cos = v_y / v, so
  // sin(drift - s_r) v = v_x cos s_r - v_y sin s_r and
  // cos(drift - s_r) v = v_y cos s_r + v_x sin s_r: no atan2, sqrt or division
  // (122 fewer VALU; -0.26 us/step). Same parity class as the ocml/libm
  // differences: the increments agree to a few ulp of v dt.
  s_r = v_r * p.dt + s_r;
  double ssr, csr;
  sincos_cw(s_r, &ssr, &csr, K);
  s_x = (v_x * csr - v_y * ssr) * p.dt + s_x;
  s_y = (v_y * csr + v_x * ssr) * p.dt + s_y;
  index = index + 1;
  EARLY_STORE2(U_SX, s_x, s_y);
  EARLY_STORE2(U_SR, s_r, v_x);
  if (!kRoll) st_out(A.i32e(U_IDX, eo4), index);
  PHASE(2);

  Obs o = make_obs(p, oc, s_x, v_x, a_x, s_y, v_y, a_y, s_r, v_r, a_r, rudder, (double)fuel);

  // exponential_reward (reward_functions.py:42-57), f_x = 0
  const double ay = fabs(s_y);
  const double f_y = div_c(ay, p.track_width, r_w) / (1.0 + exp_v(p.reward_k * (ay - p.reward_center), K));
  double reward = 0.0 - f_y;

  // termination chain :84-105 (the first true condition wins), as selects: as an
  // if/else-if chain it compiled to nested exec-mask branches (~25 SALU a step)
  const bool goal = s_x >= p.goal_line;
  int tm = (rudder > kPi / 3) | (rudder < -kPi / 3) ? SACENV_TERM_RUDDER_BROKEN : SACENV_TERM_NONE;
  tm = p.t_max <= t ? SACENV_TERM_TIMEOUT : tm;
  tm = fuel < 0 ? SACENV_TERM_OUT_OF_FUEL : tm;
  tm = (fabs(s_y) > p.oob_limit) | (s_x < 0.0) ? SACENV_TERM_OUT_OF_BOUNDS : tm;
  tm = goal ? SACENV_TERM_REACHED_GOAL : tm;
  reward = goal ? reward + 1000.0 : reward;
  // penalties :107-111
  reward = ((rudder > kPi / 4) | (rudder < -kPi / 4)) ? reward - fabs(rudder) * 100.0 : reward;
  reward = fabs(s_r) > kPi / 2 ? reward - 1.0 : reward;
  ep = ep + reward;
  uint8_t term = active ? (uint8_t)tm : (uint8_t)SACENV_TERM_NONE;  // padding lanes never end

  if (term != SACENV_TERM_NONE)  // no-return atomic: nothing on the critical path waits
    __hip_atomic_fetch_add(&A.at_e<uint32_t>(U_CNT + 4 * (term - 1), eo4), 1u, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
  if (term == SACENV_TERM_NONE && active && p.max_episode_steps > 0 && index >= p.max_episode_steps)
    term = SACENV_TERM_TRUNCATED;
  lt = (uint32_t)term - 1u < 5u ? (uint32_t)term : lt;  // codes 1..5 overwrite it, 0 and 6 keep it
  const bool ended = term != SACENV_TERM_NONE;
  PHASE(3);

  OWNER_STAMP(st_computed);
  // this step's outputs: the arena's record, or the multi-step launch's
  char* const R = kRoll ? ra->rec + (int64_t)ks * ra->rec_stride : A.b + A.ur() * A.np;
  float* const fin = kRoll ? (ra->fin != nullptr ? ra->fin + (int64_t)ks * ra->fin_stride : nullptr)
                           : A.final_obs();
  // (kRoll: kRows compiles the pooled row in or out; the step launch decides at run time)
  char* const trans = kRows != 1 ? nullptr
                              : kRoll ? (ra->trans != nullptr ? ra->trans + (int64_t)ks * ra->trans_stride : nullptr)
                                      : trans1;
  if (p.out_flags & SACENV_OUT_REWARD64) A.at_e<double>(A.ur() + 126, eo) = reward;
  if (p.out_flags & SACENV_OUT_ACCEL) {
    A.at_e<double>(A.ur() + 102, eo) = a_x;
    A.at_e<double>(A.ur() + 110, eo) = a_y;
    A.at_e<double>(A.ur() + 118, eo) = a_r;
  }
  const bool restart = ended && p.autoreset;
  if (ended) A.at_e<double>(A.ur() + 94, eo) = ep;
  // terminal obs of the envs that auto-reset (main.py:72 reset, boat_env.py:121):
  // per-lane stores (measured 0.13 us/step cheaper than a 2.8-KB block store per
  // restarting wave with two extra barriers)
  if (restart && fin != nullptr) store_obs(fin + (int64_t)e * SACENV_OBS_DIM, o);
  int cons_out = cons;
  // the record's obs row: this step's obs, or a restarting lane's first obs of
  // its next episode. The restart's ~45 per-lane selects (state, row, slot ring)
  // sit behind ONE wave-uniform branch: in most steps no lane of the wave ends
  // its episode (an episode runs up to 500 steps), and the selects are skipped.
  // the staged replay row of this step (sacenv_replay_sample_staged reads it), only
  // where a learn of this or the next segment samples it or its successor: one 64-B
  // line per row, s' (the pre-reset obs), reward, action, term | lt << 8, obs3_next
  // (written by a restarting lane below); stored before the restart selects, so the
  // pre-reset obs need not stay live across them
  bool staged = false;
  if (kRoll && kRows == 2) {
    // the lane's mark bits, one LDS read per 32 steps (a per-step read waited its
    // latency right before the test), consumed bit by bit
    if ((ks & 31) == 0) mkw = l.mk[(ks >> 5) & (kMkWords - 1)][lane];  // (n_steps <= 256 with marks)
    staged = (mkw & 1u) != 0u;
    mkw >>= 1;
    if (staged) {  // (write-through, as the record's stores: measured +70 us per launch here)
      const uint32_t so = (uint32_t)ks * 64u;
      __builtin_amdgcn_raw_buffer_store_b128(
          u4v{__float_as_uint(o.v[0]), __float_as_uint(o.v[1]), __float_as_uint(o.v[2]), __float_as_uint(o.v[3])},
          srs, s_lane, so, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          u4v{__float_as_uint(o.v[4]), __float_as_uint(o.v[5]), __float_as_uint(o.v[6]), __float_as_uint(o.v[7])},
          srs, s_lane + 16u, so, 0);
      __builtin_amdgcn_raw_buffer_store_b128(
          u4v{__float_as_uint(o.v[8]), __float_as_uint(o.v[9]), __float_as_uint(o.v[10]), __float_as_uint((float)reward)},
          srs, s_lane + 32u, so, 0);
      __builtin_amdgcn_raw_buffer_store_b128(u4v{__float_as_uint(act), (uint32_t)term | (lt << 8), 0u, 0u}, srs,
                                             s_lane + 48u, so, 0);
    }
  }
  float row[SACENV_OBS_DIM];
#pragma unroll
  for (int k = 0; k < SACENV_OBS_DIM; ++k) row[k] = o.v[k];
  float row3_new = 0.0f;  // (exp 2's pooled row: the new episode's obs[3])
  const bool any_restart = __ballot(restart) != 0ull;
  if (any_restart) {
    if (restart) {  // next episode from its pre-drawn slot: a fresh Boat (boat_env.py:152-198)
      const double sy0 = p.experiment == 2 ? (double)syn : 0.0;  // :166-169
      s_x = 0.0, s_y = sy0, s_r = 0.0, v_x = 0.0, v_y = 0.0, v_r = 0.0, rudder = 0.0;
      t = 0.0, ep = 0.0;  // :122
      index = 0;
      Obs fo;
      if (p.experiment == 2 || p.fuel0 == 0) {
        fo = make_obs(p, oc, 0.0, 0.0, 0.0, sy0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, (double)p.fuel0);
      } else {  // make_obs of the zero state, folded: (0+W)/(2W) = 0.5 and fuel0/fuel0 = 1 exactly
        constexpr float kRud0 = (float)((0.0 + kPi / 3) * (1.0 / (kPi / 3 - (-kPi / 3))));
#pragma unroll
        for (int k = 0; k < SACENV_OBS_DIM; ++k) fo.v[k] = 0.0f;
        fo.v[3] = 0.5f;
        fo.v[9] = kRud0;
        fo.v[10] = 1.0f;
      }
#pragma unroll
      for (int k = 0; k < SACENV_OBS_DIM; ++k) row[k] = fo.v[k];
      row3_new = fo.v[3];
      if (kRoll && kRows == 2 && p.experiment == 2 && staged)  // the staged row's obs3_next
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(row3_new), srs, s_lane + 56u, (uint32_t)ks * 64u, 0);
      cons_out = cons + 1;
    }
  }
  // the dynamics' fields went out as they were computed; what is left: the
  // fresh state of restarting envs (same lane, same address: the later store
  // wins), ep_reward, the next wind, and the record
  if (!kRoll && restart) {
    EARLY_STORE2(U_SX, s_x, s_y);
    EARLY_STORE2(U_SR, s_r, v_x);
    EARLY_STORE2(U_VY, v_y, v_r);
    if (!t_idx) st_out(A.f64e(U_T, eo), t);
    st_out(A.i32e(U_IDX, eo4), index);
    st_out(A.i32e(U_CONS, eo4), cons_out);
  }
  if (!kRoll) {
    st_out(A.i32e(U_LTERM, eo4), (int32_t)lt);
    EARLY_STORE2(U_RUD, rudder, ep);
    if (restart && nc > 0) {  // the new episode's first wind: the piece's y0 = y(0); at
      // t = 0 the piece is exactly y0 whatever (finite) m0, y1, m1 it still holds
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (c < nc) st_out(A.f64e(U_COEF + 32 * c, eo), y0n[c]);
    } else if (refresh) {
#pragma unroll
      for (int k = 0; k < kCoef; k += 2)
        if (k < 4 * nc) EARLY_STORE2(U_COEF + 8 * k, rq[k], rq[k + 1]);
    }
    if (hdr_refresh) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (c < nc) st_out(A.f64e(U_W0N + 8 * c, eo), y0n[c]);
      if (p.experiment == 2) st_out(A.i32e(U_SYN, eo4), syn);
    }
  } else {  // the same updates, in registers (each behind a wave-uniform branch)
    if (nc > 0 && __ballot(refresh && !restart) != 0ull && refresh && !restart) {
#pragma unroll
      for (int k = 0; k < kCoef; ++k) cf[k] = rq[k];
    }
#pragma unroll
    for (int c = 0; c < 2; ++c) y0c[c] = y0n[c];
    syc = syn;
    cons = cons_out;
    kcur = knext;
    if (any_restart && restart) {  // the next slot becomes current; grid index 0
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (c < nc) cf[4 * c] = y0n[c];
      so = sno;
      nslot = nslot + 1 == kSlots ? 0 : nslot + 1;
      sno = nslot == 0 ? lane_ring : sno + slot_bytes;
      kcur = knot_coord(p, 0);
    }
  }
  if (kRows == 3) {  // (fresh rows: streaming stores, as the obs row below)
    __builtin_nontemporal_store((float)reward, reinterpret_cast<float*>(R + 44 * A.np + eo4));
    __builtin_nontemporal_store((uint8_t)(ended ? 1 : 0), reinterpret_cast<uint8_t*>(R + 48 * A.np + e));
    __builtin_nontemporal_store(term, reinterpret_cast<uint8_t*>(R + 49 * A.np + e));
  } else {
    st_out<kWT>(*reinterpret_cast<float*>(R + 44 * A.np + eo4), (float)reward);
    st_out<kWT>(*reinterpret_cast<uint8_t*>(R + 48 * A.np + e), (uint8_t)(ended ? 1 : 0));
    st_out<kWT>(*reinterpret_cast<uint8_t*>(R + 49 * A.np + e), term);
  }
  // a restarting env's row is its new episode's first obs
  if (!kWT) {
    // write-back record (open-loop multi-step launch): each lane stores its own
    // 44-B row as 16 + 16 + 12 B (4-B aligned vector stores): 0.08 us/step
    // cheaper than the LDS-staged block below, whose LDS round trip and waits
    // sit on the step's path
    if (kRows == 3)  // every step's record to fresh rows (sacenv_boat_rollout): streaming stores
      store_row_nt<SACENV_OBS_DIM>(reinterpret_cast<float*>(R) + (int64_t)e * SACENV_OBS_DIM, row);
    else
      store_row<SACENV_OBS_DIM>(reinterpret_cast<float*>(R) + (int64_t)e * SACENV_OBS_DIM, row);
  } else {
    // obs rows through LDS, stored as write-through float4 (64 rows x 44 B = 176 float4)
#pragma unroll
    for (int k = 0; k < SACENV_OBS_DIM; ++k) l.obs[lane * SACENV_OBS_DIM + k] = row[k];
    // the rows are this wave's own LDS: a wave's LDS accesses run in issue order,
    // so only the compiler must keep the stores ahead of the loads (no workgroup
    // barrier: a step workgroup may hold several owner waves, or toy waves)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int64_t row0 = (int64_t)ob * kWave * SACENV_OBS_DIM;
    store_obs_block<SACENV_OBS_DIM, kWT>(l.obs, reinterpret_cast<float*>(R) + row0, lane);
    if (kRoll) {  // l.obs is rewritten by the next step
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  if (trans != nullptr) {  // the pooled transition row (sacenv_boat_step_pooled)
    // s' entries 0..8 = the pre-reset obs (entries 9 and 10, rudder and fuel, follow
    // on the receivers from the actions and the episode starts), reward, action,
    // term (done = term != 0) and, in experiment 2, the new episode's obs[3]
    if (!kWT) {  // per-lane rows, as the record's
      store_row<SACENV_TRANS_OBS>(reinterpret_cast<float*>(trans) + (int64_t)e * SACENV_TRANS_OBS, o.v);
    } else {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
      for (int k = 0; k < SACENV_TRANS_OBS; ++k) l.obs[lane * SACENV_TRANS_OBS + k] = o.v[k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      store_obs_block<SACENV_TRANS_OBS, kWT>(
          l.obs, reinterpret_cast<float*>(trans) + (int64_t)ob * kWave * SACENV_TRANS_OBS, lane);
    }
    constexpr int kOff = 4 * SACENV_TRANS_OBS;  // byte columns (x n_pad) after s'
    st_out<kWT>(*reinterpret_cast<float*>(trans + kOff * A.np + eo4), (float)reward);
    st_out<kWT>(*reinterpret_cast<float*>(trans + (kOff + 4) * A.np + eo4), act);
    st_out<kWT>(*reinterpret_cast<uint8_t*>(trans + (kOff + 8) * A.np + e), term);
    if (pin.experiment == 2)
      st_out<kWT>(*reinterpret_cast<float*>(trans + (kOff + 9) * A.np + eo4), row3_new);
    if (kRoll && kWT) {  // l.obs is rewritten by the next step
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
  }
  if (kHand && ra->done != nullptr) {
    // step ks's outputs visible device-wide (release: L2 write-back + wait for
    // the stores), then its done flag, write-through
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    if (lane == 0)
      __hip_atomic_store(ra->done + ob, ra->seq0 + (uint32_t)ks + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (kHand && per_step && ks + 1 < n_steps) {
    const uint32_t fv = flag_value(flag_now);
    seen = fv > seen ? fv : seen;
    failed = seen == SACENV_FLAG_ABORT;  // the producer gave up: so does this wave
    if (!act_next && !failed) {  // closed loop: the next action comes after these outputs
      seen = wait_flag(rdy, ra->seq0 + (uint32_t)ks + 2u, seen, ra->status, lane);
      failed = seen == 0u || seen == SACENV_FLAG_ABORT;
      act_cur = act_load(abase, (uint32_t)((ks + 1) * arow));
    }
  }
  PHASE(4);
  }  // steps
  if (kHand && failed && ra->done != nullptr && lane == 0)  // waiters on this wave must not hang
    __hip_atomic_store(ra->done + ob, SACENV_FLAG_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (kRoll) {  // the carried state, once
    A.f64e(U_SX, eo) = s_x, A.f64e(U_SY, eo) = s_y, A.f64e(U_SR, eo) = s_r;
    A.f64e(U_VX, eo) = v_x, A.f64e(U_VY, eo) = v_y, A.f64e(U_VR, eo) = v_r;
    A.f64e(U_RUD, eo) = rudder;
    if (!t_idx) A.f64e(U_T, eo) = t;
    A.f64e(U_EP, eo) = ep;
    A.i32e(U_IDX, eo4) = index;
    A.i32e(U_LTERM, eo4) = (int32_t)lt;
    if (p.autoreset) A.i32e(U_CONS, eo4) = cons;
#pragma unroll
    for (int k = 0; k < kCoef; ++k)
      if (k < 4 * nc) A.f64e(U_COEF + 8 * k, eo) = cf[k];
    if (p.autoreset) {
#pragma unroll
      for (int c = 0; c < 2; ++c)
        if (c < nc) A.f64e(U_W0N + 8 * c, eo) = y0c[c];
      if (p.experiment == 2) A.i32e(U_SYN, eo4) = syc;
    }
  }

#ifdef SACENV_STAMPS
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (kRoll && lane == 0) {  // phase sums (shader clocks) of this launch
    double* d = A.accel() + (int64_t)ob * 8;
    for (int i = 0; i < 4; ++i) d[i] = (double)ph[i];
    d[4] = (double)n_steps;
  } else if (lane == 0) {
    double* d = A.accel() + (int64_t)ob * 4;
    d[0] = (double)st_real0;
    d[1] = (double)__builtin_amdgcn_s_memrealtime();
    d[2] = (double)st_loaded;
    d[3] = (double)st_computed;
  }
#endif
}

// The step launch. Grid: nb_boat owner waves, then (kMixed) the waves of
// each toy arena: heterogeneous workgroups of one launch, selected by
// uniform block-index ranges. One wave per workgroup (measured against 2 and
// 4 waves, with or without LDS padding to one workgroup per CU: 6.04-6.29 us
// against 5.33-5.35).
template <bool kMixed, int kNc, bool kTIdx>
__global__ void __launch_bounds__(kWave) k_step(SacenvBoatParams p, Arena A, Tail T,
                                                const float* __restrict__ action, int nb_boat,
                                                MixedToys M, char* __restrict__ trans) {
  __shared__ OwnerLds slds;
  const int lane = threadIdx.x;
  int b = (int)blockIdx.x;
  if (!kMixed || b < nb_boat) {
    // (the parameters stay in SGPRs: VGPR copies ahead of the load burst delay it in
    // every launch, measured k_step 5.79 -> 5.37 us without them)
    owner_wave<false, kNc, kTIdx>(p, A, T, action, slds, b, lane, 1, nullptr,
                                  trans);
    return;
  }
  b -= nb_boat;
  if (b < M.nb[0]) {
    toy_wave(M.p[0], M.a[0], b, lane);
  } else if (M.n > 1) {
    toy_wave(M.p[1], M.a[1], b - M.nb[0], lane);
  }
}



// n_steps BoatEnv.step launches fused, the state in registers between the
// steps: open-loop rollouts (records per step) and the segment
// launch (the arena's record every step, actions behind per-wave flags)
//
// kVc: the fp64 constants as VGPR copies (one owner wave per SIMD: k_rollout), or
// as literals and scalar registers (k_rollout_dense: 238 VGPRs, two owner waves
// per SIMD, for grids with more owner waves than SIMDs -- 131 072 envs: 48.5
// against 44.4 G env-steps/s; at one wave per SIMD the copies win, 1.34 against
// 2.04 us per step). The same arithmetic either way: results are bit-identical.
template <int kNc, bool kTIdx, int kRows, bool kVc>
__device__ __forceinline__ void rollout_body(const SacenvBoatParams& p, const Arena& A, const Tail& T,
                                             const float* __restrict__ action, int n_steps, const RollArgs& ra,
                                             OwnerLds& slds) {
  const int ob = blockIdx.x, lane = threadIdx.x;
  uint32_t seen = 0u;
  bool hand = ra.done != nullptr;
  if (ra.ready != nullptr || ra.done != nullptr) {
    // abort protocol (sacenv.h): after a hand-off timeout anywhere, a hand-off
    // launch steps nothing; a producer that gave up published SACENV_FLAG_ABORT
    const uint32_t* rdy = ra.ready != nullptr ? ra.ready + ob : nullptr;
    const uint32_t st = flag_issue(reinterpret_cast<const uint32_t*>(ra.status));
    const uint32_t f0 = rdy != nullptr ? flag_issue(rdy) : 0u;
    bool stop = (flag_value(st) & SACENV_STATUS_HANDOFF_TIMEOUT) != 0u;
    if (!stop && rdy != nullptr) {
      seen = wait_flag(rdy, ra.seq0 + 1u, flag_value(f0), ra.status, lane);
      stop = seen == 0u || seen == SACENV_FLAG_ABORT;  // row 0 never came: nothing steps
    }
    if (stop) {
      if (ra.done != nullptr && lane == 0)  // waiters on this wave must not hang either
        __hip_atomic_store(ra.done + ob, SACENV_FLAG_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
  }
  if (ra.ready != nullptr) {
    // the rows the flag covers were written before it (the producer's release):
    // drop any stale copy of them from this XCD's L2 once, then read them plainly;
    // rows published only later are read device-coherently, step by step
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    hand = hand || seen < ra.seq0 + (uint32_t)n_steps;
  }
  if (hand) {
    if (kVc)
      owner_wave<true, kNc, kTIdx, true, kRows, true>(vreg_params(p), A, vreg_tail(T), action, slds, ob, lane,
                                                       n_steps, &ra, nullptr, seen);
    else
      owner_wave<true, kNc, kTIdx, true, kRows, false>(p, A, T, action, slds, ob, lane, n_steps, &ra, nullptr, seen);
  } else {
    if (kVc)
      owner_wave<true, kNc, kTIdx, false, kRows, true>(vreg_params(p), A, vreg_tail(T), action, slds, ob, lane,
                                                        n_steps, &ra);
    else
      owner_wave<true, kNc, kTIdx, false, kRows, false>(p, A, T, action, slds, ob, lane, n_steps, &ra);
  }
}
template <int kNc, bool kTIdx, int kRows>
__global__ void __launch_bounds__(kWave) k_rollout(SacenvBoatParams p, Arena A, Tail T,
                                                   const float* __restrict__ action, int n_steps, RollArgs ra) {
  __shared__ OwnerLds slds;
  rollout_body<kNc, kTIdx, kRows, true>(p, A, T, action, n_steps, ra, slds);
}
template <int kNc, bool kTIdx, int kRows>
__global__ void __launch_bounds__(kWave) __attribute__((amdgpu_waves_per_eu(2, 2)))
k_rollout_dense(SacenvBoatParams p, Arena A, Tail T, const float* __restrict__ action, int n_steps, RollArgs ra) {
  __shared__ OwnerLds slds;
  rollout_body<kNc, kTIdx, kRows, false>(p, A, T, action, n_steps, ra, slds);
}

// sacenv_mixed_segment (BASELINE configs[4] as one persistent launch): the
// boat's owner waves (k_rollout's open loop) and each toy arena's waves,
// heterogeneous workgroups selected by uniform block-index ranges
template <int kNc, bool kTIdx>
__global__ void __launch_bounds__(kWave) k_rollout_mixed(SacenvBoatParams p, Arena A, Tail T,
                                                         const float* __restrict__ action, int n_steps, RollArgs ra,
                                                         int nb_boat, MixedToys M) {
  __shared__ OwnerLds slds;
  const int lane = threadIdx.x;
  int b = (int)blockIdx.x;
  if (b < nb_boat) {
    owner_wave<true, kNc, kTIdx, false, 0>(vreg_params(p), A, vreg_tail(T), action, slds, b, lane, n_steps,
                                               &ra);
    return;
  }
  b -= nb_boat;
  if (b < M.nb[0]) {
    toy_roll_wave(M.p[0], M.a[0], b, lane, n_steps);
  } else if (M.n > 1) {
    toy_roll_wave(M.p[1], M.a[1], b - M.nb[0], lane, n_steps);
  }
}

__global__ void __launch_bounds__(kWave) k_toy_init(SacenvToyParams p, ToyArena T, const int32_t* __restrict__ ids,
                                                    int n, int zero_counters) {
  const int q = blockIdx.x * kWave + threadIdx.x;
  if (q >= n) return;
  const int e = ids != nullptr ? ids[q] : q;
  if (e < 0 || e >= p.n_envs) return;
  double f[5];
  float obs[2];
  toy_initial(p, f, obs);
  for (int k = 0; k < 5; ++k) T.f(k)[e] = f[k];
  T.count()[e] = 0;
  if (zero_counters)
    for (int k = 0; k < 3; ++k) T.ctr(k)[e] = 0u;
  reinterpret_cast<float2*>(T.obs())[e] = make_float2(obs[0], obs[1]);
  T.reward()[e] = 0.0f;
  T.done()[e] = 0;
  T.term()[e] = 0;
}

__global__ void __launch_bounds__(kWave) k_toy_step(SacenvToyParams p, ToyArena T) {
  toy_wave(p, T, blockIdx.x, threadIdx.x);
}

__global__ void __launch_bounds__(256) k_wind_eval(SacenvBoatParams p, Arena A, Tail T,
                                                   const int32_t* __restrict__ env_ids,
                                                   const int32_t* __restrict__ idx, int n,
                                                   double* __restrict__ out_v, double* __restrict__ out_a) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int e = env_ids[q];
  if (e < 0 || e >= p.n_envs) return;
  const int slot = p.autoreset ? A.i32(U_CONS)[e] % kSlots : 0;
  double wv, wa;
  wind_at(p, A, T.table, slot, e, idx[q], wv, wa);
  out_v[q] = wv;
  out_a[q] = wa;
}

// ---------------------------------------------------------------- host side

int check_params(const SacenvBoatParams* p) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->experiment < 1 || p->experiment > 6) return SACENV_E_EXPERIMENT;
  if (p->n_envs <= 0 || p->n_envs > (1 << 22) || p->wind_len <= 0) return SACENV_E_SIZE;  // 32-bit offsets
  if (n_curves(p->experiment) > 0 && (p->n_knots < 4 || p->n_knots > kMaxK)) return SACENV_E_KNOTS;
  if (p->n_knots < 2 || p->n_knots > kMaxK) return SACENV_E_KNOTS;
  if (n_curves(p->experiment) > 0 && !p->use_wind_table && p->wind_len < 2) return SACENV_E_SIZE;
  if (p->start_y_half < 1) return SACENV_E_RANGE;
  if (p->autoreset && (p->n_helpers < 1 || p->n_helpers > 65536)) return SACENV_E_SIZE;
  return SACENV_OK;
}

Tail make_tail(const SacenvBoatParams& p, void* arena) {
  SacenvBoatLayout L;
  compute_layout(p.n_envs, p.n_knots, p.wind_len, p.use_wind_table, (p.out_flags & SACENV_OUT_KNOTS) != 0, &L);
  char* b = static_cast<char*>(arena);
  Tail T;
  T.g = reinterpret_cast<const double*>(b + L.spline_g);
  T.table = reinterpret_cast<const double*>(b + L.wind_table);
  T.r_mx = 1.0 / p.m_plus_mx;
  T.r_my = 1.0 / p.m_plus_my;
  T.r_iz = 1.0 / p.i_plus_iz;
  T.r_nd = 1.0 / p.n_times_d;
  T.r_w = 1.0 / p.track_width;
  T.r_goal = 1.0 / p.goal_line;
  T.r_two_w = 1.0 / (p.track_width + p.track_width);
  T.r_fuel = 1.0 / (double)p.fuel0;
  T.k_front = p.c_r_front * 0.5 * p.rho * p.boat_area_front;                  // F_R, F_W
  T.k_thrust = p.n_squared * p.rho * p.d_pow4 * p.one_minus_td;               // F_T / KT
  T.k_side = p.c_r_side * 0.5 * p.rho * p.boat_area_side;                     // F_R (transverse), F_W
  T.k_rud_front = p.c_r_front * 0.5 * p.rho * p.rudder_area;                  // F_RU
  T.k_hull = p.c_r_side * 0.5 * p.rho * p.boat_area_side * p.boat_l * 5.0;    // M_hull
  T.k_rud_moment = p.c_r_side * 0.5 * p.rho * p.rudder_area * (p.boat_b / 2);  // M_rudder
  return T;
}

int launch_status() {
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? SACENV_OK : (int)err;
}

inline int blocks_for(int n, int per) { return (n + per - 1) / per; }

int check_toy(const SacenvToyParams* p) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->kind != SACENV_TOY_PARACHUTE && p->kind != SACENV_TOY_CAR) return SACENV_E_EXPERIMENT;
  if (p->n_envs <= 0) return SACENV_E_SIZE;
  return SACENV_OK;
}

ToyArena make_toy_arena(const SacenvToyParams& p, void* base) {
  return ToyArena{static_cast<char*>(base), pad64(p.n_envs)};
}

}  // namespace

extern "C" {

int sacenv_abi_version(void) { return SACENV_ABI_VERSION; }

int sacenv_stream_create_exclusive(void** stream) {
  if (stream == nullptr) return SACENV_E_NULL;
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return (int)e;
  hipDeviceProp_t prop;
  e = hipGetDeviceProperties(&prop, dev);
  if (e != hipSuccess) return (int)e;
  uint32_t mask[64];
  const int words = (prop.multiProcessorCount + 31) / 32;
  if (words > 64) return SACENV_E_SIZE;
  for (int i = 0; i < words; ++i) mask[i] = 0xFFFFFFFFu;  // every CU (extra bits are ignored)
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)words, mask);
  if (e != hipSuccess) return (int)e;
  *stream = s;
  return SACENV_OK;
}

int sacenv_stream_destroy(void* stream) {
  if (stream == nullptr) return SACENV_E_NULL;
  return (int)hipStreamDestroy((hipStream_t)stream);
}

const char* sacenv_error_string(int code) {
  switch (code) {
    case SACENV_OK: return "ok";
    case SACENV_E_NULL: return "required pointer is NULL";
    case SACENV_E_EXPERIMENT: return "Well someone tried to use an experiment that doesnt exist!";
    case SACENV_E_KNOTS:
      return "Please select at least 4 fixed_points in your config. The interpolation doesn't work "
             "otherwise! (max 16)";
    case SACENV_E_SIZE: return "size out of range";
    case SACENV_E_RANGE: return "low >= high: int(0.8*track_width) must be >= 1";
    case SACENV_E_MODE: return "call not valid in this autoreset mode";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown sacenv error";
  }
}

int sacenv_boat_layout(const SacenvBoatParams* p, SacenvBoatLayout* out) {
  const int rc = check_params(p);
  if (rc) return rc;
  if (out == nullptr) return SACENV_E_NULL;
  compute_layout(p->n_envs, p->n_knots, p->wind_len, p->use_wind_table, (p->out_flags & SACENV_OUT_KNOTS) != 0, out);
  return SACENV_OK;
}

int sacenv_boat_init(const SacenvBoatParams* p, void* arena, const uint32_t* seeds, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr || seeds == nullptr) return SACENV_E_NULL;
  const hipStream_t s = (hipStream_t)stream;
  const Arena A = make_arena(*p, arena);
  const Tail T = make_tail(*p, arena);
  hipLaunchKernelGGL(k_spline_g, dim3(1), dim3(1), 0, s, *p, const_cast<double*>(T.g));
  if ((rc = launch_status())) return rc;
  hipLaunchKernelGGL(k_seed, dim3(blocks_for(p->n_envs, kWave)), dim3(kWave), 0, s, *p, A, seeds);
  if ((rc = launch_status())) return rc;
  hipLaunchKernelGGL(k_draw, dim3(p->n_envs), dim3(kWave), 0, s, *p, A, T, 0, (const int32_t*)nullptr,
                     (const int32_t*)nullptr, (const double*)nullptr, (const int32_t*)nullptr);
  if ((rc = launch_status())) return rc;
  return p->autoreset ? sacenv_boat_refill(p, arena, stream) : SACENV_OK;  // episodes 1 .. SLOTS-1
}

int sacenv_boat_reset(const SacenvBoatParams* p, void* arena, const int32_t* ids, int32_t n_ids,
                      void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  const int nb = ids != nullptr ? n_ids : p->n_envs;
  if (nb < 0) return SACENV_E_SIZE;
  if (nb == 0) return SACENV_OK;
  const hipStream_t s = (hipStream_t)stream;
  const Arena A = make_arena(*p, arena);
  const Tail T = make_tail(*p, arena);
  hipLaunchKernelGGL(k_draw, dim3(nb), dim3(kWave), 0, s, *p, A, T, 1, ids, (const int32_t*)nullptr,
                     (const double*)nullptr, (const int32_t*)nullptr);
  return launch_status();
}

int sacenv_compact_done(const uint8_t* done, int32_t n, int32_t* ids, int32_t* count, void* stream) {
  if (n < 0) return SACENV_E_SIZE;
  if (count == nullptr || (n > 0 && (done == nullptr || ids == nullptr))) return SACENV_E_NULL;
  const int aligned = (reinterpret_cast<uintptr_t>(done) & 15u) == 0;
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, (hipStream_t)stream, done, n, aligned, ids, count);
  return launch_status();
}

int sacenv_boat_reset_list(const SacenvBoatParams* p, void* arena, const int32_t* ids, const int32_t* count,
                           void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr || ids == nullptr || count == nullptr) return SACENV_E_NULL;
  const hipStream_t s = (hipStream_t)stream;
  const Arena A = make_arena(*p, arena);
  const Tail T = make_tail(*p, arena);
  // at most one workgroup per CU-slot; each loops over its share of the device-side list
  const int grid = p->n_envs < 1024 ? p->n_envs : 1024;
  hipLaunchKernelGGL(k_draw, dim3(grid), dim3(kWave), 0, s, *p, A, T, 1, ids, (const int32_t*)nullptr,
                     (const double*)nullptr, count);
  return launch_status();
}

int sacenv_boat_reset_explicit(const SacenvBoatParams* p, void* arena, const int32_t* ids, int32_t n_ids,
                               const int32_t* start_y, const double* knots, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (p->autoreset) return SACENV_E_MODE;
  if (arena == nullptr || ids == nullptr || start_y == nullptr) return SACENV_E_NULL;
  if (n_curves(p->experiment) > 0 && !p->use_wind_table && knots == nullptr) return SACENV_E_NULL;
  if (n_ids < 0) return SACENV_E_SIZE;
  if (n_ids == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_draw, dim3(n_ids), dim3(kWave), 0, (hipStream_t)stream, *p, make_arena(*p, arena),
                     make_tail(*p, arena), 2, ids, start_y, knots, (const int32_t*)nullptr);
  return launch_status();
}

// the step kernels' wind kind and t rule (owner_wave's template arguments)
static int owner_curves(const SacenvBoatParams& p) { return p.use_wind_table ? 0 : n_curves(p.experiment); }
#define SACENV_OWNER_DISPATCH(p, LAUNCH)                                  \
  switch (owner_curves(p) * 2 + (t_from_index((p).dt) ? 1 : 0)) {         \
    case 0: LAUNCH(0, false); break;                                      \
    case 1: LAUNCH(0, true); break;                                       \
    case 2: LAUNCH(1, false); break;                                      \
    case 3: LAUNCH(1, true); break;                                       \
    case 4: LAUNCH(2, false); break;                                      \
    default: LAUNCH(2, true); break;                                      \
  }

static int boat_step(const SacenvBoatParams* p, void* arena, const float* action, char* trans, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr || action == nullptr) return SACENV_E_NULL;
  const int nb_boat = (int)(pad64(p->n_envs) / kWave);
#define SACENV_LAUNCH(NC, TI)                                                                         \
  hipLaunchKernelGGL((k_step<false, NC, TI>), dim3(nb_boat), dim3(kWave), 0, (hipStream_t)stream, *p, \
                     make_arena(*p, arena), make_tail(*p, arena), action, nb_boat, MixedToys{}, trans)
  SACENV_OWNER_DISPATCH(*p, SACENV_LAUNCH)
#undef SACENV_LAUNCH
  return launch_status();
}

int sacenv_boat_step(const SacenvBoatParams* p, void* arena, const float* action, void* stream) {
  return boat_step(p, arena, action, nullptr, stream);
}

int sacenv_boat_step_pooled(const SacenvBoatParams* p, void* arena, const float* action, void* trans,
                            void* stream) {
  if (trans == nullptr) return SACENV_E_NULL;
  if ((reinterpret_cast<uintptr_t>(trans) & 15u) != 0u) return SACENV_E_RANGE;  // float4 row stores
  return boat_step(p, arena, action, static_cast<char*>(trans), stream);
}

// k_rollout for the launch's wind kind and t rule
// More owner waves than the device has SIMDs: the two-waves-per-SIMD
// instantiation (k_rollout_dense), which keeps every owner wave resident.
static bool dense_grid(int nb_boat) {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return false;
  return nb_boat > 4 * cus;
}

static int launch_multi(const SacenvBoatParams& p, void* arena, const float* actions, int n_steps, const RollArgs& ra,
                        void* stream) {
  const int nb_boat = (int)(pad64(p.n_envs) / kWave);
  const bool dense = dense_grid(nb_boat);
#define SACENV_LAUNCH_K(KER, NC, TI)                                                                       \
  if (ra.stage != nullptr)                                                                                 \
    hipLaunchKernelGGL((KER<NC, TI, 2>), dim3(nb_boat), dim3(kWave), 0, (hipStream_t)stream, p,            \
                       make_arena(p, arena), make_tail(p, arena), actions, n_steps, ra);                   \
  else if (ra.trans != nullptr)                                                                            \
    hipLaunchKernelGGL((KER<NC, TI, 1>), dim3(nb_boat), dim3(kWave), 0, (hipStream_t)stream, p,            \
                       make_arena(p, arena), make_tail(p, arena), actions, n_steps, ra);                   \
  else if (ra.rec_stride != 0)                                                                             \
    hipLaunchKernelGGL((KER<NC, TI, 3>), dim3(nb_boat), dim3(kWave), 0, (hipStream_t)stream, p,            \
                       make_arena(p, arena), make_tail(p, arena), actions, n_steps, ra);                   \
  else                                                                                                     \
    hipLaunchKernelGGL((KER<NC, TI, 0>), dim3(nb_boat), dim3(kWave), 0, (hipStream_t)stream, p,            \
                       make_arena(p, arena), make_tail(p, arena), actions, n_steps, ra)
#define SACENV_LAUNCH(NC, TI)                  \
  if (dense) {                                 \
    SACENV_LAUNCH_K(k_rollout_dense, NC, TI);  \
  } else {                                     \
    SACENV_LAUNCH_K(k_rollout, NC, TI);        \
  }
  SACENV_OWNER_DISPATCH(p, SACENV_LAUNCH)
#undef SACENV_LAUNCH
#undef SACENV_LAUNCH_K
  return launch_status();
}

// byte offsets of the record and the status words in the arena
static int64_t A_ur_bytes(const SacenvBoatParams& p) {
  SacenvBoatLayout L;
  compute_layout(p.n_envs, p.n_knots, p.wind_len, p.use_wind_table, (p.out_flags & SACENV_OUT_KNOTS) != 0, &L);
  return L.record;
}
static int64_t status_offset(const SacenvBoatParams& p) {
  SacenvBoatLayout L;
  compute_layout(p.n_envs, p.n_knots, p.wind_len, p.use_wind_table, (p.out_flags & SACENV_OUT_KNOTS) != 0, &L);
  return L.status;
}

int sacenv_boat_rollout(const SacenvBoatParams* p, void* arena, const float* actions, int32_t n_steps,
                        void* records, float* final_obs, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr || actions == nullptr || records == nullptr) return SACENV_E_NULL;
  if (n_steps < 1 || (p->autoreset && n_steps > SACENV_REFILL_PERIOD)) return SACENV_E_SIZE;
  const int64_t np = pad64(p->n_envs);
  RollArgs ra{};
  ra.rec = static_cast<char*>(records);
  ra.rec_stride = 50 * np;
  ra.fin = final_obs;
  ra.fin_stride = np * SACENV_OBS_DIM;
  ra.act_stride = p->n_envs;
  return launch_multi(*p, arena, actions, n_steps, ra, stream);
}

int sacenv_boat_segment(const SacenvBoatParams* p, void* arena, const float* actions, int64_t action_stride,
                        int32_t n_steps, const uint32_t* act_ready, uint32_t* step_done, uint32_t seq0,
                        void* trans, int64_t trans_stride, void* stage, uint64_t* stage_marks,
                        void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr || actions == nullptr) return SACENV_E_NULL;
  if (n_steps < 1 || (p->autoreset && n_steps > SACENV_REFILL_PERIOD)) return SACENV_E_SIZE;
  if (action_stride < p->n_envs ||
      ((act_ready != nullptr || step_done != nullptr) && (uint64_t)seq0 + (uint64_t)n_steps >= 0x80000000ull))
    return SACENV_E_RANGE;
  if (trans != nullptr && ((reinterpret_cast<uintptr_t>(trans) & 15u) != 0u || (trans_stride & 15) != 0))
    return SACENV_E_RANGE;  // float4 row stores
  if (stage != nullptr && (trans != nullptr || (reinterpret_cast<uintptr_t>(stage) & 15u) != 0u))
    return SACENV_E_RANGE;  // one kind of rows per launch; float4 stores
  // the marks are staged into the wave's LDS (OwnerLds::mk: one word per step, REFILL_PERIOD
  // entries), whatever the autoreset setting
  if (stage_marks != nullptr && n_steps > SACENV_REFILL_PERIOD) return SACENV_E_SIZE;
  const Arena A = make_arena(*p, arena);
  RollArgs ra{};
  ra.rec = static_cast<char*>(arena) + A_ur_bytes(*p);
  ra.rec_stride = 0;
  ra.fin = reinterpret_cast<float*>(static_cast<char*>(arena) + A_ur_bytes(*p) + 50 * A.np);
  ra.fin_stride = 0;
  ra.trans = static_cast<char*>(trans);
  ra.trans_stride = trans_stride;
  ra.stage = static_cast<char*>(stage);
  ra.marks = reinterpret_cast<unsigned long long*>(stage_marks);
  ra.act_stride = action_stride;
  ra.ready = act_ready;
  ra.done = step_done;
  ra.seq0 = seq0;
  ra.status = reinterpret_cast<int32_t*>(static_cast<char*>(arena) + status_offset(*p)) + 1;
  return launch_multi(*p, arena, actions, n_steps, ra, stream);
}

// The segment launch's kernel resources for these params, for the closed
// loop's co-residency plan (sacenv.h): resident one-wave workgroups per CU
// (hipOccupancyMaxActiveBlocksPerMultiprocessor), the grid, VGPRs per lane as
// allocated and LDS bytes per workgroup (hipFuncGetAttributes).
int sacenv_boat_segment_occupancy(const SacenvBoatParams* p, int32_t with_trans, int32_t* blocks_per_cu,
                                  int32_t* grid, int32_t* vgprs, int32_t* lds_bytes) {
  int rc = check_params(p);
  if (rc) return rc;
  if (blocks_per_cu == nullptr || grid == nullptr || vgprs == nullptr || lds_bytes == nullptr) return SACENV_E_NULL;
  int nb = 0;
  hipError_t e = hipSuccess;
  hipFuncAttributes fa{};
  const bool dense = dense_grid((int)(pad64(p->n_envs) / kWave));  // the kernel launch_multi would pick
#define SACENV_OCC_K(KER, NC, TI)                                                                            \
  if (with_trans == 2) {                                                                                     \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, KER<NC, TI, 2>, kWave, 0);                         \
    if (e == hipSuccess) e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(KER<NC, TI, 2>));       \
  } else if (with_trans) {                                                                                   \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, KER<NC, TI, 1>, kWave, 0);                         \
    if (e == hipSuccess) e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(KER<NC, TI, 1>));       \
  } else {                                                                                                   \
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, KER<NC, TI, 0>, kWave, 0);                         \
    if (e == hipSuccess) e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(KER<NC, TI, 0>));       \
  }
#define SACENV_OCC(NC, TI)                  \
  if (dense) {                              \
    SACENV_OCC_K(k_rollout_dense, NC, TI);  \
  } else {                                  \
    SACENV_OCC_K(k_rollout, NC, TI);        \
  }
  SACENV_OWNER_DISPATCH(*p, SACENV_OCC)
#undef SACENV_OCC
#undef SACENV_OCC_K
  if (e != hipSuccess) return (int)e;
  *blocks_per_cu = nb;
  *grid = (int32_t)(pad64(p->n_envs) / kWave);
  *vgprs = fa.numRegs;
  *lds_bytes = (int32_t)fa.sharedSizeBytes;
  return SACENV_OK;
}

int sacenv_boat_refill(const SacenvBoatParams* p, void* arena, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  if (!p->autoreset) return SACENV_E_MODE;
  const Arena A = make_arena(*p, arena);
  const unsigned mask_blocks = (unsigned)((A.np / kWave + kMaskThreads / kWave - 1) / (kMaskThreads / kWave));
  hipLaunchKernelGGL(k_need_masks, dim3(mask_blocks), dim3(kMaskThreads), 0, (hipStream_t)stream, *p, A);
  if ((rc = launch_status())) return rc;
  hipLaunchKernelGGL(k_refill, dim3(p->n_helpers), dim3(kWave), 0, (hipStream_t)stream, *p, A);
  if ((rc = launch_status())) return rc;
  // the fit's item count (episodes drawn x curves) is on the device: a grid
  // that covers a typical refill in one pass (8 groups per block: 65 536
  // (episode, curve) items), grid-stride beyond it; blocks past the count exit
  // at once. Measured 0.12 us/step better than one block per owner wave.
  // (+ the twist-ahead workgroups first, np / kAheadEnvs: measured ahead of
  // twisting in the fit blocks, before or after their fits)
  const int fit_blocks = 8192 + (int)(A.np / kAheadEnvs);
  const Tail T = make_tail(*p, arena);
  if (p->n_knots == 8)
    hipLaunchKernelGGL((k_refill_fit<8, true>), dim3(fit_blocks), dim3(kWave), 0, (hipStream_t)stream, *p, A, T);
  else if (p->n_knots < 8)
    hipLaunchKernelGGL((k_refill_fit<8, false>), dim3(fit_blocks), dim3(kWave), 0, (hipStream_t)stream, *p, A, T);
  else if (p->n_knots == 16)
    hipLaunchKernelGGL((k_refill_fit<16, true>), dim3(fit_blocks), dim3(kWave), 0, (hipStream_t)stream, *p, A, T);
  else
    hipLaunchKernelGGL((k_refill_fit<16, false>), dim3(fit_blocks), dim3(kWave), 0, (hipStream_t)stream, *p, A,
                       T);
  return launch_status();
}

int sacenv_toy_layout(const SacenvToyParams* p, SacenvToyLayout* out) {
  const int rc = check_toy(p);
  if (rc) return rc;
  if (out == nullptr) return SACENV_E_NULL;
  toy_layout(p->n_envs, out);
  return SACENV_OK;
}

int sacenv_toy_init(const SacenvToyParams* p, void* arena, void* stream) {
  const int rc = check_toy(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  hipLaunchKernelGGL(k_toy_init, dim3(blocks_for(p->n_envs, kWave)), dim3(kWave), 0, (hipStream_t)stream, *p,
                     make_toy_arena(*p, arena), (const int32_t*)nullptr, p->n_envs, 1);
  return launch_status();
}

int sacenv_toy_reset(const SacenvToyParams* p, void* arena, const int32_t* ids, int32_t n_ids, void* stream) {
  const int rc = check_toy(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  const int n = ids != nullptr ? n_ids : p->n_envs;
  if (n < 0) return SACENV_E_SIZE;
  if (n == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_toy_init, dim3(blocks_for(n, kWave)), dim3(kWave), 0, (hipStream_t)stream, *p,
                     make_toy_arena(*p, arena), ids, n, 0);
  return launch_status();
}

int sacenv_toy_step(const SacenvToyParams* p, void* arena, void* stream) {
  const int rc = check_toy(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  hipLaunchKernelGGL(k_toy_step, dim3(blocks_for(p->n_envs, kWave)), dim3(kWave), 0, (hipStream_t)stream, *p,
                     make_toy_arena(*p, arena));
  return launch_status();
}

static int mixed_step(const SacenvBoatParams* bp, void* boat_arena, const float* boat_action,
                      const SacenvToyParams* toy_params, void* const* toy_arenas, int32_t n_toys,
                      char* trans, void* stream) {
  int rc;
  if (n_toys < 0 || n_toys > 2) return SACENV_E_SIZE;
  if (n_toys > 0 && (toy_params == nullptr || toy_arenas == nullptr)) return SACENV_E_NULL;
  MixedToys M{};
  M.n = n_toys;
  int nb = 0;
  for (int t = 0; t < n_toys; ++t) {
    if ((rc = check_toy(&toy_params[t]))) return rc;
    if (toy_arenas[t] == nullptr) return SACENV_E_NULL;
    M.p[t] = toy_params[t];
    M.a[t] = make_toy_arena(toy_params[t], toy_arenas[t]);
    M.nb[t] = blocks_for(toy_params[t].n_envs, kWave);
    nb += M.nb[t];
  }
  SacenvBoatParams p{};
  Arena A{};
  Tail T{};
  int nb_boat = 0;
  if (bp != nullptr) {
    if ((rc = check_params(bp))) return rc;
    if (boat_arena == nullptr || boat_action == nullptr) return SACENV_E_NULL;
    p = *bp;
    A = make_arena(p, boat_arena);
    T = make_tail(p, boat_arena);
    nb_boat = (int)(pad64(p.n_envs) / kWave);
    nb += nb_boat;
  }
  if (nb == 0) return SACENV_OK;
#define SACENV_LAUNCH(NC, TI) \
  hipLaunchKernelGGL((k_step<true, NC, TI>), dim3(nb), dim3(kWave), 0, (hipStream_t)stream, p, A, T, boat_action, nb_boat, M, trans)
  SACENV_OWNER_DISPATCH(p, SACENV_LAUNCH)
#undef SACENV_LAUNCH
  return launch_status();
}

int sacenv_mixed_step(const SacenvBoatParams* bp, void* boat_arena, const float* boat_action,
                      const SacenvToyParams* toy_params, void* const* toy_arenas, int32_t n_toys,
                      void* stream) {
  return mixed_step(bp, boat_arena, boat_action, toy_params, toy_arenas, n_toys, nullptr, stream);
}

int sacenv_mixed_step_pooled(const SacenvBoatParams* bp, void* boat_arena, const float* boat_action,
                             const SacenvToyParams* toy_params, void* const* toy_arenas, int32_t n_toys,
                             void* trans, void* stream) {
  if (bp == nullptr || trans == nullptr) return SACENV_E_NULL;
  if ((reinterpret_cast<uintptr_t>(trans) & 15u) != 0u) return SACENV_E_RANGE;
  return mixed_step(bp, boat_arena, boat_action, toy_params, toy_arenas, n_toys, static_cast<char*>(trans),
                    stream);
}

int sacenv_mixed_segment(const SacenvBoatParams* bp, void* boat_arena, const float* boat_actions,
                         int64_t action_stride, int32_t n_steps, const SacenvToyParams* toy_params,
                         void* const* toy_arenas, int32_t n_toys, void* stream) {
  int rc;
  if (n_toys < 0 || n_toys > 2) return SACENV_E_SIZE;
  if (n_toys > 0 && (toy_params == nullptr || toy_arenas == nullptr)) return SACENV_E_NULL;
  if (n_steps < 1) return SACENV_E_SIZE;
  MixedToys M{};
  M.n = n_toys;
  int nb = 0;
  for (int t = 0; t < n_toys; ++t) {
    if ((rc = check_toy(&toy_params[t]))) return rc;
    if (toy_arenas[t] == nullptr) return SACENV_E_NULL;
    M.p[t] = toy_params[t];
    M.a[t] = make_toy_arena(toy_params[t], toy_arenas[t]);
    M.nb[t] = blocks_for(toy_params[t].n_envs, kWave);
    nb += M.nb[t];
  }
  SacenvBoatParams p{};
  Arena A{};
  Tail T{};
  RollArgs ra{};
  int nb_boat = 0;
  if (bp != nullptr) {
    if ((rc = check_params(bp))) return rc;
    if (boat_arena == nullptr || boat_actions == nullptr) return SACENV_E_NULL;
    if (bp->autoreset && n_steps > SACENV_REFILL_PERIOD) return SACENV_E_SIZE;
    if (action_stride < bp->n_envs) return SACENV_E_RANGE;
    p = *bp;
    A = make_arena(p, boat_arena);
    T = make_tail(p, boat_arena);
    ra.rec = static_cast<char*>(boat_arena) + A_ur_bytes(p);
    ra.rec_stride = 0;
    ra.fin = reinterpret_cast<float*>(static_cast<char*>(boat_arena) + A_ur_bytes(p) + 50 * A.np);
    ra.fin_stride = 0;
    ra.act_stride = action_stride;
    ra.status = reinterpret_cast<int32_t*>(static_cast<char*>(boat_arena) + status_offset(p)) + 1;
    nb_boat = (int)(pad64(p.n_envs) / kWave);
    nb += nb_boat;
  }
  if (nb == 0) return SACENV_OK;
#define SACENV_LAUNCH(NC, TI)                                                                                  \
  hipLaunchKernelGGL((k_rollout_mixed<NC, TI>), dim3(nb), dim3(kWave), 0, (hipStream_t)stream, p, A, T,        \
                     boat_actions, n_steps, ra, nb_boat, M)
  SACENV_OWNER_DISPATCH(p, SACENV_LAUNCH)
#undef SACENV_LAUNCH
  return launch_status();
}

int sacenv_boat_wind_eval(const SacenvBoatParams* p, const void* arena, const int32_t* env_ids,
                          const int32_t* idx, int32_t n, double* out_velocity, double* out_angle,
                          void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if (!arena || !env_ids || !idx || !out_velocity || !out_angle) return SACENV_E_NULL;
  if (n < 0) return SACENV_E_SIZE;
  if (n == 0) return SACENV_OK;
  void* a = const_cast<void*>(arena);
  hipLaunchKernelGGL(k_wind_eval, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, *p,
                     make_arena(*p, a), make_tail(*p, a), env_ids, idx, n, out_velocity, out_angle);
  return launch_status();
}

}  // extern "C"
