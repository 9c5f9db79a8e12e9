// sacenv_boat.hip — gfx950 kernels + C ABI for the vectorised boat env.
//
// One wave64 workgroup owns 64 consecutive envs. Per step each lane runs one
// env's BoatEnv.step (boat_env.py:67-115) on float64 SoA state; envs that end
// are then reset by the WHOLE wave, one env at a time (Boat.__init__,
// boat_env.py:144-201): the per-env MT19937 twist, the randint rejection
// loop, the knot draws and the not-a-knot spline's grid min/max are spread
// across the 64 lanes, so a reset costs a few hundred cycles instead of the
// 10 000-sample scan the reference does (wind.py:80-89).
//
// Floating-point order follows the reference expression by expression
// (left-to-right products, no FMA contraction: -ffp-contract=off), so the
// only differences from the CPU step are the libm/ocml transcendentals.

#include <hip/hip_runtime.h>
#include <stdint.h>

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
constexpr double kPi = 3.141592653589793;  // np.pi

struct ResetLds {
  uint32_t blk[2][kMtN];          // current MT block, next (twisted) block
  double y[2][kMaxK];             // knot values per curve (unfolded)
  double m[2][kMaxK];             // second derivatives / 6 per curve (unfolded)
};

// ---------------------------------------------------------------- MT19937
// numpy legacy RandomState (numpy/random/src/mt19937), pinned numpy 1.23.5.

__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
  y ^= (y >> 11);
  y ^= (y << 7) & 0x9d2c5680u;
  y ^= (y << 15) & 0xefc60000u;
  y ^= (y >> 18);
  return y;
}

__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t c) {
  const uint32_t y = (a & kMtUpper) | (b & kMtLower);
  return c ^ (y >> 1) ^ ((y & 1u) ? kMtMatrixA : 0u);
}

// mt19937_gen as four lane-parallel phases: word i depends on old[i],
// old[i+1] and either old[i+397] (i < 227) or new[i-227].
__device__ void mt_twist_wave(const uint32_t* __restrict__ o, uint32_t* __restrict__ n, int lane) {
  for (int i = lane; i < kMtN - kMtM; i += kWave) n[i] = mt_mix(o[i], o[i + 1], o[i + kMtM]);
  __syncthreads();
  for (int i = (kMtN - kMtM) + lane; i < 2 * (kMtN - kMtM); i += kWave)
    n[i] = mt_mix(o[i], o[i + 1], n[i - (kMtN - kMtM)]);
  __syncthreads();
  for (int i = 2 * (kMtN - kMtM) + lane; i < kMtN - 1; i += kWave)
    n[i] = mt_mix(o[i], o[i + 1], n[i - (kMtN - kMtM)]);
  __syncthreads();
  if (lane == 0) n[kMtN - 1] = mt_mix(o[kMtN - 1], n[0], n[kMtM - 1]);
  __syncthreads();
}

// Wave-uniform view of one env's MT19937 stream. Words are handed out 64 at
// a time (lane k sees word pos+k); the 2.5 KB block is staged in LDS only
// when a window crosses the block end.
struct MtStream {
  uint32_t* gkey;
  int pos;        // offset of the next unconsumed word in the current block
  int cur;        // which ResetLds::blk holds the current block (when loaded)
  bool loaded;
  bool nxt_valid;
  bool advanced;  // current block differs from gkey
};

__device__ uint32_t mt_fetch(MtStream& st, ResetLds& l, int lane) {
  if (!st.loaded) {
    if (st.pos + kWave <= kMtN) return mt_temper(st.gkey[st.pos + lane]);
    for (int i = lane; i < kMtN; i += kWave) l.blk[0][i] = st.gkey[i];
    __syncthreads();
    st.loaded = true;
    st.cur = 0;
    st.nxt_valid = false;
  }
  while (st.pos >= kMtN) {
    if (!st.nxt_valid) mt_twist_wave(l.blk[st.cur], l.blk[st.cur ^ 1], lane);
    st.cur ^= 1;
    st.pos -= kMtN;
    st.nxt_valid = false;
    st.advanced = true;
  }
  if (st.pos + kWave > kMtN && !st.nxt_valid) {
    mt_twist_wave(l.blk[st.cur], l.blk[st.cur ^ 1], lane);
    st.nxt_valid = true;
  }
  const int i = st.pos + lane;
  const uint32_t w = (i < kMtN) ? l.blk[st.cur][i] : l.blk[st.cur ^ 1][i - kMtN];
  return mt_temper(w);
}

__device__ void mt_finish(MtStream& st, ResetLds& l, int32_t* gpos, int lane) {
  // words consumed past the block end came from the twisted block: make it current
  while (st.loaded && (st.pos > kMtN || (st.pos == kMtN && st.nxt_valid))) {
    if (!st.nxt_valid) mt_twist_wave(l.blk[st.cur], l.blk[st.cur ^ 1], lane);
    st.cur ^= 1;
    st.pos -= kMtN;
    st.nxt_valid = false;
    st.advanced = true;
  }
  if (st.loaded && st.advanced)
    for (int i = lane; i < kMtN; i += kWave) st.gkey[i] = l.blk[st.cur][i];
  if (lane == 0) *gpos = st.pos;
}

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

__device__ __forceinline__ double curve_lds(const SacenvBoatParams& p, const ResetLds& l, int c, int i) {
  const Knot k = knot_coord(p, i);
  return spline_piece(l.y[c][k.j], l.y[c][k.j + 1], l.m[c][k.j], l.m[c][k.j + 1], k.t);
}

__device__ __forceinline__ double curve_env(const SacenvBoatParams& p, const SacenvBoatState& s,
                                            int c, int e, int i) {
  const Knot k = knot_coord(p, i);
  const size_t n = (size_t)p.n_envs;
  const size_t base = ((size_t)c * p.n_knots + k.j) * n + e;
  return spline_piece(s.wind_y[base], s.wind_y[base + n], s.wind_m[base], s.wind_m[base + n], k.t);
}

__host__ __device__ __forceinline__ int n_curves(int experiment) {
  return experiment == 6 ? 2 : (experiment == 4 || experiment == 5) ? 1 : 0;
}

// Wind.get_wind(index) (wind.py:20-24) for the tables of wind.py:26-99.
__device__ __forceinline__ void wind_at(const SacenvBoatParams& p, const SacenvBoatState& s, int e,
                                        int idx, double& wv, double& wa) {
  if (idx > p.wind_len - 1) idx = p.wind_len - 1;  // reference: IndexError
  if (idx < 0) idx = 0;
  if (p.wind_table != nullptr) {
    wv = p.wind_table[idx];
    wa = p.wind_table[p.wind_len + idx];
    return;
  }
  switch (p.experiment) {
    case 3:
      wv = p.max_velocity;
      wa = p.wind_dir_rad;
      return;
    case 4:
      wv = curve_env(p, s, 0, e, idx);
      wa = p.wind_dir_rad;
      return;
    case 5: {
      wv = p.max_velocity;
      const double r = curve_env(p, s, 0, e, idx) <= 0.5 / 2 ? 0.0 : 1.0;  // wind.py:92-99
      wa = (r * kPi) + kPi / 2;
      return;
    }
    case 6:
      wv = curve_env(p, s, 0, e, idx);
      wa = curve_env(p, s, 1, e, idx);
      return;
    default:  // 1, 2: no wind
      wv = 0.0;
      wa = 0.0;
      return;
  }
}

// ---------------------------------------------------------------- observation

__device__ __forceinline__ double norm(const SacenvBoatParams& p, int k, double v) {
  return (v - p.obs_lo[k]) / (p.obs_hi[k] - p.obs_lo[k]);  // Boat.normalize, :325-326
}

struct Obs {
  float v[SACENV_OBS_DIM];
};

__device__ __forceinline__ Obs make_obs(const SacenvBoatParams& p, double s_x, double v_x, double a_x,
                                        double s_y, double v_y, double a_y, double s_r, double v_r,
                                        double a_r, double rudder, double fuel) {
  Obs o;
  o.v[0] = (float)norm(p, 0, s_x);
  o.v[1] = (float)norm(p, 1, v_x);
  o.v[2] = (float)norm(p, 2, a_x);
  o.v[3] = (float)norm(p, 3, s_y);
  o.v[4] = (float)norm(p, 4, v_y);
  o.v[5] = (float)norm(p, 5, a_y);
  o.v[6] = (float)norm(p, 6, s_r);
  o.v[7] = (float)norm(p, 7, v_r);
  o.v[8] = (float)norm(p, 8, a_r);
  o.v[9] = (float)norm(p, 9, rudder);
  o.v[10] = (float)norm(p, 10, fuel);
  return o;
}

__device__ __forceinline__ void store_obs(float* dst, const Obs& o) {
#pragma unroll
  for (int k = 0; k < SACENV_OBS_DIM; ++k) dst[k] = o.v[k];
}

// ---------------------------------------------------------------- reset

__device__ __forceinline__ double wave_min16(double v) {
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) v = fmin(v, __shfl_xor(v, off));
  return v;
}
__device__ __forceinline__ double wave_max16(double v) {
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) v = fmax(v, __shfl_xor(v, off));
  return v;
}

// Grid-sample min/max of one spline interval: the cubic is monotone between
// its critical points, so the extreme grid samples of interval j are its
// first/last grid points and the neighbours of each critical point.
__device__ void interval_extrema(const SacenvBoatParams& p, const ResetLds& l, int c, int j,
                                 double& mn, double& mx) {
  mn = INFINITY;
  mx = -INFINITY;
  const int L = p.wind_len;
  const double inv = 1.0 / p.knot_step;
  int lo = (int)ceil((double)j * inv) - 2;
  if (lo < 0) lo = 0;
  while (lo < L && knot_coord(p, lo).j < j) ++lo;
  int hi = (int)floor((double)(j + 1) * inv) + 2;
  if (hi > L - 1) hi = L - 1;
  while (hi >= 0 && knot_coord(p, hi).j > j) --hi;
  if (lo > hi) return;
  int cand[10];
  int nc = 0;
  cand[nc++] = lo;
  cand[nc++] = hi;
  const double a = l.m[c][j], b = l.m[c][j + 1];
  const double y0 = l.y[c][j], y1 = l.y[c][j + 1];
  const double qa = 3.0 * (b - a), qb = 6.0 * a, qc = y1 - y0 - 2.0 * a - b;
  double roots[2];
  int nr = 0;
  const double scale = fabs(qa) + fabs(qb) + fabs(qc);
  if (fabs(qa) <= 1e-14 * scale) {
    if (qb != 0.0) roots[nr++] = -qc / qb;
  } else {
    const double disc = qb * qb - 4.0 * qa * qc;
    if (disc >= 0.0) {
      const double sq = sqrt(disc);
      const double q = -0.5 * (qb + (qb >= 0.0 ? sq : -sq));
      roots[nr++] = q / qa;
      if (q != 0.0) roots[nr++] = qc / q;
    }
  }
  for (int r = 0; r < nr; ++r) {
    const double tr = roots[r];
    if (!(tr > -0.01 && tr < 1.01)) continue;
    const double ic = ((double)j + tr) * inv;
    const int i0 = (int)floor(ic);
    for (int d = -1; d <= 2; ++d) {
      int i = i0 + d;
      i = i < lo ? lo : (i > hi ? hi : i);
      cand[nc++] = i;
    }
  }
  for (int q = 0; q < nc; ++q) {
    const double v = curve_lds(p, l, c, cand[q]);
    mn = fmin(mn, v);
    mx = fmax(mx, v);
  }
}

// Boat(config) for env `e`, executed by all 64 lanes of the wave (e uniform).
// Draws (unless explicit) in the reference order: randint (boat_env.py:147),
// then 8 knot values per random curve (wind.py:78; velocity first in exp 6).
// Writes the wind coefficients and the RNG state; returns start_y in all
// lanes. The caller writes the scalar state and the obs row.
__device__ int32_t reset_env_wave(const SacenvBoatParams& p, const SacenvBoatState& s, ResetLds& l,
                                  int e, int lane, const int32_t* ex_start_y,
                                  const double* ex_knots) {
  const int nk = p.n_knots;
  // draws follow the reference even when a recorded wind table overrides the
  // curves; only the spline fit is skipped then
  const int ndraw = n_curves(p.experiment);
  const int ncurves = p.wind_table != nullptr ? 0 : ndraw;
  int32_t start_y;
  if (ex_start_y != nullptr) {
    start_y = *ex_start_y;
    for (int c = 0; c < ncurves; ++c)
      if (lane < nk) l.y[c][lane] = ex_knots[c * nk + lane];
  } else {
    MtStream st;
    st.gkey = s.mt_key + (size_t)e * kMtN;
    st.pos = s.mt_pos[e];
    st.cur = 0;
    st.loaded = false;
    st.nxt_valid = false;
    st.advanced = false;
    // np.random.randint(-hw, hw): masked rejection on 32-bit words
    // (numpy random_bounded_uint64_fill -> buffered_bounded_masked_uint32).
    const uint32_t rng = (uint32_t)(2 * p.start_y_half - 1);
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    uint32_t val = 0;
    for (;;) {
      const uint32_t w = mt_fetch(st, l, lane);
      const unsigned long long acc = __ballot((w & mask) <= rng);
      if (acc) {
        const int k = __ffsll((long long)acc) - 1;
        val = (uint32_t)__shfl((int)w, k) & mask;
        st.pos += k + 1;
        break;
      }
      st.pos += kWave;
    }
    start_y = -p.start_y_half + (int32_t)val;
    // np.random.sample(n): legacy_double = genrand_res53 on two words.
    for (int c = 0; c < ndraw; ++c) {
      const uint32_t w = mt_fetch(st, l, lane);
      const int src = (2 * lane) & (kWave - 1);
      const uint32_t wa = (uint32_t)__shfl((int)w, src);
      const uint32_t wb = (uint32_t)__shfl((int)w, src + 1);
      if (lane < nk) {
        const double a = (double)(wa >> 5), b = (double)(wb >> 6);
        l.y[c][lane] = (a * 67108864.0 + b) / 9007199254740992.0;
      }
      st.pos += 2 * nk;
    }
    mt_finish(st, l, s.mt_pos + e, lane);
  }
  if (ncurves > 0) {
    __syncthreads();
    const size_t n = (size_t)p.n_envs;
    // second derivatives / 6 of the not-a-knot spline: m = G @ y
    for (int c = 0; c < ncurves; ++c) {
      if (lane < nk) {
        double acc = 0.0;
        for (int k = 0; k < nk; ++k) acc += p.spline_g[lane * nk + k] * l.y[c][k];
        l.m[c][lane] = acc;
        if (s.knots_raw != nullptr) s.knots_raw[((size_t)c * nk + lane) * n + e] = l.y[c][lane];
      }
    }
    __syncthreads();
    // grid min/max per curve: lanes c*16 + j own interval j of curve c
    const int c = lane >> 4, j = lane & 15;
    double mn = INFINITY, mx = -INFINITY;
    if (c < ncurves && j < nk - 1) interval_extrema(p, l, c, j, mn, mx);
    mn = wave_min16(mn);
    mx = wave_max16(mx);
    for (int cc = 0; cc < ncurves; ++cc) {
      const double cmn = __shfl(mn, cc * 16), cmx = __shfl(mx, cc * 16);
      if (lane < nk) {
        double yv = l.y[cc][lane], mv = l.m[cc][lane];
        if (cmn < 0.0 || cmx > 1.0) {  // wind.py:87-89 min-max renormalisation
          const double span = cmx - cmn;
          yv = (yv - cmn) / span;
          mv = mv / span;
        }
        // table scaling of wind.py:86-89: velocity * max_v, angle * pi * 2;
        // exp 5 keeps the unit curve for the rectifier (wind.py:92-99).
        if (p.experiment == 4 || (p.experiment == 6 && cc == 0)) {
          yv = yv * p.max_velocity;
          mv = mv * p.max_velocity;
        } else if (p.experiment == 6 && cc == 1) {
          yv = yv * kPi * 2;
          mv = mv * kPi * 2;
        }
        const size_t o = ((size_t)cc * nk + lane) * n + e;
        s.wind_y[o] = yv;
        s.wind_m[o] = mv;
      }
    }
  }
  return start_y;
}

// scalar state + obs of a fresh Boat (boat_env.py:152-198), written by one lane
__device__ __forceinline__ void write_fresh_state(const SacenvBoatParams& p, const SacenvBoatState& s,
                                                  int e, int32_t start_y, float* obs_row) {
  const double s_y = p.experiment == 2 ? (double)start_y : 0.0;  // :166-169
  s.s_x[e] = 0.0;
  s.s_y[e] = s_y;
  s.s_r[e] = 0.0;
  s.v_x[e] = 0.0;
  s.v_y[e] = 0.0;
  s.v_r[e] = 0.0;
  s.rudder[e] = 0.0;
  s.t[e] = 0.0;
  s.ep_reward[e] = 0.0;  // :122
  s.index[e] = 0;
  s.start_y[e] = start_y;
  if (obs_row != nullptr)
    store_obs(obs_row, make_obs(p, 0.0, 0.0, 0.0, s_y, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, (double)p.fuel0));
}

// ---------------------------------------------------------------- kernels

__global__ void __launch_bounds__(kWave) k_seed(SacenvBoatParams p, SacenvBoatState s,
                                                const uint32_t* __restrict__ seeds) {
  const int e = blockIdx.x * kWave + threadIdx.x;
  if (e >= p.n_envs) return;
  // mt19937_seed (init_genrand), numpy RandomState._legacy_seeding(int)
  uint32_t x = seeds[e];
  uint32_t* key = s.mt_key + (size_t)e * kMtN;
  for (int i = 0; i < kMtN; ++i) {
    key[i] = x;
    x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
  }
  s.mt_pos[e] = kMtN;
}

__global__ void __launch_bounds__(kWave) k_reset(SacenvBoatParams p, SacenvBoatState s,
                                                 const int32_t* __restrict__ ids,
                                                 const int32_t* __restrict__ ex_start_y,
                                                 const double* __restrict__ ex_knots,
                                                 float* __restrict__ obs) {
  __shared__ ResetLds lds;
  const int b = blockIdx.x;
  const int lane = threadIdx.x;
  const int e = ids != nullptr ? ids[b] : b;
  if (e < 0 || e >= p.n_envs) return;  // uniform per block
  const int32_t* sy = ex_start_y != nullptr ? ex_start_y + b : nullptr;
  const double* kn = ex_knots != nullptr ? ex_knots + (size_t)b * 2 * p.n_knots : nullptr;
  const int32_t start_y = reset_env_wave(p, s, lds, e, lane, sy, kn);
  if (lane == 0)
    write_fresh_state(p, s, e, start_y, obs != nullptr ? obs + (size_t)e * SACENV_OBS_DIM : nullptr);
}

__global__ void __launch_bounds__(kWave) k_step(SacenvBoatParams p, SacenvBoatState s,
                                                const float* __restrict__ action,
                                                SacenvBoatStepOut out) {
  __shared__ ResetLds lds;
  const int lane = threadIdx.x;
  const int e = blockIdx.x * kWave + lane;
  const bool active = e < p.n_envs;
  bool ended = false;
  if (active) {
    double s_x = s.s_x[e], s_y = s.s_y[e], s_r = s.s_r[e];
    double v_x = s.v_x[e], v_y = s.v_y[e], v_r = s.v_r[e];
    double rudder = s.rudder[e], t = s.t[e], ep = s.ep_reward[e];
    int32_t index = s.index[e];
    const float act = action[e];
    double wv, wa;
    wind_at(p, s, e, index, wv, wa);

    // BoatEnv.step :69-73
    t = t + p.dt;
    const int32_t fuel = p.fuel0 - (index + 1);
    if (p.test_mode == 0) rudder = rudder + (double)act / 10;
    const bool first = index == 0;  // integrator counter == 0 (control_blocks.py:21-22)
    const double wsign = (double)((wv > 0.0) - (wv < 0.0));
    const double cwa = cos(wa), swa = sin(wa);

    // eom_longitudinal :213-239
    const double F_R = v_x * v_x * p.c_r_front * 0.5 * p.rho * p.boat_area_front;
    const double v_x_w = v_x * (1.0 - p.wake_friction);
    const double nD = p.n_rpm * p.propeller_diameter;
    const double J = p.n_rpm != 0.0 ? v_x_w / nD : 0.0;  // :222-224
    const double D = p.propeller_diameter;
    const double F_T = sin(J) * (p.n_rpm * p.n_rpm) * p.rho * (D * D * D * D) * (1.0 - p.thrust_deduction);
    const double F_C = v_y * (p.boat_m + p.boat_m_y) * v_r;
    const double F_W = (wv * wv * wsign * p.c_r_front * 0.5 * p.rho * p.boat_area_front) * cwa;
    const double a_x = (-F_R + F_T + F_C + F_W) / (p.boat_m + p.boat_m_x);
    v_x = first ? 3.0 : a_x * p.dt + v_x;

    // eom_transverse :241-265 (new v_x)
    const double vys = (double)((v_y > 0.0) - (v_y < 0.0));
    const double F_R2 = v_y * v_y * p.c_r_side * 0.5 * p.rho * p.boat_area_side * vys;
    const double sin_rud = sin(rudder);
    const double F_RU = sin_rud * (v_x * v_x * p.c_r_front * 0.5 * p.rho * p.rudder_area);
    const double F_C2 = v_x * (p.boat_m + p.boat_m_x) * v_r;
    const double F_W2 = (wv * wv * wsign * p.c_r_side * 0.5 * p.rho * p.boat_area_side) * swa;
    const double a_y = (-F_R2 + F_RU + F_C2 + F_W2) / (p.boat_m + p.boat_m_y);
    v_y = first ? 0.0 : a_y * p.dt + v_y;

    // eom_yawning :267-281
    const double vrs = (double)((v_r > 0.0) - (v_r < 0.0));
    const double vxs = (double)((v_x > 0.0) - (v_x < 0.0));
    const double M_hull = v_r * v_r * p.c_r_side * 0.5 * p.rho * p.boat_area_side * p.boat_l * 5.0 * vrs;
    const double M_rud = v_x * v_x * p.c_r_side * 0.5 * p.rho * p.rudder_area * sin_rud * (p.boat_b / 2) * vxs;
    const double a_r = (-M_hull + M_rud) / (p.boat_I + p.boat_Iz);
    v_r = first ? 0.0 : a_r * p.dt + v_r;

    // get_kinematics :283-306
    const double v = sqrt(v_x * v_x + v_y * v_y);
    const double drift = atan2(v_x, v_y);
    s_r = v_r * p.dt + s_r;
    const double dir = drift - s_r;
    double sd, cd;
    sincos(dir, &sd, &cd);
    s_x = (sd * v) * p.dt + s_x;
    s_y = (cd * v) * p.dt + s_y;
    index = index + 1;

    const Obs o = make_obs(p, s_x, v_x, a_x, s_y, v_y, a_y, s_r, v_r, a_r, rudder, (double)fuel);

    // exponential_reward (reward_functions.py:42-57)
    const double ay = fabs(s_y);
    const double f_y = (ay / p.track_width) / (1.0 + exp(p.reward_k * (ay - p.reward_center)));
    double reward = 0.0 - f_y;

    // termination chain :84-105
    uint8_t term = SACENV_TERM_NONE;
    if (s_x >= p.goal_line) {
      term = SACENV_TERM_REACHED_GOAL;
      reward = reward + 1000.0;
    } else if (fabs(s_y) > p.oob_limit || s_x < 0.0) {
      term = SACENV_TERM_OUT_OF_BOUNDS;
    } else if (fuel < 0) {
      term = SACENV_TERM_OUT_OF_FUEL;
    } else if (p.t_max <= t) {
      term = SACENV_TERM_TIMEOUT;
    } else if (rudder > kPi / 3 || rudder < -kPi / 3) {
      term = SACENV_TERM_RUDDER_BROKEN;
    }
    // penalties :107-111
    if (rudder > kPi / 4 || rudder < -kPi / 4) reward = reward - fabs(rudder) * 100.0;
    if (fabs(s_r) > kPi / 2) reward = reward - 1.0;
    ep = ep + reward;

    if (term != SACENV_TERM_NONE) s.counters[(size_t)(term - 1) * p.n_envs + e] += 1u;
    if (term == SACENV_TERM_NONE && p.max_episode_steps > 0 && index >= p.max_episode_steps)
      term = SACENV_TERM_TRUNCATED;
    ended = term != SACENV_TERM_NONE;

    out.reward[e] = (float)reward;
    out.done[e] = ended ? 1 : 0;
    out.term[e] = term;
    if (out.reward64 != nullptr) out.reward64[e] = reward;
    if (out.accel != nullptr) {
      out.accel[e] = a_x;
      out.accel[(size_t)p.n_envs + e] = a_y;
      out.accel[2 * (size_t)p.n_envs + e] = a_r;
    }
    if (ended && out.final_ep_reward != nullptr) out.final_ep_reward[e] = ep;
    if (ended && p.autoreset) {
      if (out.final_obs != nullptr) store_obs(out.final_obs + (size_t)e * SACENV_OBS_DIM, o);
    } else {
      store_obs(out.obs + (size_t)e * SACENV_OBS_DIM, o);
      s.s_x[e] = s_x;
      s.s_y[e] = s_y;
      s.s_r[e] = s_r;
      s.v_x[e] = v_x;
      s.v_y[e] = v_y;
      s.v_r[e] = v_r;
      s.rudder[e] = rudder;
      s.t[e] = t;
      s.ep_reward[e] = ep;
      s.index[e] = index;
    }
  }
  if (!p.autoreset) return;
  // auto-reset: the whole wave resets each ended env in turn
  unsigned long long pending = __ballot(ended);
  while (pending) {
    const int owner = __ffsll((long long)pending) - 1;
    pending &= pending - 1;
    const int er = blockIdx.x * kWave + owner;
    const int32_t start_y = reset_env_wave(p, s, lds, er, lane, nullptr, nullptr);
    if (lane == owner) write_fresh_state(p, s, er, start_y, out.obs + (size_t)er * SACENV_OBS_DIM);
    __syncthreads();
  }
}

__global__ void __launch_bounds__(256) k_wind_eval(SacenvBoatParams p, SacenvBoatState s,
                                                   const int32_t* __restrict__ env_ids,
                                                   const int32_t* __restrict__ idx, int n,
                                                   double* __restrict__ out_v,
                                                   double* __restrict__ out_a) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int e = env_ids[q];
  if (e < 0 || e >= p.n_envs) return;
  double wv, wa;
  wind_at(p, s, e, idx[q], wv, wa);
  out_v[q] = wv;
  out_a[q] = wa;
}

// ---------------------------------------------------------------- host side

int check_params(const SacenvBoatParams* p) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->experiment < 1 || p->experiment > 6) return SACENV_E_EXPERIMENT;
  if (p->n_envs <= 0 || p->wind_len <= 0) return SACENV_E_SIZE;
  if (n_curves(p->experiment) > 0 && p->wind_table == nullptr) {
    if (p->n_knots < 4 || p->n_knots > kMaxK) return SACENV_E_KNOTS;
    if (p->wind_len < 2) return SACENV_E_SIZE;
    if (p->spline_g == nullptr) return SACENV_E_NULL;
  }
  if (p->start_y_half < 1) return SACENV_E_RANGE;
  return SACENV_OK;
}

int check_state(const SacenvBoatParams* p, const SacenvBoatState* s) {
  if (s == nullptr) return SACENV_E_NULL;
  if (!s->s_x || !s->s_y || !s->s_r || !s->v_x || !s->v_y || !s->v_r || !s->rudder || !s->t ||
      !s->ep_reward || !s->index || !s->start_y || !s->mt_key || !s->mt_pos || !s->counters)
    return SACENV_E_NULL;
  if (n_curves(p->experiment) > 0 && (!s->wind_y || !s->wind_m)) return SACENV_E_NULL;
  return SACENV_OK;
}

int launch_status() {
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? SACENV_OK : (int)err;
}

inline int blocks_for(int n, int per) { return (n + per - 1) / per; }

}  // namespace

extern "C" {

int sacenv_abi_version(void) { return SACENV_ABI_VERSION; }

const char* sacenv_error_string(int code) {
  switch (code) {
    case SACENV_OK: return "ok";
    case SACENV_E_NULL: return "required pointer is NULL";
    case SACENV_E_EXPERIMENT: return "Well someone tried to use an experiment that doesnt exist!";
    case SACENV_E_KNOTS: return "Please select at least 4 fixed_points in your config (max 16).";
    case SACENV_E_SIZE: return "size out of range";
    case SACENV_E_RANGE: return "start-y range empty: int(0.8*track_width) must be >= 1";
    default: return code > 0 ? hipGetErrorString((hipError_t)code) : "unknown sacenv error";
  }
}

int sacenv_boat_seed(const SacenvBoatParams* p, const SacenvBoatState* s, const uint32_t* seeds,
                     void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if ((rc = check_state(p, s))) return rc;
  if (seeds == nullptr) return SACENV_E_NULL;
  hipLaunchKernelGGL(k_seed, dim3(blocks_for(p->n_envs, kWave)), dim3(kWave), 0, (hipStream_t)stream,
                     *p, *s, seeds);
  return launch_status();
}

int sacenv_boat_reset(const SacenvBoatParams* p, const SacenvBoatState* s, const int32_t* ids,
                      int32_t n_ids, float* obs, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if ((rc = check_state(p, s))) return rc;
  const int nb = ids != nullptr ? n_ids : p->n_envs;
  if (nb < 0) return SACENV_E_SIZE;
  if (nb == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_reset, dim3(nb), dim3(kWave), 0, (hipStream_t)stream, *p, *s, ids,
                     (const int32_t*)nullptr, (const double*)nullptr, obs);
  return launch_status();
}

int sacenv_boat_reset_explicit(const SacenvBoatParams* p, const SacenvBoatState* s,
                               const int32_t* ids, int32_t n_ids, const int32_t* start_y,
                               const double* knots, float* obs, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if ((rc = check_state(p, s))) return rc;
  if (ids == nullptr || start_y == nullptr) return SACENV_E_NULL;
  if (n_curves(p->experiment) > 0 && p->wind_table == nullptr && knots == nullptr) return SACENV_E_NULL;
  if (n_ids < 0) return SACENV_E_SIZE;
  if (n_ids == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_reset, dim3(n_ids), dim3(kWave), 0, (hipStream_t)stream, *p, *s, ids, start_y,
                     knots, obs);
  return launch_status();
}

int sacenv_boat_step(const SacenvBoatParams* p, const SacenvBoatState* s, const float* action,
                     const SacenvBoatStepOut* out, void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if ((rc = check_state(p, s))) return rc;
  if (action == nullptr || out == nullptr || !out->obs || !out->reward || !out->done || !out->term)
    return SACENV_E_NULL;
  hipLaunchKernelGGL(k_step, dim3(blocks_for(p->n_envs, kWave)), dim3(kWave), 0, (hipStream_t)stream,
                     *p, *s, action, *out);
  return launch_status();
}

int sacenv_boat_wind_eval(const SacenvBoatParams* p, const SacenvBoatState* s, const int32_t* env_ids,
                          const int32_t* idx, int32_t n, double* out_velocity, double* out_angle,
                          void* stream) {
  int rc = check_params(p);
  if (rc) return rc;
  if ((rc = check_state(p, s))) return rc;
  if (!env_ids || !idx || !out_velocity || !out_angle) return SACENV_E_NULL;
  if (n < 0) return SACENV_E_SIZE;
  if (n == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_wind_eval, dim3(blocks_for(n, 256)), dim3(256), 0, (hipStream_t)stream, *p, *s,
                     env_ids, idx, n, out_velocity, out_angle);
  return launch_status();
}

}  // extern "C"
