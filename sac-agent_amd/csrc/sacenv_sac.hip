// sacenv_sac.hip — the SAC agent on gfx950.
//
// ContinuousAgent.choose_action (agent/continuous_agent.py:57-61) for N
// observations at once, and ContinuousAgent.learn (:96-154) over the five
// networks of networks/networks.py:14-133, as fp32 MFMA kernels
// (v_mfma_f32_16x16x4_f32: f32 in, f32 accumulate, an fmaf chain per output).
//
// learn() in four launches. Every gradient of one learn() is taken at the
// parameters the call starts with: the value step (:121-125) changes only the
// value net, which neither the actor loss nor the critic loss reads; the
// critics step after the actor loss (:127-137 vs :139-150); the value-phase
// gradients that reach actor and critics are zeroed before their own losses
// (:133, :139-140). So the four losses are independent and the kernels run
// them side by side:
//
//   phase 0 (row blocks x 4 roles): actor forward + both policy draws, value
//     forward, critic 1 / 2 forward on the stored actions.
//   phase 1 (x 6): critic c at the rsample() actions with dq/da (actor loss);
//     critic c's own loss backward (target forward for value_, done-masked;
//     q_hat = scale * reward + gamma * value_); critic c at the sample()
//     actions (value target).
//   phase 2 (x 4): actor backward (min of the critics, tanh-squashed Normal
//     log-prob), value backward (value_target = min q - log_prob), each layer
//     split over two workgroups by output features.
//   phase 3: weight gradients as batch reductions (dW = dZ^T H on MFMA), Adam
//     (torch.optim.Adam, foreach form) on the four optimised nets, the target
//     soft update (:63-77), the transposes, and the four losses.
//
// Row blocks are 16 batch rows per 256-thread workgroup. A dense layer of a
// row block is Y^T = W X^T: wave w owns output features [64w, 64w + 64) as
// four 16x16 tiles; the weights are the MFMA A operand straight from L2
// (float4 per lane), the activations the B operand from LDS ([row][feature],
// 4-float pad). k runs in blocks of 16 with lane (i, kq) supplying
// k = 16 kb + 4 kq + s in step s — the same permutation on both operands, so
// each lane reads one float4 of each per block. Activations that phase 3
// reduces over the batch are stored feature-major [256][B].
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "sacenv.h"

namespace {

constexpr int kH = SACENV_SAC_HIDDEN;
constexpr int kRows = 16;      // batch rows per row-block workgroup
constexpr int kThreads = 256;  // 4 waves
constexpr int kSP = kH + 4;    // LDS row stride of an activation tile (floats)
constexpr int kXP = 20;        // LDS row stride of the padded input tile
constexpr float kLogSqrt2Pi = 0.91893853320467274f;  // math.log(math.sqrt(2 * math.pi))

typedef float f4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------- layout

struct NetOff {
  int64_t t[8];  // w1, b1, w2, b2, wh0, bh0, wh1, bh1 (-1 absent)
  int64_t size;
};

__host__ __device__ inline NetOff net_off(int in_dim, int nh) {
  NetOff o;
  int64_t p = 0;
  auto take = [&](int k, int64_t n) {
    o.t[k] = p;
    p += (n + 3) & ~int64_t(3);  // every tensor 16-B aligned
  };
  take(0, (int64_t)kH * in_dim);
  take(1, kH);
  take(2, (int64_t)kH * kH);
  take(3, kH);
  take(4, kH);
  take(5, 1);
  if (nh > 1) {
    take(6, kH);
    take(7, 1);
  } else {
    o.t[6] = o.t[7] = -1;
  }
  o.size = p;
  return o;
}

enum Shape { kActorShape = 0, kCriticShape = 1, kValueShape = 2 };
__host__ __device__ inline int net_shape(int n) { return n == 0 ? kActorShape : (n <= 2 ? kCriticShape : kValueShape); }
__host__ __device__ inline int net_in(int n, int D) { return net_shape(n) == kCriticShape ? D + 1 : D; }

// Fragment order of a 256x256 layer's kernel copy: element (n, k) of the
// [out][in] matrix sits where lane (i = n % 16, kq = (k % 16) / 4) of the
// 16x16 block (n / 16, k / 16) reads it as component k % 4 of its float4: one
// A-fragment load is 1 KB contiguous (eight full 128-B lines) instead of 16
// half-used lines of the [out][in] layout.
__host__ __device__ inline int64_t swz(int n, int k) {
  return ((int64_t)((n >> 4) * 16 + (k >> 4)) * 64 + ((k & 15) >> 2) * 16 + (n & 15)) * 4 + (k & 3);
}

// per-row fields of the scratch, f32 [B] each
enum RowField {
  F_MU, F_SR, F_SIG, F_TL, F_A1, F_LP1, F_A2, F_X2, F_LP2,   // actor forward + draws
  F_V,                                                       // value (value_ stays in the critic-loss role)
  F_QC1, F_QC2,                                              // critics at the stored actions
  F_Q1A1, F_Q2A1, F_Q1A2, F_Q2A2, F_DA1, F_DA2,              // critics at the draws, dq/da at a2
  F_GMU, F_GSR, F_GC1, F_GC2, F_GV,                          // head-output gradients
  F_LV, F_LA, F_LC1, F_LC2,                                  // per-row loss terms
  F_COUNT
};

// Activations that phase 3 reduces over the batch ([kH][B] per net) are kept in
// the same fragment order with the batch row as k: (n, r) -> block (n / 16,
// r / 16), lane (n % 16, (r % 16) / 4), component r % 4. A row block writes
// exactly one column of blocks; phase 3 loads whole 1 KB fragments.
__host__ __device__ inline int64_t act_off(int n, int r, int B) {
  return ((int64_t)((n >> 4) * (B >> 4) + (r >> 4)) * 64 + ((r & 15) >> 2) * 16 + (n & 15)) * 4 + (r & 3);
}

struct NetAct {   // [kH][B] activations of one optimised net (act_off order)
  float* h1t;
  float* h2t;
  float* dz1t;
  float* dz2t;
};

struct SacArgs {
  float* P;            // weights buffer
  unsigned long long* stamps;  // SACENV_SAC_STAMPS diagnostics: [phase][block][16] s_memrealtime
  const float* s;      // state [B][D]
  const float* act;    // action [B]
  const double* rew;   // reward [B]
  const float* s2;     // new_state [B][D]
  const uint8_t* done;
  const float* eps1;
  const float* eps2;
  float* rows;         // row fields [F_COUNT][B]
  float* xt;           // [16][B] fc1 inputs (act_off order): state, action, 1
  float* losses;
  NetAct na[4];        // actor, critic 1, critic 2, value
  int64_t net[5], am[4], av[4], w2f[5], w2tf[4];
  NetOff off[3];
  int B, D;
  float max_action, gamma, scale, inv_b;
  // Adam (torch.optim.Adam foreach form), scalars as torch casts them
  float lerp_w, b2, omb2, bc2s, eps, nstep_actor, nstep_critic;
  float tau, omtau;
};

__device__ __forceinline__ float* rowf(const SacArgs& a, int f) { return a.rows + (int64_t)f * a.B; }

#ifdef SACENV_SAC_STAMPS  // timing diagnostics: wall clock (100 MHz) per block of each phase
#define STAMP(a, ph, k)                                                                           \
  do {                                                                                            \
    if (threadIdx.x == 0)                                                                         \
      (a).stamps[((int64_t)(ph) * 1024 + blockIdx.x) * 16 + (k)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define STAMP(a, ph, k) \
  do {                  \
  } while (0)
#endif

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS
// operations, not for its global stores (__syncthreads() would drain those
// too; nothing in these kernels reads its own global stores back)
__device__ __forceinline__ void lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// ---------------------------------------------------------------- LDS tiles

struct RowLds {
  float x[kRows * kXP];
  float h1[kRows * kSP];
  float h2[kRows * kSP];
  float z[kRows * kSP];
  float g0[kRows], g1[kRows];
};

// X[j][k] = src[row0 + j][k] (k < D), acol[row0 + j] at k = D, zero to 16
__device__ __forceinline__ void load_x(float* xl, const float* __restrict__ src, int D, int row0, int nrows,
                                       const float* __restrict__ acol, int tid) {
  const int j = tid >> 4, k = tid & 15;
  float v = 0.f;
  if (j < nrows) {
    if (k < D)
      v = src[(int64_t)(row0 + j) * D + k];
    else if (k == D && acol != nullptr)
      v = acol[row0 + j];
  }
  xl[j * kXP + k] = v;
}

// feature-major [kH][B] rows row0..row0+15 -> LDS tile
__device__ __forceinline__ void load_tile_t(float* hl, const float* __restrict__ gT, int B, int row0, int tid) {
  const int j = tid & 15, fg = tid >> 4;
  float v[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) v[q] = gT[act_off(fg * 16 + q, row0 + j, B)];
#pragma unroll
  for (int q = 0; q < 16; ++q) hl[j * kSP + fg * 16 + q] = v[q];
}

__device__ __forceinline__ void store_tile_t(const float* hl, float* __restrict__ gT, int B, int row0, int tid) {
  const int j = tid & 15, fg = tid >> 4;
#pragma unroll 4
  for (int q = 0; q < 16; ++q) {
    const int f = fg * 16 + q;
    gT[act_off(f, row0 + j, B)] = hl[j * kSP + f];
  }
}

// ---------------------------------------------------------------- dense layer on MFMA

// acc[t] <- W[64w + 16t + ..][:] . X^T for the 16 rows of xl. FC1: W is
// [kH][kin] (kin <= 16, scalar loads); else [kH][kH] (float4 loads, issued
// kPrefetch k-blocks ahead: one block is 16 MFMAs = ~0.25 us, an L2 round
// trip ~1 us, and hipcc on its own pipelines one block ahead)
constexpr int kPrefetch = 8;

// the first kPrefetch k-blocks of a 256x256 layer's A fragments, issued early
struct WPre {
  f4 v[kPrefetch][4];
};
__device__ __forceinline__ const f4* frag(const float* __restrict__ Wf, int w, int t, int kb, int lane) {
  return reinterpret_cast<const f4*>(Wf + ((int64_t)((4 * w + t) * 16 + kb) * 64 + lane) * 4);
}
__device__ __forceinline__ void w_prefetch(const float* __restrict__ Wf, int lane, int w, WPre& p) {
#pragma unroll
  for (int kb = 0; kb < kPrefetch; ++kb)
#pragma unroll
    for (int t = 0; t < 4; ++t) p.v[kb][t] = *frag(Wf, w, t, kb, lane);
}

// acc[t] <- W[64w + 16t + ..][:] . X^T for the 16 rows of xl (256 x 256 layer, W
// in fragment order);
// blocks kb >= kPrefetch are loaded kPrefetch blocks ahead of their MFMAs
__device__ __forceinline__ void layer256(const float* __restrict__ W, const WPre& pre, const float* xl, int xs,
                                         int lane, int w, f4 acc[4]) {
  const int i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
  constexpr int KB = kH / 16;
  f4 av[KB][4];
#pragma unroll
  for (int kb = 0; kb < KB; ++kb) {
    if (kb + kPrefetch < KB) {
#pragma unroll
      for (int t = 0; t < 4; ++t) av[kb + kPrefetch][t] = *frag(W, w, t, kb + kPrefetch, lane);
      __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead (the scheduler sinks them)
    }
    const f4 b = *reinterpret_cast<const f4*>(xl + i * xs + 16 * kb + 4 * kq);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const float aw = kb < kPrefetch ? pre.v[kb < kPrefetch ? kb : 0][t][s] : av[kb][t][s];
        acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(aw, b[s], acc[t], 0, 0, 0);
      }
  }
}

// fc1 (K = kin <= 16): A fragments of the four tiles, loaded early
struct W1Pre {
  f4 v[4];
};
__device__ __forceinline__ void w1_prefetch(const float* __restrict__ W, int kin, int lane, int w, W1Pre& p) {
  const int i = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const float* wp = W + (64 * w + 16 * t + i) * kin;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int k = 4 * kq + s;
      p.v[t][s] = k < kin ? wp[k] : 0.f;
    }
  }
}
__device__ __forceinline__ void layer_fc1(const W1Pre& p, const float* xl, int xs, int lane, f4 acc[4]) {
  const int i = lane & 15, kq = lane >> 4;
  const f4 b = *reinterpret_cast<const f4*>(xl + i * xs + 4 * kq);
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(p.v[t][s], b[s], acc[t], 0, 0, 0);
}

// a tile's bias slice, per lane (features 64w + 16t + 4kq .. +3)
__device__ __forceinline__ void bias_prefetch(const float* __restrict__ bias, int lane, int w, f4 bv[4]) {
  const int kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) bv[t] = *reinterpret_cast<const f4*>(bias + 64 * w + 16 * t + 4 * kq);
}

// forward epilogue: y = relu(acc + bias) -> LDS tile (and feature-major global)
// lane (j = row, kq) holds features 64w + 16t + 4kq + r
__device__ __forceinline__ void epi_fwd(const f4 acc[4], const f4 bv[4], float* yl, int lane, int w,
                                        float* __restrict__ gT, int B, int row0) {
  const int j = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n0 = 64 * w + 16 * t + 4 * kq;
    const f4 bb = bv[t];
    f4 y;
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = fmaxf(acc[t][r] + bb[r], 0.f);
    *reinterpret_cast<f4*>(yl + j * kSP + n0) = y;
    if (gT != nullptr)
#pragma unroll
      for (int r = 0; r < 4; ++r) gT[act_off(n0 + r, row0 + j, B)] = y[r];
  }
}

// backward epilogue: dz = acc * [h > 0] (relu backward on the stored output)
__device__ __forceinline__ void epi_bwd(const f4 acc[4], const float* hl, float* zl, int lane, int w,
                                        float* __restrict__ gT, int B, int row0) {
  const int j = lane & 15, kq = lane >> 4;
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n0 = 64 * w + 16 * t + 4 * kq;
    const f4 h = *reinterpret_cast<const f4*>(hl + j * kSP + n0);
    f4 z;
#pragma unroll
    for (int r = 0; r < 4; ++r) z[r] = h[r] > 0.f ? acc[t][r] : 0.f;
    if (zl != nullptr) *reinterpret_cast<f4*>(zl + j * kSP + n0) = z;
    if (gT != nullptr)
#pragma unroll
      for (int r = 0; r < 4; ++r) gT[act_off(n0 + r, row0 + j, B)] = z[r];
  }
}

// sum_f w[f * ws] * h[row][f] for row = tid >> 4, in all 16 lanes of the row
__device__ __forceinline__ float row_dot(const float* hl, const float* __restrict__ wv, int ws, int tid) {
  const int j = tid >> 4, part = tid & 15;
  float s = 0.f;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const int f = q * 16 + part;
    s = fmaf(wv[f * ws], hl[j * kSP + f], s);
  }
#pragma unroll
  for (int o = 8; o > 0; o >>= 1) s += __shfl_xor(s, o, 16);
  return s;
}

// two-layer trunk on the input tile in l.x: h1, h2 in LDS (and optionally global)
// input rows (state, + acol at column D) -> fc1 -> fc2 for the 16 rows: every
// parameter load (fc1 fragments, biases, fc2's first k-blocks) is issued with
// the input loads, before the first barrier
__device__ __forceinline__ void trunk(const float* __restrict__ Pn, const NetOff& o, int kin, RowLds& l, int tid,
                                      float* h1t, float* h2t, int B, int row0, const float* __restrict__ src,
                                      int D, const float* __restrict__ acol, const float* __restrict__ w2f,
                                      const SacArgs* sa = nullptr, int ph = 0) {
  const int lane = tid & 63, w = tid >> 6;
  W1Pre w1;
  w1_prefetch(Pn + o.t[0], kin, lane, w, w1);
  f4 b1[4], b2[4];
  bias_prefetch(Pn + o.t[1], lane, w, b1);
  bias_prefetch(Pn + o.t[3], lane, w, b2);
  WPre w2;
  w_prefetch(w2f, lane, w, w2);
  load_x(l.x, src, D, row0, kRows, acol, tid);
  lds_sync();
  if (sa) STAMP(*sa, ph, 1);
  f4 acc[4];
  layer_fc1(w1, l.x, kXP, lane, acc);
  epi_fwd(acc, b1, l.h1, lane, w, h1t, B, row0);
  lds_sync();
  if (sa) STAMP(*sa, ph, 2);
  layer256(w2f, w2, l.h1, kSP, lane, w, acc);
  if (sa) STAMP(*sa, ph, 3);
  epi_fwd(acc, b2, l.h2, lane, w, h2t, B, row0);
  lds_sync();
  if (sa) STAMP(*sa, ph, 4);
}

// head backward: dz2 = (wh0 g0 + wh1 g1) * [h2 > 0] -> dz2t; dz1 = (W2^T dz2) * [h1 > 0]
// (W2^T in fragment order: w2tf)
// -> dz1t (and LDS l.h2 when keep_dz1). g0/g1 per row in l.g0/l.g1.
__device__ __forceinline__ void head_backward(const float* __restrict__ Pn, const NetOff& o,
                                              const float* __restrict__ w2tf, const WPre& pre, RowLds& l, int tid,
                                              float* dz2t, float* dz1t, int B, int row0, bool keep_dz1) {
  const int lane = tid & 63, w = tid >> 6;
  const float* wh0 = Pn + o.t[4];
  const float* wh1 = o.t[6] >= 0 ? Pn + o.t[6] : nullptr;
  for (int e = tid; e < kRows * kH; e += kThreads) {
    const int j = e >> 8, f = e & (kH - 1);
    float g = wh0[f] * l.g0[j];
    if (wh1 != nullptr) g = g + wh1[f] * l.g1[j];
    l.z[j * kSP + f] = l.h2[j * kSP + f] > 0.f ? g : 0.f;
  }
  lds_sync();
  f4 acc[4];
  layer256(w2tf, pre, l.z, kSP, lane, w, acc);
  if (dz2t != nullptr) store_tile_t(l.z, dz2t, B, row0, tid);  // l.z stays until the next barrier
  lds_sync();  // every wave has read l.z / l.h2 before l.h2 is overwritten
  epi_bwd(acc, l.h1, keep_dz1 ? l.h2 : nullptr, lane, w, dz1t, B, row0);
  lds_sync();
}

// Half of a backward layer: output features [128 h, 128 h + 128), wave w
// owning two 16x16 tiles (blocks 8h + 2w + t). Phase 2 splits each role's one
// layer over two workgroups this way (twice the workgroups, half the MFMAs
// each); every A fragment of the half is loaded before the first MFMA.
struct HalfPre {
  f4 v[kH / 16][2];
};
__device__ __forceinline__ void half_prefetch(const float* __restrict__ Wf, int lane, int nb0, HalfPre& p) {
#pragma unroll
  for (int kb = 0; kb < kH / 16; ++kb)
#pragma unroll
    for (int t = 0; t < 2; ++t)
      p.v[kb][t] = *reinterpret_cast<const f4*>(Wf + ((int64_t)((nb0 + t) * 16 + kb) * 64 + lane) * 4);
}

__device__ __forceinline__ void head_backward_half(const float* __restrict__ Pn, const NetOff& o, const HalfPre& pre,
                                                   RowLds& l, int tid, float* dz2t, float* dz1t, int B, int row0,
                                                   int h) {
  const int lane = tid & 63, w = tid >> 6, i = lane & 15, kq = lane >> 4;
  const float* wh0 = Pn + o.t[4];
  const float* wh1 = o.t[6] >= 0 ? Pn + o.t[6] : nullptr;
  for (int e = tid; e < kRows * kH; e += kThreads) {
    const int j = e >> 8, f = e & (kH - 1);
    float g = wh0[f] * l.g0[j];
    if (wh1 != nullptr) g = g + wh1[f] * l.g1[j];
    l.z[j * kSP + f] = l.h2[j * kSP + f] > 0.f ? g : 0.f;
  }
  lds_sync();
  const int nb0 = 8 * h + 2 * w;
  f4 acc[2] = {f4{0.f, 0.f, 0.f, 0.f}, f4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
  for (int kb = 0; kb < kH / 16; ++kb) {
    const f4 b = *reinterpret_cast<const f4*>(l.z + i * kSP + 16 * kb + 4 * kq);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 2; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(pre.v[kb][t][s], b[s], acc[t], 0, 0, 0);
  }
  if (h == 0 && dz2t != nullptr) store_tile_t(l.z, dz2t, B, row0, tid);
#pragma unroll
  for (int t = 0; t < 2; ++t) {  // relu backward on h1, dz1 -> global (act_off order)
    const int n0 = 16 * (nb0 + t) + 4 * kq;
    const f4 hv = *reinterpret_cast<const f4*>(l.h1 + i * kSP + n0);
#pragma unroll
    for (int r = 0; r < 4; ++r) dz1t[act_off(n0 + r, row0 + i, B)] = hv[r] > 0.f ? acc[t][r] : 0.f;
  }
}

// tanh-squashed Normal draw (networks.py:47-70): x = mean + eps * std,
// action = tanh(x) * max_action, log_prob with the tanh correction
__device__ __forceinline__ float policy_sigma(float sr, float& tl) {
  tl = tanhf(sr);
  const float ls = -5.f + 3.5f * (tl + 1.f);  // LOG_STD_MIN + 0.5 (MAX - MIN) (tanh + 1)
  return expf(ls);
}
__device__ __forceinline__ void policy_draw(float mu, float sig, float eps, float M, float& x, float& act, float& lp) {
  x = mu + eps * sig;
  act = tanhf(x) * M;
  const float u = x - mu;
  lp = -(u * u) / (2.f * (sig * sig)) - logf(sig) - kLogSqrt2Pi;
  lp = lp - logf(1.f - act * act + 1e-6f);
}

// ---------------------------------------------------------------- phase roles

__device__ void role_actor_fwd(const SacArgs& a, RowLds& l, int tid, int row0) {
  const float* Pn = a.P + a.net[0];
  const NetOff& o = a.off[kActorShape];
  trunk(Pn, o, a.D, l, tid, a.na[0].h1t, a.na[0].h2t, a.B, row0, a.s, a.D, nullptr, a.P + a.w2f[0]);
  const float mu = row_dot(l.h2, Pn + o.t[4], 1, tid) + Pn[o.t[5]];
  const float sr = row_dot(l.h2, Pn + o.t[6], 1, tid) + Pn[o.t[7]];
  if ((tid & 15) == 0) {
    const int r = row0 + (tid >> 4);
    float tl;
    const float sig = policy_sigma(sr, tl);
    float x1, a1, lp1, x2, a2, lp2;
    policy_draw(mu, sig, a.eps1[r], a.max_action, x1, a1, lp1);
    policy_draw(mu, sig, a.eps2[r], a.max_action, x2, a2, lp2);
    rowf(a, F_MU)[r] = mu;
    rowf(a, F_SR)[r] = sr;
    rowf(a, F_SIG)[r] = sig;
    rowf(a, F_TL)[r] = tl;
    rowf(a, F_A1)[r] = a1;
    rowf(a, F_LP1)[r] = lp1;
    rowf(a, F_A2)[r] = a2;
    rowf(a, F_X2)[r] = x2;
    rowf(a, F_LP2)[r] = lp2;
  }
}

// value(state) (storing the activations) or target_value(new_state); v in the row's lanes
__device__ float value_fwd(const SacArgs& a, RowLds& l, int tid, int row0, bool target) {
  const int n = target ? 4 : 3;
  const float* Pn = a.P + a.net[n];
  const NetOff& o = a.off[kValueShape];
  trunk(Pn, o, a.D, l, tid, target ? nullptr : a.na[3].h1t, target ? nullptr : a.na[3].h2t, a.B, row0,
        target ? a.s2 : a.s, a.D, nullptr, a.P + a.w2f[n], target ? nullptr : &a, 0);
  const float v = row_dot(l.h2, Pn + o.t[4], 1, tid) + Pn[o.t[5]];
  if (!target) STAMP(a, 0, 5);
  return v;
}

__device__ void role_value_fwd(const SacArgs& a, RowLds& l, int tid, int row0) {
  const float v = value_fwd(a, l, tid, row0, false);
  if ((tid & 15) == 0) rowf(a, F_V)[row0 + (tid >> 4)] = v;
}

// critic c (1, 2) on [state, acol]; returns q in the row's lanes
__device__ float critic_fwd(const SacArgs& a, RowLds& l, int tid, int row0, int c, const float* acol, bool store) {
  const float* Pn = a.P + a.net[c];
  const NetOff& o = a.off[kCriticShape];
  trunk(Pn, o, a.D + 1, l, tid, store ? a.na[c].h1t : nullptr, store ? a.na[c].h2t : nullptr, a.B, row0, a.s, a.D,
        acol, a.P + a.w2f[c]);
  return row_dot(l.h2, Pn + o.t[4], 1, tid) + Pn[o.t[5]];
}

__device__ void role_critic_stored(const SacArgs& a, RowLds& l, int tid, int row0, int c) {
  const float q = critic_fwd(a, l, tid, row0, c, a.act, true);
  if ((tid & 15) == 0) rowf(a, c == 1 ? F_QC1 : F_QC2)[row0 + (tid >> 4)] = q;
  if (c == 1) {  // X^T of the fc1 inputs for phase 3: state, action at column D, 1 at column 15 (bias)
    const int j = tid >> 4, k = tid & 15;
    a.xt[act_off(k, row0 + j, a.B)] = k == 15 ? 1.f : l.x[j * kXP + k];
  }
}

// critic c at the sample() actions: the value target's min q (:113-117)
__device__ void role_critic_sample(const SacArgs& a, RowLds& l, int tid, int row0, int c) {
  const float qa1 = critic_fwd(a, l, tid, row0, c, rowf(a, F_A1), false);
  if ((tid & 15) == 0) rowf(a, c == 1 ? F_Q1A1 : F_Q2A1)[row0 + (tid >> 4)] = qa1;
}

// critic c at the rsample() actions with dq/da through the critic (actor loss, :127-131)
__device__ void role_critic_rsample(const SacArgs& a, RowLds& l, int tid, int row0, int c) {
  const float qa2 = critic_fwd(a, l, tid, row0, c, rowf(a, F_A2), false);
  const float* Pn = a.P + a.net[c];
  const NetOff& o = a.off[kCriticShape];
  WPre pre;
  w_prefetch(a.P + a.w2tf[c], tid & 63, tid >> 6, pre);
  if ((tid & 15) == 0) l.g0[tid >> 4] = 1.f;
  lds_sync();
  head_backward(Pn, o, a.P + a.w2tf[c], pre, l, tid, nullptr, nullptr, a.B, row0, true);
  // dq/da = W1[:, D] . dz1
  const float da = row_dot(l.h2, Pn + o.t[0] + a.D, a.D + 1, tid);
  if ((tid & 15) == 0) {
    const int r = row0 + (tid >> 4);
    rowf(a, c == 1 ? F_Q1A2 : F_Q2A2)[r] = qa2;
    rowf(a, c == 1 ? F_DA1 : F_DA2)[r] = da;
  }
}

// critic c's loss backward: 0.5 mse(q, q_hat), q_hat = scale r + gamma value_ (:141-146)
// (value_ = target_value(new_state), done-masked (:108-111), computed here: one
// more layer for this role, one role fewer in phase 0 — 256 workgroups, one per CU)
__device__ void role_critic_loss(const SacArgs& a, RowLds& l, int tid, int row0, int c) {
  const NetAct& na = a.na[c];
  const float vt = value_fwd(a, l, tid, row0, true);
  if ((tid & 15) == 0) {
    const int j = tid >> 4;
    l.g1[j] = a.done[row0 + j] ? 0.f : vt;  // value_[done] = 0.0
  }
  WPre pre;
  w_prefetch(a.P + a.w2tf[c], tid & 63, tid >> 6, pre);
  lds_sync();
  load_tile_t(l.h1, na.h1t, a.B, row0, tid);
  load_tile_t(l.h2, na.h2t, a.B, row0, tid);
  if (tid < kRows) {
    const int r = row0 + tid;
    const float q = rowf(a, c == 1 ? F_QC1 : F_QC2)[r];
    const float qh = a.scale * (float)a.rew[r] + a.gamma * l.g1[tid];
    const float d = q - qh;
    const float g = d * a.inv_b;  // mse backward: (2 / B) (q - q_hat) * 0.5
    l.g0[tid] = g;
    rowf(a, c == 1 ? F_GC1 : F_GC2)[r] = g;
    rowf(a, c == 1 ? F_LC1 : F_LC2)[r] = d * d;
  }
  lds_sync();
  head_backward(a.P + a.net[c], a.off[kCriticShape], a.P + a.w2tf[c], pre, l, tid, na.dz2t, na.dz1t, a.B, row0,
                false);
}

// actor loss backward: mean(log_prob - min(q1, q2)) at the rsample() draw (:127-135)
__device__ void role_actor_bwd(const SacArgs& a, RowLds& l, int tid, int row0, int h) {
  const NetAct& na = a.na[0];
  HalfPre pre;
  half_prefetch(a.P + a.w2tf[0], tid & 63, 8 * h + 2 * (tid >> 6), pre);
  load_tile_t(l.h1, na.h1t, a.B, row0, tid);
  load_tile_t(l.h2, na.h2t, a.B, row0, tid);
  if (tid < kRows) {
    const int r = row0 + tid;
    const float ib = a.inv_b;
    const float q1 = rowf(a, F_Q1A2)[r], q2 = rowf(a, F_Q2A2)[r];
    // torch.min(q1, q2) backward: the smaller one, half each on a tie
    const float dm = -ib;
    const float g1 = q1 < q2 ? dm : (q1 == q2 ? 0.5f * dm : 0.f);
    const float g2 = q2 < q1 ? dm : (q1 == q2 ? 0.5f * dm : 0.f);
    const float M = a.max_action;
    const float mu = rowf(a, F_MU)[r], sig = rowf(a, F_SIG)[r], tl = rowf(a, F_TL)[r];
    const float x = rowf(a, F_X2)[r], act = rowf(a, F_A2)[r];
    const float e2 = a.eps2[r];
    const float th = tanhf(x);
    const float u = x - mu, var = sig * sig;
    // d/d action: -log(1 - a^2 + 1e-6) (log_prob term) and -min q
    const float dact = ib * (2.f * act / (1.f - act * act + 1e-6f)) + (g1 * rowf(a, F_DA1)[r] + g2 * rowf(a, F_DA2)[r]);
    const float dx = dact * M * (1.f - th * th) + ib * (-u / var);
    const float dmu = dx + ib * (u / var);
    const float dsig = dx * e2 + ib * (u * u * sig / (var * var) - 1.f / sig);
    const float dsr = dsig * sig * 3.5f * (1.f - tl * tl);
    l.g0[tid] = dmu;
    l.g1[tid] = dsr;
    if (h == 0) {
      rowf(a, F_GMU)[r] = dmu;
      rowf(a, F_GSR)[r] = dsr;
      rowf(a, F_LA)[r] = rowf(a, F_LP2)[r] - fminf(q1, q2);
    }
  }
  lds_sync();
  head_backward_half(a.P + a.net[0], a.off[kActorShape], pre, l, tid, na.dz2t, na.dz1t, a.B, row0, h);
}

// value loss backward: 0.5 mse(value, min q(sample()) - log_prob) (:113-124)
__device__ void role_value_bwd(const SacArgs& a, RowLds& l, int tid, int row0, int h) {
  const NetAct& na = a.na[3];
  HalfPre pre;
  half_prefetch(a.P + a.w2tf[3], tid & 63, 8 * h + 2 * (tid >> 6), pre);
  load_tile_t(l.h1, na.h1t, a.B, row0, tid);
  load_tile_t(l.h2, na.h2t, a.B, row0, tid);
  if (tid < kRows) {
    const int r = row0 + tid;
    const float target = fminf(rowf(a, F_Q1A1)[r], rowf(a, F_Q2A1)[r]) - rowf(a, F_LP1)[r];
    const float d = rowf(a, F_V)[r] - target;
    const float g = d * a.inv_b;
    l.g0[tid] = g;
    if (h == 0) {
      rowf(a, F_GV)[r] = g;
      rowf(a, F_LV)[r] = d * d;
    }
  }
  lds_sync();
  head_backward_half(a.P + a.net[3], a.off[kValueShape], pre, l, tid, na.dz2t, na.dz1t, a.B, row0, h);
}

__device__ __forceinline__ void rows_body(const SacArgs& a, RowLds& l, int phase, int vb) {
  const int tid = threadIdx.x;
  const int nrb = a.B / kRows;
  const int role = vb / nrb, row0 = (vb - role * nrb) * kRows;
  if (phase == 0) {
    if (role == 0) role_actor_fwd(a, l, tid, row0);
    else if (role == 1) role_value_fwd(a, l, tid, row0);
    else role_critic_stored(a, l, tid, row0, role - 1);
  } else if (phase == 1) {  // two-layer roles first; the one-layer ones share CUs
    if (role < 2) role_critic_rsample(a, l, tid, row0, role + 1);
    else if (role < 4) role_critic_loss(a, l, tid, row0, role - 1);
    else role_critic_sample(a, l, tid, row0, role - 3);
  } else {
    if (role < 2) role_actor_bwd(a, l, tid, row0, role);  // two halves of each backward layer
    else role_value_bwd(a, l, tid, row0, role - 2);
  }
}

// one or two workgroups per CU: registers for kPrefetch k-blocks of weights in flight
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(1, 2))) k_sac_rows(SacArgs a, int phase) {
  __shared__ RowLds l;
  STAMP(a, phase, 0);
  rows_body(a, l, phase, blockIdx.x);
  STAMP(a, phase, 15);
}

// ---------------------------------------------------------------- phase 3: gradients + Adam

__device__ __forceinline__ void adam(const SacArgs& a, float nstep, float g, float& p, float& m, float& v) {
  m = m + a.lerp_w * (g - m);            // exp_avg.lerp_(grad, 1 - beta1)
  v = v * a.b2 + (a.omb2 * g) * g;       // exp_avg_sq.mul_(beta2).addcmul_(grad, grad, 1 - beta2)
  const float den = sqrtf(v) / a.bc2s + a.eps;
  p = p + nstep * (m / den);             // param.addcdiv_(exp_avg, denom, -step_size)
}

__device__ __forceinline__ void update_elem(const SacArgs& a, int t, int64_t idx, float g) {
  float* P = a.P + a.net[t];
  float* M = a.P + a.am[t];
  float* V = a.P + a.av[t];
  float p = P[idx], m = M[idx], v = V[idx];
  adam(a, t == 0 ? a.nstep_actor : a.nstep_critic, g, p, m, v);
  P[idx] = p;
  M[idx] = m;
  V[idx] = v;
  if (t == 3) {  // update_network_parameters(): tau * value + (1 - tau) * target
    float* T = a.P + a.net[4];
    T[idx] = a.tau * p + a.omtau * T[idx];
  }
}

constexpr int kUpdLds = 4 * 32 * 33 + 128;  // fc2 tile partials + fc2.bias partials (small_params: 8 x 16 x 17)

// C k-blocks of 16 rows: every load issued before the first MFMA (the update
// launch runs one wave per SIMD: registers to spare, latency to hide); the
// dz2 fragments are also summed per lane (fc2.bias gradient)
__device__ __forceinline__ const f4* afrag(const float* __restrict__ gT, int nb, int rb, int B, int lane) {
  return reinterpret_cast<const f4*>(gT + ((int64_t)nb * (B >> 4) + rb) * 256 + lane * 4);
}
template <int C>
__device__ __forceinline__ void fc2_chunk(const float* __restrict__ dz2t, const float* __restrict__ h1t, int B,
                                          int r0, int o0, int i0, int lane, f4 acc[2][2], float cs[2]) {
  f4 A[C][2], Bv[C][2];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int rb = (r0 >> 4) + c;
#pragma unroll
    for (int so = 0; so < 2; ++so) A[c][so] = *afrag(dz2t, (o0 >> 4) + so, rb, B, lane);
#pragma unroll
    for (int si = 0; si < 2; ++si) Bv[c][si] = *afrag(h1t, (i0 >> 4) + si, rb, B, lane);
  }
  __builtin_amdgcn_sched_barrier(0);  // all loads in flight before the first MFMA
#pragma unroll
  for (int c = 0; c < C; ++c) {
#pragma unroll
    for (int so = 0; so < 2; ++so) cs[so] += ((A[c][so][0] + A[c][so][1]) + A[c][so][2]) + A[c][so][3];
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int so = 0; so < 2; ++so)
#pragma unroll
        for (int si = 0; si < 2; ++si)
          acc[so][si] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[c][so][s], Bv[c][si][s], acc[so][si], 0, 0, 0);
  }
}

// fc2.weight gradient tile (32 out x 32 in) of net t: dW = dz2^T h1 over the
// batch, each wave a quarter of the rows, then Adam and the kernel copies;
// tiles of the first in-column also take fc2.bias (sum of dz2 over the batch)
__device__ void fc2_tile(const SacArgs& a, int t, int ob, int ib, int tid, float* red) {
  const int lane = tid & 63, w = tid >> 6, kq = lane >> 4;
  const NetAct& na = a.na[t];
  const int B = a.B, rq = B / 4, rbeg = w * rq;
  const int o0 = 32 * ob, i0 = 32 * ib;
  f4 acc[2][2];
  float cs[2] = {0.f, 0.f};
#pragma unroll
  for (int so = 0; so < 2; ++so)
#pragma unroll
    for (int si = 0; si < 2; ++si) acc[so][si] = f4{0.f, 0.f, 0.f, 0.f};
  int r0 = rbeg;
  // chunks of 16 k-blocks hold 256 VGPRs of loads (one workgroup per CU); 12 + 4 stays
  // under 256 so the small-parameter workgroups can share the CUs
  constexpr int kChunk = 12;
  for (; r0 + 16 * kChunk <= rbeg + rq; r0 += 16 * kChunk)
    fc2_chunk<kChunk>(na.dz2t, na.h1t, B, r0, o0, i0, lane, acc, cs);
  for (; r0 < rbeg + rq; r0 += 64) fc2_chunk<4>(na.dz2t, na.h1t, B, r0, o0, i0, lane, acc, cs);  // rq % 64 == 0
  STAMP(a, 3, 1);
  // lane holds dW[o = 16 so + 4 kq + r][i = 16 si + (lane & 15)]
#pragma unroll
  for (int so = 0; so < 2; ++so)
#pragma unroll
    for (int si = 0; si < 2; ++si)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[(w * 32 + 16 * so + 4 * kq + r) * 33 + 16 * si + (lane & 15)] = acc[so][si][r];
  float* bred = red + 4 * 32 * 33;  // [4 waves][32] fc2.bias partials
#pragma unroll
  for (int so = 0; so < 2; ++so) {
    cs[so] += __shfl_xor(cs[so], 16, 64);
    cs[so] += __shfl_xor(cs[so], 32, 64);
    if (kq == 0) bred[w * 32 + 16 * so + (lane & 15)] = cs[so];
  }
  lds_sync();
  STAMP(a, 3, 2);
  const int o = tid >> 3, ic = (tid & 7) * 4;
  const int64_t w2 = a.off[net_shape(t)].t[2];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const int col = ic + c, n = o0 + o, k = i0 + col;
    const float g = ((red[(0 * 32 + o) * 33 + col] + red[(1 * 32 + o) * 33 + col]) + red[(2 * 32 + o) * 33 + col]) +
                    red[(3 * 32 + o) * 33 + col];
    const int64_t idx = w2 + (int64_t)n * kH + k;
    update_elem(a, t, idx, g);
    const float p = a.P[a.net[t] + idx];
    a.P[a.w2f[t] + swz(n, k)] = p;   // kernel copies: forward and backward fragment order
    a.P[a.w2tf[t] + swz(k, n)] = p;
    if (t == 3) a.P[a.w2f[4] + swz(n, k)] = a.P[a.net[4] + idx];  // the target's forward copy
  }
  if (ib == 0 && tid < 32) {
    const float g = ((bred[tid] + bred[32 + tid]) + bred[64 + tid]) + bred[96 + tid];
    update_elem(a, t, a.off[net_shape(t)].t[3] + o0 + tid, g);
  }
}

constexpr int kSmallF = 16;  // features per small-parameter workgroup (one 16x16 tile)

template <int C>
__device__ __forceinline__ void small_chunk(const NetAct& na, const float* __restrict__ xt, const float* __restrict__ g0,
                                            const float* __restrict__ g1, int B, int nb, int rb0, int lane, f4& s1,
                                            f4& s2) {
  const int j = lane & 15, kq = lane >> 4;
  f4 z1[C], x[C], h2[C], g[C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const int rb = rb0 + c, r = 16 * rb + 4 * kq;
    z1[c] = *afrag(na.dz1t, nb, rb, B, lane);
    x[c] = *afrag(xt, 0, rb, B, lane);
    h2[c] = *afrag(na.h2t, nb, rb, B, lane);
    g[c] = f4{0.f, 0.f, 0.f, 0.f};
    if (j == 0) g[c] = *reinterpret_cast<const f4*>(g0 + r);
    if (j == 1 && g1 != nullptr) g[c] = *reinterpret_cast<const f4*>(g1 + r);
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < C; ++c)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s1 = __builtin_amdgcn_mfma_f32_16x16x4f32(z1[c][s], x[c][s], s1, 0, 0, 0);
      s2 = __builtin_amdgcn_mfma_f32_16x16x4f32(h2[c][s], g[c][s], s2, 0, 0, 0);
    }
}

// fc1.weight and fc1.bias (dz1^T [X | 1]) and the head weights (h2^T G, G = the
// head-output gradients) of 16 features of net t as two 16x16 MFMA tiles over
// the batch (each wave a quarter of the rows); the head biases in block 0
__device__ void small_params(const SacArgs& a, int t, int fb, int tid, float* red) {
  const int lane = tid & 63, w = tid >> 6, kq = lane >> 4;
  const NetAct& na = a.na[t];
  const int B = a.B, in = net_in(t, a.D);
  const NetOff& o = a.off[net_shape(t)];
  const float* g0 = rowf(a, t == 0 ? F_GMU : (t == 1 ? F_GC1 : (t == 2 ? F_GC2 : F_GV)));
  const float* g1 = t == 0 ? rowf(a, F_GSR) : nullptr;
  f4 s1 = f4{0.f, 0.f, 0.f, 0.f}, s2 = f4{0.f, 0.f, 0.f, 0.f};
  const int rbq = (B >> 4) / 4, rb0 = w * rbq;  // rbq % 4 == 0
  int c0 = 0;
  for (; c0 + 8 <= rbq; c0 += 8) small_chunk<8>(na, a.xt, g0, g1, B, fb, rb0 + c0, lane, s1, s2);
  for (; c0 < rbq; c0 += 4) small_chunk<4>(na, a.xt, g0, g1, B, fb, rb0 + c0, lane, s1, s2);
  // lane holds [f = 4 kq + r][col = lane & 15] of both tiles
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    red[((w * 2 + 0) * 16 + 4 * kq + r) * 17 + (lane & 15)] = s1[r];
    red[((w * 2 + 1) * 16 + 4 * kq + r) * 17 + (lane & 15)] = s2[r];
  }
  lds_sync();
  STAMP(a, 3, 3);
  {
    const int f = tid >> 4, k = tid & 15, fg = kSmallF * fb + f;
    auto sum4 = [&](int m) {
      return ((red[((0 * 2 + m) * 16 + f) * 17 + k] + red[((1 * 2 + m) * 16 + f) * 17 + k]) +
              red[((2 * 2 + m) * 16 + f) * 17 + k]) + red[((3 * 2 + m) * 16 + f) * 17 + k];
    };
    const float a1 = sum4(0), a2 = sum4(1);
    if (k < in) update_elem(a, t, o.t[0] + (int64_t)fg * in + k, a1);  // fc1.weight
    else if (k == 15) update_elem(a, t, o.t[1] + fg, a1);              // fc1.bias (the column of ones)
    if (k == 0) update_elem(a, t, o.t[4] + fg, a2);                    // head-0 weight
    else if (k == 1 && o.t[6] >= 0) update_elem(a, t, o.t[6] + fg, a2);  // head-1 weight
  }
  if (fb == 0) {  // head biases: sums of the head-output gradients
    lds_sync();
    float s0 = 0.f, sb = 0.f;
    for (int r = tid; r < B; r += kThreads) {
      s0 += g0[r];
      if (g1 != nullptr) sb += g1[r];
    }
#pragma unroll
    for (int m = 32; m > 0; m >>= 1) {
      s0 += __shfl_xor(s0, m, 64);
      sb += __shfl_xor(sb, m, 64);
    }
    if ((tid & 63) == 0) {
      red[tid >> 6] = s0;
      red[4 + (tid >> 6)] = sb;
    }
    lds_sync();
    if (tid == 0) update_elem(a, t, o.t[5], ((red[0] + red[1]) + red[2]) + red[3]);
    if (tid == 1 && o.t[7] >= 0) update_elem(a, t, o.t[7], ((red[4] + red[5]) + red[6]) + red[7]);
  }
}

__device__ void reduce_losses(const SacArgs& a, int tid, float* xs) {
  for (int q = 0; q < 4; ++q) {  // F_LV, F_LA, F_LC1, F_LC2 are consecutive
    const float* v = rowf(a, F_LV + q);
    float s = 0.f;
    for (int r = tid; r < a.B; r += kThreads) s += v[r];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((tid & 63) == 0) xs[4 * q + (tid >> 6)] = s;
  }
  lds_sync();
  if (tid < 4 && a.losses != nullptr) {
    const float s = ((xs[4 * tid] + xs[4 * tid + 1]) + xs[4 * tid + 2]) + xs[4 * tid + 3];
    const float mean = s / (float)a.B;
    a.losses[tid] = tid == 1 ? mean : 0.5f * mean;  // 0.5 * mse for value and critics
  }
}

constexpr int kFc2Tiles = 8 * 8;  // 32x32 tiles of a 256x256 layer

// block order: the loss reduction and the 64 small-parameter blocks first (they
// finish early and their CUs then take the last fc2 tiles), then 256 fc2 tiles
constexpr int kSmallBlocks = 4 * (kH / kSmallF);

__device__ __forceinline__ void update_body(const SacArgs& a, float* sm, int b) {
  const int tid = threadIdx.x;
  if (b == 0) {
    reduce_losses(a, tid, sm);
  } else if (b <= kSmallBlocks) {
    const int q = b - 1;
    small_params(a, q / (kH / kSmallF), q % (kH / kSmallF), tid, sm);
  } else {
    // workgroups go to the 8 XCDs round-robin (b % 8): XCD x gets the 2x4 block of
    // 32x32 tiles (out rows 2(x>>1)..+1, in cols 4(x&1)..+3) of each net, so its L2
    // fetches 2 dz2 and 4 h1 row panels instead of 8 + 8
    const int u = b - 1 - kSmallBlocks;  // kSmallBlocks + 1 = 65: b % 8 == (u + 1) % 8
    const int x = b & 7, k = u >> 3;
    const int t = k >> 3, kk = k & 7;
    fc2_tile(a, t, 2 * (x >> 1) + (kk >> 2), 4 * (x & 1) + (kk & 3), tid, sm);
  }
}
constexpr int kUpdateBlocks = 1 + kSmallBlocks + 4 * kFc2Tiles;

__global__ void __launch_bounds__(kThreads) k_sac_update(SacArgs a) {
  __shared__ float sm[kUpdLds];
  STAMP(a, 3, 0);
  update_body(a, sm, blockIdx.x);
  STAMP(a, 3, 15);
}

// kernel copies of fc2.weight: fragment order for nets 0..4, transposed for 0..3
__global__ void __launch_bounds__(kThreads) k_sac_sync(SacArgs a) {
  const int t = blockIdx.y;
  const float* w2 = a.P + a.net[t] + a.off[net_shape(t)].t[2];
  for (int e = blockIdx.x * kThreads + threadIdx.x; e < kH * kH; e += gridDim.x * kThreads) {
    const int n = e >> 8, k = e & (kH - 1);
    const float v = w2[e];
    a.P[a.w2f[t] + swz(n, k)] = v;
    if (t < 4) a.P[a.w2tf[t] + swz(k, n)] = v;
  }
}

// choose_action for n rows: actor forward and the sample() draw. 64 rows per
// workgroup (four 16-row tiles against every weight fragment: 4x the MFMA
// work per weight byte of the 16-row learn kernels); fc2's output never
// leaves registers — the two heads are reduced from the accumulators.
constexpr int kActRows = 64;

struct ActLds {
  float x[kActRows * kXP];
  float h1[kActRows * kSP];
  float head[4][kActRows][2];
};

// Closed-loop hand-off with sacenv_boat_segment (sacenv.h): workgroup b's 64
// rows are owner wave b's envs. It reads its obs rows only once
// obs_ready[b] >= obs_want (the env wave published the step), and publishes
// act_ready[b] = act_value once its actions are visible device-wide.
struct ActHandoff {
  const uint32_t* obs_ready;  // null: no hand-off
  uint32_t obs_want;
  uint32_t* act_ready;
  uint32_t act_value;
  int32_t* status;            // SACENV_STATUS_HANDOFF_TIMEOUT bit (nullable)
};

__device__ __forceinline__ uint32_t flag_load(const uint32_t* f) {  // device-coherent (sc0 sc1)
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(f), 0, 4, 0x00020000);
  return (uint32_t)__builtin_amdgcn_readfirstlane((int)__builtin_amdgcn_raw_buffer_load_b32(r, 0, 0, 17));
}

constexpr int kHandoffLds = 84 * 1024;  // > 160 KB / 2: one hand-off workgroup per CU
static_assert(sizeof(ActLds) <= (size_t)kHandoffLds, "ActLds above the hand-off LDS size");

__device__ __forceinline__ void act_body(ActLds& l, const SacArgs& a, const float* __restrict__ obs, int n,
                                         const float* __restrict__ eps, float* __restrict__ out,
                                         float* __restrict__ logp, const ActHandoff& h) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, i = lane & 15, kq = lane >> 4;
  const int row0 = blockIdx.x * kActRows;
  if (h.obs_ready != nullptr) {
    // Abort protocol (shared with sacenv_boat_segment): a hand-off that timed out
    // anywhere leaves SACENV_STATUS_HANDOFF_TIMEOUT set, and every later hand-off
    // launch refuses to compute; a wave that gives up publishes SACENV_FLAG_ABORT so
    // its peer stops too instead of reading stale rows. No one waits forever.
    bool abort = false;
    if (tid < 64) {  // one wave polls (bounded: ~seconds), the workgroup waits at the barrier
      const uint32_t* f = h.obs_ready + blockIdx.x;
      abort = h.status != nullptr &&
              (flag_load(reinterpret_cast<const uint32_t*>(h.status)) & SACENV_STATUS_HANDOFF_TIMEOUT) != 0;
      uint32_t it = 0, v = abort ? 0u : flag_load(f);
      while (!abort && v < h.obs_want) {
        if (++it >= (1u << 22)) {
          if (tid == 0 && h.status != nullptr) atomicOr(h.status, SACENV_STATUS_HANDOFF_TIMEOUT);
          abort = true;
          break;
        }
        __builtin_amdgcn_s_sleep(2);
        v = flag_load(f);
      }
      abort = abort || v == SACENV_FLAG_ABORT;
    }
    if (__syncthreads_or(abort ? 1 : 0)) {
      if (tid == 0)  // the env wave waiting for this row must not hang: release it, as an abort
        __hip_atomic_store(h.act_ready + blockIdx.x, SACENV_FLAG_ABORT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // no stale L2 lines of the obs rows
  }
  const int nrows = n - row0 < kActRows ? n - row0 : kActRows;
  const float* Pn = a.P + a.net[0];
  const NetOff& o = a.off[kActorShape];
  const int D = a.D;
  for (int e = tid; e < kActRows * 16; e += kThreads) {
    const int j = e >> 4, k = e & 15;
    l.x[j * kXP + k] = (j < nrows && k < D) ? obs[(int64_t)(row0 + j) * D + k] : 0.f;
  }
  f4 acc[4][4];  // [feature tile t][row tile rt]
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) acc[t][rt] = f4{0.f, 0.f, 0.f, 0.f};
  {  // fc1 (K = obs_dim <= 16): one k-block
    f4 av[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const float* wp = Pn + o.t[0] + (64 * w + 16 * t + i) * D;
#pragma unroll
      for (int s = 0; s < 4; ++s) av[t][s] = 4 * kq + s < D ? wp[4 * kq + s] : 0.f;
    }
    lds_sync();
    f4 bx[4];
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) bx[rt] = *reinterpret_cast<const f4*>(l.x + (16 * rt + i) * kXP + 4 * kq);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][s], bx[rt][s], acc[t][rt], 0, 0, 0);
  }
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n0 = 64 * w + 16 * t + 4 * kq;
    const f4 bb = *reinterpret_cast<const f4*>(Pn + o.t[1] + n0);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) {
      f4 y;
#pragma unroll
      for (int r = 0; r < 4; ++r) y[r] = fmaxf(acc[t][rt][r] + bb[r], 0.f);
      *reinterpret_cast<f4*>(l.h1 + (16 * rt + i) * kSP + n0) = y;
      acc[t][rt] = f4{0.f, 0.f, 0.f, 0.f};
    }
  }
  lds_sync();
  const float* W2f = a.P + a.w2f[0];
#pragma unroll 4
  for (int kb = 0; kb < kH / 16; ++kb) {
    f4 av[4], bx[4];
#pragma unroll
    for (int t = 0; t < 4; ++t) av[t] = *frag(W2f, w, t, kb, lane);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt) bx[rt] = *reinterpret_cast<const f4*>(l.h1 + (16 * rt + i) * kSP + 16 * kb + 4 * kq);
#pragma unroll
    for (int s = 0; s < 4; ++s)
#pragma unroll
      for (int t = 0; t < 4; ++t)
#pragma unroll
        for (int rt = 0; rt < 4; ++rt)
          acc[t][rt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[t][s], bx[rt][s], acc[t][rt], 0, 0, 0);
  }
  // heads from the accumulators: lane (i = row in tile, kq) holds features 64w + 16t + 4kq + r
  float pm[4] = {0.f, 0.f, 0.f, 0.f}, ps[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int n0 = 64 * w + 16 * t + 4 * kq;
    const f4 bb = *reinterpret_cast<const f4*>(Pn + o.t[3] + n0);
    const f4 wm = *reinterpret_cast<const f4*>(Pn + o.t[4] + n0);
    const f4 ws = *reinterpret_cast<const f4*>(Pn + o.t[6] + n0);
#pragma unroll
    for (int rt = 0; rt < 4; ++rt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float h = fmaxf(acc[t][rt][r] + bb[r], 0.f);
        pm[rt] = fmaf(wm[r], h, pm[rt]);
        ps[rt] = fmaf(ws[r], h, ps[rt]);
      }
  }
#pragma unroll
  for (int rt = 0; rt < 4; ++rt) {
    pm[rt] += __shfl_xor(pm[rt], 16, 64);
    pm[rt] += __shfl_xor(pm[rt], 32, 64);
    ps[rt] += __shfl_xor(ps[rt], 16, 64);
    ps[rt] += __shfl_xor(ps[rt], 32, 64);
    if (kq == 0) {
      l.head[w][16 * rt + i][0] = pm[rt];
      l.head[w][16 * rt + i][1] = ps[rt];
    }
  }
  lds_sync();
  if (tid < nrows) {
    const int j = tid;
    const float mu = (((l.head[0][j][0] + l.head[1][j][0]) + l.head[2][j][0]) + l.head[3][j][0]) + Pn[o.t[5]];
    const float sr = (((l.head[0][j][1] + l.head[1][j][1]) + l.head[2][j][1]) + l.head[3][j][1]) + Pn[o.t[7]];
    float tl, x, act, lp;
    const float sig = policy_sigma(sr, tl);
    policy_draw(mu, sig, eps[row0 + j], a.max_action, x, act, lp);
    out[row0 + j] = act;
    if (logp != nullptr) logp[row0 + j] = lp;
  }
  if (h.act_ready != nullptr) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");  // the actions, device-wide
    __syncthreads();
    if (tid == 0)
      __hip_atomic_store(h.act_ready + blockIdx.x, h.act_value, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// ---------------------------------------------------------------- host side

int check(const SacenvSacParams* p) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->hidden != kH || p->n_actions != 1 || p->obs_dim < 1 || p->obs_dim > 14) return SACENV_E_SIZE;
  if (p->batch < 256 || p->batch % 256 != 0 || p->batch > (1 << 20)) return SACENV_E_SIZE;
  return SACENV_OK;
}

void make_layout(const SacenvSacParams* p, SacenvSacLayout* L) {
  const int D = p->obs_dim;
  const NetOff sh[3] = {net_off(D, 2), net_off(D + 1, 1), net_off(D, 1)};
  int64_t q = 0;
  for (int n = 0; n < 5; ++n) {
    L->net[n] = q;
    q += sh[net_shape(n)].size;
  }
  for (int n = 0; n < 4; ++n) {
    L->adam_m[n] = q;
    q += sh[net_shape(n)].size;
  }
  for (int n = 0; n < 4; ++n) {
    L->adam_v[n] = q;
    q += sh[net_shape(n)].size;
  }
  for (int n = 0; n < 5; ++n) {
    L->w2f[n] = q;
    q += (int64_t)kH * kH;
  }
  for (int n = 0; n < 4; ++n) {
    L->w2tf[n] = q;
    q += (int64_t)kH * kH;
  }
  L->total_floats = q;
  for (int s = 0; s < 3; ++s) {
    L->net_floats[s] = sh[s].size;
    for (int k = 0; k < 8; ++k) L->tensor[s][k] = sh[s].t[k];
  }
  L->scratch_bytes = (int64_t)sizeof(float) * p->batch * (16 * (int64_t)kH + F_COUNT + 16);
#ifdef SACENV_SAC_STAMPS
  L->scratch_bytes += 4 * 1024 * 16 * 8;  // [phase][block][16] u64 after the row fields
#endif
}

SacArgs make_args(const SacenvSacParams* p, float* weights) {
  SacenvSacLayout L;
  make_layout(p, &L);
  SacArgs a{};
  a.P = weights;
  for (int n = 0; n < 5; ++n) a.net[n] = L.net[n];
  for (int n = 0; n < 4; ++n) {
    a.am[n] = L.adam_m[n];
    a.av[n] = L.adam_v[n];
    a.w2tf[n] = L.w2tf[n];
  }
  for (int n = 0; n < 5; ++n) a.w2f[n] = L.w2f[n];
  a.off[0] = net_off(p->obs_dim, 2);
  a.off[1] = net_off(p->obs_dim + 1, 1);
  a.off[2] = net_off(p->obs_dim, 1);
  a.B = p->batch;
  a.D = p->obs_dim;
  a.max_action = (float)p->max_action;
  a.gamma = (float)p->gamma;
  a.scale = (float)p->reward_scale;
  a.inv_b = 1.f / (float)p->batch;
  a.tau = (float)p->tau;
  a.omtau = (float)(1.0 - p->tau);
  return a;
}

bool aligned16(const void* q) { return ((uintptr_t)q & 15u) == 0; }

}  // namespace

extern "C" int sacenv_sac_layout(const SacenvSacParams* p, SacenvSacLayout* out) {
  if (p == nullptr || out == nullptr) return SACENV_E_NULL;
  const int rc = check(p);
  if (rc != SACENV_OK) return rc;
  make_layout(p, out);
  return SACENV_OK;
}

extern "C" int sacenv_sac_sync(const SacenvSacParams* p, float* weights, void* stream) {
  const int rc = check(p);
  if (rc != SACENV_OK) return rc;
  if (weights == nullptr) return SACENV_E_NULL;
  if (!aligned16(weights)) return SACENV_E_SIZE;
  const SacArgs a = make_args(p, weights);
  hipLaunchKernelGGL(k_sac_sync, dim3(64, 5), dim3(kThreads), 0, (hipStream_t)stream, a);
  return (int)hipGetLastError();
}

__global__ void __launch_bounds__(kThreads) k_sac_act(SacArgs a, const float* __restrict__ obs, int n,
                                                        const float* __restrict__ eps, float* __restrict__ out,
                                                        float* __restrict__ logp, ActHandoff h) {
  __shared__ ActLds l;
  act_body(l, a, obs, n, eps, out, logp, h);
}

// The closed loop's form (sacenv_sac_act_handoff): the same code held to 128
// architectural VGPRs (~150 allocated, no spills) so that one policy wave fits
// beside an owner wave of the segment launch (~320 VGPRs) on a SIMD's 512,
// and launched with its LDS padded to kHandoffLds (> half of a CU's 160 KB):
// a CU then holds at most ONE policy workgroup, which always leaves room for
// the CU's owner waves -- no arrangement of dispatched policy workgroups can
// keep an owner wave out (sacenv.closed_loop's co-residency plan).
__global__ void __launch_bounds__(kThreads) __attribute__((amdgpu_num_vgpr(128)))
k_sac_act_lean(SacArgs a, const float* __restrict__ obs, int n, const float* __restrict__ eps,
               float* __restrict__ out, float* __restrict__ logp, ActHandoff h) {
  __shared__ ActLds l;
  act_body(l, a, obs, n, eps, out, logp, h);
}

static int sac_act(const SacenvSacParams* p, const float* weights, const float* obs, int32_t n, const float* eps,
                   float* action, float* log_prob, const ActHandoff& h, void* stream) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->hidden != kH || p->n_actions != 1 || p->obs_dim < 1 || p->obs_dim > 14) return SACENV_E_SIZE;
  if (n < 0) return SACENV_E_SIZE;
  if (n == 0) return SACENV_OK;
  if (weights == nullptr || obs == nullptr || eps == nullptr || action == nullptr) return SACENV_E_NULL;
  if (!aligned16(weights)) return SACENV_E_SIZE;
  SacenvSacParams q = *p;
  q.batch = 256;  // unused by the act kernel
  const SacArgs a = make_args(&q, const_cast<float*>(weights));
  const int blocks = (n + kActRows - 1) / kActRows;
  if (h.obs_ready != nullptr)  // LDS padded: at most one policy workgroup per CU (kHandoffLds)
    hipLaunchKernelGGL(k_sac_act_lean, dim3(blocks), dim3(kThreads), kHandoffLds - sizeof(ActLds),
                       (hipStream_t)stream, a, obs, (int)n, eps, action, log_prob, h);
  else
    hipLaunchKernelGGL(k_sac_act, dim3(blocks), dim3(kThreads), 0, (hipStream_t)stream, a, obs, (int)n, eps, action,
                       log_prob, h);
  return (int)hipGetLastError();
}

extern "C" int sacenv_sac_act(const SacenvSacParams* p, const float* weights, const float* obs, int32_t n,
                              const float* eps, float* action, float* log_prob, void* stream) {
  return sac_act(p, weights, obs, n, eps, action, log_prob, ActHandoff{}, stream);
}

// The hand-off act kernel's resources for the closed loop's co-residency plan
// (sacenv.h): resident workgroups per CU alone, the grid for n rows, VGPRs per
// lane (architectural + accumulation, as allocated) and LDS bytes per workgroup.
extern "C" int sacenv_sac_act_occupancy(int32_t n, int32_t* blocks_per_cu, int32_t* grid, int32_t* vgprs,
                                        int32_t* lds_bytes) {
  if (blocks_per_cu == nullptr || grid == nullptr || vgprs == nullptr || lds_bytes == nullptr) return SACENV_E_NULL;
  if (n < 0) return SACENV_E_SIZE;
  int nb = 0;
  hipError_t e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_sac_act_lean, kThreads,
                                                               kHandoffLds - sizeof(ActLds));
  if (e != hipSuccess) return (int)e;
  hipFuncAttributes fa{};
  e = hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(k_sac_act_lean));
  if (e != hipSuccess) return (int)e;
  *blocks_per_cu = nb;
  *grid = (n + kActRows - 1) / kActRows;
  *vgprs = fa.numRegs;
  *lds_bytes = kHandoffLds;  // static + the padding at launch
  return SACENV_OK;
}

extern "C" int sacenv_sac_act_handoff(const SacenvSacParams* p, const float* weights, const float* obs,
                                      int32_t n, const float* eps, float* action, const uint32_t* obs_ready,
                                      uint32_t obs_want, uint32_t* act_ready, uint32_t act_value,
                                      int32_t* status, void* stream) {
  if (obs_ready == nullptr || act_ready == nullptr) return SACENV_E_NULL;
  if (obs_want >= 0x80000000u || act_value >= 0x80000000u) return SACENV_E_RANGE;
  return sac_act(p, weights, obs, n, eps, action, nullptr, ActHandoff{obs_ready, obs_want, act_ready, act_value, status},
                 stream);
}

extern "C" int sacenv_sac_learn(const SacenvSacParams* p, float* weights, void* scratch, const float* state,
                                const float* action, const double* reward, const float* new_state,
                                const uint8_t* done, const float* eps1, const float* eps2, int32_t adam_step,
                                float* losses, void* stream) {
  const int rc = check(p);
  if (rc != SACENV_OK) return rc;
  if (weights == nullptr || scratch == nullptr || state == nullptr || action == nullptr || reward == nullptr ||
      new_state == nullptr || done == nullptr || eps1 == nullptr || eps2 == nullptr)
    return SACENV_E_NULL;
  if (adam_step < 1) return SACENV_E_RANGE;
  if (!aligned16(weights) || !aligned16(scratch)) return SACENV_E_SIZE;
  SacArgs a = make_args(p, weights);
  a.s = state;
  a.act = action;
  a.rew = reward;
  a.s2 = new_state;
  a.done = done;
  a.eps1 = eps1;
  a.eps2 = eps2;
  a.losses = losses;
  float* scr = static_cast<float*>(scratch);
  const int64_t tile = (int64_t)kH * p->batch;
  for (int t = 0; t < 4; ++t) {
    a.na[t].h1t = scr + (4 * t + 0) * tile;
    a.na[t].h2t = scr + (4 * t + 1) * tile;
    a.na[t].dz1t = scr + (4 * t + 2) * tile;
    a.na[t].dz2t = scr + (4 * t + 3) * tile;
  }
  a.rows = scr + 16 * tile;
  a.xt = a.rows + (int64_t)F_COUNT * p->batch;
  a.stamps = reinterpret_cast<unsigned long long*>(a.xt + 16 * (int64_t)p->batch);
  // torch.optim.Adam (_multi_tensor_adam): Python-float scalars, cast to f32 in the kernels
  const double b1 = p->adam_beta1, b2 = p->adam_beta2;
  const double bc1 = 1.0 - pow(b1, (double)adam_step), bc2 = 1.0 - pow(b2, (double)adam_step);
  a.lerp_w = (float)(1.0 - b1);
  a.b2 = (float)b2;
  a.omb2 = (float)(1.0 - b2);
  a.bc2s = (float)pow(bc2, 0.5);
  a.eps = (float)p->adam_eps;
  a.nstep_actor = (float)((p->lr_actor / bc1) * -1.0);
  a.nstep_critic = (float)((p->lr_critic / bc1) * -1.0);
  const int nrb = p->batch / kRows;
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(k_sac_rows, dim3(4 * nrb), dim3(kThreads), 0, s, a, 0);
  hipLaunchKernelGGL(k_sac_rows, dim3(6 * nrb), dim3(kThreads), 0, s, a, 1);
  hipLaunchKernelGGL(k_sac_rows, dim3(4 * nrb), dim3(kThreads), 0, s, a, 2);
  hipLaunchKernelGGL(k_sac_update, dim3(kUpdateBlocks), dim3(kThreads), 0, s, a);
  return (int)hipGetLastError();
}
