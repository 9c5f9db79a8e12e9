// sacenv_replay.hip — gfx950 device replay buffer + C ABI (include/sacenv.h).
//
// agent/buffer.py:3-35 on the GPU. The step records of every env are appended
// in env order with the reference's ring rule (index = mem_cntr % mem_size,
// buffer.py:14). Sampling is np.random.choice(min(mem_cntr, mem_size), batch)
// (buffer.py:27), which numpy's legacy RandomState computes as a
// masked-rejection randint on 32-bit MT19937 words. One wave draws the whole
// batch: 64 candidate words per window, a ballot keeps the accepted ones in
// order, and the stream advances by exactly the words numpy consumes. The
// gather of the sampled rows is a plain element-parallel copy.
//
// The buffer's arrays are row-major per transition (the policy reads whole
// rows); the store is coalesced along the flattened row-major element index.

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sacenv.h"

namespace {

constexpr int kWave = 64;
constexpr int kMtN = SACENV_MT_N;
constexpr int kMtM = 397;
constexpr uint32_t kMtUpper = 0x80000000u;
constexpr uint32_t kMtLower = 0x7fffffffu;
constexpr uint32_t kMtMatrixA = 0x9908b0dfu;

#include "mt19937.h"

__host__ __device__ inline int64_t align256(int64_t x) { return (x + 255) / 256 * 256; }

__host__ __device__ inline void replay_layout(const SacenvReplayParams& p, SacenvReplayLayout* o) {
  const int64_t M = p.mem_size;
  int64_t off = 0;
  o->state = off;
  off = align256(off + 4 * M * p.obs_dim);
  o->new_state = off;
  off = align256(off + 4 * M * p.obs_dim);
  o->action = off;
  off = align256(off + 4 * M * p.act_dim);
  o->reward = off;
  off = align256(off + 8 * M);
  o->terminal = off;
  off = align256(off + M);
  o->mem_cntr = off;
  off += 256;
  o->mt_key = off;
  off = align256(off + 4 * kMtN);
  o->mt_pos = off;
  off += 256;
  o->total_bytes = off;
}

struct RB {
  char* b;
  SacenvReplayLayout L;
  __device__ float* state() const { return reinterpret_cast<float*>(b + L.state); }
  __device__ float* new_state() const { return reinterpret_cast<float*>(b + L.new_state); }
  __device__ float* action() const { return reinterpret_cast<float*>(b + L.action); }
  __device__ double* reward() const { return reinterpret_cast<double*>(b + L.reward); }
  __device__ uint8_t* terminal() const { return reinterpret_cast<uint8_t*>(b + L.terminal); }
  __device__ int64_t* cntr() const { return reinterpret_cast<int64_t*>(b + L.mem_cntr); }
  __device__ uint32_t* key() const { return reinterpret_cast<uint32_t*>(b + L.mt_key); }
  __device__ int32_t* pos() const { return reinterpret_cast<int32_t*>(b + L.mt_pos); }
};

struct DrawLds {
  uint32_t blk[2][kMtN];
};

__global__ void __launch_bounds__(kWave) k_rb_init(RB r, uint32_t seed) {
  if (threadIdx.x != 0) return;
  uint32_t x = seed;  // init_genrand (numpy RandomState._legacy_seeding)
  for (int i = 0; i < kMtN; ++i) {
    r.key()[i] = x;
    x = 1812433253u * (x ^ (x >> 30)) + (uint32_t)(i + 1);
  }
  *r.pos() = kMtN;
  *r.cntr() = 0;
}

// store_transition for rows [0, n): row i -> (mem_cntr + i) % M. Rows that a
// later row of the same call overwrites (i < n - M) are skipped, so the ring
// ends exactly as n sequential calls leave it. Element-parallel over the
// (n - first) x (D + A + 1) stored columns with 32-bit index math. mem_cntr
// advances in a second launch (k_rb_advance), after every workgroup has read
// it: stream order instead of a grid-wide atomic (one word takes ~90
// returning atomics/µs) or an agent-scope acq_rel fence per workgroup.
__global__ void __launch_bounds__(256) k_rb_store(SacenvReplayParams p, RB r, int64_t n, int64_t offset,
                                                  const float* __restrict__ state,
                                                  const float* __restrict__ action,
                                                  const void* __restrict__ reward,
                                                  const float* __restrict__ new_state,
                                                  const float* __restrict__ final_state,
                                                  const uint8_t* __restrict__ code,
                                                  uint8_t* __restrict__ last_term) {
  const int64_t M = p.mem_size, c0 = *r.cntr() + offset;
  const int64_t first = n > M ? n - M : 0;
  const uint32_t rows = (uint32_t)(n - first);
  const uint32_t base = (uint32_t)((c0 + first) % M);  // ring row of stored row 0
  const uint32_t D = (uint32_t)p.obs_dim, A = (uint32_t)p.act_dim, Mu = (uint32_t)M;
  const uint32_t nD = rows * D, nA = rows * A, stored = nD + nA + rows;
  // with last_term, rows a later row overwrites still update their env's byte
  const uint32_t total = stored + (last_term != nullptr ? (uint32_t)first : 0u);
  for (uint32_t q = blockIdx.x * blockDim.x + threadIdx.x; q < total; q += gridDim.x * blockDim.x) {
    if (q < nD) {
      const uint32_t j = q / D, k = q - j * D;
      uint32_t row = base + j;
      row = row >= Mu ? row - Mu : row;
      const int64_t src = (first + j) * (int64_t)D + k;
      r.state()[(int64_t)row * D + k] = state[src];
      const float* ns = (final_state != nullptr && code[first + j] != 0) ? final_state : new_state;
      r.new_state()[(int64_t)row * D + k] = ns[src];
    } else if (q < nD + nA) {
      const uint32_t qq = q - nD, j = qq / A, k = qq - j * A;
      uint32_t row = base + j;
      row = row >= Mu ? row - Mu : row;
      r.action()[(int64_t)row * A + k] = action[(first + j) * (int64_t)A + k];
    } else if (q < stored) {
      const uint32_t j = q - nD - nA;
      uint32_t row = base + j;
      row = row >= Mu ? row - Mu : row;
      const int64_t i = first + j;
      r.reward()[row] = p.reward_f32 ? (double)static_cast<const float*>(reward)[i]
                                     : static_cast<const double*>(reward)[i];
      uint32_t cd = code[i];
      if (last_term != nullptr) {
        // main.py:83 tests info['termination'], which only the termination
        // chain writes (boat_env.py:84-105) and reset never clears (:120-126):
        // codes 1..5 overwrite env i's last termination, others keep it
        if (cd >= 1u && cd <= 5u) last_term[i] = (uint8_t)cd;
        else cd = last_term[i];
      }
      r.terminal()[row] = (uint8_t)((p.terminal_mask >> (cd < 31 ? cd : 31)) & 1u);
    } else {
      const int64_t i = q - stored;  // a row the ring drops: only its env's byte
      const uint32_t cd = code[i];
      if (cd >= 1u && cd <= 5u) last_term[i] = (uint8_t)cd;
    }
  }
}

__global__ void k_rb_advance(RB r, int64_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *r.cntr() += n;  // buffer.py:22
}

// np.random.choice(max_mem, batch) with replace=True, p=None: numpy legacy
// randint(0, max_mem) -> masked rejection on 32-bit words (rng = max_mem-1;
// rng == 0 draws nothing). One wave; words in order, accepted words fill the
// batch in order, the stream stops after the batch-th accepted word.
__global__ void __launch_bounds__(kWave) k_rb_draw(SacenvReplayParams p, RB r, int batch,
                                                   int64_t* __restrict__ idx) {
  __shared__ DrawLds l;
  const int lane = threadIdx.x;
  const int64_t cnt = *r.cntr();
  const int64_t max_mem = cnt < p.mem_size ? cnt : p.mem_size;
  const uint64_t rng = (uint64_t)(max_mem - 1);
  if (rng == 0) {  // numpy: off + 0, no words consumed
    for (int i = lane; i < batch; i += kWave) idx[i] = 0;
    return;
  }
  uint32_t mask = (uint32_t)rng;
  mask |= mask >> 1;
  mask |= mask >> 2;
  mask |= mask >> 4;
  mask |= mask >> 8;
  mask |= mask >> 16;
  MtStream st;
  st.gkey = r.key();
  st.pos = *r.pos();
  st.cur = 0;
  st.loaded = false;
  st.nxt_valid = false;
  st.advanced = false;
  int filled = 0;
  while (filled < batch) {
    const uint32_t w = mt_fetch(st, l, lane) & mask;
    const bool acc = w <= (uint32_t)rng;
    const unsigned long long bal = __ballot(acc);
    const int before = __popcll(bal & ((1ull << lane) - 1ull));
    const int take = batch - filled;
    if (acc && before < take) idx[filled + before] = (int64_t)w;
    const int total = __popcll(bal);
    if (total >= take) {
      // the take-th accepted word ends the draw: consume up to and including it
      unsigned long long b = bal;
      for (int t = 1; t < take; ++t) b &= b - 1ull;
      st.pos += __ffsll((long long)b);
      filled = batch;
    } else {
      st.pos += kWave;
      filled += total;
    }
  }
  mt_finish(st, l, r.pos(), lane);
}

// Sharded rows (sacenv_replay_sample_shard): ring row p holds the transition
// with the latest global sequence number s <= mem_cntr - 1, s = p (mod M); this
// shard wrote it iff (s mod period) is in [lo, hi). Rows of other shards come
// out as zero bits.
struct Shard {
  int64_t period, lo, hi;  // period 0: every row is this shard's
};
__device__ __forceinline__ bool owns(const Shard& sh, int64_t cnt, int64_t M, int64_t row) {
  if (sh.period == 0) return true;
  const int64_t s = row + M * ((cnt - 1 - row) / M);
  const int64_t u = s % sh.period;
  return u >= sh.lo && u < sh.hi;
}

__global__ void __launch_bounds__(256) k_rb_gather(SacenvReplayParams p, RB r, int batch,
                                                   const int64_t* __restrict__ idx, float* __restrict__ st,
                                                   float* __restrict__ ac, double* __restrict__ rw,
                                                   float* __restrict__ ns, uint8_t* __restrict__ tm, Shard sh) {
  const int D = p.obs_dim, A = p.act_dim;
  const int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t nd = (int64_t)batch * D, na = (int64_t)batch * A;
  const int64_t cnt = *r.cntr(), M = p.mem_size;
  if (q < nd) {
    const int64_t i = q / D, k = q - i * D, row = idx[i];
    const bool own = owns(sh, cnt, M, row);
    if (st) st[q] = own ? r.state()[row * D + k] : 0.f;
    if (ns) ns[q] = own ? r.new_state()[row * D + k] : 0.f;
  } else if (q < nd + na) {
    const int64_t qq = q - nd, i = qq / A, k = qq - i * A, row = idx[i];
    if (ac) ac[qq] = owns(sh, cnt, M, row) ? r.action()[row * A + k] : 0.f;
  } else if (q < nd + na + batch) {
    const int64_t i = q - nd - na, row = idx[i];
    const bool own = owns(sh, cnt, M, row);
    if (rw) rw[i] = own ? r.reward()[row] : 0.0;
    if (tm) tm[i] = own ? r.terminal()[row] : (uint8_t)0;
  }
}

// ---------------------------------------------------------------------------
// The staged sampler (sacenv_replay_sample_staged): the pooled buffer of
// main.py:81-90 -- every rank's envs storing one transition each per step, one
// learn() (sample_buffer, buffer.py:24-35) after every step -- sampled straight
// out of the segments of transition rows the persistent step launch wrote
// (sacenv_boat_segment's `trans`), with no store into a ring. A ring of M rows
// that takes `period` rows per step holds the last M sequence numbers; with M <=
// seg * period every row learn k can reach lies in this segment's or the
// previous segment's rows, so the two staged segments ARE the ring.

// The persistent info['termination'] (main.py:83, boat_env.py:24-32,84-105,
// 120-126) per row: codes 1..5 overwrite the env's last termination, 0 and 6
// keep it; terminal = (terminal_mask >> last) & 1. One thread per 4 envs walks
// the segment's rows in order: u32 loads (4 envs' codes, coalesced across the
// threads of a row), kChunk rows in flight before the serial carry.
__global__ void __launch_bounds__(256) k_rb_stage_terminal(const uint8_t* __restrict__ rows, int64_t row_bytes,
                                                           int64_t term_off, int n_steps, int n, int n_pad,
                                                           uint32_t terminal_mask, uint8_t* __restrict__ last_term,
                                                           uint8_t* __restrict__ terminal) {
  constexpr int kChunk = 32;
  const int e0 = 4 * (blockIdx.x * blockDim.x + threadIdx.x);
  if (e0 >= n) return;
  uint32_t lt[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) lt[q] = e0 + q < n ? last_term[e0 + q] : 0u;
  for (int j0 = 0; j0 < n_steps; j0 += kChunk) {
    uint32_t c[kChunk];
#pragma unroll
    for (int j = 0; j < kChunk; ++j)
      c[j] = j0 + j < n_steps ? *reinterpret_cast<const uint32_t*>(rows + (int64_t)(j0 + j) * row_bytes + term_off + e0)
                              : 0u;
#pragma unroll
    for (int j = 0; j < kChunk; ++j) {
      uint32_t out = 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t cq = (c[j] >> (8 * q)) & 0xFFu;
        lt[q] = (cq >= 1u && cq <= 5u) ? cq : lt[q];
        out |= ((terminal_mask >> lt[q]) & 1u) << (8 * q);
      }
      if (j0 + j < n_steps) *reinterpret_cast<uint32_t*>(terminal + (int64_t)(j0 + j) * n_pad + e0) = out;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (e0 + q < n) last_term[e0 + q] = (uint8_t)lt[q];
}

// mt19937_gen over one block with a whole workgroup (>= 227 threads): the three
// lane-parallel phases of mt_twist_wave, one word per thread each.
__device__ __forceinline__ void mt_twist_block(const uint32_t* __restrict__ o, uint32_t* __restrict__ n, int tid) {
  constexpr int kD = kMtN - kMtM;  // 227
  if (tid < kD) n[tid] = mt_mix(o[tid], o[tid + 1], o[tid + kMtM]);
  __syncthreads();
  if (tid < kD) n[kD + tid] = mt_mix(o[kD + tid], o[kD + tid + 1], n[tid]);
  __syncthreads();
  if (tid < kMtN - 1 - 2 * kD) n[2 * kD + tid] = mt_mix(o[2 * kD + tid], o[2 * kD + tid + 1], n[kD + tid]);
  __syncthreads();
  if (tid == 0) n[kMtN - 1] = mt_mix(o[kMtN - 1], n[0], n[kMtM - 1]);
  __syncthreads();
}

// n_batches consecutive np.random.choice(min(cntr_k, M), batch) calls on one
// stream, cntr_k = cntr0 + (k + 1) * period (learn k follows step k's stores).
// One workgroup of kDrawThreads: a whole 624-word block is tempered and tested
// at once (thread i: word i), accepted words are ranked with a ballot per wave
// and a prefix over the waves; a batch that completes inside the block ends at
// its last accepted word, and the next batch re-tests the block from there
// (its range may differ while cntr < M). The stream advances exactly as numpy's.
constexpr int kDrawThreads = 1024;
__global__ void __launch_bounds__(kDrawThreads) k_rb_draw_many(SacenvReplayParams p, RB r, int batch, int nb,
                                                               int64_t cntr0, int64_t period,
                                                               int64_t* __restrict__ idx) {
  __shared__ uint32_t blk[2][kMtN];
  __shared__ int wcnt[kDrawThreads / kWave];
  __shared__ int s_end;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  constexpr int kWaves = kDrawThreads / kWave;
  for (int i = tid; i < kMtN; i += kDrawThreads) blk[0][i] = r.key()[i];
  int cur = 0, pos = *r.pos();
  bool advanced = false;
  __syncthreads();
  int k = 0, filled = 0;
  while (k < nb) {
    const int64_t c = cntr0 + (int64_t)(k + 1) * period;
    const int64_t max_mem = c < p.mem_size ? c : p.mem_size;
    const uint32_t rng = (uint32_t)(max_mem - 1);
    if (c < batch || rng == 0u) {  // learn() returns before sampling (continuous_agent.py:97-98),
      // or numpy's off + 0: no words consumed
      for (int i = tid; i < batch; i += kDrawThreads) idx[(int64_t)k * batch + i] = c < batch ? -1 : 0;
      ++k;
      continue;
    }
    uint32_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    if (pos >= kMtN) {
      mt_twist_block(blk[cur], blk[cur ^ 1], tid);
      cur ^= 1;
      pos = 0;
      advanced = true;
    }
    const bool valid = tid >= pos && tid < kMtN;
    const uint32_t w = valid ? (mt_temper(blk[cur][tid]) & mask) : 0u;
    const bool acc = valid && w <= rng;
    const unsigned long long bal = __ballot(acc);
    if (lane == 0) wcnt[wv] = __popcll(bal);
    __syncthreads();
    int excl = 0, total = 0;
#pragma unroll
    for (int q = 0; q < kWaves; ++q) {
      const int v = wcnt[q];
      excl += q < wv ? v : 0;
      total += v;
    }
    const int rank = excl + __popcll(bal & ((1ull << lane) - 1ull));
    const int take = batch - filled;
    if (acc && rank < take) idx[(int64_t)k * batch + filled + rank] = (int64_t)w;
    if (total >= take) {  // the take-th accepted word ends batch k
      if (acc && rank == take - 1) s_end = tid;
      __syncthreads();
      pos = s_end + 1;
      ++k;
      filled = 0;
    } else {
      filled += total;
      pos = kMtN;
    }
    __syncthreads();  // wcnt / s_end are rewritten by the next round
  }
  if (advanced)
    for (int i = tid; i < kMtN; i += kDrawThreads) r.key()[i] = blk[cur][i];
  if (tid == 0) *r.pos() = pos;
}

struct Staged {
  const char* cur;         // rows of segment g
  const char* prev;        // rows of segment g - 1 (g = 0: row seg-1 holds the reset obs, term 0)
  const uint8_t* tcur;     // k_rb_stage_terminal's terminal bytes [seg][n_pad] of segment g
  const uint8_t* tprev;    // ... of segment g - 1
  int64_t row_bytes, period, offset, g;
  int n, n_pad, seg, exp2;
  float first[SACENV_OBS_DIM];
};

// One thread per sampled row (batch b, row i): ring row idx -> the sequence
// number it holds at learn b (the latest s = idx mod M below cntr_b) -> (step,
// global env); this rank's rows are read from the staged segments: s' the row's
// obs, s the previous step's s' (or the fresh-Boat obs where that step ended:
// first_obs, exp 2 with that row's obs3_next), the reward and action, the
// terminal byte. Output per batch, 32-bit words (sample_many's packing):
// reward f64 [B] | state [B][11] | new_state [B][11] | action [B] | terminal [B];
// rows of other ranks are zero words, so a SUM all-reduce assembles the batch.
__global__ void __launch_bounds__(256) k_rb_gather_staged(SacenvReplayParams p, Staged S, int batch, int nb,
                                                          const int64_t* __restrict__ idx,
                                                          uint32_t* __restrict__ words, int64_t per) {
  constexpr int D = SACENV_OBS_DIM;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)batch * nb) return;
  const int b = (int)(t / batch), i = (int)(t - (int64_t)b * batch);
  const int64_t M = p.mem_size;
  const int64_t cntr = (S.g * S.seg + b + 1) * S.period;
  const int64_t row = idx[t];  // -1: no learn at this step (fewer rows than a batch)
  const int64_t s = row < 0 ? 0 : row + M * ((cntr - 1 - row) / M);
  const int64_t q = s / S.period, u = s - q * S.period;
  const bool own = row >= 0 && u >= S.offset && u < S.offset + S.n;
  uint32_t* const W = words + (int64_t)b * per;
  float sn[D], sv[D];
  float rw = 0.f, ac = 0.f;
  uint32_t tm = 0u;
#pragma unroll
  for (int k = 0; k < D; ++k) sn[k] = sv[k] = 0.f;
  if (own) {
    const int e = (int)(u - S.offset);
    int64_t j = q - S.g * S.seg;  // >= -seg + 1 (M <= seg * period)
    const bool in_cur = j >= 0;
    j = in_cur ? j : j + S.seg;
    const char* R = (in_cur ? S.cur : S.prev) + j * S.row_bytes;
    // the previous step's row: same segment, or the last row of the previous one
    const char* P = j > 0 ? R - S.row_bytes : S.prev + (int64_t)(S.seg - 1) * S.row_bytes;
    const float* rs = reinterpret_cast<const float*>(R) + (int64_t)e * D;
    const float* ps = reinterpret_cast<const float*>(P) + (int64_t)e * D;
    const int64_t np = S.n_pad;
    rw = reinterpret_cast<const float*>(R + 44 * np)[e];
    ac = reinterpret_cast<const float*>(R + 48 * np)[e];
    tm = (in_cur ? S.tcur : S.tprev)[j * np + e];
    const bool pdone = reinterpret_cast<const uint8_t*>(P + 52 * np)[e] != 0;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      sn[k] = rs[k];
      sv[k] = pdone ? S.first[k] : ps[k];
    }
    if (S.exp2 && pdone) sv[3] = reinterpret_cast<const float*>(P + 53 * np)[e];
  }
  const double r64 = (double)rw;
  uint64_t rb;
  __builtin_memcpy(&rb, &r64, 8);
  W[2 * i] = (uint32_t)rb;
  W[2 * i + 1] = (uint32_t)(rb >> 32);
  uint32_t* const st = W + 2 * batch + (int64_t)i * D;
  uint32_t* const ns = W + 2 * batch + (int64_t)batch * D + (int64_t)i * D;
#pragma unroll
  for (int k = 0; k < D; ++k) {
    st[k] = __float_as_uint(sv[k]);
    ns[k] = __float_as_uint(sn[k]);
  }
  W[2 * batch + 2 * (int64_t)batch * D + i] = __float_as_uint(ac);
  W[2 * batch + 2 * (int64_t)batch * D + batch + i] = tm;
}

int check_replay(const SacenvReplayParams* p) {
  if (p == nullptr) return SACENV_E_NULL;
  if (p->mem_size <= 0 || p->mem_size > 0x7FFFFFFFLL || p->obs_dim <= 0 || p->act_dim <= 0)
    return SACENV_E_SIZE;  // 32-bit ring rows; randint on 32-bit words
  return SACENV_OK;
}

RB make_rb(const SacenvReplayParams& p, void* arena) {
  RB r;
  r.b = static_cast<char*>(arena);
  replay_layout(p, &r.L);
  return r;
}

int status() {
  const hipError_t err = hipGetLastError();
  return err == hipSuccess ? SACENV_OK : (int)err;
}

}  // namespace

extern "C" {

int sacenv_replay_layout(const SacenvReplayParams* p, SacenvReplayLayout* out) {
  const int rc = check_replay(p);
  if (rc) return rc;
  if (out == nullptr) return SACENV_E_NULL;
  replay_layout(*p, out);
  return SACENV_OK;
}

int sacenv_replay_init(const SacenvReplayParams* p, void* arena, uint32_t seed, void* stream) {
  const int rc = check_replay(p);
  if (rc) return rc;
  if (arena == nullptr) return SACENV_E_NULL;
  hipLaunchKernelGGL(k_rb_init, dim3(1), dim3(kWave), 0, (hipStream_t)stream, make_rb(*p, arena), seed);
  return status();
}

static int store(const SacenvReplayParams* p, void* arena, int64_t n, int64_t offset, int64_t advance,
                 const float* state, const float* action, const void* reward, const float* new_state,
                 const float* final_state, const uint8_t* code, uint8_t* last_term, void* stream) {
  int rc = check_replay(p);
  if (rc) return rc;
  if (n < 0) return SACENV_E_SIZE;
  if (n == 0 && advance == n) return SACENV_OK;
  if (!arena || !state || !action || !reward || !new_state || !code) return SACENV_E_NULL;
  const int64_t rows = n > p->mem_size ? p->mem_size : n;
  const int64_t total = rows * ((int64_t)p->obs_dim + p->act_dim + 1) + (last_term ? n - rows : 0);
  if (total >= (1LL << 32)) return SACENV_E_SIZE;  // 32-bit element index per call
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const RB r = make_rb(*p, arena);
  if (n > 0) {
    hipLaunchKernelGGL(k_rb_store, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *p, r, n, offset,
                       state, action, reward, new_state, final_state, code, last_term);
    if ((rc = status())) return rc;
  }
  hipLaunchKernelGGL(k_rb_advance, dim3(1), dim3(kWave), 0, (hipStream_t)stream, r, advance);
  return status();
}

int sacenv_replay_store_env(const SacenvReplayParams* p, void* arena, int64_t n, const float* state,
                            const float* action, const void* reward, const float* new_state,
                            const float* final_state, const uint8_t* code, uint8_t* last_term,
                            void* stream) {
  return store(p, arena, n, 0, n, state, action, reward, new_state, final_state, code, last_term, stream);
}

int sacenv_replay_store_shard(const SacenvReplayParams* p, void* arena, int64_t n, int64_t offset, int64_t period,
                              const float* state, const float* action, const void* reward, const float* new_state,
                              const float* final_state, const uint8_t* code, uint8_t* last_term, void* stream) {
  if (p == nullptr) return SACENV_E_NULL;
  if (offset < 0 || n < 0 || period <= 0 || offset + n > period || n > p->mem_size) return SACENV_E_RANGE;
  return store(p, arena, n, offset, period, state, action, reward, new_state, final_state, code, last_term, stream);
}

int sacenv_replay_store(const SacenvReplayParams* p, void* arena, int64_t n, const float* state,
                        const float* action, const void* reward, const float* new_state,
                        const float* final_state, const uint8_t* code, void* stream) {
  return sacenv_replay_store_env(p, arena, n, state, action, reward, new_state, final_state, code,
                                 nullptr, stream);
}

static int sample(const SacenvReplayParams* p, void* arena, int32_t batch, int64_t stored, int64_t* idx,
                  float* state, float* action, double* reward, float* new_state, uint8_t* terminal,
                  const Shard& sh, void* stream) {
  int rc = check_replay(p);
  if (rc) return rc;
  if (batch < 0) return SACENV_E_SIZE;
  if (stored <= 0) return SACENV_E_SIZE;  // np.random.choice(0, n) raises
  if (arena == nullptr || idx == nullptr) return SACENV_E_NULL;
  if (batch == 0) return SACENV_OK;
  const RB r = make_rb(*p, arena);
  hipLaunchKernelGGL(k_rb_draw, dim3(1), dim3(kWave), 0, (hipStream_t)stream, *p, r, batch, idx);
  if ((rc = status())) return rc;
  const int64_t total = (int64_t)batch * (p->obs_dim + p->act_dim + 1);
  hipLaunchKernelGGL(k_rb_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *p,
                     r, batch, idx, state, action, reward, new_state, terminal, sh);
  return status();
}

int sacenv_replay_sample(const SacenvReplayParams* p, void* arena, int32_t batch, int64_t stored,
                         int64_t* idx, float* state, float* action, double* reward, float* new_state,
                         uint8_t* terminal, void* stream) {
  return sample(p, arena, batch, stored, idx, state, action, reward, new_state, terminal, Shard{0, 0, 0}, stream);
}

int sacenv_replay_sample_shard(const SacenvReplayParams* p, void* arena, int32_t batch, int64_t stored,
                               int64_t offset, int64_t n, int64_t period, int64_t* idx, float* state,
                               float* action, double* reward, float* new_state, uint8_t* terminal,
                               void* stream) {
  if (offset < 0 || n < 0 || period <= 0 || offset + n > period) return SACENV_E_RANGE;
  return sample(p, arena, batch, stored, idx, state, action, reward, new_state, terminal,
                Shard{period, offset, offset + n}, stream);
}

static int check_staged(const SacenvReplayParams* p, const SacenvStagedParams* sp) {
  int rc = check_replay(p);
  if (rc) return rc;
  if (sp == nullptr) return SACENV_E_NULL;
  if (p->obs_dim != SACENV_OBS_DIM || p->act_dim != 1) return SACENV_E_SIZE;  // the boat's rows
  if (sp->n <= 0 || sp->n_pad < sp->n || (sp->n_pad & 63) != 0 || sp->seg <= 0) return SACENV_E_SIZE;
  if (sp->offset < 0 || sp->period <= 0 || sp->offset + sp->n > sp->period) return SACENV_E_RANGE;
  return SACENV_OK;
}

static int64_t staged_row_bytes(const SacenvStagedParams* sp) {
  return (int64_t)(sp->experiment == 2 ? SACENV_TRANS_BYTES_EXP2 : SACENV_TRANS_BYTES) * sp->n_pad;
}

int sacenv_replay_stage_terminal(const SacenvReplayParams* p, const SacenvStagedParams* sp, const void* rows,
                                 int32_t n_steps, uint8_t* last_term, uint8_t* terminal, void* stream) {
  int rc = check_staged(p, sp);
  if (rc) return rc;
  if (n_steps < 0 || n_steps > sp->seg) return SACENV_E_SIZE;
  if (!rows || !last_term || !terminal) return SACENV_E_NULL;
  if (n_steps == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_rb_stage_terminal, dim3((unsigned)((sp->n + 1023) / 1024)), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const uint8_t*>(rows), staged_row_bytes(sp), (int64_t)52 * sp->n_pad, n_steps, sp->n,
                     sp->n_pad, p->terminal_mask, last_term, terminal);
  return status();
}

int sacenv_replay_sample_staged(const SacenvReplayParams* p, void* arena, const SacenvStagedParams* sp, int64_t g,
                                const void* rows_cur, const uint8_t* term_cur, const void* rows_prev,
                                const uint8_t* term_prev, int32_t batch, int32_t n_batches, int64_t* idx,
                                uint32_t* words, void* stream) {
  int rc = check_staged(p, sp);
  if (rc) return rc;
  if (g < 0 || batch < 0 || n_batches < 0 || n_batches > sp->seg) return SACENV_E_SIZE;
  // every row learn k can reach lies in segments g and g-1 (and a row's predecessor too)
  if (p->mem_size > (int64_t)sp->seg * sp->period) return SACENV_E_RANGE;
  if (!arena || !rows_cur || !term_cur || !rows_prev || !term_prev || !idx || !words) return SACENV_E_NULL;
  if (batch == 0 || n_batches == 0) return SACENV_OK;
  if ((g * sp->seg + 1) * sp->period > (int64_t)1 << 62) return SACENV_E_RANGE;
  const RB r = make_rb(*p, arena);
  hipLaunchKernelGGL(k_rb_draw_many, dim3(1), dim3(kDrawThreads), 0, (hipStream_t)stream, *p, r, batch, n_batches,
                     g * sp->seg * sp->period, sp->period, idx);
  if ((rc = status())) return rc;
  Staged S;
  S.cur = static_cast<const char*>(rows_cur);
  S.prev = static_cast<const char*>(rows_prev);
  S.tcur = term_cur;
  S.tprev = term_prev;
  S.row_bytes = staged_row_bytes(sp);
  S.period = sp->period;
  S.offset = sp->offset;
  S.g = g;
  S.n = sp->n;
  S.n_pad = sp->n_pad;
  S.seg = sp->seg;
  S.exp2 = sp->experiment == 2;
  for (int k = 0; k < SACENV_OBS_DIM; ++k) S.first[k] = sp->first_obs[k];
  const int64_t total = (int64_t)batch * n_batches;
  const int64_t per = (int64_t)batch * (2 * SACENV_OBS_DIM + 1 + 3);
  hipLaunchKernelGGL(k_rb_gather_staged, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     *p, S, batch, n_batches, idx, words, per);
  return status();
}

}  // extern "C"
