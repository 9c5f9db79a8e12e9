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
// returning atomics/µs) or an agent-scope acq_rel fence per workgroup. With the
// count from the host (host_cntr >= 0) no workgroup reads it, so the first one
// writes the advanced count and the second launch goes (one fixed launch cost,
// ~5 us, per stored step).
__global__ void __launch_bounds__(256) k_rb_store(SacenvReplayParams p, RB r, int64_t host_cntr, int64_t advance,
                                                  int64_t n, int64_t offset,
                                                  const float* __restrict__ state,
                                                  const float* __restrict__ action,
                                                  const void* __restrict__ reward,
                                                  const float* __restrict__ new_state,
                                                  const float* __restrict__ final_state,
                                                  const uint8_t* __restrict__ code,
                                                  uint8_t* __restrict__ last_term) {
  const int64_t M = p.mem_size, c0 = (host_cntr >= 0 ? host_cntr : *r.cntr()) + offset;
  if (host_cntr >= 0 && blockIdx.x == 0 && threadIdx.x == 0) *r.cntr() = host_cntr + advance;  // buffer.py:22
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
// rng == 0 draws nothing); words in order, accepted words fill the batch in
// order, the stream stops after the batch-th accepted word: k_rb_draw_many below
// (one 1 024-thread workgroup).

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
  // (an index outside the ring -- a caller's, sacenv_replay_gather -- reads nothing: zero bits)
  if (q < nd) {
    const int64_t i = q / D, k = q - i * D, row = idx[i];
    const bool own = row >= 0 && row < M && owns(sh, cnt, M, row);
    if (st) st[q] = own ? r.state()[row * D + k] : 0.f;
    if (ns) ns[q] = own ? r.new_state()[row * D + k] : 0.f;
  } else if (q < nd + na) {
    const int64_t qq = q - nd, i = qq / A, k = qq - i * A, row = idx[i];
    if (ac) ac[qq] = row >= 0 && row < M && owns(sh, cnt, M, row) ? r.action()[row * A + k] : 0.f;
  } else if (q < nd + na + batch) {
    const int64_t i = q - nd - na, row = idx[i];
    const bool own = row >= 0 && row < M && owns(sh, cnt, M, row);
    if (rw) rw[i] = own ? r.reward()[row] : 0.0;
    if (tm) tm[i] = own ? r.terminal()[row] : (uint8_t)0;
  }
}

// ---------------------------------------------------------------------------
// The staged sampler: the pooled buffer of main.py:78-90 -- every rank's envs
// storing one transition each per step, one learn() (sample_buffer,
// buffer.py:24-35) after every step -- sampled out of the rows the persistent
// step launch wrote (sacenv_boat_segment's `stage`), with no ring. A ring of M
// rows that takes `period` rows per step holds the last M sequence numbers;
// with M <= seg * period every row learn k of segment g can reach (and the row
// before it, for s) lies in segment g or g - 1, so two staged segments ARE the
// ring. The index draws depend only on the sampling stream and the counts
// stored, so segment g's are drawn before it steps, and the launch writes only
// the rows some learn will read (sacenv_replay_stage_mark).

struct StagedGeom {
  int64_t period, offset, g;
  int n, n_pad, seg, exp2;
  double r_mem, r_period;  // 1 / mem_size, 1 / period (host IEEE divisions)
};

// floor(x / d) for 0 <= x < 2^52 and 0 < d < 2^31 from the rounded reciprocal rd:
// the double estimate is off by at most one, fixed by one step each way (a 64-bit
// integer division is a ~50-instruction sequence on the GPU)
__device__ __forceinline__ int64_t div_floor(int64_t x, int64_t d, double rd) {
  int64_t q = (int64_t)((double)x * rd);
  q -= q * d > x ? 1 : 0;
  q += (q + 1) * d <= x ? 1 : 0;
  return q;
}

// The staged segment buffers are ENV-MAJOR (round 6): env e's 64-B row of step j of a
// segment at (e x seg + j) x 64, its mark bits in the ceil(seg / 64) words from e x
// that, bit j % 64 -- a row and its predecessor (the row before it: its s) share a
// mark word (one atomic) and mostly a 128-B line.
__device__ __forceinline__ int64_t stage_row(const StagedGeom& G, int e, int64_t j) {
  return ((int64_t)e * G.seg + j) * 64;
}
__device__ __forceinline__ void mark_rows(unsigned long long* __restrict__ marks, const StagedGeom& G, int e,
                                          int64_t j, unsigned long long bits) {
  const int W = (G.seg + 63) / 64;
  atomicOr(&marks[(int64_t)e * W + (j >> 6)], bits << (j & 63));
}

// ring row `row` at learn time (cntr rows stored) -> (global step q, global env u)
__device__ __forceinline__ void resolve(int64_t row, int64_t cntr, int64_t M, const StagedGeom& G, int64_t* q,
                                        int64_t* u) {
  // the latest sequence number = row (mod M) below cntr
  const int64_t s = row + M * div_floor(cntr - 1 - row, M, G.r_mem);
  *q = div_floor(s, G.period, G.r_period);
  *u = s - *q * G.period;
}

// n_batches consecutive np.random.choice(min(cntr_k, M), batch) calls on one
// stream, cntr_k = cntr0 + (k + 1) * period (learn k follows step k's stores),
// learns with cntr_k < batch skipped (continuous_agent.py:97-98: idx = -1, no
// words). The general path (ranges that change between learns): one workgroup;
// a whole 624-word block is tempered and tested at once (thread i: word i),
// accepted words are ranked with a ballot per wave and a prefix over the
// waves; a batch that completes inside the block ends at its last accepted
// word, and the next batch re-tests the block from there.
constexpr int kDrawThreads = 1024;
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

// kSample: one sample_buffer(batch) at the device count (sacenv_replay_sample: no
// learn() skip below batch rows; graph-capturable like the store), else the nb
// learns of a staged segment at counts cntr0 + (k + 1) * period.
template <bool kSample = false>
__global__ void __launch_bounds__(kDrawThreads) k_rb_draw_many(SacenvReplayParams p, RB r, int batch, int nb,
                                                               int64_t cntr0, int64_t period,
                                                               int64_t* __restrict__ idx) {
  __shared__ uint32_t blk[2][kMtN];
  __shared__ int wcnt[kDrawThreads / kWave];
  __shared__ int s_end;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  constexpr int kWaves = kDrawThreads / kWave;
  int cur = 0, pos = *r.pos();
  if (pos < 0) {  // a poisoned stream (a staged draw ran short): draw nothing, keep the poison
    for (int64_t i = tid; i < (int64_t)nb * batch; i += kDrawThreads) idx[i] = -1;
    return;
  }
  for (int i = tid; i < kMtN; i += kDrawThreads) blk[0][i] = r.key()[i];
  bool advanced = false;
  __syncthreads();
  int k = 0, filled = 0;
  while (k < nb) {
    const int64_t c = kSample ? *r.cntr() : cntr0 + (int64_t)(k + 1) * period;
    const int64_t max_mem = c < p.mem_size ? c : p.mem_size;
    const uint32_t rng = (uint32_t)(max_mem - 1);
    const bool skip = !kSample && c < batch;
    if (skip || rng == 0u) {  // learn() returns before sampling, or numpy's off + 0: no words
      for (int i = tid; i < batch; i += kDrawThreads) idx[(int64_t)k * batch + i] = skip ? -1 : 0;
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

// The steady-state path (every learn of the segment draws from the same range
// [0, M)): the accepted words are numbered over the whole stream, word by word,
// so the draws split into (1) the MT blocks the segment may need, generated
// by one wave -- the only sequential part, the recurrence itself; (2) accepted
// words counted per 1 024-word tile, all tiles at once; (3) a prefix over the
// tiles; (4) every tile ranking its accepted words and writing idx[rank] for
// rank < n_batches * batch, the tile holding the last one handing the stream
// on (the block it lies in and the position after it).
constexpr int kTile = 1024, kTileThreads = 256;

// The stream's MT blocks for one segment's draws: block 0 is the block holding
// the next word (the key, or its successor when pos = 624), then one twist per
// block -- the only sequential part of the draws. Thread l (l < 227) owns the
// words l, l + 227 and l + 454 of every block: mt19937_gen's word i depends on
// new word i - 227 from i = 227 on, so the three phases of a twist chain inside
// the thread (w0 = mix(o[l], o[l+1], o[l+397]), w1 = mix(o[l+227], o[l+228], w0),
// w2 = mix(o[l+454], o[l+455], w1); word 623 = mix(o[623], new[0], new[396])),
// and a block costs one LDS round trip (the old block's neighbours) and one
// barrier instead of three dependent phases.
constexpr int kChainThreads = 256;
__global__ void __launch_bounds__(kChainThreads) k_mt_chain(RB r, uint32_t* __restrict__ out, int n_blocks,
                                                            int* __restrict__ ctrl) {
  constexpr int kD = kMtN - kMtM;  // 227
  __shared__ uint32_t buf[2][kMtN];
  const int l = threadIdx.x;
  const int pos = *r.pos();
  if (l == 0) {
    ctrl[2] = 0;                          // no shortfall yet
    ctrl[3] = pos >= kMtN ? 0 : pos;      // p0: the next word's position in block 0 (-1: poisoned)
  }
  if (pos < 0) return;  // a poisoned stream: nothing generated, the draws below draw nothing
  for (int i = l; i < kMtN; i += kChainThreads) {
    const uint32_t v = r.key()[i];
    buf[0][i] = v;
    if (pos < kMtN) out[i] = v;
  }
  __syncthreads();
  int cur = 0;
  for (int b = pos < kMtN ? 1 : 0; b < n_blocks; ++b) {
    const uint32_t* o = buf[cur];
    uint32_t* n = buf[cur ^ 1];
    uint32_t* g = out + (int64_t)b * kMtN;
    if (l < kD) {
      const uint32_t o0 = o[l], o1 = o[l + 1], o397 = o[l + kMtM], o227 = o[l + kD], o228 = o[l + kD + 1];
      const bool has2 = l < kMtN - 1 - 2 * kD;  // words 454..622
      const uint32_t o454 = o[has2 ? l + 2 * kD : 0], o455 = o[has2 ? l + 2 * kD + 1 : 0];
      const uint32_t w0 = mt_mix(o0, o1, o397);
      const uint32_t w1 = mt_mix(o227, o228, w0);
      n[l] = w0;
      g[l] = w0;
      n[l + kD] = w1;
      g[l + kD] = w1;
      if (has2) {
        const uint32_t w2 = mt_mix(o454, o455, w1);
        n[l + 2 * kD] = w2;
        g[l + 2 * kD] = w2;
      } else if (l == kMtN - 1 - 2 * kD) {  // word 623: new[0] (thread 0's w0) redone here, new[396] = w1
        const uint32_t n0 = mt_mix(o[0], o[1], o[kMtM]);
        const uint32_t w2 = mt_mix(o[kMtN - 1], n0, w1);
        n[kMtN - 1] = w2;
        g[kMtN - 1] = w2;
      }
    }
    __syncthreads();
    cur ^= 1;
  }
}

struct DrawPlan {
  const uint32_t* blocks;  // the generated blocks; stream word t is block (p0 + t) / 624, word (p0 + t) % 624
  int p0;                  // position of the stream's next word in block 0 (ctrl[3], set by k_mt_chain)
  int64_t n_words;         // words generated from p0 on
  uint32_t rng, mask;
  int64_t need;            // accepted words wanted: n_batches * batch
  int* tile_cnt;           // [tiles]
  int* tile_off;           // [tiles] exclusive prefix
  int* ctrl;               // [0] tile holding the last wanted word (-1: too few words), [1] total accepted,
                           // [2] 1 = too few words generated (no draw made), [3] p0
};

__device__ __forceinline__ void plan_start(DrawPlan& d, int64_t n_blocks) {
  d.p0 = d.ctrl[3];
  d.n_words = n_blocks * kMtN - d.p0;
}

__device__ __forceinline__ uint32_t plan_word(const DrawPlan& d, int64_t t, bool* acc) {
  const int64_t gp = d.p0 + t;
  const int64_t b = gp / kMtN;
  const uint32_t w = mt_temper(d.blocks[b * kMtN + (gp - b * kMtN)]) & d.mask;
  *acc = t < d.n_words && w <= d.rng;
  return w;
}

__global__ void __launch_bounds__(kTileThreads) k_draw_count(DrawPlan d, int64_t n_blocks) {
  __shared__ int wc[kTileThreads / kWave];
  plan_start(d, n_blocks);
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  if (d.p0 < 0) {  // a poisoned stream: no words (the scan then finds too few, the emit draws nothing)
    if (tid == 0) d.tile_cnt[blockIdx.x] = 0;
    return;
  }
  int c = 0;
#pragma unroll
  for (int q = 0; q < kTile / kTileThreads; ++q) {
    bool acc;
    const int64_t t = t0 + q * kTileThreads + tid;
    if (t < d.n_words) plan_word(d, t, &acc);
    else acc = false;
    c += acc ? 1 : 0;
  }
  // wave sum, then the workgroup's
  for (int o = kWave / 2; o > 0; o >>= 1) c += __shfl_xor(c, o);
  if (lane == 0) wc[wv] = c;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
    for (int i = 0; i < kTileThreads / kWave; ++i) t += wc[i];
    d.tile_cnt[blockIdx.x] = t;
  }
}

__global__ void __launch_bounds__(1024) k_draw_scan(DrawPlan d, int tiles) {
  __shared__ int part[1024 / kWave];
  __shared__ int carry;
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  if (tid == 0) {
    carry = 0;
    d.ctrl[0] = -1;
  }
  __syncthreads();
  for (int base = 0; base < tiles; base += 1024) {
    const int i = base + tid;
    const int v = i < tiles ? d.tile_cnt[i] : 0;
    int x = v;  // inclusive scan in the wave
    for (int o = 1; o < kWave; o <<= 1) {
      const int y = __shfl_up(x, o);
      x += lane >= o ? y : 0;
    }
    if (lane == kWave - 1) part[wv] = x;
    __syncthreads();
    int before = carry;
    for (int w = 0; w < wv; ++w) before += part[w];
    const int excl = before + x - v;
    if (i < tiles) {
      d.tile_off[i] = excl;
      if (excl < d.need && excl + v >= d.need) d.ctrl[0] = i;
    }
    __syncthreads();
    if (tid == 1023) carry = excl + v;
    __syncthreads();
  }
  if (tid == 0) d.ctrl[1] = carry;
}

__global__ void __launch_bounds__(kTileThreads) k_draw_emit(DrawPlan d, RB r, int64_t n_blocks,
                                                              int64_t* __restrict__ idx) {
  __shared__ int wc[kTileThreads / kWave];
  plan_start(d, n_blocks);
  __shared__ int64_t s_end;   // stream position after the last wanted word (this tile only)
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const int last = d.ctrl[0];
  if (last < 0) {  // too few words generated (never at the planned margin): report, draw nothing;
    // the stream position -1 marks the arena (StagedReplay.check raises)
    if (blockIdx.x == 0 && tid == 0) {
      d.ctrl[2] = 1;
      *r.pos() = -1;
    }
    return;
  }
  if ((int)blockIdx.x > last) return;
  const int64_t t0 = (int64_t)blockIdx.x * kTile;
  int run = d.tile_off[blockIdx.x];
  if (tid == 0) s_end = -1;
#pragma unroll
  for (int q = 0; q < kTile / kTileThreads; ++q) {
    const int64_t t = t0 + q * kTileThreads + tid;
    bool acc = false;
    uint32_t w = 0u;
    if (t < d.n_words) w = plan_word(d, t, &acc);
    const unsigned long long bal = __ballot(acc);
    __syncthreads();  // wc of the previous round read
    if (lane == 0) wc[wv] = __popcll(bal);
    __syncthreads();
    int before = 0, total = 0;
#pragma unroll
    for (int i = 0; i < kTileThreads / kWave; ++i) {
      before += i < wv ? wc[i] : 0;
      total += wc[i];
    }
    const int64_t rank = (int64_t)run + before + __popcll(bal & ((1ull << lane) - 1ull));
    if (acc && rank < d.need) idx[rank] = (int64_t)w;
    if (acc && rank == d.need - 1) s_end = d.p0 + t + 1;
    run += total;
  }
  __syncthreads();
  if (s_end >= 0) {  // this tile ends the segment's draws: the stream's state after them
    int64_t b = s_end / kMtN;
    int pos = (int)(s_end - b * kMtN);
    if (pos == 0) {  // block b is not generated yet: keep block b-1, twist first next time
      b -= 1;
      pos = kMtN;
    }
    for (int i = tid; i < kMtN; i += kTileThreads) r.key()[i] = d.blocks[b * kMtN + i];
    if (tid == 0) *r.pos() = pos;
  }
}

// Marks the rows of segment g that a learn will read: every sampled row of
// the learns of segments g and g + 1 (idx_g, idx_n) that lies in segment g on
// this rank, and the row before it (its s). One thread per sampled row.
__global__ void __launch_bounds__(256) k_rb_stage_mark(SacenvReplayParams p, StagedGeom G,
                                                       const int64_t* __restrict__ idx_g,
                                                       const int64_t* __restrict__ idx_n, int batch, int nb,
                                                       unsigned long long* __restrict__ marks, int64_t total) {
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t per = (int64_t)batch * nb;
  if (t >= total) return;
  const bool nxt = t >= per;
  const int64_t tt = nxt ? t - per : t;
  const int64_t row = (nxt ? idx_n : idx_g)[tt];
  if (row < 0) return;  // no learn at that step
  const int k = (int)(tt / batch);
  const int64_t cntr = ((G.g + (nxt ? 1 : 0)) * G.seg + k + 1) * G.period;
  int64_t q, u;
  resolve(row, cntr, p.mem_size, G, &q, &u);
  if (u < G.offset || u >= G.offset + G.n) return;
  const int e = (int)(u - G.offset);
  const int64_t j = q - G.g * G.seg;  // the row's step in segment g (or outside it)
  if (j >= 1 && j < G.seg && (j & 63) != 0) {  // row and predecessor in one word
    mark_rows(marks, G, e, j - 1, 3ull);
    return;
  }
#pragma unroll
  for (int d = 0; d < 2; ++d)  // the row, and its predecessor (s)
    if (j - d >= 0 && j - d < G.seg) mark_rows(marks, G, e, j - d, 1ull);
}

struct StagedRows {
  const char* cur;   // segment g's 64-B rows [n_pad][seg] (env-major)
  const char* prev;  // segment g - 1's (g = 0: its last row holds the reset obs, term 0)
  float first[SACENV_OBS_DIM];
};

// One thread per sampled row (batch b, row i): the ring row -> (step, global
// env) at learn b; this rank's rows are read from the staged segments: s' =
// the row's obs, s = the previous step's s' (or the fresh-Boat obs where that
// step ended: first_obs, exp 2 with that row's obs3_next), reward, action,
// terminal = (terminal_mask >> last_term) & 1. Output per batch, 32-bit words
// (sample_many's packing): reward f64 [B] | state [B][11] | new_state [B][11] |
// action [B] | terminal [B]; other ranks' rows are zero words, so a SUM
// all-reduce assembles the batch.
__global__ void __launch_bounds__(256) k_rb_gather_staged(SacenvReplayParams p, StagedGeom G, StagedRows S,
                                                          int batch, int nb, const int64_t* __restrict__ idx,
                                                          uint32_t* __restrict__ words, int64_t per) {
  constexpr int D = SACENV_OBS_DIM;
  const int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (t >= (int64_t)batch * nb) return;
  const int b = (int)(t / batch), i = (int)(t - (int64_t)b * batch);
  const int64_t row = idx[t];  // -1: no learn at this step (fewer rows than a batch)
  int64_t q = 0, u = -1;
  if (row >= 0) resolve(row, (G.g * G.seg + b + 1) * G.period, p.mem_size, G, &q, &u);
  const bool own = u >= G.offset && u < G.offset + G.n;
  uint32_t* const W = words + (int64_t)b * per;
  float sn[16], sv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) sn[k] = sv[k] = 0.f;
  uint32_t tm = 0u;
  if (own) {
    const int e = (int)(u - G.offset);
    int64_t j = q - G.g * G.seg;  // > -seg (M <= seg * period)
    const bool in_cur = j >= 0;
    j = in_cur ? j : j + G.seg;
    const float4* R = reinterpret_cast<const float4*>((in_cur ? S.cur : S.prev) + stage_row(G, e, j));
    const float4* P = j > 0 ? R - 4 : reinterpret_cast<const float4*>(S.prev + stage_row(G, e, G.seg - 1));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 x = R[k], y = P[k];
      sn[4 * k] = x.x, sn[4 * k + 1] = x.y, sn[4 * k + 2] = x.z, sn[4 * k + 3] = x.w;
      sv[4 * k] = y.x, sv[4 * k + 1] = y.y, sv[4 * k + 2] = y.z, sv[4 * k + 3] = y.w;
    }
    const bool pdone = (__float_as_uint(sv[13]) & 0xFFu) != 0u;
    const float o3 = sv[14];
#pragma unroll
    for (int k = 0; k < D; ++k) sv[k] = pdone ? S.first[k] : sv[k];
    if (G.exp2 && pdone) sv[3] = o3;
    tm = (p.terminal_mask >> ((__float_as_uint(sn[13]) >> 8) & 0xFFu)) & 1u;
  }
  const double r64 = (double)sn[11];
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
  W[2 * batch + 2 * (int64_t)batch * D + i] = __float_as_uint(sn[12]);
  W[2 * batch + 2 * (int64_t)batch * D + batch + i] = tm;
}

// ---------------------------------------------------------------------------
// The counter-based sampler (sacenv_replay_stage_draw_ctr). Each learn still
// samples np.random.choice(min(c, M), batch)'s distribution -- `batch` rows
// uniform with replacement over the rows stored -- but from Philox4x64-10
// (Salmon, Moraes, Dror, Shaw, SC'11; numpy ships it as np.random.Philox)
// keyed by the seed and counted by (draw, learn, attempt) instead of one
// MT19937 stream: every draw of every learn is independent of the others, so a
// segment's seg x batch draws run at once -- no 624-word chain that one
// workgroup has to walk -- and the thread that draws a row also marks it.
__device__ __forceinline__ void philox4x64_10(uint64_t c[4], uint64_t k0, uint64_t k1) {
  constexpr uint64_t kM0 = 0xD2E7470EE14C6C93ull, kM1 = 0xCA5A826395121157ull;  // multipliers
  constexpr uint64_t kW0 = 0x9E3779B97F4A7C15ull, kW1 = 0xBB67AE8584CAA73Bull;  // Weyl key bumps
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t hi0 = __umul64hi(kM0, c[0]), lo0 = kM0 * c[0];
    const uint64_t hi1 = __umul64hi(kM1, c[2]), lo1 = kM1 * c[2];
    const uint64_t n0 = hi1 ^ c[1] ^ k0, n2 = hi0 ^ c[3] ^ k1;
    c[0] = n0;
    c[1] = lo1;
    c[2] = n2;
    c[3] = lo0;
    k0 += kW0;
    k1 += kW1;
  }
}

// Draw i of global learn L over [0, rng]: word i % 4 of the Philox4x64-10 blocks at
// counters (i / 4, L, j, 0) under key (seed, 0), j = 0, 1, ...: the first whose bits
// under `mask` (the smallest 2^k - 1 >= rng) are <= rng -- numpy's masked rejection.
// One block serves four draws (`blk`, the block at j = 0 of counter c): a retry (each
// word fails with probability < 1/2) takes the draw's word of the next block.
__device__ __forceinline__ int64_t ctr_draw4(uint64_t seed, int64_t L, int i, uint64_t rng, uint64_t mask,
                                             const uint64_t blk[4]) {
  if (rng == 0) return 0;  // numpy's off + 0: no words
  const int w = i & 3;
  uint64_t v = (w == 0 ? blk[0] : w == 1 ? blk[1] : w == 2 ? blk[2] : blk[3]) & mask;
  for (uint64_t j = 1; v > rng && j < 64; ++j) {  // (64 failed words: probability < 2^-64)
    uint64_t c[4] = {(uint64_t)(i >> 2), (uint64_t)L, j, 0ull};
    philox4x64_10(c, seed, 0ull);
    v = (w == 0 ? c[0] : w == 1 ? c[1] : w == 2 ? c[2] : c[3]) & mask;
  }
  return v <= rng ? (int64_t)v : 0;
}

__device__ __forceinline__ uint64_t range_mask(uint64_t rng) {
  uint64_t m = rng;
  m |= m >> 1;
  m |= m >> 2;
  m |= m >> 4;
  m |= m >> 8;
  m |= m >> 16;
  m |= m >> 32;
  return m;
}

constexpr int kPackTile = 256;

// the tile's records before this thread's (the block's waves in order): returns the
// exclusive rank, *tile_total the tile's count
__device__ __forceinline__ int tile_rank(bool take, int* wcnt, int* tile_total) {
  const int tid = threadIdx.x, lane = tid & (kWave - 1), wv = tid / kWave;
  const unsigned long long bal = __ballot(take);
  if (lane == 0) wcnt[wv] = __popcll(bal);
  __syncthreads();
  int before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kPackTile / kWave; ++w) {
    const int c = wcnt[w];
    before += w < wv ? c : 0;
    total += c;
  }
  *tile_total = total;
  return before + __popcll(bal & ((1ull << lane) - 1ull));
}

// The all-gather form of the exchange. Each rank packs the rows IT owns of the
// segment's learns -- one 25-word record per sampled row: slot (learn x batch +
// draw) | terminal << 31, reward f32, state [11], new_state [11], action -- into
// a chunk of `cap` records behind a 4-word header (record count); rank 0 also
// packs the rows of skipped learns (all zero). One all-gather of the chunks and
// an unpack on every rank rebuild sacenv_replay_sample_staged's `words`, bit for
// bit: every slot comes from exactly one rank. The records sit in slot order (a
// count per 256-slot tile, then each tile's prefix over the tiles before it: no
// atomics -- one count word taking every wave's atomic cost ~100 us a segment --
// and the chunk is the same bytes run to run).
constexpr int kRecWords = 2 + 2 * SACENV_OBS_DIM + 1;  // 25
constexpr int kChunkHdr = 4;

// One 256-slot tile of side work in LDS: the tile's records (the pack assembles them
// here and writes them out as one contiguous run; the unpack reads its run in here:
// coalesced dwords instead of a 100-B stride per lane), the per-wave counts, the
// tile's first record.
struct SideLds {
  uint32_t rec[kPackTile * kRecWords];  // the tile's records
  uint32_t meta[kPackTile];             // unpack: the record's learn's words offset
  uint32_t meta2[kPackTile];            // unpack: the record's draw within its learn
  int wcnt[kPackTile / kWave];
  int base;
};

// Segment G.g's learns, slots [tile x 256, tile x 256 + 256): idx[k][i] (-1: the
// learn is skipped, fewer than `batch` rows stored) and the marks of the rows they
// read on this rank -- the row and its predecessor (its s) -- in segment G.g
// (marks_cur) or G.g - 1 (marks_prev; with M <= seg x period a row lies in one of
// the two). One draw per thread (the four threads of an aligned four compute their
// shared Philox block each: ~200 integer ops, cheaper than any exchange); with
// tile_cnt, also the records this tile's pack will write (so the pack needs no
// count pass).
__device__ __forceinline__ void draw_ctr_tile(const SacenvReplayParams& p, const StagedGeom& G, uint64_t seed,
                                              int batch, int nb, int64_t* __restrict__ idx,
                                              unsigned long long* __restrict__ marks_prev,
                                              unsigned long long* __restrict__ marks_cur, int* __restrict__ tile_cnt,
                                              int skip_owner, int64_t tile, int* wcnt) {
  const int total = batch * nb;  // (< 2^31: check_ctr_shape)
  const int t = (int)(tile * kPackTile) + (int)threadIdx.x;
  const int64_t M = p.mem_size;
  bool take = false;  // (a slot the all-gather's pack of this segment takes on this rank)
  if (t < total) {
    const int k = t / batch, i = t - k * batch;
    const int64_t L = G.g * G.seg + k, cntr = (L + 1) * G.period;
    if (cntr < batch) {  // continuous_agent.py:97-98: learn() returns before sampling
      idx[t] = -1;
      take = skip_owner != 0;
    } else {
      const uint64_t rng = (uint64_t)((cntr < M ? cntr : M) - 1);
      uint64_t blk[4] = {(uint64_t)(i >> 2), (uint64_t)L, 0ull, 0ull};  // the block of this draw's four
      philox4x64_10(blk, seed, 0ull);
      const int64_t row = ctr_draw4(seed, L, i, rng, range_mask(rng), blk);
      idx[t] = row;
      int64_t q, u;
      resolve(row, cntr, M, G, &q, &u);
      if (u >= G.offset && u < G.offset + G.n) {
        take = true;
        const int e = (int)(u - G.offset);
        // the row and its predecessor (s); the predecessor of segment g's first row is
        // segment g - 1's last (a learn of segment g reaches no row before step 1 of
        // segment g - 1: M <= seg x period); step -1 is the reset obs begin() staged
        int64_t j = q - G.g * G.seg;
        unsigned long long* const mk = j >= 0 ? marks_cur : marks_prev;
        j = j >= 0 ? j : j + G.seg;
        if (j >= 1 && (j & 63) != 0) {  // both in one word: one atomic
          if (mk != nullptr) mark_rows(mk, G, e, j - 1, 3ull);
        } else {
          if (mk != nullptr) mark_rows(mk, G, e, j, 1ull);
          if (q >= 1) {
            unsigned long long* const mp = j >= 1 ? mk : marks_prev;  // (j = 0: segment g - 1's last)
            if (mp != nullptr) mark_rows(mp, G, e, j >= 1 ? j - 1 : G.seg - 1, 1ull);
          }
        }
      }
    }
  }
  if (tile_cnt != nullptr) {  // the pack's per-tile record counts, drawn ahead
    int tile_total;
    tile_rank(take, wcnt, &tile_total);
    if (threadIdx.x == 0 && (int64_t)tile * kPackTile < total) tile_cnt[tile] = tile_total;
  }
}

// do this rank's records include slot t (its row, or rank 0 a skipped learn's zero row)?
__device__ __forceinline__ bool pack_takes(const SacenvReplayParams& p, const StagedGeom& G, int batch, int64_t t,
                                           int64_t row, int skip_owner, int64_t* q, int64_t* u) {
  *q = 0;
  *u = -1;
  if (row >= 0) resolve(row, (G.g * G.seg + t / batch + 1) * G.period, p.mem_size, G, q, u);
  return (*u >= G.offset && *u < G.offset + G.n) || (row == -1 && skip_owner);
}

// The records of tile `tile` (slots tile x 256 ...): each taking thread forms its
// record in LDS at its rank within the tile, then the block writes the tile's run
// [base, base + count) of the chunk with coalesced dword stores (records past `cap`
// are dropped: the header's count says so and the unpack flags it). The last tile
// writes the header's count.
__device__ __forceinline__ void pack_tile(const SacenvReplayParams& p, const StagedGeom& G, const StagedRows& S,
                                          int batch, int nb, const int64_t* __restrict__ idx,
                                          uint32_t* __restrict__ chunk, int64_t cap, int skip_owner,
                                          const int* __restrict__ tile_cnt, int64_t tile, int64_t n_tiles,
                                          SideLds& l) {
  constexpr int D = SACENV_OBS_DIM;
  const int tid = threadIdx.x;
  if (tid < kWave) {  // this tile's first record: the counts of the tiles before it (8 loads in flight per lane)
    int s = 0;
    for (int64_t b0 = 0; b0 < tile; b0 += 8 * kWave) {
      int v[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const int64_t i = b0 + r * kWave + tid;
        v[r] = i < tile ? tile_cnt[i] : 0;
      }
#pragma unroll
      for (int r = 0; r < 8; ++r) s += v[r];
    }
    for (int o = kWave / 2; o > 0; o >>= 1) s += __shfl_xor(s, o);
    if (tid == 0) l.base = s;
  }
  const int64_t t = tile * kPackTile + tid;
  const bool live = t < (int64_t)batch * nb;
  const int64_t row = live ? idx[t] : -2;
  int64_t q = 0, u = -1;
  const bool take = live && pack_takes(p, G, batch, t, row, skip_owner, &q, &u);
  const bool own = take && row >= 0;
  int tile_total;
  const int rank = tile_rank(take, l.wcnt, &tile_total);  // (its barrier also publishes l.base)
  const int64_t base = l.base;
  if (tile == n_tiles - 1 && tid == 0) chunk[0] = (uint32_t)(base + tile_total);  // the record count
  float sn[16], sv[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) sn[k] = sv[k] = 0.f;
  uint32_t tm = 0u;
  if (own) {  // (as k_rb_gather_staged)
    const int e = (int)(u - G.offset);
    int64_t j = q - G.g * G.seg;
    const bool in_cur = j >= 0;
    j = in_cur ? j : j + G.seg;
    const float4* R = reinterpret_cast<const float4*>((in_cur ? S.cur : S.prev) + stage_row(G, e, j));
    const float4* P = j > 0 ? R - 4 : reinterpret_cast<const float4*>(S.prev + stage_row(G, e, G.seg - 1));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float4 x = R[k], y = P[k];
      sn[4 * k] = x.x, sn[4 * k + 1] = x.y, sn[4 * k + 2] = x.z, sn[4 * k + 3] = x.w;
      sv[4 * k] = y.x, sv[4 * k + 1] = y.y, sv[4 * k + 2] = y.z, sv[4 * k + 3] = y.w;
    }
    const bool pdone = (__float_as_uint(sv[13]) & 0xFFu) != 0u;
    const float o3 = sv[14];
#pragma unroll
    for (int k = 0; k < D; ++k) sv[k] = pdone ? S.first[k] : sv[k];
    if (G.exp2 && pdone) sv[3] = o3;
    tm = (p.terminal_mask >> ((__float_as_uint(sn[13]) >> 8) & 0xFFu)) & 1u;
  }
  if (take) {
    uint32_t* const rec = l.rec + rank * kRecWords;
    rec[0] = (uint32_t)t | (tm << 31);
    rec[1] = __float_as_uint(sn[11]);
#pragma unroll
    for (int k = 0; k < D; ++k) {
      rec[2 + k] = __float_as_uint(sv[k]);
      rec[2 + D + k] = __float_as_uint(sn[k]);
    }
    rec[2 + 2 * D] = __float_as_uint(sn[12]);
  }
  __syncthreads();
  int64_t nrec = tile_total;
  if (base + nrec > cap) nrec = cap - base;  // (past cap: dropped; the count tells the unpack)
  if (nrec <= 0) return;
  uint32_t* const dst = chunk + kChunkHdr + base * kRecWords;
  const int nw = (int)nrec * kRecWords;
  for (int w = tid; w < nw; w += kPackTile) dst[w] = l.rec[w];
}

// Records [j0, j0 + 256) of chunk r -> sacenv_replay_sample_staged's words: the run
// is read into LDS with coalesced dwords, then one thread per record scatters it to
// its slot. A count above cap sets status bit 0 (the first tile of the chunk).
__device__ __forceinline__ void unpack_tile(const uint32_t* __restrict__ gathered, int64_t chunk_words, int64_t cap,
                                            int batch, uint32_t* __restrict__ words, int64_t per,
                                            int32_t* __restrict__ status, int64_t blk, int64_t tiles_per_chunk,
                                            SideLds& l) {
  constexpr int D = SACENV_OBS_DIM;
  const int tid = threadIdx.x;
  const int64_t r = blk / tiles_per_chunk;
  const int64_t j0 = (blk - r * tiles_per_chunk) * kPackTile;
  const uint32_t* const hdr = gathered + r * chunk_words;
  int64_t cnt = hdr[0];
  if (j0 == 0 && tid == 0 && cnt > cap) atomicOr(status, 1);
  cnt = cnt < cap ? cnt : cap;
  const int nrec = (int)(cnt - j0 < kPackTile ? cnt - j0 : kPackTile);
  if (nrec <= 0) return;  // (uniform over the block)
  const uint32_t* const src = hdr + kChunkHdr + j0 * kRecWords;
  for (int w = tid; w < nrec * kRecWords; w += kPackTile) l.rec[w] = src[w];
  __syncthreads();
  if (tid < nrec) {  // the record's batch: words offset of learn b, draw i (i < 2^31 / 26)
    const uint32_t slot = l.rec[tid * kRecWords] & 0x7FFFFFFFu;
    const uint32_t b = slot / (uint32_t)batch, i = slot - b * (uint32_t)batch;
    l.meta[tid] = (uint32_t)(b * per);  // (n_batches x per < 2^32: the host's size checks)
    l.meta2[tid] = i;
  }
  __syncthreads();
  // one output word per thread, so consecutive lanes write consecutive words where the
  // records' slots are consecutive (a 100-B record per lane scattered 26 partial lines)
  const int64_t B = batch;
  for (int w = tid; w < nrec * 2; w += kPackTile) {  // reward f64: two words each
    const int q = w >> 1;
    const uint32_t m = l.meta[q], i = l.meta2[q];
    const double r64 = (double)__uint_as_float(l.rec[q * kRecWords + 1]);
    uint64_t rb;
    __builtin_memcpy(&rb, &r64, 8);
    words[(int64_t)m + 2 * (int64_t)i + (w & 1)] = (w & 1) ? (uint32_t)(rb >> 32) : (uint32_t)rb;
  }
  for (int w = tid; w < nrec * D; w += kPackTile) {  // state
    const int q = w / D, k = w - q * D;
    const uint32_t m = l.meta[q], i = l.meta2[q];
    words[(int64_t)m + 2 * B + (int64_t)i * D + k] = l.rec[q * kRecWords + 2 + k];
  }
  for (int w = tid; w < nrec * D; w += kPackTile) {  // new_state
    const int q = w / D, k = w - q * D;
    const uint32_t m = l.meta[q], i = l.meta2[q];
    words[(int64_t)m + 2 * B + B * D + (int64_t)i * D + k] = l.rec[q * kRecWords + 2 + D + k];
  }
  if (tid < nrec) {  // action, terminal
    const uint32_t m = l.meta[tid], i = l.meta2[tid];
    const uint32_t* const rec = l.rec + tid * kRecWords;
    uint32_t* const W = words + (int64_t)m;
    W[2 * B + 2 * B * D + i] = rec[2 + 2 * D];
    W[2 * B + 2 * B * D + B + i] = rec[0] >> 31;
  }
}

__global__ void __launch_bounds__(kPackTile) k_rb_draw_ctr(SacenvReplayParams p, StagedGeom G, uint64_t seed,
                                                           int batch, int nb, int64_t* __restrict__ idx,
                                                           unsigned long long* __restrict__ marks_prev,
                                                           unsigned long long* __restrict__ marks_cur,
                                                           int* __restrict__ tile_cnt, int skip_owner) {
  __shared__ int wcnt[kPackTile / kWave];
  draw_ctr_tile(p, G, seed, batch, nb, idx, marks_prev, marks_cur, tile_cnt, skip_owner, blockIdx.x, wcnt);
}

__global__ void __launch_bounds__(kPackTile) k_rb_pack_count(SacenvReplayParams p, StagedGeom G, int batch, int nb,
                                                             const int64_t* __restrict__ idx, int skip_owner,
                                                             int* __restrict__ tile_cnt) {
  __shared__ int wcnt[kPackTile / kWave];
  const int64_t t = blockIdx.x * (int64_t)kPackTile + threadIdx.x;
  int64_t q, u;
  const bool take = t < (int64_t)batch * nb && pack_takes(p, G, batch, t, idx[t], skip_owner, &q, &u);
  int total;
  tile_rank(take, wcnt, &total);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = total;
}

__global__ void __launch_bounds__(kPackTile) k_rb_pack_staged(SacenvReplayParams p, StagedGeom G, StagedRows S, int batch,
                                                              int nb, const int64_t* __restrict__ idx,
                                                              uint32_t* __restrict__ chunk, int64_t cap, int skip_owner,
                                                              const int* __restrict__ tile_cnt) {
  __shared__ SideLds l;
  pack_tile(p, G, S, batch, nb, idx, chunk, cap, skip_owner, tile_cnt, blockIdx.x, gridDim.x, l);
}

__global__ void __launch_bounds__(kPackTile) k_rb_unpack_staged(const uint32_t* __restrict__ gathered,
                                                                int64_t chunk_words, int64_t cap, int batch,
                                                                uint32_t* __restrict__ words, int64_t per,
                                                                int32_t* __restrict__ status, int64_t tiles_per_chunk) {
  __shared__ SideLds l;
  unpack_tile(gathered, chunk_words, cap, batch, words, per, status, blockIdx.x, tiles_per_chunk, l);
}

// A segment's side work in ONE launch (sacenv_replay_stage_side): the unpack of one
// segment's collected chunks, the pack of the next segment's rows and the draws of a
// later segment, on disjoint buffers (the host checks) -- three launches, their
// boundaries and their tails become one, and the three kinds of blocks share the GPU
// (each alone leaves it mostly idle: ~1 000 short-lived blocks bound by latency).
// Block ranges: the pack's tiles, the unpack's, then the draws' (measured in bench's
// runner: 36.5-36.7 G for this order, 36.0 with the draws first; alone 23.2 vs 27.5 us).
struct SideArgs {
  SacenvReplayParams p;
  int batch, nb, skip_owner, world;
  // draws
  StagedGeom Gd;
  uint64_t seed;
  int64_t* d_idx;
  unsigned long long* marks_prev;
  unsigned long long* marks_cur;
  int* d_tiles;
  int64_t n_draw;
  // pack
  StagedGeom Gp;
  StagedRows S;
  const int64_t* p_idx;
  const int* p_tiles;
  uint32_t* chunk;
  int64_t cap, n_pack;
  // unpack
  const uint32_t* gathered;
  uint32_t* words;
  int32_t* status;
  int64_t chunk_words, per, u_tiles, n_unpack;
};

__global__ void __launch_bounds__(kPackTile) k_rb_side(SideArgs a) {
  __shared__ SideLds l;
  int64_t b = blockIdx.x;
  if (b < a.n_pack) {
    pack_tile(a.p, a.Gp, a.S, a.batch, a.nb, a.p_idx, a.chunk, a.cap, a.skip_owner, a.p_tiles, b, a.n_pack, l);
    return;
  }
  b -= a.n_pack;
  if (b < a.n_unpack) {
    unpack_tile(a.gathered, a.chunk_words, a.cap, a.batch, a.words, a.per, a.status, b, a.u_tiles, l);
    return;
  }
  b -= a.n_unpack;
  draw_ctr_tile(a.p, a.Gd, a.seed, a.batch, a.nb, a.d_idx, a.marks_prev, a.marks_cur, a.d_tiles, a.skip_owner, b,
                l.wcnt);
}

// A stand-in for a collective's kernel on one GPU (bench.py's replay_path at N =
// 1): `workgroups` workgroups of 256 threads -- the channels of an RCCL kernel --
// copy `n16` 16-B units and then stay resident until `min_ticks` of the 100-MHz
// realtime clock have passed since they started (an RCCL kernel lives as long as
// its transfer over the links, not as long as a local copy): what the owner waves
// of a segment launch share their CUs with while the exchange runs beside them.
__global__ void __launch_bounds__(256) k_copy_standin(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                      int64_t n16, uint64_t min_ticks) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (int64_t q = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; q < n16; q += (int64_t)gridDim.x * blockDim.x)
    dst[q] = src[q];
  while (__builtin_amdgcn_s_memrealtime() - t0 < min_ticks) __builtin_amdgcn_s_sleep(8);
}

// 32-bit words of one learn's batch in sacenv_replay_sample_staged's packing
int64_t words_per_batch(int32_t batch) { return (int64_t)batch * (2 * SACENV_OBS_DIM + 1 + 3); }

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
                 const float* final_state, const uint8_t* code, uint8_t* last_term, void* stream,
                 int64_t host_cntr = -1) {
  int rc = check_replay(p);
  if (rc) return rc;
  if (n < 0) return SACENV_E_SIZE;
  if (host_cntr >= 0 && n == 0) host_cntr = -1;  // nothing to launch: advance as before
  if (n == 0 && advance == n) return SACENV_OK;
  if (!arena || !state || !action || !reward || !new_state || !code) return SACENV_E_NULL;
  const int64_t rows = n > p->mem_size ? p->mem_size : n;
  const int64_t total = rows * ((int64_t)p->obs_dim + p->act_dim + 1) + (last_term ? n - rows : 0);
  if (total >= (1LL << 32)) return SACENV_E_SIZE;  // 32-bit element index per call
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  const RB r = make_rb(*p, arena);
  if (n > 0) {
    hipLaunchKernelGGL(k_rb_store, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, *p, r, host_cntr,
                       advance, n, offset, state, action, reward, new_state, final_state, code, last_term);
    if ((rc = status())) return rc;
    if (host_cntr >= 0) return SACENV_OK;
  }
  hipLaunchKernelGGL(k_rb_advance, dim3(1), dim3(kWave), 0, (hipStream_t)stream, r, advance);
  return status();
}

int sacenv_replay_store_env_at(const SacenvReplayParams* p, void* arena, int64_t cntr, int64_t n, const float* state,
                               const float* action, const void* reward, const float* new_state,
                               const float* final_state, const uint8_t* code, uint8_t* last_term, void* stream) {
  if (cntr < 0) return SACENV_E_RANGE;
  return store(p, arena, n, 0, n, state, action, reward, new_state, final_state, code, last_term, stream, cntr);
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
  // one 1 024-thread workgroup: a twist per 624 words and one ballot-and-scan round per
  // block instead of one wave's 64-word rounds (9.8 -> ~4 us per 1 024 draws)
  hipLaunchKernelGGL(k_rb_draw_many<true>, dim3(1), dim3(kDrawThreads), 0, (hipStream_t)stream, *p, r, batch, 1,
                     (int64_t)0, (int64_t)0, idx);
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
  // every row a learn can reach (and the row before it) lies in this segment or the previous one
  if (p->mem_size > (int64_t)sp->seg * sp->period) return SACENV_E_RANGE;
  return SACENV_OK;
}

// the sequence numbers of segments g and g + 1 stay below 2^52 (div_floor's range)
static bool staged_range_ok(const SacenvStagedParams* sp, int64_t g) {
  if (sp->period >= ((int64_t)1 << 31)) return false;
  return g < (((int64_t)1 << 52) / ((int64_t)sp->seg * sp->period)) - 2;
}

static StagedGeom geom(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g) {
  StagedGeom G;
  G.r_mem = 1.0 / (double)p->mem_size;
  G.r_period = 1.0 / (double)sp->period;
  G.period = sp->period;
  G.offset = sp->offset;
  G.g = g;
  G.n = sp->n;
  G.n_pad = sp->n_pad;
  G.seg = sp->seg;
  G.exp2 = sp->experiment == 2;
  return G;
}

// the steady-state draw's generated blocks: enough for n_batches * batch accepted
// words with a 5 % margin over the expected count (at 262 144 draws of [0, 10^6)
// the count's standard deviation is 0.04 % of it: 120 sigma), + 3 blocks for the
// start position and small draws
static int64_t draw_blocks(const SacenvReplayParams* p, int32_t batch, int32_t n_batches) {
  const uint64_t rng = (uint64_t)(p->mem_size - 1);
  uint64_t mask = rng;
  for (int sh = 1; sh < 64; sh <<= 1) mask |= mask >> sh;
  const double acc = (double)(rng + 1) / (double)(mask + 1);
  const double need = (double)batch * n_batches;
  return (int64_t)(need / acc * 1.05 / kMtN) + 3;
}

static int64_t draw_tiles(int64_t blocks) { return (blocks * kMtN + kTile - 1) / kTile; }

static int64_t scratch_bytes(const SacenvReplayParams* p, int32_t batch, int32_t n_batches) {
  const int64_t K = draw_blocks(p, batch, n_batches), T = draw_tiles(K);
  return align256(4 * K * kMtN) + 2 * align256(4 * T) + 256;
}

int sacenv_replay_stage_scratch_bytes(const SacenvReplayParams* p, int32_t batch, int32_t n_batches,
                                      int64_t* bytes) {
  const int rc = check_replay(p);
  if (rc) return rc;
  if (bytes == nullptr) return SACENV_E_NULL;
  if (batch < 0 || n_batches < 0) return SACENV_E_SIZE;
  *bytes = scratch_bytes(p, batch, n_batches);
  return SACENV_OK;
}

int sacenv_replay_stage_draw(const SacenvReplayParams* p, void* arena, const SacenvStagedParams* sp, int64_t g,
                             int32_t batch, int32_t n_batches, int64_t* idx, void* scratch, int64_t scratch_size,
                             void* stream) {
  int rc = check_staged(p, sp);
  if (rc) return rc;
  if (g < 0 || batch < 0 || n_batches < 0 || n_batches > sp->seg) return SACENV_E_SIZE;
  if (!arena || !idx) return SACENV_E_NULL;
  if (batch == 0 || n_batches == 0) return SACENV_OK;
  if (!staged_range_ok(sp, g)) return SACENV_E_RANGE;
  const RB r = make_rb(*p, arena);
  const int64_t cntr0 = g * sp->seg * sp->period;
  const int64_t M = p->mem_size;
  const bool steady = cntr0 + sp->period >= M && cntr0 + sp->period >= batch && M >= 2;
  if (!steady) {  // the first learns of a buffer (ranges below M, skipped learns): one workgroup
    hipLaunchKernelGGL(k_rb_draw_many<false>, dim3(1), dim3(kDrawThreads), 0, (hipStream_t)stream, *p, r, batch,
                       n_batches, cntr0, sp->period, idx);
    return status();
  }
  if (!scratch) return SACENV_E_NULL;
  if (scratch_size < scratch_bytes(p, batch, n_batches)) return SACENV_E_SIZE;
  const int64_t K = draw_blocks(p, batch, n_batches), T = draw_tiles(K);
  char* sc = static_cast<char*>(scratch);
  DrawPlan d;
  d.blocks = reinterpret_cast<const uint32_t*>(sc);
  d.tile_cnt = reinterpret_cast<int*>(sc + align256(4 * K * kMtN));
  d.tile_off = reinterpret_cast<int*>(sc + align256(4 * K * kMtN) + align256(4 * T));
  d.ctrl = reinterpret_cast<int*>(sc + align256(4 * K * kMtN) + 2 * align256(4 * T));
  d.rng = (uint32_t)(M - 1);
  uint32_t mask = d.rng;
  for (int sh = 1; sh < 32; sh <<= 1) mask |= mask >> sh;
  d.mask = mask;
  d.need = (int64_t)batch * n_batches;
  d.p0 = -1;       // (read by the kernels from ctrl[3], which k_mt_chain sets)
  d.n_words = -1;
  hipLaunchKernelGGL(k_mt_chain, dim3(1), dim3(kChainThreads), 0, (hipStream_t)stream, r,
                     reinterpret_cast<uint32_t*>(sc), (int)K, d.ctrl);
  if ((rc = status())) return rc;
  hipLaunchKernelGGL(k_draw_count, dim3((unsigned)T), dim3(kTileThreads), 0, (hipStream_t)stream, d, (int64_t)K);
  if ((rc = status())) return rc;
  hipLaunchKernelGGL(k_draw_scan, dim3(1), dim3(1024), 0, (hipStream_t)stream, d, (int)T);
  if ((rc = status())) return rc;
  hipLaunchKernelGGL(k_draw_emit, dim3((unsigned)T), dim3(kTileThreads), 0, (hipStream_t)stream, d, r, (int64_t)K,
                     idx);
  return status();
}

int sacenv_replay_stage_mark(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g,
                             const int64_t* idx_g, const int64_t* idx_next, int32_t batch, int32_t n_batches,
                             uint64_t* marks, void* stream) {
  int rc = check_staged(p, sp);
  if (rc) return rc;
  if (g < 0 || batch < 0 || n_batches < 0 || n_batches > sp->seg) return SACENV_E_SIZE;
  if (!idx_g || !marks) return SACENV_E_NULL;
  if (!staged_range_ok(sp, g)) return SACENV_E_RANGE;
  const hipError_t e = hipMemsetAsync(marks, 0, (size_t)sp->n_pad * ((sp->seg + 63) / 64) * 8, (hipStream_t)stream);
  if (e != hipSuccess) return (int)e;
  const int64_t per = (int64_t)batch * n_batches;
  if (per == 0) return SACENV_OK;
  // without the next segment's draws, only this segment's learns mark
  const int64_t total = idx_next != nullptr ? 2 * per : per;
  hipLaunchKernelGGL(k_rb_stage_mark, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     *p, geom(p, sp, g), idx_g, idx_next != nullptr ? idx_next : idx_g, batch, n_batches,
                     reinterpret_cast<unsigned long long*>(marks), total);
  return status();
}

int sacenv_replay_sample_staged(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g,
                                const void* stage_cur, const void* stage_prev, const int64_t* idx, int32_t batch,
                                int32_t n_batches, uint32_t* words, void* stream) {
  int rc = check_staged(p, sp);
  if (rc) return rc;
  if (g < 0 || batch < 0 || n_batches < 0 || n_batches > sp->seg) return SACENV_E_SIZE;
  if (!stage_cur || !stage_prev || !idx || !words) return SACENV_E_NULL;
  if (!staged_range_ok(sp, g)) return SACENV_E_RANGE;
  if (((reinterpret_cast<uintptr_t>(stage_cur) | reinterpret_cast<uintptr_t>(stage_prev)) & 15u) != 0u)
    return SACENV_E_RANGE;
  if (batch == 0 || n_batches == 0) return SACENV_OK;
  StagedRows S;
  S.cur = static_cast<const char*>(stage_cur);
  S.prev = static_cast<const char*>(stage_prev);
  for (int k = 0; k < SACENV_OBS_DIM; ++k) S.first[k] = sp->first_obs[k];
  const int64_t total = (int64_t)batch * n_batches;
  const int64_t per = (int64_t)batch * (2 * SACENV_OBS_DIM + 1 + 3);
  hipLaunchKernelGGL(k_rb_gather_staged, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     *p, geom(p, sp, g), S, batch, n_batches, idx, words, per);
  return status();
}

int sacenv_replay_gather(const SacenvReplayParams* p, void* arena, int32_t batch, const int64_t* idx, float* state,
                         float* action, double* reward, float* new_state, uint8_t* terminal, void* stream) {
  int rc = check_replay(p);
  if (rc) return rc;
  if (batch < 0) return SACENV_E_SIZE;
  if (arena == nullptr || idx == nullptr) return SACENV_E_NULL;
  if (batch == 0) return SACENV_OK;
  const int64_t total = (int64_t)batch * (p->obs_dim + p->act_dim + 1);
  hipLaunchKernelGGL(k_rb_gather, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *p,
                     make_rb(*p, arena), batch, idx, state, action, reward, new_state, terminal, Shard{0, 0, 0});
  return status();
}

static int check_ctr_shape(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g, int32_t batch,
                           int32_t n_batches) {
  const int rc = check_staged(p, sp);
  if (rc) return rc;
  if (g < 0 || batch < 0 || n_batches < 0 || n_batches > sp->seg) return SACENV_E_SIZE;
  if ((int64_t)batch * n_batches >= ((int64_t)1 << 31)) return SACENV_E_SIZE;  // slot numbers: 31 bits
  if (!staged_range_ok(sp, g)) return SACENV_E_RANGE;
  return SACENV_OK;
}

int sacenv_replay_stage_draw_ctr(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g,
                                 int32_t batch, int32_t n_batches, uint64_t seed, int64_t* idx, uint64_t* marks_prev,
                                 uint64_t* marks_cur, int32_t* tiles, void* stream) {
  const int rc = check_ctr_shape(p, sp, g, batch, n_batches);
  if (rc) return rc;
  if (idx == nullptr) return SACENV_E_NULL;
  const int64_t total = (int64_t)batch * n_batches;
  if (total == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_rb_draw_ctr, dim3((unsigned)((total + kPackTile - 1) / kPackTile)), dim3(kPackTile), 0,
                     (hipStream_t)stream, *p, geom(p, sp, g), seed, batch, n_batches, idx,
                     reinterpret_cast<unsigned long long*>(marks_prev), reinterpret_cast<unsigned long long*>(marks_cur),
                     tiles, sp->offset == 0 ? 1 : 0);
  return status();
}

// rows of the window [c - W, c) of sequence numbers whose (s mod period) lies in [o, o + n)
static double window_rows(int64_t c, int64_t W, int64_t period, int64_t o, int64_t n) {
  auto F = [&](int64_t x) {
    int64_t r = x % period - o;
    r = r < 0 ? 0 : (r > n ? n : r);
    return (x / period) * n + r;
  };
  return (double)(F(c) - F(c - W));
}

// The chunk of sacenv_replay_stage_pack for this shape, the same on every rank: the
// most records any rank packs in expectation over any segment (each learn's rows
// owned in proportion to the rank's share of the ring window; rank 0 also the
// skipped learns' rows), + 8 standard deviations (the count is a sum of
// independent draws: variance <= mean) + 64, at most every slot.
static int64_t chunk_cap(const SacenvReplayParams* p, const SacenvStagedParams* sp, int32_t batch, int32_t nb) {
  const int64_t P = sp->period, n = sp->n, M = p->mem_size, world = P / n, total = (int64_t)batch * nb;
  if (world == 1) return total;
  // after the first learn whose window is the whole ring, every learn's window has the
  // same alignment (c is a multiple of period): the rank shares repeat
  const int64_t g_last = (M / P) / sp->seg + 2;
  double worst = 0.0;
  for (int64_t g = 0; g <= g_last; ++g)
    for (int64_t r = 0; r < world; ++r) {
      double e = 0.0;
      for (int k = 0; k < nb; ++k) {
        const int64_t c = (g * sp->seg + k + 1) * P;
        if (c < batch) {
          e += r == 0 ? batch : 0;
          continue;
        }
        const int64_t W = c < M ? c : M;
        e += (double)batch * window_rows(c, W, P, r * n, n) / (double)W;
      }
      worst = e > worst ? e : worst;
    }
  const int64_t cap = (int64_t)(worst + 8.0 * sqrt(worst) + 64.0) + 1;
  return cap < total ? cap : total;
}

int sacenv_replay_stage_chunk(const SacenvReplayParams* p, const SacenvStagedParams* sp, int32_t batch,
                              int32_t n_batches, int64_t* cap_rows, int64_t* chunk_bytes) {
  const int rc = check_ctr_shape(p, sp, 0, batch, n_batches);
  if (rc) return rc;
  if (cap_rows == nullptr || chunk_bytes == nullptr) return SACENV_E_NULL;
  if (sp->period % sp->n != 0) return SACENV_E_RANGE;  // every rank holds n envs
  const int64_t cap = chunk_cap(p, sp, batch, n_batches);
  *cap_rows = cap;
  *chunk_bytes = align256(4 * (kChunkHdr + cap * kRecWords));
  return SACENV_OK;
}

int sacenv_replay_stage_pack(const SacenvReplayParams* p, const SacenvStagedParams* sp, int64_t g,
                             const void* stage_cur, const void* stage_prev, const int64_t* idx, int32_t batch,
                             int32_t n_batches, int64_t cap, void* chunk, int32_t* tiles, int32_t counted,
                             void* stream) {
  int rc = check_ctr_shape(p, sp, g, batch, n_batches);
  if (rc) return rc;
  if (!stage_cur || !stage_prev || !idx || !chunk || !tiles) return SACENV_E_NULL;
  if (((reinterpret_cast<uintptr_t>(stage_cur) | reinterpret_cast<uintptr_t>(stage_prev)) & 15u) != 0u ||
      (reinterpret_cast<uintptr_t>(chunk) & 3u) != 0u || cap < 0)
    return SACENV_E_RANGE;
  const int64_t total = (int64_t)batch * n_batches;
  if (total == 0) {  // no records: only the count
    const hipError_t e = hipMemsetAsync(chunk, 0, 4 * kChunkHdr, (hipStream_t)stream);
    return e == hipSuccess ? SACENV_OK : (int)e;
  }
  StagedRows S;
  S.cur = static_cast<const char*>(stage_cur);
  S.prev = static_cast<const char*>(stage_prev);
  for (int k = 0; k < SACENV_OBS_DIM; ++k) S.first[k] = sp->first_obs[k];
  const StagedGeom G = geom(p, sp, g);
  const int skip_owner = sp->offset == 0 ? 1 : 0;
  const unsigned T = (unsigned)((total + kPackTile - 1) / kPackTile);
  if (!counted) {  // (the counter-based draw wrote the tile counts already)
    hipLaunchKernelGGL(k_rb_pack_count, dim3(T), dim3(kPackTile), 0, (hipStream_t)stream, *p, G, batch, n_batches,
                       idx, skip_owner, tiles);
    if ((rc = status())) return rc;
  }
  hipLaunchKernelGGL(k_rb_pack_staged, dim3(T), dim3(kPackTile), 0, (hipStream_t)stream, *p, G, S, batch, n_batches,
                     idx, static_cast<uint32_t*>(chunk), cap, skip_owner, tiles);
  return status();
}

int sacenv_replay_stage_unpack(int32_t world, int64_t chunk_bytes, int64_t cap, int32_t batch, int32_t n_batches,
                               const void* gathered, uint32_t* words, int32_t* status_word, void* stream) {
  if (world < 1 || cap < 0 || batch < 0 || n_batches < 0) return SACENV_E_SIZE;
  if ((int64_t)batch * n_batches >= ((int64_t)1 << 31) || (int64_t)world * cap >= ((int64_t)1 << 31))
    return SACENV_E_SIZE;
  if (chunk_bytes < 4 * (kChunkHdr + cap * kRecWords) || (chunk_bytes & 3) != 0) return SACENV_E_SIZE;
  if ((int64_t)n_batches * words_per_batch(batch) >= ((int64_t)1 << 32)) return SACENV_E_SIZE;  // 32-bit offsets
  if (!gathered || !words || !status_word) return SACENV_E_NULL;
  const int64_t tiles = (cap + kPackTile - 1) / kPackTile;
  if (tiles == 0 || batch == 0) return SACENV_OK;
  hipLaunchKernelGGL(k_rb_unpack_staged, dim3((unsigned)(world * tiles)), dim3(kPackTile), 0, (hipStream_t)stream,
                     static_cast<const uint32_t*>(gathered), chunk_bytes / 4, cap, batch, words, words_per_batch(batch),
                     status_word, tiles);
  return status();
}

int sacenv_replay_stage_side(const SacenvReplayParams* p, const SacenvStagedParams* sp, int32_t batch,
                             int32_t n_batches, const SacenvStageSide* w, void* stream) {
  if (w == nullptr) return SACENV_E_NULL;
  const bool draw = w->draw_g >= 0, pack = w->pack_g >= 0, unpack = w->gathered != nullptr;
  int rc = check_ctr_shape(p, sp, draw ? w->draw_g : 0, batch, n_batches);
  if (rc) return rc;
  if (pack && (rc = check_ctr_shape(p, sp, w->pack_g, batch, n_batches))) return rc;
  const int64_t total = (int64_t)batch * n_batches;
  const int64_t tiles = (total + kPackTile - 1) / kPackTile;
  SideArgs a = {};
  a.p = *p;
  a.batch = batch;
  a.nb = n_batches;
  a.skip_owner = sp->offset == 0 ? 1 : 0;
  if (draw) {
    if (!w->draw_idx || !w->marks_cur || !w->draw_tiles) return SACENV_E_NULL;
    a.Gd = geom(p, sp, w->draw_g);
    a.seed = w->seed;
    a.d_idx = w->draw_idx;
    a.marks_prev = reinterpret_cast<unsigned long long*>(w->marks_prev);
    a.marks_cur = reinterpret_cast<unsigned long long*>(w->marks_cur);
    a.d_tiles = w->draw_tiles;
    a.n_draw = tiles;
  }
  if (pack || unpack) {
    if (w->cap < 0 || w->cap > total) return SACENV_E_SIZE;
    if ((int64_t)w->world * w->cap >= ((int64_t)1 << 31)) return SACENV_E_SIZE;
    a.cap = w->cap;
  }
  if (pack) {
    if (!w->stage_cur || !w->stage_prev || !w->pack_idx || !w->pack_tiles || !w->chunk) return SACENV_E_NULL;
    if (((reinterpret_cast<uintptr_t>(w->stage_cur) | reinterpret_cast<uintptr_t>(w->stage_prev)) & 15u) != 0u ||
        (reinterpret_cast<uintptr_t>(w->chunk) & 3u) != 0u)
      return SACENV_E_RANGE;
    // the roles run side by side: the pack must not read what the draws write
    if (draw && (w->pack_idx == w->draw_idx || w->pack_tiles == w->draw_tiles)) return SACENV_E_RANGE;
    a.Gp = geom(p, sp, w->pack_g);
    a.S.cur = static_cast<const char*>(w->stage_cur);
    a.S.prev = static_cast<const char*>(w->stage_prev);
    for (int k = 0; k < SACENV_OBS_DIM; ++k) a.S.first[k] = sp->first_obs[k];
    a.p_idx = w->pack_idx;
    a.p_tiles = w->pack_tiles;
    a.chunk = static_cast<uint32_t*>(w->chunk);
    a.n_pack = tiles;
  }
  if (unpack) {
    if (w->world < 1) return SACENV_E_SIZE;
    if (w->chunk_bytes < 4 * (kChunkHdr + w->cap * kRecWords) || (w->chunk_bytes & 3) != 0) return SACENV_E_SIZE;
    if ((int64_t)n_batches * words_per_batch(batch) >= ((int64_t)1 << 32)) return SACENV_E_SIZE;  // 32-bit offsets
    if (!w->words || !w->status_word) return SACENV_E_NULL;
    // nor the unpack read the chunk the pack writes
    if (pack && static_cast<const char*>(w->gathered) < static_cast<const char*>(w->chunk) + w->chunk_bytes &&
        static_cast<const char*>(w->chunk) < static_cast<const char*>(w->gathered) + w->world * w->chunk_bytes)
      return SACENV_E_RANGE;
    a.gathered = static_cast<const uint32_t*>(w->gathered);
    a.words = w->words;
    a.status = w->status_word;
    a.world = w->world;
    a.chunk_words = w->chunk_bytes / 4;
    a.per = words_per_batch(batch);
    a.u_tiles = (w->cap + kPackTile - 1) / kPackTile;
    a.n_unpack = w->world * a.u_tiles;
  }
  const int64_t blocks = a.n_draw + a.n_pack + a.n_unpack;
  if (total == 0 || blocks == 0) {
    if (pack && w->chunk) {  // no records: only the count
      const hipError_t e = hipMemsetAsync(w->chunk, 0, 4 * kChunkHdr, (hipStream_t)stream);
      return e == hipSuccess ? SACENV_OK : (int)e;
    }
    return SACENV_OK;
  }
  hipLaunchKernelGGL(k_rb_side, dim3((unsigned)blocks), dim3(kPackTile), 0, (hipStream_t)stream, a);
  return status();
}

int sacenv_copy_standin(const void* src, void* dst, int64_t bytes, int32_t workgroups, double min_us, void* stream) {
  if (bytes < 0 || (bytes & 15) != 0 || workgroups < 1 || workgroups > 4096 || !(min_us >= 0.0) || min_us > 1e5)
    return SACENV_E_SIZE;
  if ((bytes > 0 && (!src || !dst)) ||
      ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15u) != 0u)
    return bytes > 0 && (!src || !dst) ? SACENV_E_NULL : SACENV_E_RANGE;
  hipLaunchKernelGGL(k_copy_standin, dim3((unsigned)workgroups), dim3(256), 0, (hipStream_t)stream,
                     static_cast<const uint4*>(src), static_cast<uint4*>(dst), bytes / 16,
                     (uint64_t)(min_us * 100.0));
  return status();
}

}  // extern "C"
