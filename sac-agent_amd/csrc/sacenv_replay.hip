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

}  // extern "C"
