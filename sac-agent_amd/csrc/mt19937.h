// mt19937.h — numpy-legacy MT19937 (numpy/random/src/mt19937, pinned numpy
// 1.23.5) for one wave64: lane-parallel twist in LDS, 64-word windows.
// Included INSIDE an anonymous namespace of each .hip translation unit (after
// kWave and the kMt* constants); the LDS type L has `uint32_t blk[2][624]`.
#pragma once

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
  int pos;   // offset of the next unconsumed word in the current block
  int cur;   // which L::blk holds the current block (when loaded)
  bool loaded;
  bool nxt_valid;
  bool advanced;  // current block differs from gkey
};

template <class L>
__device__ uint32_t mt_fetch(MtStream& st, L& l, int lane) {
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

template <class L>
__device__ void mt_finish(MtStream& st, L& l, int32_t* gpos, int lane) {
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

