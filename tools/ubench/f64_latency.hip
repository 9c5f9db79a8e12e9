// Microbenchmark: dependent vs independent v_fma_f64 issue on gfx950, one wave
// per SIMD. Prints shader cycles (s_memtime) per FMA for 1, 2, 4 and 8
// interleaved chains, and for a v_fma_f32 chain. Build: hipcc --offload-arch=gfx950 -O3.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int kChains, typename T>
__global__ void chain(T* out, long long* cyc, T a, T b, int iters) {
  T x[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) x[c] = (T)(threadIdx.x + c);
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 64; ++u)
#pragma unroll
      for (int c = 0; c < kChains; ++c) x[c] = __builtin_fma(x[c], a, b);
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  T s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += x[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// one dependent f64 chain with a wave-uniform guard branch every 16 FMAs
__global__ void guarded(double* out, long long* cyc, double a, double b, int iters) {
  double x = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
#pragma unroll
      for (int k = 0; k < 16; ++k) x = __builtin_fma(x, a, b);
      if (__ballot(!(__builtin_fabs(x) <= 1e30)) != 0ull) x = sin(x);
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = x;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int kChains, typename T>
void run(const char* name, int blocks) {
  T* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(T) * blocks * 256);
  (void)hipMalloc(&cyc, sizeof(long long) * blocks);
  const int iters = 64;
  chain<kChains, T><<<blocks, 256>>>(out, cyc, (T)0.999, (T)1e-3, iters);
  (void)hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  chain<kChains, T><<<blocks, 256>>>(out, cyc, (T)0.999, (T)1e-3, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  long long h[4];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  const double n = (double)iters * 64 * kChains;
  printf("%-10s chains %d: %.2f cycles per fma per wave (wall %.3f ms, %.2f ns per fma)\n", name, kChains,
         h[0] / n, ms, ms * 1e6 / n);
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  const int blocks = 256;  // 256 CUs x 4 waves: one wave per SIMD
  run<1, double>("f64", blocks);
  run<2, double>("f64", blocks);
  run<4, double>("f64", blocks);
  run<8, double>("f64", blocks);
  {
    double* out;
    long long* cyc;
    (void)hipMalloc(&out, sizeof(double) * blocks * 256);
    (void)hipMalloc(&cyc, sizeof(long long) * blocks);
    guarded<<<blocks, 256>>>(out, cyc, 0.999, 1e-3, 64);
    guarded<<<blocks, 256>>>(out, cyc, 0.999, 1e-3, 64);
    long long h;
    (void)hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
    printf("f64 guarded chain: %.2f cycles per fma (16 fma + 1 guard)\n", h / (64.0 * 64));
  }
  run<1, float>("f32", blocks);
  run<4, float>("f32", blocks);
  return 0;
}
