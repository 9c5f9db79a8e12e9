// Microbenchmark: FP64 VALU issue and dependent latency on gfx950.
//
// For each op (v_fma_f64, v_mul_f64, v_add_f64, v_fma_f32, an f64 FMA chain with an
// independent integer chain beside it, v_rcp_f64) and each number of independent
// chains per lane (1, 2, 4, 8), one kernel runs 64 x 64 x chains ops per lane at 1 and
// 2 waves per SIMD (256 workgroups of 256 or 512 threads on 256 CUs). Reported:
//   cyc/inst/wave  shader cycles (s_memtime) per instruction of one wave
//   cyc/inst/SIMD  the same divided by the waves sharing the SIMD: the SIMD's issue
//                  interval for this op (4.0 = one wave64 instruction every 4 cycles)
//   TFLOP/s        chip-wide, from the wall time of the launch (FMA = 2 flops)
// Build: hipcc --offload-arch=gfx950 -O3 -o f64_latency f64_latency.hip
#include <hip/hip_runtime.h>
#include <cstdio>

enum Op { kFma64, kMul64, kAdd64, kFma32, kFma64Int, kRcp64 };

template <int kOp, int kChains>
__global__ void __launch_bounds__(512) chain(double* out, long long* cyc, double a, double b, int iters) {
  double x[kChains];
  float xf[kChains];
  int xi[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    x[c] = (double)(threadIdx.x + c) * 1e-3 + 1.0;
    xf[c] = (float)x[c];
    xi[c] = threadIdx.x + c;
  }
  const float af = (float)a, bf = (float)b;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 64; ++u) {
#pragma unroll
      for (int c = 0; c < kChains; ++c) {
        if constexpr (kOp == kFma64) {
          x[c] = __builtin_fma(x[c], a, b);
        } else if constexpr (kOp == kMul64) {
          x[c] = x[c] * a;
        } else if constexpr (kOp == kAdd64) {
          x[c] = x[c] + b;
        } else if constexpr (kOp == kFma32) {
          xf[c] = __builtin_fmaf(xf[c], af, bf);
        } else if constexpr (kOp == kFma64Int) {
          x[c] = __builtin_fma(x[c], a, b);
          xi[c] = xi[c] * 3 + 7;
        } else {
          x[c] = __builtin_amdgcn_rcp(x[c]);
        }
      }
    }
    asm volatile("" ::: "memory");
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = 0;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += x[c] + (double)xf[c] + (double)xi[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char* kNames[] = {"v_fma_f64", "v_mul_f64", "v_add_f64", "v_fma_f32", "fma_f64+int", "v_rcp_f64"};

template <int kOp, int kChains>
void run(int waves_per_simd) {
  const int blocks = 256, threads = 256 * waves_per_simd, iters = 64;
  double* out;
  long long* cyc;
  const int nw = blocks * threads / 64;
  (void)hipMalloc(&out, sizeof(double) * blocks * threads);
  (void)hipMalloc(&cyc, sizeof(long long) * nw);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  chain<kOp, kChains><<<blocks, threads>>>(out, cyc, 0.999, 1e-3, iters);
  (void)hipEventRecord(e0);
  chain<kOp, kChains><<<blocks, threads>>>(out, cyc, 0.999, 1e-3, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  long long* h = new long long[nw];
  (void)hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < nw; ++i) mean += (double)h[i];
  mean /= nw;
  const double n = (double)iters * 64 * kChains;   // instructions of the measured op per wave
  const double flops = (kOp == kFma64 || kOp == kFma32 || kOp == kFma64Int) ? 2.0 : 1.0;
  printf("%-12s chains %d waves/SIMD %d: %6.2f cyc/inst/wave  %5.2f cyc/inst/SIMD  %6.1f TFLOP/s  (%.3f ms)\n",
         kNames[kOp], kChains, waves_per_simd, mean / n, mean / n / waves_per_simd,
         flops * n * 64.0 * nw / (ms * 1e-3) / 1e12, ms);
  delete[] h;
  (void)hipFree(out);
  (void)hipFree(cyc);
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
}

template <int kOp>
void sweep() {
  for (int w = 1; w <= 2; ++w) {
    run<kOp, 1>(w);
    run<kOp, 2>(w);
    run<kOp, 4>(w);
    run<kOp, 8>(w);
  }
}

int main() {
  sweep<kFma64>();
  sweep<kMul64>();
  sweep<kAdd64>();
  sweep<kFma32>();
  sweep<kFma64Int>();
  sweep<kRcp64>();
  return 0;
}
