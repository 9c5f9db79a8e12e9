// Microbenchmark: issue cost of the non-FMA instructions the segment step loop
// executes (conversions, rounding, ldexp, compare+select, AGPR reads, moves,
// readfirstlane, SALU interleaved with f64 FMAs), one wave per SIMD, 8
// independent streams per lane (asm volatile: nothing is hoisted or merged).
// Prints shader cycles (s_memtime) per instruction of one wave; compare with
// f64_latency's v_fma_f64 (~5.1 independent, ~5.8 dependent at one wave/SIMD).
// Build: hipcc --offload-arch=gfx950 -O3 -o valu_mix valu_mix.hip
#include <hip/hip_runtime.h>
#include <cstdio>

enum Op {
  kFma64, kCvtF32F64, kCvtI32F64, kCvtF64I32, kRndne64, kLdexp64, kFract64, kCmpSel64, kMov64,
  kAccRead, kReadFirstLane, kFmaSalu, kFmaMov32, kDiv64, kMul64F32Mix, kNops
};
static const char* kNames[] = {"v_fma_f64",     "v_cvt_f32_f64", "v_cvt_i32_f64",   "v_cvt_f64_i32",
                               "v_rndne_f64",   "v_ldexp_f64",   "v_fract_f64",     "cmp_f64+cndmask",
                               "v_mov_b64",     "accvgpr_read",  "readfirstlane",   "fma_f64+s_add",
                               "fma_f64+v_mov32", "x/y f64 (div)", "mul_f64+mul_f32", "fma_f64+s_nop0"};
static const int kInstPer[] = {1, 1, 1, 1, 1, 1, 1, 2, 1, 1, 1, 2, 2, 1, 2, 2};  // asm instructions per op

template <int kOp>
__global__ void __launch_bounds__(256) bench(double* out, long long* cyc, double a, double b, int iters) {
  constexpr int C = 8;
  double x[C], y[C];
  float f[C];
  int n[C];
  int acc_src = threadIdx.x;
#pragma unroll
  for (int c = 0; c < C; ++c) {
    x[c] = (double)(threadIdx.x + c) * 1e-3 + 1.0;
    y[c] = x[c] * 0.5;
    f[c] = 0.f;
    n[c] = c;
  }
  int s_acc = 0;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if constexpr (kOp == kFma64) {
          asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(x[c]) : "v"(a), "v"(b));
        } else if constexpr (kOp == kCvtF32F64) {
          asm volatile("v_cvt_f32_f64 %0, %1" : "=v"(f[c]) : "v"(x[c]));
        } else if constexpr (kOp == kCvtI32F64) {
          asm volatile("v_cvt_i32_f64 %0, %1" : "=v"(n[c]) : "v"(x[c]));
        } else if constexpr (kOp == kCvtF64I32) {
          asm volatile("v_cvt_f64_i32 %0, %1" : "=v"(y[c]) : "v"(n[c]));
        } else if constexpr (kOp == kRndne64) {
          asm volatile("v_rndne_f64 %0, %1" : "=v"(y[c]) : "v"(x[c]));
        } else if constexpr (kOp == kLdexp64) {
          asm volatile("v_ldexp_f64 %0, %1, %2" : "=v"(y[c]) : "v"(x[c]), "v"(n[c]));
        } else if constexpr (kOp == kFract64) {
          asm volatile("v_fract_f64 %0, %1" : "=v"(y[c]) : "v"(x[c]));
        } else if constexpr (kOp == kCmpSel64) {
          asm volatile("v_cmp_gt_f64 vcc, %1, %2\n\tv_cndmask_b32 %0, %3, %4, vcc"
                       : "=v"(n[c]) : "v"(x[c]), "v"(y[c]), "v"(n[c]), "v"(acc_src) : "vcc");
        } else if constexpr (kOp == kMov64) {
          asm volatile("v_mov_b64 %0, %1" : "=v"(y[c]) : "v"(x[c]));
        } else if constexpr (kOp == kAccRead) {
          int r;
          asm volatile("v_accvgpr_read_b32 %0, %1" : "=v"(r) : "a"(acc_src));
          n[c] = r;
        } else if constexpr (kOp == kReadFirstLane) {
          int r;
          asm volatile("v_readfirstlane_b32 %0, %1" : "=s"(r) : "v"(n[c]));
          s_acc += r;
        } else if constexpr (kOp == kFmaSalu) {
          asm volatile("v_fma_f64 %0, %0, %2, %3\n\ts_add_u32 %1, %1, 1"
                       : "+v"(x[c]), "+s"(s_acc) : "v"(a), "v"(b) : "scc");
        } else if constexpr (kOp == kFmaMov32) {
          asm volatile("v_fma_f64 %0, %0, %2, %3\n\tv_mov_b32 %1, %4"
                       : "+v"(x[c]), "=v"(n[c]) : "v"(a), "v"(b), "v"(acc_src));
        } else if constexpr (kOp == kDiv64) {
          x[c] = a / x[c];
        } else if constexpr (kOp == kMul64F32Mix) {
          asm volatile("v_mul_f64 %0, %0, %2\n\tv_mul_f32 %1, %1, %3"
                       : "+v"(x[c]), "+v"(f[c]) : "v"(a), "v"((float)b));
        } else {
          asm volatile("v_fma_f64 %0, %0, %1, %2\n\ts_nop 0" : "+v"(x[c]) : "v"(a), "v"(b));
        }
      }
    }
    asm volatile("" ::: "memory");
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  double s = (double)s_acc;
#pragma unroll
  for (int c = 0; c < C; ++c) s += x[c] + y[c] + (double)f[c] + (double)n[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int kOp>
void run() {
  const int blocks = 256, threads = 256, iters = 64, nw = blocks * threads / 64;
  double* out;
  long long* cyc;
  (void)hipMalloc(&out, sizeof(double) * blocks * threads);
  (void)hipMalloc(&cyc, sizeof(long long) * nw);
  bench<kOp><<<blocks, threads>>>(out, cyc, 0.999, 1e-3, iters);
  bench<kOp><<<blocks, threads>>>(out, cyc, 0.999, 1e-3, iters);
  (void)hipDeviceSynchronize();
  long long* h = new long long[nw];
  (void)hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
  double mean = 0;
  for (int i = 0; i < nw; ++i) mean += (double)h[i];
  mean /= nw;
  const double ops = (double)iters * 16 * 8;
  printf("%-18s %6.2f cyc/op  %6.2f cyc/instruction (one wave per SIMD)\n", kNames[kOp], mean / ops,
         mean / ops / kInstPer[kOp]);
  delete[] h;
  (void)hipFree(out);
  (void)hipFree(cyc);
}

int main() {
  run<kFma64>();
  run<kCvtF32F64>();
  run<kCvtI32F64>();
  run<kCvtF64I32>();
  run<kRndne64>();
  run<kLdexp64>();
  run<kFract64>();
  run<kCmpSel64>();
  run<kMov64>();
  run<kAccRead>();
  run<kReadFirstLane>();
  run<kFmaSalu>();
  run<kFmaMov32>();
  run<kDiv64>();
  run<kMul64F32Mix>();
  run<kNops>();
  return 0;
}
