// Probe: does a one-wave-per-SIMD step-shaped kernel (1024 waves x 64 lanes,
// ~160 B read + ~120 B written per lane, then launch boundary) run faster with
// 16-B per-lane accesses (paired fields) than with 8-B per-lane SoA accesses?
// Writes are sc1 (write-through) as in k_step. Prints us per launch.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

constexpr int NF_R = 20, NF_W = 15;  // 8-B fields read / written per env

template <class T> __device__ __forceinline__ void st_wt(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) k8(const double* __restrict__ in, double* __restrict__ out, int np, int iters) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double f[NF_R];
#pragma unroll
  for (int k = 0; k < NF_R; ++k) f[k] = in[(size_t)k * np + e];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NF_R; ++k) acc = acc * 1.0000001 + f[k];
  for (int i = 0; i < iters; ++i) acc = fma(acc, 0.999999, 1e-9);
#pragma unroll
  for (int k = 0; k < NF_W; ++k) st_wt(&out[(size_t)k * np + e], acc + f[k]);
}

__global__ void __launch_bounds__(64) k16(const double2* __restrict__ in, double2* __restrict__ out, int np, int iters) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double2 f[NF_R / 2];
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) f[k] = in[(size_t)k * np + e];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) acc = (acc * 1.0000001 + f[k].x) * 1.0000001 + f[k].y;
  for (int i = 0; i < iters; ++i) acc = fma(acc, 0.999999, 1e-9);
#pragma unroll
  for (int k = 0; k < (NF_W + 1) / 2; ++k) {
    double2 v = make_double2(acc + f[k].x, acc + f[k].y);
    // 16-B write-through store: two 8-B atomics would split it; use nontemporal 16-B
    __builtin_nontemporal_store(v.x, &out[(size_t)k * np + e].x);
    __builtin_nontemporal_store(v.y, &out[(size_t)k * np + e].y);
  }
}

__global__ void __launch_bounds__(64) k16p(const double2* __restrict__ in, double2* __restrict__ out, int np, int iters) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double2 f[NF_R / 2];
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) f[k] = in[(size_t)k * np + e];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) acc = (acc * 1.0000001 + f[k].x) * 1.0000001 + f[k].y;
  for (int i = 0; i < iters; ++i) acc = fma(acc, 0.999999, 1e-9);
#pragma unroll
  for (int k = 0; k < (NF_W + 1) / 2; ++k) out[(size_t)k * np + e] = make_double2(acc + f[k].x, acc + f[k].y);
}

__global__ void __launch_bounds__(64) k8p(const double* __restrict__ in, double* __restrict__ out, int np, int iters) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double f[NF_R];
#pragma unroll
  for (int k = 0; k < NF_R; ++k) f[k] = in[(size_t)k * np + e];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NF_R; ++k) acc = acc * 1.0000001 + f[k];
  for (int i = 0; i < iters; ++i) acc = fma(acc, 0.999999, 1e-9);
#pragma unroll
  for (int k = 0; k < NF_W; ++k) out[(size_t)k * np + e] = acc + f[k];
}

typedef unsigned int u4v __attribute__((ext_vector_type(4)));
__global__ void __launch_bounds__(64) k16s(const double2* __restrict__ in, double2* __restrict__ out, int np, int iters) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double2 f[NF_R / 2];
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) f[k] = in[(size_t)k * np + e];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < NF_R / 2; ++k) acc = (acc * 1.0000001 + f[k].x) * 1.0000001 + f[k].y;
  for (int i = 0; i < iters; ++i) acc = fma(acc, 0.999999, 1e-9);
  __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
#pragma unroll
  for (int k = 0; k < (NF_W + 1) / 2; ++k) {
    double2 v = make_double2(acc + f[k].x, acc + f[k].y);
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, v), r, (uint32_t)(((size_t)k * np + e) * 16), 0, 16);
  }
}

int main() {
  const int np = 65536, waves = np / 64;
  double *a, *b;
  CHECK(hipMalloc(&a, (size_t)NF_R * np * 8 * 2));
  CHECK(hipMalloc(&b, (size_t)NF_R * np * 8 * 2));
  CHECK(hipMemset(a, 0, (size_t)NF_R * np * 8 * 2));
  CHECK(hipMemset(b, 0, (size_t)NF_R * np * 8 * 2));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int reps = 2000;
  for (int iters : {0, 300}) {
    for (int v = 0; v < 5; ++v) {
      for (int round = 0; round < 2; ++round) {
        hipGraph_t g;
        hipGraphExec_t ge;
        CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
        for (int r = 0; r < 128; ++r) {
          // ping-pong so each launch reads what the previous one wrote
          double* src = (r & 1) ? b : a;
          double* dst = (r & 1) ? a : b;
          if (v == 0) hipLaunchKernelGGL(k8, dim3(waves), dim3(64), 0, s, src, dst, np, iters);
          if (v == 1) hipLaunchKernelGGL(k16, dim3(waves), dim3(64), 0, s, (double2*)src, (double2*)dst, np, iters);
          if (v == 2) hipLaunchKernelGGL(k8p, dim3(waves), dim3(64), 0, s, src, dst, np, iters);
          if (v == 3) hipLaunchKernelGGL(k16p, dim3(waves), dim3(64), 0, s, (double2*)src, (double2*)dst, np, iters);
          if (v == 4) hipLaunchKernelGGL(k16s, dim3(waves), dim3(64), 0, s, (double2*)src, (double2*)dst, np, iters);
        }
        CHECK(hipStreamEndCapture(s, &g));
        CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
        for (int w = 0; w < 3; ++w) CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e0, s));
        for (int w = 0; w < reps / 128; ++w) CHECK(hipGraphLaunch(ge, s));
        CHECK(hipEventRecord(e1, s));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        const char* nm[] = {"8B sc1 stores", "16B nt stores", "8B plain", "16B plain", "16B sc1 buffer"};
        printf("iters %3d %-14s round %d: %.3f us/launch\n", iters, nm[v], round, ms * 1e3 / (reps / 128 * 128));
        CHECK(hipGraphExecDestroy(ge));
        CHECK(hipGraphDestroy(g));
      }
    }
  }
  return 0;
}
