// Calibration of the rocprofv3 memory-side byte counters for k_step's access
// pattern (MI355X_MICROARCH.md: "other access widths are uncalibrated").
// k_calib8: one wave per 64 envs, 20 SoA f64 fields loaded per lane (8 B),
// 15 f64 fields stored per lane with write-through (sc1) stores, as k_step.
// k_calib16: the same bytes with 16-B per-lane accesses.
// Known bytes per launch: read 20 x 8 x 65536 = 10 485 760, write 15 x 8 x
// 65536 = 7 864 320. Run under rocprofv3 --pmc; tools/pmc_summary.py reads it.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void __launch_bounds__(64) k_calib8(const double* __restrict__ in, double* __restrict__ out, int np) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double f[20], acc = 0.0;
#pragma unroll
  for (int k = 0; k < 20; ++k) f[k] = in[(size_t)k * np + e];
#pragma unroll
  for (int k = 0; k < 20; ++k) acc += f[k];
#pragma unroll
  for (int k = 0; k < 15; ++k)
    __hip_atomic_store(&out[(size_t)k * np + e], acc + f[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ void __launch_bounds__(64) k_calib16(const double2* __restrict__ in, double2* __restrict__ out, int np) {
  const int e = blockIdx.x * 64 + threadIdx.x;
  double2 f[10];
  double acc = 0.0;
#pragma unroll
  for (int k = 0; k < 10; ++k) f[k] = in[(size_t)k * np + e];
#pragma unroll
  for (int k = 0; k < 10; ++k) acc += f[k].x + f[k].y;
#pragma unroll
  for (int k = 0; k < 7; ++k) out[(size_t)k * np + e] = make_double2(acc + f[k].x, acc + f[k].y);
  // the 15th field: 8 B (the write total matches k_calib8's)
  out[(size_t)7 * np + e].x = acc;
}

int main() {
  const int np = 65536;
  double *a, *b;
  CHECK(hipMalloc(&a, (size_t)20 * np * 8));
  CHECK(hipMalloc(&b, (size_t)16 * np * 8));
  CHECK(hipMemset(a, 0, (size_t)20 * np * 8));
  CHECK(hipMemset(b, 0, (size_t)16 * np * 8));
  for (int r = 0; r < 20; ++r) {
    hipLaunchKernelGGL(k_calib8, dim3(np / 64), dim3(64), 0, 0, a, b, np);
    hipLaunchKernelGGL(k_calib16, dim3(np / 64), dim3(64), 0, 0, (const double2*)a, (double2*)b, np);
  }
  CHECK(hipDeviceSynchronize());
  printf("calib ok: read 10485760 B, write 7864320 B per launch\n");
  return 0;
}
