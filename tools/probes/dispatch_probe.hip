// Dispatch cost of a refill-shaped grid: an (almost) empty kernel launched as
// 8 192 one-wave workgroups (k_refill's shape) and as 2 048 four-wave ones, each
// wave doing a short dependent load chain, timed with HIP events over 200
// launches. Writes one line per shape.
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_chain(const int* __restrict__ in, int* __restrict__ out, int hops) {
  int v = (int)(blockIdx.x * blockDim.x + threadIdx.x) & 1023;
  for (int h = 0; h < hops; ++h) v = in[v];
  if (v == -7) out[0] = v;  // never: keeps the chain
}

int main() {
  int *in, *out;
  hipMalloc(&in, 1024 * sizeof(int));
  hipMalloc(&out, sizeof(int));
  int host[1024];
  for (int i = 0; i < 1024; ++i) host[i] = (i * 7 + 3) & 1023;
  hipMemcpy(in, host, sizeof(host), hipMemcpyHostToDevice);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int shapes[][2] = {{8192, 64}, {4096, 128}, {2048, 256}, {1024, 512}};
  for (int hops : {0, 8}) {
    for (const auto& s : shapes) {
      for (int w = 0; w < 20; ++w) hipLaunchKernelGGL(k_chain, dim3(s[0]), dim3(s[1]), 0, 0, in, out, hops);
      hipEventRecord(a, 0);
      for (int r = 0; r < 200; ++r) hipLaunchKernelGGL(k_chain, dim3(s[0]), dim3(s[1]), 0, 0, in, out, hops);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0.f;
      hipEventElapsedTime(&ms, a, b);
      printf("grid %5d x %3d threads, %d dependent loads per lane: %7.2f us per launch\n", s[0], s[1], hops,
             ms * 1e3f / 200.f);
    }
  }
  return 0;
}
