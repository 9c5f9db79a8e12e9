// Diagnostic: which XCD each workgroup of a 1536-block launch runs on, over
// consecutive launches (eager and graph-replayed). Answers whether an env
// block's L2 (per-XCD) is the same from one step launch to the next.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>

__global__ void probe(int* out, int launch, int nb) {
  if (threadIdx.x != 0) return;
  unsigned x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(x));
  out[launch * nb + blockIdx.x] = (int)x;
}

int main() {
  const int nb = 1536, L = 24;
  int* d;
  hipMalloc(&d, sizeof(int) * nb * L);
  hipStream_t s;
  hipStreamCreate(&s);
  for (int l = 0; l < L / 2; ++l) hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d, l, nb);
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
  for (int l = L / 2; l < L; ++l) hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d, l, nb);
  hipStreamEndCapture(s, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  hipGraphLaunch(ge, s);
  hipStreamSynchronize(s);
  std::vector<int> h(nb * L);
  hipMemcpy(h.data(), d, sizeof(int) * nb * L, hipMemcpyDeviceToHost);
  for (int l = 0; l < L; ++l) {
    int same = 0, rr = 0;
    for (int b = 0; b < nb; ++b) {
      same += h[l * nb + b] == h[b];
      rr += h[l * nb + b] == (h[l * nb] + b) % 8;
    }
    printf("launch %2d (%s): block0..7 xcd:", l, l < L / 2 ? "eager" : "graph");
    for (int b = 0; b < 8; ++b) printf(" %d", h[l * nb + b]);
    printf(" | same-as-launch0 %4d/%d | round-robin-from-block0 %4d/%d\n", same, nb, rr, nb);
  }
  return 0;
}
