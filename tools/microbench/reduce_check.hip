// reduce_check.hip -- checks vr_stage.h wave_min / wave_max (DPP + permlane swaps) against a
// brute-force reduction over random inputs, every lane and every wave.
// Build: hipcc --offload-arch=gfx950 -O3 -I../../volume_renderer_amd/csrc reduce_check.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include "vr_stage.h"

__global__ void k(const int *in, int *bad) {
  const int lane = threadIdx.x & 63;
  const int base = (blockIdx.x * blockDim.x + threadIdx.x) & ~63;
  const int v = in[base + lane];
  const int mn = vr::wave_min(v), mx = vr::wave_max(v);
  int bmn = in[base], bmx = in[base];
  for (int i = 1; i < 64; ++i) {
    bmn = min(bmn, in[base + i]);
    bmx = max(bmx, in[base + i]);
  }
  if (mn != bmn || mx != bmx) atomicAdd(bad, 1);
}

int main() {
  const int n = 64 * 4096;
  int *h = new int[n];
  unsigned s = 12345u;
  for (int i = 0; i < n; ++i) {
    s = s * 1664525u + 1013904223u;
    h[i] = (int)(s >> 8) % 4000 - 2000;
  }
  int *d, *bad, hb = 0;
  hipMalloc(&d, n * sizeof(int));
  hipMalloc(&bad, sizeof(int));
  hipMemcpy(d, h, n * sizeof(int), hipMemcpyHostToDevice);
  hipMemcpy(bad, &hb, sizeof(int), hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(d, bad);
  hipMemcpy(&hb, bad, sizeof(int), hipMemcpyDeviceToHost);
  printf("wave_min/wave_max mismatching lanes: %d of %d\n", hb, n);
  return hb != 0;
}
