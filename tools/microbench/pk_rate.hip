// pk_rate.hip -- issue rate of v_pk_fma_f32 vs v_fma_f32 on one SIMD (independent chains).
#include <hip/hip_runtime.h>
#include <stdio.h>
typedef float v2 __attribute__((ext_vector_type(2)));
template <int PK>
__global__ __launch_bounds__(256) void k(float *out, float a, float b, int iters) {
  float x[16];
  v2 y[8];
#pragma unroll
  for (int i = 0; i < 16; ++i) x[i] = threadIdx.x + i;
#pragma unroll
  for (int i = 0; i < 8; ++i) y[i] = v2{(float)threadIdx.x + i, (float)i};
  for (int it = 0; it < iters; ++it) {
    if (PK) {
#pragma unroll
      for (int i = 0; i < 8; ++i) y[i] = __builtin_elementwise_fma(y[i], v2{a, a}, v2{b, b});
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) x[i] = fmaf(x[i], a, b);
    }
  }
  float s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += x[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) s += y[i].x + y[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
int main() {
  float *o;
  hipMalloc(&o, 256 * 1024 * 16 * sizeof(float));
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 20000, blocks = 256 * 16;
  for (int rep = 0; rep < 2; ++rep)
    for (int pk = 0; pk < 2; ++pk) {
      hipEventRecord(e0);
      if (pk) k<1><<<blocks, 256>>>(o, 0.999f, 0.001f, iters);
      else k<0><<<blocks, 256>>>(o, 0.999f, 0.001f, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      const double fmas = (double)blocks * 256 * iters * 16;
      printf("%s: %.3f ms  %.1f TFLOP/s (fp32 FMA lanes)\n", pk ? "v_pk_fma_f32" : "v_fma_f32   ", ms, 2 * fmas / ms / 1e9);
    }
  return 0;
}
