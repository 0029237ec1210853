// exp_check.hip -- how the device's exponentials round exp(-x) for the opacity's small arguments
// (DESIGN.md s6): the device library expf, __expf's form exp2(x * log2 e) on v_exp_f32, and the
// Taylor form exp_neg_rn of vr_sampling.h, each against glibc's expf on the host (the oracle's),
// over every STRIDE-th positive float below 2^-7.  Prints, per method: inputs, results differing
// from glibc, and how many of those are above / below it (a one-sided excess is a bias).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <vector>

__device__ __forceinline__ float exp_neg_rn_dev(float x) {
  const float x2 = x * x;
  const float q = fmaf(x, x * (1.f / 24.f) + (-1.f / 6.f), 0.5f);
  return 1.f + fmaf(x2, q, -x);
}

__global__ void k(const float *x, float *o, size_t n) {
  const size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float v = x[i];
  o[3 * i + 0] = expf(-v);
  o[3 * i + 1] = __builtin_amdgcn_exp2f((-v) * 0x1.715476p+0f);
  o[3 * i + 2] = exp_neg_rn_dev(v);
}

int main() {
  const uint32_t stride = 101;
  std::vector<float> xs;
  for (uint32_t u = 1;; u += stride) {
    float x;
    memcpy(&x, &u, 4);
    if (!(x < 0x1p-7f)) break;
    xs.push_back(x);
  }
  const size_t n = xs.size();
  float *dx, *dout;
  if (hipMalloc(&dx, n * 4) || hipMalloc(&dout, 3 * n * 4)) return 1;
  hipMemcpy(dx, xs.data(), n * 4, hipMemcpyHostToDevice);
  k<<<(unsigned)((n + 255) / 256), 256>>>(dx, dout, n);
  std::vector<float> out(3 * n);
  hipMemcpy(out.data(), dout, 3 * n * 4, hipMemcpyDeviceToHost);
  const char *names[3] = {"device expf", "exp2(x*log2e) (v_exp_f32)", "exp_neg_rn (Taylor)"};
  for (int m = 0; m < 3; ++m) {
    size_t diff = 0, up = 0, dn = 0;
    for (size_t i = 0; i < n; ++i) {
      const float g = expf(-xs[i]), d = out[3 * i + m];
      if (d != g) {
        ++diff;
        (d > g ? up : dn)++;
      }
    }
    printf("%-28s inputs %zu differ %zu (%.4f %%) above %zu below %zu\n", names[m], n, diff, 100.0 * diff / n, up, dn);
  }
  return 0;
}
