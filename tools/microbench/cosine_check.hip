// cosine_check.hip -- how close the gfx950 hardware square root / reciprocal square root / reciprocal
// come to the correctly rounded IEEE results the oracle's cosines use (the fast
// shading's parity): over every fp32 significand in [1, 4) (two binades: sqrt depends on the
// exponent's parity), count the inputs where
//   v_sqrt_f32(x) != RN(sqrt x),  v_rsq_f32(x) != RN(1 / sqrt x),  v_rcp_f32(x) != RN(1 / x),
// and for the short quotient q = fma(fma(-b, a y, a), y, a y), y = v_rcp_f32(b) (no Newton step on
// y), the pairs (a, b) -- b every significand in [1, 2), a 64 pseudo-random values in [2^-8, 2) --
// where q != RN(a / b).  References in double (innocuous double rounding for sqrt and division).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>

__global__ void unary(unsigned long long *cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (2u << 23)) return;
  const float x = __uint_as_float(0x3f800000u + i);  // [1, 4)
  const float s_ref = (float)sqrt((double)x);
  const float r_ref = (float)(1.0 / sqrt((double)x));
  const float c_ref = (float)(1.0 / (double)x);
  if (__builtin_amdgcn_sqrtf(x) != s_ref) atomicAdd(cnt + 0, 1ull);
  if (__builtin_amdgcn_rsqf(x) != r_ref) atomicAdd(cnt + 1, 1ull);
  if (__builtin_amdgcn_rcpf(x) != c_ref) atomicAdd(cnt + 2, 1ull);
  // the oracle's RN(1 / RN(sqrt x)) against the hardware rsq
  if (__builtin_amdgcn_rsqf(x) != (float)(1.0 / (double)s_ref)) atomicAdd(cnt + 3, 1ull);
}

__global__ void quot(unsigned long long *cnt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= (1u << 23)) return;
  const float b = __uint_as_float(0x3f800000u | i);
  const float y = __builtin_amdgcn_rcpf(b);
  uint32_t h = i * 2654435761u + 12345u;
  for (int k = 0; k < 64; ++k) {
    h ^= h << 13; h ^= h >> 17; h ^= h << 5;
    const float a = __uint_as_float(0x3b800000u + h % (0x3fffffffu - 0x3b800000u));
    const float q0 = a * y;
    const float q = fmaf(fmaf(-b, q0, a), y, q0);
    if (q != (float)((double)a / (double)b)) atomicAdd(cnt + 4, 1ull);
  }
}

int main() {
  unsigned long long *d, h[5] = {0, 0, 0, 0, 0};
  if (hipMalloc(&d, sizeof h)) return 1;
  hipMemset(d, 0, sizeof h);
  hipLaunchKernelGGL(unary, dim3((2u << 23) / 256), dim3(256), 0, 0, d);
  hipLaunchKernelGGL(quot, dim3((1u << 23) / 256), dim3(256), 0, 0, d);
  if (hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost)) return 1;
  const double nu = (double)(2u << 23), nq = (double)(1u << 23) * 64;
  printf("v_sqrt_f32 != RN(sqrt):            %llu of %.0f (%.3g)\n", h[0], nu, h[0] / nu);
  printf("v_rsq_f32  != RN(1/sqrt):          %llu of %.0f (%.3g)\n", h[1], nu, h[1] / nu);
  printf("v_rcp_f32  != RN(1/x):             %llu of %.0f (%.3g)\n", h[2], nu, h[2] / nu);
  printf("v_rsq_f32  != RN(1/RN(sqrt)):      %llu of %.0f (%.3g)\n", h[3], nu, h[3] / nu);
  printf("short quotient != RN(a/b):         %llu of %.0f (%.3g)\n", h[4], nq, h[4] / nq);
  return 0;
}
