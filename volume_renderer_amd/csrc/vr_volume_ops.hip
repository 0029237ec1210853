// vr_volume_ops.hip -- the MATLAB-side volume preprocessing of the reference, on the device
// (SURVEY.md 8f row 4): the illumination LUT generator, Volume.normalize and Volume.resize.  A
// 1024^3 single volume is 4 GiB; in the reference these run on the host in MATLAB before the data
// is uploaded (examples/example1.m, example3.m:86-89).
//
//   hg_lut_kernel      HenyeyGreenstein(N, g)        src/C/mex/HenyeyGreenstein.cc:29-96
//   minmax / normalize Volume.normalize(min, max)    src/matlab/VolumeRender/Volume.m:208-220
//   resize_dim_kernel  Volume.resize(newsize)        src/matlab/VolumeRender/Volume.m:93-106
//                      (imresize3, cubic, antialiasing when shrinking; weights from the host)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "vr_device.h"

namespace vr {

// HenyeyGreenstein.cc:52-88 for the element (c, a, b) at c*N*N + a*N + b.  The sines and cosines of
// k*pi/N come from the host (sinf / cosf there, so they are the host generator's own values); the
// rest is the generator's single-precision expression, op for op (the power of 3 from the device
// math library, which is where device and host can differ).
__global__ __launch_bounds__(256) void hg_lut_kernel(uint32_t n, const float *__restrict__ sn, const float *__restrict__ cs,
                                                     float g, float g2, float num, float *__restrict__ out) {
  const uint64_t total = (uint64_t)n * n * n;
  const float inv4pi = 1.f / (4.f * ((float)3.141592653589793238462643383279502884197169399375105820));
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < total; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t b = (uint32_t)(q % n), a = (uint32_t)((q / n) % n), c = (uint32_t)(q / ((uint64_t)n * n));
    const float s = sn[c], co = cs[c];
    const float lx = sn[a], lz = cs[a];
    const float rx = 1.f * lx + 0.f * 0.f + 0.f * lz;
    const float ry = 0.f * lx + co * 0.f + s * lz;
    const float rz = 0.f * lx + -s * 0.f + co * lz;
    const float ix = sn[b], iz = cs[b];
    const float cos_theta = rx * ix + ry * 0.f + rz * iz;
    const float den = sqrtf(powf((1.f + g2 - (2.f * g * cos_theta)), 3.f));
    out[q] = inv4pi * (num / den);
  }
}

// MATLAB max / min of single data (NaN omitted; all-NaN or empty gives NaN): ordered-integer
// atomics over the finite-or-infinite values.
__device__ __forceinline__ uint32_t ordered(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float unordered(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

__global__ __launch_bounds__(256) void minmax_kernel(const float *__restrict__ d, uint64_t n, uint32_t *mm) {
  uint32_t lo = 0xffffffffu, hi = 0u;  // ordered min / max of the non-NaN values
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const float v = d[q];
    if (v == v) {
      const uint32_t o = ordered(v);
      lo = min(lo, o);
      hi = max(hi, o);
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    lo = min(lo, (uint32_t)__shfl_xor((int)lo, off, 64));
    hi = max(hi, (uint32_t)__shfl_xor((int)hi, off, 64));
  }
  if ((threadIdx.x & 63) == 0) {
    atomicMin(mm, lo);
    atomicMax(mm + 1, hi);
  }
}

// Volume.normalize (Volume.m:208-220) in MATLAB's single arithmetic: (Data - min) * single(newMax -
// newMin) / (max - min) + single(newMin), every operation rounded to single, left to right.
__global__ __launch_bounds__(256) void normalize_kernel(const float *__restrict__ d, uint64_t n, const uint32_t *mm,
                                                        float range, float new_min, float *__restrict__ out) {
  const bool any = mm[0] != 0xffffffffu;  // some non-NaN value
  const float mn = any ? unordered(mm[0]) : __uint_as_float(0x7fc00000u);
  const float mx = any ? unordered(mm[1]) : __uint_as_float(0x7fc00000u);
  const float span = mx - mn;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const float t1 = d[q] - mn;
    const float t2 = t1 * range;
    const float t3 = t2 / span;
    out[q] = t3 + new_min;
  }
}

// One separable pass of imresize3 along axis `dim` of a column-major (n0, n1, n2) volume: output
// index o along the axis takes sum_p w[o*P + p] * in[idx[o*P + p]] in double, in p order, rounded
// to single (the contributions w / idx -- kernel weights and mirrored indices -- are computed on
// the host, vr_capi.hip resize_contributions).
__global__ __launch_bounds__(256) void resize_dim_kernel(const float *__restrict__ in, uint64_t n0, uint64_t n1,
                                                         uint64_t n2, int dim, uint64_t out_len,
                                                         const double *__restrict__ w, const int32_t *__restrict__ idx,
                                                         int32_t P, float *__restrict__ out) {
  const uint64_t m0 = dim == 0 ? out_len : n0, m1 = dim == 1 ? out_len : n1, m2 = dim == 2 ? out_len : n2;
  const uint64_t total = m0 * m1 * m2;
  const uint64_t stride = dim == 0 ? 1 : (dim == 1 ? n0 : n0 * n1);
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < total; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i0 = q % m0, r = q / m0, i1 = r % m1, i2 = r / m1;
    const uint64_t o = dim == 0 ? i0 : (dim == 1 ? i1 : i2);
    const uint64_t base = (dim == 0 ? 0 : i0) + (dim == 1 ? 0 : i1 * n0) + (dim == 2 ? 0 : i2 * n0 * n1);
    double acc = 0.0;
    for (int32_t p = 0; p < P; ++p) {
      const double wt = w[o * (uint64_t)P + (uint64_t)p];
      const double v = (double)in[base + (uint64_t)idx[o * (uint64_t)P + (uint64_t)p] * stride];
      acc = acc + wt * v;
    }
    out[q] = (float)acc;
  }
}

static unsigned grid_for(uint64_t n, unsigned cap) {
  const uint64_t b = (n + 255) / 256;
  return (unsigned)(b < cap ? (b ? b : 1) : cap);
}

hipError_t launch_hg_lut(uint32_t n, const float *sn, const float *cs, float g, float g2, float num, float *out,
                         hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(hg_lut_kernel, dim3(grid_for((uint64_t)n * n * n, 65536)), dim3(256), 0, s, n, sn, cs, g, g2, num,
                     out);
  return hipGetLastError();
}

hipError_t launch_normalize(const float *d, uint64_t n, uint32_t *mm, float range, float new_min, float *out,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  hipError_t rc = hipMemsetAsync(mm, 0xff, sizeof(uint32_t), s);
  if (rc == hipSuccess) rc = hipMemsetAsync(mm + 1, 0, sizeof(uint32_t), s);
  if (rc != hipSuccess) return rc;
  hipLaunchKernelGGL(minmax_kernel, dim3(grid_for(n, 16384)), dim3(256), 0, s, d, n, mm);
  hipLaunchKernelGGL(normalize_kernel, dim3(grid_for(n, 65536)), dim3(256), 0, s, d, n, (const uint32_t *)mm, range,
                     new_min, out);
  return hipGetLastError();
}

hipError_t launch_resize_dim(const float *in, const uint64_t dims[3], int dim, uint64_t out_len, const double *w,
                             const int32_t *idx, int32_t P, float *out, hipStream_t s) {
  const uint64_t total = (dim == 0 ? out_len : dims[0]) * (dim == 1 ? out_len : dims[1]) * (dim == 2 ? out_len : dims[2]);
  if (!total) return hipSuccess;
  hipLaunchKernelGGL(resize_dim_kernel, dim3(grid_for(total, 65536)), dim3(256), 0, s, in, dims[0], dims[1], dims[2], dim,
                     out_len, w, idx, P, out);
  return hipGetLastError();
}

}  // namespace vr
