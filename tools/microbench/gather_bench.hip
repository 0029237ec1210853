// gather_bench.hip -- gfx950 microbenchmark for the ray-march design decisions.
// Measures, per CU, the sustained rate of
//   (1) global dword / dwordx2 / dwordx4 gathers with K distinct 128-B lines per wave-instruction
//       from tables of increasing size (L1/L2/MALL/HBM resident),
//   (2) LDS ds_read_b32 gathers with random addresses,
//   (3) dependent VALU chains vs independent (v_fma), v_exp/v_rsq/v_sqrt issue cost.
// Build: hipcc --offload-arch=gfx950 -O3 gather_bench.hip -o gather_bench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <vector>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// Each lane owns a pseudo-random walk; per iteration it loads from addr = base + f(lane group, iter).
// `lines` = distinct 128-B lines per wave-instruction (lanes share a line in groups of 64/lines).
template <int VEC>
__global__ __launch_bounds__(256) void gather_kernel(const float *__restrict__ tab, uint64_t tab_floats,
                                                     int iters, int lines, float *__restrict__ sink) {
  // 8 independent loads per iteration; addresses from a cheap xorshift, masks only (no division)
  const int lane = threadIdx.x & 63;
  const int per = 64 / lines;
  const int group = lane / per;
  const int within = lane % per;
  uint32_t s = (blockIdx.x * 4 + (threadIdx.x >> 6)) * 2654435761u + group * 40503u + 12345u;
  const uint32_t line_mask = (uint32_t)(tab_floats / 32) - 1u;
  const uint32_t off = (uint32_t)((within * VEC) & 31);
  float acc = 0.f;
  for (int it = 0; it < iters; it += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s ^= s << 13; s ^= s >> 17; s ^= s << 5;
      const uint64_t idx = (uint64_t)(s & line_mask) * 32 + off;
      if (VEC == 1) v[k] = tab[idx];
      else if (VEC == 2) { float2 q = *reinterpret_cast<const float2 *>(tab + idx); v[k] = q.x + q.y; }
      else { float4 q = *reinterpret_cast<const float4 *>(tab + idx); v[k] = (q.x + q.y) + (q.z + q.w); }
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (acc == 1234.5f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void lds_gather_kernel(int iters, int span, float *__restrict__ sink) {
  __shared__ float lds[16384];
  for (int i = threadIdx.x; i < 16384; i += 256) lds[i] = (float)i;
  __syncthreads();
  uint32_t s = threadIdx.x * 2654435761u + blockIdx.x + 1;
  const uint32_t mask = (uint32_t)span - 1u;
  float acc = 0.f;
  for (int it = 0; it < iters; it += 8) {
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      s ^= s << 13; s ^= s >> 17; s ^= s << 5;
      v[k] = lds[s & mask];
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) acc += v[k];
  }
  if (acc == 1234.5f) sink[0] = acc;
}

__global__ __launch_bounds__(256) void valu_kernel(int iters, float *__restrict__ sink, float a0) {
  float a = a0 + threadIdx.x, b = a0 * 2, c = a0 * 3, d = a0 * 4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      a = fmaf(a, 1.0001f, 0.5f); b = fmaf(b, 0.9999f, 0.25f);
      c = fmaf(c, 1.0002f, 0.125f); d = fmaf(d, 0.9998f, 0.0625f);
    }
  }
  if (a + b + c + d == 1234.5f) sink[0] = a;
}

__global__ __launch_bounds__(256) void trans_kernel(int iters, float *__restrict__ sink, float a0) {
  float a = a0 + threadIdx.x * 1e-3f, b = a0 * 0.5f, c = a0 * 0.25f, d = a0 * 0.125f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a = __builtin_amdgcn_rsqf(a + 1.f); b = __builtin_amdgcn_exp2f(b * 0.5f);
      c = __builtin_amdgcn_rsqf(c + 1.f); d = __builtin_amdgcn_exp2f(d * 0.5f);
    }
  }
  if (a + b + c + d == 1234.5f) sink[0] = a;
}

static float time_ms(hipEvent_t e0, hipEvent_t e1) { float ms; CHECK(hipEventElapsedTime(&ms, e0, e1)); return ms; }

int main() {
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  const int cus = prop.multiProcessorCount;
  printf("device %s CUs %d clock %d kHz\n", prop.name, cus, prop.clockRate);
  float *sink;
  CHECK(hipMalloc(&sink, 4));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const int blocks = cus * 8, iters = 2000;
  const double ghz = 2.4;
  std::vector<uint64_t> sizes = {8ull << 10, 1ull << 20, 16ull << 20, 512ull << 20, 4096ull << 20};
  float *tab;
  CHECK(hipMalloc(&tab, sizes.back()));
  CHECK(hipMemset(tab, 0, sizes.back()));
  for (int vec : {1, 2, 4}) {
    for (uint64_t bytes : sizes) {
      for (int lines : {1, 4, 16, 64}) {
        auto run = [&]() {
          if (vec == 1) hipLaunchKernelGGL(gather_kernel<1>, dim3(blocks), dim3(256), 0, 0, tab, bytes / 4, iters, lines, sink);
          if (vec == 2) hipLaunchKernelGGL(gather_kernel<2>, dim3(blocks), dim3(256), 0, 0, tab, bytes / 4, iters, lines, sink);
          if (vec == 4) hipLaunchKernelGGL(gather_kernel<4>, dim3(blocks), dim3(256), 0, 0, tab, bytes / 4, iters, lines, sink);
        };
        run();
        CHECK(hipEventRecord(e0));
        run();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        const double ms = time_ms(e0, e1);
        const double winst = (double)blocks * 4 * iters;  // wave-instructions
        const double cyc_per_inst_cu = ms * 1e-3 * ghz * 1e9 / (winst / cus);
        printf("gather vec%d table %8llu KB lines/inst %2d : %7.2f cycles per wave-load per CU, %8.1f GB/s useful\n",
               vec, (unsigned long long)(bytes >> 10), lines, cyc_per_inst_cu,
               winst * 64 * 4 * vec / (ms * 1e-3) / 1e9);
      }
    }
  }
  for (int span : {64, 1024, 16384}) {
    hipLaunchKernelGGL(lds_gather_kernel, dim3(blocks), dim3(256), 0, 0, iters, span, sink);
    CHECK(hipEventRecord(e0));
    hipLaunchKernelGGL(lds_gather_kernel, dim3(blocks), dim3(256), 0, 0, iters, span, sink);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    const double ms = time_ms(e0, e1);
    const double winst = (double)blocks * 4 * iters;
    printf("lds gather span %5d floats: %6.2f cycles per wave ds_read per CU\n", span,
           ms * 1e-3 * ghz * 1e9 / (winst / cus));
  }
  for (int k = 0; k < 2; ++k) {
    CHECK(hipEventRecord(e0));
    if (k == 0) hipLaunchKernelGGL(valu_kernel, dim3(blocks), dim3(256), 0, 0, iters, sink, 1.f);
    else hipLaunchKernelGGL(trans_kernel, dim3(blocks), dim3(256), 0, 0, iters, sink, 1.f);
    CHECK(hipEventRecord(e1));
    CHECK(hipEventSynchronize(e1));
    const double ms = time_ms(e0, e1);
    const double ops = (double)blocks * 4 * iters * (k == 0 ? 64 : 32);  // wave-instructions
    printf("%s: %.2f cycles per wave-instruction per SIMD (%.1f Gwave-inst/s)\n", k == 0 ? "v_fma chain x4" : "rsq/exp2",
           ms * 1e-3 * ghz * 1e9 / (ops / (cus * 4)), ops / (ms * 1e-3) / 1e9);
  }
  printf("done\n");
  return 0;
}
