// valu_rates.hip -- issue throughput of the VALU instruction classes the ray-march uses
// (cycles per wave-instruction per SIMD, 16 independent chains per lane, 8 waves per SIMD).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

#define KERNEL(NAME, ASM)                                                                    \
  __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t c, int iters) {        \
    uint32_t v[16];                                                                          \
    for (int i = 0; i < 16; ++i) v[i] = threadIdx.x * 16 + i;                                \
    uint64_t w[16];                                                                          \
    for (int i = 0; i < 16; ++i) w[i] = v[i];                                                \
    (void)w;                                                                                 \
    for (int it = 0; it < iters; ++it) {                                                     \
      _Pragma("unroll") for (int i = 0; i < 16; ++i) { ASM; }                                \
    }                                                                                        \
    uint32_t s = 0;                                                                          \
    for (int i = 0; i < 16; ++i) s += v[i] + (uint32_t)w[i];                                 \
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;                                          \
  }

KERNEL(k_fma, asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_fmac, asm volatile("v_fmac_f32 %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_mul, asm volatile("v_mul_f32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_addf, asm volatile("v_add_f32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_subf, asm volatile("v_sub_f32 %0, %1, %0" : "+v"(v[i]) : "v"(c)))
KERNEL(k_maxf, asm volatile("v_max_f32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_med3f, asm volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_pkfma, asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(w[i]) : "v"((uint64_t)c)))
KERNEL(k_pkmul, asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(w[i]) : "v"((uint64_t)c)))
KERNEL(k_pkadd, asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(w[i]) : "v"((uint64_t)c)))
KERNEL(k_addu, asm volatile("v_add_u32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_add3u, asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_and, asm volatile("v_and_b32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_mini, asm volatile("v_min_i32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_med3i, asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_mad24, asm volatile("v_mad_u32_u24 %0, %0, %1, %2" : "+v"(v[i]) : "v"(c), "v"(v[(i + 1) & 15])))
KERNEL(k_cvt, asm volatile("v_cvt_i32_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_cvtf, asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(v[i])))
KERNEL(k_floor, asm volatile("v_floor_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_fract, asm volatile("v_fract_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_rndne, asm volatile("v_rndne_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_cnd, asm volatile("v_cmp_gt_f32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc" : "+v"(v[i]) : "v"(c) : "vcc"))
KERNEL(k_cmp, asm volatile("v_cmp_gt_f32 vcc, %0, %1" : : "v"(v[i]), "v"(c) : "vcc"))
KERNEL(k_mullo, asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(v[i]) : "v"(c)))
KERNEL(k_lshl64, asm volatile("v_lshl_add_u64 %0, %0, 2, %0" : "+v"(w[i])))
KERNEL(k_sqrt, asm volatile("v_sqrt_f32 %0, %0" : "+v"(v[i])))
KERNEL(k_mov, asm volatile("v_mov_b32 %0, %1" : "=v"(v[i]) : "v"(v[(i + 1) & 15])))
KERNEL(k_readlane, asm volatile("v_readlane_b32 s2, %0, 3" : : "v"(v[i]) : "s2"))

typedef void (*kfn)(uint32_t *, uint32_t, int);
int main() {
  uint32_t *o;
  hipMalloc(&o, 256u * 2048 * 16 * 4);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct { const char *n; kfn f; } ks[] = {
      {"v_fma_f32", k_fma}, {"v_fmac_f32", k_fmac}, {"v_mul_f32", k_mul}, {"v_add_f32", k_addf}, {"v_sub_f32", k_subf}, {"v_max_f32", k_maxf}, {"v_med3_f32", k_med3f}, {"v_pk_fma_f32", k_pkfma}, {"v_pk_mul_f32", k_pkmul}, {"v_pk_add_f32", k_pkadd}, {"v_add_u32", k_addu}, {"v_add3_u32", k_add3u}, {"v_and_b32", k_and}, {"v_min_i32", k_mini}, {"v_med3_i32", k_med3i}, {"v_mad_u32_u24", k_mad24}, {"v_cvt_i32_f32", k_cvt}, {"v_cvt_f32_i32", k_cvtf}, {"v_floor_f32", k_floor}, {"v_fract_f32", k_fract}, {"v_rndne_f32", k_rndne}, {"v_cmp+v_cndmask", k_cnd}, {"v_cmp_gt_f32", k_cmp}, {"v_mul_lo_u32", k_mullo}, {"v_lshl_add_u64", k_lshl64}, {"v_sqrt_f32", k_sqrt}, {"v_mov_b32", k_mov}, {"v_readlane_b32", k_readlane}};
  int dev;
  hipGetDevice(&dev);
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, dev);
  const int cus = p.multiProcessorCount, iters = 4000, blocks = cus * 8;  // 8 waves per SIMD
  printf("CUs %d, clock %d kHz (cycles/wave-instr use this clock)\n", cus, p.clockRate);
  for (auto &k : ks) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEventRecord(e0);
      k.f<<<blocks, 256>>>(o, 0x3f7ff000u, iters);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      if (rep) {
        const double winstr = (double)blocks * 4 * iters * 16 / (cus * 4.0);  // per SIMD
        const double cyc = ms * 1e-3 * p.clockRate * 1e3;
        printf("%-16s %.2f cycles/wave-instr/SIMD (%.3f ms)\n", k.n, cyc / winstr, ms);
      }
    }
  }
  return 0;
}
