// vr_stage.h -- per-wave LDS staging of the emission volume for the march kernels:
// wave reductions, the staged box, the tap-pair range of a chunk, the box copy and the trilinear
// fetch that reads the slot when the 2x2x2 cell lies in it (global memory otherwise, same
// arithmetic).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <type_traits>

#include "vr_device.h"
#include "vr_sampling.h"

namespace vr {

// Wave slot sizes (floats).  The march kernel is built for both and the host picks per frame
// from the camera's texels per pixel (vr_capi.hip): the 8x8-ray footprint grows with it.
#ifndef VR_LDS_CAP
#define VR_LDS_CAP 1664        // 6.5 KiB: 26 KiB per workgroup -> 6 workgroups (24 waves) per CU
#endif
#ifndef VR_LDS_CAP_MARCH
// 8 KiB (2040 floats: 5 workgroups per CU, the register-bound occupancy of the march kernel at 96
// VGPRs, so the larger slot costs no wave) for the 32-bit on-the-fly / emission-only launches --
// round 5, with every full frame heavy-first: metric frame 27.24-27.57 -> 26.18-26.50 ms on two
// boxes (r5aw, r5ax), the P = 2 part 15.62 -> 14.87; lookup-gradient (C3 29.4 -> 30.1) and 64-bit
// (C5 226.1 -> 228.7) launches keep VR_LDS_CAP
#define VR_LDS_CAP_MARCH 2040
#endif
#ifndef VR_LDS_CAP_WIDE
// 10 KiB: 4 workgroups per CU, for footprints above ~1.5 texels/pixel and every K = 4 launch (round 5:
// 2560 instead of 3072 floats -- C2 12.23 -> 10.93-10.97 ms, P = 8 part 4.89-4.93 -> 4.82-4.87, r5t;
// 2304 / 2048 floats: C2 11.18-11.22 / 11.88-11.93 ms, P = 4 part 8.25 / 8.33 vs 8.00, r5u)
#define VR_LDS_CAP_WIDE 2560
#endif
#ifndef VR_STAGE_UNROLL
#define VR_STAGE_UNROLL 4  // loads in flight per lane while staging
#endif
#ifndef VR_STAGE_NT
#define VR_STAGE_NT 0  // 1 (A/B): staging loads with the non-temporal hint (L2 streaming policy)
#endif
#ifndef VR_CHUNK
#define VR_CHUNK 32      // samples per staged chunk (halved while the box does not fit)
#endif
#ifndef VR_ATTEMPTS
#define VR_ATTEMPTS 3    // box attempts per chunk: S = VR_CHUNK, /2, /4, ...
#endif

// Wave-wide min / max without LDS: DPP row rotations reduce each 16-lane row, then the gfx950
// permlane16 / permlane32 swaps combine the rows (each returns both halves of the exchange, whose
// min / max is the xor-16 / xor-32 partner's).  Result made wave-uniform.
template <bool MAX>
__device__ __forceinline__ int wave_reduce(int v) {
  int o = __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false);  // row_ror:8
  v = MAX ? max(v, o) : min(v, o);
  o = __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false);  // row_ror:4
  v = MAX ? max(v, o) : min(v, o);
  o = __builtin_amdgcn_update_dpp(v, v, 0x122, 0xf, 0xf, false);  // row_ror:2
  v = MAX ? max(v, o) : min(v, o);
  o = __builtin_amdgcn_update_dpp(v, v, 0x121, 0xf, 0xf, false);  // row_ror:1
  v = MAX ? max(v, o) : min(v, o);
  const auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = MAX ? max((int)p16[0], (int)p16[1]) : min((int)p16[0], (int)p16[1]);
  const auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = MAX ? max((int)p32[0], (int)p32[1]) : min((int)p32[0], (int)p32[1]);
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int wave_min(int v) { return wave_reduce<false>(v); }
__device__ __forceinline__ int wave_max(int v) { return wave_reduce<true>(v); }

// wave_reduce<false> of two int16 fields packed in one dword, component-wise (v_pk_min_i16): the
// chunk box's six bounds in three reductions (plan_chunk, VR_PACKED_BOUNDS).
typedef short vr_s2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int pk_min(int a, int b) {
  return __builtin_bit_cast(int, __builtin_elementwise_min(__builtin_bit_cast(vr_s2, a), __builtin_bit_cast(vr_s2, b)));
}
__device__ __forceinline__ int wave_min2(int v) {
  v = pk_min(v, __builtin_amdgcn_update_dpp(v, v, 0x128, 0xf, 0xf, false));  // row_ror:8
  v = pk_min(v, __builtin_amdgcn_update_dpp(v, v, 0x124, 0xf, 0xf, false));  // row_ror:4
  v = pk_min(v, __builtin_amdgcn_update_dpp(v, v, 0x122, 0xf, 0xf, false));  // row_ror:2
  v = pk_min(v, __builtin_amdgcn_update_dpp(v, v, 0x121, 0xf, 0xf, false));  // row_ror:1
  const auto p16 = __builtin_amdgcn_permlane16_swap(v, v, false, false);
  v = pk_min((int)p16[0], (int)p16[1]);
  const auto p32 = __builtin_amdgcn_permlane32_swap(v, v, false, false);
  v = pk_min((int)p32[0], (int)p32[1]);
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ int pk2(int lo16, int hi16) { return (lo16 & 0xffff) | (int)((uint32_t)hi16 << 16); }
__device__ __forceinline__ int pk_lo(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int pk_hi(int v) { return v >> 16; }
#ifndef VR_PACKED_BOUNDS
#define VR_PACKED_BOUNDS 1
#endif

#ifndef VR_RELOAD_TEX
#define VR_RELOAD_TEX 0
#endif

#ifndef VR_ODD_PITCH
// LDS row / plane pitches: 0 dense (ex, ex * ey); 1 always odd (measured slower: the larger slots
// overflow more); 2 odd when the padded box still fits the slot, dense otherwise
#define VR_ODD_PITCH 0
#endif

// Staged box: padded-volume index ranges [r0, r0 + e) per axis, stored in the slot with row
// pitch px and plane pitch pxy (odd, so that rows and planes start on rotating banks).
struct Box {
  int rx, ry, rz, ex, ey, ez, px, pxy;
};

// Trilinear interpolation of the staged cell whose (x, y, z) = (0, 0, 0) corner is slot word a.
__device__ __forceinline__ float lds_tri(const float *L, const Box &B, int a, float wx, float wy, float wz) {
  const float c00 = lerp(L[a], L[a + 1], wx);
  const float c10 = lerp(L[a + B.px], L[a + B.px + 1], wx);
  const float c01 = lerp(L[a + B.pxy], L[a + B.pxy + 1], wx);
  const float c11 = lerp(L[a + B.pxy + B.px], L[a + B.pxy + B.px + 1], wx);
  const float c0 = lerp(c00, c10, wy), c1 = lerp(c01, c11, wy);
  return lerp(c0, c1, wz);
}

// The partial sums of one staged trilinear fetch (lds_tri's c00 .. c1), kept by the centre sample
// for the gradient taps that share them (half_grad_lds).
struct Cell {
  float c00, c10, c01, c11, c0, c1;
};
__device__ __forceinline__ float lds_tri_cell(const float *L, const Box &B, int a, float wx, float wy, float wz,
                                              Cell &C) {
  C.c00 = lerp(L[a], L[a + 1], wx);
  C.c10 = lerp(L[a + B.px], L[a + B.px + 1], wx);
  C.c01 = lerp(L[a + B.pxy], L[a + B.pxy + 1], wx);
  C.c11 = lerp(L[a + B.pxy + B.px], L[a + B.pxy + B.px + 1], wx);
  C.c0 = lerp(C.c00, C.c10, wy);
  C.c1 = lerp(C.c01, C.c11, wy);
  return lerp(C.c0, C.c1, wz);
}

// The six half-texel gradient taps of the fast variant (vr_sampling.h half_taps) from the slot, for
// a sample whose centre cell (slot word ac, partial sums C, weights wx wy wz) and tap cells all lie
// in the staged box.  Each tap is the trilinear fetch fetch_at would take -- same voxels, same
// weights, the same lerps in the same order (x, then y, then z) -- but what two taps or a tap and
// the centre compute alike is computed once: the x taps read their three voxels per row (the minus
// and plus cells share the middle one); the y taps' x-interpolated rows are the centre's c00 .. c11
// except one extra row pair; the z taps' xy-interpolated planes are the centre's c0, c1 except one
// extra plane.  20 voxels and 27 lerps instead of 48 voxels and 42 lerps, with no per-tap box
// test.  Returns the unhalved differences (plus - minus) per axis.
__device__ __forceinline__ f3 half_grad_lds(const float *L, const Box &B, int ac, const AxS &sx, const AxS &sy,
                                            const AxS &sz, float wx, float wy, float wz, const Cell &C) {
  f3 g;
  {  // x: cells a - 1 (minus) and a (plus), a = i + hi; three voxels per (y, z) row from a - 1
    const float tx = sx.w + (sx.hi ? -0.5f : 0.5f);
    const int w = ac + (sx.hi ? 0 : -1);
    float m[4], p[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int o = w + ((r & 1) ? B.px : 0) + ((r & 2) ? B.pxy : 0);
      const float x0 = L[o], x1 = L[o + 1], x2 = L[o + 2];
      m[r] = lerp(x0, x1, tx);
      p[r] = lerp(x1, x2, tx);
    }
    const float gm = lerp(lerp(m[0], m[1], wy), lerp(m[2], m[3], wy), wz);
    const float gp = lerp(lerp(p[0], p[1], wy), lerp(p[2], p[3], wy), wz);
    g.x = gp - gm;
  }
  {  // y: rows b - 1, b, b + 1 (b = j + hi) of the x-interpolated values; one row pair is new
    const float ty = sy.w + (sy.hi ? -0.5f : 0.5f);
    const int w = ac + (sy.hi ? 2 * B.px : -B.px);
    const float e0 = lerp(L[w], L[w + 1], wx), e1 = lerp(L[w + B.pxy], L[w + B.pxy + 1], wx);
    const float y00 = sy.hi ? C.c00 : e0, y01 = sy.hi ? C.c10 : C.c00, y02 = sy.hi ? e0 : C.c10;  // z
    const float y10 = sy.hi ? C.c01 : e1, y11 = sy.hi ? C.c11 : C.c01, y12 = sy.hi ? e1 : C.c11;  // z + 1
    const float gm = lerp(lerp(y00, y01, ty), lerp(y10, y11, ty), wz);
    const float gp = lerp(lerp(y01, y02, ty), lerp(y11, y12, ty), wz);
    g.y = gp - gm;
  }
  {  // z: planes c - 1, c, c + 1 (c = k + hi) of the xy-interpolated values; one plane is new
    const float tz = sz.w + (sz.hi ? -0.5f : 0.5f);
    const int w = ac + (sz.hi ? 2 * B.pxy : -B.pxy);
    const float q0 = lerp(L[w], L[w + 1], wx), q1 = lerp(L[w + B.px], L[w + B.px + 1], wx);
    const float pe = lerp(q0, q1, wy);
    const float z0 = sz.hi ? C.c0 : pe, z1 = sz.hi ? C.c1 : C.c0, z2 = sz.hi ? pe : C.c1;
    g.z = lerp(z1, z2, tz) - lerp(z0, z1, tz);
  }
  return g;
}

// Slot coordinates of a tap pair base and whether the cell [l, l+1] lies in the box along it.
__device__ __forceinline__ int slot_coord(int i, int r) { return (int)((uint32_t)i + 1u - (uint32_t)r); }
__device__ __forceinline__ bool in_box(int l, int e) {
  return (VR_ABLATE & 16) || (unsigned)l < (unsigned)(e - 1);
}

// A texture's parameters re-read from the kernel-argument segment at the point of use (scalar loads)
// for the rare global-memory taps: behind the empty asm the compiler cannot hoist the loads out of
// the sample loop, so they do not hold SGPRs across it (the loop's SGPRs spill to VGPR lanes
// otherwise, and every spilled value costs a v_readlane per use).
__device__ __forceinline__ DevTex reload(const DevTex &t) {
#if VR_RELOAD_TEX == 1
  typedef const volatile __attribute__((address_space(4))) DevTex *cptr;
  cptr q = (cptr)&t;
  DevTex u;
  u.p = q->p;
  u.nx = q->nx;
  u.ny = q->ny;
  u.nz = q->nz;
  u.px = q->px;
  u.pxy = q->pxy;
  return u;
#elif VR_RELOAD_TEX == 2
  typedef const __attribute__((address_space(4))) DevTex *cptr;
  cptr q = (cptr)&t;
  asm volatile("" : "+s"(q));
  return *q;
#else
  return t;
#endif
}

// Trilinear fetch of the staged emission texture: the slot when the 2x2x2 cell lies in the box
// (`in`, with slot word `a`), global memory otherwise -- the same interpolation either way.  The
// axes are unclamped (axis_raw); the global path clamps them.
template <bool BIG>
__device__ __forceinline__ float fetch_at(const DevTex &t, const float *L, const Box &B, bool in, int a,
                                          const Ax &ax, const Ax &ay, const Ax &az) {
  if (in) return lds_tri(L, B, a, ax.w, ay.w, az.w);
  const DevTex u = reload(t);
  return fetch<BIG>(u, clamp_ax(ax, u.nx), clamp_ax(ay, u.ny), clamp_ax(az, u.nz));
}

// Padded index range [lo, hi] (inclusive) of the tap pairs of one axis for a coordinate range.
// `off` includes the staging margin (RenderParams::tap_off): it bounds the drift between the
// predicted end position fma(step, k, pos) and the k sequentially rounded pos += step additions.
// `edge`: set when the range is clamped to the apron, i.e. some tap of the range is a clamped tap at a
// volume face, whose voxels a box cannot hold (then only the per-sample slot test is exact).
__device__ __forceinline__ void axis_range(float c0, float c1, float off, int n, int &lo, int &hi, bool &edge) {
  const float cmin = fminf(c0, c1) - off, cmax = fmaxf(c0, c1) + off;
  const int a = (int)floorf(cmin), b = (int)floorf(cmax);
  edge = edge || a < -1 || b > n - 1;
  lo = min(max(a, -1), n - 1) + 1;
  hi = min(max(b, -1), n - 1) + 2;
}

// Element-wise copy of box B into the slot (any box shape and pitch).  Returns whether any
// staged voxel is non-zero (NaN counts as non-zero), for the whole wave.
__device__ __forceinline__ bool stage_box_elems(float *L, const DevTex &t, const Box &B, int lane) {
  bool nz = false;
  const uint32_t ex = (uint32_t)B.ex, ey = (uint32_t)B.ey;
  const uint32_t V = ex * ey * (uint32_t)B.ez;
  uint32_t x = (uint32_t)lane % ex;
  uint32_t r = (uint32_t)lane / ex;
  uint32_t y = r % ey, z = r / ey;
  const uint32_t sx = 64u % ex, sr = 64u / ex;
  for (uint32_t q0 = (uint32_t)lane; q0 < V; q0 += 256u) {
    float v[4];
    uint32_t li[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = q0 + 64u * j;
      li[j] = z * (uint32_t)B.pxy + y * (uint32_t)B.px + x;
      if (q < V) {
        const uint64_t o = ((uint64_t)(B.rz + z) * t.pxy + (uint64_t)(B.ry + y) * t.px) + (uint64_t)(B.rx + x);
        v[j] = t.p[o];
        nz |= (v[j] != 0.f);
      }
      x += sx;
      y += sr;
      if (x >= ex) {
        x -= ex;
        ++y;
      }
      while (y >= ey) {
        y -= ey;
        ++z;
      }
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t q = q0 + 64u * j;
      if (q < V) L[li[j]] = v[j];
    }
  }
  return __any(nz);
}


#ifndef VR_STAGE_GLDS
#define VR_STAGE_GLDS 0  // (A/B) stage dense boxes with LDS-DMA loads (global_load_lds_dword)
#endif

// Copy a densely pitched box B into the slot with LDS-DMA loads: a dense slot is the box's V voxels
// in x-fastest order, so slot words q0 .. q0 + 63 of one wave pass are the lane-linear destination
// of one global_load_lds_dword (LDS address = slot + 4 q0 + 4 lane); no VGPR holds a voxel and no
// ds_write is issued.  The non-zero test reads the slot back (one word per lane per pass).
template <bool BIG>
__device__ __forceinline__ bool stage_box_glds(float *L, const DevTex &t, const Box &B, int lane) {
  const uint32_t ex = (uint32_t)B.ex, ey = (uint32_t)B.ey;
  const uint32_t V = ex * ey * (uint32_t)B.ez;
  uint32_t x = (uint32_t)lane % ex, r = (uint32_t)lane / ex;
  uint32_t y = r % ey;
  const float *src = t.p + ((uint64_t)(B.rz + r / ey) * t.pxy + (uint64_t)(B.ry + y) * t.px + (uint64_t)(B.rx + x));
  const uint32_t sx = 64u % ex, sr = 64u / ex;
  const int64_t g_step = (int64_t)sx + (int64_t)sr * (int64_t)t.px;
  const int64_t g_row = (int64_t)t.px - (int64_t)ex, g_wrap = (int64_t)t.pxy - (int64_t)ey * (int64_t)t.px;
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the previous chunk's slot reads are done
  for (uint32_t q0 = 0; q0 < V; q0 += 64u) {
    if (q0 + (uint32_t)lane < V)
      __builtin_amdgcn_global_load_lds((const void *)src, (__attribute__((address_space(3))) void *)(L + q0), 4, 0, 0);
    x += sx;
    y += sr;
    src += g_step;
    if (x >= ex) {
      x -= ex;
      ++y;
      src += g_row;
    }
    while (y >= ey) {
      y -= ey;
      src += g_wrap;
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the slot is written
  uint32_t acc = 0;
  for (uint32_t q = (uint32_t)lane; q < V; q += 64u) acc |= __float_as_uint(L[q]);
  return __any((acc & 0x7fffffffu) != 0u);
}

// Copy box B of the apron volume into the wave's LDS slot (row-major, x fastest).  A wave pass
// moves 64 / ex whole rows (lane -> (row slot, x)); row offsets advance incrementally, relative to
// a wave-uniform base pointer, so a pass costs a handful of adds instead of per-element 64-bit
// index products.  Returns whether any staged voxel is non-zero (NaN counts as non-zero), for
// the whole wave.
template <bool BIG>
__device__ __forceinline__ bool stage_box(float *L, const DevTex &t, const Box &B, int lane) {
  const int ex = B.ex, ey = B.ey;
  if (VR_STAGE_GLDS && B.px == ex && B.pxy == ex * ey &&
      (BIG || (uint64_t)t.pxy * (uint64_t)B.ez * 4u < 0xFFFFFFFFull))
    return stage_box_glds<BIG>(L, t, B, lane);
  if (ex > 64) return stage_box_elems(L, t, B, lane);
  if (!BIG && (uint64_t)t.pxy * (uint64_t)B.ez * 4u >= 0xFFFFFFFFull)  // 32-bit byte offsets overflow
    return stage_box_elems(L, t, B, lane);
  typedef typename std::conditional<BIG, uint64_t, uint32_t>::type off_t;
  const int per = 64 / ex;  // rows per pass (wave-uniform)
  const int rr = lane / ex, xr = lane - rr * ex;
  const int rows = ey * B.ez;
  const int n = rr < per ? (rows - rr + per - 1) / per : 0;  // passes with a row for this lane
  int y = rr % ey;
  const int z = rr / ey;
  const char *base = reinterpret_cast<const char *>(
      t.p + ((uint64_t)B.rz * t.pxy + (uint64_t)B.ry * t.px + (uint64_t)B.rx));  // uniform
  off_t g = ((off_t)z * t.pxy + (off_t)y * t.px + (off_t)xr) * 4u;               // bytes
  const off_t g_row = (off_t)per * t.px * 4u;
  const off_t g_wrap = ((off_t)t.pxy - (off_t)ey * t.px) * 4u;
  int l = z * B.pxy + y * B.px + xr;  // slot word
  const int l_row = per * B.px;
  const int l_wrap = B.pxy - ey * B.px;  // plane padding (0 for dense pitches)
  uint32_t acc = 0;
  for (int k0 = 0; k0 < n; k0 += VR_STAGE_UNROLL) {
    float v[VR_STAGE_UNROLL];
    int li[VR_STAGE_UNROLL];
#pragma unroll
    for (int j = 0; j < VR_STAGE_UNROLL; ++j) {
      li[j] = l;
      if (k0 + j < n) {
        const float *src = reinterpret_cast<const float *>(base + g);
        v[j] = VR_STAGE_NT ? __builtin_nontemporal_load(src) : *src;
      }
      l += l_row;
      g += g_row;
      y += per;
      while (y >= ey) {
        y -= ey;
        g += g_wrap;
        l += l_wrap;
      }
    }
#pragma unroll
    for (int j = 0; j < VR_STAGE_UNROLL; ++j) {
      if (k0 + j < n) {
        L[li[j]] = v[j];
        acc |= __float_as_uint(v[j]) & 0x7fffffffu;
      }
    }
  }
  return __any(acc != 0u);
}

#ifndef VR_PARTIAL
#define VR_PARTIAL 1     // stage a centred sub-box when no whole box fits (taps outside: global)
#endif

// Chunk set-up: the box of every tap the wave's live rays take in their next S samples, S halved
// (up to VR_ATTEMPTS tries) until the box fits the slot.  When none fits, the last box is shrunk
// about its centre until it does (partial = true): taps outside it read global memory (the
// fetch checks every cell against the box), and the chunk may not be leaped.  The predicted end
// position fma(step, k, pos) is bounded against the k sequentially rounded additions by
// RenderParams::tap_off.
template <int CAP>
__device__ __forceinline__ void plan_chunk(const RenderParams &P, bool alive, const f3 &pos, const f3 &step,
                                           float t, float tfar, int &S, bool &staged, bool &partial, Box &B,
                                           int *vol_out = nullptr, bool *edge_out = nullptr, int s0 = VR_CHUNK) {
  const DevTex &E = P.em;
  const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);
  const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
  const float tstep = P.tstep;
  S = s0;  // the first attempt (VR_CHUNK, or the wave's guess from its last chunk: VR_ADAPTIVE_S)
  staged = false;
  partial = false;
  B = Box{0, 0, 0, 1, 1, 1, 1, 1};
  for (int attempt = 0;; ++attempt) {
    int lo[3] = {0x3fffffff, 0x3fffffff, 0x3fffffff}, hi[3] = {-0x3fffffff, -0x3fffffff, -0x3fffffff};
    bool edge = false;
    if (alive) {
      const float rem = (tfar - t) / tstep;  // samples left before the exit test fires
      const int s_eff = (rem < (float)S) ? max((int)rem + 2, 1) : S;
      const float k = (float)(s_eff - 1);
      const f3 pe = mk(fmaf(step.x, k, pos.x), fmaf(step.y, k, pos.y), fmaf(step.z, k, pos.z));
      axis_range(((pos.x - bmin.x) * bsc.x) * E.fnx - 0.5f, ((pe.x - bmin.x) * bsc.x) * E.fnx - 0.5f,
                 P.tap_off[0], E.nx, lo[0], hi[0], edge);
      axis_range(((pos.y - bmin.y) * bsc.y) * E.fny - 0.5f, ((pe.y - bmin.y) * bsc.y) * E.fny - 0.5f,
                 P.tap_off[1], E.ny, lo[1], hi[1], edge);
      axis_range(((pos.z - bmin.z) * bsc.z) * E.fnz - 0.5f, ((pe.z - bmin.z) * bsc.z) * E.fnz - 0.5f,
                 P.tap_off[2], E.nz, lo[2], hi[2], edge);
    }
    if (VR_PACKED_BOUNDS && E.nx < 16000 && E.ny < 16000 && E.nz < 16000) {
      // padded bounds lie in [0, n + 1] (and the dead-lane sentinels are clamped to +-16383), so
      // they fit int16 fields: lo x/y, lo z / -hi x, -hi y / -hi z, each pair in one reduction
      const int c = 16383;
      const int a = wave_min2(pk2(min(lo[0], c), min(lo[1], c)));
      const int b = wave_min2(pk2(min(lo[2], c), min(-hi[0], c)));
      const int d = wave_min2(pk2(min(-hi[1], c), min(-hi[2], c)));
      B.rx = pk_lo(a);
      B.ry = pk_hi(a);
      B.rz = pk_lo(b);
      B.ex = -pk_hi(b) - B.rx + 1;
      B.ey = -pk_lo(d) - B.ry + 1;
      B.ez = -pk_hi(d) - B.rz + 1;
    } else {
      B.rx = wave_min(lo[0]);
      B.ry = wave_min(lo[1]);
      B.rz = wave_min(lo[2]);
      B.ex = wave_max(hi[0]) - B.rx + 1;
      B.ey = wave_max(hi[1]) - B.ry + 1;
      B.ez = wave_max(hi[2]) - B.rz + 1;
    }
    B.px = VR_ODD_PITCH == 1 ? (B.ex | 1) : B.ex;
    B.pxy = VR_ODD_PITCH == 1 ? ((B.px * B.ey) | 1) : B.px * B.ey;
    if (vol_out) *vol_out = B.pxy * B.ez;
    if (B.ex <= 0 || B.ey <= 0 || B.ez <= 0) return;  // no live ray
    if (B.pxy * B.ez <= CAP) {
      if (VR_ODD_PITCH == 2) {  // rows and planes on rotating banks, if the slot has room
        const int px = B.ex | 1, pxy = (px * B.ey) | 1;
        if (pxy * B.ez <= CAP) {
          B.px = px;
          B.pxy = pxy;
        }
      }
      staged = true;
      if (edge_out) *edge_out = __any(edge);
      return;
    }
    if (S <= (VR_CHUNK >> (VR_ATTEMPTS - 1))) break;  // the shortest chunk did not fit either
    S >>= 1;
  }
#if VR_PARTIAL
  // shrink the largest extent about the centre until the sub-box fits (wave-uniform scalars)
  int e[3] = {B.ex, B.ey, B.ez}, r[3] = {B.rx, B.ry, B.rz};
  while (e[0] * e[1] * e[2] > CAP) {
    const int a = (e[0] >= e[1] && e[0] >= e[2]) ? 0 : (e[1] >= e[2] ? 1 : 2);
    if (e[a] <= 2) break;
    r[a] += e[a] & 1;  // trim alternately from the low and the high side
    --e[a];
  }
  B.rx = r[0]; B.ry = r[1]; B.rz = r[2];
  B.ex = e[0]; B.ey = e[1]; B.ez = e[2];
  B.px = B.ex;
  B.pxy = B.ex * B.ey;
  if (B.pxy * B.ez <= CAP) {
    staged = true;
    partial = true;
    return;
  }
#endif
  S >>= 1;  // no box fits: march S/2 samples from global memory
}

// The launch's RenderParams in the kernel-argument segment (march_kernel: the first argument, at
// offset 0; march_views_kernel: view v's entry), for parameters read at their point of use with
// scalar loads the compiler cannot hoist (the empty-space probe's: read once per probe, not held in
// SGPRs across the sample loop).  Formed from __builtin_amdgcn_kernarg_segment_ptr, never from the
// address of the by-value parameter (which may be a private copy).
typedef const __attribute__((address_space(4))) RenderParams *KParams;
__device__ __forceinline__ KParams kparams_fresh(KParams kp) {
  asm volatile("" : "+s"(kp));
  return kp;
}

// Empty-space probe (round 5): whether every centre tap of the live rays' next L
// samples lies in bricks of the emission texture's occupancy map (RenderParams::occ) that hold only
// +-0 -- then each of those samples has em = ab = 0 and opacity exactly 0, adds exactly nothing
// (skip_empty), and the rays may leap the L samples replaying only the recurrences, as the
// empty-chunk leap does after staging an all-zero box.  Here no box is staged: one byte per brick
// of the box's bricks is read (one load per lane, two for up to 128 bricks), so a run through
// empty space costs a box reduction and one round trip per L samples instead of a staging copy per
// chunk.  The box is the centre cells' range with RenderParams::probe_off as the margin (the
// gradient taps do not matter: an opacity-0 sample is never shaded).  Returns 1: empty (leap),
// 0: a brick is occupied, -1: the box spans more than 128 bricks (undecided).  Wave-uniform.
__device__ __forceinline__ int probe_run(const RenderParams &P, KParams kp0, bool alive, const f3 &pos,
                                         const f3 &step, float t, float tfar, int L, int lane) {
  const KParams kp = kparams_fresh(kp0);
  const DevTex &E = P.em;
  const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);
  const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
  int lo[3] = {0x3fffffff, 0x3fffffff, 0x3fffffff}, hi[3] = {-0x3fffffff, -0x3fffffff, -0x3fffffff};
  bool edge = false;
  if (alive) {
    const float rem = (tfar - t) / P.tstep;  // samples left before the exit test fires
    const int s_eff = (rem < (float)L) ? max((int)rem + 2, 1) : L;
    const float k = (float)(s_eff - 1);
    const f3 pe = mk(fmaf(step.x, k, pos.x), fmaf(step.y, k, pos.y), fmaf(step.z, k, pos.z));
    axis_range(((pos.x - bmin.x) * bsc.x) * E.fnx - 0.5f, ((pe.x - bmin.x) * bsc.x) * E.fnx - 0.5f,
               kp->probe_off[0], E.nx, lo[0], hi[0], edge);
    axis_range(((pos.y - bmin.y) * bsc.y) * E.fny - 0.5f, ((pe.y - bmin.y) * bsc.y) * E.fny - 0.5f,
               kp->probe_off[1], E.ny, lo[1], hi[1], edge);
    axis_range(((pos.z - bmin.z) * bsc.z) * E.fnz - 0.5f, ((pe.z - bmin.z) * bsc.z) * E.fnz - 0.5f,
               kp->probe_off[2], E.nz, lo[2], hi[2], edge);
  }
  // brick ranges of the box (padded coordinates >> VR_OCC_LOG): lo in the low, -hi in the high int16 field
  const int c = 16383;
  const int a = wave_min2(pk2(min(lo[0] >> VR_OCC_LOG, c), min(lo[1] >> VR_OCC_LOG, c)));
  const int b = wave_min2(pk2(min(lo[2] >> VR_OCC_LOG, c), min(-(hi[0] >> VR_OCC_LOG), c)));
  const int d = wave_min2(pk2(min(-(hi[1] >> VR_OCC_LOG), c), min(-(hi[2] >> VR_OCC_LOG), c)));
  const int bx = pk_lo(a), by = pk_hi(a), bz = pk_lo(b);
  const int cx = -pk_hi(b) - bx + 1, cy = -pk_lo(d) - by + 1, cz = -pk_hi(d) - bz + 1;
  if (cx <= 0 || cy <= 0 || cz <= 0) return 1;  // no live ray
  const int cnt = cx * cy * cz;
  if (cnt > 128) return -1;
  // lane q -> brick q and q + 64 of the box (x fastest); the divisions by the uniform extents in fp32
  // (q < 128 and extents <= 128: exact quotients after the truncation)
  const float rcx = 1.f / (float)cx, rcy = 1.f / (float)cy;
  const uint8_t *occ = kp->occ;
  const uint32_t obx = kp->occ_bx, obxy = kp->occ_bxy;
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int q = lane + 64 * j;
    if (q < cnt) {
      const int qz = (int)(((float)q + 0.5f) * (rcx * rcy));
      const int r = q - qz * cx * cy;
      const int qy = (int)(((float)r + 0.5f) * rcx);
      const int qx = r - qy * cx;
      v |= occ[(uint32_t)(bz + qz) * obxy + (uint32_t)(by + qy) * obx + (uint32_t)(bx + qx)];
    }
  }
  return __any(v != 0u) ? 0 : 1;
}

// Per-lane empty-space probe (round 6): whether every centre tap of each live lane's own next L
// samples lies in +-0 bricks -- the test for waves whose rays are too far apart for one box
// (probe_run's -1).  Rays that graze a volume face enter it at very different depths (a column of
// pixels whose rays run almost parallel to the face: rotate(30,10,0) at 1920x1080, the 8 columns
// next to the silhouette), so a wave's live rays spread along the face, its probe box spans
// hundreds of bricks and its chunk boxes stage only partially: before round 6 such a block marched
// its ~7000 empty samples per ray with global gathers, up to 55 ms.  Here each lane walks its own
// run in segments of at most VR_LANE_SEG texels per axis; a segment's box (its end points' cells
// widened by probe_off, as probe_run's box) spans at most 2 bricks per axis, whose bytes are ORed.
// Consecutive segments share their end points bit for bit (both from the same expression), so the
// segments cover the run's box end to end.  Returns 1 (all empty: leap) or 0.  Wave-uniform.
#ifndef VR_LANE_SEG
#define VR_LANE_SEG 4.0f
#endif
// The walk of one lane (no wave operations inside, every launch constant an argument).  Inlined it
// weighs on the sample loop of every launch although it rarely runs (round 6, same box: metric frame
// 25.34-25.40 vs 24.89-25.00 ms without the lane probe, C3 28.8-28.9 vs 27.5-27.7); out of line
// (VR_PROBE_LANES_CALL=1) the call's register saves spill more (metric kernel 5 VGPRs), so inline.
#ifndef VR_PROBE_LANES_CALL
#define VR_PROBE_LANES_CALL 0
#endif
#if VR_PROBE_LANES_CALL
#define VR_LANES_ATTR __attribute__((noinline))
#else
#define VR_LANES_ATTR __forceinline__
#endif
__device__ VR_LANES_ATTR uint32_t probe_lane_walk(const uint8_t *occ, uint32_t obx, uint32_t obxy, float a0x, float a0y,
                                                  float a0z, float a1x, float a1y, float a1z, float ox, float oy,
                                                  float oz, int nx, int ny, int nz) {
  const float a0[3] = {a0x, a0y, a0z}, a1[3] = {a1x, a1y, a1z}, off[3] = {ox, oy, oz};
  const int n[3] = {nx, ny, nz};
  const float span = fmaxf(fabsf(a1x - a0x), fmaxf(fabsf(a1y - a0y), fabsf(a1z - a0z)));
  const int nseg = max(1, (int)ceilf(span * (1.f / VR_LANE_SEG)));
  const float inv = 1.f / (float)nseg;
  uint32_t v = 0;
  for (int j = 0; j < nseg && v == 0u; ++j) {
    // segment j: from fraction j / nseg to (j + 1) / nseg of the run, per axis
    int blo[3], bhi[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
      const float s = a1[d] - a0[d];
      const float c0 = j == 0 ? a0[d] : fmaf(s, (float)j * inv, a0[d]);
      const float c1 = j + 1 == nseg ? a1[d] : fmaf(s, (float)(j + 1) * inv, a0[d]);
      int lo, hi;
      bool edge = false;
      axis_range(c0, c1, off[d], n[d], lo, hi, edge);
      blo[d] = lo >> VR_OCC_LOG;
      bhi[d] = hi >> VR_OCC_LOG;
    }
    for (int bz = blo[2]; bz <= bhi[2]; ++bz)
      for (int by = blo[1]; by <= bhi[1]; ++by)
        for (int bx = blo[0]; bx <= bhi[0]; ++bx) v |= occ[(uint32_t)bz * obxy + (uint32_t)by * obx + (uint32_t)bx];
  }
  return v;
}
__device__ __forceinline__ int probe_lanes(const RenderParams &P, KParams kp0, bool alive, const f3 &pos,
                                           const f3 &step, float t, float tfar, int L) {
  // (every launch constant read through the argument segment at its point of use: the probe is rare,
  // and values held for it across the sample loop would cost the loop registers)
  const KParams kp = kparams_fresh(kp0);
  uint32_t v = 0;
  if (alive) {
    const float rem = (tfar - t) / kp->tstep;  // as probe_run
    const int s_eff = (rem < (float)L) ? max((int)rem + 2, 1) : L;
    const float k = (float)(s_eff - 1);
    const f3 pe = mk(fmaf(step.x, k, pos.x), fmaf(step.y, k, pos.y), fmaf(step.z, k, pos.z));
    v = probe_lane_walk(kp->occ, kp->occ_bx, kp->occ_bxy,
                        ((pos.x - kp->bmin[0]) * kp->bscale[0]) * kp->em.fnx - 0.5f,
                        ((pos.y - kp->bmin[1]) * kp->bscale[1]) * kp->em.fny - 0.5f,
                        ((pos.z - kp->bmin[2]) * kp->bscale[2]) * kp->em.fnz - 0.5f,
                        ((pe.x - kp->bmin[0]) * kp->bscale[0]) * kp->em.fnx - 0.5f,
                        ((pe.y - kp->bmin[1]) * kp->bscale[1]) * kp->em.fny - 0.5f,
                        ((pe.z - kp->bmin[2]) * kp->bscale[2]) * kp->em.fnz - 0.5f, kp->probe_off[0],
                        kp->probe_off[1], kp->probe_off[2], kp->em.nx, kp->em.ny, kp->em.nz);
  }
  return __any(v != 0u) ? 0 : 1;
}

// The empty-chunk leap: every tap of the chunk lies in the staged all-zero box, so each sample has
// em = ab = 0, alpha = 1 - exp(-0) = 0 and adds exactly 0 (skip_empty proves the shading term
// finite).  Only the march recurrences run, in the reference's order.
// cap (all four): the sample-count cap, P.max_steps unless given (a chord split's front half, A,
// stops at its split index: vr_march.hip SPLIT)
__device__ __forceinline__ void leap(const RenderParams &P, int S, bool &alive, int32_t &nsteps, float &t,
                                     float tfar, f3 &pos, const f3 &step, int cap = -1) {
  const int mx = cap < 0 ? P.max_steps : cap;
  for (int k = 0; k < S && alive; ++k) {
    ++nsteps;
    if (nsteps >= mx) {
      alive = false;
    } else {
      t += P.tstep;
      if (t > tfar) alive = false;
      else pos = mk(pos.x + step.x, pos.y + step.y, pos.z + step.z);
    }
  }
}

// The same recurrence as leap() for a wave-uniform count, without branches: a lane whose sample
// stopped existing keeps advancing, but its state is never read again (`alive` stays false), so
// the live lanes see exactly leap()'s additions.
__device__ __forceinline__ void advance(const RenderParams &P, int n, bool &alive, int32_t &nsteps, float &t,
                                        float tfar, f3 &pos, const f3 &step, int cap = -1) {
  const int mx = cap < 0 ? P.max_steps : cap;
  for (int k = 0; k < n; ++k) {
    ++nsteps;
    t += P.tstep;
    pos = mk(pos.x + step.x, pos.y + step.y, pos.z + step.z);
    alive = alive && nsteps < mx && !(t > tfar);
  }
}

// advance() for a tame launch (tstep > 0, finite): the additions of n samples, then one exit test
// (t only grows and nsteps only counts up, so the intermediate tests are implied by the last).
__device__ __forceinline__ void advance_n(const RenderParams &P, int n, bool &alive, int32_t &nsteps, float &t,
                                          float tfar, f3 &pos, const f3 &step, int cap = -1) {
  for (int k = 0; k < n; ++k) {
    t += P.tstep;
    pos = mk(pos.x + step.x, pos.y + step.y, pos.z + step.z);
  }
  nsteps += n;
  alive = alive && nsteps < (cap < 0 ? P.max_steps : cap) && !(t > tfar);
}

// advance() by a compile-time count for a tame launch (tstep > 0, finite): t only grows and nsteps
// only counts up, so the exit tests of the intermediate samples are implied by the last one's --
// the same `alive`, with the same rounded additions, and one test instead of n.
template <int N>
__device__ __forceinline__ void advance_k(const RenderParams &P, bool &alive, int32_t &nsteps, float &t, float tfar,
                                          f3 &pos, const f3 &step, int cap = -1) {
#pragma unroll
  for (int k = 0; k < N; ++k) {
    t += P.tstep;
    pos = mk(pos.x + step.x, pos.y + step.y, pos.z + step.z);
  }
  nsteps += N;
  alive = alive && nsteps < (cap < 0 ? P.max_steps : cap) && !(t > tfar);
}

}  // namespace vr
