// vr_sampling.h -- device helpers shared by the gfx950 kernels: vector ops with the oracle's fma
// contraction, the CUDA linear-filter address computation (normalized coords, clamp) and the
// trilinear fetch from the apron layout of vr_device.h.  See DESIGN.md s4 for the arithmetic.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "vr_device.h"

namespace vr {

#define VR_PI ((float)3.14159265358979323846f)  // volumeRender_kernel.cu:20

struct f3 {
  float x, y, z;
};
__device__ __forceinline__ f3 mk(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)); }

typedef float f2a4 __attribute__((ext_vector_type(2), aligned(4)));
typedef float f4a8 __attribute__((ext_vector_type(4), aligned(8)));

// One axis of the linear-filter address computation (normalized coords, clamp addressing):
// pair base i' = clamp(floor(c*n - 0.5), -1, n-1) and the 8-bit weight.  The clamp runs on the
// float floor before the conversion (one v_med3 instead of v_max + v_min: the same integer for
// every floor value, +-inf included).  NANCHK = false skips the NaN -> 0 substitution where the
// caller has proven the coordinate finite.
struct Ax {
  int i;
  float w;
};
// The 8-bit filter weight rint(frac(xb) * 256) / 256 of a coordinate xb with floor fl, as
// rint(256 xb) / 256 - fl in one fma: 256 xb is exact, 256 fl an even integer (so the rounding,
// ties to even included, commutes with it), and the result a multiple of 1/256 in [0, 1] --
// bit-identical, NaN / inf alike, one VALU less than the sub, mul, rint, mul sequence.
__device__ __forceinline__ float weight8(float xb, float fl) {
  return fmaf(rintf(xb * 256.f), 1.f / 256.f, -fl);
}
template <bool NANCHK = true>
__device__ __forceinline__ Ax axis(float c, int n, float fn) {
  if (NANCHK) c = (c != c) ? 0.f : c;  // NaN coordinate -> 0
  const float xb = c * fn - 0.5f;
  const float fl = floorf(xb);
  const float w = weight8(xb, fl);
  (void)n;
  return Ax{(int)__builtin_amdgcn_fmed3f(fl, -1.f, fn - 1.f), w};
}

// The pair base without the clamp, and the weight.  Wherever the cell [i, i+1] lies inside a
// staged box the clamp is the identity (box coordinates are clamped indices: an index below -1 or
// above n-1 cannot fall in the box), so the LDS path uses this and the global path clamps.
template <bool NANCHK = true>
__device__ __forceinline__ Ax axis_raw(float c, float fn) {
  if (NANCHK) c = (c != c) ? 0.f : c;  // NaN coordinate -> 0
  const float xb = c * fn - 0.5f;
  const float fl = floorf(xb);
  const float w = weight8(xb, fl);
  return Ax{(int)fl, w};
}
__device__ __forceinline__ Ax clamp_ax(const Ax &a, int n) { return Ax{min(max(a.i, -1), n - 1), a.w}; }

// axis_raw plus the half-texel split of the raw fraction (frac(xb) >= 0.5), for the fast
// gradient taps of a half-texel tap offset (half_taps below).
struct AxS {
  int i;
  float w;
  bool hi;
};
template <bool NANCHK = true>
__device__ __forceinline__ AxS axis_raw_s(float c, float fn) {
  if (NANCHK) c = (c != c) ? 0.f : c;  // NaN coordinate -> 0 (every tap of it is then the centre's
                                       // clamped edge voxel: g = 0, as the reference's NaN taps)
  const float xb = c * fn - 0.5f;
  const float fl = floorf(xb);
  const float r = xb - fl;
  const float w = rintf(r * 256.f) * (1.f / 256.f);
  return AxS{(int)fl, w, r >= 0.5f};
}
// axis_raw_s of a power-of-two cube (box [-1, 1]: bmin = -1, bscale = 1/2; n = 2 hs a power of
// two -- the half-texel tap launch, vr_capi.hip half_texel_taps): the sampler's coordinate
// ((p - bmin) * bscale) * n - 1/2 is fma(p + 1, hs, -1/2) bit for bit -- p - (-1) is p + 1, and
// the products by 1/2 and n (hs) are exact power-of-two scalings, so the fma's single rounding is
// that of the final subtraction.  A NaN coordinate (p + 1 NaN) is taken as c = 0, i.e. p + 1 = 0.
template <bool NANCHK = true>
__device__ __forceinline__ AxS axis_cube_s(float p, float hs) {
  float a = p + 1.f;
  if (NANCHK) a = (a != a) ? 0.f : a;
  const float xb = fmaf(a, hs, -0.5f);
  const float fl = floorf(xb);
  const float r = xb - fl;
  const float w = rintf(r * 256.f) * (1.f / 256.f);
  return AxS{(int)fl, w, r >= 0.5f};
}

// The two taps xb +- 1/2 of an axis derived from the centre's (fast shading variant, DESIGN.md
// s4): with xb' = xb + 1/2 computed exactly, floor(xb') = i + hi and the quantized weight of
// frac(xb') is w + 1/2 - hi (rint((r + 1/2 - hi) * 256) = rint(r * 256) + 128 - 256 hi: adding an
// even integer keeps round-half-even); xb - 1/2 has the same weight on the cell one lower.  The
// reference forms each tap coordinate from pos +- gstep in fp32, which can differ from xb +- 1/2
// in its last bits; the difference reaches an 8-bit weight or a cell only at rounding boundaries.
__device__ __forceinline__ void half_taps(const AxS &a, Ax &plus, Ax &minus) {
  const int ip = a.i + (a.hi ? 1 : 0);
  const float wt = a.w + (a.hi ? -0.5f : 0.5f);
  plus = Ax{ip, wt};
  minus = Ax{ip - 1, wt};
}

// Correctly rounded sqrtf for x >= 0, NaN or +inf.  The device library's sqrtf scales inputs
// below 2^-96 and patches +-0 / inf by class; for x == 0 or x >= 2^-96 its remaining steps (the
// hardware root corrected by one ulp either way from two fma residuals) give the identical result
// on their own, so when every lane of the wave is in that range the scaling is skipped.
__device__ __forceinline__ float sqrt_cr(float x) {
  const uint32_t u = __float_as_uint(x);
  if (__builtin_expect(__all(u - 1u >= 0x0f7fffffu), 1)) {  // x == 0, x >= 2^-96 (or x < 0, NaN)
    const float s = __builtin_amdgcn_sqrtf(x);
    const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
    const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
    const float r = (rm <= 0.f) ? sm : s;
    return (rp > 0.f) ? sp : r;
  }
  return sqrtf(x);
}

// sqrt_cr over a group of values with one wave-wide guard (fewer, larger basic blocks for the
// scheduler): the fast path when every lane's every value qualifies, else the library sqrtf.
__device__ __forceinline__ float sqrt_fast(float x) {
  const float s = __builtin_amdgcn_sqrtf(x);
  const float sm = __uint_as_float(__float_as_uint(s) - 1u), sp = __uint_as_float(__float_as_uint(s) + 1u);
  const float rm = fmaf(-sm, s, x), rp = fmaf(-sp, s, x);
  const float r = (rm <= 0.f) ? sm : s;
  return (rp > 0.f) ? sp : r;
}
template <int N>
__device__ __forceinline__ void sqrt_cr_n(const float (&x)[N], float (&out)[N]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < N; ++i) ok = ok && (__float_as_uint(x[i]) - 1u >= 0x0f7fffffu);
  if (__builtin_expect(__all(ok), 1)) {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = sqrt_fast(x[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) out[i] = sqrtf(x[i]);
  }
}

__device__ __forceinline__ float lerp(float a, float b, float w) { return fmaf(w, b - a, a); }

// Trilinear fetch from the apron layout given the three axes.
template <bool BIG>
__device__ __forceinline__ float fetch(const DevTex &t, const Ax &ax, const Ax &ay, const Ax &az) {
  const float *b;
  if (BIG) {
    const uint64_t o = ((uint64_t)(az.i + 1) * t.pxy + (uint64_t)(ay.i + 1) * t.px) + (uint64_t)(ax.i + 1);
    b = t.p + o;
  } else {
    const uint32_t o = ((uint32_t)(az.i + 1) * t.pxy + (uint32_t)(ay.i + 1) * t.px) + (uint32_t)(ax.i + 1);
    b = t.p + o;
  }
  const f2a4 r00 = *reinterpret_cast<const f2a4 *>(b);
  const f2a4 r10 = *reinterpret_cast<const f2a4 *>(b + t.px);
  const f2a4 r01 = *reinterpret_cast<const f2a4 *>(b + t.pxy);
  const f2a4 r11 = *reinterpret_cast<const f2a4 *>(b + t.pxy + t.px);
  const float c00 = lerp(r00.x, r00.y, ax.w), c10 = lerp(r10.x, r10.y, ax.w);
  const float c01 = lerp(r01.x, r01.y, ax.w), c11 = lerp(r11.x, r11.y, ax.w);
  const float c0 = lerp(c00, c10, ay.w), c1 = lerp(c01, c11, ay.w);
  return lerp(c0, c1, az.w);
}

// Axis of a texture whose offsets are formed in fp32 (fetch_small): the floor kept as a float
// (the value axis() would convert) and the weight.
struct AxF {
  float fl;
  float w;
};

// axis_f for a LUT coordinate, an angle / pi: in [0, 1] or NaN (acosf / acospi of a quotient
// that is NaN or rounds past +-1).  One v_med3 does the NaN -> 0 substitution (the median of NaN,
// 0 and 1 is min3 = 0 under the hardware's NaN rule) and keeps c in [0, 1], where the floor of
// c*n - 0.5 is already in [-1, n-1]: the same axis as axis_f, without its compare, select and clamp.
template <bool FMA = false>
__device__ __forceinline__ AxF axis_lut(float c, float fn) {
  c = __builtin_amdgcn_fmed3f(c, 0.f, 1.f);
  const float xb = FMA ? fmaf(c, fn, -0.5f) : c * fn - 0.5f;  // FMA: the fast variant's shading
  const float fl = floorf(xb);
  return AxF{fl, weight8(xb, fl)};
}

// Trilinear fetch from a texture of fewer than 2^22 padded voxels (the illumination LUT): the
// byte offset 4*((i'z+1)*pxy + (i'y+1)*px + (i'x+1)) is an integer below 2^24, so it is formed
// exactly with three fmas on the float floors and converted once; the four row loads then use
// the wave-uniform base with 32-bit offsets.  Same interpolation as fetch().
__device__ __forceinline__ float fetch_small(const DevTex &t, const AxF &ax, const AxF &ay, const AxF &az) {
  const uint32_t o = (uint32_t)fmaf(az.fl, t.fpxy4, fmaf(ay.fl, t.fpx4, fmaf(ax.fl, 4.f, t.fbase4)));
  const uint32_t px4 = t.px * 4u, pxy4 = t.pxy * 4u;
  const char *b = reinterpret_cast<const char *>(t.p);
  const f2a4 r00 = *reinterpret_cast<const f2a4 *>(b + o);
  const f2a4 r10 = *reinterpret_cast<const f2a4 *>(b + (o + px4));
  const f2a4 r01 = *reinterpret_cast<const f2a4 *>(b + (o + pxy4));
  const f2a4 r11 = *reinterpret_cast<const f2a4 *>(b + (o + pxy4 + px4));
  const float c00 = lerp(r00.x, r00.y, ax.w), c10 = lerp(r10.x, r10.y, ax.w);
  const float c01 = lerp(r01.x, r01.y, ax.w), c11 = lerp(r11.x, r11.y, ax.w);
  const float c0 = lerp(c00, c10, ay.w), c1 = lerp(c01, c11, ay.w);
  return lerp(c0, c1, az.w);
}
// Two fetch_small lookups sharing the x axis, all eight row loads issued before the first lerp.
__device__ __forceinline__ void fetch_small2(const DevTex &t, const AxF &ax, const AxF &ay0, const AxF &az0,
                                             const AxF &ay1, const AxF &az1, float &v0, float &v1) {
  const float ox = fmaf(ax.fl, 4.f, t.fbase4);
  const uint32_t o0 = (uint32_t)fmaf(az0.fl, t.fpxy4, fmaf(ay0.fl, t.fpx4, ox));
  const uint32_t o1 = (uint32_t)fmaf(az1.fl, t.fpxy4, fmaf(ay1.fl, t.fpx4, ox));
  const uint32_t px4 = t.px * 4u, pxy4 = t.pxy * 4u;
  const char *b = reinterpret_cast<const char *>(t.p);
  const f2a4 a00 = *reinterpret_cast<const f2a4 *>(b + o0);
  const f2a4 a10 = *reinterpret_cast<const f2a4 *>(b + (o0 + px4));
  const f2a4 a01 = *reinterpret_cast<const f2a4 *>(b + (o0 + pxy4));
  const f2a4 a11 = *reinterpret_cast<const f2a4 *>(b + (o0 + pxy4 + px4));
  const f2a4 b00 = *reinterpret_cast<const f2a4 *>(b + o1);
  const f2a4 b10 = *reinterpret_cast<const f2a4 *>(b + (o1 + px4));
  const f2a4 b01 = *reinterpret_cast<const f2a4 *>(b + (o1 + pxy4));
  const f2a4 b11 = *reinterpret_cast<const f2a4 *>(b + (o1 + pxy4 + px4));
  {
    const float c00 = lerp(a00.x, a00.y, ax.w), c10 = lerp(a10.x, a10.y, ax.w);
    const float c01 = lerp(a01.x, a01.y, ax.w), c11 = lerp(a11.x, a11.y, ax.w);
    v0 = lerp(lerp(c00, c10, ay0.w), lerp(c01, c11, ay0.w), az0.w);
  }
  {
    const float c00 = lerp(b00.x, b00.y, ax.w), c10 = lerp(b10.x, b10.y, ax.w);
    const float c01 = lerp(b01.x, b01.y, ax.w), c11 = lerp(b11.x, b11.y, ax.w);
    v1 = lerp(lerp(c00, c10, ay1.w), lerp(c01, c11, ay1.w), az1.w);
  }
}
// The same lookups from the texture's z-paired copy (DevTex::zp, entries {v(i), v(i + pxy)}): a
// 16-byte load at entry i holds the x-pair of plane z and of plane z + 1, so one lookup is two row
// loads (rows y and y + 1) where fetch_small takes four, and touches half the cache lines.  The
// lerps are fetch_small's, in its order, on the same values: bit-identical.
#ifndef VR_LUT_ZPAIR
#define VR_LUT_ZPAIR 1
#endif
__device__ __forceinline__ float lerp_zrows(const f4a8 &r0, const f4a8 &r1, const AxF &ax, const AxF &ay,
                                            const AxF &az) {
  const float c00 = lerp(r0.x, r0.z, ax.w), c10 = lerp(r1.x, r1.z, ax.w);
  const float c01 = lerp(r0.y, r0.w, ax.w), c11 = lerp(r1.y, r1.w, ax.w);
  const float c0 = lerp(c00, c10, ay.w), c1 = lerp(c01, c11, ay.w);
  return lerp(c0, c1, az.w);
}
__device__ __forceinline__ float fetch_small_z(const DevTex &t, const AxF &ax, const AxF &ay, const AxF &az) {
  const uint32_t o = (uint32_t)fmaf(az.fl, t.fpxy4, fmaf(ay.fl, t.fpx4, fmaf(ax.fl, 4.f, t.fbase4)));
  const uint32_t o2 = o + o, px8 = t.px * 8u;  // entries are 8 bytes
  const char *b = reinterpret_cast<const char *>(t.zp);
  const f4a8 r0 = *reinterpret_cast<const f4a8 *>(b + o2);
  const f4a8 r1 = *reinterpret_cast<const f4a8 *>(b + (o2 + px8));
  return lerp_zrows(r0, r1, ax, ay, az);
}
__device__ __forceinline__ void fetch_small2_z(const DevTex &t, const AxF &ax, const AxF &ay0, const AxF &az0,
                                               const AxF &ay1, const AxF &az1, float &v0, float &v1) {
  const float ox = fmaf(ax.fl, 4.f, t.fbase4);
  const uint32_t o0 = (uint32_t)fmaf(az0.fl, t.fpxy4, fmaf(ay0.fl, t.fpx4, ox));
  const uint32_t o1 = (uint32_t)fmaf(az1.fl, t.fpxy4, fmaf(ay1.fl, t.fpx4, ox));
  const uint32_t px8 = t.px * 8u;
  const char *b = reinterpret_cast<const char *>(t.zp);
  const f4a8 a0 = *reinterpret_cast<const f4a8 *>(b + (o0 + o0));
  const f4a8 a1 = *reinterpret_cast<const f4a8 *>(b + (o0 + o0 + px8));
  const f4a8 b0 = *reinterpret_cast<const f4a8 *>(b + (o1 + o1));
  const f4a8 b1 = *reinterpret_cast<const f4a8 *>(b + (o1 + o1 + px8));
  v0 = lerp_zrows(a0, a1, ax, ay0, az0);
  v1 = lerp_zrows(b0, b1, ax, ay1, az1);
}
__device__ __forceinline__ Ax to_ax(const AxF &a) { return Ax{(int)a.fl, a.w}; }

// The LUT value of one light (0 if the illumination texture is unbound).
template <bool FMA = false>
__device__ __forceinline__ float lut_light(const DevTex &lut, const AxF &la, float beta, float gamma) {
  if (lut.p == nullptr) return 0.f;
  if (lut.one) {
    const float q = lut.p[0];
    return fmaf(0.5f, q - q, q);
  }
  const AxF lb = axis_lut<FMA>(beta, lut.fny), lg = axis_lut<FMA>(gamma, lut.fnz);
  if (lut.small) return fetch_small(lut, la, lb, lg);
  return fetch<false>(lut, to_ax(la), to_ax(lb), to_ax(lg));
}

// Trilinear fetch of the three lookup-gradient textures at once from their interleaved copy
// (RenderParams::gvec): eight aligned 16-byte corner loads, and each component goes through exactly
// the interpolation fetch() applies to its own texture.  VR_GVEC_BRICK: padded voxel (X, Y, Z) is
// entry ((Z/2 * by + Y/2) * bx + X/2) * 8 + (X&1) + 2 (Y&1) + 4 (Z&1) -- a cell's corners span
// 1-8 lines (3.4 on average) where rows of the padded volume take 4-8 (4.5), and a wave's oblique
// footprint touches fewer lines.  Without it: rows of the padded volume (pitches of `t`).
// (Split into the eight corner loads and their interpolation; round 5 measured the loads issued
// before the emission fetch slower -- C3 30.3-30.4 ms at 4 waves per SIMD, 34.8 at 5 with spills,
// vs 28.8-29.0, r5w.)
struct GvCell {
  float4 a00, b00, a10, b10, a01, b01, a11, b11;
};
template <bool BIG>
__device__ __forceinline__ GvCell gvec_load(const float *gvec, const DevTex &t, uint32_t row8, uint32_t plane8,
                                            const Ax &ax, const Ax &ay, const Ax &az) {
  GvCell q;
  if (VR_GVEC_BRICK) {
    const uint32_t X = (uint32_t)(ax.i + 1), Y = (uint32_t)(ay.i + 1), Z = (uint32_t)(az.i + 1);
    const uint32_t dx = (X & 1u) ? 7u : 1u, dy = (Y & 1u) ? row8 - 2u : 2u, dz = (Z & 1u) ? plane8 - 4u : 4u;
    const uint32_t xy = ((X >> 1) << 3) + (X & 1u) + (Y >> 1) * row8 + ((Y & 1u) << 1) + ((Z & 1u) << 2);
    uint64_t o;
    if (BIG) o = (uint64_t)(Z >> 1) * plane8 + xy;
    else o = (Z >> 1) * plane8 + xy;
    const float4 *b = reinterpret_cast<const float4 *>(gvec) + o;
    q.a00 = b[0], q.b00 = b[dx], q.a10 = b[dy], q.b10 = b[dy + dx];
    q.a01 = b[dz], q.b01 = b[dz + dx], q.a11 = b[dz + dy], q.b11 = b[dz + dy + dx];
  } else {
    uint64_t o;
    if (BIG) o = ((uint64_t)(az.i + 1) * t.pxy + (uint64_t)(ay.i + 1) * t.px) + (uint64_t)(ax.i + 1);
    else o = ((uint32_t)(az.i + 1) * t.pxy + (uint32_t)(ay.i + 1) * t.px) + (uint32_t)(ax.i + 1);
    const float4 *b = reinterpret_cast<const float4 *>(gvec) + o;
    q.a00 = b[0], q.b00 = b[1], q.a10 = b[t.px], q.b10 = b[t.px + 1];
    q.a01 = b[t.pxy], q.b01 = b[t.pxy + 1], q.a11 = b[t.pxy + t.px], q.b11 = b[t.pxy + t.px + 1];
  }
  return q;
}
__device__ __forceinline__ f3 gvec_lerp(const GvCell &q, const Ax &ax, const Ax &ay, const Ax &az) {
  f3 r;
#define VR_TRI(c)                                                                                  \
  {                                                                                                \
    const float c00 = lerp(q.a00.c, q.b00.c, ax.w), c10 = lerp(q.a10.c, q.b10.c, ax.w);            \
    const float c01 = lerp(q.a01.c, q.b01.c, ax.w), c11 = lerp(q.a11.c, q.b11.c, ax.w);            \
    const float c0 = lerp(c00, c10, ay.w), c1 = lerp(c01, c11, ay.w);                              \
    r.c = lerp(c0, c1, az.w);                                                                      \
  }
  VR_TRI(x)
  VR_TRI(y)
  VR_TRI(z)
#undef VR_TRI
  return r;
}
template <bool BIG>
__device__ __forceinline__ f3 fetch_vec(const float *gvec, const DevTex &t, uint32_t row8, uint32_t plane8,
                                        const Ax &ax, const Ax &ay, const Ax &az) {
  return gvec_lerp(gvec_load<BIG>(gvec, t, row8, plane8, ax, ay, az), ax, ay, az);
}

// tex3D on any texture state (unbound -> 0, 1x1x1 -> single voxel through the same lerp algebra).
template <bool BIG>
__device__ __forceinline__ float tex3d(const DevTex &t, float x, float y, float z) {
  if (t.p == nullptr) return 0.f;  // wave-uniform
  if (t.one) {
    const float v = t.p[0];
    return fmaf(0.5f, v - v, v);  // == lerp(v, v, w) for every w (NaN/inf/-0 included)
  }
  return fetch<BIG>(t, axis(x, t.nx, t.fnx), axis(y, t.ny, t.fny), axis(z, t.nz, t.fnz));
}


#ifndef VR_MIN_WAVES
#define VR_MIN_WAVES 1
#endif

// Workgroup -> 16x16-pixel tile.  tile_mode 1 (XCD-aware): workgroups are dealt
// round-robin to the 8 XCDs (b % 8 share one, observed -- a speed assumption only), so block b
// is mapped to tile `within` of super-tile s = (b/8/64)*8 + b%8, a super-tile being 8x8 tiles
// (128x128 pixels): each XCD's L2 then serves the rays of one or two compact image regions
// instead of 128 scattered tiles.  The map is a bijection onto the padded super-tile grid;
// blocks past the image do nothing.
__device__ __forceinline__ bool tile_of_block(const RenderParams &P, int &tx, int &ty) {
  const int b = blockIdx.x;
  const int ntx = (P.part_cols + 15) >> 4, nty = (P.height + 15) >> 4;
  if (P.tile_mode == 0) {
    tx = b % ntx;
    ty = b / ntx;
  } else {
    const int nsx = (ntx + 7) >> 3;
    const int j = b >> 3, s = ((j >> 6) << 3) + (b & 7), w = j & 63;
    tx = (s % nsx) * 8 + (w & 7);
    ty = (s / nsx) * 8 + (w >> 3);
  }
  return tx < ntx && ty < nty;
}

// Primary ray of pixel (x, y) and its box intersection (volumeRender_kernel.cu:388-425), op for
// op as the oracle.  Returns hit; tnear is already clamped to 0.
__device__ __forceinline__ bool ray_setup(const RenderParams &P, int x, int y, f3 &o, f3 &d, float &tnear,
                                          float &tfar, int view = 0) {
  const float u = fmaf((float)x / P.fw, 2.f, -1.f);
  const float v = fmaf(((float)y / P.fh) * 2.f, P.ratio, -P.ratio);
  o = view ? mk(P.eye2[0], P.eye2[1], P.eye2[2]) : mk(P.eye[0], P.eye[1], P.eye[2]);
  f3 du;
  du.x = fmaf(P.focal, P.zdir[0], fmaf(v, P.ydir[0], u * P.nx_[0]));
  du.y = fmaf(P.focal, P.zdir[1], fmaf(v, P.ydir[1], u * P.nx_[1]));
  du.z = fmaf(P.focal, P.zdir[2], fmaf(v, P.ydir[2], u * P.nx_[2]));
  const float inv = 1.f / sqrt_cr(dot3(du, du));
  d = mk(du.x * inv, du.y * inv, du.z * inv);
  const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);
  const f3 bmax = mk(-P.bmin[0], -P.bmin[1], -P.bmin[2]);
  const f3 id = mk(1.f / d.x, 1.f / d.y, 1.f / d.z);
  float tmin = ((id.x < 0.f ? bmax.x : bmin.x) - o.x) * id.x;
  float tmax = ((id.x < 0.f ? bmin.x : bmax.x) - o.x) * id.x;
  const float tymin = ((id.y < 0.f ? bmax.y : bmin.y) - o.y) * id.y;
  const float tymax = ((id.y < 0.f ? bmin.y : bmax.y) - o.y) * id.y;
  bool hit = !((tmin > tymax) || (tymin > tmax));
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  const float tzmin = ((id.z < 0.f ? bmax.z : bmin.z) - o.z) * id.z;
  const float tzmax = ((id.z < 0.f ? bmin.z : bmax.z) - o.z) * id.z;
  hit = hit && !((tmin > tzmax) || (tzmin > tmax));
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  tnear = tmin < 0.f ? 0.f : tmin;
  tfar = tmax;
  return hit;
}

// shade() of volumeRender_kernel.cu:308-353 after the gradient: per light, the three angles and
// the LUT lookup, accumulated as ((refl*light)*lc)*color + result.  `refl` is Fr * R(p).
#ifndef VR_ABLATE
#define VR_ABLATE 0  // diagnostic builds only (tools/ablate_build.sh): 1 LUT, 2 angles, 4 taps, 8 exp,
                     // 16 no staged-box check, 32 no lookup-gradient fetch
#endif

// a / b for the arguments of the angle acosf calls, bit-identical to IEEE a / b wherever it can
// matter: the compiler's correctly rounded sequence (Newton-refined reciprocal, two residual
// corrections) without its v_div_scale / v_div_fixup range handling, which is the identity for
// 2^-40 <= |b| <= 2^40 and |a| <= 2^40 (tools/microbench: 2^33 random pairs, 0 mismatches).  Here
// |a| <= |b| (Cauchy-Schwarz, up to rounding), and a tiny quotient gives acosf == pi/2 however it
// rounds, so only b is tested; a wave with any other lane takes '/'.
__device__ __forceinline__ float div_acos_arg(float a, float b) {
  const uint32_t ub = __float_as_uint(b) & 0x7fffffffu;
  if (__builtin_expect(__all(ub - 0x2b800000u <= 0x28000000u), 1)) {
    const float y0 = __builtin_amdgcn_rcpf(b);
    const float y1 = fmaf(fmaf(-b, y0, 1.f), y0, y0);
    const float q0 = a * y1;
    const float q1 = fmaf(fmaf(-b, q0, a), y1, q0);
    return fmaf(fmaf(-b, q1, a), y1, q1);
  }
  return a / b;
}

__device__ __forceinline__ float div_fast(float a, float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float y1 = fmaf(fmaf(-b, y0, 1.f), y0, y0);
  const float q0 = a * y1;
  const float q1 = fmaf(fmaf(-b, q0, a), y1, q0);
  return fmaf(fmaf(-b, q1, a), y1, q1);
}
// a / b with one residual correction on the hardware reciprocal (no Newton step on it): not always
// correctly rounded (tools/microbench/cosine_check.hip counts how often it is not).
__device__ __forceinline__ float div_short(float a, float b) {
  const float y = __builtin_amdgcn_rcpf(b);
  const float q0 = a * y;
  return fmaf(fmaf(-b, q0, a), y, q0);
}
// div_acos_arg over a group with one wave-wide guard (see div_acos_arg for the exactness argument).
template <int N>
__device__ __forceinline__ void div_acos_n(const float (&a)[N], const float (&b)[N], float (&q)[N]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < N; ++i) ok = ok && ((__float_as_uint(b[i]) & 0x7fffffffu) - 0x2b800000u <= 0x28000000u);
  if (__builtin_expect(__all(ok), 1)) {
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = div_fast(a[i], b[i]);
  } else {
#pragma unroll
    for (int i = 0; i < N; ++i) q[i] = a[i] / b[i];
  }
}

// x / pi, correctly rounded, for x = 0, NaN or x >= 2^-100 -- the range of acosf: x * RN(1/pi)
// corrected by one fma residual step (3 VALU instead of the 12 of a general IEEE divide).  Equal to
// the IEEE quotient for every such fp32 x (exhaustive check: tools/microbench/divpi_check.c).
__device__ __forceinline__ float divpi(float x) {
  const float r = 0x1.45f306p-2f;  // RN(1 / (float)pi)
  const float q = x * r;
  return fmaf(fmaf(-q, VR_PI, x), r, q);
}

// acos(q) / pi for the fast shading variant.  VR_FAST_ACOS 0: the device library's acospi (one
// rounding, ~21 VALU); 1: acospi(t) = sqrt(1 - t) * P8(t) on t = |q| (the form of Abramowitz &
// Stegun 4.4.46; P8 a weighted least-squares fit at Chebyshev nodes of acos(t) / (pi sqrt(1 - t)),
// relative approximation error 2.4e-9), acospi(q) = 1 - acospi(-q) for q < 0: 13 VALU.  In fp32,
// over every q in [-1, 1]: 94 % correctly rounded, at most 1.95 ulp.  NaN and |q| > 1 give NaN as
// acosf does (sqrt of a negative).
#ifndef VR_FAST_ACOS
#define VR_FAST_ACOS 1
#endif
#ifndef VR_ACOS_LITERALS
#define VR_ACOS_LITERALS 1
#endif
#ifndef VR_FAST_NLEN
#define VR_FAST_NLEN 1  // 1: the fast variant takes the unit normal's length as 1 (shade_lights)
#endif
#ifndef VR_FAST_COS
#define VR_FAST_COS 1  // 1: the fast variant's cosines as dot * rsq * rsq; 0: correctly rounded (ablation)
#endif
#ifndef VR_FAST_NX
#define VR_FAST_NX 0  // 1: the fast variant's unit normal as the oracle's, -(g * (1 / sqrtf(g.g))), bit for bit
#endif
#ifndef VR_FAST_GX
#define VR_FAST_GX 0  // 1: the fast variant's gamma cosines correctly rounded (the oracle's quotient)
#endif
#ifndef VR_FAST_NXQ
#define VR_FAST_NXQ 0  // 1: the fast normal as -(g * v_rcp(v_sqrt(g.g))) (the oracle's op sequence, hardware ops)
#endif
#ifndef VR_FAST_GXQ
#define VR_FAST_GXQ 0  // 1: gamma's cosine as dot / (v_sqrt(lip.lip) v_sqrt(lop.lop)), one-correction quotient
#endif
#ifndef VR_FAST_HYBQ
// gamma's cosine as the oracle's correctly rounded quotient where |cos gamma| > VR_HYB_TG (parity
// ablation, round 4): 2 per lane with the compiler's IEEE sequences, 1 per wave with the guarded
// sequences, 0 never (default: VR_FAST_CLAMP takes care of what they fixed, at a fraction of their
// +5 % cost).
#define VR_FAST_HYBQ 0
#endif
#ifndef VR_FAST_HYBRID
#define VR_FAST_HYBRID 0  // 1: rsq shading, and XN + XG shading where gamma is ill-conditioned (shade_fast)
#endif
#ifndef VR_HYB_TA
#define VR_HYB_TA 0.01f  // hybrid: |lip|^2 < TA |li|^2 (view within asin(0.1) of the normal), same for lights
#endif
#ifndef VR_HYB_TG
#define VR_HYB_TG 0.999f  // |cos gamma| > TG: the oracle's quotient (VR_FAST_HYBQ; below gamma = 0.0245 the
                          // LUT taps clamp to one voxel and the weight no longer matters)
#endif
#ifndef VR_HYB_TU
// ... and |cos gamma| < TU: beyond it gamma is within 0.0245 of 0 or pi, where both taps of the LUT's
// gamma axis are the same voxel (the weight does not matter); 2: no upper bound
#define VR_HYB_TU 2.f
#endif
#ifndef VR_RSQ_NR
#define VR_RSQ_NR 0  // 1: one Newton step on every cosine's hardware rsq
#endif
// rsq of a cosine normalisation (VR_RSQ_NR: one Newton step y (1 + (1 - x y^2) / 2))
__device__ __forceinline__ float rsq_c(float x) {
  const float y = __builtin_amdgcn_rsqf(x);
#if VR_RSQ_NR
  const float r = fmaf(-(x * y), y, 1.f);
  return fmaf(r * 0.5f, y, y);
#else
  return y;
#endif
}
// RN(1 / RN(sqrt(x))), the oracle's 1.f / sqrtf(x), for x >= 0: the correctly rounded root and
// the compiler's correctly rounded reciprocal sequence without its range fix-ups where every lane
// of the wave has x = 0 or 2^-80 <= x <= 2^80 (the root then in [2^-40, 2^40], div_fast's identity
// range); x = 0 gives +inf, as 1 / 0.  Other waves take the library operations.
__device__ __forceinline__ float rcp_sqrt_cr(float x) {
  const uint32_t u = __float_as_uint(x);
  if (__builtin_expect(__all(u == 0u || u - 0x17800000u <= 0x50000000u), 1)) {
    const float r = div_fast(1.f, sqrt_fast(x));
    return u == 0u ? __builtin_inff() : r;
  }
  return 1.f / sqrtf(x);
}
extern "C" __device__ float __ocml_acospi_f32(float);
__device__ __forceinline__ float acospi_q(float q);
// acos(q) / pi of a fast-shading cosine (shade_fast).  VR_FAST_CLAMP (default 1, inside acospi_q at
// no cost; 2: an explicit compare and select here): a cosine the rsq product rounds below -1 is
// taken as -1, NaN kept.  Where the exact cosine lies within a few ulps
// of -1 (a back-facing normal, a light opposite the view in the tangent plane) the rsq product and
// the oracle's correctly rounded quotient round past -1 independently, and past it acosf is NaN,
// which the LUT lookup reads as the coordinate 0 -- the LUT at angle 0 instead of pi.  The fp64
// oracle never rounds past; taking the cosine as -1 agrees with it everywhere and with the fp32
// oracle wherever that one does not round past either (where it does, the envelope |fp32 - fp64|
// holds the difference).  Past +1 needs no care: angle 0 and the NaN's coordinate 0 read the same
// LUT voxels.  This was the whole of the fast shading's remaining SURVEY 8c gap.
#ifndef VR_FAST_CLAMP
#define VR_FAST_CLAMP 1
#endif
__device__ __forceinline__ float acospi_f(float q) {
  if (VR_FAST_CLAMP == 2) q = q < -1.f ? -1.f : q;  // (the explicit form: a compare and a select)
  return acospi_q(q);
}
__device__ __forceinline__ float acospi_q(float q) {
#if VR_ABLATE & 2
  return fmaf(q, -0.5f, 0.5f);  // diagnostic: the angle's cost removed (wrong image)
#endif
#if VR_FAST_ACOS
  const float t = fabsf(q);
#if VR_ACOS_LITERALS
  // the Horner steps as VOP2 v_fmaak_f32 with the coefficient as a literal: written as plain fmaf the
  // compiler folds |q| into VOP3 fmas, which take no literal on gfx950, and holds the eight
  // coefficients in SGPRs across the sample loop -- where they push other values into v_readlane
  // spills.  Same single rounding per step (d = s0 * s1 + K).
  float p;
  asm("v_mov_b32 %0, 0x3967ab32\n\t"
      "v_fmaak_f32 %0, %0, %1, 0xbaa77072\n\t"
      "v_fmaak_f32 %0, %0, %1, 0x3b67639e\n\t"
      "v_fmaak_f32 %0, %0, %1, 0xbbd8c4b8\n\t"
      "v_fmaak_f32 %0, %0, %1, 0x3c2a004e\n\t"
      "v_fmaak_f32 %0, %0, %1, 0xbc83f1fe\n\t"
      "v_fmaak_f32 %0, %0, %1, 0x3ce82823\n\t"
      "v_fmaak_f32 %0, %0, %1, 0xbd8be5f3\n\t"
      "v_fmaak_f32 %0, %0, %1, 0x3f000000"
      : "=&v"(p)
      : "v"(t));
#else
  float p = 2.209365193e-04f;
  p = fmaf(p, t, -1.277460018e-03f);
  p = fmaf(p, t, 3.530717921e-03f);
  p = fmaf(p, t, -6.615247577e-03f);
  p = fmaf(p, t, 1.037604921e-02f);
  p = fmaf(p, t, -1.610660180e-02f);
  p = fmaf(p, t, 2.833945118e-02f);
  p = fmaf(p, t, -6.830968708e-02f);
  p = fmaf(p, t, 0.5f);
#endif
  // VR_FAST_CLAMP 1: sqrt(|1 - t|) -- a free source modifier -- is the clamp of acospi_f for the few
  // ulps a rounded cosine can exceed 1 in magnitude (the result within sqrt(ulp) of 0 or 1, in the
  // LUT's clamped end cell either way) and keeps NaN; with 1 - t alone they are NaN (coordinate 0)
  const float r = __builtin_amdgcn_sqrtf(VR_FAST_CLAMP == 1 ? fabsf(1.f - t) : 1.f - t) * p;
  // q < 0 ? 1 - r : r without a compare: fma(-1, r, 1) rounds as 1 - r, fma(1, r, 0) is r (q = -0
  // takes the first form: 1 - 0.5 = 0.5 = r, the same value)
  const float sg = __builtin_copysignf(1.f, q);
  return fmaf(sg, r, fmaf(-0.5f, sg, 0.5f));
#else
  return __ocml_acospi_f32(q);
#endif
}

// exp(-x) rounded to nearest, as the oracle's expf (glibc, < 0.502 ulp) gives it: for |x| < 2^-7
// (every sample of a 1024^3 volume at Fa <= 25) the Taylor form 1 + c, c = fma(x^2, q, -x),
// q = 1/2 - x/6 + x^2/24, in fp32 -- -x is exact inside the fma, so c carries one rounding of a
// term ~x^2/2 and the sum 1 + c rounds once at the granularity of the result; measured against
// glibc's expf over 2.9e8 inputs in (-2^-7, 2^-7): 0.005 % differ (by one ulp), where the device
// library's expf and the hardware exp2 differ far more often and with a bias.  That bias matters:
// alpha = 1 - exp(-x) cancels, so one ulp of the exponential is ~2e-4 of a sample's opacity at this
// step size, and a one-sided rounding adds up along every ray (C4's structure channel: 0.03 % of
// the pixel value, rms 0.9 of the fp32 envelope).  Other x: exp in double, rounded.
// Five fast VALU and no transcendental, against the mul, exp2 and sub of __expf.
// the rare general case out of line (one copy per object instead of one per kernel variant)
__device__ __attribute__((noinline)) float exp_neg_rn_general(float x) { return (float)exp(-(double)x); }
// small: the host proved |x| < 2^-7 for every sample of the launch (RenderParams::small_x).
__device__ __forceinline__ float exp_neg_rn(float x, bool small = false) {
  const float x2 = x * x;
  // q = 1/2 - x/6 + x^2/24: its own rounding enters c only through x^2 q (relative 2^-23 of a term
  // below 2^-15), so the inner term is a mul and an add with literal operands (VOP2) -- an fma would
  // need one of its constants held in a register across the sample loop
  const float q = fmaf(x, x * (1.f / 24.f) + (-1.f / 6.f), 0.5f);
  float e = 1.f + fmaf(x2, q, -x);
  if (!small && __builtin_expect(!__all(fabsf(x) < 0x1p-7f), 0))  // wave-uniform: large or non-finite x
    if (!(fabsf(x) < 0x1p-7f)) e = exp_neg_rn_general(x);
  return e;
}

// 1 - __expf(-a * dx) (volumeRender_kernel.cu:456), both shading variants: the oracle's expf
// (exp_neg_rn) -- x = a * dx rounded, then the exponential of its negation, as the oracle's
// expf((-a) * dx) (negation is exact).
// VR_OPACITY_EXP2 1 (a build switch, off by default): the reference's own form instead, __expf as
// CUDA defines it -- exp2(x * log2 e) on the hardware exponential (v_exp_f32), the fast intrinsic of
// volumeRender_kernel.cu:456 -- kept as the model of __expf; no fixture of the reference pins either
// rounding (DESIGN.md s4 "opacity": the oracle's expf was chosen for its unbiased rounding).
#ifndef VR_OPACITY_EXP2
#define VR_OPACITY_EXP2 0
#endif
template <bool FAST>
__device__ __forceinline__ float opacity(float a, float tstep, bool small = false) {
#if VR_ABLATE & 8
  return a * tstep;
#elif VR_OPACITY_EXP2
  return 1.f - __builtin_amdgcn_exp2f(-(a * tstep) * 1.44269504088896341f);
#else
  return 1.f - exp_neg_rn(a * tstep, small);
#endif
}

// FAST = false: op for op the oracle's shading (correctly rounded roots and quotients; only acosf
// comes from the device library).  FAST = true (the default): the angle cosines as
// dot(a,b) * rsq(a.a) * rsq(b.b) with the hardware reciprocal square root (1 ulp, as the
// reference's own rsqrtf normalize) and acos/pi in one step; within the parity tolerance of
// SURVEY.md 8c, about 10 % faster at the metric configuration.
// TAME (vr_march.hip sample_at): the launch's LUT, if it has lights, is a bound grid of fewer than
// 2^22 padded voxels (RenderParams::tame), so only the fetch_small path is compiled.
// The frame's light list through the constant address space: the list never changes during a launch,
// so its (wave-uniform) loads are scalar loads in every kernel -- through a generic pointer the
// compiler keeps them scalar only where no store of the kernel might alias them (in the slab kernel,
// whose resume-point stores are inside the march, they became vector loads, 3 per light pair).
__device__ __forceinline__ DevLight light_at(const RenderParams &P, int i) {
  typedef const __attribute__((address_space(4))) DevLight *cptr;
  const cptr q = (cptr)P.lights + i;  // generic -> constant: an address-space cast
  return DevLight{q->px, q->py, q->pz, q->cr, q->cg, q->cb};
}
// The same for the voxel of a single-voxel texture (the tame reflection term).
__device__ __forceinline__ float voxel0(const float *p) {
  typedef const __attribute__((address_space(4))) float *cptr;
  return ((cptr)p)[0];
}

// The fast variant's shading (shade_lights FAST).  XN: the unit normal bit for bit as the oracle's
// (the correctly rounded 1 / sqrtf); XG: gamma's cosine as the oracle's correctly rounded quotient.
// NEED: set `need` where the sample's gamma is ill-conditioned -- the view or a light direction
// within asin(sqrt(VR_HYB_TA)) of the normal (its projection onto the tangent plane cancels, so the
// normal's last bits decide its direction) or a gamma cosine beyond +-VR_HYB_TG (acos amplifies the
// cosine's rounding there) -- where the hybrid shading (VR_FAST_HYBRID) takes XN + XG.
// NL (round 6): the launch's light count when the kernel was specialised on it (2: the metric frame
// and examples/example1.m; 1: examples/example2.m and example3.m -- the lights are the caller's
// hoisted `pre`, no light loop, no masks of the loop bounds held across the sample loop); 0:
// P.num_lights.
template <bool TAME, bool XN, bool XG, bool NEED, int NL = 0>
__device__ __forceinline__ void shade_fast(const RenderParams &P, const f3 g, const f3 pos, const f3 o,
                                          const float refl, float &ir, float &ig, float &ib, bool &need,
                                          const DevLight *pre = nullptr) {
  static_assert(NL == 0 || ((NL == 1 || NL == 2) && TAME), "specialised for hoisted lights only");
  const int nl = NL ? NL : P.num_lights;
  // n = -g * rsq(g.g): rsq(0) = inf gives the reference's NaN normal for a zero gradient
  float ginv;
  if constexpr (XN) ginv = rcp_sqrt_cr(dot3(g, g));  // the oracle's 1 / sqrtf(g.g), bit for bit
  else if (VR_FAST_NXQ) ginv = __builtin_amdgcn_rcpf(__builtin_amdgcn_sqrtf(dot3(g, g)));
  else ginv = __builtin_amdgcn_rsqf(dot3(g, g));
  const f3 n = mk(-(g.x * ginv), -(g.y * ginv), -(g.z * ginv));
  const f3 li = mk(o.x - pos.x, o.y - pos.y, o.z - pos.z);
  const float dli = dot3(li, n);
  const f3 lip = mk(fmaf(-dli, n.x, li.x), fmaf(-dli, n.y, li.y), fmaf(-dli, n.z, li.z));
  // |n| is 1 to within the rsq's ulp: its length is not divided out again (VR_FAST_NLEN 0 does)
#if VR_FAST_NLEN
  const float rn = 1.f;
#else
  const float rn = rsq_c(dot3(n, n));
#endif
  // XG: gamma's cosine as the oracle's dot(lip, lop) / (|lip| |lop|): `rlip` then holds |lip|
  const float lip2 = dot3(lip, lip), li2 = dot3(li, li);
  const float rlip = XG ? sqrt_cr(lip2) : (VR_FAST_GXQ ? __builtin_amdgcn_sqrtf(lip2) : rsq_c(lip2));
  // the cosine of gamma for light vector lo (its projection lop); NEED: the sample is in a region
  // where gamma is ill-conditioned (see shade_lights)
  auto gamma_q = [&](const f3 &lo, const f3 &lop) {
    const float lop2 = dot3(lop, lop);
    float q;
    if constexpr (XG) q = div_acos_arg(dot3(lip, lop), rlip * sqrt_cr(lop2));
    else if (VR_FAST_GXQ) q = div_short(dot3(lip, lop), rlip * __builtin_amdgcn_sqrtf(lop2));
    else q = dot3(lip, lop) * (rlip * rsq_c(lop2));
    if constexpr (NEED) need = need || fabsf(q) > VR_HYB_TG || lop2 < VR_HYB_TA * dot3(lo, lo);
    if constexpr (VR_FAST_HYBQ == 2 && !XG && !NEED) {
      // per lane, no wave-wide guard: near |cos| = 1 (where acos amplifies the cosine's rounding) the
      // oracle's quotient dot / (sqrtf(lip.lip) sqrtf(lop.lop)) with the compiler's IEEE sequences
      const float aq = fabsf(q);
      if (__builtin_expect(aq > VR_HYB_TG && aq < VR_HYB_TU, 0)) q = dot3(lip, lop) / (sqrtf(lip2) * sqrtf(lop2));
    } else if constexpr (VR_FAST_HYBQ == 1 && !XG && !NEED) {
      // near |cos| = 1 acos amplifies the cosine's rounding: there the oracle's quotient
      const bool nd = fabsf(q) > VR_HYB_TG;
      if (__builtin_expect(__any(nd), 0)) {
        const float qx = div_acos_arg(dot3(lip, lop), sqrt_cr(lip2) * sqrt_cr(lop2));
        if (nd) q = qx;
      }
    }
    return q;
  };
  if constexpr (NEED) need = lip2 < VR_HYB_TA * li2;
  const float alpha_n = acospi_f(dot3(n, li) * (rn * rsq_c(li2)));
  const AxF la = axis_lut<true>(alpha_n, P.lut.fnx);
  int i = 0;
  if (TAME || (P.lut.p != nullptr && P.lut.small && !P.lut.one)) {
    // the common LUT (bound, below 2^22 padded voxels): one wave-uniform test for the frame's
    // lights; a pair's eight LUT row loads are issued together, ahead of their lerps
    for (; i + 1 < nl; i += 2) {
      // pre: the first pair held in registers by the caller (vr_march.hip VR_LIGHTS_HOIST)
      const DevLight L0 = NL == 2 ? pre[0] : ((pre && i == 0) ? pre[0] : light_at(P, i));
      const DevLight L1 = NL == 2 ? pre[1] : ((pre && i == 0) ? pre[1] : light_at(P, i + 1));
      const f3 lo0 = mk(L0.px - pos.x, L0.py - pos.y, L0.pz - pos.z);
      const f3 lo1 = mk(L1.px - pos.x, L1.py - pos.y, L1.pz - pos.z);
      const float dlo0 = dot3(lo0, n), dlo1 = dot3(lo1, n);
      const f3 lop0 = mk(fmaf(-dlo0, n.x, lo0.x), fmaf(-dlo0, n.y, lo0.y), fmaf(-dlo0, n.z, lo0.z));
      const f3 lop1 = mk(fmaf(-dlo1, n.x, lo1.x), fmaf(-dlo1, n.y, lo1.y), fmaf(-dlo1, n.z, lo1.z));
      const float beta0 = acospi_f(dlo0 * (rn * rsq_c(dot3(lo0, lo0))));
      const float gamma0 = acospi_f(gamma_q(lo0, lop0));
      const float beta1 = acospi_f(dlo1 * (rn * rsq_c(dot3(lo1, lo1))));
      const float gamma1 = acospi_f(gamma_q(lo1, lop1));
      float light0, light1;
#if VR_ABLATE & 1  // diagnostic: the LUT fetch's cost removed (wrong image)
      light0 = beta0 + gamma0 + la.w;
      light1 = beta1 + gamma1 + la.w;
#else
      if (TAME && VR_LUT_ZPAIR)  // the host binds a tame launch's LUT with its z-paired copy
        fetch_small2_z(P.lut, la, axis_lut<true>(beta0, P.lut.fny), axis_lut<true>(gamma0, P.lut.fnz),
                       axis_lut<true>(beta1, P.lut.fny), axis_lut<true>(gamma1, P.lut.fnz), light0, light1);
      else
        fetch_small2(P.lut, la, axis_lut<true>(beta0, P.lut.fny), axis_lut<true>(gamma0, P.lut.fnz),
                     axis_lut<true>(beta1, P.lut.fny), axis_lut<true>(gamma1, P.lut.fnz), light0, light1);
#endif
      const float rl0 = refl * light0;
      ir = fmaf(rl0 * L0.cr, P.color[0], ir);
      ig = fmaf(rl0 * L0.cg, P.color[1], ig);
      ib = fmaf(rl0 * L0.cb, P.color[2], ib);
      const float rl1 = refl * light1;
      ir = fmaf(rl1 * L1.cr, P.color[0], ir);
      ig = fmaf(rl1 * L1.cg, P.color[1], ig);
      ib = fmaf(rl1 * L1.cb, P.color[2], ib);
    }
  }
  if constexpr (!TAME) for (; i + 1 < nl; i += 2) {
    const DevLight L0 = light_at(P, i), L1 = light_at(P, i + 1);
    const f3 lo0 = mk(L0.px - pos.x, L0.py - pos.y, L0.pz - pos.z);
    const f3 lo1 = mk(L1.px - pos.x, L1.py - pos.y, L1.pz - pos.z);
    const float dlo0 = dot3(lo0, n), dlo1 = dot3(lo1, n);
    const f3 lop0 = mk(fmaf(-dlo0, n.x, lo0.x), fmaf(-dlo0, n.y, lo0.y), fmaf(-dlo0, n.z, lo0.z));
    const f3 lop1 = mk(fmaf(-dlo1, n.x, lo1.x), fmaf(-dlo1, n.y, lo1.y), fmaf(-dlo1, n.z, lo1.z));
    const float beta0 = acospi_f(dlo0 * (rn * rsq_c(dot3(lo0, lo0))));
    const float gamma0 = acospi_f(gamma_q(lo0, lop0));
    const float beta1 = acospi_f(dlo1 * (rn * rsq_c(dot3(lo1, lo1))));
    const float gamma1 = acospi_f(gamma_q(lo1, lop1));
    const float light0 = lut_light<true>(P.lut, la, beta0, gamma0);
    const float light1 = lut_light<true>(P.lut, la, beta1, gamma1);
    const float rl0 = refl * light0;
    ir = fmaf(rl0 * L0.cr, P.color[0], ir);
    ig = fmaf(rl0 * L0.cg, P.color[1], ig);
    ib = fmaf(rl0 * L0.cb, P.color[2], ib);
    const float rl1 = refl * light1;
    ir = fmaf(rl1 * L1.cr, P.color[0], ir);
    ig = fmaf(rl1 * L1.cg, P.color[1], ig);
    ib = fmaf(rl1 * L1.cb, P.color[2], ib);
  }
  if (i < nl) {
    const DevLight L = NL == 1 ? pre[0] : light_at(P, i);
    const f3 lo = mk(L.px - pos.x, L.py - pos.y, L.pz - pos.z);
    const float dlo = dot3(lo, n);
    const f3 lop = mk(fmaf(-dlo, n.x, lo.x), fmaf(-dlo, n.y, lo.y), fmaf(-dlo, n.z, lo.z));
    const float beta = acospi_f(dlo * (rn * rsq_c(dot3(lo, lo))));
    const float gamma = acospi_f(gamma_q(lo, lop));
    const float rl = refl * (TAME ? (VR_LUT_ZPAIR ? fetch_small_z(P.lut, la, axis_lut<true>(beta, P.lut.fny),
                                                                 axis_lut<true>(gamma, P.lut.fnz))
                                                  : fetch_small(P.lut, la, axis_lut<true>(beta, P.lut.fny),
                                                                axis_lut<true>(gamma, P.lut.fnz)))
                                  : lut_light<true>(P.lut, la, beta, gamma));
    ir = fmaf(rl * L.cr, P.color[0], ir);
    ig = fmaf(rl * L.cg, P.color[1], ig);
    ib = fmaf(rl * L.cb, P.color[2], ib);
  }
}

template <bool FAST, bool TAME = false, int NL = 0>
__device__ __forceinline__ void shade_lights(const RenderParams &P, const f3 g, const f3 pos, const f3 o,
                                             const float refl, float &ir, float &ig, float &ib,
                                             const DevLight *pre = nullptr) {
#if !VR_FAST_COS
  if constexpr (FAST) {
    // VR_FAST_COS 0 (parity ablation): the normal and the angle cosines in the exact variant's
    // correctly rounded op sequence (the oracle's), only acos/pi as acospi_q and the opacity as
    // exp2 differ from it
    const float ginv = 1.f / sqrt_cr(dot3(g, g));
    const f3 n = mk(-(g.x * ginv), -(g.y * ginv), -(g.z * ginv));
    const f3 li = mk(o.x - pos.x, o.y - pos.y, o.z - pos.z);
    const float dli = dot3(li, n);
    const f3 lip = mk(fmaf(-dli, n.x, li.x), fmaf(-dli, n.y, li.y), fmaf(-dli, n.z, li.z));
    float sq_in[3] = {dot3(n, n), dot3(li, li), dot3(lip, lip)}, sq[3];
    sqrt_cr_n<3>(sq_in, sq);
    const float nlen = sq[0], liplen = sq[2];
    float alpha_n;
    {
      const float num[1] = {dot3(n, li)}, den[1] = {nlen * sq[1]};
      float q[1];
      div_acos_n<1>(num, den, q);
      alpha_n = acospi_q(q[0]);
    }
    const AxF la = axis_lut<true>(alpha_n, P.lut.fnx);
    for (int i = 0; i < P.num_lights; ++i) {
      const DevLight L = light_at(P, i);
      const f3 lo = mk(L.px - pos.x, L.py - pos.y, L.pz - pos.z);
      const float dlo = dot3(lo, n);
      const f3 lop = mk(fmaf(-dlo, n.x, lo.x), fmaf(-dlo, n.y, lo.y), fmaf(-dlo, n.z, lo.z));
      float li_in[2] = {dot3(lo, lo), dot3(lop, lop)}, ln[2];
      sqrt_cr_n<2>(li_in, ln);
      const float num[2] = {dot3(n, lo), dot3(lip, lop)}, den[2] = {nlen * ln[0], liplen * ln[1]};
      float q[2];
      div_acos_n<2>(num, den, q);
      const float rl = refl * lut_light<true>(P.lut, la, acospi_q(q[0]), acospi_q(q[1]));
      ir = fmaf(rl * L.cr, P.color[0], ir);
      ig = fmaf(rl * L.cg, P.color[1], ig);
      ib = fmaf(rl * L.cb, P.color[2], ib);
    }
  } else
#endif
  if constexpr (FAST) {
#if VR_FAST_HYBRID
    // the rsq-based shading everywhere, and where gamma is ill-conditioned (NEED) the sample's
    // shading again with the oracle's normal and gamma cosines (per lane: the image does not depend
    // on which lanes share a wave)
    bool need = false;
    const float ir0 = ir, ig0 = ig, ib0 = ib;
    shade_fast<TAME, false, false, true>(P, g, pos, o, refl, ir, ig, ib, need);
    if (__any(need)) {
      float er = ir0, eg = ig0, eb = ib0;
      bool unused = false;
      shade_fast<TAME, true, true, false>(P, g, pos, o, refl, er, eg, eb, unused);
      if (need) {
        ir = er;
        ig = eg;
        ib = eb;
      }
    }
#else
    bool unused = false;
    shade_fast<TAME, VR_FAST_NX, VR_FAST_GX, false, NL>(P, g, pos, o, refl, ir, ig, ib, unused, pre);
#endif
  } else {
    // surface normal n = -normalize(g); normalize(0) = 0 * inf = NaN as in the reference.
    // Correctly rounded 1/sqrtf, bit-identical to the oracle: the projections li - (li.n)n below
    // cancel when the view ray is parallel to n, and gamma then depends on every bit of n.
    const float ginv = 1.f / sqrt_cr(dot3(g, g));
    const f3 n = mk(-(g.x * ginv), -(g.y * ginv), -(g.z * ginv));
    const f3 li = mk(o.x - pos.x, o.y - pos.y, o.z - pos.z);  // lightIn = eye - pos
    const float dli = dot3(li, n);
    const f3 lip = mk(fmaf(-dli, n.x, li.x), fmaf(-dli, n.y, li.y), fmaf(-dli, n.z, li.z));
    // angle(a,b)/pi = acos(dot(a,b) / (length(a)*length(b))) / PI, op for op as the oracle; the
    // square roots and quotients of one stage share a guard (sqrt_cr_n, div_acos_n)
    float sq_in[3] = {dot3(n, n), dot3(li, li), dot3(lip, lip)}, sq[3];
    sqrt_cr_n<3>(sq_in, sq);
    const float nlen = sq[0], liplen = sq[2];
    float alpha_n;
    {
#if VR_ABLATE & 2
      alpha_n = dot3(n, li) * 0.1f;
#else
      const float num[1] = {dot3(n, li)}, den[1] = {nlen * sq[1]};
      float q[1];
      div_acos_n<1>(num, den, q);
      alpha_n = divpi(acosf(q[0]));
#endif
    }
    const AxF la = axis_lut(alpha_n, P.lut.fnx);
    // lights two at a time: both angle pairs, then both LUT fetches (their loads overlap), then the
    // accumulation in light order, exactly as the reference's sequential loop
    int i = 0;
    for (; i + 1 < P.num_lights; i += 2) {
      const DevLight L0 = light_at(P, i), L1 = light_at(P, i + 1);
      const f3 lo0 = mk(L0.px - pos.x, L0.py - pos.y, L0.pz - pos.z);  // lightOut
      const f3 lo1 = mk(L1.px - pos.x, L1.py - pos.y, L1.pz - pos.z);
      const float dlo0 = dot3(lo0, n), dlo1 = dot3(lo1, n);
      const f3 lop0 = mk(fmaf(-dlo0, n.x, lo0.x), fmaf(-dlo0, n.y, lo0.y), fmaf(-dlo0, n.z, lo0.z));
      const f3 lop1 = mk(fmaf(-dlo1, n.x, lo1.x), fmaf(-dlo1, n.y, lo1.y), fmaf(-dlo1, n.z, lo1.z));
      float beta0, gamma0, beta1, gamma1;
#if VR_ABLATE & 2
      beta0 = dot3(n, lo0) * 0.01f; gamma0 = dot3(lip, lo0) * 0.01f + liplen;
      beta1 = dot3(n, lo1) * 0.01f; gamma1 = dot3(lip, lo1) * 0.01f + liplen;
#else
      float li_in[4] = {dot3(lo0, lo0), dot3(lop0, lop0), dot3(lo1, lo1), dot3(lop1, lop1)}, ln[4];
      sqrt_cr_n<4>(li_in, ln);
      const float num[4] = {dot3(n, lo0), dot3(lip, lop0), dot3(n, lo1), dot3(lip, lop1)};
      const float den[4] = {nlen * ln[0], liplen * ln[1], nlen * ln[2], liplen * ln[3]};
      float q[4];
      div_acos_n<4>(num, den, q);
      beta0 = divpi(acosf(q[0]));
      gamma0 = divpi(acosf(q[1]));
      beta1 = divpi(acosf(q[2]));
      gamma1 = divpi(acosf(q[3]));
#endif
#if VR_ABLATE & 1
      const float light0 = beta0 + gamma0 + la.w, light1 = beta1 + gamma1 + la.w;
#else
      const float light0 = lut_light(P.lut, la, beta0, gamma0);
      const float light1 = lut_light(P.lut, la, beta1, gamma1);
#endif
      const float rl0 = refl * light0;
      ir = fmaf(rl0 * L0.cr, P.color[0], ir);
      ig = fmaf(rl0 * L0.cg, P.color[1], ig);
      ib = fmaf(rl0 * L0.cb, P.color[2], ib);
      const float rl1 = refl * light1;
      ir = fmaf(rl1 * L1.cr, P.color[0], ir);
      ig = fmaf(rl1 * L1.cg, P.color[1], ig);
      ib = fmaf(rl1 * L1.cb, P.color[2], ib);
    }
    if (i < P.num_lights) {
      const DevLight L = light_at(P, i);
      const f3 lo = mk(L.px - pos.x, L.py - pos.y, L.pz - pos.z);
      const float dlo = dot3(lo, n);
      const f3 lop = mk(fmaf(-dlo, n.x, lo.x), fmaf(-dlo, n.y, lo.y), fmaf(-dlo, n.z, lo.z));
#if VR_ABLATE & 2
      const float beta = dot3(n, lo) * 0.01f, gamma = dot3(lip, lo) * 0.01f + liplen;
#else
      float li_in[2] = {dot3(lo, lo), dot3(lop, lop)}, ln[2];
      sqrt_cr_n<2>(li_in, ln);
      const float num[2] = {dot3(n, lo), dot3(lip, lop)}, den[2] = {nlen * ln[0], liplen * ln[1]};
      float q[2];
      div_acos_n<2>(num, den, q);
      const float beta = divpi(acosf(q[0])), gamma = divpi(acosf(q[1]));
#endif
#if VR_ABLATE & 1
      const float light = beta + gamma + la.w;
#else
      const float light = lut_light(P.lut, la, beta, gamma);
#endif
      const float rl = refl * light;
      ir = fmaf(rl * L.cr, P.color[0], ir);
      ig = fmaf(rl * L.cg, P.color[1], ig);
      ib = fmaf(rl * L.cb, P.color[2], ib);
    }
  }
}

}  // namespace vr
