// vr_march.hip -- the LDS-staged ray-march kernel for gfx950 ("wave slab staging").
//
// Why: a lit sample needs 7 trilinear fetches of the emission volume (centre + 6 gradient taps,
// volumeRender_kernel.cu:212-253, :444) -- 28 paired gathers that each touch ~8 L2 lines for a
// wave of 64 rays.  Measured on MI355X that is L2-request bound (16% L2 misses, 258 GB/frame
// beyond L2 for a 4.3 GB volume, VALU ~20% busy).  Here each wave (an 8x8-pixel tile) marches in
// chunks of S samples: it bounds the stencil footprint of its live rays for the next S samples
// (rays of a tile enter through one axis-aligned box face and advance in lockstep, so the
// footprint is a thin slab), copies that box of the apron-layout volume into its private LDS
// slot with coalesced loads, and takes every emission/gradient tap of the chunk from LDS.
// A tap outside the staged box (or a chunk whose box exceeds the slot) reads global memory
// through exactly the same arithmetic, so the result never depends on the staging.
//
// The per-sample arithmetic is the oracle's (vr_sampling.h).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>
#include <stdlib.h>
#include <algorithm>
#include <type_traits>

#ifndef VR_MARCH_K
#define VR_MARCH_K 1  // depth lanes of this object file (see below)
#endif
#ifndef VR_MERGED_BOUNDS
#define VR_MERGED_BOUNDS 1  // one wave-uniform slot test for the centre and the half-texel taps
#endif
#ifndef VR_WHOLE_BOX
// 1: in a chunk whose whole tap box is staged (not partial; tame waves, not a slab), every tap of
// every sample lies in the box by construction (plan_chunk: the box of all taps of the live rays'
// next S samples, the drift of the rounded position additions in its halo), so the per-sample
// merged slot test is not evaluated.  VR_CHECK_WHOLE=1 (diagnostic build): evaluated anyway, and a
// sample it fails is reported with printf.
#define VR_WHOLE_BOX 1
#endif
#ifndef VR_CHECK_WHOLE
#define VR_CHECK_WHOLE 0
#endif
#ifndef VR_LIGHTS_HOIST
#define VR_LIGHTS_HOIST 1  // tame launches: the first light pair held in registers across the march
#endif
#ifndef VR_REFL_HOIST
#define VR_REFL_HOIST 1  // tame launches: the reflection's single voxel read once per wave (sample_at)
#endif
#ifndef VR_ADAPTIVE_S
#define VR_ADAPTIVE_S 1
#endif
#ifndef VR_WHOLE_SPLIT
#define VR_WHOLE_SPLIT 1  // K > 1: the sample loop compiled twice, for whole chunks and the others
#endif
#ifndef VR_COUNT_K
// 1 (diagnostic builds): the counter variant is also built for K > 1 -- the chunk statistics of the
// production depth lanes (staged / leaped / global chunks, S histogram, wave iterations); its sample
// sums stay the K = 1 variant's (host: VR_COUNT_PROD=1 routes a counted launch here)
#define VR_COUNT_K 0
#endif
#if VR_CHECK_WHOLE
static __device__ unsigned long long vr_whole_violations;  // (diagnostic build) samples the whole-box rule misses
#endif
#ifndef VR_BRANCHFREE_LEAP
#define VR_BRANCHFREE_LEAP 1  // empty-chunk leap of K = 1 lanes without per-step branches
#endif
#ifndef VR_CHUNK_PER_LANE
#define VR_CHUNK_PER_LANE 16  // chunk length per depth lane for K >= 2 (samples per ray per chunk)
#endif
#ifndef VR_CHUNK
// samples per ray per staged chunk: the chunk set-up (box reduction + staging copy) is paid once
// per S / K iterations, so longer chunks for more depth lanes (fewer rays -> thinner boxes)
#define VR_CHUNK (VR_MARCH_K >= 2 ? VR_CHUNK_PER_LANE * VR_MARCH_K : 32)
#endif
// the host's staging halo covers chunks of up to this many sequential position additions
// (vr_capi.hip chunk_samples): a longer chunk could leap over a tap outside its staged box
static_assert(VR_CHUNK <= (VR_MARCH_K >= 2 ? 16 * VR_MARCH_K : 32), "chunk longer than the host's halo margin");

#include "vr_device.h"
#include "vr_sampling.h"
#include "vr_stage.h"

namespace vr {

// Built twice (Makefile): VR_MARCH_FAST=1 -> vr::fast (the default shading),
// VR_MARCH_FAST=0 -> vr::exact (op for op the oracle's).  Everything else is shared.
#ifndef VR_MARCH_FAST
#define VR_MARCH_FAST 1
#endif
#if VR_MARCH_FAST
namespace fast {
#else
namespace exact {
#endif

// Depth lanes: each object file is built for one K = VR_MARCH_K (Makefile).  A wave
// marches 64 / K rays with K lanes per ray; per iteration the K lanes of a ray take its next K
// consecutive samples and then composite them in order.  K = 1 is the plain one-lane-per-ray march.
#define VR_CAT2(a, b) a##b
#define VR_CAT(a, b) VR_CAT2(a, b)

// Value of lane (group base + I) of this lane's K-lane group.  K = 2, 4: one DPP quad_perm move;
// K = 8: ds_swizzle in 32-lane bit mode (and 0x18, or I).
template <int K, int I>
__device__ __forceinline__ float group_lane(float v) {
  if constexpr (K == 1) {
    return v;
  } else if constexpr (K == 2) {  // quad_perm reads lanes of the same quad: no old value needed
    constexpr int ctrl = I | (I << 2) | ((2 + I) << 4) | ((2 + I) << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, true));
  } else if constexpr (K == 4) {
    constexpr int ctrl = I | (I << 2) | (I << 4) | (I << 6);
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), ctrl, 0xf, 0xf, true));
  } else {
    static_assert(K == 8, "depth lanes: K in {1, 2, 4, 8}");
    return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(v), 0x18 | (I << 5)));
  }
}

// Per-lane march state carried across chunks.
struct Ray {
  f3 o, pos, step;
  float t, tfar;
  float sr, sg, sb, sa;
  int32_t nsteps, nlit;
  bool alive;
  bool mine;  // K > 1: this lane's current sample exists (see march)
  bool past;  // slab mode: the ray left this rank's slab still unfinished (the next slab goes on)
};

// Slab mode: the ray's resume point -- the recurrence state (t, pos, sample index) of its next
// sample, the first one this slab does not own -- goes straight to the state planes 5-9 of P.out
// at pixel index kk (registers are the march's limit; a ray hands off once).
__device__ __forceinline__ void store_resume(const RenderParams &P, uint32_t kk, float t, const f3 &pos, int32_t n) {
  const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
  P.out[kk + 5 * plane] = t;
  P.out[kk + 6 * plane] = pos.x;
  P.out[kk + 7 * plane] = pos.y;
  P.out[kk + 8 * plane] = pos.z;
  P.out[kk + 9 * plane] = __int_as_float(n);
}

// K > 1, called by whole groups: (t, p, n) = (t0, p0, n0) of the first lane (in sample order) of
// this lane's group with flagf != 0, in every lane of the group (I descending: the lowest flagged
// lane writes last).
template <int K, int I = K - 1>
__device__ __forceinline__ void first_of_group(float flagf, float t0, const f3 &p0, int32_t n0, float &t, f3 &p,
                                               int32_t &n) {
  if constexpr (I >= 0) {
    const float x = group_lane<K, I>(p0.x), y = group_lane<K, I>(p0.y), z = group_lane<K, I>(p0.z);
    const float tt = group_lane<K, I>(t0);
    const int32_t nn = __float_as_int(group_lane<K, I>(__int_as_float(n0)));
    if (group_lane<K, I>(flagf) != 0.f) {
      t = tt;
      p = mk(x, y, z);
      n = nn;
    }
    first_of_group<K, I - 1>(flagf, t0, p0, n0, t, p, n);
  }
}

struct ChunkStats {
  uint32_t staged, leap, fall, iter, lit, probe, probe_fail;
};

#ifndef VR_CUBE_AXIS
#define VR_CUBE_AXIS 1  // the half-texel tap launch forms its axes as axis_cube_s (2 VALU instead of 4 per axis)
#endif
#ifndef VR_PROBE
#define VR_PROBE 1  // the empty-space probe (vr_stage.h probe_run); 0: staged empty-chunk leaps only
#endif
#ifndef VR_NL2
#define VR_NL2 1  // round 6: the two-light march specialised (march_kernel, shade_fast NL)
#endif
#ifndef VR_PARK
#define VR_PARK 1  // round 6: wave-front alignment of rays far apart along their direction (march)
#endif
#ifndef VR_PARK_SAMPLES
#define VR_PARK_SAMPLES (2 * VR_CHUNK)  // parked: more than this many steps ahead of the wave's hindmost ray
#endif
#ifndef VR_REPROBE_PARTIAL
#define VR_REPROBE_PARTIAL 1  // after a partial chunk the probe runs again before the next chunk
#endif
#ifndef VR_PRELEAP
#define VR_PRELEAP 1  // round 6: per-lane leaps of empty runs before the march of a wave whose rays are far apart
#endif
#ifndef VR_PRELEAP_SPREAD
#define VR_PRELEAP_SPREAD 256  // ... more than this many steps apart (the grazing tiles of rotate(30,10,0): 900-2700)
#endif
#ifndef VR_PROBE_LANES
#define VR_PROBE_LANES 0  // round 6: per-lane probes inside the march loop for waves whose rays are far apart
                          // (vr_stage.h probe_lanes; measured: +0.4 ms metric, +1.2 ms C3 -- VR_PRELEAP instead)
#endif
#ifndef VR_PROBE_BISECT
// 1: a probe that finds data (or too many bricks) retries at half the run length, down to
// VR_PROBE_MIN -- the run stops closer to the data (same box: metric 28.4-28.6 -> 27.5 ms, C2 14.6 ->
// 12.8 ms, P = 8 part 5.27 -> 5.07 ms, r5e)
#define VR_PROBE_BISECT 1
#endif
#ifndef VR_PROBE_MIN
#define VR_PROBE_MIN (2 * VR_CHUNK)  // the probe's first run after the march enters empty space
#endif

// One sample of a ray at position `pos` (volumeRender_kernel.cu:444-474): the emission /
// absorption fetch, opacity, and for a lit, non-empty sample the gradient and the shading.  Returns
// the premultiplied colour (r, g, b) and the opacity; `shaded` says whether shading ran.
template <int MODE, bool AB_ALIAS, bool SHARE2, bool BIG, bool NANCHK, int NL = 0>
__device__ __forceinline__ void sample_at(const RenderParams &P, const float *L, const Box &B, bool staged, bool whole,
                                          const f3 pos, const f3 o, float &r, float &gg, float &b, float &alpha,
                                          bool &shaded, float rv = 0.f, const DevLight *pre = nullptr) {
  const DevTex &E = P.em;
  const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);
  const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
  const float tstep = P.tstep;
  const f3 ps = mk((pos.x - bmin.x) * bsc.x, (pos.y - bmin.y) * bsc.y, (pos.z - bmin.z) * bsc.z);
  // unclamped axes (axis_raw): exact on the LDS path, clamped by fetch_at on the global one.
  // The fast variant's half-texel gradient taps need the raw fraction's half split as well.
  // MODE 1 with SHARE2: the launch is known to take the half-texel taps (P.tap_half; the exact
  // tap code is not compiled in, which frees registers); without it P.tap_half decides per sample.
  constexpr bool HALF_TAPS = VR_MARCH_FAST && MODE == 1;
  constexpr bool HALF_ONLY = HALF_TAPS && SHARE2;
  AxS sx{}, sy{}, sz{};
  Ax ax, ay, az;
  if constexpr (HALF_ONLY && VR_CUBE_AXIS) {
    // the half-texel tap launch is a power-of-two cube (vr_capi.hip half_texel_taps): the
    // coordinate in one add and one fma, bit-identical (vr_sampling.h axis_cube_s)
    sx = axis_cube_s<NANCHK>(pos.x, P.cube_hs[0]);
    sy = axis_cube_s<NANCHK>(pos.y, P.cube_hs[1]);
    sz = axis_cube_s<NANCHK>(pos.z, P.cube_hs[2]);
    ax = Ax{sx.i, sx.w};
    ay = Ax{sy.i, sy.w};
    az = Ax{sz.i, sz.w};
  } else if constexpr (HALF_TAPS) {
    sx = axis_raw_s<NANCHK>(ps.x, E.fnx);
    sy = axis_raw_s<NANCHK>(ps.y, E.fny);
    sz = axis_raw_s<NANCHK>(ps.z, E.fnz);
    ax = Ax{sx.i, sx.w};
    ay = Ax{sy.i, sy.w};
    az = Ax{sz.i, sz.w};
  } else {
    ax = axis_raw<NANCHK>(ps.x, E.fnx);
    ay = axis_raw<NANCHK>(ps.y, E.fny);
    az = axis_raw<NANCHK>(ps.z, E.fnz);
  }
  // centre cell in the slot; the gradient taps below differ from it along one axis only
  const int lx = slot_coord(ax.i, B.rx), ly = slot_coord(ay.i, B.ry), lz = slot_coord(az.i, B.rz);
  // (the per-axis box tests, evaluated where used: only the paths that are not wholly staged need them)
#define inx in_box(lx, B.ex)
#define iny in_box(ly, B.ey)
#define inz in_box(lz, B.ez)
  const int ayz = lz * B.pxy + ly * B.px;  // slot word of (0, ly, lz)
  const int ac = ayz + lx;
  Cell C;  // the centre's partial sums, for the half-texel taps (valid where the centre is staged)
  float em_s;
  // The half-texel taps of every lane in the slot (cells a - 1 .. a + 1 per axis, a = i + hi): then
  // the centre cell is too (a - 1 >= 0 and a + 1 <= e - 2 put i in [0, e - 2]), so one wave-uniform
  // test serves the centre fetch and the gradient, with no per-lane branch on either
  bool full = false;
  if constexpr (HALF_ONLY && VR_MERGED_BOUNDS) {
    if (VR_WHOLE_BOX && !VR_CHECK_WHOLE && whole) {
      full = true;  // (wave-uniform) a whole box: every tap inside by construction
    } else {
      full = __all(staged && (unsigned)(lx + (sx.hi ? 1 : 0) - 1) < (unsigned)(B.ex - 2) &&
                   (unsigned)(ly + (sy.hi ? 1 : 0) - 1) < (unsigned)(B.ey - 2) &&
                   (unsigned)(lz + (sz.hi ? 1 : 0) - 1) < (unsigned)(B.ez - 2));
#if VR_CHECK_WHOLE
      if (whole && !full && __lane_id() == __builtin_amdgcn_readfirstlane(__lane_id())) {
        const unsigned long long c = atomicAdd(&vr_whole_violations, 1ull);
        if (c < 8 || c % 100000 == 0)
          printf("VR_CHECK_WHOLE: whole box misses a tap (#%llu): cell %d %d %d box %d %d %d + %d %d %d\n", c, ax.i,
                 ay.i, az.i, B.rx, B.ry, B.rz, B.ex, B.ey, B.ez);
      }
#endif
    }
  }
  if constexpr (HALF_TAPS) {
    if (full) em_s = lds_tri_cell(L, B, ac, ax.w, ay.w, az.w, C);
    else if (staged && inx && iny && inz) em_s = lds_tri_cell(L, B, ac, ax.w, ay.w, az.w, C);
    else {
      const DevTex U = reload(E);
      em_s = fetch<BIG>(U, clamp_ax(ax, U.nx), clamp_ax(ay, U.ny), clamp_ax(az, U.nz));
    }
  } else {
    em_s = fetch_at<BIG>(E, L, B, staged && inx && iny && inz, ac, ax, ay, az);
  }
  const float ab_s = AB_ALIAS ? em_s : tex3d<BIG>(P.ab, ps.x, ps.y, ps.z);
  const float e = P.fe * em_s;
  const float a = P.fa * ab_s;
  // NANCHK = false is the tame fast path (march_kernel: finite rays of a launch with P.tame): every
  // launch-wide test below was decided by the host (vr_capi.hip), so none of them holds a uniform
  // mask in SGPRs across the sample loop (such masks spill to VGPR lanes and cost a v_readlane pair
  // per use)
  constexpr bool TAME = !NANCHK;
  if constexpr (TAME) alpha = opacity<VR_MARCH_FAST>(a, tstep, true);
  else alpha = P.small_x ? opacity<VR_MARCH_FAST>(a, tstep, true) : opacity<VR_MARCH_FAST>(a, tstep);
  const float eds = e * tstep;
  float ir = 0.f, ig = 0.f, ib = 0.f;
  const bool skip = TAME ? alpha == 0.f : (P.skip_empty && alpha == 0.f && (P.eds_finite || fabsf(eds) <= 3.0e38f));
  shaded = MODE != 0 && !skip;
  if (MODE != 0 && !skip) {
    f3 g;
    if ((MODE == 1 && (VR_ABLATE & 4)) || (MODE == 2 && (VR_ABLATE & 32))) {  // diagnostics: no gradient fetch
      g = mk(ps.x, ps.y, em_s);
    } else if (HALF_TAPS && (HALF_ONLY || P.tap_half) &&
               (full || __all(staged && (unsigned)(lx + (sx.hi ? 1 : 0) - 1) < (unsigned)(B.ex - 2) &&
                     (unsigned)(ly + (sy.hi ? 1 : 0) - 1) < (unsigned)(B.ey - 2) &&
                     (unsigned)(lz + (sz.hi ? 1 : 0) - 1) < (unsigned)(B.ez - 2)))) {
      // every shading lane's taps lie in the staged box (the tap cells a - 1 .. a + 1 per axis,
      // a = i + hi): the taps from the slot with their shared voxels and partial sums
      // unhalved: the fast shading uses g only through n = -g * rsq(g.g), which the exact factor 2
      // leaves bit-identical (4x scales g.g by a power of two; rsq halves exactly)
      g = half_grad_lds(L, B, ac, sx, sy, sz, ax.w, ay.w, az.w, C);
    } else if (HALF_TAPS && (HALF_ONLY || P.tap_half)) {
      // fast variant, gradient offset of exactly half a texel on every axis (a power-of-two cube,
      // vr_capi.hip half_texel_taps): each axis' two taps derived from the centre's (half_taps);
      // in the slot the plus tap's cell is the centre's, or the next one along the axis, and the
      // minus tap's lies one row / plane below it
      const bool syz = staged && iny && inz, sxz = staged && inx && inz, sxy = staged && inx && iny;
      Ax p, m;
      half_taps(sx, p, m);
      int l = lx + (sx.hi ? 1 : 0);
      int a = ac + (sx.hi ? 1 : 0);
      g.x = fetch_at<BIG>(E, L, B, syz && in_box(l, B.ex), a, p, ay, az) -
            fetch_at<BIG>(E, L, B, syz && in_box(l - 1, B.ex), a - 1, m, ay, az);
      half_taps(sy, p, m);
      l = ly + (sy.hi ? 1 : 0);
      a = ac + (sy.hi ? B.px : 0);
      g.y = fetch_at<BIG>(E, L, B, sxz && in_box(l, B.ey), a, ax, p, az) -
            fetch_at<BIG>(E, L, B, sxz && in_box(l - 1, B.ey), a - B.px, ax, m, az);
      half_taps(sz, p, m);
      l = lz + (sz.hi ? 1 : 0);
      a = ac + (sz.hi ? B.pxy : 0);
      g.z = fetch_at<BIG>(E, L, B, sxy && in_box(l, B.ez), a, ax, ay, p) -
            fetch_at<BIG>(E, L, B, sxy && in_box(l - 1, B.ez), a - B.pxy, ax, ay, m);  // unhalved, as above
    } else if (MODE == 1) {  // computeGradient on tex_emission (gem == em), world offsets +-gstep
      const float xp = ((pos.x + P.gstep[0]) - bmin.x) * bsc.x;
      const float xm = ((pos.x - P.gstep[0]) - bmin.x) * bsc.x;
      const float yp = ((pos.y + P.gstep[1]) - bmin.y) * bsc.y;
      const float ym = ((pos.y - P.gstep[1]) - bmin.y) * bsc.y;
      const float zp = ((pos.z + P.gstep[2]) - bmin.z) * bsc.z;
      const float zm = ((pos.z - P.gstep[2]) - bmin.z) * bsc.z;
      const bool syz = staged && iny && inz, sxz = staged && inx && inz, sxy = staged && inx && iny;
      const Ax axp = axis_raw<NANCHK>(xp, E.fnx), axm = axis_raw<NANCHK>(xm, E.fnx);
      const int lxp = slot_coord(axp.i, B.rx), lxm = slot_coord(axm.i, B.rx);
      g.x = fetch_at<BIG>(E, L, B, syz && in_box(lxp, B.ex), ayz + lxp, axp, ay, az) -
            fetch_at<BIG>(E, L, B, syz && in_box(lxm, B.ex), ayz + lxm, axm, ay, az);
      const Ax ayp = axis_raw<NANCHK>(yp, E.fny), aym = axis_raw<NANCHK>(ym, E.fny);
      const int lyp = slot_coord(ayp.i, B.ry), lym = slot_coord(aym.i, B.ry);
      const int axz = lz * B.pxy + lx;
      g.y = fetch_at<BIG>(E, L, B, sxz && in_box(lyp, B.ey), axz + lyp * B.px, ax, ayp, az) -
            fetch_at<BIG>(E, L, B, sxz && in_box(lym, B.ey), axz + lym * B.px, ax, aym, az);
      const Ax azp = axis_raw<NANCHK>(zp, E.fnz), azm = axis_raw<NANCHK>(zm, E.fnz);
      const int lzp = slot_coord(azp.i, B.rz), lzm = slot_coord(azm.i, B.rz);
      const int axy = ly * B.px + lx;
      g.z = fetch_at<BIG>(E, L, B, sxy && in_box(lzp, B.ez), axy + lzp * B.pxy, ax, ay, azp) -
            fetch_at<BIG>(E, L, B, sxy && in_box(lzm, B.ez), axy + lzm * B.pxy, ax, ay, azm);
      g = mk(g.x * 0.5f, g.y * 0.5f, g.z * 0.5f);
    } else if (MODE == 2 && SHARE2) {
      const Ax cx = clamp_ax(ax, E.nx), cy = clamp_ax(ay, E.ny), cz = clamp_ax(az, E.nz);
      if (P.gvec)
        g = fetch_vec<BIG>(P.gvec, P.gx, P.gv_row8, P.gv_plane8, cx, cy, cz);
      else
        g = mk(fetch<BIG>(P.gx, cx, cy, cz), fetch<BIG>(P.gy, cx, cy, cz), fetch<BIG>(P.gz, cx, cy, cz));
    } else {
      g = mk(tex3d<BIG>(P.gx, ps.x, ps.y, ps.z), tex3d<BIG>(P.gy, ps.x, ps.y, ps.z),
             tex3d<BIG>(P.gz, ps.x, ps.y, ps.z));
    }
    float refl;
    if constexpr (TAME) {  // the emission sample or the single voxel, selected by a 32-bit mask (v_bfi)
      // VR_REFL_HOIST: the single voxel loaded once per wave before the march (rv), not per sample
      const float v = VR_REFL_HOIST ? rv : voxel0(P.re.p);
      const uint32_t m = P.re_mask;
      refl = P.fr * __uint_as_float((__float_as_uint(em_s) & m) | (__float_as_uint(fmaf(0.5f, v - v, v)) & ~m));
    } else {
      refl = P.fr * (P.re_is_em ? em_s : tex3d<BIG>(P.re, ps.x, ps.y, ps.z));
    }
    shade_lights<VR_MARCH_FAST, TAME, NL>(P, g, pos, o, refl, ir, ig, ib, pre);
  }
  r = fmaf(eds, P.color[0], ir) * alpha;
  gg = fmaf(eds, P.color[1], ig) * alpha;
  b = fmaf(eds, P.color[2], ib) * alpha;
#undef inx
#undef iny
#undef inz
}

// Front-to-back compositing of one sample and the march recurrences of volumeRender_kernel.cu:
// 476-492, in the reference's order: early exit on sum.a > thr before t > tfar; pos += step only
// while the ray goes on.
// thr / cap: the exit threshold and the sample cap (P.thr / P.max_steps).
__device__ __forceinline__ void composite(const RenderParams &P, Ray &R, float r, float gg, float b, float alpha,
                                          float thr, int cap) {
  const float om = 1.f - R.sa;
  R.sr = fmaf(om, r, R.sr);
  R.sg = fmaf(om, gg, R.sg);
  R.sb = fmaf(om, b, R.sb);
  R.sa = fmaf(om, alpha, R.sa);
  ++R.nsteps;
  if (R.sa > thr || R.nsteps >= cap) {
    R.alive = false;
  } else {
    R.t += P.tstep;
    if (R.t > R.tfar) R.alive = false;
    else R.pos = mk(R.pos.x + R.step.x, R.pos.y + R.step.y, R.pos.z + R.step.z);
  }
}

// Whether any lane of this lane's K-lane group has b set (called by whole groups).  K = 2, 4: DPP
// quad_perm swaps within the group (no 64-bit ballot arithmetic); K = 8: the ballot.
#ifndef VR_GROUP_ANY_DPP
#define VR_GROUP_ANY_DPP 1
#endif
template <int K>
__device__ __forceinline__ bool group_any(bool b) {
  if constexpr ((K == 2 || K == 4) && VR_GROUP_ANY_DPP) {
    int v = b ? 1 : 0;
    v |= __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, true);  // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (K == 4) v |= __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, true);  // [2,3,0,1]: lane ^ 2
    return v != 0;
  } else {
    const uint64_t m = __ballot(b);
    const int base = (int)(__lane_id() & ~(uint32_t)(K - 1));
    return ((m >> base) & ((1ull << K) - 1)) != 0ull;
  }
}

// The largest v over this lane's K-lane group (called by whole groups): acc = v to start.
template <int K, int I = 0>
__device__ __forceinline__ int group_max_i(int v, int acc) {
  if constexpr (K == 1 || I == K) {
    return acc;
  } else {
    return group_max_i<K, I + 1>(v, max(acc, __float_as_int(group_lane<K, I>(__int_as_float(v)))));
  }
}

// Composite the existing samples (a prefix of the K; exf = 1 where this lane's sample exists) of a
// depth-lane group in order, every lane of the group alike; the ray stops at the first sum.a > thr
// (volumeRender_kernel.cu:482).
// ZF (tame waves): a missing sample is composited as its zeros, without the existence test -- an
// exact no-op there: fma(1 - sum.a, 0, s) = s for the finite sums of a tame launch (never -0: they
// start at +0 and an exact zero sum rounds to +0), and the exit test sees the unchanged sum.a,
// which a live ray has already passed.  Saves the broadcast and test of exf per group lane.
#ifndef VR_ZERO_FILL
#define VR_ZERO_FILL 1
#endif
template <int K, int I, bool ZF = false>
__device__ __forceinline__ void composite_group(const RenderParams &P, Ray &R, float exf, float r, float gg, float b,
                                                float alpha, float thr) {
  if constexpr (I < K) {
    const float ri = group_lane<K, I>(r), gi = group_lane<K, I>(gg), bi = group_lane<K, I>(b),
                ai = group_lane<K, I>(alpha);
    // sample I of the group exists iff group lane I's does (the existing samples are a prefix)
    if ((ZF || group_lane<K, I>(exf) != 0.f) && R.alive) {
      const float om = 1.f - R.sa;
      R.sr = fmaf(om, ri, R.sr);
      R.sg = fmaf(om, gi, R.sg);
      R.sb = fmaf(om, bi, R.sb);
      R.sa = fmaf(om, ai, R.sa);
      if (R.sa > thr) R.alive = false;
    }
    composite_group<K, I + 1, ZF>(P, R, exf, r, gg, b, alpha, thr);
  }
}

// The chunked march of one wave.  NANCHK = false when every live ray of the wave has a finite
// start position and step: all volume coordinates are then finite and the NaN -> 0 substitution
// of the sampler is skipped (the LUT coordinates, which are NaN for a zero gradient, keep it).
// MODE 0: no lights; 1: on-the-fly gradient from the staged emission texture (gem == em);
// 2: lookup gradient (gx/gy/gz from global memory, at the centre's axes when SHARE2).
// K > 1 (depth lanes): lane `sub` of a ray's group owns samples sub, sub + K, sub + 2K, ...: its
// pos / t / nsteps (= sample index) follow the reference's recurrence from the ray start (sub
// steps, then K per iteration: the same sequence of rounded additions as one lane taking every
// sample), and `mine` says whether its sample exists (t <= tfar and index < max_steps; t is
// non-decreasing, so the existing samples of a group are a prefix).  Per iteration each lane
// takes its sample, then every lane composites the group's samples in order; `alive` (the ray:
// not stopped by sum.a > thr and some sample left) is the same in all K lanes.  Bit-identical to
// K = 1; samples after an early exit are computed and discarded.
// SLAB (sort-last bricks): the emission texture holds planes of one z-slab of a
// larger volume, and only the samples this slab owns (slab_z0 <= p.z < slab_z1 in normalized
// coordinates) are fetched and composited.  A ray arrives with the recurrence state of its next
// sample (the resume point the previous slab handed off, or its start); samples before the slab
// (only when a sweep does not begin at an end slab) replay the recurrences, so every owned sample
// has the position, t and step count of the one-volume march.  A ray stops here when it
// terminates, or at its first sample beyond the slab in its direction of travel (`past`), whose
// state becomes the resume point (store_resume).
// NL: the launch's light count if the kernel is specialised on it (2; sample_at / shade_fast), else 0.
template <int K, int MODE, bool AB_ALIAS, bool COUNT, bool SHARE2, bool BIG, bool NANCHK, int CAP, bool SLAB = false,
          int NL = 0>
__device__ __forceinline__ void march(const RenderParams &P, float *L, int lane, Ray &R, ChunkStats &C,
                                      uint32_t kk = 0, KParams kp = nullptr, uint32_t gw = 0) {
  static_assert(!COUNT || K == 1 || VR_COUNT_K, "the counter variant is built for K = 1 only (VR_COUNT_K: all K)");
  static_assert(!SLAB || (!COUNT && BIG), "slab mode: no counters, 64-bit addressing");
  const int cap = P.max_steps;
  const float thr = P.thr;
  const float sbz = P.bmin[2], ssz = P.bscale[2];
  // slab mode: the ray has left the slab in its direction of travel (normalized z of its sample)
  auto beyond = [&](float zn) { return R.step.z >= 0.f ? zn >= P.slab_z1 : zn < P.slab_z0; };
  const DevTex &E = P.em;
  const int sub = lane & (K - 1);
  if constexpr (K > 1) {  // R.nsteps: 0, or the resume point's index (slab mode)
    R.mine = R.alive;
    leap(P, sub, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);  // to this lane's first sample
    R.alive = group_any<K>(R.mine);
  }

  // VR_ADAPTIVE_S: the first box attempt of a chunk is twice the length the wave's last chunk
  // staged (its box grows little from one chunk to the next), and the shortest after a partial box,
  // instead of always VR_CHUNK halved until it fits: fewer box reductions per chunk.  The samples
  // are the same whatever the chunk length (the staging never changes a result).
  int s0 = VR_CHUNK;
  // Empty-space probe (vr_stage.h probe_run; tame waves, absorption = emission, not the slab march):
  // ps > 0 -- the next probe's run length (doubled after each empty run, up to VR_PROBE_MAX); 0 --
  // off (a probe found data: the staged chunks go on until they find data themselves); -1 -- armed
  // (a chunk found data; the next empty chunk restarts the probe at VR_PROBE_MIN).  Rays start in
  // front of the data, so the probe starts on.
  constexpr bool PROBE = VR_PROBE && !NANCHK && AB_ALIAS && !SLAB;
  int ps = VR_PROBE_MIN;
  // the tame reflection's single voxel (sample_at), held in a register across the march: an opaque
  // copy, so that the compiler does not re-issue the invariant load in every sample
  float rv = 0.f;
  if constexpr (!NANCHK && VR_REFL_HOIST) {
    if (P.tame && P.re.p) rv = voxel0(P.re.p);
    asm volatile("" : "+v"(rv));
  }
  // VR_LIGHTS_HOIST: the first light pair likewise (shade_fast), when the frame has two or more
  DevLight pre2[2];
  const DevLight *pre = nullptr;
  // (only where the registers fit without lowering occupancy or spilling: not K = 1, the slab or
  // counter variants, nor the 64-bit, separate-absorption or full-gradient-tap ones)
  if constexpr (!NANCHK && VR_LIGHTS_HOIST && MODE != 0 && K > 1 && AB_ALIAS && SHARE2 && !BIG && !SLAB && !COUNT) {
    // (NL = 1: the single light in pre2[0])
    const bool two = NL == 2 || (NL == 0 && P.num_lights >= 2);
    for (int j = 0; j < 2; ++j) {
      pre2[j] = (two || (NL == 1 && j == 0)) ? light_at(P, j) : DevLight{0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      asm volatile("" : "+v"(pre2[j].px), "+v"(pre2[j].py), "+v"(pre2[j].pz), "+v"(pre2[j].cr), "+v"(pre2[j].cg),
                   "+v"(pre2[j].cb));
    }
    if (two || NL == 1) pre = pre2;
  }
  // the recurrences of n samples whose every sample adds exactly nothing (an empty-chunk leap or an
  // empty probe run); tame waves: one exit test after the n additions (advance_n; t only grows)
  auto leap_run = [&](int n) __attribute__((always_inline)) {
    if constexpr (K == 1) {
      if (COUNT || !VR_BRANCHFREE_LEAP) leap(P, n, R.alive, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);  // exact counts
      else if constexpr (!NANCHK) advance_n(P, n, R.alive, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
      else advance(P, n, R.alive, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
    } else {
      if constexpr (!NANCHK) advance_n(P, n, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
      else advance(P, n, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
      R.alive = R.alive && group_any<K>(R.mine);
    }
  };
  // the state a pre-leap launch left for this wave (preleap_kernel), if any: the rays start there
  if constexpr (PROBE && VR_PRELEAP && !COUNT) {
    if (kp != nullptr) {
      const KParams kq = kparams_fresh(kp);
      if (kq->pre_flag != nullptr) {
        const uint32_t f = __builtin_amdgcn_readfirstlane(kq->pre_flag[gw]);
        if (__builtin_expect(f != 0u, 0)) {
          const float4 *st = kq->pre_state + ((size_t)(f - 1u) * 64u + (uint32_t)lane) * 2u;
          const float4 a = st[0], b = st[1];
          R.t = a.x;
          R.pos = mk(a.y, a.z, a.w);
          R.nsteps = __float_as_int(b.x);
          const int fl = __float_as_int(b.y);
          R.alive = (fl & 1) != 0;
          R.mine = (fl & 2) != 0;
        }
      }
    }
  }
  while (__any(R.alive)) {
    if constexpr (PROBE) {
      if (ps > 0 && kp != nullptr && kparams_fresh(kp)->occ != nullptr) {
        const bool live = K > 1 ? (R.alive && R.mine) : R.alive;
        // a box of too many bricks (the wave's rays far apart): each lane's own run (probe_lanes)
        auto probe = [&](int len) __attribute__((always_inline)) {
          const int r = probe_run(P, kp, live, R.pos, R.step, R.t, R.tfar, len, lane);
          return (VR_PROBE_LANES && r < 0) ? probe_lanes(P, kp, live, R.pos, R.step, R.t, R.tfar, len) : r;
        };
        int e = probe(ps);
        // an occupied (or too large) box: runs half as long until one is empty or the shortest fails
        while (VR_PROBE_BISECT && e <= 0 && ps > VR_PROBE_MIN) {
          ps >>= 1;
          e = probe(ps);
        }
        if (e > 0) {
          if (COUNT) ++C.probe;
          leap_run(ps);
          ps = min(2 * ps, (int)VR_PROBE_MAX);
          continue;
        }
        if (COUNT) ++C.probe_fail;
        ps = 0;
      }
    }
    // ---- chunk set-up: the box of every tap the live rays take in the next S samples --------
    int S;
    bool staged, partial;
    Box B;
    int box_vol = 0;
    bool edge = true;  // the box is clamped at a volume face (set by plan_chunk when it stages a whole box)
    plan_chunk<CAP>(P, K > 1 ? (R.alive && R.mine) : R.alive, R.pos, R.step, R.t, R.tfar, S, staged, partial, B,
                    COUNT ? &box_vol : nullptr, &edge, s0);
    // Wave-front alignment (round 6): when the chunk's box does not fit whole, the rays may be far
    // apart along their direction rather than across it -- a tile whose rays enter the volume through
    // a face at a grazing angle, or across an edge of the box, starts them up to hundreds of texels
    // apart at the same sample index (45 texels at rotate(125,61,0), 420 at rotate(30,10,0)), and
    // their chunks stage partially and gather from global memory.  All rays share the eye, so t is
    // each ray's distance from it: the rays more than VR_PARK_SAMPLES steps ahead of the wave's
    // hindmost are parked for this chunk (no box, no samples, no recurrence), and the box is planned
    // for the others.  A parked ray's samples are taken later, by the same recurrence, so the image
    // is the same; the hindmost ray always advances, so every ray finishes.
    // (a parked ray's mark is the sign of its t -- t >= 0 otherwise -- so that nothing per lane is
    // held across the sample loop; it has alive = false meanwhile, and every lane of a parked ray's
    // group is parked, so no group operation of the chunk reads it)
    bool parked_any = false;  // wave-uniform
    if constexpr (VR_PARK && !SLAB && !NANCHK) {
      if (!staged || partial) {
        const bool lv = K > 1 ? (R.alive && R.mine) : R.alive;
        // (t >= 0 for every ray: its float bits order as integers)
        const int tmin = wave_min(lv ? __float_as_int(R.t) : 0x7f7fffff);
        bool pk = lv && R.t > __int_as_float(tmin) + (float)VR_PARK_SAMPLES * P.tstep;
        if constexpr (K > 1) pk = group_any<K>(pk);  // (a ray's K lanes together)
        if (__any(pk)) {
          parked_any = true;
          if (pk) {
            R.alive = false;
            R.t = -R.t;
          }
          plan_chunk<CAP>(P, K > 1 ? (R.alive && R.mine) : R.alive, R.pos, R.step, R.t, R.tfar, S, staged, partial,
                          B, COUNT ? &box_vol : nullptr, &edge, s0);
        }
      }
    }
    auto unpark = [&]() __attribute__((always_inline)) {
      if (parked_any && __float_as_int(R.t) < 0) {  // (-0 too)
        R.t = -R.t;
        R.alive = true;
      }
    };
    if (VR_ADAPTIVE_S)
      s0 = (staged && !partial) ? min(2 * S, (int)VR_CHUNK) : (int)(VR_CHUNK >> (VR_ATTEMPTS - 1));
    bool inside = true;  // slab mode: every sample of this chunk lies in the slab
    if constexpr (SLAB) {
      // a chunk none of whose samples this slab owns is not staged: its samples only replay the
      // recurrences (before the slab) or hand the ray off at the first one beyond it, sample by
      // sample, so the resume point is exact
      bool own = false, in = true;
      if (R.alive) {
        const float zs = (R.pos.z - sbz) * ssz;
        const float ze = (fmaf(R.step.z, (float)(S - 1), R.pos.z) - sbz) * ssz;
        own = fmaxf(zs, ze) + P.slab_margin >= P.slab_z0 && fminf(zs, ze) - P.slab_margin < P.slab_z1;
        in = fminf(zs, ze) - P.slab_margin >= P.slab_z0 && fmaxf(zs, ze) + P.slab_margin < P.slab_z1;
      }
      if (!__any(own)) staged = false;
      inside = __all(in);  // every sample of the chunk is owned: no per-sample test
      // only this slab's planes are resident: clamp the staged box to them (the owned samples'
      // taps lie inside; the others are not fetched)
      const int z_lo = max(B.rz, P.slab_pk0), z_hi = min(B.rz + B.ez, P.slab_pk1);
      if (staged) {
        if (z_hi - z_lo < 3) {  // (the half-texel tap test assumes boxes of >= 3 planes)
          staged = false;
        } else {
          B.rz = z_lo;
          B.ez = z_hi - z_lo;
        }
      }
    }
    if (COUNT && lane == 0) {  // diagnostics: box volume of partial/failed chunks, S of staged ones
      if (!staged || partial) atomicAdd(P.steps + 8 + min(box_vol >> 8, 31), 1ull);
      else atomicAdd(P.steps + 40 + (S >= 32 ? 0 : (S >= 16 ? 1 : (S >= 8 ? 2 : 3))), 1ull);
      if (staged) atomicAdd(P.steps + 45, (unsigned long long)(B.pxy * B.ez));  // staging volume (floats)
    }
    bool empty = false;
    if (staged) {
      const bool nonzero = stage_box<BIG>(L, E, B, lane);  // always stage: the samples read the slot
      // leap only when the absorption texture is the staged one: a zero emission box says nothing
      // about the opacity of a separate absorption texture (the simEmAb slot path)
      // slab mode: only a chunk wholly inside the slab (a leap must not carry a ray past its hand-off
      // sample: the samples beyond are the next slab's, and its data is not in this box)
      empty = AB_ALIAS && P.skip_empty && !partial && !nonzero && (!SLAB || inside);
    }
    __builtin_amdgcn_wave_barrier();
    if (COUNT) ++(staged && !partial ? (empty ? C.leap : C.staged) : C.fall);
    // wave-uniform (sample_at: VR_WHOLE_BOX), held as one scalar rather than a lane mask
    const bool whole = __builtin_amdgcn_readfirstlane((!NANCHK && !SLAB && staged && !partial && !edge) ? 1 : 0) != 0;

    if (empty) {
      // (the leap's additions are unconditional: not on a parked ray)
      if (!parked_any) leap_run(S);
      else if (__float_as_int(R.t) >= 0) leap_run(S);
      unpark();
      if (PROBE && ps < 0) ps = VR_PROBE_MIN;  // back in empty space after data: probe again
      continue;
    }
    // data: armed; after a partial chunk (rays far apart, no chunk of theirs can be found empty by
    // staging) the probe runs again before the next chunk -- one probe costs far less than a chunk of
    // global gathers (VR_PROBE_LANES)
    if (PROBE) ps = (VR_PROBE_LANES && VR_REPROBE_PARTIAL && partial) ? (int)VR_PROBE_MIN : -1;

    // ---- S samples ---------------------------------------------------------------------------
    if constexpr (K == 1) {
      for (int k = 0; k < S && R.alive; ++k) {
        if (SLAB && !inside) {
          const float zn = (R.pos.z - sbz) * ssz;  // the sampler's own p.z
          if (!(zn >= P.slab_z0 && zn < P.slab_z1)) {
            if (beyond(zn)) {  // this sample is the next slab's first
              store_resume(P, kk, R.t, R.pos, R.nsteps);
              R.alive = false;
              R.past = true;
            } else {  // before the slab: the recurrences of one sample (composite without colour)
              ++R.nsteps;
              if (R.nsteps >= P.max_steps) {
                R.alive = false;
              } else {
                R.t += P.tstep;
                if (R.t > R.tfar) R.alive = false;
                else R.pos = mk(R.pos.x + R.step.x, R.pos.y + R.step.y, R.pos.z + R.step.z);
              }
            }
            continue;
          }
        }
        float r, gg, b, alpha;
        bool shaded;
        sample_at<MODE, AB_ALIAS, SHARE2, BIG, NANCHK, NL>(P, L, B, staged, whole, R.pos, R.o, r, gg, b, alpha, shaded,
                                                       rv, pre);
        if (COUNT) {
          ++C.iter;
          C.lit += (MODE != 0 && __any(shaded)) ? 1u : 0u;
          R.nlit += shaded ? 1 : 0;
        }
        composite(P, R, r, gg, b, alpha, thr, cap);
      }
    } else {
      // WC: the chunk's box is whole (sample_at skips its slot test); a separate copy of the loop,
      // so that the test and its flag are not carried through the samples of a whole chunk
      auto samples = [&](auto wc) {
      constexpr bool WC = decltype(wc)::value;
      for (int k = 0; k < S && R.alive; k += K) {
        float r = 0.f, gg = 0.f, b = 0.f, alpha = 0.f;
        bool ex = R.mine, take = R.mine;
        if (SLAB && !inside) {
          // a sample beyond the slab ends the ray here (beyond is monotone along the ray, so the
          // group's existing samples stay a prefix); one before it adds exactly nothing (colour 0,
          // opacity 0: the sums and the exit test are unchanged)
          const float zn = (R.pos.z - sbz) * ssz;
          if (ex && beyond(zn)) ex = false;
          take = ex && zn >= P.slab_z0 && zn < P.slab_z1;
        }
        bool shaded = false;
        if (take) {
          sample_at<MODE, AB_ALIAS, SHARE2, BIG, NANCHK, NL>(P, L, B, staged, WC || (!VR_WHOLE_SPLIT && whole), R.pos,
                                                         R.o, r, gg, b, alpha, shaded, rv, pre);
        }
        if (COUNT) {
          ++C.iter;
          C.lit += (MODE != 0 && __any(shaded)) ? 1u : 0u;
        }
        composite_group<K, 0, VR_ZERO_FILL && !NANCHK && !SLAB>(P, R, ex ? 1.f : 0.f, r, gg, b, alpha, thr);
        if (SLAB && !inside) {
          if (R.alive && group_any<K>(R.mine && !ex)) {  // left the slab still unfinished
            // the next slab resumes at the group's first sample beyond this one (samples of a
            // group are in lane order: the first flagged lane of the group stores it)
            float t = R.t;
            f3 p = R.pos;
            int32_t n = R.nsteps;
            first_of_group<K>((R.mine && !ex) ? 1.f : 0.f, R.t, R.pos, R.nsteps, t, p, n);
            if (sub == 0) store_resume(P, kk, t, p, n);  // one store per pixel, from lane 0 as the others
            R.alive = false;
            R.past = true;
          }
        }
        if constexpr (!NANCHK && !SLAB)  // tame: t is non-decreasing (tstep > 0), one test after K steps
          advance_k<K>(P, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
        else
          advance(P, K, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);  // to sample + K
        R.alive = R.alive && group_any<K>(R.mine);
      }
      };
      // (only the half-texel tap launch has the slot test that a whole chunk skips, sample_at)
      if constexpr (VR_WHOLE_SPLIT && !NANCHK && !SLAB && VR_MARCH_FAST && MODE == 1 && SHARE2) {
        if (whole) samples(std::true_type{});
        else samples(std::false_type{});
      } else {
        samples(std::false_type{});
      }
    }
    unpark();
    __builtin_amdgcn_wave_barrier();
  }
}

__device__ __forceinline__ bool finite3(const f3 &v) {
  return fabsf(v.x) <= 3.4e38f && fabsf(v.y) <= 3.4e38f && fabsf(v.z) <= 3.4e38f;
}

// Occupancy of the march: 6.5 KiB wave slots (1664 floats, the largest for which six 4-wave
// workgroups fit the 160 KiB LDS at its allocation granularity) fit 6 workgroups (24 waves) per
// CU, which 80 VGPRs allow (6 waves per SIMD; ~2 VGPRs spill).  Measured on MI355X: the metric
// frame 43.8 ms (10 KiB, 16 waves) -> 42.6 (6 KiB) -> 41.2 (6.5 KiB; 1704 floats: 5 workgroups,
// 41.9) at K = 2.  A scheduled launch (few rounds, heavy waves first) keeps the uncapped allocation: its
// longest waves share a SIMD with fewer others (one rank's share at P = 8: 7.2 ms vs 7.7 capped).
// Round 3, after the whole-box changes (fewer instructions between the loads a wave waits for): 5
// waves per SIMD with a 96-VGPR budget (no spills) beat 6 with 80 -- same box, three rounds,
// 31.25-31.40 vs 31.64-31.90 ms; 5 waves with 7.9 KiB slots (2016 floats) 31.42-31.54 (r3bg).
#ifndef VR_MARCH_MIN_EU
#define VR_MARCH_MIN_EU 5
#endif
#ifndef VR_SCHED1_MIN_EU
#define VR_SCHED1_MIN_EU 1  // a short (scheduled) launch's occupancy cap (A/B; 1: uncapped registers)
#endif
constexpr int march_min_eu(int cap, int sched) {
  return cap <= VR_LDS_CAP_MARCH ? (sched != 1 ? VR_MARCH_MIN_EU : VR_SCHED1_MIN_EU) : 1;
}
#ifndef VR_WG_WAVES
#define VR_WG_WAVES 4  // waves per workgroup: a 16x16 block stays on one XCD (1 wave: same speed, 2x HBM traffic)
#endif

// One wave marches one tile of 64 / K rays (K = 1: 8x8 pixels, 2: 4x8, 4: 4x4, 8: 2x4; lane ->
// ray lane / K, ray -> (x = ray / th, y = ray % th)).  Tile t is quadrant (t & 3) of block
// (t >> 2), a block being 2x2 tiles (16x16 pixels at K = 1), blocks row-major,
// t = blockIdx.x * VR_WG_WAVES + wave.
template <int K>
struct TileShape {
  static constexpr int LR = (K == 1 ? 6 : K == 2 ? 5 : K == 4 ? 4 : 3);  // log2 rays per wave
  static constexpr int LK = 6 - LR;                                         // log2 K
#ifndef VR_TILE_WLOG
#define VR_TILE_WLOG -1  // log2 tile width override (A/B; -1: square-ish, the taller for odd LR)
#endif
  static constexpr int LW = (VR_TILE_WLOG >= 0 && VR_TILE_WLOG <= LR) ? VR_TILE_WLOG : LR / 2;
  static constexpr int TW = 1 << LW, TH = 1 << (LR - LW);  // tile width, height
};

// XCD runs: the dispatcher deals workgroup b to XCD b % 8, so row-major blocks b and b + 1 land on
// different XCDs (and L2s).  With run R > 1, full groups of 8R workgroups are renumbered so that
// XCD x takes R consecutive blocks of the group (g * 8R + x * R + j, j-th of its turns); the tail
// keeps dispatch order.  A bijection of the grid: the image is the same for any R.
__device__ __forceinline__ uint32_t xcd_block(uint32_t b, uint32_t n, int run) {
  if (run <= 1) return b;
  const uint32_t R = (uint32_t)run, gs = 8u * R, g = b / gs;
  if ((g + 1) * gs > n) return b;
  const uint32_t r = b - g * gs;
  return g * gs + (r & 7u) * R + (r >> 3);
}

// SCHED: the launch follows P.wg_order and records each block's duration in P.wg_cost (separate
// instantiations: the hooks cost when compiled in, even unused).  SCHED 1: a short launch (few
// rounds; uncapped registers, its longest waves share a SIMD with few others); 2: a full frame
// (the occupancy cap of the unscheduled kernel); 3: a full frame following the order without
// recording durations.  (Round 4: two chord-split schedules, SCHED 4 / 5, measured slower and
// removed in round 5 -- DESIGN.md s8, s9.)
// SCHED 4 (round 5, fused stereo with paired tiles, P.pair_shift > 0; DESIGN.md s9 "shared reads"):
// each wave marches half a tile of each eye -- the right eye's rays of columns c .. c + TW - 1 and
// the left eye's of columns c + pair_shift .., the shift chosen so that the two bundles converge at
// the volume's centre -- so that one staged box (the union of the two bundles' footprints) serves
// both eyes.  Columns are counted on a virtual image of part_cols + pair_shift columns: the left
// eye's pixel at virtual column xv, the right eye's at xv - pair_shift; every pixel of each eye
// is marched once.  Unpartitioned frames only.
// NL (round 6, VR_NL2): 2 / 1 -- a launch of exactly two lights (the metric frame, examples/example1.m)
// or one (examples/example2.m, example3.m), whose tame march shades the lights it holds in registers
// without a light loop (shade_fast NL); 0 -- any light count.
template <int K, int MODE, bool AB_ALIAS, bool COUNT, bool SHARE2, bool BIG, int CAP, int SCHED, int NL>
__global__ __launch_bounds__(64 * VR_WG_WAVES, march_min_eu(CAP, SCHED)) void march_kernel(const RenderParams P) {
  using TS = TileShape<K>;
  __shared__ float lds[VR_WG_WAVES][CAP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float *L = lds[wave];
  constexpr bool ORDERED = SCHED >= 1 && SCHED <= 3;
  constexpr bool TIMED = SCHED == 1 || SCHED == 2;  // SCHED 3: the order only
  constexpr bool PAIRED = SCHED == 4;
  const uint64_t clk0 = TIMED ? __builtin_amdgcn_s_memrealtime() : 0;
  uint32_t wgo = ORDERED ? P.wg_order[blockIdx.x] : xcd_block(blockIdx.x, gridDim.x, P.xcd_run);
  if (!ORDERED && P.block_rot) {  // (A/B, VR_BLOCK_ROT_ROWS) a rotation of the row-major order
    wgo += P.block_rot;
    if (wgo >= gridDim.x) wgo -= gridDim.x;
  }
  // the longest blocks (first in the order) issue ahead of the short ones that fill in beside them
  if (ORDERED && blockIdx.x < P.prio_blocks) __builtin_amdgcn_s_setprio(2);
  int view, lc, y;
  if constexpr (PAIRED) {
    constexpr int TH2 = TS::TH / 2, HR = (64 / K) / 2;  // rows and rays of each eye's half tile
    const int tile = (int)wgo * VR_WG_WAVES + wave;
    const int nbx = (P.part_cols + P.pair_shift + 2 * TS::TW - 1) / (2 * TS::TW);
    const int blk = tile >> 2, quad = tile & 3;
    const int ray = lane >> TS::LK, rr = ray & (HR - 1);
    view = ray >= HR ? 0 : 1;  // 0: the left eye (P.out), 1: the right eye (P.out2)
    const int xv = (blk % nbx) * (2 * TS::TW) + (quad & 1) * TS::TW + rr / TH2;
    y = (blk / nbx) * (2 * TH2) + (quad >> 1) * TH2 + rr % TH2;
    lc = view ? xv - P.pair_shift : xv;
  } else {
    // fused stereo: the second view's workgroups follow the first's (same rays, other eye)
    view = (P.views > 1 && wgo >= P.view_blocks) ? 1 : 0;
    const uint32_t wg = view ? wgo - P.view_blocks : wgo;
    const int tile = (int)wg * VR_WG_WAVES + wave;
    const int nbx = (P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW);
    const int blk = tile >> 2, quad = tile & 3;
    const int ray = lane >> TS::LK;
    lc = (blk % nbx) * (2 * TS::TW) + (quad & 1) * TS::TW + (ray / TS::TH);
    y = (blk / nbx) * (2 * TS::TH) + (quad >> 1) * TS::TH + (ray % TS::TH);
  }
  float *const out = view ? P.out2 : P.out;
  const bool active = (!PAIRED || lc >= 0) && (lc < P.part_cols) && (y < P.height);
  Ray R;
  R.o = mk(0.f, 0.f, 0.f);
  R.pos = R.o;
  R.step = R.o;
  R.t = 0.f;
  R.tfar = -1.f;
  R.sr = R.sg = R.sb = R.sa = 0.f;
  R.nsteps = R.nlit = 0;
  R.alive = false;
  ChunkStats C{0, 0, 0, 0, 0, 0, 0};
  if (active) {
    const int blk = lc / P.block_cols, within = lc - blk * P.block_cols;
    const int x = (P.part + blk * P.num_parts) * P.block_cols + within;
    f3 d;
    float tnear;
    R.alive = ray_setup(P, x, y, R.o, d, tnear, R.tfar, view);
    R.pos = mk(fmaf(d.x, tnear, R.o.x), fmaf(d.y, tnear, R.o.y), fmaf(d.z, tnear, R.o.z));
    R.step = mk(d.x * P.tstep, d.y * P.tstep, d.z * P.tstep);
    R.t = tnear;
  }
  // every coordinate the march forms from a finite start and step is finite; a tame launch takes
  // the fast path (sample_at: TAME)
  if (P.tame && __all(!R.alive || (finite3(R.pos) && finite3(R.step))))
    march<K, MODE, AB_ALIAS, COUNT, SHARE2, BIG, false, CAP, false, NL>(
        P, L, lane, R, C, 0u, (KParams)__builtin_amdgcn_kernarg_segment_ptr(), wgo * VR_WG_WAVES + (uint32_t)wave);
  else
    march<K, MODE, AB_ALIAS, COUNT, SHARE2, BIG, true, CAP>(P, L, lane, R, C);

  if (active && (lane & (K - 1)) == 0) {
    const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
    const size_t kk = (size_t)lc * (size_t)P.height + (size_t)y;
    out[kk] = R.sr;
    out[kk + plane] = R.sg;
    out[kk + 2 * plane] = R.sb;
  }
  if (TIMED) {  // this block's duration, for the next launch's schedule
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t d = __builtin_amdgcn_s_memrealtime() - clk0;
      P.wg_cost[wgo] = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
      if (P.wg_start) P.wg_start[wgo] = (uint32_t)clk0;
    }
  }
  if (COUNT) {
    // (K > 1: the lanes' sample indices are not the ray's sample count -- the sums are the K = 1 variant's)
    unsigned long long s = K == 1 ? (unsigned long long)R.nsteps : 0ull, l = K == 1 ? (unsigned long long)R.nlit : 0ull;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      s += __shfl_xor(s, off, 64);
      l += __shfl_xor(l, off, 64);
    }
    if (lane == 0 && s) atomicAdd(P.steps, s);
    if (lane == 0 && l) atomicAdd(P.steps + 1, l);
    if (lane == 0) {  // per-wave chunk counts (uniform values)
      atomicAdd(P.steps + 2, (unsigned long long)C.staged);
      atomicAdd(P.steps + 3, (unsigned long long)C.leap);
      atomicAdd(P.steps + 4, (unsigned long long)C.fall);
      atomicAdd(P.steps + 5, (unsigned long long)C.iter);
      atomicAdd(P.steps + 6, (unsigned long long)C.lit);
      atomicAdd(P.steps + 7, (unsigned long long)C.probe);
      atomicAdd(P.steps + 44, (unsigned long long)C.probe_fail);
    }
  }
}

// Pre-leap launch (round 6, VR_PRELEAP; DESIGN.md s5 "Rays far apart in one wave"): a wave whose
// live rays start more than VR_PRELEAP_SPREAD steps apart along their direction (a tile of rays
// entering the volume through a face at a grazing angle: the columns next to the silhouette at
// rotate(30,10,0) start 900-2700 samples apart) cannot probe one box for them all, so before the
// march each of its rays walks the occupancy map along its own runs of VR_PROBE_MAX samples
// (probe_lane_walk: segments of at most 4 texels per axis, each segment's brick box widened by the
// probe margin) and leaps every run whose cells all lie in +-0 bricks -- exact as the probe's leap,
// run by run (the margin covers one run's drift) -- until a run finds data; a ray's K lanes leap
// together.  The states go to a slot the march wave starts from (RenderParams::pre_flag / pre_state).
// A separate launch: the same code inside the march cost every launch ~2 % (code placement), though
// it rarely ran.  Same workgroups and ray mapping as march_kernel (not paired stereo tiles).
template <int K>
__global__ __launch_bounds__(64 * VR_WG_WAVES) void preleap_kernel(const RenderParams P) {
  using TS = TileShape<K>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t wgo = blockIdx.x;
  const uint32_t gw = wgo * VR_WG_WAVES + (uint32_t)wave;
  const int view = (P.views > 1 && wgo >= P.view_blocks) ? 1 : 0;
  const uint32_t wg = view ? wgo - P.view_blocks : wgo;
  const int tile = (int)wg * VR_WG_WAVES + wave;
  const int nbx = (P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW);
  const int blk = tile >> 2, quad = tile & 3;
  const int ray = lane >> TS::LK;
  const int lc = (blk % nbx) * (2 * TS::TW) + (quad & 1) * TS::TW + (ray / TS::TH);
  const int y = (blk / nbx) * (2 * TS::TH) + (quad >> 1) * TS::TH + (ray % TS::TH);
  const bool active = lc < P.part_cols && y < P.height;
  Ray R;
  R.pos = mk(0.f, 0.f, 0.f);
  R.step = R.pos;
  R.t = 0.f;
  R.tfar = -1.f;
  R.nsteps = 0;
  R.alive = false;
  if (active) {
    const int pb = lc / P.block_cols, within = lc - pb * P.block_cols;
    const int x = (P.part + pb * P.num_parts) * P.block_cols + within;
    f3 o, d;
    float tnear;
    R.alive = ray_setup(P, x, y, o, d, tnear, R.tfar, view);
    R.pos = mk(fmaf(d.x, tnear, o.x), fmaf(d.y, tnear, o.y), fmaf(d.z, tnear, o.z));
    R.step = mk(d.x * P.tstep, d.y * P.tstep, d.z * P.tstep);
    R.t = tnear;
  }
  const int cap = P.max_steps;
  uint32_t flag = 0;
  // the march's tame waves only (march_kernel: finite starts and steps; the probe needs the map)
  if (P.tame && P.occ != nullptr && __all(!R.alive || (finite3(R.pos) && finite3(R.step)))) {
    if constexpr (K > 1) {  // to this lane's first sample, as march()
      R.mine = R.alive;
      leap(P, lane & (K - 1), R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
      R.alive = group_any<K>(R.mine);
    } else {
      R.mine = R.alive;
    }
    const bool lv0 = K > 1 ? (R.alive && R.mine) : R.alive;
    const int tmn = wave_min(lv0 ? __float_as_int(R.t) : 0x7f7fffff);
    const int tmx = wave_max(lv0 ? __float_as_int(R.t) : 0);
    if (__int_as_float(tmx) > __int_as_float(tmn) + (float)VR_PRELEAP_SPREAD * P.tstep) {
      const KParams kq = (KParams)__builtin_amdgcn_kernarg_segment_ptr();
      bool go = lv0;
      while (group_any<K>(go)) {  // (a ray's K lanes decide together)
        uint32_t v = 0;
        if (go) {
          const float rem = (R.tfar - R.t) / P.tstep;
          const int s_eff = (rem < (float)VR_PROBE_MAX) ? max((int)rem + 2, 1) : (int)VR_PROBE_MAX;
          const float k = (float)(s_eff - 1);
          const f3 pe = mk(fmaf(R.step.x, k, R.pos.x), fmaf(R.step.y, k, R.pos.y), fmaf(R.step.z, k, R.pos.z));
          v = probe_lane_walk(P.occ, P.occ_bx, P.occ_bxy, ((R.pos.x - P.bmin[0]) * P.bscale[0]) * P.em.fnx - 0.5f,
                              ((R.pos.y - P.bmin[1]) * P.bscale[1]) * P.em.fny - 0.5f,
                              ((R.pos.z - P.bmin[2]) * P.bscale[2]) * P.em.fnz - 0.5f,
                              ((pe.x - P.bmin[0]) * P.bscale[0]) * P.em.fnx - 0.5f,
                              ((pe.y - P.bmin[1]) * P.bscale[1]) * P.em.fny - 0.5f,
                              ((pe.z - P.bmin[2]) * P.bscale[2]) * P.em.fnz - 0.5f, kq->probe_off[0],
                              kq->probe_off[1], kq->probe_off[2], P.em.nx, P.em.ny, P.em.nz);
        }
        const bool data = group_any<K>(v != 0u);
        if (go && !data) {
          if constexpr (K == 1) {
            advance_n(P, (int)VR_PROBE_MAX, R.alive, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
            go = R.alive;
          } else {
            advance_n(P, (int)VR_PROBE_MAX, R.mine, R.nsteps, R.t, R.tfar, R.pos, R.step, cap);
            go = group_any<K>(R.mine);
          }
        } else {
          go = false;
        }
      }
      if constexpr (K > 1) R.alive = R.alive && group_any<K>(R.mine);
      if constexpr (K == 1) R.mine = R.alive;
      uint32_t slot = 0;
      if (lane == 0) slot = atomicAdd(P.pre_count, 1u);
      slot = __builtin_amdgcn_readfirstlane(slot);
      if (slot < P.pre_cap) {  // (no slot left: the wave marches from its start, as without)
        float4 *st = P.pre_state + ((size_t)slot * 64u + (uint32_t)lane) * 2u;
        st[0] = make_float4(R.t, R.pos.x, R.pos.y, R.pos.z);
        st[1] = make_float4(__int_as_float(R.nsteps), __int_as_float((R.alive ? 1 : 0) | (R.mine ? 2 : 0)), 0.f, 0.f);
        flag = slot + 1u;
      }
    }
  }
  if (lane == 0) const_cast<uint32_t *>(P.pre_flag)[gw] = flag;
}

#if !VR_ISA_PROBE
hipError_t VR_CAT(launch_preleap_k, VR_MARCH_K)(const RenderParams &P, hipStream_t s) {
  constexpr int K = VR_MARCH_K;
  using TS = TileShape<K>;
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  if (!P.pre_flag || !P.pre_state || !P.pre_count || P.pair_shift) return hipErrorInvalidValue;
  const uint64_t tiles = (uint64_t)((P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW)) *
                         (uint64_t)((P.height + 2 * TS::TH - 1) / (2 * TS::TH)) * 4;
  const uint32_t per_view = (uint32_t)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES);
  hipLaunchKernelGGL(preleap_kernel<K>, dim3(per_view * (P.views > 1 ? 2u : 1u)), dim3(64 * VR_WG_WAVES), 0, s, P);
  return hipGetLastError();
}
#endif

#if VR_MARCH_K <= 4
// One wave's tile of workgroup `wg` of a view: ray setup, the march, the pixel store into `out` --
// march_kernel's body for the multi-view launch below.  (march_kernel keeps its own copy: routed
// through this function its register allocation changes, and the metric kernel is measured as is.)
template <int K, int MODE, bool AB_ALIAS, bool COUNT, bool SHARE2, bool BIG, int CAP>
__device__ __forceinline__ void march_tile(const RenderParams &P, float *L, int lane, int wave, uint32_t wg,
                                           int view, float *out, Ray &R, ChunkStats &C, KParams kp) {
  using TS = TileShape<K>;
  const int tile = (int)wg * VR_WG_WAVES + wave;
  const int nbx = (P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW);
  const int blk = tile >> 2, quad = tile & 3;
  const int ray = lane >> TS::LK;
  const int lc = (blk % nbx) * (2 * TS::TW) + (quad & 1) * TS::TW + (ray / TS::TH);
  const int y = (blk / nbx) * (2 * TS::TH) + (quad >> 1) * TS::TH + (ray % TS::TH);
  const bool active = (lc < P.part_cols) && (y < P.height);
  R.o = mk(0.f, 0.f, 0.f);
  R.pos = R.o;
  R.step = R.o;
  R.t = 0.f;
  R.tfar = -1.f;
  R.sr = R.sg = R.sb = R.sa = 0.f;
  R.nsteps = R.nlit = 0;
  R.alive = false;
  if (active) {
    const int blk = lc / P.block_cols, within = lc - blk * P.block_cols;
    const int x = (P.part + blk * P.num_parts) * P.block_cols + within;
    f3 d;
    float tnear;
    R.alive = ray_setup(P, x, y, R.o, d, tnear, R.tfar, view);
    R.pos = mk(fmaf(d.x, tnear, R.o.x), fmaf(d.y, tnear, R.o.y), fmaf(d.z, tnear, R.o.z));
    R.step = mk(d.x * P.tstep, d.y * P.tstep, d.z * P.tstep);
    R.t = tnear;
  }
  // every coordinate the march forms from a finite start and step is finite; a tame launch takes
  // the fast path (sample_at: TAME)
  if (P.tame && __all(!R.alive || (finite3(R.pos) && finite3(R.step))))
    march<K, MODE, AB_ALIAS, COUNT, SHARE2, BIG, false, CAP>(P, L, lane, R, C, 0u, kp);
  else
    march<K, MODE, AB_ALIAS, COUNT, SHARE2, BIG, true, CAP>(P, L, lane, R, C);

  if (active && (lane & (K - 1)) == 0) {
    const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
    const size_t kk = (size_t)lc * (size_t)P.height + (size_t)y;
    out[kk] = R.sr;
    out[kk + plane] = R.sg;
    out[kk + 2 * plane] = R.sb;
  }
}

// Fused views (vr_render_channels): the channels of a multi-channel frame, and of
// each its stereo eyes, in one launch.  Every view has its own RenderParams (volumes, factors,
// colour, lights, eye, output), all of them kernel arguments (scalar loads at a uniform offset;
// pointers loaded from the argument segment stay global, which a device-memory table would lose),
// and the same image and partition; view v marches workgroups [v * per_view, (v+1) * per_view).
template <int K, int MODE, bool AB_ALIAS, int CAP>
__global__ __launch_bounds__(64 * VR_WG_WAVES, march_min_eu(CAP, false)) void march_views_kernel(
    const RenderViews V, uint32_t per_view) {
  __shared__ float lds[VR_WG_WAVES][CAP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const uint32_t view = blockIdx.x / per_view;
  const RenderParams &P = V.p[view];
  Ray R;
  ChunkStats C{0, 0, 0, 0, 0, 0, 0};
  // (view's RenderParams in the argument segment: V is the kernel's first argument)
  const KParams kp = (KParams)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() +
                               (size_t)view * sizeof(RenderParams));
  march_tile<K, MODE, AB_ALIAS, false, false, false, CAP>(P, lds[wave], lane, wave, blockIdx.x - view * per_view, 0,
                                                          P.out, R, C, kp);
}

#if !VR_ISA_PROBE
// Host entry (launch_march_views_k1 / _k2 / _k4): V.p[0 .. nviews) share the image, partition,
// gradient mode (0 or 1), absorption aliasing and slot size; 32-bit addressing only.
hipError_t VR_CAT(launch_march_views_k, VR_MARCH_K)(const RenderViews &V, uint32_t nviews, int mode, bool ab_alias,
                                                   hipStream_t s) {
  constexpr int K = VR_MARCH_K;
  using TS = TileShape<K>;
  const RenderParams &P0 = V.p[0];
  if (nviews > VR_VIEWS_MAX) return hipErrorInvalidValue;
  if (P0.part_cols <= 0 || P0.height <= 0 || nviews == 0) return hipSuccess;
  if (mode > 1 || P0.steps || P0.wg_order) return hipErrorInvalidValue;
  for (uint32_t v = 1; v < nviews; ++v)
    if (V.p[v].part_cols != P0.part_cols || V.p[v].height != P0.height || V.p[v].wide_slot != P0.wide_slot)
      return hipErrorInvalidValue;
  const uint64_t tiles = (uint64_t)((P0.part_cols + 2 * TS::TW - 1) / (2 * TS::TW)) *
                         (uint64_t)((P0.height + 2 * TS::TH - 1) / (2 * TS::TH)) * 4;
  const uint32_t per_view = (uint32_t)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES);
  if ((uint64_t)per_view * nviews > 0x7fffffffull) return hipErrorInvalidValue;
  const dim3 grid(per_view * nviews), blk(64 * VR_WG_WAVES);
#define VR_VIEWS_LAUNCH(M, A)                                                                                    \
  do {                                                                                                           \
    if (P0.wide_slot)                                                                                            \
      hipLaunchKernelGGL((march_views_kernel<K, M, A, VR_LDS_CAP_WIDE>), grid, blk, 0, s, V, per_view);         \
    else                                                                                                         \
      hipLaunchKernelGGL((march_views_kernel<K, M, A, VR_LDS_CAP>), grid, blk, 0, s, V, per_view);              \
  } while (0)
  if (mode == 0) {
    if (ab_alias) VR_VIEWS_LAUNCH(0, true);
    else VR_VIEWS_LAUNCH(0, false);
  } else {
    if (ab_alias) VR_VIEWS_LAUNCH(1, true);
    else VR_VIEWS_LAUNCH(1, false);
  }
#undef VR_VIEWS_LAUNCH
  return hipGetLastError();
}

#endif  // !VR_ISA_PROBE
// Sort-last slab launch: one wave per 8x8 tile of the image part (the columns of
// the image partition, vr_partition); per pixel the ray state is read from P.slab_in (null: a
// fresh ray), marched through this slab's samples and written to P.out as VR_SLAB_PLANES
// [plane_cols][H] planes: premultiplied r, g, b, alpha; 1 if the ray goes on past this slab; and
// the resume point of a ray that goes on -- t, pos.x, pos.y, pos.z and the sample index (int32
// bits) of its next sample -- so the next slab continues the recurrences where this one stopped
// instead of replaying them from the ray start.  Rays whose direction does not match the sweep
// (P.slab_dir: +1 = rays with dir.z >= 0 in ascending slab order, -1 = dir.z < 0 descending; 0 =
// both, for the top slab, where the descending rays start) pass their state through (a fresh ray's
// resume point is its start).
// SH / SCHED as for march_kernel: the half-texel tap launch; the longest-first schedule.
#ifndef VR_SLAB_MIN_EU
#define VR_SLAB_MIN_EU 6  // the slab kernel keeps 6 waves per SIMD (5 measured no faster, r3ag)
#endif
template <int K, int MODE, bool SH, int CAP, bool SCHED>
__global__ __launch_bounds__(64 * VR_WG_WAVES, (CAP <= VR_LDS_CAP && !SCHED) ? VR_SLAB_MIN_EU : 1) void march_slab_kernel(
    const RenderParams P) {
  using TS = TileShape<K>;
  __shared__ float lds[VR_WG_WAVES][CAP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float *L = lds[wave];
  const uint64_t clk0 = SCHED ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint32_t wg = SCHED ? P.wg_order[blockIdx.x] : blockIdx.x;
  if (SCHED && blockIdx.x < P.prio_blocks) __builtin_amdgcn_s_setprio(2);
  const int tile = (int)wg * VR_WG_WAVES + wave;
  const int nbx = (P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW);
  const int blk = tile >> 2, quad = tile & 3;
  const int ray = lane >> TS::LK;
  const int lc = (blk % nbx) * (2 * TS::TW) + (quad & 1) * TS::TW + (ray / TS::TH);  // local column
  const int y = (blk / nbx) * (2 * TS::TH) + (quad >> 1) * TS::TH + (ray % TS::TH);
  const bool active = (lc < P.part_cols) && (y < P.height);
  const int pb = lc / P.block_cols;
  const int x = (P.part + pb * P.num_parts) * P.block_cols + (lc - pb * P.block_cols);
  const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
  const uint32_t kk = (uint32_t)lc * (uint32_t)P.height + (uint32_t)y;  // plane < 2^32 (host check)
  Ray R;
  R.o = mk(0.f, 0.f, 0.f);
  R.pos = R.o;
  R.step = R.o;
  R.t = 0.f;
  R.tfar = -1.f;
  R.sr = R.sg = R.sb = R.sa = 0.f;
  R.nsteps = R.nlit = 0;
  R.alive = false;
  R.mine = false;
  R.past = false;
  bool go_on = true;  // the incoming state: the ray has not terminated
  ChunkStats C{0, 0, 0, 0, 0, 0, 0};
  if (active) {
    f3 d;
    float tnear;
    const bool hit = ray_setup(P, x, y, R.o, d, tnear, R.tfar);
    R.pos = mk(fmaf(d.x, tnear, R.o.x), fmaf(d.y, tnear, R.o.y), fmaf(d.z, tnear, R.o.z));
    R.step = mk(d.x * P.tstep, d.y * P.tstep, d.z * P.tstep);
    R.t = tnear;
    if (P.slab_in) {
      R.sr = P.slab_in[kk];
      R.sg = P.slab_in[kk + plane];
      R.sb = P.slab_in[kk + 2 * plane];
      R.sa = P.slab_in[kk + 3 * plane];
      go_on = P.slab_in[kk + 4 * plane] != 0.f;
      if (go_on) {  // resume at the next sample
        R.t = P.slab_in[kk + 5 * plane];
        R.pos = mk(P.slab_in[kk + 6 * plane], P.slab_in[kk + 7 * plane], P.slab_in[kk + 8 * plane]);
        R.nsteps = __float_as_int(P.slab_in[kk + 9 * plane]);
      }
    }
    const bool mine_dir = P.slab_dir == 0 || (P.slab_dir > 0) == (R.step.z >= 0.f);
    R.alive = hit && go_on && mine_dir;
    R.past = go_on && !mine_dir;  // another sweep's ray: passed through unchanged
    if (!hit) R.past = false;
  }
  // the resume point as it stands (a ray passed through keeps it; one handed off below replaces it)
  if (active && (lane & (K - 1)) == 0) store_resume(P, kk, R.t, R.pos, R.nsteps);
  if (P.tame && __all(!R.alive || (finite3(R.pos) && finite3(R.step))))
    march<K, MODE, true, false, SH, true, false, CAP, true>(P, L, lane, R, C, kk);
  else
    march<K, MODE, true, false, SH, true, true, CAP, true>(P, L, lane, R, C, kk);
  if (SCHED) {
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t d = __builtin_amdgcn_s_memrealtime() - clk0;
      P.wg_cost[wg] = d > 0xffffffffull ? 0xffffffffu : (uint32_t)d;
    }
  }
  if (active && (lane & (K - 1)) == 0) {
    P.out[kk] = R.sr;
    P.out[kk + plane] = R.sg;
    P.out[kk + 2 * plane] = R.sb;
    P.out[kk + 3 * plane] = R.sa;
    P.out[kk + 4 * plane] = R.past ? 1.f : 0.f;
  }
}

#if !VR_ISA_PROBE
// Host entry of the slab launch (launch_march_slab_k1 / _k2 / _k4): MODE 0 or 1, absorption
// aliasing emission, the emission texture addressed with 64-bit offsets from its virtual base.
template <int MODE, bool SH, int CAP>
static void launch_slab_c(const RenderParams &P, dim3 grid, hipStream_t s) {
  constexpr int K = VR_MARCH_K;
  const dim3 blk(64 * VR_WG_WAVES);
  if (P.wg_order) hipLaunchKernelGGL((march_slab_kernel<K, MODE, SH, CAP, true>), grid, blk, 0, s, P);
  else hipLaunchKernelGGL((march_slab_kernel<K, MODE, SH, CAP, false>), grid, blk, 0, s, P);
}

template <int MODE, bool SH>
static void launch_slab_m(const RenderParams &P, dim3 grid, hipStream_t s) {
  if (P.wide_slot) launch_slab_c<MODE, SH, VR_LDS_CAP_WIDE>(P, grid, s);
  else launch_slab_c<MODE, SH, VR_LDS_CAP>(P, grid, s);
}

hipError_t VR_CAT(launch_march_slab_k, VR_MARCH_K)(const RenderParams &P, int mode, hipStream_t s) {
  constexpr int K = VR_MARCH_K;
  using TS = TileShape<K>;
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  if (mode > 1) return hipErrorInvalidValue;
  const uint64_t tiles = (uint64_t)((P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW)) *
                         (uint64_t)((P.height + 2 * TS::TH - 1) / (2 * TS::TH)) * 4;
  const dim3 grid((unsigned)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES));
  if (P.wg_order && (P.sched_blocks != grid.x || !P.wg_cost || K == 1)) return hipErrorInvalidValue;
  if (mode == 0) launch_slab_m<0, false>(P, grid, s);
  else if (VR_MARCH_FAST && P.tap_half) launch_slab_m<1, true>(P, grid, s);
  else launch_slab_m<1, false>(P, grid, s);
  return hipGetLastError();
}
#endif  // !VR_ISA_PROBE
#endif

#if !VR_ISA_PROBE
// VR_INJECT_BAD_LAUNCH=1 (tests only): the march launch asks for 2048 work-items per workgroup, more
// than a gfx950 workgroup holds, so the runtime rejects it before dispatch -- the reporting path of
// a failed launch (tests/test_gpu_streams.py::test_failed_launch_is_reported_by_its_call).  Read
// per launch.
static bool inject_bad_launch() {
  const char *ev = test_switches_on() ? getenv("VR_INJECT_BAD_LAUNCH") : nullptr;
  return ev && ev[0] == '1';
}

// One march_kernel launch; a lit launch of one or two lights takes the NL = 1 / 2 kernel where the
// lights are hoisted (march: VR_LIGHTS_HOIST's conditions).
template <int KK, int MODE, bool AB, bool CNT, bool SH, bool BG, int CAP, int SC>
static void launch_one(const RenderParams &P, dim3 grid, dim3 blk, hipStream_t s) {
  // (on-the-fly gradient launches only: the lookup-gradient march, C3, measured 0.8 % slower with it,
  // 27.65-27.70 vs 27.44-27.47 ms, r6v)
  constexpr bool NL2 = VR_NL2 && VR_LIGHTS_HOIST && MODE == 1 && KK > 1 && AB && SH && !BG && !CNT;
  const int nl = (NL2 && (P.num_lights == 2 || P.num_lights == 1)) ? P.num_lights : 0;
  if (NL2 && nl == 2) hipLaunchKernelGGL((march_kernel<KK, MODE, AB, CNT, SH, BG, CAP, SC, NL2 ? 2 : 0>), grid, blk, 0, s, P);
  else if (NL2 && nl == 1) hipLaunchKernelGGL((march_kernel<KK, MODE, AB, CNT, SH, BG, CAP, SC, NL2 ? 1 : 0>), grid, blk, 0, s, P);
  else hipLaunchKernelGGL((march_kernel<KK, MODE, AB, CNT, SH, BG, CAP, SC, 0>), grid, blk, 0, s, P);
  note_march_kernel(VR_MARCH_FAST, KK, MODE, AB, CNT, SH, BG, CAP, SC, nl);
}

// BS: the addressing variants this instantiation holds (1: 32-bit, 2: 64-bit, 3: both) -- the
// narrow slot differs between them (launch_m), the kernel count does not.
template <int MODE, bool AB, bool SH, int CAP, int BS = 3>
static hipError_t launch_c(const RenderParams &P, dim3 grid, hipStream_t s, bool big) {
  constexpr int K = VR_MARCH_K;
  const dim3 blk(inject_bad_launch() ? 2048 : 64 * VR_WG_WAVES);
  const bool sched = P.wg_order && P.wg_cost;
  // scheduled kernels: K > 1, fast variant, absorption = emission only (otherwise the names below
  // alias the SCHED 0 kernel; the host schedules no other launch, vr_capi.hip attach_schedule)
  constexpr bool SCH = K > 1 && VR_MARCH_FAST && AB;
  constexpr int S1 = SCH ? 1 : 0, S2 = SCH ? 2 : 0, S3 = SCH ? 3 : 0;
#define VR_LAUNCH(KK, CNT, BG, SC) launch_one<KK, MODE, AB, CNT, SH, BG, CAP, SC>(P, grid, blk, s)
#define VR_LAUNCH_B(KK, CNT, SC)                                                                           \
  do {                                                                                                    \
    if (big) {                                                                                            \
      if constexpr ((BS & 2) != 0) VR_LAUNCH(KK, CNT, true, SC);                                          \
      else return hipErrorInvalidValue;                                                                   \
    } else {                                                                                              \
      if constexpr ((BS & 1) != 0) VR_LAUNCH(KK, CNT, false, SC);                                         \
      else return hipErrorInvalidValue;                                                                   \
    }                                                                                                     \
  } while (0)
  // paired stereo tiles (SCHED 4): the lit, half-texel-tap, absorption = emission, default-slot,
  // 32-bit launch of K > 1 only (a measurement of what the eyes' staged boxes share)
  constexpr bool PAIRK = K > 1 && VR_MARCH_FAST && AB && MODE == 1 && SH && CAP == VR_LDS_CAP_MARCH && (BS & 1);
  if (P.pair_shift) {
    if constexpr (PAIRK) {
      if (big || sched || (P.steps && !VR_COUNT_K)) return hipErrorInvalidValue;
      if (P.steps) VR_LAUNCH(K, VR_COUNT_K != 0, false, 4);
      else VR_LAUNCH(K, false, false, 4);
      return hipGetLastError();
    } else {
      return hipErrorInvalidValue;
    }
  }
  // (the counter variant: instantiated in the K = 1 object only -- or at every K in a VR_COUNT_K build)
  if constexpr (K == 1 || VR_COUNT_K) {
    if (P.steps) {
      VR_LAUNCH_B(K, true, 0);
      return hipGetLastError();
    }
  }
  if (P.steps) {
    return hipErrorInvalidValue;
  } else if (sched && !SCH) {  // the exact variant and separate absorption have no scheduled kernels
    return hipErrorInvalidValue;
  } else if (K > 1 && sched && P.sched_full == 1) {  // a full frame, durations measured
    VR_LAUNCH_B(K, false, S2);
  } else if (K > 1 && sched && P.sched_full == 2) {  // a full frame in the last measured order
    VR_LAUNCH_B(K, false, S3);
  } else if (K > 1 && sched) {  // a short launch (few waves per slot), longest first
    VR_LAUNCH_B(K, false, S1);
  } else {
    VR_LAUNCH_B(K, false, 0);
  }
#undef VR_LAUNCH_B
#undef VR_LAUNCH
  return hipGetLastError();
}

// The wave slot of a launch: wide (P.wide_slot), else 8 KiB for a 32-bit launch without lookup
// gradients and 6.5 KiB for the others (vr_stage.h VR_LDS_CAP_MARCH).
template <int MODE, bool AB, bool SH>
static hipError_t launch_m(const RenderParams &P, dim3 grid, hipStream_t s, bool big) {
  if (P.wide_slot) return launch_c<MODE, AB, SH, VR_LDS_CAP_WIDE>(P, grid, s, big);
  // (the exact-arithmetic variant, a parity reference, keeps 6.5 KiB everywhere: 0.5 MiB less code)
  if constexpr (MODE == 2 || !VR_MARCH_FAST)
    return launch_c<MODE, AB, SH, VR_LDS_CAP>(P, grid, s, big);
  else
    return big ? launch_c<MODE, AB, SH, VR_LDS_CAP, 2>(P, grid, s, big)
               : launch_c<MODE, AB, SH, VR_LDS_CAP_MARCH, 1>(P, grid, s, big);
}

// Host entry (launch_march_k1 / _k2 / _k4 / _k8, one per object file): the staged kernel needs a
// bound, non-constant emission texture; for MODE 1 the gradient texture must be the emission
// texture itself (the reference's tex_emission binding).  The counter variant (P.steps) exists
// for K = 1 only; the host routes counted launches there.
// Number of workgroups launch_march_k<K> uses for this frame (the schedule's length).
uint32_t VR_CAT(march_blocks_k, VR_MARCH_K)(const RenderParams &P) {
  using TS = TileShape<VR_MARCH_K>;
  if (P.part_cols <= 0 || P.height <= 0) return 0;
  const uint64_t tiles = (uint64_t)((P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW)) *
                         (uint64_t)((P.height + 2 * TS::TH - 1) / (2 * TS::TH)) * 4;
  return (uint32_t)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES);
}

hipError_t VR_CAT(launch_march_k, VR_MARCH_K)(const RenderParams &P, int mode, bool ab_alias, bool share, bool big,
                                              hipStream_t s) {
  using TS = TileShape<VR_MARCH_K>;
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  if (VR_MARCH_K != 1 && !VR_COUNT_K && P.steps) return hipErrorInvalidValue;
  const uint64_t tiles = (uint64_t)((P.part_cols + 2 * TS::TW - 1) / (2 * TS::TW)) *
                         (uint64_t)((P.height + 2 * TS::TH - 1) / (2 * TS::TH)) * 4;
  const uint32_t per_view = (uint32_t)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES);
  if (P.views > 1 && (P.view_blocks != per_view || !P.out2)) return hipErrorInvalidValue;
  dim3 grid(per_view * (P.views > 1 ? 2u : 1u));
  if (P.pair_shift) {  // paired stereo tiles (march_kernel SCHED 4): half tiles of each eye over the virtual width
    if (P.views != 2 || P.num_parts != 1 || P.pair_shift < 0 || P.wg_order) return hipErrorInvalidValue;
    const uint64_t ptiles = (uint64_t)((P.part_cols + P.pair_shift + 2 * TS::TW - 1) / (2 * TS::TW)) *
                            (uint64_t)((P.height + TS::TH - 1) / TS::TH) * 4;
    grid = dim3((unsigned)((ptiles + VR_WG_WAVES - 1) / VR_WG_WAVES));
  }
  if (P.wg_order && (P.sched_blocks != grid.x || !P.wg_cost || VR_MARCH_K == 1))
    return hipErrorInvalidValue;  // a schedule of another grid, or for K = 1 (not built)
  switch (mode) {
    case 0: return ab_alias ? launch_m<0, true, false>(P, grid, s, big) : launch_m<0, false, false>(P, grid, s, big);
    case 1:  // SH: the half-texel tap launch (fast variant only; see sample_at)
      if (VR_MARCH_FAST && P.tap_half)
        return ab_alias ? launch_m<1, true, true>(P, grid, s, big) : launch_m<1, false, true>(P, grid, s, big);
      return ab_alias ? launch_m<1, true, false>(P, grid, s, big) : launch_m<1, false, false>(P, grid, s, big);
    default:
      if (share) return ab_alias ? launch_m<2, true, true>(P, grid, s, big) : launch_m<2, false, true>(P, grid, s, big);
      return ab_alias ? launch_m<2, true, false>(P, grid, s, big) : launch_m<2, false, false>(P, grid, s, big);
  }
}

#else
// ISA probe (tools/isa_probe.sh): only the metric frame's production instantiation and the matching
// sort-last slab kernel, for a quick look at their code without compiling every variant.
template __global__ void march_kernel<2, 1, true, false, true, false, VR_LDS_CAP_MARCH, 0, 2>(const RenderParams P);
template __global__ void march_kernel<2, 2, true, false, true, false, VR_LDS_CAP, 0, 0>(const RenderParams P);  // C3
template __global__ void march_slab_kernel<2, 1, true, VR_LDS_CAP, false>(const RenderParams P);
#endif  // !VR_ISA_PROBE
}  // namespace fast / exact
}  // namespace vr
