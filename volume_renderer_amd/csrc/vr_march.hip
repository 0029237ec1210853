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

// Per-lane march state carried across chunks.
struct Ray {
  f3 o, pos, step;
  float t, tfar;
  float sr, sg, sb, sa;
  int32_t nsteps, nlit;
  bool alive;
};

struct ChunkStats {
  uint32_t staged, leap, fall, iter, lit;
};

// The chunked march of one wave.  NANCHK = false when every live ray of the wave has a finite
// start position and step: all volume coordinates are then finite and the NaN -> 0 substitution
// of the sampler is skipped (the LUT coordinates, which are NaN for a zero gradient, keep it).
// MODE 0: no lights; 1: on-the-fly gradient from the staged emission texture (gem == em);
// 2: lookup gradient (gx/gy/gz from global memory, at the centre's axes when SHARE2).
template <int MODE, bool AB_ALIAS, bool COUNT, bool SHARE2, bool BIG, bool NANCHK, int CAP>
__device__ __forceinline__ void march(const RenderParams &P, float *L, int lane, Ray &R, ChunkStats &C) {
  const DevTex &E = P.em;
  const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);
  const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
  const float tstep = P.tstep, thr = P.thr;

  while (__any(R.alive)) {
    // ---- chunk set-up: the box of every tap the live rays take in the next S samples --------
    int S;
    bool staged, partial;
    Box B;
    int box_vol = 0;
    plan_chunk<CAP>(P, R.alive, R.pos, R.step, R.t, R.tfar, S, staged, partial, B, COUNT ? &box_vol : nullptr);
    if (COUNT && lane == 0) {  // diagnostics: box volume of partial/failed chunks, S of staged ones
      if (!staged || partial) atomicAdd(P.steps + 8 + min(box_vol >> 8, 31), 1ull);
      else atomicAdd(P.steps + 40 + (S >= 32 ? 0 : (S >= 16 ? 1 : (S >= 8 ? 2 : 3))), 1ull);
    }
    bool empty = false;
    if (staged) {
      const bool nonzero = stage_box<BIG>(L, E, B, lane);  // always stage: the samples read the slot
      // leap only when the absorption texture is the staged one: a zero emission box says nothing
      // about the opacity of a separate absorption texture (the simEmAb slot path)
      empty = AB_ALIAS && P.skip_empty && !partial && !nonzero;
    }
    __builtin_amdgcn_wave_barrier();
    if (COUNT) ++(staged && !partial ? (empty ? C.leap : C.staged) : C.fall);

    if (empty) {
      leap(P, S, R.alive, R.nsteps, R.t, R.tfar, R.pos, R.step);
      continue;
    }

    // ---- S samples ---------------------------------------------------------------------------
    for (int k = 0; k < S && R.alive; ++k) {
      const f3 pos = R.pos;
      const f3 ps = mk((pos.x - bmin.x) * bsc.x, (pos.y - bmin.y) * bsc.y, (pos.z - bmin.z) * bsc.z);
      // unclamped axes (axis_raw): exact on the LDS path, clamped by fetch_at on the global one
      const Ax ax = axis_raw<NANCHK>(ps.x, E.fnx), ay = axis_raw<NANCHK>(ps.y, E.fny),
               az = axis_raw<NANCHK>(ps.z, E.fnz);
      // centre cell in the slot; the gradient taps below differ from it along one axis only
      const int lx = slot_coord(ax.i, B.rx), ly = slot_coord(ay.i, B.ry), lz = slot_coord(az.i, B.rz);
      const bool inx = in_box(lx, B.ex), iny = in_box(ly, B.ey), inz = in_box(lz, B.ez);
      const int ayz = lz * B.pxy + ly * B.px;  // slot word of (0, ly, lz)
      const int ac = ayz + lx;
      const float em_s = fetch_at<BIG>(E, L, B, staged && inx && iny && inz, ac, ax, ay, az);
      const float ab_s = AB_ALIAS ? em_s : tex3d<BIG>(P.ab, ps.x, ps.y, ps.z);
      const float e = P.fe * em_s;
      const float a = P.fa * ab_s;
      const float alpha = opacity<VR_MARCH_FAST>(a, tstep);
      const float eds = e * tstep;
      float ir = 0.f, ig = 0.f, ib = 0.f;
      const bool skip = P.skip_empty && alpha == 0.f && fabsf(eds) <= 3.0e38f;
      if (COUNT) {
        ++C.iter;
        C.lit += (MODE != 0 && __any(!skip)) ? 1u : 0u;
      }
      if (MODE != 0 && !skip) {
        if (COUNT) ++R.nlit;
        f3 g;
        if (MODE == 1 && (VR_ABLATE & 4)) {
          g = mk(ps.x, ps.y, em_s);
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
        } else if (SHARE2) {
          const Ax cx = clamp_ax(ax, E.nx), cy = clamp_ax(ay, E.ny), cz = clamp_ax(az, E.nz);
          if (P.gvec)
            g = fetch_vec<BIG>(P.gvec, P.gx, cx, cy, cz);
          else
            g = mk(fetch<BIG>(P.gx, cx, cy, cz), fetch<BIG>(P.gy, cx, cy, cz), fetch<BIG>(P.gz, cx, cy, cz));
        } else {
          g = mk(tex3d<BIG>(P.gx, ps.x, ps.y, ps.z), tex3d<BIG>(P.gy, ps.x, ps.y, ps.z),
                 tex3d<BIG>(P.gz, ps.x, ps.y, ps.z));
        }
        const float refl = P.fr * (P.re_is_em ? em_s : tex3d<BIG>(P.re, ps.x, ps.y, ps.z));
        shade_lights<VR_MARCH_FAST>(P, g, pos, R.o, refl, ir, ig, ib);
      }
      const float r = fmaf(eds, P.color[0], ir) * alpha;
      const float gg = fmaf(eds, P.color[1], ig) * alpha;
      const float b = fmaf(eds, P.color[2], ib) * alpha;
      const float om = 1.f - R.sa;
      R.sr = fmaf(om, r, R.sr);
      R.sg = fmaf(om, gg, R.sg);
      R.sb = fmaf(om, b, R.sb);
      R.sa = fmaf(om, alpha, R.sa);
      ++R.nsteps;
      if (R.sa > thr || R.nsteps >= P.max_steps) {
        R.alive = false;
      } else {
        R.t += tstep;
        if (R.t > R.tfar) R.alive = false;
        else R.pos = mk(pos.x + R.step.x, pos.y + R.step.y, pos.z + R.step.z);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

__device__ __forceinline__ bool finite3(const f3 &v) {
  return fabsf(v.x) <= 3.4e38f && fabsf(v.y) <= 3.4e38f && fabsf(v.z) <= 3.4e38f;
}

#ifndef VR_WG_WAVES
#define VR_WG_WAVES 4  // waves per workgroup: a 16x16 block stays on one XCD (1 wave: same speed, 2x HBM traffic)
#endif

// One wave marches one 8x8-pixel tile (lane -> (x = lane >> 3, y = lane & 7)).  Tile t is quadrant
// (t & 3) of 16x16 block (t >> 2), blocks row-major, t = blockIdx.x * VR_WG_WAVES + wave.  With
// single-wave workgroups a wave whose rays end early releases its LDS slot at once instead of
// holding it until the slowest wave of a larger workgroup has finished.
template <int MODE, bool AB_ALIAS, bool COUNT, bool SHARE2, bool BIG, int CAP>
__global__ __launch_bounds__(64 * VR_WG_WAVES) void march_kernel(const RenderParams P) {
  __shared__ float lds[VR_WG_WAVES][CAP];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  float *L = lds[wave];
  const int tile = blockIdx.x * VR_WG_WAVES + wave;
  const int nbx = (P.part_cols + 15) >> 4;
  const int blk16 = tile >> 2, quad = tile & 3;
  const int lc = (blk16 % nbx) * 16 + (quad & 1) * 8 + (lane >> 3);
  const int y = (blk16 / nbx) * 16 + (quad >> 1) * 8 + (lane & 7);
  const bool active = (lc < P.part_cols) && (y < P.height);
  Ray R;
  R.o = mk(0.f, 0.f, 0.f);
  R.pos = R.o;
  R.step = R.o;
  R.t = 0.f;
  R.tfar = -1.f;
  R.sr = R.sg = R.sb = R.sa = 0.f;
  R.nsteps = R.nlit = 0;
  R.alive = false;
  ChunkStats C{0, 0, 0, 0, 0};
  if (active) {
    const int blk = lc / P.block_cols, within = lc - blk * P.block_cols;
    const int x = (P.part + blk * P.num_parts) * P.block_cols + within;
    f3 d;
    float tnear;
    R.alive = ray_setup(P, x, y, R.o, d, tnear, R.tfar);
    R.pos = mk(fmaf(d.x, tnear, R.o.x), fmaf(d.y, tnear, R.o.y), fmaf(d.z, tnear, R.o.z));
    R.step = mk(d.x * P.tstep, d.y * P.tstep, d.z * P.tstep);
    R.t = tnear;
  }
  // every coordinate the march forms from a finite start and step is finite
  if (__all(!R.alive || (finite3(R.pos) && finite3(R.step))))
    march<MODE, AB_ALIAS, COUNT, SHARE2, BIG, false, CAP>(P, L, lane, R, C);
  else
    march<MODE, AB_ALIAS, COUNT, SHARE2, BIG, true, CAP>(P, L, lane, R, C);

  if (active) {
    const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
    const size_t kk = (size_t)lc * (size_t)P.height + (size_t)y;
    P.out[kk] = R.sr;
    P.out[kk + plane] = R.sg;
    P.out[kk + 2 * plane] = R.sb;
  }
  if (COUNT) {
    unsigned long long s = (unsigned long long)R.nsteps, l = (unsigned long long)R.nlit;
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
    }
  }
}

template <int MODE, bool AB, bool SH, int CAP>
static hipError_t launch_c(const RenderParams &P, dim3 grid, hipStream_t s, bool big) {
  const dim3 blk(64 * VR_WG_WAVES);
  if (P.steps) {
    if (big) hipLaunchKernelGGL((march_kernel<MODE, AB, true, SH, true, CAP>), grid, blk, 0, s, P);
    else hipLaunchKernelGGL((march_kernel<MODE, AB, true, SH, false, CAP>), grid, blk, 0, s, P);
  } else {
    if (big) hipLaunchKernelGGL((march_kernel<MODE, AB, false, SH, true, CAP>), grid, blk, 0, s, P);
    else hipLaunchKernelGGL((march_kernel<MODE, AB, false, SH, false, CAP>), grid, blk, 0, s, P);
  }
  return hipGetLastError();
}

template <int MODE, bool AB, bool SH>
static hipError_t launch_m(const RenderParams &P, dim3 grid, hipStream_t s, bool big) {
  return P.wide_slot ? launch_c<MODE, AB, SH, VR_LDS_CAP_WIDE>(P, grid, s, big)
                     : launch_c<MODE, AB, SH, VR_LDS_CAP>(P, grid, s, big);
}

// Host entry: the staged kernel needs a bound, non-constant emission texture; for MODE 1 the
// gradient texture must be the emission texture itself (the reference's tex_emission binding).
hipError_t launch_march(const RenderParams &P, int mode, bool ab_alias, bool share, bool big, hipStream_t s) {
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  const uint64_t tiles = (uint64_t)((P.part_cols + 15) / 16) * (uint64_t)((P.height + 15) / 16) * 4;
  const dim3 grid((unsigned)((tiles + VR_WG_WAVES - 1) / VR_WG_WAVES));
  switch (mode) {
    case 0: return ab_alias ? launch_m<0, true, false>(P, grid, s, big) : launch_m<0, false, false>(P, grid, s, big);
    case 1: return ab_alias ? launch_m<1, true, false>(P, grid, s, big) : launch_m<1, false, false>(P, grid, s, big);
    default:
      if (share) return ab_alias ? launch_m<2, true, true>(P, grid, s, big) : launch_m<2, false, true>(P, grid, s, big);
      return ab_alias ? launch_m<2, true, false>(P, grid, s, big) : launch_m<2, false, false>(P, grid, s, big);
  }
}

}  // namespace fast / exact
}  // namespace vr
