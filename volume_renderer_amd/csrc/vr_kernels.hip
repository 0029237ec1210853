// vr_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the volume ray-marcher.
//
// render_kernel: one lane per primary ray, a wave = an 8x8-pixel tile, a 256-thread workgroup =
// 16x16 pixels.  Front-to-back emission/absorption compositing with early ray termination,
// software trilinear sampling with the CUDA linear-filter semantics of the reference's tex3D
// (/root/reference/src/C/vr/volumeRender_kernel.cu:544-548), on-the-fly (:212-253) or lookup
// (:266-276) gradient, Henyey-Greenstein LUT shading per light (:308-353).
//
// Numerics: the ray set-up, the march recurrences (t += tstep, pos += step), the
// sample coordinates, the 8-bit filter weights and the lerps follow the oracle op for op (explicit
// fmaf, -ffp-contract=off), so sample positions and texel fetches are bit-identical to the oracle.
// Shading: FAST (the default) forms the angle cosines with the hardware reciprocal square root and
// __expf as exp2 (vr_sampling.h shade_lights / opacity); FAST = false is the oracle's op sequence
// with correctly rounded sqrt/div, only expf/acosf from the device math library.
//
// Memory: volumes live in the apron layout of vr_device.h, so every trilinear fetch
// is 4 x global_load_dwordx2 (one per (y,z) row of the 2x2x2 cell) with no per-tap clamping; the
// six gradient taps reuse the centre sample's weights on the two unshifted axes; a 1x1x1 texture
// (the class default VolumeReflection = Volume(1)) is one scalar load.  Samples whose opacity is
// exactly 0 contribute exactly 0 and skip gradient+shading when the host has proven every other
// term finite (skip_empty).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <math.h>

#include "vr_device.h"
#include "vr_sampling.h"

namespace vr {

// MODE 0: no light sources (shade() contributes exactly 0); 1: on-the-fly gradient; 2: lookup.
// SHARE: the gradient texture(s) have the emission texture's dims, so the unshifted axes of the
// gradient taps (MODE 1) / all axes of the lookups (MODE 2) are the centre sample's.
template <int MODE, bool AB_ALIAS, bool BIG, bool COUNT, bool SHARE, bool FAST>
__global__ __launch_bounds__(256, VR_MIN_WAVES) void render_kernel(const RenderParams P) {
  // 16x16 pixel workgroup tile; wave w owns the 8x8 quadrant (w & 1, w >> 1); lane -> (x, y)
  // with y fastest so that the column-major output stores of a lane octet are contiguous.
  int tx, ty;
  if (!tile_of_block(P, tx, ty)) return;  // whole workgroup: uniform
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = tx * 16 + (wave & 1) * 8 + (lane >> 3);  // local (partition) column
  const int y = ty * 16 + (wave >> 1) * 8 + (lane & 7);
  const bool active = (lc < P.part_cols) && (y < P.height);
  int32_t nsteps = 0, nlit = 0;
  if (active) {
    const int blk = lc / P.block_cols, within = lc - blk * P.block_cols;
    const int x = (P.part + blk * P.num_parts) * P.block_cols + within;

    f3 o, d;
    float tnear, tfar;
    const bool hit = ray_setup(P, x, y, o, d, tnear, tfar);  // volumeRender_kernel.cu:388-425
    const f3 bmin = mk(P.bmin[0], P.bmin[1], P.bmin[2]);

    float sr = 0.f, sg = 0.f, sb = 0.f, sa = 0.f;
    if (hit) {
      const float tstep = P.tstep, thr = P.thr;
      const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
      f3 pos = mk(fmaf(d.x, tnear, o.x), fmaf(d.y, tnear, o.y), fmaf(d.z, tnear, o.z));
      const f3 step = mk(d.x * tstep, d.y * tstep, d.z * tstep);
      float t = tnear;
      for (;;) {
        const f3 ps = mk((pos.x - bmin.x) * bsc.x, (pos.y - bmin.y) * bsc.y, (pos.z - bmin.z) * bsc.z);
        // centre sample (emission slot; absorption aliases it unless the slots differ)
        float em_s = 0.f;
        Ax ax{0, 0.f}, ay{0, 0.f}, az{0, 0.f};
        if (P.em.p != nullptr) {
          if (P.em.one) {
            const float q = P.em.p[0];
            em_s = fmaf(0.5f, q - q, q);
          } else {
            ax = axis(ps.x, P.em.nx, P.em.fnx);
            ay = axis(ps.y, P.em.ny, P.em.fny);
            az = axis(ps.z, P.em.nz, P.em.fnz);
            em_s = fetch<BIG>(P.em, ax, ay, az);
          }
        }
        const float ab_s = AB_ALIAS ? em_s : tex3d<BIG>(P.ab, ps.x, ps.y, ps.z);
        const float e = P.fe * em_s;
        const float a = P.fa * ab_s;
        const float alpha = opacity<FAST>(a, tstep);
        const float eds = e * tstep;
        float ir = 0.f, ig = 0.f, ib = 0.f;
        // opacity exactly 0 and a finite emission term: the sample adds exactly 0 (every other
        // term is finite by the host's scan), so gradient and shading are skipped.
        const bool skip = P.skip_empty && alpha == 0.f && fabsf(eds) <= 3.0e38f;
        if (MODE != 0 && !skip) {
          if (COUNT) ++nlit;
          f3 g;
          if (MODE == 1) {
            const float xp = ((pos.x + P.gstep[0]) - bmin.x) * bsc.x;
            const float xm = ((pos.x - P.gstep[0]) - bmin.x) * bsc.x;
            const float yp = ((pos.y + P.gstep[1]) - bmin.y) * bsc.y;
            const float ym = ((pos.y - P.gstep[1]) - bmin.y) * bsc.y;
            const float zp = ((pos.z + P.gstep[2]) - bmin.z) * bsc.z;
            const float zm = ((pos.z - P.gstep[2]) - bmin.z) * bsc.z;
            if (SHARE && FAST && P.tap_half) {  // half-texel taps derived from the centre (vr_march.hip)
              const DevTex &T = P.gem;
              Ax p, m;
              half_taps(axis_raw_s(ps.x, T.fnx), p, m);
              g.x = fetch<BIG>(T, clamp_ax(p, T.nx), ay, az) - fetch<BIG>(T, clamp_ax(m, T.nx), ay, az);
              half_taps(axis_raw_s(ps.y, T.fny), p, m);
              g.y = fetch<BIG>(T, ax, clamp_ax(p, T.ny), az) - fetch<BIG>(T, ax, clamp_ax(m, T.ny), az);
              half_taps(axis_raw_s(ps.z, T.fnz), p, m);
              g.z = fetch<BIG>(T, ax, ay, clamp_ax(p, T.nz)) - fetch<BIG>(T, ax, ay, clamp_ax(m, T.nz));
            } else if (SHARE) {  // gem == em: reuse the centre's axes on the unshifted coordinates
              const DevTex &T = P.gem;
              g.x = fetch<BIG>(T, axis(xp, T.nx, T.fnx), ay, az) - fetch<BIG>(T, axis(xm, T.nx, T.fnx), ay, az);
              g.y = fetch<BIG>(T, ax, axis(yp, T.ny, T.fny), az) - fetch<BIG>(T, ax, axis(ym, T.ny, T.fny), az);
              g.z = fetch<BIG>(T, ax, ay, axis(zp, T.nz, T.fnz)) - fetch<BIG>(T, ax, ay, axis(zm, T.nz, T.fnz));
            } else {
              g.x = tex3d<BIG>(P.gem, xp, ps.y, ps.z) - tex3d<BIG>(P.gem, xm, ps.y, ps.z);
              g.y = tex3d<BIG>(P.gem, ps.x, yp, ps.z) - tex3d<BIG>(P.gem, ps.x, ym, ps.z);
              g.z = tex3d<BIG>(P.gem, ps.x, ps.y, zp) - tex3d<BIG>(P.gem, ps.x, ps.y, zm);
            }
            g = mk(g.x * 0.5f, g.y * 0.5f, g.z * 0.5f);
          } else {
            if (SHARE)
              g = mk(fetch<BIG>(P.gx, ax, ay, az), fetch<BIG>(P.gy, ax, ay, az), fetch<BIG>(P.gz, ax, ay, az));
            else
              g = mk(tex3d<BIG>(P.gx, ps.x, ps.y, ps.z), tex3d<BIG>(P.gy, ps.x, ps.y, ps.z),
                     tex3d<BIG>(P.gz, ps.x, ps.y, ps.z));
          }
          const float refl = P.fr * (P.re_is_em ? em_s : tex3d<BIG>(P.re, ps.x, ps.y, ps.z));
          shade_lights<FAST>(P, g, pos, o, refl, ir, ig, ib);
        }
        const float r = fmaf(eds, P.color[0], ir) * alpha;
        const float gg = fmaf(eds, P.color[1], ig) * alpha;
        const float b = fmaf(eds, P.color[2], ib) * alpha;
        const float om = 1.f - sa;
        sr = fmaf(om, r, sr);
        sg = fmaf(om, gg, sg);
        sb = fmaf(om, b, sb);
        sa = fmaf(om, alpha, sa);
        ++nsteps;
        if (sa > thr) break;
        if (nsteps >= P.max_steps) break;
        t += tstep;
        if (t > tfar) break;
        pos = mk(pos.x + step.x, pos.y + step.y, pos.z + step.z);
      }
    }
    // column-major planar output of this partition, kernel.cu:496-506 (misses write 0 here:
    // the reference memsets the buffer, volumeRender.cpp:271)
    const size_t plane = (size_t)P.plane_cols * (size_t)P.height;
    const size_t k = (size_t)lc * (size_t)P.height + (size_t)y;
    P.out[k] = sr;
    P.out[k + plane] = sg;
    P.out[k + 2 * plane] = sb;
  }
  if (COUNT) {  // steps[0] += samples, steps[1] += samples that ran gradient + shading
    unsigned long long s = (unsigned long long)nsteps, l = (unsigned long long)nlit;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      s += __shfl_xor(s, off, 64);
      l += __shfl_xor(l, off, 64);
    }
    if (lane == 0 && s) atomicAdd(P.steps, s);
    if (lane == 0 && l) atomicAdd(P.steps + 1, l);
  }
}

// Scatter num_parts gathered partition images into the full [H, W, 3] image.
__global__ __launch_bounds__(256) void assemble_kernel(const float *__restrict__ parts, int64_t w,
                                                       int64_t h, int32_t bc, int32_t np,
                                                       int64_t max_cols, float *__restrict__ out) {
  const int64_t total = w * h;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t x = i / h, y = i - x * h;
    const int64_t b = x / bc, within = x - b * bc;
    const int64_t p = b % np, j = b / np;
    const int64_t lc = j * bc + within;
    const float *src = parts + (size_t)p * (size_t)(max_cols * h * 3);
    const size_t plane_in = (size_t)max_cols * h;
    const size_t k = (size_t)lc * h + y;
    out[i] = src[k];
    out[i + total] = src[k + plane_in];
    out[i + 2 * total] = src[k + 2 * plane_in];
  }
}

// V_shell(n), SURVEY.md 8d: normalized voxel centres x=(i+.5)/n ..., r = |(x,y,z) - .5|,
// v = clamp(1 - |r - .32|/.14, 0, 1) * (.6 + .4 sin(6 pi x) sin(6 pi y) sin(6 pi z))
//     + .05 (x + 2y + 3z)/6 [v > 0]
__global__ __launch_bounds__(256) void synth_shell_kernel(float *__restrict__ out, uint64_t n, uint64_t z_first,
                                                          uint64_t nz) {
  const uint64_t total = n * n * nz;
  const double inv = 1.0 / (double)n;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = i % n, bq = i / n, b = bq % n, c = bq / n + z_first;
    const double x = (a + 0.5) * inv, y = (b + 0.5) * inv, z = (c + 0.5) * inv;
    const double dx = x - 0.5, dy = y - 0.5, dz = z - 0.5;
    const double r = sqrt(dx * dx + dy * dy + dz * dz);
    double v = 1.0 - fabs(r - 0.32) / 0.14;
    v = v < 0.0 ? 0.0 : (v > 1.0 ? 1.0 : v);
    if (v > 0.0) {
      const double tp = 6.0 * M_PI;
      v = v * (0.6 + 0.4 * sin(tp * x) * sin(tp * y) * sin(tp * z)) + 0.05 * (x + 2.0 * y + 3.0 * z) / 6.0;
    }
    out[i] = (float)v;
  }
}

// ---- upload into the apron layout ------------------------------------------------------------

// Copy a dense column-major nx*ny*nz volume into the padded buffer, writing the replicated apron in
// the same pass: padded voxel (i, j, k) = T[clamp(i-1)][clamp(j-1)][clamp(k-1)].
__global__ __launch_bounds__(256) void pad_volume_kernel(const float *__restrict__ src, float *__restrict__ dst,
                                                         int32_t nx, int32_t ny, int32_t nz) {
  const uint64_t px = (uint64_t)nx + 2, py = (uint64_t)ny + 2, pz = (uint64_t)nz + 2;
  const uint64_t total = px * py * pz;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = q % px, r = q / px, j = r % py, k = r / py;
    const uint64_t si = i == 0 ? 0 : (i > (uint64_t)nx ? (uint64_t)nx - 1 : i - 1);
    const uint64_t sj = j == 0 ? 0 : (j > (uint64_t)ny ? (uint64_t)ny - 1 : j - 1);
    const uint64_t sk = k == 0 ? 0 : (k > (uint64_t)nz ? (uint64_t)nz - 1 : k - 1);
    dst[q] = src[(sk * (uint64_t)ny + sj) * (uint64_t)nx + si];
  }
}

// Padded planes [k0, k1) of the apron layout (vr_device.h) from source planes [z0, ...) held at src
// (a chunk of the volume, or the whole of it), one padded row per workgroup iteration: a coalesced
// read of the source row, a coalesced write of the padded row with its two border copies; the
// statistics of the written values (nonfinite flag, max |x| -- border copies repeat interior
// values, so they change neither) are folded in on the way (the upload path, vr_resources.h).
__global__ __launch_bounds__(256) void pad_planes_kernel(const float *__restrict__ src, int64_t z0, int32_t nx,
                                                         int32_t ny, int32_t nz, float *__restrict__ dst, int64_t k0,
                                                         uint64_t rows, BufStats *st) {
  const uint64_t px = (uint64_t)nx + 2, py = (uint64_t)ny + 2;
  uint32_t bad = 0;
  float mx = 0.f;
  for (uint64_t row = blockIdx.x; row < rows; row += gridDim.x) {
    const uint64_t k = (uint64_t)k0 + row / py;
    const int64_t j = (int64_t)(row % py);
    const int64_t kk = (int64_t)k - 1, jj = j - 1;
    const int64_t sk = (kk < 0 ? 0 : (kk > (int64_t)nz - 1 ? (int64_t)nz - 1 : kk)) - z0;
    const int64_t sj = jj < 0 ? 0 : (jj > (int64_t)ny - 1 ? (int64_t)ny - 1 : jj);
    const float *s = src + ((uint64_t)sk * (uint64_t)ny + (uint64_t)sj) * (uint64_t)nx;
    float *d = dst + (k * py + (uint64_t)j) * px;
    for (uint32_t i = threadIdx.x; i < px; i += blockDim.x) {
      const uint32_t si = i == 0 ? 0u : (i > (uint32_t)nx ? (uint32_t)nx - 1 : i - 1);
      const float v = s[si];
      d[i] = v;
      if (!(fabsf(v) <= 3.4028234e38f)) bad = 1;
      else mx = fmaxf(mx, fabsf(v));
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    bad |= __shfl_xor(bad, off, 64);
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  __shared__ uint32_t sb[4];
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = bad;
    sm[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t bb = sb[0] | sb[1] | sb[2] | sb[3];
    const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    if (bb) atomicOr(&st->nonfinite, 1u);
    atomicMax(reinterpret_cast<unsigned int *>(&st->maxabs), __float_as_uint(m));  // m >= 0
  }
}

// nonfinite flag and max |x| of a dense buffer (one atomic pair per workgroup)
__global__ __launch_bounds__(256) void stats_kernel(const float *__restrict__ src, uint64_t n, BufStats *st) {
  uint32_t bad = 0;
  float mx = 0.f;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const float v = src[q];
    if (!(fabsf(v) <= 3.4028234e38f)) bad = 1;
    else mx = fmaxf(mx, fabsf(v));
  }
  for (int off = 32; off > 0; off >>= 1) {
    bad |= __shfl_xor(bad, off, 64);
    mx = fmaxf(mx, __shfl_xor(mx, off, 64));
  }
  __shared__ uint32_t sb[4];
  __shared__ float sm[4];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = bad;
    sm[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t bb = sb[0] | sb[1] | sb[2] | sb[3];
    const float m = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
    if (bb) atomicOr(&st->nonfinite, 1u);
    atomicMax(reinterpret_cast<unsigned int *>(&st->maxabs), __float_as_uint(m));  // m >= 0
  }
}

// ------------------------------------------------------------------------------------------------
// launch helpers (called from vr_capi.hip)

template <int MODE, bool AB, bool BIG, bool SH>
static hipError_t launch4(const RenderParams &P, dim3 grid, hipStream_t s) {
  if (P.fast_shade) {
    if (P.steps)
      hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, true, SH, true>), grid, dim3(256), 0, s, P);
    else
      hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, false, SH, true>), grid, dim3(256), 0, s, P);
  } else {
    if (P.steps)
      hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, true, SH, false>), grid, dim3(256), 0, s, P);
    else
      hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, false, SH, false>), grid, dim3(256), 0, s, P);
  }
  return hipGetLastError();
}

template <int MODE, bool AB>
static hipError_t launch3(const RenderParams &P, bool big, bool share, dim3 grid, hipStream_t s) {
  if (big) return share ? launch4<MODE, AB, true, true>(P, grid, s) : launch4<MODE, AB, true, false>(P, grid, s);
  return share ? launch4<MODE, AB, false, true>(P, grid, s) : launch4<MODE, AB, false, false>(P, grid, s);
}

template <int MODE>
static hipError_t launch2(const RenderParams &P, bool ab_alias, bool big, bool share, dim3 grid, hipStream_t s) {
  return ab_alias ? launch3<MODE, true>(P, big, share, grid, s) : launch3<MODE, false>(P, big, share, grid, s);
}

hipError_t launch_render(const RenderParams &P, int mode, bool ab_alias, bool big, bool share, hipStream_t s) {
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  const uint64_t ntx = (P.part_cols + 15) / 16, nty = (P.height + 15) / 16;
  uint64_t blocks = ntx * nty;
  if (P.tile_mode == 1) {
    const uint64_t nsuper = ((ntx + 7) / 8) * ((nty + 7) / 8);
    blocks = ((nsuper + 7) / 8) * 512;
  }
  dim3 grid((unsigned)blocks);
  switch (mode) {
    case 0: return launch2<0>(P, ab_alias, big, false, grid, s);
    case 1: return launch2<1>(P, ab_alias, big, share, grid, s);
    default: return launch2<2>(P, ab_alias, big, share, grid, s);
  }
}

hipError_t launch_assemble(const float *parts, int64_t w, int64_t h, int32_t bc, int32_t np,
                           int64_t max_cols, float *out, hipStream_t s) {
  const int64_t total = w * h;
  if (total <= 0) return hipSuccess;
  int64_t blocks = (total + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(assemble_kernel, dim3((unsigned)blocks), dim3(256), 0, s, parts, w, h, bc, np,
                     max_cols, out);
  return hipGetLastError();
}

// MATLAB [gx, gy, gz] = gradient(Data) for single Data(d0, d1, d2) (Volume.m:181-205): gx along
// dim 2 (d1), gy along dim 1 (d0), gz along dim 3 (d2); (f(i+1) - f(i-1)) / 2 inside, one-sided
// differences at the ends, 0 along a dimension of extent 1.  fp32 like MATLAB's single gradient:
// bit-identical to the numpy restatement (oracle.matlab_gradient).  One thread per voxel, x
// fastest: the three neighbour pairs are coalesced rows / L2-resident planes.
__device__ __forceinline__ float grad1(const float *p, uint64_t i, uint64_t stride, uint32_t c, uint32_t n) {
  if (n < 2) return 0.f;
  if (c == 0) return p[i + stride] - p[i];
  if (c == n - 1) return p[i] - p[i - stride];
  return (p[i + stride] - p[i - stride]) / 2.f;
}

__global__ __launch_bounds__(256) void gradient_kernel(const float *__restrict__ d, uint32_t n0, uint32_t n1,
                                                       uint32_t n2, float *__restrict__ gx,
                                                       float *__restrict__ gy, float *__restrict__ gz) {
  const uint64_t total = (uint64_t)n0 * n1 * n2, plane = (uint64_t)n0 * n1;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < total;
       q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t k = q / plane, r = q - k * plane;
    const uint32_t j = (uint32_t)(r / n0), i = (uint32_t)(r - (uint64_t)j * n0);
    gy[q] = grad1(d, q, 1, i, n0);
    gx[q] = grad1(d, q, n0, j, n1);
    gz[q] = grad1(d, q, plane, (uint32_t)k, n2);
  }
}

hipError_t launch_gradient(const float *d, const uint64_t dims[3], float *gx, float *gy, float *gz, hipStream_t s) {
  const uint64_t total = dims[0] * dims[1] * dims[2];
  if (!total) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 262144) blocks = 262144;
  hipLaunchKernelGGL(gradient_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d, (uint32_t)dims[0],
                     (uint32_t)dims[1], (uint32_t)dims[2], gx, gy, gz);
  return hipGetLastError();
}

// out[e] = (a, b, c, 0) of padded voxel e: rows of the padded volume, or (VR_GVEC_BRICK) 2x2x2
// bricks, entry ((Z/2 * by + Y/2) * bx + X/2) * 8 + (X&1) + 2 (Y&1) + 4 (Z&1) (vr_sampling.h
// fetch_vec), the bricks past an odd padded edge zero-filled.
__global__ __launch_bounds__(256) void interleave3_kernel(const float *__restrict__ a, const float *__restrict__ b,
                                                          const float *__restrict__ c, float4 *__restrict__ out,
                                                          uint64_t n, uint32_t px, uint32_t py, uint32_t pz) {
  const uint32_t bx = (px + 1) >> 1, by = (py + 1) >> 1;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t src = i;
    if (VR_GVEC_BRICK) {
      const uint64_t brick = i >> 3, e = i & 7u;
      const uint64_t bz = brick / ((uint64_t)bx * by), rem = brick - bz * bx * by;
      const uint32_t byi = (uint32_t)(rem / bx), bxi = (uint32_t)(rem - (uint64_t)byi * bx);
      const uint32_t X = 2u * bxi + (uint32_t)(e & 1u), Y = 2u * byi + (uint32_t)((e >> 1) & 1u);
      const uint64_t Z = 2u * bz + (e >> 2);
      if (X >= px || Y >= py || Z >= pz) {
        out[i] = make_float4(0.f, 0.f, 0.f, 0.f);
        continue;
      }
      src = (Z * py + Y) * px + X;
    }
    out[i] = make_float4(a[src], b[src], c[src], 0.f);
  }
}

// Entries of the interleaved lookup gradient of a padded px x py x pz volume.
uint64_t interleave3_entries(uint32_t px, uint32_t py, uint32_t pz) {
  if (!VR_GVEC_BRICK) return (uint64_t)px * py * pz;
  return 8ull * ((px + 1) >> 1) * ((py + 1) >> 1) * ((pz + 1) >> 1);
}

// out: interleave3_entries entries (gx, gy, gz, 0) of the lookup gradient (RenderParams::gvec).
// (Round 4 also measured a z-paired and a packed 12-byte layout, both slower; removed in round 5.)
hipError_t launch_interleave3(const float *a, const float *b, const float *c, float *out, uint32_t px,
                              uint32_t py, uint32_t pz, hipStream_t s) {
  const uint64_t n = interleave3_entries(px, py, pz);
  if (!n) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 262144) blocks = 262144;
  hipLaunchKernelGGL(interleave3_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, b, c,
                     reinterpret_cast<float4 *>(out), n, px, py, pz);
  return hipGetLastError();
}

// Channel sum of a multi-channel frame (vr_render_channels): out[e][i] = in[0][e][i] + in[1][e][i]
// + ... in channel order, i.e. MATLAB's `main + structure` (example3.m:239) on the views' images
// (nv views per channel, img floats each).
__global__ void sum_channels_kernel(const float *__restrict__ in, uint32_t nch, uint32_t nv, uint64_t img,
                                    float *__restrict__ out) {
  const uint64_t n = img * nv;
  for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < n; k += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t e = k / img, i = k - e * img;
    float acc = in[e * img + i];
    for (uint32_t c = 1; c < nch; ++c) acc = acc + in[((uint64_t)c * nv + e) * img + i];
    out[k] = acc;
  }
}

hipError_t launch_sum_channels(const float *in, uint32_t nch, uint32_t nv, uint64_t img, float *out, hipStream_t s) {
  const uint64_t n = img * nv;
  if (!n || !nch) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(sum_channels_kernel, dim3((unsigned)blocks), dim3(256), 0, s, in, nch, nv, img, out);
  return hipGetLastError();
}

// Longest-first schedule of the march workgroups: order[] lists the tile blocks by
// their last measured duration, longest first, in 256 log-spaced buckets (8 per octave; order
// within a bucket is arbitrary).  The march writes the same image for any order.  One workgroup.
__device__ __forceinline__ uint32_t cost_bucket(uint32_t c) {
  if (c == 0) return 0;
  const uint32_t lz = __clz(c), e = 31u - lz;                        // floor(log2 c)
  const uint32_t m = e >= 3 ? (c >> (e - 3)) & 7u : (c << (3 - e)) & 7u;  // next 3 bits
  return min(255u, e * 8u + m);
}

__global__ __launch_bounds__(1024) void order_kernel(const uint32_t *__restrict__ cost, uint32_t n,
                                                     uint32_t *__restrict__ order) {
  __shared__ uint32_t hist[256];
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) atomicAdd(&hist[cost_bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive offsets, largest bucket first
    uint32_t acc = 0;
    for (int b = 255; b >= 0; --b) {
      const uint32_t c = hist[b];
      hist[b] = acc;
      acc += c;
    }
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) order[atomicAdd(&hist[cost_bucket(cost[i])], 1u)] = i;
}

// Full-frame schedule: the heavy blocks (measured duration >= max / div) first, longest first, then
// every other block in ascending (row-major) order -- the bulk keeps the L2 locality of
// neighbouring tiles running together, and no heavy block starts late enough to form the tail.
// tail_pct / wg_slots: only when the longest block lasts at least tail_pct % of the packed frame
// (sum of durations / resident workgroups) does it risk forming a tail; otherwise the order is
// plain row-major.
__global__ __launch_bounds__(1024) void order_heavy_kernel(const uint32_t *__restrict__ cost, uint32_t n,
                                                           uint32_t div, uint32_t tail_pct, uint32_t wg_slots,
                                                           uint32_t *__restrict__ order) {
  __shared__ uint32_t hist[256];
  __shared__ uint32_t scan[1024];
  __shared__ uint32_t smax, nheavy, base;
  __shared__ unsigned long long ssum;
  if (threadIdx.x == 0) {
    smax = 0;
    nheavy = 0;
    ssum = 0;
  }
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) hist[i] = 0;
  __syncthreads();
  uint32_t m = 0;
  unsigned long long sum = 0;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    m = max(m, cost[i]);
    sum += cost[i];
  }
  atomicMax(&smax, m);
  atomicAdd(&ssum, sum);
  __syncthreads();
  const unsigned long long packed = ssum / (unsigned long long)max(wg_slots, 1u);
  const bool tail = (unsigned long long)smax * 100ull >= packed * (unsigned long long)tail_pct;
  // no tail: every block "light", i.e. row-major
  const uint32_t thr = tail ? max(smax / max(div, 1u), 1u) : 0xffffffffu;
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (cost[i] >= thr) atomicAdd(&hist[cost_bucket(cost[i])], 1u);
  __syncthreads();
  if (threadIdx.x == 0) {  // exclusive offsets of the heavy blocks, largest bucket first
    uint32_t acc = 0;
    for (int b = 255; b >= 0; --b) {
      const uint32_t c = hist[b];
      hist[b] = acc;
      acc += c;
    }
    nheavy = acc;
    base = acc;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x)
    if (cost[i] >= thr) order[atomicAdd(&hist[cost_bucket(cost[i])], 1u)] = i;
  // the rest in ascending block order: a block-wide exclusive scan per chunk of 1024 blocks
  for (uint32_t c0 = 0; c0 < n; c0 += blockDim.x) {
    const uint32_t i = c0 + threadIdx.x;
    const uint32_t f = (i < n && cost[i] < thr) ? 1u : 0u;
    scan[threadIdx.x] = f;
    __syncthreads();
    for (uint32_t off = 1; off < blockDim.x; off <<= 1) {
      const uint32_t v = threadIdx.x >= off ? scan[threadIdx.x - off] : 0u;
      __syncthreads();
      scan[threadIdx.x] += v;
      __syncthreads();
    }
    if (f) order[base + scan[threadIdx.x] - 1u] = i;
    __syncthreads();
    if (threadIdx.x == blockDim.x - 1) base += scan[threadIdx.x];
    __syncthreads();
  }
  (void)nheavy;
}

// heavy_div 0: longest first (short launches); else the full-frame order of order_heavy_kernel
// with tail = (tail_pct << 32) | resident workgroups.
hipError_t launch_order(const uint32_t *cost, uint32_t n, uint32_t *order, hipStream_t s, uint32_t heavy_div,
                        uint64_t tail) {
  if (!n) return hipSuccess;
  if (heavy_div)
    hipLaunchKernelGGL(order_heavy_kernel, dim3(1), dim3(1024), 0, s, cost, n, heavy_div, (uint32_t)(tail >> 32),
                       (uint32_t)tail, order);
  else hipLaunchKernelGGL(order_kernel, dim3(1), dim3(1024), 0, s, cost, n, order);
  return hipGetLastError();
}

__global__ __launch_bounds__(256) void iota_kernel(uint32_t *__restrict__ order, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) order[i] = i;
}

hipError_t launch_iota(uint32_t *order, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(iota_kernel, dim3((n + 255) / 256), dim3(256), 0, s, order, n);
  return hipGetLastError();
}

hipError_t launch_synth_shell(float *out, uint64_t n, uint64_t z_first, uint64_t nz, hipStream_t s) {
  const uint64_t total = n * n * nz;
  if (!total) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(synth_shell_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, n, z_first, nz);
  return hipGetLastError();
}

hipError_t launch_pad(const float *src, float *dst, int32_t nx, int32_t ny, int32_t nz, hipStream_t s) {
  const uint64_t total = ((uint64_t)nx + 2) * ((uint64_t)ny + 2) * ((uint64_t)nz + 2);
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(pad_volume_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, nx, ny, nz);
  return hipGetLastError();
}

hipError_t launch_pad_planes(const float *src, int64_t z0, int32_t nx, int32_t ny, int32_t nz, float *dst, int64_t k0,
                             int64_t k1, BufStats *st, hipStream_t s) {
  const uint64_t rows = (uint64_t)(k1 - k0) * ((uint64_t)ny + 2);
  if (!rows || nx <= 0 || ny <= 0 || nz <= 0) return hipSuccess;
  // a few workgroups per CU that loop over rows: few dispatches, so an upload that runs beside a
  // render (which holds most CU slots) is not held back by workgroup dispatch
  const uint64_t blocks = rows < 2048 ? rows : 2048;
  hipLaunchKernelGGL(pad_planes_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, z0, nx, ny, nz, dst, k0, rows, st);
  return hipGetLastError();
}

// The z-paired copy of a small padded texture (the illumination LUT, fetch_small_z): entry i holds
// voxel i and its +z neighbour i + pxy (itself in the last plane, which no lookup's lower corner is
// in), so one 16-byte load at entry i gives the x-pair of two consecutive planes.
__global__ void zpair_kernel(const float *src, float *dst, uint32_t n, uint32_t pxy) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = src[i], b = i + pxy < n ? src[i + pxy] : a;
  reinterpret_cast<float2 *>(dst)[i] = make_float2(a, b);
}

// Occupancy map of a padded (apron-layout) volume for the march's empty-space probe (vr_stage.h
// probe_run): one byte per 8x8x8 brick, 1 when any voxel of the brick is non-zero (NaN included,
// +-0 not: the test the staging copy applies to its box, vr_stage.h stage_box).  A workgroup takes a
// 256-voxel run of x in one (y, z) brick row and ORs its 64 rows (coalesced 1 KiB row loads); eight
// consecutive lanes then hold one brick.
__global__ __launch_bounds__(256) void occupancy_kernel(const float *__restrict__ p, uint32_t px, uint32_t py,
                                                        uint32_t pz, uint8_t *__restrict__ occ, uint32_t obx,
                                                        uint32_t oby, float inv_scale) {
  constexpr uint32_t E = 1u << VR_OCC_LOG;  // brick edge
  const uint32_t x = blockIdx.x * 256u + threadIdx.x;
  const uint32_t by = blockIdx.y, bz = blockIdx.z;
  uint32_t acc = 0;
  float sum = 0.f;
  if (x < px) {
    const uint64_t pxy = (uint64_t)px * py;
#pragma unroll 8
    for (uint32_t k = 0; k < E * E; ++k) {
      const uint32_t y = by * E + (k & (E - 1)), z = bz * E + (k >> VR_OCC_LOG);
      if (y < py && z < pz) {
        const uint32_t u = __float_as_uint(p[(uint64_t)z * pxy + (uint64_t)y * px + x]) & 0x7fffffffu;
        acc |= u;
        sum += __uint_as_float(u);
      }
    }
  }
#pragma unroll
  for (uint32_t m = 1; m < E; m <<= 1) {
    acc |= (uint32_t)__shfl_xor((int)acc, (int)m, 64);
    sum += __shfl_xor(sum, (int)m, 64);
  }
  // the byte: 0 iff every voxel is +-0 (what the probe tests); otherwise the brick's mean |voxel| in
  // 1/255 of the volume's largest (1 at least; 255 for NaN / inf), the schedule predictor's density
  if ((threadIdx.x & (E - 1)) == 0 && x < px) {
    uint8_t q = 0;
    if (acc != 0u) {
      const float m = sum * (1.f / (float)(E * E * E)) * inv_scale;
      q = (m == m && m < 254.5f) ? (uint8_t)fmaxf(1.f, ceilf(m)) : (uint8_t)255;
    }
    occ[((uint64_t)bz * oby + by) * obx + (x >> VR_OCC_LOG)] = q;
  }
}

// inv_scale: 255 / the volume's largest |voxel| (0 if unknown: every occupied brick reads 1)
hipError_t launch_occupancy(const float *p, uint32_t px, uint32_t py, uint32_t pz, uint8_t *occ, float inv_scale,
                            hipStream_t s) {
  if (!px || !py || !pz) return hipSuccess;
  constexpr uint32_t E = 1u << VR_OCC_LOG;
  const uint32_t obx = (px + E - 1) / E, oby = (py + E - 1) / E, obz = (pz + E - 1) / E;
  if (oby > 65535 || obz > 65535) return hipErrorInvalidValue;
  hipLaunchKernelGGL(occupancy_kernel, dim3((px + 255) / 256, oby, obz), dim3(256), 0, s, p, px, py, pz, occ, obx,
                     oby, inv_scale);
  return hipGetLastError();
}

// Predicted block costs (round 6, DESIGN.md s5 "history-free schedule"): the cost of march tile
// block b (workgroup b of the launch; views x nb_view blocks, view-major) from the emission
// texture's occupancy map alone -- no earlier frame of the same camera needed.  A block lasts as
// long as its slowest wave; a wave iterates in lockstep over its rays' sample indices until its
// last ray ends, and an iteration is cheap when none of its rays' samples is in an occupied brick
// (the probe leaps up to 512 such samples at a time) and costly when any is (staged taps, gradient,
// shading for the whole wave).  So one predictor wave per block walks 16 rays of each of the
// block's four march waves (a 4 x 4 grid over each wave's tile) through the map in lockstep, m
// samples (~8 texels) per step: per march wave it counts the steps where any of its rays is alive
// and, VR_PRED_W_OCC times over, the steps where any of them is in an occupied brick; a ray ends at
// its exit from the box or where the optical depth of the bricks' mean densities (Fa x mean |v| x
// tstep per sample) reaches the early-exit threshold -log(1 - thr).  The block's cost is its most
// costly wave's.  Only the order of the blocks follows from it: the image is the same for any order.
#ifndef VR_PRED_W_OCC
#define VR_PRED_W_OCC 16
#endif
__global__ __launch_bounds__(256) void predict_cost_kernel(const RenderParams P, uint32_t nb_view, uint32_t nbx,
                                                           int32_t tw, int32_t th, int32_t m, float dens, float xthr,
                                                           uint32_t *__restrict__ cost) {
  const uint32_t b = (blockIdx.x * 256u + threadIdx.x) >> 6;  // the tile block (wave-uniform)
  const int lane = (int)(threadIdx.x & 63u), q = lane >> 4, r = lane & 15;
  const uint32_t nb = nb_view * (P.views > 1 ? 2u : 1u);
  if (b >= nb) return;  // (whole waves)
  const int view = b >= nb_view ? 1 : 0;
  const uint32_t bb = view ? b - nb_view : b;
  // march wave q of the block covers the tile (q & 1, q >> 1) of TW x TH pixels (vr_march.hip)
  const int lc = (int)(bb % nbx) * 2 * tw + (q & 1) * tw + ((2 * (r & 3) + 1) * tw) / 8;
  const int y = (int)(bb / nbx) * 2 * th + (q >> 1) * th + ((2 * (r >> 2) + 1) * th) / 8;
  float ns = 0.f, g0x = 0.f, g0y = 0.f, g0z = 0.f, dx = 0.f, dy = 0.f, dz = 0.f;
  if (lc < P.part_cols && y < P.height) {
    const int pb = lc / P.block_cols;
    const int x = (P.part + pb * P.num_parts) * P.block_cols + (lc - pb * P.block_cols);
    f3 o, d;
    float tnear, tfar;
    if (ray_setup(P, x, y, o, d, tnear, tfar, view) && tfar >= tnear) {
      ns = fminf(floorf((tfar - tnear) / P.tstep) + 1.f, (float)P.max_steps);
      // texel coordinate + 1/2 per axis (its floor is the padded centre cell), at the first sample
      // and per sample
      const float sx = P.bscale[0] * P.em.fnx, sy = P.bscale[1] * P.em.fny, sz = P.bscale[2] * P.em.fnz;
      g0x = fmaf(fmaf(d.x, tnear, o.x) - P.bmin[0], sx, 0.5f);
      g0y = fmaf(fmaf(d.y, tnear, o.y) - P.bmin[1], sy, 0.5f);
      g0z = fmaf(fmaf(d.z, tnear, o.z) - P.bmin[2], sz, 0.5f);
      dx = d.x * P.tstep * sx;
      dy = d.y * P.tstep * sy;
      dz = d.z * P.tstep * sz;
    }
  }
  const int obx = (int)P.occ_bx, oby = (int)(P.occ_bxy / P.occ_bx);
  const int obz = (P.em.nz + 2 + (1 << VR_OCC_LOG) - 1) >> VR_OCC_LOG;
  constexpr float inv = 1.f / (float)(1 << VR_OCC_LOG);
  const float fm = (float)m;
  float depth = 0.f, alive_s = 0.f, occ_s = 0.f;
  const uint64_t gmask = 0xffffull << (16 * q);
  for (float k0 = 0.f;; k0 += fm) {
    const bool live = k0 < ns;
    bool occ = false;
    if (live) {
      const float kc = fmaf(0.5f, fminf(fm, ns - k0), k0);
      const int ix = min(max((int)floorf(fmaf(dx, kc, g0x) * inv), 0), obx - 1);
      const int iy = min(max((int)floorf(fmaf(dy, kc, g0y) * inv), 0), oby - 1);
      const int iz = min(max((int)floorf(fmaf(dz, kc, g0z) * inv), 0), obz - 1);
      const uint32_t qv = P.occ[((uint32_t)iz * (uint32_t)oby + (uint32_t)iy) * (uint32_t)obx + (uint32_t)ix];
      if (qv) {
        occ = true;
        depth = fmaf(dens * (float)qv, fm, depth);
        if (depth > xthr) ns = k0;  // the ray's early exit, as far as the mean densities tell
      }
    }
    const uint64_t lv = __ballot(live), oc = __ballot(occ);
    if (lv == 0ull) break;
    alive_s += (lv & gmask) ? fm : 0.f;
    occ_s += (oc & gmask) ? fm : 0.f;
  }
  float c = fmaf(occ_s, (float)VR_PRED_W_OCC, alive_s) + 16.f;
  c = fmaxf(c, __shfl_xor(c, 16, 64));
  c = fmaxf(c, __shfl_xor(c, 32, 64));
  if (lane == 0) cost[b] = (uint32_t)fminf(c, 4.0e9f);
}

// tw x th: the launch's march-wave tile in pixels (TW x TH of its depth lanes, vr_march.hip
// TileShape); m: samples per predictor step
hipError_t launch_predict_cost(const RenderParams &P, uint32_t nb_view, uint32_t nbx, int32_t tw, int32_t th,
                               int32_t m, float dens, float xthr, uint32_t *cost, hipStream_t s) {
  const uint64_t n = (uint64_t)nb_view * (P.views > 1 ? 2u : 1u);
  if (!n || !P.occ || !P.occ_bx || P.part_cols <= 0 || P.height <= 0 || m < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(predict_cost_kernel, dim3((unsigned)((n * 64 + 255) / 256)), dim3(256), 0, s, P, nb_view, nbx,
                     tw, th, m, dens, xthr, cost);
  return hipGetLastError();
}

hipError_t launch_zpair(const float *src, float *dst, uint32_t n, uint32_t pxy, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(zpair_kernel, dim3((n + 255) / 256), dim3(256), 0, s, src, dst, n, pxy);
  return hipGetLastError();
}

hipError_t launch_stats(const float *src, uint64_t n, BufStats *st, hipStream_t s) {
  if (!n) return hipSuccess;
  uint64_t blocks = (n + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(stats_kernel, dim3((unsigned)blocks), dim3(256), 0, s, src, n, st);
  return hipGetLastError();
}

}  // namespace vr
