// vr_kernels.hip -- gfx950 (MI355X, CDNA4) kernels of the volume ray-marcher.
//
// render_kernel: one lane per primary ray, a wave = an 8x8-pixel tile, a 256-thread workgroup =
// 16x16 pixels.  Front-to-back emission/absorption compositing with early ray termination,
// software trilinear sampling with the CUDA linear-filter semantics of the reference's tex3D
// (/root/reference/src/C/vr/volumeRender_kernel.cu:544-548), on-the-fly (:212-253) or lookup
// (:266-276) gradient, Henyey-Greenstein LUT shading per light (:308-353).  The arithmetic follows
// the contract of DESIGN.md s4 op for op (explicit fmaf, -ffp-contract=off) so that the HIP path and
// the CPU oracle (oracle/vr_oracle.c) agree to the last bit wherever libm's expf/acosf do.
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
__device__ __forceinline__ float len3(f3 a) { return sqrtf(dot3(a, a)); }
__device__ __forceinline__ float angle3(f3 a, f3 b) {
  return acosf(dot3(a, b) / (len3(a) * len3(b)));
}

// One axis of the linear-filter address computation (normalized coords, clamp addressing).
__device__ __forceinline__ float tex_axis(float c, int n, int &i0, int &i1) {
  c = (c != c) ? 0.f : c;  // NaN coordinate -> 0
  const float xb = c * (float)n - 0.5f;
  const float fl = floorf(xb);
  const float w = rintf((xb - fl) * 256.f) * (1.f / 256.f);
  const int i = (int)fl;
  i0 = min(max(i, 0), n - 1);
  i1 = min(max(i + 1, 0), n - 1);
  return w;
}

__device__ __forceinline__ float lerp(float a, float b, float w) { return fmaf(w, b - a, a); }

template <bool BIG>
__device__ __forceinline__ float tex3d(const DevTex &t, float x, float y, float z) {
  if (t.p == nullptr) return 0.f;  // unbound texture reads 0 (wave-uniform branch)
  int x0, x1, y0, y1, z0, z1;
  const float wx = tex_axis(x, t.nx, x0, x1);
  const float wy = tex_axis(y, t.ny, y0, y1);
  const float wz = tex_axis(z, t.nz, z0, z1);
  const float *p = t.p;
  float v[8];
  if (BIG) {
    const uint64_t sy = (uint64_t)t.nx, sz = (uint64_t)t.nx * (uint64_t)t.ny;
    const uint64_t r00 = y0 * sy + z0 * sz, r10 = y1 * sy + z0 * sz;
    const uint64_t r01 = y0 * sy + z1 * sz, r11 = y1 * sy + z1 * sz;
    v[0] = p[r00 + x0]; v[1] = p[r00 + x1]; v[2] = p[r10 + x0]; v[3] = p[r10 + x1];
    v[4] = p[r01 + x0]; v[5] = p[r01 + x1]; v[6] = p[r11 + x0]; v[7] = p[r11 + x1];
  } else {
    const uint32_t sy = (uint32_t)t.nx, sz = (uint32_t)t.nx * (uint32_t)t.ny;
    const uint32_t r00 = y0 * sy + z0 * sz, r10 = y1 * sy + z0 * sz;
    const uint32_t r01 = y0 * sy + z1 * sz, r11 = y1 * sy + z1 * sz;
    v[0] = p[r00 + x0]; v[1] = p[r00 + x1]; v[2] = p[r10 + x0]; v[3] = p[r10 + x1];
    v[4] = p[r01 + x0]; v[5] = p[r01 + x1]; v[6] = p[r11 + x0]; v[7] = p[r11 + x1];
  }
  const float c00 = lerp(v[0], v[1], wx), c10 = lerp(v[2], v[3], wx);
  const float c01 = lerp(v[4], v[5], wx), c11 = lerp(v[6], v[7], wx);
  const float c0 = lerp(c00, c10, wy), c1 = lerp(c01, c11, wy);
  return lerp(c0, c1, wz);
}

// MODE 0: no light sources (shade() contributes exactly 0); 1: on-the-fly gradient; 2: lookup.
template <int MODE, bool AB_ALIAS, bool BIG, bool COUNT>
__global__ __launch_bounds__(256) void render_kernel(const RenderParams P) {
  // 16x16 pixel workgroup tile; wave w owns the 8x8 quadrant (w & 1, w >> 1); lane -> (x, y)
  // with y fastest so that the column-major output stores of a lane octet are contiguous.
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lc = blockIdx.x * 16 + (wave & 1) * 8 + (lane >> 3);  // local (partition) column
  const int y = blockIdx.y * 16 + (wave >> 1) * 8 + (lane & 7);
  const bool active = (lc < P.part_cols) && (y < P.height);
  int32_t nsteps = 0;
  if (active) {
    const int blk = lc / P.block_cols, within = lc - blk * P.block_cols;
    const int x = (P.part + blk * P.num_parts) * P.block_cols + within;

    // ray, volumeRender_kernel.cu:388-413
    const float u = fmaf((float)x / P.fw, 2.f, -1.f);
    const float v = fmaf(((float)y / P.fh) * 2.f, P.ratio, -P.ratio);
    const f3 o = mk(P.eye[0], P.eye[1], P.eye[2]);
    f3 du;
    du.x = fmaf(P.focal, P.zdir[0], fmaf(v, P.ydir[0], u * P.nx_[0]));
    du.y = fmaf(P.focal, P.zdir[1], fmaf(v, P.ydir[1], u * P.nx_[1]));
    du.z = fmaf(P.focal, P.zdir[2], fmaf(v, P.ydir[2], u * P.nx_[2]));
    const float inv = 1.f / sqrtf(dot3(du, du));
    const f3 d = mk(du.x * inv, du.y * inv, du.z * inv);

    // intersectBox, :155-199
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

    float sr = 0.f, sg = 0.f, sb = 0.f, sa = 0.f;
    if (hit) {
      const float tnear = tmin < 0.f ? 0.f : tmin;
      const float tfar = tmax;
      const float tstep = P.tstep, thr = P.thr;
      const f3 bsc = mk(P.bscale[0], P.bscale[1], P.bscale[2]);
      f3 pos = mk(fmaf(d.x, tnear, o.x), fmaf(d.y, tnear, o.y), fmaf(d.z, tnear, o.z));
      const f3 step = mk(d.x * tstep, d.y * tstep, d.z * tstep);
      float t = tnear;
      for (;;) {
        const f3 ps = mk((pos.x - bmin.x) * bsc.x, (pos.y - bmin.y) * bsc.y, (pos.z - bmin.z) * bsc.z);
        const float em_s = tex3d<BIG>(P.em, ps.x, ps.y, ps.z);
        const float ab_s = AB_ALIAS ? em_s : tex3d<BIG>(P.ab, ps.x, ps.y, ps.z);
        const float e = P.fe * em_s;
        const float a = P.fa * ab_s;
        const float alpha = 1.f - expf(-a * tstep);
        const float eds = e * tstep;
        float ir = 0.f, ig = 0.f, ib = 0.f;
        if (MODE != 0) {
          f3 g;
          if (MODE == 1) {
            const float xp = ((pos.x + P.gstep[0]) - bmin.x) * bsc.x;
            const float xm = ((pos.x - P.gstep[0]) - bmin.x) * bsc.x;
            const float yp = ((pos.y + P.gstep[1]) - bmin.y) * bsc.y;
            const float ym = ((pos.y - P.gstep[1]) - bmin.y) * bsc.y;
            const float zp = ((pos.z + P.gstep[2]) - bmin.z) * bsc.z;
            const float zm = ((pos.z - P.gstep[2]) - bmin.z) * bsc.z;
            g.x = tex3d<BIG>(P.gem, xp, ps.y, ps.z) - tex3d<BIG>(P.gem, xm, ps.y, ps.z);
            g.y = tex3d<BIG>(P.gem, ps.x, yp, ps.z) - tex3d<BIG>(P.gem, ps.x, ym, ps.z);
            g.z = tex3d<BIG>(P.gem, ps.x, ps.y, zp) - tex3d<BIG>(P.gem, ps.x, ps.y, zm);
            g = mk(g.x * 0.5f, g.y * 0.5f, g.z * 0.5f);
          } else {
            g = mk(tex3d<BIG>(P.gx, ps.x, ps.y, ps.z), tex3d<BIG>(P.gy, ps.x, ps.y, ps.z),
                   tex3d<BIG>(P.gz, ps.x, ps.y, ps.z));
          }
          const float ginv = 1.f / sqrtf(dot3(g, g));
          const f3 n = mk(-(g.x * ginv), -(g.y * ginv), -(g.z * ginv));
          const float refl = P.fr * tex3d<BIG>(P.re, ps.x, ps.y, ps.z);
          const f3 li = mk(o.x - pos.x, o.y - pos.y, o.z - pos.z);
          const float nlen = len3(n), lilen = len3(li);
          const float alpha_n = acosf(dot3(n, li) / (nlen * lilen)) / VR_PI;
          const float dli = dot3(li, n);
          const f3 lip = mk(fmaf(-dli, n.x, li.x), fmaf(-dli, n.y, li.y), fmaf(-dli, n.z, li.z));
          const float liplen = len3(lip);
          for (int i = 0; i < P.num_lights; ++i) {
            const DevLight L = P.lights[i];
            const f3 lo = mk(L.px - pos.x, L.py - pos.y, L.pz - pos.z);
            const float beta = acosf(dot3(n, lo) / (nlen * len3(lo))) / VR_PI;
            const float dlo = dot3(lo, n);
            const f3 lop = mk(fmaf(-dlo, n.x, lo.x), fmaf(-dlo, n.y, lo.y), fmaf(-dlo, n.z, lo.z));
            const float gamma = acosf(dot3(lip, lop) / (liplen * len3(lop))) / VR_PI;
            const float light = tex3d<false>(P.lut, alpha_n, beta, gamma);
            const float rl = refl * light;
            ir = fmaf(rl * L.cr, P.color[0], ir);
            ig = fmaf(rl * L.cg, P.color[1], ig);
            ib = fmaf(rl * L.cb, P.color[2], ib);
          }
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
  if (COUNT) {
    unsigned long long s = (unsigned long long)nsteps;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
    if (lane == 0 && s) atomicAdd(P.steps, s);
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
__global__ __launch_bounds__(256) void synth_shell_kernel(float *__restrict__ out, uint64_t n) {
  const uint64_t total = n * n * n;
  const double inv = 1.0 / (double)n;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t a = i % n, bq = i / n, b = bq % n, c = bq / n;
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

// ------------------------------------------------------------------------------------------------
// launch helpers (called from vr_capi.hip)

template <int MODE, bool AB, bool BIG>
static hipError_t launch3(const RenderParams &P, dim3 grid, hipStream_t s) {
  if (P.steps)
    hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, true>), grid, dim3(256), 0, s, P);
  else
    hipLaunchKernelGGL((render_kernel<MODE, AB, BIG, false>), grid, dim3(256), 0, s, P);
  return hipGetLastError();
}

template <int MODE>
static hipError_t launch2(const RenderParams &P, bool ab_alias, bool big, dim3 grid, hipStream_t s) {
  if (ab_alias) return big ? launch3<MODE, true, true>(P, grid, s) : launch3<MODE, true, false>(P, grid, s);
  return big ? launch3<MODE, false, true>(P, grid, s) : launch3<MODE, false, false>(P, grid, s);
}

hipError_t launch_render(const RenderParams &P, int mode, bool ab_alias, bool big, hipStream_t s) {
  if (P.part_cols <= 0 || P.height <= 0) return hipSuccess;
  dim3 grid((unsigned)((P.part_cols + 15) / 16), (unsigned)((P.height + 15) / 16));
  switch (mode) {
    case 0: return launch2<0>(P, ab_alias, big, grid, s);
    case 1: return launch2<1>(P, ab_alias, big, grid, s);
    default: return launch2<2>(P, ab_alias, big, grid, s);
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

hipError_t launch_synth_shell(float *out, uint64_t n, hipStream_t s) {
  const uint64_t total = n * n * n;
  if (!total) return hipSuccess;
  uint64_t blocks = (total + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  hipLaunchKernelGGL(synth_shell_kernel, dim3((unsigned)blocks), dim3(256), 0, s, out, n);
  return hipGetLastError();
}

}  // namespace vr
