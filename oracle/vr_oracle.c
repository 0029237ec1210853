/*
 * oracle/vr_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * Scalar CPU restatement of the reference's per-pixel volume ray march so that the HIP path in
 * volume_renderer_amd/ can be checked against it.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load this file's shared object.
 *
 * PARITY STATUS: "parity unpinned" for the ray march.  The reference (CUDA <= 11 legacy texture
 * references + MATLAB mex, /root/reference/src/C/vr/volumeRender_kernel.cu) cannot be built or run
 * in this image and ships no tests, golden images or fixtures.  This file
 * is a line-by-line restatement of the reference's arithmetic; the only reference-pinned values
 * on this path are the Henyey-Greenstein LUT known answers (the LUT restatement is
 * oracle/vr_oracle_host.c; tests/test_oracle.py checks it against them).
 *
 * Arithmetic contract (shared with the HIP kernel, written out in DESIGN.md section 4):
 *   - IEEE fp32 (or fp64 for the envelope build, -DOR_DOUBLE), compiled with -ffp-contract=off.
 *   - Every `a*b + c` site of the reference that nvcc (--fmad=true) contracts is written as an
 *     explicit fma(); everything else is an individually rounded op in source order.
 *   - rsqrtf(d) (helper_math.h normalize) is modelled as 1/sqrtf(d); __expf as expf; acos as acosf.
 *   - tex3D with cudaFilterModeLinear + cudaAddressModeClamp + normalized coords
 *     (volumeRender_kernel.cu:544-548) is modelled per axis as xB = c*N - 0.5, i = floor(xB),
 *     w = rint(frac(xB)*256)/256 (9-bit fixed-point weights, 8 fractional bits), taps clamped to
 *     [0, N-1]; lerp(a, b, w) = fma(w, b - a, a), order x -> y -> z.  A NaN coordinate is treated
 *     as 0.  An unbound texture reads 0.
 *
 * Assumption variants (tools/parity_band.py): the reference's output depends on
 * details this image cannot observe; each -D switch below replaces one assumption by a plausible
 * alternative so that the spread of "equally faithful" fp32 renders can be measured:
 *   OR_VAR_TRUNC      8-bit filter weights by truncation instead of round-to-nearest-even
 *   OR_VAR_AXIS_FMA   the sampler's c*N - 0.5 as one fused multiply-add
 *   OR_VAR_LERP_2MUL  the CUDA guide's filter formula (1 - w)*a + w*b instead of fma(w, b - a, a)
 *   OR_VAR_NOFMA      no contraction anywhere (nvcc --fmad=false)
 *   OR_VAR_RSQRT_CR   helper_math normalize with a correctly rounded rsqrt instead of 1/sqrtf
 *   OR_VAR_EXP2       __expf as exp2f(x * log2 e) (the intrinsic's formulation) instead of expf
 *   OR_VAR_NAN_PROP   a NaN texture coordinate makes the fetch NaN instead of sampling at 0
 */
#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifdef OR_VAR_NOFMA
#define FMA_IMPL(a, b, c) ((a) * (b) + (c))
#endif

#ifdef OR_DOUBLE
typedef double real;
#define FMA fma
#define SQRT sqrt
#define EXP exp
#define ACOS acos
#define FLOOR floor
#define RINT rint
#define OR_SUFFIX(name) name##_f64
#else
typedef float real;
#ifdef OR_VAR_NOFMA
#define FMA(a, b, c) FMA_IMPL(a, b, c)
#else
#define FMA fmaf
#endif
#define SQRT sqrtf
#define EXP expf
#define ACOS acosf
#define FLOOR floorf
#define RINT rintf
#define OR_SUFFIX(name) name##_f32
#endif

/* A bound texture: column-major fp32 volume, x (d0) fastest.  data == NULL: unbound (reads 0). */
typedef struct or_tex {
  const float *data;
  int64_t nx, ny, nz;
} or_tex;

/* Everything d_render reads (volumeRender.h:81-109 RenderOptions + the kernel arguments
 * volumeRender_kernel.cu:365-368 + the device globals :55-120), already marshalled. */
typedef struct or_params {
  int64_t width, height;             /* image W x H (RenderOptions.image_width/height)        */
  float factor_emission;             /* Fe                                                     */
  float factor_absorption;           /* Fa                                                     */
  float factor_reflection;           /* Fr                                                     */
  float boxmin[3], boxmax[3];        /* initRender volumeRender.cpp:125-131                    */
  float rot[4][3];                   /* float4x3: m[0..2] = X,Y,Z; m[3] = (xoff, f, dist)       */
  float opacity_threshold;
  float tstep;                       /* initRender volumeRender.cpp:133-145                    */
  float color[3];                    /* aColor                                                 */
  float grad_step[3];                /* volumeRender.cpp:273-275                               */
  int32_t grad_method;               /* 0 compute (kernel.cu:212-253), 1 lookup (:266-276)     */
  int32_t num_lights;                /* c_numLightSources                                      */
  const float *lights;               /* [num_lights][6]: position xyz (kernel order), color rgb */
  int64_t max_steps;                 /* safety cap on samples per ray: never reached
                                        by a ray that terminates; bounds the t-stall case        */
  or_tex em;                         /* texture selected by d_idxEmmission  (kernel.cu:444)    */
  or_tex ab;                         /* texture selected by d_idxAbsorption (kernel.cu:446)    */
  or_tex re;                         /* texture selected by d_idxReflection (kernel.cu:343)    */
  or_tex grad_em;                    /* tex_emission binding used by computeGradient (:225)    */
  or_tex gx, gy, gz;                 /* tex_gradientX/Y/Z (:270-275)                           */
  or_tex lut;                        /* tex_illumination (:346)                                */
} or_params;

#define OR_PI ((float)3.14159265358979323846f) /* volumeRender_kernel.cu:20 */

typedef struct vec3 { real x, y, z; } vec3;

static inline vec3 v3(real x, real y, real z) { vec3 r = {x, y, z}; return r; }
static inline vec3 v3f(const float *p) { return v3((real)p[0], (real)p[1], (real)p[2]); }

/* helper_math.h dot(a,b) = a.x*b.x + a.y*b.y + a.z*b.z, contracted by nvcc to an fma chain. */
static inline real dot3(vec3 a, vec3 b) { return FMA(a.z, b.z, FMA(a.y, b.y, a.x * b.x)); }
/* helper_math.h length(v) = sqrtf(dot(v,v)) */
static inline real len3(vec3 a) { return SQRT(dot3(a, a)); }
/* helper_math.h normalize(v) = v * rsqrtf(dot(v,v)); rsqrtf modelled as 1/sqrtf. */
static inline vec3 normalize3(vec3 a) {
#ifdef OR_VAR_RSQRT_CR
  real inv = (real)(1.0 / sqrt((double)dot3(a, a)));
#else
  real inv = (real)1 / SQRT(dot3(a, a));
#endif
  return v3(a.x * inv, a.y * inv, a.z * inv);
}

/* One axis of the CUDA linear-filter address computation (normalized coords, clamp). */
static inline real tex_axis(real c, int64_t n, int64_t *i0, int64_t *i1) {
  if (c != c) c = (real)0; /* NaN coordinate -> 0 (assumption) */
#ifdef OR_VAR_AXIS_FMA
  real xb = FMA(c, (real)n, (real)-0.5);
#else
  real xb = c * (real)n - (real)0.5;
#endif
  real fl = FLOOR(xb);
#ifdef OR_VAR_TRUNC
  real w = FLOOR((xb - fl) * (real)256) * ((real)1 / (real)256);
#else
  real w = RINT((xb - fl) * (real)256) * ((real)1 / (real)256);
#endif
  int64_t i = (int64_t)fl;
  int64_t a = i, b = i + 1;
  *i0 = a < 0 ? 0 : (a > n - 1 ? n - 1 : a);
  *i1 = b < 0 ? 0 : (b > n - 1 ? n - 1 : b);
  return w;
}

#ifdef OR_VAR_LERP_2MUL
static inline real lerp(real a, real b, real w) { return ((real)1 - w) * a + w * b; }
#else
static inline real lerp(real a, real b, real w) { return FMA(w, b - a, a); }
#endif

/* tex3D(tex, x, y, z) on a bound fp32 texture, volumeRender_kernel.cu:544-548 semantics. */
static real tex3d(const or_tex *t, real x, real y, real z) {
  if (!t->data) return (real)0; /* unbound texture reference reads 0 (assumption) */
#ifdef OR_VAR_NAN_PROP
  if (x != x || y != y || z != z) return (real)NAN;
#endif
  int64_t x0, x1, y0, y1, z0, z1;
  real wx = tex_axis(x, t->nx, &x0, &x1);
  real wy = tex_axis(y, t->ny, &y0, &y1);
  real wz = tex_axis(z, t->nz, &z0, &z1);
  const float *d = t->data;
  int64_t sy = t->nx, sz = t->nx * t->ny;
#define T(i, j, k) ((real)d[(i) + (j) * sy + (k) * sz])
  real c00 = lerp(T(x0, y0, z0), T(x1, y0, z0), wx);
  real c10 = lerp(T(x0, y1, z0), T(x1, y1, z0), wx);
  real c01 = lerp(T(x0, y0, z1), T(x1, y0, z1), wx);
  real c11 = lerp(T(x0, y1, z1), T(x1, y1, z1), wx);
#undef T
  real c0 = lerp(c00, c10, wy);
  real c1 = lerp(c01, c11, wy);
  return lerp(c0, c1, wz);
}

/* angle(a,b) = acos(dot(a,b) / (length(a)*length(b)))   volumeRender_kernel.cu:284-287 */
static inline real angle3(vec3 a, vec3 b) { return ACOS(dot3(a, b) / (len3(a) * len3(b))); }

/* shade(), volumeRender_kernel.cu:308-353, with the gradient dispatch of :316-319. */
static vec3 shade(const or_params *P, vec3 ps, vec3 pos, vec3 eye, vec3 bmin, vec3 bscale) {
  vec3 g;
  if (P->grad_method == 0) {
    /* computeGradient :212-253 -- world offsets +-gradStep, always samples tex_emission. */
    real sx = (real)P->grad_step[0], sy = (real)P->grad_step[1], sz = (real)P->grad_step[2];
    real xp = ((pos.x + sx) - bmin.x) * bscale.x, xm = ((pos.x - sx) - bmin.x) * bscale.x;
    real yp = ((pos.y + sy) - bmin.y) * bscale.y, ym = ((pos.y - sy) - bmin.y) * bscale.y;
    real zp = ((pos.z + sz) - bmin.z) * bscale.z, zm = ((pos.z - sz) - bmin.z) * bscale.z;
    /* the untouched components equal the centre sample's: (pos.y + 0 - bmin.y)*s == ps.y */
    g.x = tex3d(&P->grad_em, xp, ps.y, ps.z) - tex3d(&P->grad_em, xm, ps.y, ps.z);
    g.y = tex3d(&P->grad_em, ps.x, yp, ps.z) - tex3d(&P->grad_em, ps.x, ym, ps.z);
    g.z = tex3d(&P->grad_em, ps.x, ps.y, zp) - tex3d(&P->grad_em, ps.x, ps.y, zm);
    g = v3(g.x * (real)0.5, g.y * (real)0.5, g.z * (real)0.5);
  } else {
    /* lookupGradient :266-276 */
    g = v3(tex3d(&P->gx, ps.x, ps.y, ps.z), tex3d(&P->gy, ps.x, ps.y, ps.z),
           tex3d(&P->gz, ps.x, ps.y, ps.z));
  }
  vec3 nn = normalize3(g);
  vec3 n = v3(-nn.x, -nn.y, -nn.z); /* -1.f * normalize(...) */
  vec3 col = v3f(P->color);
  vec3 result = v3(0, 0, 0);
  for (int32_t i = 0; i < P->num_lights; ++i) {
    vec3 lp = v3f(P->lights + 6 * i), lc = v3f(P->lights + 6 * i + 3);
    vec3 lo = v3(lp.x - pos.x, lp.y - pos.y, lp.z - pos.z);     /* lightOut */
    vec3 li = v3(eye.x - pos.x, eye.y - pos.y, eye.z - pos.z);  /* lightIn  */
    real alpha = angle3(n, li) / (real)OR_PI;
    real beta = angle3(n, lo) / (real)OR_PI;
    real dlo = dot3(lo, n), dli = dot3(li, n);
    /* v - dot(v,n)*n, contracted to fma(-d, n, v) */
    vec3 lop = v3(FMA(-dlo, n.x, lo.x), FMA(-dlo, n.y, lo.y), FMA(-dlo, n.z, lo.z));
    vec3 lip = v3(FMA(-dli, n.x, li.x), FMA(-dli, n.y, li.y), FMA(-dli, n.z, li.z));
    real gamma = angle3(lip, lop) / (real)OR_PI;
    real refl = (real)P->factor_reflection * tex3d(&P->re, ps.x, ps.y, ps.z);
    real light = tex3d(&P->lut, alpha, beta, gamma);
    real rl = refl * light;
    result.x = FMA(rl * lc.x, col.x, result.x);
    result.y = FMA(rl * lc.y, col.y, result.y);
    result.z = FMA(rl * lc.z, col.z, result.z);
  }
  return result;
}

/* intersectBox, volumeRender_kernel.cu:155-199 (slab test, Williams et al.) */
static int intersect_box(vec3 o, vec3 d, vec3 bmin, vec3 bmax, real *tnear, real *tfar) {
  vec3 inv = v3((real)1 / d.x, (real)1 / d.y, (real)1 / d.z);
  int sx = inv.x < 0, sy = inv.y < 0, sz = inv.z < 0;
  real px[2] = {bmin.x, bmax.x}, py[2] = {bmin.y, bmax.y}, pz[2] = {bmin.z, bmax.z};
  real tmin = (px[sx] - o.x) * inv.x;
  real tmax = (px[1 - sx] - o.x) * inv.x;
  real tymin = (py[sy] - o.y) * inv.y;
  real tymax = (py[1 - sy] - o.y) * inv.y;
  if ((tmin > tymax) || (tymin > tmax)) return 0;
  if (tymin > tmin) tmin = tymin;
  if (tymax < tmax) tmax = tymax;
  real tzmin = (pz[sz] - o.z) * inv.z;
  real tzmax = (pz[1 - sz] - o.z) * inv.z;
  if ((tmin > tzmax) || (tzmin > tmax)) return 0;
  if (tzmin > tmin) tmin = tzmin;
  if (tzmax < tmax) tmax = tzmax;
  *tnear = tmin;
  *tfar = tmax;
  return 1;
}

/* d_render for one pixel (x, y), volumeRender_kernel.cu:365-507.  Writes rgb (misses leave
 * rgb untouched, i.e. 0 after the caller's memset, volumeRender.cpp:271).  Returns #samples. */
static uint64_t render_pixel(const or_params *P, int64_t x, int64_t y, real rgb[3]) {
  const real W = (real)P->width, H = (real)P->height;
  const real tstep = (real)P->tstep, thr = (real)P->opacity_threshold;
  const real Fe = (real)P->factor_emission, Fa = (real)P->factor_absorption;
  const vec3 bmin = v3f(P->boxmin), bmax = v3f(P->boxmax);
  /* 2D image plane in [-1,1], :388-390 */
  real u = FMA((real)x / W, (real)2, (real)-1);
  real ratio = H / W;
  real v = FMA(((real)y / H) * (real)2, ratio, -ratio);
  const vec3 bscale =
      v3((real)1 / (bmax.x - bmin.x), (real)1 / (bmax.y - bmin.y), (real)1 / (bmax.z - bmin.z));
  /* camera, :399-413 */
  const real xoff = (real)P->rot[3][0], f = (real)P->rot[3][1], dist = (real)P->rot[3][2];
  const vec3 X = v3f(P->rot[0]), Y = v3f(P->rot[1]), Z = v3f(P->rot[2]);
  vec3 o = v3(FMA(-dist, Z.x, xoff * X.x), FMA(-dist, Z.y, xoff * X.y), FMA(-dist, Z.z, xoff * X.z));
  vec3 nX = normalize3(X);
  vec3 du = v3(FMA(f, Z.x, FMA(v, Y.x, u * nX.x)), FMA(f, Z.y, FMA(v, Y.y, u * nX.y)),
               FMA(f, Z.z, FMA(v, Y.z, u * nX.z)));
  vec3 d = normalize3(du);
  real tnear = 0, tfar = 0;
  if (!intersect_box(o, d, bmin, bmax, &tnear, &tfar)) return 0;
  if (tnear < (real)0) tnear = (real)0;
  real sr = 0, sg = 0, sb = 0, sa = 0;
  real t = tnear;
  vec3 pos = v3(FMA(d.x, tnear, o.x), FMA(d.y, tnear, o.y), FMA(d.z, tnear, o.z));
  const vec3 step = v3(d.x * tstep, d.y * tstep, d.z * tstep);
  const vec3 col = v3f(P->color);
  uint64_t n = 0;
  for (;;) {
    vec3 ps = v3((pos.x - bmin.x) * bscale.x, (pos.y - bmin.y) * bscale.y, (pos.z - bmin.z) * bscale.z);
    real em_s = tex3d(&P->em, ps.x, ps.y, ps.z);
    real ab_s = (P->ab.data == P->em.data && P->ab.nx == P->em.nx && P->ab.ny == P->em.ny &&
                 P->ab.nz == P->em.nz)
                    ? em_s
                    : tex3d(&P->ab, ps.x, ps.y, ps.z);
    real e = Fe * em_s;
    real a = Fa * ab_s;
#ifdef OR_VAR_EXP2
    real alpha = (real)1 - exp2f((-a * tstep) * 0x1.715476p+0f);
#else
    real alpha = (real)1 - EXP(-a * tstep);
#endif
    real eds = e * tstep;
    vec3 ill = v3(0, 0, 0);
    /* shade() runs unconditionally in the reference; with no lights its result is exactly 0
     * and the gradient it computes is unused, so it is skipped here. */
    if (P->num_lights > 0) ill = shade(P, ps, pos, o, bmin, bscale);
    real r = FMA(eds, col.x, ill.x) * alpha;
    real g = FMA(eds, col.y, ill.y) * alpha;
    real b = FMA(eds, col.z, ill.z) * alpha;
    real om = (real)1 - sa;
    sr = FMA(om, r, sr);
    sg = FMA(om, g, sg);
    sb = FMA(om, b, sb);
    sa = FMA(om, alpha, sa);
    ++n;
    if (sa > thr) break;
    if ((int64_t)n >= P->max_steps) break;
    t += tstep;
    if (t > tfar) break;
    pos = v3(pos.x + step.x, pos.y + step.y, pos.z + step.z);
  }
  rgb[0] = sr;
  rgb[1] = sg;
  rgb[2] = sb;
  return n;
}

/* Render the pixel columns listed in `cols` (NULL: all W columns) into the column-major planar
 * image out[x*H + y + c*W*H] (volumeRender_kernel.cu:496-506).  Pixels not rendered are left as
 * they are (callers zero `out`).  Returns the total number of samples taken (steps). */
uint64_t OR_SUFFIX(or_render)(const or_params *P, float *out, const int64_t *cols, int64_t ncols,
                              int nthreads) {
  const int64_t W = P->width, H = P->height;
  if (W <= 0 || H <= 0) return 0;
  if (!cols) ncols = W;
  uint64_t total = 0;
#ifdef _OPENMP
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads) reduction(+ : total)
#endif
  for (int64_t ci = 0; ci < ncols; ++ci) {
    int64_t x = cols ? cols[ci] : ci;
    if (x < 0 || x >= W) continue;
    for (int64_t y = 0; y < H; ++y) {
      real rgb[3] = {0, 0, 0};
      uint64_t n = render_pixel(P, x, y, rgb);
      total += n;
      if (n) {
        int64_t k = x * H + y;
        out[k] = (float)rgb[0];
        out[k + W * H] = (float)rgb[1];
        out[k + 2 * W * H] = (float)rgb[2];
      }
    }
  }
  return total;
}

/* Render an explicit list of pixels (x[i], y[i]) into out[3*i + c]; returns total samples. */
uint64_t OR_SUFFIX(or_render_pixels)(const or_params *P, const int64_t *xs, const int64_t *ys,
                                     int64_t n, float *out, uint64_t *steps, int nthreads) {
  uint64_t total = 0;
#ifdef _OPENMP
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads) reduction(+ : total)
#endif
  for (int64_t i = 0; i < n; ++i) {
    real rgb[3] = {0, 0, 0};
    uint64_t s = render_pixel(P, xs[i], ys[i], rgb);
    out[3 * i] = (float)rgb[0];
    out[3 * i + 1] = (float)rgb[1];
    out[3 * i + 2] = (float)rgb[2];
    if (steps) steps[i] = s;
    total += s;
  }
  return total;
}

/* Single tex3D fetch (sampler known-answer tests). */
float OR_SUFFIX(or_tex3d)(const float *data, int64_t nx, int64_t ny, int64_t nz, float x, float y,
                          float z) {
  or_tex t = {data, nx, ny, nz};
  return (float)tex3d(&t, (real)x, (real)y, (real)z);
}
