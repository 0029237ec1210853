/*
 * oracle/vr_oracle_host.c -- TEST INFRASTRUCTURE ONLY (the checker, never the product).
 *
 * CPU restatement of the reference's host-side arithmetic on the render path:
 *   - initRender box / step size        /root/reference/src/C/vr/volumeRender.cpp:112-156
 *   - gradient step                      /root/reference/src/C/vr/volumeRender.cpp:273-275
 *   - Henyey-Greenstein LUT generator    /root/reference/src/C/mex/HenyeyGreenstein.cc:39-91
 *     (+ rotateAroundX / operator* of   /root/reference/src/C/vr/illumination/float3.h:77-106)
 *
 * PARITY STATUS: the HG LUT is pinned by the known-answer values the reference's own generator
 * produced (LUT[0]=3.580975, LUT[1]=3.336926, LUT[64]=3.336926,
 * LUT[64^3-1]=0.004934164 at N=64, g=0.8), checked in tests/test_oracle.py.  initRender is
 * straight-line fp32 arithmetic; it is unpinned (no reference output exists for it).
 * Compile with -ffp-contract=off and without -ffast-math (build: oracle/Makefile).
 */
#include <math.h>
#include <stddef.h>
#include <stdint.h>

/* initRender: box extents and ray step.  es = element size in kernel order (x,y,z), i.e. the
 * MATLAB ElementSizeUm reversed (render.cpp:195 make_float3Inv). */
void or_init_render(uint64_t w, uint64_t h, uint64_t d, const float es[3], float boxmin[3],
                    float boxmax[3], float *tstep) {
  boxmax[0] = 1.f;
  boxmax[1] = (es[1] * (float)h) / ((float)w * es[0]);
  boxmax[2] = (es[2] * (float)d) / ((float)w * es[0]);
  for (int i = 0; i < 3; ++i) boxmin[i] = -1.f * boxmax[i];
  /* diagonals are computed in size_t arithmetic, then converted for sqrtf */
  float dxy = sqrtf((float)(w * w + h * h));
  float dyz = sqrtf((float)(h * h + d * d));
  float dxz = sqrtf((float)(w * w + d * d));
  float maxDiagonal = fminf(dxy, fminf(dyz, dxz)); /* named "max", computes the min */
  *tstep = 1.f / (2.2f * maxDiagonal);
}

/* gradientStep = (1/W, 1/H, 1/D) of the emission extent */
void or_grad_step(uint64_t w, uint64_t h, uint64_t d, float out[3]) {
  out[0] = 1.f / (float)w;
  out[1] = 1.f / (float)h;
  out[2] = 1.f / (float)d;
}

#define HG_PI ((float)3.141592653589793238462643383279502884197169399375105820)

/* Henyey-Greenstein N^3 LUT, value at linear index c*N*N + a*N + b (MATLAB array (b,a,c)). */
int or_hg_lut(unsigned n, float g, float *out) {
  if (g > 1 || g < -1) return 1;
  float frac_half = HG_PI / n;
  size_t page = (size_t)n * n;
  for (unsigned c = 0; c < n; ++c) {
    float gamma = c * frac_half;
    float s = sinf(gamma), co = cosf(gamma);
    for (unsigned a = 0; a < n; ++a) {
      float alpha = a * frac_half;
      /* lightOut = (sin a, 0, cos a) times rotateAroundX(gamma), whose columns are
       * (1,0,0), (0,c,-s), (0,s,c) (float3.h:96-104); operator* sums column-wise (:80-82). */
      float lx = sinf(alpha), ly = 0.f, lz = cosf(alpha);
      float rx = 1.f * lx + 0.f * ly + 0.f * lz;
      float ry = 0.f * lx + co * ly + s * lz;
      float rz = 0.f * lx + -s * ly + co * lz;
      for (unsigned b = 0; b < n; ++b) {
        float beta = b * frac_half;
        float ix = sinf(beta), iy = 0.f, iz = cosf(beta);
        float cosTheta = rx * ix + ry * iy + rz * iz;
        float numerator = (1.f - powf(g, 2.f));
        float denominator = sqrtf(powf((1.f + powf(g, 2.f) - (2.f * g * cosTheta)), 3.f));
        out[(size_t)c * page + (size_t)a * n + b] = 1.f / (4.f * HG_PI) * (numerator / denominator);
      }
    }
  }
  return 0;
}
