// vr_device.h -- types shared by the host driver (vr_capi.hip) and the gfx950 kernels
// (vr_kernels.hip).  Pure data; no torch types, no CUDA shims.
#pragma once
#include <stdint.h>

namespace vr {

// A bound "texture": fp32 volume in HBM, column-major, x (d0) fastest.  p == nullptr means the
// texture reference is unbound and reads 0 (the reference's unbound tex3D).
struct DevTex {
  const float *p;
  int32_t nx, ny, nz;
  int32_t pad_;
};

// One light in kernel order (position reversed from MATLAB, render.cpp:167-168).
struct DevLight {
  float px, py, pz;
  float cr, cg, cb;
};

// Everything one render launch reads.  Per-frame constants that the reference recomputes per
// pixel with identical IEEE arithmetic (boxScale, ray origin, normalize(X), ratio) are hoisted to
// the host (bit-identical: same ops, same rounding, -ffp-contract=off on both sides).
struct RenderParams {
  int32_t width, height;          // full image W x H
  float fw, fh;                   // (float)W, (float)H
  float ratio;                    // H / (float)W                        kernel.cu:389
  float fe, fa, fr;               // factor emission / absorption / reflection
  float bmin[3];                  // boxmin                              volumeRender.cpp:131
  float bscale[3];                // 1 / (boxmax - boxmin)               kernel.cu:396
  float eye[3];                   // xoff*X - dist*Z                     kernel.cu:407-410
  float nx_[3];                   // normalize(X)                        kernel.cu:413
  float ydir[3], zdir[3];         // Y, Z columns
  float focal;                    // f
  float thr, tstep;
  int32_t max_steps;              // safety cap on samples per ray (never reached
                                  // by a terminating ray, stops the reference's t-stall hang)
  float color[3];
  float gstep[3];                 // gradient step (world units)          volumeRender.cpp:273-275
  int32_t num_lights;
  const DevLight *lights;
  DevTex em, ab, re, gem, gx, gy, gz, lut;
  // image-space partition (vr_partition): local column lc -> global column
  int32_t block_cols, part, num_parts, part_cols;
  int32_t plane_cols;             // column stride of the output planes (part 0's column count)
  float *out;                     // [3][plane_cols][H]: column-major planar image of the part
  unsigned long long *steps;      // optional sample counter
};

}  // namespace vr
