// vr_device.h -- types shared by the host driver (vr_capi.hip) and the gfx950 kernels
// (vr_kernels.hip).  Pure data; no torch types, no CUDA shims.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime.h>  // (float4)

namespace vr {

// A bound "texture": an fp32 volume resident in HBM in the apron layout of DESIGN.md s5 -- the
// logical nx*ny*nz column-major volume (x fastest) surrounded by a one-voxel border that
// replicates the edge voxels, i.e. P[k][j][i] = T[clamp(k-1)][clamp(j-1)][clamp(i-1)] for
// i in [0, nx+1] etc.  With it the clamp-addressed tap pair (clamp(i), clamp(i+1)) of the linear
// filter is always the contiguous pair P[i'+1], P[i'+2] with i' = clamp(i, -1, n-1): one 8-byte
// load per row, no per-tap clamping.  p == nullptr means the texture reference is unbound and
// reads 0.
struct DevTex {
  const float *p;
  int32_t nx, ny, nz;
  uint32_t px;    // nx + 2 (row pitch, elements)
  uint32_t pxy;   // (nx + 2) * (ny + 2) (plane pitch, elements)
  float fnx, fny, fnz;  // (float)n for the coordinate transform
  int32_t one;    // 1x1x1 volume: every fetch is the single voxel
  int32_t small;  // padded size < 2^22 voxels: byte offsets are exact in fp32 (fetch_small)
                  // (VR_NO_SMALL_LUT=1 forces the general path, a test switch)
  float fpx4, fpxy4, fbase4;  // 4*px, 4*pxy, 4*(pxy+px+1): byte-offset terms for fetch_small
  const float *zp;  // small textures: the z-paired copy (vr_kernels.hip zpair_kernel), or null
};

// Longest run of samples the march's empty-space probe leaps at once (vr_stage.h probe_run); the
// host's probe margin (RenderParams::probe_off) covers the position drift of that many additions.
#ifndef VR_PROBE_MAX
#define VR_PROBE_MAX 512
#endif

// log2 of the occupancy map's brick edge (voxels of the padded volume per brick and axis)
#ifndef VR_OCC_LOG
#define VR_OCC_LOG 3
#endif

// Layout of the interleaved lookup gradient (RenderParams::gvec): 1 -- 2x2x2 bricks of padded
// voxels, one 128-byte line each (vr_kernels.hip interleave3_kernel, vr_sampling.h fetch_vec);
// 0 -- rows of the padded volume.
#ifndef VR_GVEC_BRICK
#define VR_GVEC_BRICK 1
#endif

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
  float eye2[3];                  // fused stereo: the second view's eye (views == 2)
  float nx_[3];                   // normalize(X)                        kernel.cu:413
  float ydir[3], zdir[3];         // Y, Z columns
  float focal;                    // f
  float thr, tstep;
  int32_t max_steps;              // safety cap on samples per ray (never reached
                                  // by a terminating ray, stops the reference's t-stall hang)
  float color[3];
  float gstep[3];                 // gradient step (world units)          volumeRender.cpp:273-275
  float tap_off[3];               // gradient tap offset in emission texels (staging halo)
  int32_t tap_half;               // MODE 1: the tap offset is half a texel on every axis (fast
                                  // variant derives the taps from the centre, vr_sampling.h)
  float cube_hs[3];               // tap_half: n / 2 per axis of the power-of-two box [-1, 1]^3 (axis_cube_s)
  int32_t num_lights;
  const DevLight *lights;
  DevTex em, ab, re, gem, gx, gy, gz, lut;
  const float *gvec;              // lookup gradient interleaved, (gx, gy, gz, 0) per padded voxel, or null
  uint32_t gv_row8, gv_plane8;    // VR_GVEC_BRICK: entries per row / plane of 2x2x2 bricks (vr_sampling.h)
  int32_t re_is_em;               // reflection texture == emission texture (sample reused)
  int32_t skip_empty;             // alpha == 0 samples may skip shading (exactly 0 contribution)
  int32_t small_x;                // every |Fa * ab(p) * tstep| < 2^-7: opacity without a range test
  int32_t eds_finite;             // every |Fe * em(p) * tstep| finite: empty skip without its test
  // "tame" launch (the march's fast path, vr_march.hip): skip_empty, eds_finite and small_x hold,
  // the reflection texture is the emission texture or a single voxel, and the LUT (if lights) is a
  // bound grid below 2^22 padded voxels -- every launch-wide test of the sample loop decided here
  int32_t tame;
  uint32_t re_mask;               // tame: ~0 if the reflection sample is the emission sample, else 0
  float tau;                      // host only: texels a pixel spans at the volume (depth_lanes)
  int32_t lookup;                 // host only: a lookup-gradient frame (depth_lanes, wave slot)
  int32_t tile_mode;              // 0: row-major tiles, 1: XCD-aware super-tiles (general kernel)
  int32_t xcd_run;                // march, unscheduled: runs of this many consecutive blocks per XCD (0/1: off)
  uint32_t block_rot;             // march, unscheduled: workgroup b marches block (b + block_rot) mod grid
  int32_t wide_slot;              // march: 10 KiB wave slots instead of 6.5 KiB (vr_stage.h)
  int32_t fast_shade;             // 1: hardware-rsq shading and exp2 opacity (default); 0: the oracle's ops
  // image-space partition (vr_partition): local column lc -> global column
  int32_t block_cols, part, num_parts, part_cols;
  int32_t plane_cols;             // column stride of the output planes (part 0's column count)
  float *out;                     // [3][plane_cols][H]: column-major planar image of the part
  float *out2;                    // fused stereo: the second view's image
  int32_t views;                  // 1, or 2 = both stereo eyes in one launch (vr_render_stereo)
  int32_t pair_shift;             // views 2: 0 (each workgroup one eye), or paired tiles -- a wave
                                  // marches the right eye's columns c.. with the left eye's c + shift..
  uint32_t view_blocks;           // workgroups per view (the launch has views x view_blocks)
  // launch schedule: workgroup b marches tile block wg_order[b] (null: b); each
  // block's duration in s_memrealtime ticks is stored to wg_cost[block] (null: not recorded)
  const uint32_t *wg_order;
  uint32_t *wg_cost;
  uint32_t *wg_start;             // diagnostics (VR_SCHED_DUMP): each timed block's start tick (low 32 bits)
  uint32_t sched_blocks;          // length of wg_order / wg_cost (must equal the launch's grid)
  uint32_t sched_full;            // 0: a short launch's schedule (longest first, timed); full frames
                                  // (occupancy-capped kernel, heavy blocks first or row-major): 1 timed,
                                  // 2 following the last measured order without timing
  uint32_t prio_blocks;           // scheduled launch: the first prio_blocks workgroups (the longest)
                                  // run at raised wave priority
  // empty-space probe (round 5, vr_stage.h probe_run): the emission texture's occupancy map -- one
  // byte per 8x8x8 brick of the padded volume, 0 when every voxel of the brick is +-0 -- or null;
  // its row and plane pitch in bricks; per axis the probe's margin in texels (the centre taps'
  // rounding margin plus the drift of VR_PROBE_MAX sequential position additions)
  const uint8_t *occ;
  uint32_t occ_bx, occ_bxy;
  float probe_off[3];
  unsigned long long *steps;      // optional sample counter
  // sort-last slab launch (vr_render_slab): owned normalized z range [slab_z0,
  // slab_z1), the margin of the chunk ownership test, the resident padded planes [slab_pk0,
  // slab_pk1) of the emission texture, the sweep direction, the incoming ray state (or null)
  float slab_z0, slab_z1, slab_margin;
  int32_t slab_pk0, slab_pk1, slab_dir;
  const float *slab_in;
  // pre-leap (round 6, vr_march.hip preleap_kernel): per march wave (workgroup x 4 + wave) 0, or
  // 1 + the slot whose 64 lanes' ray states (two float4 each: t, pos; sample index, alive | mine << 1)
  // the march starts from; the slot counter and the number of slots
  const uint32_t *pre_flag;
  float4 *pre_state;
  uint32_t *pre_count;
  uint32_t pre_cap;
};

// The views of one multi-view launch (vr_render_channels), passed by value: 4 x 832 B of kernel
// arguments.
#define VR_VIEWS_MAX 4
struct RenderViews {
  RenderParams p[VR_VIEWS_MAX];
};

// Per-buffer statistics computed on the device at upload (used to prove the empty-sample skip
// exact): any non-finite voxel, and the largest magnitude.
struct BufStats {
  uint32_t nonfinite;
  float maxabs;
};

// Host side: the demangled name of the march kernel a launch entry just enqueued (vr_capi.hip;
// read back by vr_last_march_kernel, so that bench.py can name the kernel it times and match the
// profiler's counters to exactly that instantiation).
void note_march_kernel(bool fast, int K, int mode, bool ab, bool count, bool share, bool big, int cap, int sched,
                       int nl);
// Host side: whether vr_set_option("test_switches", 1) enabled the test-only environment switches.
bool test_switches_on();

}  // namespace vr
