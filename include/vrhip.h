/*
 * vrhip.h -- C-ABI of libvrhip.so, the MI355X (gfx950) volume ray-marcher.
 *
 * The entry points mirror, one for one, the command protocol of the reference's CUDA mex
 * `volumeRender` (/root/reference/src/C/mex/render.cpp:50-278) plus its two helper mex files, so
 * that a thin mexFunction adaptor (mex/volumeRender_mex.cpp) keeps the MATLAB
 * classes VolumeRender / Volume / LightSource working unchanged.  Plain pointers and sizes only.
 *
 * Conventions (identical to what the mex receives from MATLAB):
 *   - volumes are MATLAB single arrays Data(d0,d1,d2), column-major, d0 fastest; a 2-D array has
 *     d2 = 1 (volumeRender.cpp:320-339).  Data pointers are borrowed for the call only.
 *   - the rendered image is MATLAB single [H, W, 3], column-major: out[x*H + y + c*W*H]
 *     (volumeRender_kernel.cu:496-506, render.cpp:248).
 *   - every function returns VR_OK (0) or an error code; vr_last_error() gives the message
 *     (the reference's mexErrMsgTxt text where one exists).  Errors are thread-local.
 */
#ifndef VRHIP_H_
#define VRHIP_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum vr_status {
  VR_OK = 0,
  VR_ERR_ARGUMENT = 1,   /* bad argument count/shape (render.cpp:51-56,60-61,68-69,136-140) */
  VR_ERR_HANDLE = 2,     /* "Handle not valid." (class_handle.hpp:64-72)                      */
  VR_ERR_VRAM = 3,       /* "insufficient free VRAM!" (mmanager.hxx:144-173)                   */
  VR_ERR_DEVICE = 4,     /* a HIP runtime error (reference ignores them, common.h:43-47)        */
  VR_ERR_UNSUPPORTED = 5 /* request outside what this build implements                          */
};

/* Where vr_volume.data lives. */
enum vr_location { VR_HOST = 0, VR_DEVICE = 1 };

/* A MATLAB `Volume` as the mex reads it (mxMake_volume, volumeRender.cpp:307-342):
 * Data (single), its dims, and TimeLastUpdate.  `location` VR_DEVICE lets device-resident data
 * (e.g. a torch tensor) be synced without a host round trip. */
typedef struct vr_volume {
  const float *data;
  uint64_t dims[3];      /* d0, d1, d2 (d2 = 1 for 2-D data)          */
  uint64_t last_update;  /* TimeLastUpdate (ms timestamp, see vr_timestamp) */
  int32_t location;      /* enum vr_location                           */
  int32_t reserved;
} vr_volume;

/* A MATLAB `LightSource` (LightSource.m:40-64): Position and Color exactly as stored in MATLAB.
 * The position is reversed into kernel order internally (render.cpp:167-168). */
typedef struct vr_light {
  float position[3];
  float color[3];
} vr_light;

/* The positional arguments of volumeRender('render', h, ...) (render.cpp:142-240,
 * caller VolumeRender.m:563-581), in the order and units MATLAB passes them. */
typedef struct vr_render_args {
  const vr_light *lights;         /* LightSources (prhs[2])                                  */
  int64_t num_lights;             /* mxGetN(LightSources); < 0: the logical `false`           */
  const vr_volume *illumination;  /* VolumeIllumination (prhs[3]); NULL: the logical `false`  */
  float factors[3];               /* single([FactorEmission FactorReflection FactorAbsorption]) */
  float element_size_um[3];       /* single(ElementSizeUm), MATLAB order (reversed inside)    */
  uint64_t resolution[2];         /* uint64([H W]) = flip(ImageResolution)                    */
  float rotation_flipped[9];      /* single(flip(RotationMatrix)), column-major as passed      */
  float props[3];                 /* single([CameraXOffset FocalLength DistanceToObject])     */
  float opacity_threshold;        /* single(OpacityThreshold)                                 */
  float color[3];                 /* single(Color)                                            */
} vr_render_args;

/* Image-space partition for multi-GPU rendering: columns are cut into blocks of
 * `block_cols`; block b belongs to part (b % num_parts).  A part's output is the column-major
 * planar image of only its columns, in increasing x, with a fixed column stride max_cols =
 * vr_partition_columns(w, {block_cols, part 0, num_parts}) (part 0 owns the most columns):
 * element (y, local column j, channel c) at c*max_cols*H + j*H + y. */
typedef struct vr_partition {
  int32_t block_cols;
  int32_t part;
  int32_t num_parts;
  int32_t reserved;
} vr_partition;

typedef struct vr_context vr_context; /* the reference's MManager handle (mmanager.hxx:25) */

/* --- the mex commands --------------------------------------------------------------------- */

/* 'new' (render.cpp:58-65): a persistent handle bound to the current HIP device. */
int vr_new(vr_context **out);

/* 'new' for a multi-device group (SURVEY.md 8e inside the library, so that the MATLAB classes reach
 * every GPU of the node through the unchanged mex protocol; the reference picks one device,
 * volumeRender.cpp:77-87).  devices[0] is the primary: 'sync_volumes' uploads there once and copies
 * the bound volumes to the other devices over xGMI (peer copies); 'render' (and vr_render_device
 * without a partition or counters) renders column part k of the frame (16-column blocks dealt
 * round-robin) on devices[k], gathers the parts to the primary with peer copies and assembles the
 * image there -- bit-identical to the one-device render.  vr_render_stereo and vr_render_channels on
 * group handles split their fused launches across the devices the same way; vr_render_slab and a
 * vr_render_device call with a partition or counters run on the primary only.  A device may repeat
 * (a rehearsal on one GPU). */
int vr_new_multi(const int32_t *devices, int32_t n, vr_context **out);

/* 'delete' (render.cpp:72-79 -> ~MManager, mmanager.hxx:103-105).  Like the reference's
 * cudaDeviceReset this frees every handle's device volumes and resets the module-global render
 * state (texture bindings, slot indices, lights, gradient method). */
int vr_delete(vr_context *h);

/* 'mem_info' (render.cpp:85-87, mmanager.hxx:218-284): writes the report into buf. */
int vr_mem_info(vr_context *h, char *buf, size_t buflen);

/* 'sync_volumes' (render.cpp:93-129): note the order Emission, Reflection, Absorption.
 * The reference keys on the argument count (render.cpp:105-113), mapped to the gradient pointers:
 *   dx, dy, dz all non-NULL  -- nrhs == 9: the gradient volumes are taken (gradient lookup);
 *   all NULL                 -- nrhs == 6: the handle's gradient volumes are reset (on-the-fly);
 *   dx (nrhs 7) or dx, dy (nrhs 8) non-NULL, the rest NULL -- any other count (an adaptor passes
 *                              nrhs 7, 8 or > 9 this way): the handle KEEPS its previous gradient
 *                              volumes and the given ones are not read; the method is set to
 *                              on-the-fly, and the sync re-enters lookup mode if kept gradient
 *                              volumes exist (mmanager.hxx:193-200). */
int vr_sync_volumes(vr_context *h, uint64_t time_last_mem_sync, const vr_volume *emission,
                    const vr_volume *reflection, const vr_volume *absorption, const vr_volume *dx,
                    const vr_volume *dy, const vr_volume *dz);

/* 'render' (render.cpp:134-277): renders into the caller-owned host image out[H*W*3]. */
int vr_render(vr_context *h, const vr_render_args *args, float *out);

/* --- the helper mex files ------------------------------------------------------------------- */

/* HenyeyGreenstein(N[, g]) (HenyeyGreenstein.cc:29-96): out[N*N*N], MATLAB array (b, a, c). */
int vr_henyey_greenstein(uint32_t n, float g, float *out);

/* timestamp (timestamp.cpp:17-33): ms since the epoch, low 32 bits only (it is stored through an
 * int*), zero-extended -- exactly the value the reference hands to MATLAB. */
uint64_t vr_timestamp(void);

/* Fused stereo: VolumeRender.render with CameraXOffset != 0
 * (VolumeRender.m:278-307) renders the pair as two 'render' calls with camera offsets +base and
 * -base.  This renders both eyes of the same frame in one launch: args->props[0] is ignored, the
 * left image (offset -base) goes to out_left, the right (+base) to out_right, each [H, W, 3] as
 * vr_render writes it, bit-identical to the two separate renders. */
int vr_render_stereo(vr_context *h, const vr_render_args *args, float base, float *out_left, float *out_right);

/* vr_render_stereo into device memory on `stream` (asynchronous, as vr_render_device; one-device
 * handles; d_steps as vr_render_device's, over both eyes).  VR_STEREO_PAIR=1 marches the pair with
 * paired tiles (a wave holds the right eye's column c and the left eye's column
 * c + shift, one staged box for both) -- a measurement switch, images bit-identical. */
int vr_render_stereo_device(vr_context *h, const vr_render_args *args, float base, float *d_left, float *d_right,
                            unsigned long long *d_steps, void *stream);

/* Multi-channel frame (replaces the per-channel loops of examples/example3.m:
 * 61-233 -- sync a channel's volumes, render, next channel -- and the sum at example3.m:239).  A
 * channel is one VolumeRender object: its handle (distinct per channel), the arguments of its
 * 'sync_volumes' (volumeRender.cpp:600-633; dx/dy/dz NULL = on-the-fly gradient) and of its
 * 'render'.  Channel i equals vr_sync_volumes + vr_render on it (stereo != 0: vr_render_stereo
 * with `base`, left then right) were its handle the only one: before the channel's sync, the
 * texture bindings its handle's last sync left are restored (the reference's textures are module
 * globals, kernel.cu:49-120, so with one object per channel an unchanged channel would render the
 * previous channel's volumes).  Every channel must have the same resolution.
 * The channels' frames are marched together (one launch per gradient-mode / absorption / shading
 * group).  vr_render_channels writes channel i's view e (e = 0 left / only, 1 right; eyes = 1 or
 * 2) to out[(i * eyes + e) * H*W*3 ...], each laid out as vr_render's image; the caller adds them
 * (example3.m:239 adds in double). */
typedef struct vr_channel {
  vr_context *handle;
  uint64_t time_last_mem_sync;
  const vr_volume *emission, *reflection, *absorption;
  const vr_volume *dx, *dy, *dz;
  const vr_render_args *args;
} vr_channel;
int vr_render_channels(const vr_channel *channels, int32_t n, int32_t stereo, float base, float *out);
/* Device variant: channel i's view e (e = 0 left / only, 1 right) into
 * d_out + (i * eyes + e) * H*W*3, on `stream` (asynchronous; the syncs are not). */
int vr_render_channels_device(const vr_channel *channels, int32_t n, int32_t stereo, float base, float *d_out,
                              void *stream);
/* fp32 channel sum on the device: d_out[e][k] = d_in[0][e][k] + d_in[1][e][k] + ... (channel order,
 * fp32 additions) for n channels x views images of image_floats floats each. */
int vr_sum_channels_device(const float *d_in, int32_t n, int32_t views, uint64_t image_floats, float *d_out,
                           void *stream);

/* --- device-side extensions (multi-GPU, benchmarking; no MATLAB counterpart) ------------------ */

/* 'render' without the host round trip: writes the (partitioned, if part != NULL) image to the
 * device buffer d_out on `stream` (a hipStream_t; NULL = default stream).  Asynchronous.
 * If d_steps != NULL it points to VR_NUM_COUNTERS (48) counters: d_steps[0] += ray-march samples
 * taken, d_steps[1] += samples that evaluated gradient + shading (the others had opacity exactly
 * 0), d_steps[2..4] += LDS-staged chunks, all-empty (leaped) chunks, global-memory chunks,
 * d_steps[5..6] += wave sample iterations, of which any lane shaded; d_steps[7] += empty-space
 * probe runs leaped; d_steps[8..39] histogram of the box volume (floats, bins of
 * 256, last bin open) of chunks that fell back to global memory; d_steps[40..43] staged chunks with
 * S = 32, 16, 8, 4; d_steps[44] += probes that found data; d_steps[45] += floats staged into LDS.
 * [2..45] are filled by the LDS-staged kernel only. */
#define VR_NUM_COUNTERS 48
int vr_render_device(vr_context *h, const vr_render_args *args, const vr_partition *part,
                     float *d_out, unsigned long long *d_steps, void *stream);

/* Number of columns a part owns for image width w. */
int64_t vr_partition_columns(int64_t w, const vr_partition *part);

/* Scatter gathered part images (num_parts slabs of max_cols*H*3 floats each, part p at
 * d_parts + p*max_cols*H*3) into the full [H, W, 3] image d_out, on `stream`. */
int vr_assemble_partitions(const float *d_parts, int64_t w, int64_t h, int32_t block_cols,
                           int32_t num_parts, int64_t max_cols, float *d_out, void *stream);

/* --- sort-last slabs (volumes larger than one GPU; no MATLAB counterpart: the
 * reference aborts when a volume does not fit, mmanager.hxx:144-173) ----------------------------
 * The bound emission volume (the last vr_sync_volumes on any handle, as for vr_render) holds
 * planes [z_first, z_first + d2) of a volume of depth `depth` (d0, d1 as synced).  The render marches every ray of the full W x H image over the
 * samples it owns, those with z0 <= p.z * depth < z1 (p the normalized sample position; z0 = -inf
 * / z1 = +inf for the end slabs), with positions, step counts and early exit exactly as the
 * one-volume march.  part (NULL = the whole image) restricts the render to the columns of an
 * image partition (the tiles of a pipelined multi-GPU sweep).  Ray state: VR_SLAB_PLANES planes
 * of cols*H floats, [c][local column][y] (cols = vr_partition_columns): premultiplied r, g, b,
 * alpha; 1 if the ray continues past this slab; and for such a ray its resume point -- t, the
 * position x, y, z and the sample index (int32 bits) of its next sample -- from which the next
 * slab continues the march without replaying it.  d_state_in NULL = fresh rays, may equal
 * d_state_out.  direction +1 handles the rays with dir.z >= 0 (run the slabs in ascending z),
 * -1 those with dir.z < 0 (descending), 0 both (the top slab, where the descending rays start:
 * its ascending launch marches them too); other rays pass through.  Chaining both sweeps over all
 * slabs gives the one-volume image bit for bit in the first three planes.  Compute gradient or
 * emission-absorption only; absorption must alias emission (the reference's default). */
#define VR_SLAB_PLANES 10
typedef struct vr_slab {
  uint64_t depth;    /* global depth D of the emission volume                          */
  uint64_t z_first;  /* global index of the first synced plane                         */
  double z0, z1;     /* owned range of p.z * D                                         */
  int32_t direction; /* +1 / -1 / 0                                                     */
  int32_t reserved;
} vr_slab;
int vr_render_slab(vr_context *h, const vr_render_args *args, const vr_slab *slab, const vr_partition *part,
                   const float *d_state_in, float *d_state_out, void *stream);

/* Planes [*first, *first + *count) of a volume of dims (d0, d1, D) a slab owning [z0, z1) must
 * hold: the trilinear taps and the gradient taps of its samples (element size in MATLAB order). */
int vr_slab_planes(const uint64_t dims[3], const float element_size_um[3], double z0, double z1, uint64_t *first,
                   uint64_t *count);

/* Depth lanes (lanes per ray) the march kernel uses for a launch of part_cols x
 * height rays on the current device at about one texel per pixel: 1, 2, 4 or 8 (VR_DEPTH_LANES
 * overrides).  A render also weighs the texels its pixels span (denser sampling: more lanes).
 * Launches with few waves per wave slot of the device also follow a longest-first schedule. */
int vr_depth_lanes(int64_t part_cols, int64_t height);
/* The same for a render whose pixels span `texels_per_pixel` texels at the volume
 * (dist * d0 / (W * f) for the reference's camera). */
int vr_depth_lanes_tau(int64_t part_cols, int64_t height, double texels_per_pixel);

/* Synthetic test volume V_shell(n) of SURVEY.md 8d, generated on the device into d_out[n^3]. */
int vr_synth_shell_device(float *d_out, uint64_t n, void *stream);

/* Planes [z_first, z_first + count) of V_shell(n) into d_out[n*n*count] (a sort-last slab's share). */
int vr_synth_shell_planes_device(float *d_out, uint64_t n, uint64_t z_first, uint64_t count, void *stream);

/* Volume.grad on the device (Volume.m:181-205, MATLAB gradient() of single data): for the
 * column-major d_data[d0*d1*d2] writes d_gx (along dim 2), d_gy (along dim 1), d_gz (along dim 3),
 * central differences inside and one-sided at the ends, bit-identical to MATLAB's single-precision
 * gradient.  All pointers are device memory; asynchronous on `stream`. */
int vr_gradient_device(const float *d_data, const uint64_t dims[3], float *d_gx, float *d_gy, float *d_gz,
                       void *stream);

/* --- the MATLAB-side volume preprocessing on the device ----------------- */

/* HenyeyGreenstein(N, g) (HenyeyGreenstein.cc:29-96) into device memory d_out[N*N*N], same layout as
 * vr_henyey_greenstein.  The sines / cosines are the host generator's; the power of 3 comes from the
 * device math library, so elements can differ from the host LUT in the last bits (measured at
 * most 3 ulp, ~91 % bit-identical; tests/test_volume_ops.py bounds it at 4 ulp).  Returns when the LUT is written. */
int vr_henyey_greenstein_device(uint32_t n, float g, float *d_out, void *stream);

/* Volume.normalize(newMin, newMax) (Volume.m:208-220) of n single values on the device:
 * (x - min) * single(newMax - newMin) / (max - min) + single(newMin) in MATLAB's single arithmetic,
 * min / max omitting NaN.  d_out may equal d_in.  Asynchronous on `stream`. */
int vr_normalize_device(const float *d_in, uint64_t n, double new_min, double new_max, float *d_out, void *stream);

/* Volume.resize(newsize) (Volume.m:93-106: imresize3, or imresize for 2-D data) of a column-major
 * (d0, d1, d2) single volume on the device into d_out[out0*out1*out2]: MATLAB's default cubic
 * kernel, antialiasing when shrinking, mirrored ends, separable passes (double accumulation, single
 * result) along the axes in order of increasing scale.  Returns when done. */
int vr_resize_device(const float *d_in, const uint64_t in_dims[3], const uint64_t out_dims[3], float *d_out,
                     void *stream);

/* The weights / 0-based indices of one resize axis (out_len x *P, row-major), for tests. */
int vr_resize_contributions(uint64_t in_len, uint64_t out_len, int32_t *P, double *w, int32_t *idx);

/* Host-side reproduction of the upload/slot state machine (syncWithDevice,
 * volumeRender_kernel.cu:739-867) for unit tests: returns the slot indices after a sync with the
 * given similarity/update flags starting from `idx` (emission, absorption, reflection). */
int vr_debug_slot_transition(const int32_t idx_in[3], int32_t sim_em_ab, int32_t sim_em_re,
                             int32_t sim_ab_re, int32_t req_em, int32_t req_ab, int32_t req_re,
                             int32_t idx_out[3], int32_t unbound_out[3]);

/* Last error message of this thread ("" if none). */
const char *vr_last_error(void);

/* HIP errors the library did not return to a caller (process-wide; the reference ignores every CUDA
 * error, common.h:43-47): errors of its own calls that it handled with a fallback (an optional
 * buffer, a launch schedule, timing events, an already enabled peer mapping) and errors found
 * pending in the calling thread's HIP error state at an API entry (raised elsewhere; a device fault
 * found there fails that call with VR_ERR_DEVICE).  Every other HIP error fails the call that met
 * it.  Returns how many since the library was loaded and writes the last (up to 32) into buf, one
 * per line, newest last: "<kind>: <hipError name> (<code>) at <site>". */
int64_t vr_hip_errors(char *buf, size_t buflen);

/* The demangled name of the march kernel instantiation the last render launched (the process's
 * last staged-march launch), e.g. "vr::fast::march_kernel<2, 1, true, false, true, false, 1664, 0>":
 * bench.py names the kernel it times with it and keys the profiler's counters to it. */
int vr_last_march_kernel(char *buf, size_t buflen);

/* Process-wide options (round 6; no reference counterpart).  "test_switches" = 1 lets the library
 * read the kernel-variant and schedule switches the GPU tests and the measurement tools set through
 * the environment (VR_NO_LDS, VR_DEPTH_LANES, VR_SCHED, ... -- INTEGRATION.md "Runtime switches");
 * by default (0) they are ignored, so a MATLAB session's environment cannot select them.  Returns
 * VR_ERR_ARGUMENT for an unknown name. */
int vr_set_option(const char *name, int64_t value);

/* Library build identification ("libvrhip <version> gfx950 ..."). */
const char *vr_version(void);

#ifdef __cplusplus
}
#endif
#endif /* VRHIP_H_ */
