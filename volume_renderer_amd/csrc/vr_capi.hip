// vr_capi.hip -- host driver and C-ABI of libvrhip.so (declared in include/vrhip.h).
//
// Replaces, for the MI355X:
//   - the mex command dispatcher /root/reference/src/C/mex/render.cpp:50-278 (marshalling kept)
//   - the host render driver     /root/reference/src/C/vr/volumeRender.cpp:112-300
//   - the persistent memory manager + handle /root/reference/src/C/vr/mm/mmanager.hxx,
//     class_handle.hpp (same handle contract: signature check, dedup by (ptr, last_update, size))
//   - the upload / texture-binding state machine /root/reference/src/C/vr/volumeRender_kernel.cu:
//     600-867, re-expressed as host state: "textures" are bindings of device buffers (fp32 volumes
//     resident in HBM, read by the software sampler of vr_kernels.hip), the slot indices d_idx* and
//     the light list stay module-global exactly as in the reference.
// Every HIP call is checked (the reference ignores errors in release builds, common.h:43-47).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <map>
#include <set>
#include <array>
#include <sstream>
#include <string>
#include <queue>
#include <vector>

#include "../../include/vrhip.h"
#include "vr_device.h"
#include "vr_resources.h"

#ifndef VR_WITH_K8
#define VR_WITH_K8 0  // the K = 8 march objects (diagnostic build, make DIAG=1)
#endif
#if VR_WITH_K8
#define VR_K8(k8, k4) k8
#define VR_EXACT_K4(k4, k2) k4
#else
#define VR_K8(k8, k4) k4  // never selected: depth_lanes returns 8 only in a K = 8 build
// The exact-arithmetic variant (a parity reference, VR_EXACT_SHADE=1) is built for K = 1, 2 only
// (libvrhip.so size); exact_lanes caps its depth lanes at 2 -- the image is the same for every K.
#define VR_EXACT_K4(k4, k2) k2
#endif
int exact_lanes(int K, bool fast) { return (fast || VR_WITH_K8) ? K : std::min(K, 2); }

namespace vr {
hipError_t launch_render(const RenderParams &P, int mode, bool ab_alias, bool big, bool share, hipStream_t s);
// vr_march.hip built with VR_MARCH_FAST=1 / 0 (namespaces fast / exact) and VR_MARCH_K = 1, 2, 4, 8
#define VR_DECL_MARCH(ns)                                                                                 \
  namespace ns {                                                                                         \
  hipError_t launch_march_k1(const RenderParams &, int, bool, bool, bool, hipStream_t);                  \
  hipError_t launch_march_k2(const RenderParams &, int, bool, bool, bool, hipStream_t);                  \
  hipError_t launch_march_k4(const RenderParams &, int, bool, bool, bool, hipStream_t);                  \
  hipError_t launch_march_k8(const RenderParams &, int, bool, bool, bool, hipStream_t);                  \
  hipError_t launch_march_slab_k1(const RenderParams &, int, hipStream_t);                                \
  hipError_t launch_march_views_k1(const RenderViews &, uint32_t, int, bool, hipStream_t);                 \
  hipError_t launch_march_views_k2(const RenderViews &, uint32_t, int, bool, hipStream_t);                 \
  hipError_t launch_march_views_k4(const RenderViews &, uint32_t, int, bool, hipStream_t);                 \
  hipError_t launch_march_slab_k2(const RenderParams &, int, hipStream_t);                                \
  hipError_t launch_march_slab_k4(const RenderParams &, int, hipStream_t);                                \
  uint32_t march_blocks_k1(const RenderParams &);                                                        \
  uint32_t march_blocks_k2(const RenderParams &);                                                        \
  uint32_t march_blocks_k4(const RenderParams &);                                                        \
  uint32_t march_blocks_k8(const RenderParams &);                                                        \
  hipError_t launch_preleap_k1(const RenderParams &, hipStream_t);                                       \
  hipError_t launch_preleap_k2(const RenderParams &, hipStream_t);                                       \
  hipError_t launch_preleap_k4(const RenderParams &, hipStream_t);                                       \
  hipError_t launch_preleap_k8(const RenderParams &, hipStream_t);                                       \
  }
VR_DECL_MARCH(fast)
VR_DECL_MARCH(exact)
#undef VR_DECL_MARCH
hipError_t launch_order(const uint32_t *cost, uint32_t n, uint32_t *order, hipStream_t s, uint32_t heavy_div,
                        uint64_t tail);
hipError_t launch_iota(uint32_t *order, uint32_t n, hipStream_t s);
hipError_t launch_pad(const float *src, float *dst, int32_t nx, int32_t ny, int32_t nz, hipStream_t s);
hipError_t launch_stats(const float *src, uint64_t n, BufStats *st, hipStream_t s);
hipError_t launch_zpair(const float *src, float *dst, uint32_t n, uint32_t pxy, hipStream_t s);
hipError_t launch_occupancy(const float *p, uint32_t px, uint32_t py, uint32_t pz, uint8_t *occ, float inv_scale,
                            hipStream_t s);
hipError_t launch_predict_cost(const RenderParams &P, uint32_t nb_view, uint32_t nbx, int32_t tw, int32_t th,
                               int32_t m, float dens, float xthr, uint32_t *cost, hipStream_t s);
uint64_t interleave3_entries(uint32_t px, uint32_t py, uint32_t pz);
hipError_t launch_interleave3(const float *a, const float *b, const float *c, float *out, uint32_t px,
                              uint32_t py, uint32_t pz, hipStream_t s);
hipError_t launch_sum_channels(const float *in, uint32_t nch, uint32_t nv, uint64_t img, float *out, hipStream_t s);
hipError_t launch_assemble(const float *parts, int64_t w, int64_t h, int32_t bc, int32_t np,
                           int64_t max_cols, float *out, hipStream_t s);
hipError_t launch_synth_shell(float *out, uint64_t n, uint64_t z_first, uint64_t nz, hipStream_t s);
hipError_t launch_gradient(const float *d, const uint64_t dims[3], float *gx, float *gy, float *gz, hipStream_t s);
hipError_t launch_hg_lut(uint32_t n, const float *sn, const float *cs, float g, float g2, float num, float *out,
                         hipStream_t s);
hipError_t launch_normalize(const float *d, uint64_t n, uint32_t *mm, float range, float new_min, float *out,
                            hipStream_t s);
hipError_t launch_resize_dim(const float *in, const uint64_t dims[3], int dim, uint64_t out_len, const double *w,
                             const int32_t *idx, int32_t P, float *out, hipStream_t s);
}  // namespace vr

#ifndef VR_DEPTH_ROUNDS_K1
#define VR_DEPTH_ROUNDS_K1 16.0  // K = 1 needs >= this many K = 1 waves per device wave slot (and sparse sampling)
#endif
#ifndef VR_DEPTH_ROUNDS_K2
#define VR_DEPTH_ROUNDS_K2 3.0   // K = 2 at >= this many, K = 4 below
#endif
#ifndef VR_SCHED_HEAVY_DIV
#define VR_SCHED_HEAVY_DIV 16  // full-frame schedule: heavy = duration >= the longest block's / this
#endif
#ifndef VR_SCHED_TAIL_PCT
// heavy-first only when the longest block >= this % of the packed frame.  Round 5: 0, i.e. every full
// frame heavy-first -- with the empty-space probe the metric frame's ramp-down (the blocks started
// last, ~3.5 ms each, 3.9-4.5 ms below 90 % residency, r5ad) outweighs the row-major order's L2
// locality: 27.50-27.62 -> 26.42-26.51 ms same box (heavy = longest / 16; / 8 26.47-26.62, / 32
// 26.37-26.64, / 4 26.80-27.17, / 2 28.27-28.82; r5ae, r5af); C3 28.83 -> 28.62, C2 and C5 unchanged
#define VR_SCHED_TAIL_PCT 0
#endif
#ifndef VR_SCHED_REMEASURE
#define VR_SCHED_REMEASURE 16  // full frames: block durations re-measured every this many launches
#endif
#ifndef VR_DEPTH_TAU_K4
#define VR_DEPTH_TAU_K4 1.5      // K = 4 from this many texels per pixel (depth_lanes)
#endif
#ifndef VR_DEPTH_TAU_K1
#define VR_DEPTH_TAU_K1 0.5      // K = 1 (with >= VR_DEPTH_ROUNDS_K1 rounds) below this many
#endif

#ifndef VR_PRELEAP_LAUNCH
#define VR_PRELEAP_LAUNCH 1  // round 6: the pre-leap launch before scheduled tame marches (vr_march.hip preleap_kernel)
#endif
#define VR_WG_WAVES_HOST 4  // waves per march workgroup (vr_march.hip VR_WG_WAVES)
#ifndef VR_SCHED_ROUNDS
#define VR_SCHED_ROUNDS 6.0      // longest-first schedule below this many K = 1 waves per wave slot
#endif

namespace {
std::atomic<int> g_test_switches{0};  // vr_set_option("test_switches"), see test_env below
}
namespace vr {
bool test_switches_on() { return g_test_switches.load() != 0; }
std::string &last_march_kernel() {
  static std::string name;
  return name;
}

void note_march_kernel(bool fast, int K, int mode, bool ab, bool count, bool share, bool big, int cap, int sched,
                       int nl) {
  char b[160];
  auto tf = [](bool v) { return v ? "true" : "false"; };
  std::snprintf(b, sizeof b, "vr::%s::march_kernel<%d, %d, %s, %s, %s, %s, %d, %d, %d>", fast ? "fast" : "exact", K,
                mode, tf(ab), tf(count), tf(share), tf(big), cap, sched, nl);
  last_march_kernel() = b;
}
}  // namespace vr

namespace {

thread_local std::string g_last_error;

int fail(int code, const std::string &msg) {
  g_last_error = msg;
  return code;
}

using vr_host::HipError;

#define VR_HIP(call)                                 \
  do {                                               \
    trace_pending(#call);                            \
    hipError_t e_ = (call);                          \
    if (e_ != hipSuccess) throw HipError{e_, #call}; \
  } while (0)

// VR_TRACE_STALE=1 (diagnostics): name the checked call before which this thread's HIP error state
// already held an error (one a later hipGetLastError-based check would otherwise report)
inline void trace_pending(const char *what) {
  static const bool on = [] {
    const char *ev = std::getenv("VR_TRACE_STALE");
    return ev && ev[0] == '1';
  }();
  if (!on) return;
  const hipError_t e = hipPeekAtLastError();
  if (e != hipSuccess) std::fprintf(stderr, "VR_TRACE_STALE before %s: %s\n", what, hipGetErrorString(e));
}

// texture ids = the reference's vr::VolumeType (volumeRender.h:149-157)
enum TexId { T_EM = 0, T_AB = 1, T_RE = 2, T_DX = 3, T_DY = 4, T_DZ = 5, T_LIGHT = 6, T_COUNT = 7 };
enum GradMethod { G_COMPUTE = 0, G_LOOKUP = 1 };

// Host-side record of a MATLAB Volume (vr::Volume, volumeRender.h:61-70).
struct VolRec {
  const float *data = nullptr;
  uint64_t dims[3] = {0, 0, 0};
  uint64_t memory_size = 0;
  uint64_t last_update = 0;
  int32_t location = VR_HOST;
};
// operator== (volumeRender.cpp:24-26)
bool same(const VolRec &a, const VolRec &b) {
  return a.data == b.data && a.last_update == b.last_update && a.memory_size == b.memory_size;
}

VolRec make_rec(const vr_volume *v) {
  VolRec r;
  if (!v) return r;
  r.data = v->data;
  for (int i = 0; i < 3; ++i) r.dims[i] = v->dims[i];
  r.memory_size = v->dims[0] * v->dims[1] * v->dims[2] * sizeof(float);
  r.last_update = v->last_update;
  r.location = v->location;
  return r;
}

// A device-resident volume (the cudaArray analog): fp32 in HBM in the apron layout of
// vr_device.h ((d0+2) x (d1+2) x (d2+2), edge-replicated border), plus its upload statistics.
struct DevBuf {
  float *ptr = nullptr;
  uint64_t dims[3] = {0, 0, 0};
  uint64_t bytes = 0;  // padded allocation size
  int device = 0;
  bool nonfinite = false;
  float maxabs = 0.f;
  uint64_t version = 0;  // bumped by every upload into this buffer
  // the MATLAB Volume it was uploaded from (VolRec identity: data pointer, TimeLastUpdate, size)
  const float *src_data = nullptr;
  uint64_t src_last_update = 0, src_bytes = 0;
  // completions of the launches / peer copies that read it (vr_resources.h): it is neither
  // rewritten nor freed before all of them
  vr_host::Readers readers;
  // a replica: completion of the peer copy that fills it (a launch on any stream waits for it)
  vr_host::EventPtr ready;
  // multi-device group (vr_new_multi): its copies on the other devices, and the version each copies
  std::map<int, std::shared_ptr<DevBuf>> replicas;
  std::map<int, uint64_t> replica_of;
  // the illumination LUT (small textures bound to the LUT slot): its z-paired copy (zpair_kernel),
  // from which the fast shading's lookups take two 16-byte loads per light instead of four 8-byte
  float *zpair = nullptr;
  uint64_t zpair_bytes = 0;
  // occupancy map (volumes of at least VR_OCC_MIN_VOXELS padded voxels; vr_kernels.hip
  // occupancy_kernel): one byte per 8^3 brick, read by the march's empty-space probe
  uint8_t *occ = nullptr;
  uint64_t occ_bytes = 0;
  ~DevBuf() {
    if (zpair) vr_host::pooled_free(zpair, zpair_bytes, device, vr_host::Readers(readers));
    if (occ) vr_host::pooled_free(occ, occ_bytes, device, vr_host::Readers(readers));
    vr_host::pooled_free(ptr, bytes, device, std::move(readers));
  }
};
using BufPtr = std::shared_ptr<DevBuf>;

}  // namespace

// The MManager analog: per-handle last-synced volumes and their device buffers.
struct vr_context {
  uint32_t signature = 0xFF00F0A5u;  // class_handle.hpp:40
  int device = 0;
  uint64_t time_last_mem_sync = 0;
  VolRec vol[T_COUNT];
  BufPtr buf[T_COUNT];
  float *d_out = nullptr;  // cached output buffer for the host-return path
  size_t d_out_bytes = 0;
  // launch schedules of the march, one per frame shape: per tile block the
  // duration measured by its last launch, and the longest-first order built from it
  struct Schedule {
    uint32_t *d_cost = nullptr, *d_order = nullptr;
    uint32_t blocks = 0;
    bool measured = false;
    uint32_t frames = 0;       // full frames launched since the last measured one
    bool order_stale = false;  // costs measured since the order was last computed
    // full frames: the measured durations copied to the host (asynchronously, after the launch) to
    // decide whether the heaviest block would form a tail
    uint32_t *h_cost = nullptr;
    hipEvent_t copied = nullptr;
    uint32_t renders = 0;  // full frames: renders of this frame key so far
    bool copy_pending = false, decided = false, tail = false;
    // round 6: the frame (camera, volume upload, opacity parameters, frame_key) the durations were
    // measured on, and the one the order in d_order was predicted for (0: none)
    uint64_t key = 0, pred_key = 0;
    // round 6: the pre-leap launch's buffers (vr_march.hip preleap_kernel): a flag per march wave,
    // ray-state slots for pre_cap waves, the slot counter
    uint32_t *pre_flag = nullptr, *pre_count = nullptr;
    float4 *pre_state = nullptr;
    uint32_t pre_waves = 0, pre_cap = 0;
  };
  std::map<std::string, Schedule> sched;
  // vr_render_channels: the views' RenderParams and lights in device memory (reused per call)
  float *d_chan = nullptr;             // per-view images of the host entry
  size_t d_chan_bytes = 0;
  // the module-global texture bindings as this handle's last sync left them (vr_render_channels
  // restores them before the channel's sync); weak: they never keep a buffer alive
  std::weak_ptr<DevBuf> snap_bind[T_COUNT];
  int32_t snap_idx[3] = {0, 0, 0};
  int32_t snap_grad = 0;
  bool has_snap = false;
  // multi-device group (vr_new_multi, SURVEY.md 8e inside the library): the primary (this handle,
  // the API's) holds one child per further device; each child renders a column partition of the
  // frame with replicas of the primary's bound volumes on its device, and its part is gathered
  // to the primary over xGMI (peer copies) and assembled there
  std::vector<vr_context *> children;
  vr_context *parent = nullptr;
  hipStream_t gstream = nullptr;  // child: its device's stream (replica copies, render, gather)
  hipEvent_t gdone = nullptr;     // child: its part has landed on the primary
  // child: whether copies between it and the primary go over a peer mapping (xGMI); without one
  // (hipDeviceCanAccessPeer 0, or VR_GROUP_PEER=0) they are staged through pinned host memory
  bool peer = true;
  float *d_part = nullptr;        // child: its part image; primary: all parts
  size_t d_part_bytes = 0;
  // child without a peer mapping: the pinned staging buffer of its part gather, kept across frames
  // (the gather's D2H waits for the previous frame's assembly, so the last H2D has read it), and the
  // completion of the last H2D that read it
  void *pin = nullptr;
  size_t pin_bytes = 0;
  vr_host::EventPtr pin_read;
  // the last launch's kernel time on this context's device (events around the march launch of
  // do_render / a fused channel launch), reported by mem_info; created on first use
  hipEvent_t tev[2] = {nullptr, nullptr};
  bool timed = false;
};

namespace {

// Module-global device state of the reference (volumeRender_kernel.cu:49-120): texture bindings,
// slot indices, gradient method, light list.  Shared by all handles, reset by 'delete'.
struct TexUnit {
  BufPtr bind[T_COUNT];
  int32_t idx_em = T_EM, idx_ab = T_EM, idx_re = T_RE;  // kernel.cu:75-85
  int32_t grad_method = G_COMPUTE;                       // kernel.cu:55
  std::vector<vr::DevLight> lights;                      // c_numLightSources = lights.size(); staged
                                                         // per launch (vr_host::LaunchRec::stage)
  // lookup gradient, interleaved (gx, gy, gz, 0) per padded voxel, built from the bound gradient
  // textures when their dims equal the emission's; rebuilt when any of them changes
  struct GVec {
    std::shared_ptr<DevBuf> buf;
    const DevBuf *src[3] = {nullptr, nullptr, nullptr};
    uint64_t ver[3] = {0, 0, 0};
  };
  std::map<int, GVec> gvec;  // per device (a multi-device group renders on every device)
};

std::mutex g_mu;
// The module state and the resource lists of vr_resources.h are never destroyed: at process exit
// their destructors would run in an order unrelated to their use (a binding's buffer returning its
// memory to an already destroyed pool, events destroyed after the runtime's own teardown) -- the
// process exit releases the device memory anyway.
TexUnit &g_tex = *new TexUnit();
uint64_t g_version = 0;
uint64_t next_version() { return ++g_version; }
std::set<vr_context *> g_contexts;

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) VR_HIP(hipSetDevice(dev));
  }
  ~DeviceGuard() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

void reset_tex_unit() {
  for (auto &b : g_tex.bind) b.reset();
  g_tex.gvec.clear();
  g_tex.idx_em = T_EM;
  g_tex.idx_ab = T_EM;
  g_tex.idx_re = T_RE;
  g_tex.grad_method = G_COMPUTE;
  g_tex.lights.clear();
}

bool valid(vr_context *h) { return h && g_contexts.count(h) && h->signature == 0xFF00F0A5u; }

bool env_flag(const char *name) {
  const char *ev = std::getenv(name);
  return ev && ev[0] == '1';
}
bool env_flag_off(const char *name) {
  const char *ev = std::getenv(name);
  return ev && ev[0] == '0';
}
// A/B and diagnostic switches (INTEGRATION.md "Runtime switches"): read by a DIAG=1 build only
// (Makefile; -DVR_DIAG=1), ignored by the default library
#ifndef VR_DIAG
#define VR_DIAG 0
#endif
const char *diag_env(const char *name) { return VR_DIAG ? std::getenv(name) : nullptr; }
bool diag_flag(const char *name) {
  const char *ev = diag_env(name);
  return ev && ev[0] == '1';
}
// Test switches (round 6, INTEGRATION.md "Runtime switches"): the kernel-variant and schedule
// switches the GPU tests and the measurement tools set through the environment are read only after
// vr_set_option("test_switches", 1) (tests/conftest.py, bench.py diagnostics, tools/) or in a DIAG=1
// build, so that a MATLAB session's environment never selects them.  The production switches
// (VR_EXACT_SHADE, VR_ALWAYS_REUPLOAD, VR_GROUP_PEER, the upload ring's) are read always.
const char *test_env(const char *name) { return (VR_DIAG || g_test_switches.load()) ? std::getenv(name) : nullptr; }
bool test_flag(const char *name) {
  const char *ev = test_env(name);
  return ev && ev[0] == '1';
}
bool test_flag_off(const char *name) {
  const char *ev = test_env(name);
  return ev && ev[0] == '0';
}

// syncVolume (kernel.cu:659-672): unbind the texture, drop the old array, upload the volume into a
// device buffer and bind it.  The handle's previous buffer of the slot is rewritten in place when
// nothing else holds it and no launch still reads it; otherwise a fresh buffer is taken and the old
// one is freed when its last launch completes (a render of the previous frame may be in flight on
// another stream while this frame's volumes upload, vr_resources.h).
// The LUT's z-paired copy (DevBuf::zpair) for a texture small enough for fetch_small and not a
// single voxel; rebuilt with every upload into the buffer (the buffer's readers have completed).
// VR_NO_ZPAIR=1: none (the fast kernels then shade without the tame path, an A/B switch).
void build_zpair(DevBuf *b, hipStream_t s) {
  const uint64_t padded = (b->dims[0] + 2) * (b->dims[1] + 2) * (b->dims[2] + 2);
  const bool want = padded < (1ull << 22) && !(b->dims[0] == 1 && b->dims[1] == 1 && b->dims[2] == 1) &&
                    !diag_flag("VR_NO_ZPAIR");
  if (!want) {
    if (b->zpair) vr_host::pooled_free(b->zpair, b->zpair_bytes, b->device, vr_host::Readers(b->readers));
    b->zpair = nullptr;
    b->zpair_bytes = 0;
    return;
  }
  const uint64_t bytes = 2 * padded * sizeof(float);
  if (!b->zpair || b->zpair_bytes != bytes) {
    if (b->zpair) vr_host::pooled_free(b->zpair, b->zpair_bytes, b->device, vr_host::Readers(b->readers));
    b->zpair = nullptr;
    b->zpair_bytes = 0;
    // (the size is recorded only once the allocation exists: a failed allocation leaves no buffer
    // that a later upload of the same size would take for allocated)
    VR_HIP(vr_host::pooled_alloc(reinterpret_cast<void **>(&b->zpair), bytes, b->device));
    b->zpair_bytes = bytes;
  }
  const uint32_t pxy = (uint32_t)((b->dims[0] + 2) * (b->dims[1] + 2));
  VR_HIP(vr::launch_zpair(b->ptr, b->zpair, (uint32_t)padded, pxy, s));
  VR_HIP(hipStreamSynchronize(s));
}

// The occupancy map of buffer b (DevBuf::occ) for the march's empty-space probe, rebuilt with every
// upload into it (its readers have completed); none for small volumes (the probe needs a map only
// where leaps are long) or with VR_NO_PROBE=1.
#ifndef VR_OCC_MIN_VOXELS
#define VR_OCC_MIN_VOXELS (1ull << 18)
#endif
void build_occupancy(DevBuf *b, hipStream_t s) {
  const uint64_t px = b->dims[0] + 2, py = b->dims[1] + 2, pz = b->dims[2] + 2;
  const bool want = px * py * pz >= VR_OCC_MIN_VOXELS && px < (1ull << 31) && !test_flag("VR_NO_PROBE");
  constexpr uint64_t E = 1u << VR_OCC_LOG;  // brick edge
  const uint64_t bytes = want ? ((px + E - 1) / E) * ((py + E - 1) / E) * ((pz + E - 1) / E) : 0;
  if (!want || b->occ_bytes != bytes) {
    if (b->occ) vr_host::pooled_free(b->occ, b->occ_bytes, b->device, vr_host::Readers(b->readers));
    b->occ = nullptr;
    b->occ_bytes = 0;
  }
  if (!want) return;
  if (!b->occ) {
    VR_HIP(vr_host::pooled_alloc(reinterpret_cast<void **>(&b->occ), bytes, b->device));
    b->occ_bytes = bytes;
  }
  // (the bytes also carry each brick's mean |voxel| for the schedule predictor, in 1/255 of the largest)
  const float inv = (!b->nonfinite && b->maxabs > 0.f) ? 255.f / b->maxabs : 0.f;
  VR_HIP(vr::launch_occupancy(b->ptr, (uint32_t)px, (uint32_t)py, (uint32_t)pz, b->occ, std::isfinite(inv) ? inv : 0.f,
                              s));
  VR_HIP(hipStreamSynchronize(s));
}

void sync_volume(vr_context *h, int tex, int slot) {
  g_tex.bind[tex].reset();
  const VolRec &v = h->vol[slot];
  const uint64_t n = v.dims[0] * v.dims[1] * v.dims[2];
  const uint64_t padded = n ? (v.dims[0] + 2) * (v.dims[1] + 2) * (v.dims[2] + 2) * sizeof(float) : 0;
  BufPtr b = h->buf[slot];
  if (!(b && b.use_count() == 2 && b->bytes == padded && b->device == h->device && b->readers.done())) {
    h->buf[slot].reset();
    b = std::make_shared<DevBuf>();
    b->device = h->device;
    b->bytes = padded;
    if (padded) VR_HIP(vr_host::pooled_alloc(reinterpret_cast<void **>(&b->ptr), padded, h->device));
  }
  for (int i = 0; i < 3; ++i) b->dims[i] = v.dims[i];
  b->nonfinite = false;
  b->maxabs = 0.f;
  b->readers.clear();  // a fresh buffer, or one whose readers all completed
  if (n) {
    if (!v.data) throw HipError{hipErrorInvalidValue, "volume data is NULL"};
    vr_host::Uploader &U = vr_host::uploaders()[h->device];
    VR_HIP(U.init(h->device));
    vr::BufStats st{0u, 0.f};
    VR_HIP(U.upload(v.data, v.location == VR_DEVICE, (int32_t)v.dims[0], (int32_t)v.dims[1], (int32_t)v.dims[2],
                    b->ptr, &st));
    b->nonfinite = st.nonfinite != 0;
    b->maxabs = st.maxabs;
    if (tex == T_LIGHT) build_zpair(b.get(), U.stream);
    else if (tex <= T_RE) build_occupancy(b.get(), U.stream);  // (only these can be bound as emission)
  } else {
    build_occupancy(b.get(), nullptr);  // (an empty volume: drops a previous map)
  }
  b->version = next_version();
  b->src_data = v.data;
  b->src_last_update = v.last_update;
  b->src_bytes = v.memory_size;
  h->buf[slot] = b;
  g_tex.bind[tex] = b;
}

// setIlluminationTexture / setGradientTextures (kernel.cu:682-722) re-upload their volume on every
// call.  Here the upload is skipped when the texture is still bound to a buffer uploaded from the
// same Volume -- the identity the reference's own dedup uses for the emission / absorption /
// reflection volumes (data pointer, TimeLastUpdate, size; volumeRender.cpp:24-26).  The image is
// the same; the LUT (1 MiB) and in lookup mode the three gradient volumes (12 GiB at 1024^3) stop
// crossing PCIe per render.  VR_ALWAYS_REUPLOAD=1 restores the reference's behaviour.
void sync_volume_if_changed(vr_context *h, int tex, int slot) {
  const BufPtr &b = g_tex.bind[tex];
  const VolRec &v = h->vol[slot];
  if (b && h->buf[slot] == b && b->device == h->device && v.data && b->src_data == v.data &&
      b->src_last_update == v.last_update && b->src_bytes == v.memory_size && v.last_update != 0 &&
      !env_flag("VR_ALWAYS_REUPLOAD"))
    return;
  sync_volume(h, tex, slot);
}

// The decisions of syncWithDevice (kernel.cu:739-867) over an abstract state, so that the real
// state and vr_debug_slot_transition run the very same code.
template <class S>
void sync_decisions(S &s, bool simEmAb, bool simEmRe, bool simAbRe, bool reqEm, bool reqAb, bool reqRe) {
  bool updEm = false, updAb = false, updRe = false;
  if (reqEm) {
    if (!updEm) { s.upload(T_EM); updEm = true; }
    if (simEmRe && !updRe) { s.reference(T_RE, T_RE, &S::idx_re, T_EM); updRe = true; }
    if (simEmAb && !updAb) { s.reference(T_AB, T_AB, &S::idx_ab, T_EM); updAb = true; }
  }
  if (reqAb) {
    if (!updAb) { s.upload(T_AB); updAb = true; }
    if (simAbRe && !updRe) { s.reference(T_RE, T_RE, &S::idx_re, T_AB); updRe = true; }
    // kernel.cu:817-819 passes the absorption array for the emission texture (unreachable)
    if (simEmAb && !updEm) { s.reference(T_EM, T_AB, &S::idx_em, T_AB); updEm = true; }
  }
  if (reqRe) {
    if (!updRe) { s.upload(T_RE); updRe = true; }
    if (simAbRe && !updAb) { s.reference(T_AB, T_AB, &S::idx_ab, T_RE); updAb = true; }
    // kernel.cu:853-856: the "simEmAb" test guards Emission <- Reflection (reachable)
    if (simEmAb && !updEm) { s.reference(T_EM, T_EM, &S::idx_em, T_RE); updEm = true; }
  }
}

struct RealState {
  vr_context *h;
  int32_t idx_em, idx_ab, idx_re;  // shadow copies, written back after the decisions
  void upload(int slot) { sync_volume(h, slot, slot); }
  // referenceTexture (kernel.cu:631-648)
  void reference(int tex, int bufslot, int32_t RealState::*idx, int target) {
    if (h->buf[bufslot]) {
      g_tex.bind[tex].reset();
      h->buf[bufslot].reset();
    }
    this->*idx = target;
  }
};

struct DebugState {
  bool present[3] = {true, true, true};
  bool bound[3] = {true, true, true};
  int32_t idx_em, idx_ab, idx_re;
  void upload(int slot) { present[slot] = true; bound[slot] = true; }
  void reference(int tex, int bufslot, int32_t DebugState::*idx, int target) {
    if (present[bufslot]) {
      bound[tex] = false;
      present[bufslot] = false;
    }
    this->*idx = target;
  }
};

// MManager::getRequiredMemory (mmanager.hxx:110-133)
uint64_t required_memory(const vr_context *h) {
  const VolRec &em = h->vol[T_EM], &ab = h->vol[T_AB], &re = h->vol[T_RE];
  uint64_t r = em.memory_size;
  if (!same(em, ab) && !same(re, ab)) r += ab.memory_size;
  if (!same(em, re) && !same(re, ab)) r += re.memory_size;
  r += h->vol[T_DX].memory_size + h->vol[T_DY].memory_size + h->vol[T_DZ].memory_size;
  return r;
}

// MManager::checkFreeDeviceMemory (mmanager.hxx:144-173)
int check_free_device_memory(uint64_t required) {
  size_t free_b = 0, total_b = 0;
  VR_HIP(hipMemGetInfo(&free_b, &total_b));
  if (free_b >= required) return VR_OK;
  int dev = 0;  // pooled / retired buffers are free memory to MATLAB's eyes: release them, recheck
  VR_HIP(hipGetDevice(&dev));
  vr_host::pool_clear(dev);
  vr_host::prune_retired(true);
  VR_HIP(hipMemGetInfo(&free_b, &total_b));
  if (free_b >= required) return VR_OK;
  std::ostringstream os;
  os << "insufficient free VRAM!\n"
     << "\tTotal Memory (MB): \t" << total_b / (1024 * 1024) << "\n"
     << "\tFree Memory (MB): \t" << free_b / (1024 * 1024) << "\n"
     << "\tRequired memory (MB): \t" << required / (1024 * 1024) << "\n";
  return fail(VR_ERR_VRAM, os.str());
}

void reset_gradients(vr_context *h) {  // MManager::resetGradients (mmanager.hxx:206-213)
  for (int s : {T_DX, T_DY, T_DZ}) {
    h->buf[s].reset();
    h->vol[s] = VolRec();
  }
}

// MManager::sync (mmanager.hxx:178-201)
void mm_sync(vr_context *h) {
  if ((h->vol[T_DX].last_update == 0 && h->buf[T_DX]) || (h->vol[T_DY].last_update == 0 && h->buf[T_DY]) ||
      (h->vol[T_DZ].last_update == 0 && h->buf[T_DZ]))
    reset_gradients(h);
  const VolRec &em = h->vol[T_EM], &ab = h->vol[T_AB], &re = h->vol[T_RE];
  const uint64_t T = h->time_last_mem_sync;
  RealState s{h, g_tex.idx_em, g_tex.idx_ab, g_tex.idx_re};
  sync_decisions(s, same(em, ab), same(em, re), same(ab, re), em.last_update > T || T == 0,
                 ab.last_update > T || T == 0, re.last_update > T || T == 0);
  g_tex.idx_em = s.idx_em;
  g_tex.idx_ab = s.idx_ab;
  g_tex.idx_re = s.idx_re;
  if (h->vol[T_DX].last_update != 0 && h->vol[T_DY].last_update != 0 && h->vol[T_DZ].last_update != 0) {
    // setGradientTextures (kernel.cu:703-722): (re-)upload all three, then lookup mode
    sync_volume_if_changed(h, T_DX, T_DX);
    sync_volume_if_changed(h, T_DY, T_DY);
    sync_volume_if_changed(h, T_DZ, T_DZ);
    g_tex.grad_method = G_LOOKUP;
  }
}

vr::DevTex dev_tex(const BufPtr &b) {
  vr::DevTex t{};
  if (b && b->ptr) {
    t.p = b->ptr;
    t.nx = (int32_t)b->dims[0];
    t.ny = (int32_t)b->dims[1];
    t.nz = (int32_t)b->dims[2];
    t.px = (uint32_t)(b->dims[0] + 2);
    t.pxy = (uint32_t)((b->dims[0] + 2) * (b->dims[1] + 2));
    t.fnx = (float)t.nx;
    t.fny = (float)t.ny;
    t.fnz = (float)t.nz;
    t.one = (t.nx == 1 && t.ny == 1 && t.nz == 1);
    const uint64_t padded = (b->dims[0] + 2) * (b->dims[1] + 2) * (b->dims[2] + 2);
    t.small = padded < (1ull << 22) && !test_flag("VR_NO_SMALL_LUT");
    t.fpx4 = 4.f * (float)t.px;
    t.fpxy4 = 4.f * (float)t.pxy;
    t.fbase4 = 4.f * (float)(t.pxy + t.px + 1);
    t.zp = t.small ? b->zpair : nullptr;
  }
  return t;
}

bool is_big(const vr::DevTex &t) {
  return t.p && ((uint64_t)t.nx + 2) * ((uint64_t)t.ny + 2) * ((uint64_t)t.nz + 2) > 0xFFFFFFFFull;
}

bool same_tex(const vr::DevTex &a, const vr::DevTex &b) {
  return a.p == b.p && a.nx == b.nx && a.ny == b.ny && a.nz == b.nz;
}
bool same_dims(const vr::DevTex &a, const vr::DevTex &b) {
  return a.nx == b.nx && a.ny == b.ny && a.nz == b.nz;
}

// finite and comfortably below FLT_MAX (a texture that is unbound reads 0)
bool tame(const BufPtr &b) { return !b || !b->ptr || (!b->nonfinite && b->maxabs < 1e30f); }

// Whether the fast variant may derive the on-the-fly gradient taps from the centre's axes
// (vr_sampling.h half_taps): a cube of power-of-two edge n with isotropic element
// size, i.e. on every axis box [-1, 1] (bscale 1/2), gstep = 1/n exact and a tap offset of exactly
// half a texel.  Then the reference's tap coordinate ((pos + 2^-k) + 1) * 1/2 * n - 1/2 equals the
// centre's xb +- 1/2 exactly -- adding 2^-k (a multiple of the ulp of pos + 1 in [1, 2)) commutes with
// the rounding of pos + 1 -- except for samples within half a texel of a plane where pos, pos +- 2^-k
// or pos + 1 changes binade (pos = 0, +-2^-j), where the two can differ by an ulp of pos before the
// 8-bit weight quantization (measured: tests/test_gpu_parity.py::test_half_texel_taps).
// VR_EXACT_TAPS=1 turns it off.
int32_t half_texel_taps(const vr::RenderParams &P, int mode, float fnz) {
  if (mode != 1 || test_flag("VR_EXACT_TAPS")) return 0;
  const float n[3] = {P.em.fnx, P.em.fny, fnz};
  for (int i = 0; i < 3; ++i) {
    int e = 0;
    if (!(n[i] >= 2.f) || std::frexp(n[i], &e) != 0.5f) return 0;  // power of two
    if (P.gstep[i] != 1.f / n[i] || P.bscale[i] != 0.5f || P.bmin[i] != -1.f) return 0;
  }
  return 1;
}

// initRender (volumeRender.cpp:112-156) + the per-frame constants of d_render.
struct Frame {
  vr::RenderParams P;
  double drift1[3] = {0, 0, 0};  // staging-halo rounding margin per chunk sample (set_chunk_halo)
  int mode = 0;
  bool ab_alias = false, big = false, share = false;
  bool degenerate = false;
  vr_context::Schedule *sched_copy = nullptr;  // a timed full-frame launch: copy its durations back
  vr_context::Schedule *sched = nullptr;       // the launch shape's schedule (attach_schedule)
};


// Per-sample bound of the drift between a predicted position fma(step, k, pos) and k sequentially
// rounded additions, in emission texels per axis: |pos| <= |box| + |eye| (fp32 rounding 1.2e-7 per
// operation, two per step).  eye2: the second eye of a fused stereo launch, whose rays start
// elsewhere (the bound must cover both eyes).
void drift_bound(Frame &F, const float *eye2) {
  const vr::RenderParams &P = F.P;
  double pmax = 0.0;
  for (int i = 0; i < 3; ++i) {
    double e = std::fabs(P.eye[i]);
    if (eye2) e = std::max(e, (double)std::fabs(eye2[i]));
    pmax = std::max(pmax, (double)std::fabs(P.bmin[i]) + e);
  }
  for (int i = 0; i < 3; ++i) {
    const float n = i == 0 ? P.em.fnx : (i == 1 ? P.em.fny : P.em.fnz);
    F.drift1[i] = 2.0 * pmax * 1.2e-7 * (double)P.bscale[i] * (double)n;
    // the empty-space probe's box: the centre taps (the cell of floor(c n - 1/2)) with the staging
    // margin of 1/16 texel, plus the drift of up to VR_PROBE_MAX sequential additions.  Set here, with
    // the drift, so that every launch path gets it -- the fused multi-view march included (ADVICE r5:
    // it copied F.P before set_chunk_halo and probed with a zero margin)
    F.P.probe_off[i] = (float)(0.0625 + (double)VR_PROBE_MAX * F.drift1[i]);
  }
}

int build_frame(vr_context *h, const vr_render_args *a, Frame &F, uint64_t depth_override = 0) {
  vr::RenderParams &P = F.P;
  std::memset(&P, 0, sizeof(P));
  const uint64_t H = a->resolution[0], W = a->resolution[1];
  if (W > 0x7FFFFFFF || H > 0x7FFFFFFF || W * H > (1ull << 40))
    return fail(VR_ERR_UNSUPPORTED, "image resolution too large");
  P.width = (int32_t)W;
  P.height = (int32_t)H;
  P.fw = (float)W;
  P.fh = (float)H;
  P.ratio = (float)H / (float)W;
  // factors = [Fe Fr Fa] -> initRender(..., Fe, Fr, Fa, ...)
  P.fe = a->factors[0];
  P.fr = a->factors[1];
  P.fa = a->factors[2];
  // element size reversed (make_float3Inv, render.cpp:35-37,195)
  const float es[3] = {a->element_size_um[2], a->element_size_um[1], a->element_size_um[0]};
  const VolRec &ev = h->vol[T_EM];  // extent of the handle's emission volume (render.cpp:245)
  const uint64_t vw = ev.dims[0], vh = ev.dims[1], vd = depth_override ? depth_override : ev.dims[2];
  float bmax[3];
  bmax[0] = 1.f;
  bmax[1] = (es[1] * (float)vh) / ((float)vw * es[0]);
  bmax[2] = (es[2] * (float)vd) / ((float)vw * es[0]);
  for (int i = 0; i < 3; ++i) P.bmin[i] = -1.f * bmax[i];
  const float dxy = sqrtf((float)(vw * vw + vh * vh));
  const float dyz = sqrtf((float)(vh * vh + vd * vd));
  const float dxz = sqrtf((float)(vw * vw + vd * vd));
  const float mind = fminf(dxy, fminf(dyz, dxz));
  P.tstep = 1.f / (2.2f * mind);
  P.thr = a->opacity_threshold;
  for (int i = 0; i < 3; ++i) {
    P.bscale[i] = 1.f / (bmax[i] - P.bmin[i]);
    P.color[i] = a->color[i];
  }
  P.gstep[0] = 1.f / (float)vw;  // volumeRender.cpp:273-275
  P.gstep[1] = 1.f / (float)vh;
  P.gstep[2] = 1.f / (float)vd;
  // rotation: m[j] = column j of R, un-flipping MATLAB's flip(R) (render.cpp:211-221)
  const float *r = a->rotation_flipped;
  const float X[3] = {r[2], r[1], r[0]}, Y[3] = {r[5], r[4], r[3]}, Z[3] = {r[8], r[7], r[6]};
  const float xoff = a->props[0], f = a->props[1], dist = a->props[2];
  for (int i = 0; i < 3; ++i) {
    P.eye[i] = fmaf(-dist, Z[i], xoff * X[i]);
    P.ydir[i] = Y[i];
    P.zdir[i] = Z[i];
  }
  const float xx = fmaf(X[2], X[2], fmaf(X[1], X[1], X[0] * X[0]));
  const float xinv = 1.f / sqrtf(xx);
  for (int i = 0; i < 3; ++i) P.nx_[i] = X[i] * xinv;
  P.focal = f;
  // textures through the slot indices (getTexture, kernel.cu:127-144)
  P.em = dev_tex(g_tex.bind[g_tex.idx_em]);
  {  // the emission buffer's occupancy map (the empty-space probe; null: none, no probe)
    const BufPtr &eb = g_tex.bind[g_tex.idx_em];
    P.occ = (eb && eb->ptr && eb->occ) ? eb->occ : nullptr;
    constexpr uint64_t E = 1u << VR_OCC_LOG;
    P.occ_bx = P.occ ? (uint32_t)((eb->dims[0] + 2 + E - 1) / E) : 0u;
    P.occ_bxy = P.occ ? P.occ_bx * (uint32_t)((eb->dims[1] + 2 + E - 1) / E) : 0u;
  }
  P.ab = dev_tex(g_tex.bind[g_tex.idx_ab]);
  P.re = dev_tex(g_tex.bind[g_tex.idx_re]);
  P.gem = dev_tex(g_tex.bind[T_EM]);
  P.gx = dev_tex(g_tex.bind[T_DX]);
  P.gy = dev_tex(g_tex.bind[T_DY]);
  P.gz = dev_tex(g_tex.bind[T_DZ]);
  P.lut = dev_tex(g_tex.bind[T_LIGHT]);
  P.num_lights = (int32_t)g_tex.lights.size();
  P.lights = nullptr;  // staged per launch on the launch's stream (stage_frame)
  F.mode = P.num_lights == 0 ? 0 : (g_tex.grad_method == G_LOOKUP ? 2 : 1);
  F.ab_alias = same_tex(P.ab, P.em);
  const bool em_grid = P.em.p && !P.em.one;  // the centre sample computes its three axes
  if (F.mode == 1)
    F.share = em_grid && same_tex(P.gem, P.em);
  else if (F.mode == 2)
    F.share = em_grid && P.gx.p && P.gy.p && P.gz.p && !P.gx.one && same_dims(P.gx, P.em) &&
              same_dims(P.gy, P.em) && same_dims(P.gz, P.em);
  P.re_is_em = same_tex(P.re, P.em) && P.em.p != nullptr;
  // staging halo per axis, in emission texels (vr_stage.h axis_range): the gradient tap offset
  // gstep * bscale * n (0.5 for a cube) plus a margin that bounds the drift between a predicted
  // position fma(step, k, pos) and k sequentially rounded additions (|pos| <= |box| + |eye|), per
  // sample of the chunk; set_chunk_halo scales it by the launch's chunk length
  {
    drift_bound(F, nullptr);
    for (int i = 0; i < 3; ++i) {
      const float n = i == 0 ? P.em.fnx : (i == 1 ? P.em.fny : P.em.fnz);
      P.tap_off[i] = (float)((F.mode == 1 ? (double)P.gstep[i] * P.bscale[i] * n : 0.0) + 0.0625);
    }
    P.tap_half = half_texel_taps(P, F.mode, P.em.fnz);
    // (n / 2 per axis, exact: n a power of two)
    P.cube_hs[0] = P.tap_half ? P.em.fnx * 0.5f : 0.f;
    P.cube_hs[1] = P.tap_half ? P.em.fny * 0.5f : 0.f;
    P.cube_hs[2] = P.tap_half ? P.em.fnz * 0.5f : 0.f;
  }
  // Empty-sample skip: a sample with alpha == 0 adds fma(eds, c, ill) * 0 to the
  // sum; that is exactly +-0 (a no-op) whenever the illumination term `ill` is finite, which holds
  // if the reflection texture, the LUT, the light colours, the colour and Fr are finite and small.
  {
    const BufPtr &rb = g_tex.bind[g_tex.idx_re];
    const BufPtr &lb = g_tex.bind[T_LIGHT];
    bool ok = tame(rb) && tame(lb) && std::isfinite(P.fr) && std::fabs(P.fr) < 1e3f;
    double bound = 1.0;
    for (int i = 0; i < 3; ++i) {
      ok = ok && std::isfinite(P.color[i]) && std::fabs(P.color[i]) < 1e3f;
      bound = std::max(bound, (double)std::fabs(P.color[i]));
    }
    double lmax = 0.0;
    for (const auto &L : g_tex.lights) {
      for (float c : {L.cr, L.cg, L.cb}) {
        ok = ok && std::isfinite(c);
        lmax = std::max(lmax, (double)std::fabs(c));
      }
    }
    const double rmax = (rb && rb->ptr) ? rb->maxabs : 0.0, lutmax = (lb && lb->ptr) ? lb->maxabs : 0.0;
    ok = ok && (double)std::fabs(P.fr) * rmax * lutmax * lmax * bound * (double)(g_tex.lights.size() + 1) < 1e36;
    P.skip_empty = ok ? 1 : 0;
    if (const char *ev = test_env("VR_NO_EMPTY_SKIP"))  // A/B switch for measurements
      if (ev[0] == '1') P.skip_empty = 0;
  }
  // Per-sample range tests the upload statistics decide for the whole launch (vr_sampling.h): every
  // opacity argument |Fa * ab(p) * tstep| below 2^-7 (the exponential's Taylor form needs no
  // per-sample check), and every |Fe * em(p) * tstep| finite (the empty-sample skip needs no
  // per-sample magnitude test).  A trilinear sample never exceeds its texture's largest |voxel|.
  {
    const BufPtr &eb = g_tex.bind[g_tex.idx_em], &ab = g_tex.bind[g_tex.idx_ab];
    auto vmax = [](const BufPtr &b) { return (b && b->ptr) ? (b->nonfinite ? INFINITY : (double)b->maxabs) : 0.0; };
    const double xa = std::fabs((double)P.fa) * vmax(ab) * (double)P.tstep;
    const double xe = std::fabs((double)P.fe) * vmax(eb) * (double)P.tstep;
    P.small_x = (std::isfinite(xa) && xa < 0x1p-7 * 0.999) ? 1 : 0;
    P.eds_finite = (std::isfinite(xe) && xe < 1e38) ? 1 : 0;
    if (diag_flag("VR_NO_RANGE_FLAGS")) P.small_x = P.eds_finite = 0;  // A/B switch (DIAG build)
  }
  {
    const bool re_ok = P.re_is_em || (P.re.p && P.re.one);
    const bool lut_ok = g_tex.lights.empty() || (P.lut.p && P.lut.small && !P.lut.one && P.lut.zp);
    // (tstep > 0: the march's t only grows, which advance_k relies on)
    const bool step_ok = std::isfinite(P.tstep) && P.tstep > 0.f;
    P.tame = (P.skip_empty && P.eds_finite && P.small_x && re_ok && lut_ok && step_ok && !diag_flag("VR_NO_TAME")) ? 1
                                                                                                            : 0;
    P.re_mask = P.re_is_em ? 0xffffffffu : 0u;
  }
  F.big = is_big(P.em) || is_big(P.ab) || is_big(P.re) || is_big(P.gem) || is_big(P.gx) || is_big(P.gy) ||
          is_big(P.gz) || test_flag("VR_FORCE_BIG");  // test switch: the 64-bit path on small volumes
  // the lookup gradient's bricked copy has 8 ceil(px/2) ceil(py/2) ceil(pz/2) entries, more than the
  // padded voxels: just under 2^32 voxels its 32-bit entry index would wrap (e.g. 1623^3)
  if (F.mode == 2 && P.gx.p &&
      vr::interleave3_entries(P.gx.px, P.gx.pxy / P.gx.px, (uint32_t)P.gx.nz + 2u) > 0xFFFFFFFFull)
    F.big = true;
  if (is_big(P.lut)) return fail(VR_ERR_UNSUPPORTED, "illumination volume larger than 2^32 voxels");
  bool finite = std::isfinite(P.tstep) && P.tstep > 0.f;
  for (int i = 0; i < 3; ++i) finite = finite && std::isfinite(P.bmin[i]) && std::isfinite(P.bscale[i]);
  // a sample-count cap every wave reaches: 2x the longest chord through the box in steps
  const double diag = std::sqrt(4.0 * ((double)bmax[0] * bmax[0] + (double)bmax[1] * bmax[1] +
                                       (double)bmax[2] * bmax[2]));
  const double cap = 2.0 * diag / (double)P.tstep + 64.0;
  P.max_steps = (finite && cap < 2.0e9) ? (int32_t)cap : 2000000000;
  F.degenerate = !finite;  // no synced emission volume: nothing to march through (renders zeros)
  return VR_OK;
}

// copyLightSources + setIlluminationTexture (render.cpp:145-191, kernel.cu:600-609,682-689)
void upload_lights(vr_context *h, const vr_render_args *a) {
  if (a->num_lights < 0 || !a->illumination) return;  // either argument is the logical false
  const size_t n = (size_t)a->num_lights;
  g_tex.lights.resize(n);
  for (size_t l = 0; l < n; ++l) {
    const vr_light &L = a->lights[l];
    g_tex.lights[l] = vr::DevLight{L.position[2], L.position[1], L.position[0], L.color[0], L.color[1],
                                   L.color[2]};
  }
  h->vol[T_LIGHT] = make_rec(a->illumination);
  sync_volume_if_changed(h, T_LIGHT, T_LIGHT);
}

// What a launch reads (vr_resources.h): every bound texture buffer (and the interleaved lookup
// gradient) is marked with the launch's completion event by finish(); the frame's light list is
// staged on the launch stream.
using LaunchRec = vr_host::LaunchRec<BufPtr>;
void wait_ready(const BufPtr &b, hipStream_t s) {  // a replica's peer copy, possibly on another stream
  if (b && !vr_host::done(b->ready)) VR_HIP(hipStreamWaitEvent(s, b->ready->e, 0));
}
void bind_reads(LaunchRec &L) {
  for (const BufPtr &b : g_tex.bind)
    if (b) {
      wait_ready(b, L.stream);
      L.reads.push_back(b);
    }
  for (const auto &kv : g_tex.gvec)
    if (kv.second.buf && kv.first == L.device) {
      wait_ready(kv.second.buf, L.stream);  // built by a launch on another stream, maybe still running
      L.reads.push_back(kv.second.buf);
    }
}
void stage_frame(LaunchRec &L, vr::RenderParams &P, const std::vector<vr::DevLight> &lights) {
  const void *d = nullptr;
  VR_HIP(L.stage(lights.data(), lights.size() * sizeof(vr::DevLight), &d));
  P.lights = static_cast<const vr::DevLight *>(d);
}

int64_t part_columns(int64_t w, int32_t bc, int32_t part, int32_t np) {
  if (w <= 0) return 0;
  if (np <= 1) return w;
  const int64_t nblocks = (w + bc - 1) / bc;
  int64_t cols = 0;
  for (int64_t b = part; b < nblocks; b += np) cols += std::min<int64_t>(bc, w - b * bc);
  return cols;
}

int validate_partition(const vr_partition *p) {
  if (!p) return VR_OK;
  if (p->num_parts < 1 || p->part < 0 || p->part >= p->num_parts || p->block_cols < 1)
    return fail(VR_ERR_ARGUMENT, "invalid partition");
  return VR_OK;
}


// Longest chunk (samples per ray) of the march built for K depth lanes (vr_march.hip VR_CHUNK);
// the staging halo's rounding margin covers that many sequential additions.
int chunk_samples(int K) { return K >= 2 ? 16 * K : 32; }
void set_chunk_halo(Frame &F, int K) {
  for (int i = 0; i < 3; ++i) {
    F.P.tap_off[i] += (float)(chunk_samples(K) * F.drift1[i]);
  }
}

void free_views(vr_context *h) {
  if (h->d_chan) (void)hipFree(h->d_chan);
  h->d_chan = nullptr;
  h->d_chan_bytes = 0;
}

void free_schedules(vr_context *h) {
  for (auto &kv : h->sched) {
    if (kv.second.copied) (void)hipEventSynchronize(kv.second.copied);
    if (kv.second.d_cost) (void)hipFree(kv.second.d_cost);
    if (kv.second.d_order) (void)hipFree(kv.second.d_order);
    if (kv.second.h_cost) (void)hipHostFree(kv.second.h_cost);
    if (kv.second.pre_flag) (void)hipFree(kv.second.pre_flag);
    if (kv.second.pre_count) (void)hipFree(kv.second.pre_count);
    if (kv.second.pre_state) (void)hipFree(kv.second.pre_state);
    if (kv.second.copied) (void)hipEventDestroy(kv.second.copied);
  }
  h->sched.clear();
}

// Depth lanes of the march kernel (lanes per ray).  One wave marches 64 / K rays;
// its run time is that of its longest ray, so the launch lasts at least as long as the slowest
// wave however many the GPU runs at once.  With few waves per wave slot of the device (a small
// image, or one GPU's share of a multi-GPU partition) K > 1 cuts that tail K-fold; with many,
// K = 1 avoids the per-group compositing overhead.  VR_DEPTH_LANES=1/2/4/8 overrides.
int device_wave_slots() {
  static int slots = 0;
  if (!slots) {
    int dev = 0, cus = 256;
    if (hipGetDevice(&dev) == hipSuccess) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, dev) == hipSuccess && prop.multiProcessorCount > 0)
        cus = prop.multiProcessorCount;
    }
    slots = cus * 16;  // the heuristics' unit: 16 waves per CU (the march runs 20-24 per CU)
  }
  return slots;
}

// Depth lanes of a launch from its length (K = 1 waves per device wave slot) and the texels a pixel
// spans (P.tau; 0 = unknown, taken as 1).  Few rounds: K = 4 shortens the tail.  Otherwise the
// staged box -- the hull of a wave's ray bundle over a chunk -- decides: its lateral extent grows
// with tau and with the tile (64 / K rays), and a hull that overflows the slot halves the chunk and
// restages.  Measured on MI355X (ms): tau 2.0 (C2, 1024x768, 3 rounds) K = 4 19.5, K = 2 29.8,
// K = 8 25.1; tau 1.07 (metric, 7.9 rounds) K = 2 36.5, K = 4 37.6, K = 1 51.7; tau 1.0 (C5,
// 4096^2, 64 rounds) K = 2 293.6, K = 4 338.5, K = 1 348.7.  K = 1 only for sparse sampling.
#ifndef VR_COUNT_K
#define VR_COUNT_K 0  // 1 (diagnostic build, as vr_march.hip): counter variants at every depth-lane count
#endif
#ifndef VR_XCD_RUN
#define VR_XCD_RUN 0  // march workgroups -> XCD runs (vr_march.hip xcd_block); 0: dispatch order
#endif

int depth_lanes(const vr::RenderParams &P) {
  if (const char *ev = test_env("VR_DEPTH_LANES")) {
    const int k = std::atoi(ev);
    if (k == 1 || k == 2 || k == 4 || (k == 8 && VR_WITH_K8)) return k;
  }
  const double waves = std::ceil(P.part_cols / 8.0) * std::ceil(P.height / 8.0);  // at K = 1
  const double rounds = waves / device_wave_slots();
  const double tau = P.tau > 0.f ? (double)P.tau : 1.0;
  // a lookup-gradient frame: K = 4, whose four consecutive samples per ray gather mostly the same
  // corner lines of the gradient copy -- C3 (tau 1.07, 7.9 rounds) 27.90-27.99 ms with 6.5 KiB slots
  // vs 28.87-28.94 at K = 2 (r5z); K = 4 with 10 KiB slots 29.8, K = 1 52.4 (r5y)
  if (P.lookup) return 4;
  if (rounds < VR_DEPTH_ROUNDS_K2 || tau >= VR_DEPTH_TAU_K4) return 4;
  if (rounds >= VR_DEPTH_ROUNDS_K1 && tau < VR_DEPTH_TAU_K1) return 1;
  return 2;
}

// texels a pixel spans at the volume, tau = dist * vw / (W * f) (pixel pitch 2/W on the image plane
// at f, box x-extent 2 = vw texels), and the wave slot size it asks for at the launch's depth lanes:
// wide (10 KiB, vr_stage.h) slots once the hull of a wave's tile passes tau 1.5 (K <= 2, tau 2.0:
// 18 % faster than 6.5 KiB), and for every K = 4 launch (round 5, below).  VR_WIDE_SLOT=0/1 overrides (A/B).
void set_tau_and_slot(vr::RenderParams &P, const vr_render_args *a, double vw) {
  const double f = std::fabs((double)a->props[1]), dist = std::fabs((double)a->props[2]);
  const double tau = (f > 0 && P.width > 0) ? dist * vw / ((double)P.width * f) : 1e30;
  P.tau = (float)std::min(tau, 1e30);
  // Round 5: with the empty-space probe the wide slots win for every K = 4 launch -- C2 (tau 2.0)
  // 12.18-12.20 vs 13.13 ms at 12 KiB (r5p), 10.90-10.93 ms at 10 KiB (r5u), the P = 8 / P = 4
  // parts of the metric frame (tau 1.07, short launches) 4.85-4.87 vs 5.26-5.27 / 8.48-8.51 vs
  // 8.81-8.83 ms (r5s; 10 KiB: 4.82-5.00 / 8.00, r5t-u); at K = 2 they still lose below
  // tau 1.5 (metric frame 30.2-30.3 vs 26.9-27.0 ms, P = 2 parts 15.15 vs 14.80-14.84 ms).  Round 4
  // measured the opposite at K = 4 (20.7 vs 19.5 ms at C2), when every empty chunk staged its box.
  const int K = P.steps ? 1 : depth_lanes(P);
  P.wide_slot = (tau > 1.5 || (K >= 4 && !P.lookup)) ? 1 : 0;  // (lookup frames: r5y above)
  if (const char *ev = test_env("VR_WIDE_SLOT")) P.wide_slot = std::atoi(ev) ? 1 : 0;
}

// The render command proper (render.cpp:134-259 minus the mxArray plumbing).
// d_out2 / eye2 (optional): fused stereo -- the same frame seen from a second eye position, into a
// second image, in the same launch (vr_render_stereo).
// fusable (optional, vr_render_channels): a frame the multi-view march can take (staged march,
// gradient mode 0/1, 32-bit addressing) is only prepared -- F.P complete, *fusable = 1, nothing
// launched; any other frame is rendered here as usual and *fusable = 0.
// Longest-first schedule: a frame of the same shape as an earlier one launches its workgroups in
// the order of that frame's measured block durations, so the long tiles start first instead of
// forming the tail (the image is the same for any order).  VR_SCHED=0: off.  Only for short
// launches (< VR_SCHED_ROUNDS K = 1 waves per device wave slot): with many rounds the tail is a
// small part of the frame and the row-major order keeps neighbouring tiles (which share voxels in
// L2) running together (metric frame: 43.6 ms row-major, 45.0 ms sorted).
// Full frames (>= VR_SCHED_ROUNDS) follow a heavy-first schedule (order_heavy_kernel: the previous
// launch's heaviest blocks first, the rest row-major): a block of rays grazing dense structure can
// last a whole frame (33 ms of 36 at rotate(30,10,0)) and, started in row-major order, forms a tail
// the rest of the frame cannot fill.  VR_SCHED=0: no schedule; VR_SCHED_FULL=0: none for full frames.
bool short_launch(const vr::RenderParams &P) {
  const double rounds = std::ceil(P.part_cols / 8.0) * std::ceil(P.height / 8.0) * std::max(1, (int)P.views) /
                        device_wave_slots();
  return rounds < VR_SCHED_ROUNDS;
}
// Very long launches (>= VR_SCHED_LPT_ROUNDS K = 1 waves per wave slot) take the short launches'
// longest-first schedule as well: C5 (V_shell(2048), 4096^2, 64 rounds) 216.6-217.1 vs 219.1-219.6 ms
// heavy-first (r5as); the metric frame (7.9 rounds) keeps heavy-first (26.58-26.60 vs 26.32-26.53, r5ae).
#ifndef VR_SCHED_LPT_ROUNDS
#define VR_SCHED_LPT_ROUNDS 32.0
#endif
bool lpt_launch(const vr::RenderParams &P) {
  const double rounds = std::ceil(P.part_cols / 8.0) * std::ceil(P.height / 8.0) * std::max(1, (int)P.views) /
                        device_wave_slots();
  return rounds < VR_SCHED_ROUNDS || rounds >= VR_SCHED_LPT_ROUNDS;
}
bool want_schedule(const vr::RenderParams &P) {
  // fused stereo (two views in one launch, vr_render_stereo) is scheduled over both views' blocks;
  // not the paired-tile measurement (VR_STEREO_PAIR), nor the multi-view channel kernel
  if (P.views > 2 || (P.views == 2 && test_flag("VR_STEREO_PAIR")) || test_flag_off("VR_SCHED")) return false;
  return test_flag("VR_SCHED") || short_launch(P) || !test_flag_off("VR_SCHED_FULL");
}

// launch_order's tail argument: (tail_pct << 32) | resident workgroups; tail_pct 0 = heavy-first.
uint64_t wg_tail_arg(uint32_t tail_pct) {
  return (uint64_t)tail_pct << 32 | (uint64_t)(device_wave_slots() / 16 * 6);
}

// What a tile block's cost depends on beyond the launch shape (round 6): the camera (eyes, axes,
// focal length), the sampling (box, step), the opacity parameters and the volume -- the emission
// buffer and the upload its occupancy map was built from.  A schedule measured or predicted under
// another key is stale (a movie turns the camera every frame, examples/example2.m:53-66).
uint64_t frame_key(const vr::RenderParams &P) {
  uint64_t h = 1469598103934665603ull;  // FNV-1a
  auto mix = [&h](const void *p, size_t n) {
    const unsigned char *c = static_cast<const unsigned char *>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  };
  mix(P.eye, sizeof P.eye);
  mix(P.eye2, sizeof P.eye2);
  mix(P.nx_, sizeof P.nx_);
  mix(P.ydir, sizeof P.ydir);
  mix(P.zdir, sizeof P.zdir);
  mix(&P.focal, sizeof P.focal);
  mix(P.bmin, sizeof P.bmin);
  mix(&P.tstep, sizeof P.tstep);
  mix(&P.thr, sizeof P.thr);
  mix(&P.fa, sizeof P.fa);
  mix(&P.fe, sizeof P.fe);
  mix(&P.em.p, sizeof P.em.p);
  mix(&P.occ, sizeof P.occ);
  const BufPtr &eb = g_tex.bind[g_tex.idx_em];
  const uint64_t ver = (eb && eb->ptr == P.em.p) ? eb->version : 0;
  mix(&ver, sizeof ver);
  return h | 1u;  // never 0
}

#ifndef VR_PRED_STEP_TEXELS
#define VR_PRED_STEP_TEXELS 8.0  // the predictor's step along a ray, in texels (one occupancy brick)
#endif
// The predicted block costs of this launch into cost[] (vr_kernels.hip predict_cost_kernel): from
// the emission texture's occupancy map, the early exit modelled with the absorption (= emission,
// the scheduled launches' aliasing) bricks' mean densities.
hipError_t predict_costs(const vr::RenderParams &P, int K, uint32_t nb_view, uint32_t *cost, hipStream_t stream) {
  const int TW = K == 1 ? 8 : (K == 2 ? 4 : (K == 4 ? 4 : 2)), TH = K <= 2 ? 8 : 4;  // vr_march.hip TileShape
  const uint32_t nbx = (uint32_t)((P.part_cols + 2 * TW - 1) / (2 * TW));
  const BufPtr &eb = g_tex.bind[g_tex.idx_em];
  double dens = 0.0;
  if (eb && !eb->nonfinite && P.fa > 0.f && std::isfinite(P.fa))
    dens = (double)P.fa * (double)eb->maxabs / 255.0 * (double)P.tstep;
  const double xthr = P.thr < 1.f ? -std::log1p(-(double)std::max(P.thr, 0.f)) : 1e30;
  // samples per predictor step: ~VR_PRED_STEP_TEXELS texels along the axis a sample advances most on
  double tpa = 0.0;  // texels per world unit, largest axis
  for (int i = 0; i < 3; ++i) {
    const float n = i == 0 ? P.em.fnx : (i == 1 ? P.em.fny : P.em.fnz);
    tpa = std::max(tpa, (double)P.bscale[i] * (double)n);
  }
  const double per = (double)P.tstep * tpa;  // texels per sample at most
  const int m = (int)std::max(1.0, std::min(4096.0, std::floor(VR_PRED_STEP_TEXELS / std::max(per, 1e-9))));
  const hipError_t rc = vr::launch_predict_cost(P, nb_view, nbx, TW, TH, m, (float)dens, (float)std::min(xthr, 1e30),
                                                cost, stream);
  // VR_SCHED_PRED_DUMP=file (DIAG build): append the predicted costs as tools/sched_dump.py's records
  if (const char *dump = rc == hipSuccess ? diag_env("VR_SCHED_PRED_DUMP") : nullptr) {
    const uint32_t nb = nb_view * (uint32_t)std::max(1, (int)P.views);
    std::vector<uint32_t> c(nb);
    VR_HIP(hipMemcpyAsync(c.data(), cost, (size_t)nb * 4, hipMemcpyDeviceToHost, stream));
    VR_HIP(hipStreamSynchronize(stream));
    const uint32_t hdr[4] = {(uint32_t)K, (uint32_t)P.part, (uint32_t)P.num_parts, nb};
    if (FILE *f = std::fopen(dump, "ab")) {
      std::fwrite(hdr, 4, 4, f);
      std::fwrite(c.data(), 4, c.size(), f);
      std::fclose(f);
    }
  }
  return rc;
}

// Attach the schedule of this launch shape (`extra` tells launches of one shape apart, e.g. the
// slab and sweep of a sort-last launch) to P: wg_order / wg_cost / sched_blocks / prio_blocks.
hipError_t attach_schedule(vr_context *h, vr::RenderParams &P, Frame &F, int K, hipStream_t stream,
                           const char *extra) {
  typedef uint32_t (*blocks_fn)(const vr::RenderParams &);
  static const blocks_fn bfns[4] = {vr::fast::march_blocks_k1, vr::fast::march_blocks_k2, vr::fast::march_blocks_k4,
                                    VR_K8(vr::fast::march_blocks_k8, vr::fast::march_blocks_k4)};
  const int ki = K == 1 ? 0 : K == 2 ? 1 : K == 4 ? 2 : 3;
  const uint32_t nb_view = bfns[ki](P);
  const uint32_t nb = nb_view * (uint32_t)std::max(1, (int)P.views);  // (fused stereo: both views' blocks)
  // keyed by stream too: the order buffer of one stream is never rewritten under another's launch
  char key[300];
  std::snprintf(key, sizeof key, "%d/%d/%d/%d/%d/%d/%d/%d/%d/%u/%p/%s", K, P.width, P.height, P.part, P.num_parts,
                P.block_cols, F.mode, P.wide_slot, P.fast_shade, nb, (void *)stream, extra);
  vr_context::Schedule &S = h->sched[key];
  F.sched = &S;
  if (!S.d_cost && nb) {
    hipError_t e = hipMalloc(&S.d_cost, nb * sizeof(uint32_t));
    if (e == hipSuccess) e = hipMalloc(&S.d_order, nb * sizeof(uint32_t));
    if (e != hipSuccess) {
      vr_host::consume(e, "hipMalloc (launch schedule; the launch runs unscheduled)");
      if (S.d_cost) (void)hipFree(S.d_cost);
      S.d_cost = nullptr;
      S.d_order = nullptr;
    }
    S.blocks = nb;
  }
  if (!(S.d_cost && S.blocks == nb)) return hipSuccess;
  hipError_t rc = hipSuccess;
  const bool full = !lpt_launch(P) && !test_flag("VR_SCHED");  // VR_SCHED=1: longest-first everywhere
  // Round 6: block costs predicted from the occupancy map (predict_costs) wherever no measurement of
  // this very frame exists -- every full frame, and a short launch whose camera or volume changed.
  // VR_SCHED_MEASURED=1 (DIAG build, A/B): the round-5 schedules from measured durations only.
  const uint64_t fkey = frame_key(P);
  const bool predict = P.occ && P.occ_bx && !diag_flag("VR_SCHED_MEASURED");
  if (!full) {  // short launch: every launch measured, ordered longest first by the previous one
    P.sched_full = 0;
    if (S.measured && S.key == fkey) {
      rc = vr::launch_order(S.d_cost, nb, S.d_order, stream, 0u, 0u);
    } else if (predict) {  // no measurement of this frame: longest first by the predicted costs
      rc = predict_costs(P, K, nb_view, S.d_cost, stream);
      if (rc == hipSuccess) rc = vr::launch_order(S.d_cost, nb, S.d_order, stream, 0u, 0u);
    } else {  // first launch of this frame without a map: row-major order, durations recorded
      rc = vr::launch_iota(S.d_order, nb, stream);
    }
    S.measured = true;  // (this launch records its durations)
    S.key = fkey;
    S.pred_key = 0;
  } else {
    // Full frame.  Round 6: the first render of a frame (camera, volume: frame_key) follows the
    // heavy-first order (order_heavy_kernel) of the block costs predicted from the occupancy map,
    // untimed -- a movie turns the camera every frame (examples/example2.m:53-66), so most of its
    // frames are first renders; the second render of the same frame runs timed in that order, and
    // once its durations have reached the host every later render follows the heavy-first order of
    // the measured durations (re-measured every VR_SCHED_REMEASURE-th render; a timed full-frame
    // kernel costs ~5 %).  Without a map (small volumes) the first render is the timed row-major
    // launch.  Whether the heaviest measured block would form a tail (>= VR_SCHED_TAIL_PCT % of the
    // packed frame: the sum of durations over the resident workgroups) decides between the
    // heavy-first order and none (round 5: VR_SCHED_TAIL_PCT 0, always heavy-first).
    if (S.key != fkey) {  // another camera or volume: what was measured does not describe this frame
      if (S.copy_pending) {
        (void)hipEventSynchronize(S.copied);
        S.copy_pending = false;
      }
      S.measured = S.decided = S.tail = S.order_stale = false;
      S.frames = S.renders = 0;
      S.key = fkey;
    }
    ++S.renders;
    uint32_t every = VR_SCHED_REMEASURE;
    if (const char *ev = test_env("VR_SCHED_REMEASURE")) every = (uint32_t)std::max(1, std::atoi(ev));
    uint32_t heavy_div = VR_SCHED_HEAVY_DIV;
    if (const char *ev = diag_env("VR_SCHED_HEAVY_DIV")) heavy_div = (uint32_t)std::max(1, std::atoi(ev));
    uint32_t tail_pct = VR_SCHED_TAIL_PCT;
    if (const char *ev = test_env("VR_SCHED_TAIL_PCT")) tail_pct = (uint32_t)std::max(0, std::atoi(ev));
    if (!S.h_cost) {
      hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&S.h_cost), nb * sizeof(uint32_t));
      if (e == hipSuccess) e = hipEventCreateWithFlags(&S.copied, hipEventDisableTiming);
      if (e != hipSuccess) {
        vr_host::consume(e, "hipHostMalloc / hipEventCreate (full-frame schedule; none used)");
        return hipSuccess;  // no schedule
      }
    }
    if (S.copy_pending && vr_host::query_done(S.copied, "hipEventQuery (schedule durations)")) {  // arrived
      S.copy_pending = false;
      uint64_t sum = 0;
      uint32_t mx = 0;
      for (uint32_t i = 0; i < nb; ++i) {
        sum += S.h_cost[i];
        mx = std::max(mx, S.h_cost[i]);
      }
      const uint64_t wg_slots = std::max<uint64_t>(1, (uint64_t)(device_wave_slots() / 16 * 6));
      S.tail = (uint64_t)mx * 100u >= (sum / wg_slots) * tail_pct;
      S.decided = true;
      S.order_stale = true;
    }
    if (predict && !S.decided) {  // nothing measured of this frame (yet): the predicted order
      if (S.pred_key != fkey) {
        rc = predict_costs(P, K, nb_view, S.d_cost, stream);
        if (rc == hipSuccess) rc = vr::launch_order(S.d_cost, nb, S.d_order, stream, heavy_div, wg_tail_arg(0));
        S.pred_key = rc == hipSuccess ? fkey : 0;
      }
      // (VR_SCHED_PREDICT_ONLY=1, DIAG build: never measured -- the predictor's own order, A/B)
      if (S.renders >= 2 && !S.measured && !diag_flag("VR_SCHED_PREDICT_ONLY")) {  // a repeated frame: measured once
        S.measured = true;
        S.frames = 0;
        P.sched_full = 1;
        F.sched_copy = &S;
      } else {
        P.sched_full = 2;
      }
    } else {
      S.pred_key = 0;  // (d_cost holds durations from here on)
      bool measure = !S.measured;
      if (S.measured && !S.copy_pending && ++S.frames >= every) measure = true;
      if (measure) {
        S.frames = 0;
        if (S.decided && S.tail) {  // measured in the heavy-first order the frames use
          if (S.order_stale) rc = vr::launch_order(S.d_cost, nb, S.d_order, stream, heavy_div, wg_tail_arg(0));
        } else {
          rc = vr::launch_iota(S.d_order, nb, stream);
        }
        S.order_stale = false;
        S.measured = true;
        P.sched_full = 1;  // timed; the durations are copied back after the launch
        F.sched_copy = &S;
      } else if (S.decided && S.tail) {
        if (S.order_stale) {
          rc = vr::launch_order(S.d_cost, nb, S.d_order, stream, heavy_div, wg_tail_arg(0));
          S.order_stale = false;
        }
        P.sched_full = 2;  // the heavy-first order, untimed
      } else {
        return hipSuccess;  // no tail (or not known yet): the unscheduled row-major launch
      }
    }
  }
  if (rc != hipSuccess) return rc;
  P.wg_order = S.d_order;
  P.wg_cost = S.d_cost;
  P.sched_blocks = nb;
  // the first round of workgroups (the longest ones) at raised wave priority (A/B: VR_PRIO_BLOCKS);
  // none for a full frame, whose first blocks are only the heavy ones
  P.prio_blocks = P.sched_full ? 0u : (uint32_t)(device_wave_slots() / 4);
  if (const char *ev = diag_env("VR_PRIO_BLOCKS")) P.prio_blocks = (uint32_t)std::atoi(ev);
  return hipSuccess;
}

// Launch timing for mem_info (the context's device must be current).
void time_mark(vr_context *h, int which, hipStream_t stream) {
  if (!h->tev[0]) {
    hipError_t e = hipEventCreate(&h->tev[0]);
    if (e == hipSuccess) e = hipEventCreate(&h->tev[1]);
    if (e != hipSuccess) {
      vr_host::consume(e, "hipEventCreate (mem_info kernel timing; not timed)");
      return;
    }
  }
  const hipError_t e = hipEventRecord(h->tev[which], stream);
  if (e != hipSuccess) vr_host::consume(e, "hipEventRecord (mem_info kernel timing; not timed)");
  if (which == 1) h->timed = true;
}

int do_render(vr_context *h, const vr_render_args *a, const vr_partition *part, float *d_out,
              unsigned long long *d_steps, hipStream_t stream, Frame &F, float *d_out2 = nullptr,
              const float *eye2 = nullptr, int *fusable = nullptr) {
  if (fusable) *fusable = 0;
  if (a->num_lights > 0 && !a->lights) return fail(VR_ERR_ARGUMENT, "lights is NULL");
  uint64_t required = required_memory(h);
  if (a->num_lights >= 0 && a->illumination) {
    required += a->illumination->dims[0] * a->illumination->dims[1] * a->illumination->dims[2] * 4 +
                (uint64_t)a->num_lights * sizeof(vr::DevLight);
    int rc = check_free_device_memory(required);
    if (rc) return rc;
  }
  upload_lights(h, a);
  required += a->resolution[0] * a->resolution[1] * sizeof(float) * 3;
  int rc = check_free_device_memory(required);
  if (rc) return rc;
  rc = build_frame(h, a, F);
  if (rc) return rc;
  rc = validate_partition(part);
  if (rc) return rc;
  vr::RenderParams &P = F.P;
  P.block_cols = part ? part->block_cols : std::max<int32_t>(P.width, 1);
  P.part = part ? part->part : 0;
  P.num_parts = part ? part->num_parts : 1;
  P.part_cols = (int32_t)part_columns(P.width, P.block_cols, P.part, P.num_parts);
  P.plane_cols = (int32_t)part_columns(P.width, P.block_cols, 0, P.num_parts);
  P.out = d_out;
  P.steps = d_steps;
  P.tile_mode = 0;
  P.lookup = F.mode == 2 ? 1 : 0;
  set_tau_and_slot(P, a, (double)h->vol[T_EM].dims[0]);  // depth lanes and wave slot size
  // shading arithmetic: hardware rsq / exp2 by default; VR_EXACT_SHADE=1 selects
  // the oracle's correctly rounded op sequence (bit-identical to oracle/vr_oracle.c up to acosf)
  P.fast_shade = env_flag("VR_EXACT_SHADE") ? 0 : 1;
  if (const char *ev = test_env("VR_TILE_MODE")) P.tile_mode = std::atoi(ev) ? 1 : 0;  // A/B switch
  // XCD runs of 16 blocks for lookup-gradient frames (their gathers of the gradient copy are the
  // launch's HBM traffic: C3 36.4 -> 35.7 ms, round 4); the compute-gradient march is indifferent
  P.xcd_run = F.mode == 2 ? 32 : VR_XCD_RUN;  // (round 5: 32 / 16 -> 31.24-31.26 / 31.43-31.67 ms, r5p)
  if (const char *ev = test_env("VR_XCD_RUN")) P.xcd_run = std::max(0, std::atoi(ev));  // A/B switch
  P.block_rot = 0;  // set at the launch (block rows of the launch's depth lanes)
  const size_t out_bytes = (size_t)P.plane_cols * (size_t)P.height * 3 * sizeof(float);
  if (d_out2) {
    P.views = 2;
    P.out2 = d_out2;
    for (int i = 0; i < 3; ++i) P.eye2[i] = eye2[i];
    drift_bound(F, eye2);  // the staging halo covers the second eye's rays too
  }
  if (F.degenerate) {
    if (out_bytes) VR_HIP(hipMemsetAsync(d_out, 0, out_bytes, stream));
    if (out_bytes && d_out2) VR_HIP(hipMemsetAsync(d_out2, 0, out_bytes, stream));
    return VR_OK;
  }
  // LDS-staged march (vr_march.hip) whenever the emission texture is a real grid and, for the
  // on-the-fly gradient, is also the gradient texture; the plain kernel covers everything else.
  // Both produce bit-identical images (tests/test_gpu_parity.py::test_kernel_variants...).
  const bool march = P.em.p && !P.em.one && (F.mode != 1 || F.share) && !test_flag("VR_NO_LDS");
  P.gvec = nullptr;
  if (march && F.mode == 2 && F.share && !test_flag("VR_NO_GVEC")) {
    // interleave the three gradient textures (one 16-byte load per voxel instead of three 4-byte
    // gathers from three volumes); without memory for it the kernel gathers them separately
    const BufPtr &bx = g_tex.bind[T_DX], &by = g_tex.bind[T_DY], &bz = g_tex.bind[T_DZ];
    TexUnit::GVec &G = g_tex.gvec[h->device];
    const uint32_t gpx = P.gx.px, gpy = P.gx.pxy / P.gx.px, gpz = (uint32_t)P.gx.nz + 2u;
    bool fresh = G.buf != nullptr;
    const DevBuf *src[3] = {bx.get(), by.get(), bz.get()};
    for (int i = 0; i < 3 && fresh; ++i) fresh = G.src[i] == src[i] && G.ver[i] == src[i]->version;
    if (!fresh) {
      G.buf.reset();
      const uint64_t n = vr::interleave3_entries(gpx, gpy, gpz);
      auto gv = std::make_shared<DevBuf>();
      gv->device = h->device;
      gv->bytes = n * 4 * sizeof(float);
      const hipError_t ea = vr_host::pooled_alloc(reinterpret_cast<void **>(&gv->ptr), gv->bytes, h->device);
      if (ea == hipSuccess) {
        for (const BufPtr *b : {&bx, &by, &bz}) wait_ready(*b, stream);
        VR_HIP(vr::launch_interleave3(bx->ptr, by->ptr, bz->ptr, gv->ptr, gpx, gpy, gpz, stream));
        // launches on other streams (another handle, a group's other children on this device) find
        // the copy fresh and wait for this event before reading it (bind_reads)
        VR_HIP(vr_host::record_event(stream, gv->ready));
        G.buf = gv;
        for (int i = 0; i < 3; ++i) {
          G.src[i] = src[i];
          G.ver[i] = src[i]->version;
        }
      } else {
        vr_host::consume(ea, "pooled_alloc (interleaved lookup gradient; three separate gathers instead)");
        gv->ptr = nullptr;
      }
    }
    if (G.buf) {
      P.gvec = G.buf->ptr;
      P.gv_row8 = 8u * ((gpx + 1) >> 1);
      P.gv_plane8 = P.gv_row8 * ((gpy + 1) >> 1);
    }
  }
  if (fusable && march && F.mode <= 1 && !F.big && !P.steps) {
    *fusable = 1;
    return VR_OK;
  }
  LaunchRec L;
  L.stream = stream;
  L.device = h->device;
  bind_reads(L);
  stage_frame(L, P, g_tex.lights);
  if (march) {
    // the counter variant: K = 1 (VR_COUNT_PROD=1 with a VR_COUNT_K=1 build: the production K's chunk
    // statistics; its sample sums are then 0)
    // (VR_COUNT_PROD is honoured by a VR_COUNT_K build only: a normal build has no counted K > 1 kernel)
    const int K = (P.steps && !(VR_COUNT_K && test_flag("VR_COUNT_PROD"))) ? 1
                                                                          : exact_lanes(depth_lanes(P), P.fast_shade);
    set_chunk_halo(F, K);
    typedef hipError_t (*launch_fn)(const vr::RenderParams &, int, bool, bool, bool, hipStream_t);
    typedef uint32_t (*blocks_fn)(const vr::RenderParams &);
    static const launch_fn fns[2][4] = {
        {vr::exact::launch_march_k1, vr::exact::launch_march_k2,
         VR_EXACT_K4(vr::exact::launch_march_k4, vr::exact::launch_march_k2),
         VR_K8(vr::exact::launch_march_k8, vr::exact::launch_march_k2)},
        {vr::fast::launch_march_k1, vr::fast::launch_march_k2, vr::fast::launch_march_k4,
         VR_K8(vr::fast::launch_march_k8, vr::fast::launch_march_k4)}};
    const int ki = K == 1 ? 0 : K == 2 ? 1 : K == 4 ? 2 : 3;
    // (the exact-arithmetic variant is a parity reference: built without the scheduled kernels)
    // (scheduled kernels exist for absorption = emission only: vr_march.hip launch_c)
    if (!P.steps && K > 1 && P.fast_shade && F.ab_alias && want_schedule(P))
      VR_HIP(attach_schedule(h, P, F, K, stream, ""));
    if (P.views > 1) {
      static const blocks_fn vfns[4] = {vr::fast::march_blocks_k1, vr::fast::march_blocks_k2,
                                        vr::fast::march_blocks_k4,
                                        VR_K8(vr::fast::march_blocks_k8, vr::fast::march_blocks_k4)};
      P.view_blocks = vfns[ki](P);
      // VR_STEREO_PAIR=1 (measurement): paired tiles -- the left eye's rays of
      // column c + shift share a wave (and its staged box) with the right eye's of column c, the
      // shift (whole tiles) making the two bundles meet at the volume's centre, at distance `dist`
      // from the eyes: base * W * f / dist columns
      if (test_flag("VR_STEREO_PAIR") && K > 1 && P.fast_shade && F.mode == 1 && F.ab_alias && P.tap_half &&
          !P.wide_slot && !F.big && P.num_parts == 1 && !P.wg_order) {
        const double base = std::fabs((double)a->props[0]), f = std::fabs((double)a->props[1]),
                     dist = std::fabs((double)a->props[2]);
        const int TW = 4;  // tile width at K = 2, 4 (vr_march.hip TileShape)
        const double cols = dist > 0 ? base * (double)P.width * f / dist : 0.0;
        P.pair_shift = (int32_t)std::min<double>(std::floor(cols / TW + 0.5) * TW, (double)P.width);
        if (const char *ev = test_env("VR_STEREO_PAIR_SHIFT")) P.pair_shift = std::max(0, std::atoi(ev));
      }
    }
    // diagnostics (VR_SCHED_DUMP): a timed launch also records its blocks' start ticks
    const char *dump = (P.wg_cost && P.sched_full != 2) ? test_env("VR_SCHED_DUMP") : nullptr;
    uint32_t *d_start = nullptr;
    if (dump) {
      const hipError_t e = hipMalloc(reinterpret_cast<void **>(&d_start), (size_t)P.sched_blocks * 4);
      if (e == hipSuccess) P.wg_start = d_start;
      else vr_host::consume(e, "hipMalloc (VR_SCHED_DUMP start ticks; not recorded)");
    }
    // VR_BLOCK_ROT_ROWS=r (A/B): the unscheduled launch starts at block row r of the row-major order
    // and wraps (the light top rows then fill the ramp-down of the heavy middle band)
    if (const char *ev = test_env("VR_BLOCK_ROT_ROWS")) {
      const int TW = K == 1 ? 8 : (K == 2 ? 4 : (K == 4 ? 4 : 2));
      const uint32_t nbx = (uint32_t)((P.part_cols + 2 * TW - 1) / (2 * TW));
      typedef uint32_t (*bfn)(const vr::RenderParams &);
      static const bfn bf[4] = {vr::fast::march_blocks_k1, vr::fast::march_blocks_k2, vr::fast::march_blocks_k4,
                                VR_K8(vr::fast::march_blocks_k8, vr::fast::march_blocks_k4)};
      const uint32_t nb = bf[ki](P) * (P.views > 1 ? 2u : 1u);
      const uint64_t rot = (uint64_t)std::max(0, std::atoi(ev)) * nbx;
      P.block_rot = nb ? (uint32_t)(rot % nb) : 0u;
    }
    // the pre-leap launch (vr_march.hip preleap_kernel, round 6): scheduled tame launches with an
    // occupancy map; its buffers live with the launch shape's schedule (one per stream)
    if (VR_PRELEAP_LAUNCH && F.sched && F.sched->blocks && P.occ && P.tame && !P.pair_shift && P.fast_shade &&
        !test_flag("VR_NO_PRELEAP")) {
      vr_context::Schedule &S = *F.sched;
      const uint32_t waves = S.blocks * (uint32_t)VR_WG_WAVES_HOST;
      if (S.pre_waves != waves) {
        if (S.pre_flag) (void)hipFree(S.pre_flag);
        if (S.pre_state) (void)hipFree(S.pre_state);
        S.pre_flag = nullptr;
        S.pre_state = nullptr;
        S.pre_waves = S.pre_cap = 0;
        const uint32_t cap = std::max<uint32_t>(64u, waves / 8u);  // slots: an eighth of the waves
        hipError_t e = S.pre_count ? hipSuccess : hipMalloc(reinterpret_cast<void **>(&S.pre_count), 4);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&S.pre_flag), (size_t)waves * 4);
        if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&S.pre_state), (size_t)cap * 64 * 2 * sizeof(float4));
        if (e == hipSuccess) {
          S.pre_waves = waves;
          S.pre_cap = cap;
        } else {
          vr_host::consume(e, "hipMalloc (pre-leap buffers; the launch marches without)");
        }
      }
      if (S.pre_waves == waves) {
        P.pre_flag = S.pre_flag;
        P.pre_state = S.pre_state;
        P.pre_count = S.pre_count;
        P.pre_cap = S.pre_cap;
        typedef hipError_t (*pre_fn)(const vr::RenderParams &, hipStream_t);
        static const pre_fn pfns[4] = {vr::fast::launch_preleap_k1, vr::fast::launch_preleap_k2,
                                       vr::fast::launch_preleap_k4,
                                       VR_K8(vr::fast::launch_preleap_k8, vr::fast::launch_preleap_k4)};
        VR_HIP(hipMemsetAsync(S.pre_count, 0, 4, stream));
        VR_HIP(pfns[ki](P, stream));
      }
    }
    time_mark(h, 0, stream);
    {
      const hipError_t e = fns[P.fast_shade ? 1 : 0][ki](P, F.mode, F.ab_alias, F.share, F.big, stream);
      if (e != hipSuccess) throw HipError{e, "the march kernel launch (launch_march_k)"};
    }
    time_mark(h, 1, stream);
    if (F.sched_copy) {  // a timed full frame: its block durations to the host, for the tail test
      vr_context::Schedule &S = *F.sched_copy;
      VR_HIP(hipMemcpyAsync(S.h_cost, S.d_cost, (size_t)S.blocks * sizeof(uint32_t), hipMemcpyDeviceToHost, stream));
      VR_HIP(hipEventRecord(S.copied, stream));
      S.copy_pending = true;
      F.sched_copy = nullptr;
    }
    if (dump) {  // diagnostics: append block durations (and, in DUMP.start, their start ticks)
      std::vector<uint32_t> c(P.sched_blocks), st(d_start ? P.sched_blocks : 0);
      VR_HIP(hipMemcpyAsync(c.data(), P.wg_cost, c.size() * 4, hipMemcpyDeviceToHost, stream));
      if (d_start) VR_HIP(hipMemcpyAsync(st.data(), d_start, st.size() * 4, hipMemcpyDeviceToHost, stream));
      VR_HIP(hipStreamSynchronize(stream));
      if (d_start) (void)hipFree(d_start);
      const uint32_t hdr[4] = {(uint32_t)K, (uint32_t)P.part, (uint32_t)P.num_parts, P.sched_blocks};
      if (FILE *f = std::fopen(dump, "ab")) {
        std::fwrite(hdr, 4, 4, f);
        std::fwrite(c.data(), 4, c.size(), f);
        std::fclose(f);
      }
      if (d_start)
        if (FILE *f = std::fopen((std::string(dump) + ".start").c_str(), "ab")) {
          std::fwrite(hdr, 4, 4, f);
          std::fwrite(st.data(), 4, st.size(), f);
          std::fclose(f);
        }
    }
  } else {
    VR_HIP(vr::launch_render(P, F.mode, F.ab_alias, F.big, F.share, stream));
    if (P.views > 1) {  // the general kernel renders one view per launch
      for (int i = 0; i < 3; ++i) P.eye[i] = P.eye2[i];
      P.out = P.out2;
      VR_HIP(vr::launch_render(P, F.mode, F.ab_alias, F.big, F.share, stream));
    }
  }
  VR_HIP(L.finish());
  return VR_OK;
}

// Sort-last slab render: the handle's emission volume holds planes
// [z_first, z_first + d2) of a volume of depth `depth`; the frame is built for the whole volume
// (box, step, gradient offsets) and the march takes the samples of [z0, z1) only.
int do_render_slab(vr_context *h, const vr_render_args *a, const vr_slab *sl, const vr_partition *part,
                   const float *d_in, float *d_out, hipStream_t stream, Frame &F) {
  if (!sl || !d_out) return fail(VR_ERR_ARGUMENT, "slab / output is NULL");
  if (sl->depth == 0 || sl->z_first >= sl->depth || (sl->direction < -1 || sl->direction > 1))
    return fail(VR_ERR_ARGUMENT, "invalid slab");
  if (a->num_lights > 0 && !a->lights) return fail(VR_ERR_ARGUMENT, "lights is NULL");
  upload_lights(h, a);
  int rc = build_frame(h, a, F, sl->depth);
  if (rc) return rc;
  vr::RenderParams &P = F.P;
  if (F.degenerate || !P.em.p || P.em.one) return fail(VR_ERR_UNSUPPORTED, "slab render needs a synced emission volume");
  // the planes resident are those of the BOUND emission texture (the last sync_volumes of any
  // handle, as every render reads -- render.cpp binds globally); the slab must lie inside them
  const uint64_t res_nz = (uint64_t)P.em.nz, res_nx = (uint64_t)P.em.nx;
  if (sl->z_first + res_nz > sl->depth) return fail(VR_ERR_ARGUMENT, "invalid slab: bound planes exceed the depth");
  if (F.mode == 2 || !F.ab_alias) return fail(VR_ERR_UNSUPPORTED, "slab render: lookup gradients / separate absorption");
  // the resident planes addressed by their global padded index: virtual base z_first planes back
  const bool re_em = P.re_is_em != 0;
  P.occ = nullptr;  // (the probe is not used by the slab march; the map would be the slab's own)
  P.em.p = P.em.p - (ptrdiff_t)(sl->z_first * (uint64_t)P.em.pxy);
  P.em.nz = (int32_t)sl->depth;
  P.em.fnz = (float)sl->depth;
  P.gem = P.em;
  if (re_em) P.re = P.em;
  P.ab = P.em;
  // resident padded planes holding the right data: the synced planes, plus the edge-replicating
  // apron planes only at the ends of the whole volume
  P.slab_pk0 = (int32_t)(sl->z_first + (sl->z_first > 0 ? 1 : 0));
  P.slab_pk1 = (int32_t)(sl->z_first + res_nz + 1 + (sl->z_first + res_nz == sl->depth ? 1 : 0));
  const double D = (double)sl->depth;
  P.slab_z0 = std::isfinite(sl->z0) ? (float)(sl->z0 / D) : -INFINITY;
  P.slab_z1 = std::isfinite(sl->z1) ? (float)(sl->z1 / D) : INFINITY;
  // the z halo of build_frame was sized by the resident depth: redo it for the whole volume
  {
    double pmax = 0.0;
    for (int i = 0; i < 3; ++i) pmax = std::max(pmax, (double)std::fabs(P.bmin[i]) + std::fabs(P.eye[i]));
    F.drift1[2] = 2.0 * pmax * 1.2e-7 * (double)P.bscale[2] * D;
    P.tap_off[2] = (float)((F.mode == 1 ? (double)P.gstep[2] * P.bscale[2] * D : 0.0) + 0.0625);
    P.tap_half = half_texel_taps(P, F.mode, (float)D);  // judged on the whole volume, as one render
    for (int i = 0; i < 3; ++i)  // (the cube's n / 2 per axis, the whole volume's depth on z)
      P.cube_hs[i] = P.tap_half ? (i == 0 ? P.em.fnx : i == 1 ? P.em.fny : (float)D) * 0.5f : 0.f;
  }
  P.slab_dir = sl->direction;
  P.slab_in = d_in;
  rc = validate_partition(part);
  if (rc) return rc;
  P.block_cols = part ? part->block_cols : std::max<int32_t>(P.width, 1);
  P.part = part ? part->part : 0;
  P.num_parts = part ? part->num_parts : 1;
  P.part_cols = (int32_t)part_columns(P.width, P.block_cols, P.part, P.num_parts);
  P.plane_cols = P.part_cols;  // the state of a part is dense: VR_SLAB_PLANES [part_cols][H] planes
  if ((uint64_t)P.part_cols * (uint64_t)P.height >= (1ull << 32))
    return fail(VR_ERR_UNSUPPORTED, "slab render: more than 2^32 rays in one part");
  P.out = d_out;
  P.fast_shade = env_flag("VR_EXACT_SHADE") ? 0 : 1;
  P.steps = nullptr;
  // depth lanes (and slot) as for the one-volume march of the whole frame: the tiles of a sweep run
  // back to back and overlap on the sweep's streams, so one tile's launch tail is not the frame's
  // (4 tiles on one MI355X: 1.25x the plain render at the frame's K = 2, 1.36x at a tile's K = 4)
  const int32_t tile_cols = P.part_cols;
  P.part_cols = P.width;
  set_tau_and_slot(P, a, (double)res_nx);
  int K = depth_lanes(P);
  P.part_cols = tile_cols;
  if (K > 4) K = 4;
  K = exact_lanes(K, P.fast_shade);
  set_chunk_halo(F, K);
  P.slab_margin = P.tap_off[2] / P.em.fnz;  // bound of the chunk ownership test, normalized
  typedef hipError_t (*slab_fn)(const vr::RenderParams &, int, hipStream_t);
  static const slab_fn sfns[2][3] = {
      {vr::exact::launch_march_slab_k1, vr::exact::launch_march_slab_k2,
       VR_EXACT_K4(vr::exact::launch_march_slab_k4, vr::exact::launch_march_slab_k2)},
      {vr::fast::launch_march_slab_k1, vr::fast::launch_march_slab_k2, vr::fast::launch_march_slab_k4}};
  LaunchRec L;
  L.stream = stream;
  L.device = h->device;
  bind_reads(L);
  stage_frame(L, P, g_tex.lights);
  if (K > 1 && want_schedule(P) && short_launch(P)) {  // a tile of a sweep: longest-first schedule
    char extra[120];
    std::snprintf(extra, sizeof extra, "slab/%llu/%llu/%g/%g/%d", (unsigned long long)sl->depth,
                  (unsigned long long)sl->z_first, sl->z0, sl->z1, sl->direction);
    VR_HIP(attach_schedule(h, P, F, K, stream, extra));
  }
  VR_HIP(sfns[P.fast_shade ? 1 : 0][K == 1 ? 0 : (K == 2 ? 1 : 2)](P, F.mode, stream));
  VR_HIP(L.finish());
  return VR_OK;
}

// ---- multi-device group (vr_new_multi) ----------------------------------------------------------

// A device-to-device copy through pinned host memory, for device pairs without a peer mapping: the
// D2H is issued on `ss` (a stream of sdev) -- synchronously when ss is null --, the H2D on `ds` (a
// stream of ddev) after it.  Through the caller's pinned buffer `stage` (which the caller keeps
// until the H2D has completed), or through one allocated here and released when the H2D has
// completed (or at once if a call fails).  Returns the completion event of the H2D.
vr_host::EventPtr staged_copy(void *dst, int ddev, hipStream_t ds, const void *src, int sdev, hipStream_t ss,
                              size_t bytes, void *stage = nullptr) {
  struct Own {  // the buffer allocated here, freed on an error path
    void *p = nullptr;
    ~Own() {
      if (p) (void)hipHostFree(p);
    }
  } own;
  void *pin = stage;
  if (!pin) {
    VR_HIP(hipHostMalloc(&own.p, bytes, hipHostMallocDefault));
    pin = own.p;
  }
  vr_host::EventPtr e1, e2;
  {
    DeviceGuard g(sdev);
    if (ss) {
      VR_HIP(hipMemcpyAsync(pin, src, bytes, hipMemcpyDeviceToHost, ss));
      VR_HIP(vr_host::record_event(ss, e1));
    } else {
      VR_HIP(hipMemcpy(pin, src, bytes, hipMemcpyDeviceToHost));
    }
  }
  DeviceGuard g(ddev);
  if (e1) VR_HIP(hipStreamWaitEvent(ds, e1->e, 0));
  VR_HIP(hipMemcpyAsync(dst, pin, bytes, hipMemcpyHostToDevice, ds));
  VR_HIP(vr_host::record_event(ds, e2));
  if (own.p) {
    vr_host::free_when_done(own.p, ddev, vr_host::readers_of(e2), true);
    own.p = nullptr;
  }
  return e2;
}

// The copy of buffer b on device `dev`, refreshed when b was re-uploaded since (peer copy over xGMI on
// the device's group stream; a replica a launch still reads is replaced, not overwritten).
BufPtr replicate(const BufPtr &b, int dev, hipStream_t s, bool peer = true) {
  if (!b) return b;
  if (b->device == dev && !test_flag("VR_GROUP_REPLICATE")) return b;  // test switch: copy on one device too
  BufPtr &r = b->replicas[dev];
  if (r && r->bytes == b->bytes && b->replica_of[dev] == b->version) return r;
  if (!(r && r->bytes == b->bytes && r->readers.done())) {
    r = std::make_shared<DevBuf>();
    r->device = dev;
    r->bytes = b->bytes;
    if (b->bytes) {
      DeviceGuard dg(dev);
      VR_HIP(vr_host::pooled_alloc(reinterpret_cast<void **>(&r->ptr), b->bytes, dev));
    }
  }
  if (b->bytes) {
    vr_host::EventPtr ev;
    if (peer) {
      VR_HIP(hipMemcpyPeerAsync(r->ptr, dev, b->ptr, b->device, b->bytes, s));
      // the occupancy map along with it (peer copies only; a staged replica marches without probes)
      if (b->occ && r->occ_bytes != b->occ_bytes) {
        if (r->occ) vr_host::pooled_free(r->occ, r->occ_bytes, dev, vr_host::Readers(r->readers));
        r->occ = nullptr;
        r->occ_bytes = 0;
        DeviceGuard dg(dev);
        VR_HIP(vr_host::pooled_alloc(reinterpret_cast<void **>(&r->occ), b->occ_bytes, dev));
        r->occ_bytes = b->occ_bytes;
      }
      if (b->occ) VR_HIP(hipMemcpyPeerAsync(r->occ, dev, b->occ, b->device, b->occ_bytes, s));
      VR_HIP(vr_host::record_event(s, ev));
    }
    if (!(peer && b->occ) && r->occ) {  // no map copied: none (a stale one would leap wrongly)
      vr_host::pooled_free(r->occ, r->occ_bytes, dev, vr_host::Readers(r->readers));
      r->occ = nullptr;
      r->occ_bytes = 0;
    }
    if (!peer) {  // no peer mapping: through pinned host memory (b is resident: its D2H runs now)
      if (b->ready) vr_host::wait(b->ready);
      ev = staged_copy(r->ptr, dev, s, b->ptr, b->device, nullptr, b->bytes);
    }
    // the copy reads b and writes r: neither is rewritten, pooled or freed before it completes
    b->readers.add(ev);
    r->readers.add(ev);
    r->ready = ev;
  }
  for (int i = 0; i < 3; ++i) r->dims[i] = b->dims[i];
  r->nonfinite = b->nonfinite;
  r->maxabs = b->maxabs;
  r->src_data = b->src_data;
  r->src_last_update = b->src_last_update;
  r->src_bytes = b->src_bytes;
  r->version = next_version();
  b->replica_of[dev] = b->version;
  return r;
}

// Whether device a may map b's memory (the mapping enabled); false: copies between them are staged
// through pinned host memory (staged_copy).
bool enable_peer(int a, int b) {
  if (a == b) return true;
  int ok = 0;
  const hipError_t q = hipDeviceCanAccessPeer(&ok, a, b);
  if (q != hipSuccess) {
    vr_host::consume(q, "hipDeviceCanAccessPeer (group peer mapping; copies staged through the host)");
    return false;
  }
  if (!ok) return false;
  DeviceGuard dg(a);
  const hipError_t e = hipDeviceEnablePeerAccess(b, 0);
  if (e == hipSuccess) return true;
  vr_host::consume(e, "hipDeviceEnablePeerAccess (group peer mapping)");
  return e == hipErrorPeerAccessAlreadyEnabled;
}

// After a sync of the primary: the children record the same volumes, and the bound volumes are
// copied to their devices now (one H2D to the primary, then peer copies), not in the render.
void group_sync(vr_context *h) {
  for (vr_context *c : h->children) {
    DeviceGuard dg(c->device);
    for (int t = 0; t < T_COUNT; ++t) c->vol[t] = h->vol[t];
    c->time_last_mem_sync = h->time_last_mem_sync;
    for (int t = 0; t < T_COUNT; ++t)
      if (t != T_LIGHT && g_tex.bind[t]) (void)replicate(g_tex.bind[t], c->device, c->gstream, c->peer);
  }
}

// Part buffers of a group frame of `nviews` images: the primary's h->d_part holds every device's
// parts view-major (view v, device k at (v * n + k) * part_floats: one view's parts are contiguous,
// as vr_assemble_partitions reads them); a child's d_part its own nviews parts.
void ensure_part_buffers(vr_context *h, int n, size_t part_floats, int nviews) {
  const size_t pb = (size_t)n * (size_t)nviews * part_floats * sizeof(float);
  if (h->d_part_bytes < pb) {
    if (h->d_part) VR_HIP(hipFree(h->d_part));
    h->d_part = nullptr;
    h->d_part_bytes = 0;
    VR_HIP(vr_host::device_alloc(reinterpret_cast<void **>(&h->d_part), pb));
    h->d_part_bytes = pb;
  }
  for (vr_context *c : h->children) {
    DeviceGuard dg(c->device);
    const size_t cb = (size_t)nviews * part_floats * sizeof(float);
    if (c->d_part_bytes < cb) {
      if (c->d_part) VR_HIP(hipFree(c->d_part));
      c->d_part = nullptr;
      c->d_part_bytes = 0;
      VR_HIP(vr_host::device_alloc(reinterpret_cast<void **>(&c->d_part), cb));
      c->d_part_bytes = cb;
    }
  }
}

// Bind, for a render on child c, the replicas of the primary's bindings `saved` on c's device (the
// LUT is c's own upload, which do_render keeps resident).
void bind_replicas(vr_context *h, vr_context *c, const BufPtr (&saved)[T_COUNT]) {
  for (int t = 0; t < T_COUNT; ++t) c->vol[t] = h->vol[t];
  for (int t = 0; t < T_COUNT; ++t)
    g_tex.bind[t] = t == T_LIGHT ? c->buf[T_LIGHT] : replicate(saved[t], c->device, c->gstream, c->peer);
}

// Gather every child's parts (nviews images each) into the primary's part buffer over xGMI and
// assemble each view into d_outs[v] on the primary's `stream`.
void group_gather_assemble(vr_context *h, int nviews, size_t part_floats, int64_t W, int64_t H, int32_t bc,
                           int64_t maxc, float *const *d_outs, hipStream_t stream) {
  const int n = 1 + (int)h->children.size();
  for (int k = 1; k < n; ++k) {
    vr_context *c = h->children[k - 1];
    DeviceGuard dg(c->device);
    // the previous frame's assembly has read these slots of the primary's part buffer
    VR_HIP(hipStreamWaitEvent(c->gstream, h->gdone, 0));
    if (c->peer) {
      for (int v = 0; v < nviews; ++v)
        VR_HIP(hipMemcpyPeerAsync(h->d_part + ((size_t)v * n + k) * part_floats, h->device,
                                  c->d_part + (size_t)v * part_floats, c->device, part_floats * sizeof(float),
                                  c->gstream));
    } else {  // no peer mapping: D2H on the child's stream, H2D on the primary's (after the previous
              // frame's assembly, which read these slots, in that stream's order), through the
              // child's persistent pinned buffer (its previous contents read by that assembly's H2Ds)
      const size_t vb = part_floats * sizeof(float);
      if (c->pin_bytes < (size_t)nviews * vb) {
        if (c->pin) vr_host::free_when_done(c->pin, c->device, vr_host::readers_of(c->pin_read), true);
        c->pin = nullptr;
        c->pin_bytes = 0;
        c->pin_read.reset();
        VR_HIP(hipHostMalloc(&c->pin, (size_t)nviews * vb, hipHostMallocDefault));
        c->pin_bytes = (size_t)nviews * vb;
      }
      for (int v = 0; v < nviews; ++v)
        c->pin_read = staged_copy(h->d_part + ((size_t)v * n + k) * part_floats, h->device, stream,
                                  c->d_part + (size_t)v * part_floats, c->device, c->gstream, vb,
                                  static_cast<char *>(c->pin) + (size_t)v * vb);
    }
    VR_HIP(hipEventRecord(c->gdone, c->gstream));
  }
  for (vr_context *c : h->children) VR_HIP(hipStreamWaitEvent(stream, c->gdone, 0));
  for (int v = 0; v < nviews; ++v)
    VR_HIP(vr::launch_assemble(h->d_part + (size_t)v * n * part_floats, W, H, bc, n, maxc, d_outs[v], stream));
  VR_HIP(hipEventRecord(h->gdone, stream));
}

// 'render' on a group: child k renders column part k (16-column blocks dealt round-robin, as
// bench.py's ranks), the primary part 0; the children's parts are peer-copied into the primary's
// part buffer and assembled there into d_out (the primary's device, on `stream`).  With d_out2 /
// eye2 every device renders its part of both eyes of a stereo pair (vr_render_stereo) in one launch.
// The module-global bindings are the primary's again when this returns.
int group_render(vr_context *h, const vr_render_args *a, float *d_out, hipStream_t stream, float *d_out2 = nullptr,
                 const float *eye2 = nullptr) {
  const int n = 1 + (int)h->children.size();
  const int nviews = d_out2 ? 2 : 1;
  const int32_t bc = 16;
  const int64_t W = (int64_t)a->resolution[1], H = (int64_t)a->resolution[0];
  vr_partition p0{bc, 0, n, 0};
  const int64_t maxc = part_columns(W, bc, 0, n);
  const size_t part_floats = (size_t)maxc * (size_t)H * 3;
  if (!part_floats) {
    Frame F;
    return do_render(h, a, nullptr, d_out, nullptr, stream, F, d_out2, eye2);
  }
  ensure_part_buffers(h, n, part_floats, nviews);
  // the primary's part first: it uploads the frame's lights / LUT and binds them.  Its slots of the
  // part buffer are read by the previous frame's assembly, which may run on another stream.
  VR_HIP(hipStreamWaitEvent(stream, h->gdone, 0));
  Frame F0;
  int rc = do_render(h, a, &p0, h->d_part, nullptr, stream, F0, d_out2 ? h->d_part + (size_t)n * part_floats : nullptr,
                     eye2);
  if (rc) return rc;
  BufPtr saved[T_COUNT];
  for (int t = 0; t < T_COUNT; ++t) saved[t] = g_tex.bind[t];
  for (int k = 1; k < n && !rc; ++k) {
    vr_context *c = h->children[k - 1];
    DeviceGuard dg(c->device);
    bind_replicas(h, c, saved);
    vr_partition pk{bc, k, n, 0};
    Frame F;
    rc = do_render(c, a, &pk, c->d_part, nullptr, c->gstream, F, d_out2 ? c->d_part + part_floats : nullptr, eye2);
  }
  for (int t = 0; t < T_COUNT; ++t) g_tex.bind[t] = saved[t];
  if (rc) return rc;
  float *outs[2] = {d_out, d_out2};
  group_gather_assemble(h, nviews, part_floats, W, H, bc, maxc, outs, stream);
  return VR_OK;
}

// Group streams are never destroyed.  Events recorded on them (replica copies, group renders) live on
// after the group is deleted -- in the reader lists of buffers that stay bound, pooled or retired --
// and a later query of such an event reads the runtime's stream object: destroyed, that read gave
// spurious stream-capture errors (hipErrorCapturedEvent / hipErrorStreamCaptureUnsupported from
// unrelated calls, intermittently).  A deleted group's streams wait here for the next group.
std::map<int, std::vector<hipStream_t>> &idle_streams() {
  static std::map<int, std::vector<hipStream_t>> &m = *new std::map<int, std::vector<hipStream_t>>();
  return m;
}
hipError_t take_stream(int dev, hipStream_t *s) {  // dev is current
  std::vector<hipStream_t> &v = idle_streams()[dev];
  if (!v.empty()) {
    *s = v.back();
    v.pop_back();
    return hipSuccess;
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}
void give_stream(int dev, hipStream_t s) {  // s is idle
  if (s) idle_streams()[dev].push_back(s);
}

void delete_children(vr_context *h) {
  for (vr_context *c : h->children) {
    DeviceGuard dg(c->device);
    (void)hipStreamSynchronize(c->gstream);
    for (auto &b : c->buf) b.reset();
    if (c->d_part) (void)hipFree(c->d_part);
    if (c->d_out) (void)hipFree(c->d_out);
    if (c->pin) vr_host::free_when_done(c->pin, c->device, vr_host::readers_of(c->pin_read), true);
    c->pin = nullptr;
    free_schedules(c);
    free_views(c);
    if (c->gdone) (void)hipEventDestroy(c->gdone);
    for (hipEvent_t e : c->tev)
      if (e) (void)hipEventDestroy(e);
    give_stream(c->device, c->gstream);
    delete c;
  }
  h->children.clear();
}

// At entry, an error already in this thread's HIP error state (another library's, or an
// asynchronous device fault) is logged, and a device fault fails the call (vr_host::check_pending):
// this call's own checks then see only its own errors.
#define VR_GUARD_BEGIN \
  try {                \
    vr_host::check_pending(__func__);
#define VR_GUARD_END                                                                             \
  }                                                                                              \
  catch (const HipError &e) {                                                                    \
    return fail(VR_ERR_DEVICE, std::string(hipGetErrorString(e.e)) + " in " + e.what);           \
  }                                                                                              \
  catch (const std::bad_alloc &) {                                                               \
    return fail(VR_ERR_DEVICE, "host out of memory");                                            \
  }

double mb(uint64_t b) { return (double)b / (1024.0 * 1024.0); }

// imresize's contributions along one axis (Volume.resize -> imresize3, Volume.m:93-106; MATLAB's
// default: cubic kernel of width 4, antialiasing when shrinking): per output index o (1-based x),
// u = x/scale + (1 - 1/scale)/2, the P = ceil(width) + 2 taps from floor(u - width/2), weights
// h(u - index) normalised by their row sum, indices mirrored at the ends ([1..n, n..1]), columns
// that are zero for every output removed.  Double precision throughout; 0-based indices out.
double cubic(double x) {
  const double ax = std::fabs(x), ax2 = ax * ax, ax3 = ax * ax * ax;
  return (1.5 * ax3 - 2.5 * ax2 + 1.0) * (ax <= 1.0 ? 1.0 : 0.0) +
         (-0.5 * ax3 + 2.5 * ax2 - 4.0 * ax + 2.0) * ((1.0 < ax && ax <= 2.0) ? 1.0 : 0.0);
}
void resize_contributions(uint64_t in_len, uint64_t out_len, std::vector<double> &w, std::vector<int32_t> &idx,
                          int32_t &P) {
  const double scale = (double)out_len / (double)in_len;
  const bool aa = scale < 1.0;
  const double width = aa ? 4.0 / scale : 4.0;
  const int32_t P0 = (int32_t)std::ceil(width) + 2;
  std::vector<double> w0((size_t)out_len * P0);
  std::vector<int64_t> i0((size_t)out_len * P0);
  for (uint64_t o = 0; o < out_len; ++o) {
    const double x = (double)(o + 1);
    const double u = x / scale + 0.5 * (1.0 - 1.0 / scale);
    const double left = std::floor(u - width / 2.0);
    double sum = 0.0;
    for (int32_t p = 0; p < P0; ++p) {
      const double ind = left + p;
      const double d = u - ind;
      const double h = aa ? scale * cubic(scale * d) : cubic(d);
      w0[o * P0 + p] = h;
      i0[o * P0 + p] = (int64_t)ind;
      sum = sum + h;
    }
    for (int32_t p = 0; p < P0; ++p) w0[o * P0 + p] = w0[o * P0 + p] / sum;
  }
  // mirror: aux = [1:n, n:-1:1], index -> aux(mod(index - 1, 2n) + 1)
  const int64_t n = (int64_t)in_len, m = 2 * n;
  for (auto &i : i0) {
    int64_t k = (i - 1) % m;
    if (k < 0) k += m;
    i = k < n ? k : (m - 1 - k);  // 0-based
  }
  std::vector<char> keep(P0, 0);
  for (uint64_t o = 0; o < out_len; ++o)
    for (int32_t p = 0; p < P0; ++p)
      if (w0[o * P0 + p] != 0.0) keep[p] = 1;
  P = 0;
  for (int32_t p = 0; p < P0; ++p) P += keep[p];
  w.assign((size_t)out_len * P, 0.0);
  idx.assign((size_t)out_len * P, 0);
  for (uint64_t o = 0; o < out_len; ++o) {
    int32_t q = 0;
    for (int32_t p = 0; p < P0; ++p) {
      if (!keep[p]) continue;
      w[o * P + q] = w0[o * P0 + p];
      idx[o * P + q] = (int32_t)i0[o * P0 + p];
      ++q;
    }
  }
}

}  // namespace

extern "C" {

int vr_new(vr_context **out) {
  if (!out) return fail(VR_ERR_ARGUMENT, "New: One output expected.");
  std::lock_guard<std::mutex> lk(g_mu);
  VR_GUARD_BEGIN
  int dev = 0;
  VR_HIP(hipGetDevice(&dev));
  vr_context *h = new vr_context();
  h->device = dev;
  g_contexts.insert(h);
  *out = h;
  g_last_error.clear();
  return VR_OK;
  VR_GUARD_END
}

int vr_new_multi(const int32_t *devices, int32_t n, vr_context **out) {
  if (!out) return fail(VR_ERR_ARGUMENT, "New: One output expected.");
  if (!devices || n < 1) return fail(VR_ERR_ARGUMENT, "no devices");
  std::lock_guard<std::mutex> lk(g_mu);
  int count = 0;
  if (hipGetDeviceCount(&count) != hipSuccess) return fail(VR_ERR_DEVICE, "no HIP device");
  for (int i = 0; i < n; ++i)
    if (devices[i] < 0 || devices[i] >= count) return fail(VR_ERR_ARGUMENT, "invalid device index");
  VR_GUARD_BEGIN
  DeviceGuard dg(devices[0]);
  vr_context *h = new vr_context();
  h->device = devices[0];
  VR_HIP(hipEventCreateWithFlags(&h->gdone, hipEventDisableTiming));
  // VR_GROUP_PEER=0 (test switch): every child as if without a peer mapping (host-staged copies)
  const bool no_peer = env_flag_off("VR_GROUP_PEER");
  for (int i = 1; i < n; ++i) {
    const bool peer = enable_peer(devices[0], devices[i]) && enable_peer(devices[i], devices[0]) && !no_peer;
    DeviceGuard dk(devices[i]);
    vr_context *c = new vr_context();
    c->device = devices[i];
    c->peer = peer;
    c->parent = h;
    h->children.push_back(c);
    VR_HIP(take_stream(c->device, &c->gstream));
    VR_HIP(hipEventCreateWithFlags(&c->gdone, hipEventDisableTiming));
  }
  g_contexts.insert(h);
  *out = h;
  g_last_error.clear();
  return VR_OK;
  VR_GUARD_END
}

int vr_delete(vr_context *h) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  VR_GUARD_BEGIN
  // ~MManager -> cudaDeviceReset(): every handle's device memory and the module globals go.
  reset_tex_unit();
  for (vr_context *c : g_contexts) {
    for (vr_context *k : c->children)  // a group's children: their buffers go with the device reset
      for (auto &b : k->buf) b.reset();
    for (auto &b : c->buf) b.reset();
    if (c->d_out) (void)hipFree(c->d_out);
    c->d_out = nullptr;
    c->d_out_bytes = 0;
    free_schedules(c);
    free_views(c);
  }
  delete_children(h);
  if (h->gdone) (void)hipEventDestroy(h->gdone);
  for (hipEvent_t e : h->tev)
    if (e) (void)hipEventDestroy(e);
  if (h->d_part) (void)hipFree(h->d_part);
  g_contexts.erase(h);
  h->signature = 0;
  delete h;
  // cudaDeviceReset waits for and drops everything: so do the retired buffers here
  (void)hipDeviceSynchronize();
  vr_host::prune_retired(true);
  vr_host::pool_clear();
  return VR_OK;
  VR_GUARD_END
}

int vr_mem_info(vr_context *h, char *buf, size_t buflen) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  size_t free_b = 0, total_b = 0;
  VR_HIP(hipMemGetInfo(&free_b, &total_b));
  const VolRec &em = h->vol[T_EM], &ab = h->vol[T_AB], &re = h->vol[T_RE];
  auto ptr = [&](int s) { return (const void *)(h->buf[s] ? h->buf[s]->ptr : nullptr); };
  std::ostringstream os;
  os << "Memory Information\n"
     << "------------------------------" << "last sync (timestamp): " << h->time_last_mem_sync << "\n\n"
     << "\tGPU\n\t---\n"
     << "\t\tTotal Memory (MB): \t" << mb(total_b) << "\n"
     << "\t\tFree Memory (MB): \t" << mb(free_b) << "\n"
     << "\t\tUsed Memory (MB): \t" << mb(total_b - free_b) << "\n\n"
     << "\t\tVolumes\n\t\t-------\n"
     << "\t\tEmission (MB): " << mb(em.memory_size) << " ptr: " << ptr(T_EM) << "\n"
     << "\t\tAbsorption (MB): " << mb(ab.memory_size) << " ptr: " << ptr(T_AB) << "\n"
     << "\t\tReflection (MB): " << mb(re.memory_size) << " ptr: " << ptr(T_RE) << "\n"
     << "\t\tdX (MB): " << mb(h->vol[T_DX].memory_size) << " ptr: " << ptr(T_DX) << "\n"
     << "\t\tdY (MB): " << mb(h->vol[T_DY].memory_size) << " ptr: " << ptr(T_DY) << "\n"
     << "\t\tdZ (MB): " << mb(h->vol[T_DZ].memory_size) << " ptr: " << ptr(T_DZ) << "\n"
     << "\t\tlight (MB): " << mb(h->vol[T_LIGHT].memory_size) << " ptr: " << ptr(T_LIGHT) << "\n"
     << "\t\treusable buffers (MB): " << mb(vr_host::pool_bytes(h->device)) << "\n\n"
     << "\t\tSimilarity of Volumes\n\t\t---------------------\n"
     << "\t\t\tEm\tAb\tRe\n"
     << "\t\tEm\t1\t\n"
     << "\t\tAb\t" << same(em, ab) << "\t1\n"
     << "\t\tRe\t" << same(em, re) << "\t" << same(ab, re) << "\t1\n\n"
     << "\t\tSlots (emission/absorption/reflection): " << g_tex.idx_em << " " << g_tex.idx_ab << " "
     << g_tex.idx_re << ", gradient method: " << (g_tex.grad_method == G_LOOKUP ? "lookup" : "compute")
     << ", lights: " << g_tex.lights.size() << "\n";
  // per-device residency and the last launch's kernel time (SURVEY.md s5 "Metrics"): the primary
  // and, for a group (vr_new_multi), every child with the replicas of the bound volumes it holds
  os << "\n\tDevices\n\t-------\n";
  static const char *const tex_names[T_COUNT] = {"Emission", "Absorption", "Reflection", "dX", "dY", "dZ", "light"};
  std::vector<vr_context *> ctxs{h};
  ctxs.insert(ctxs.end(), h->children.begin(), h->children.end());
  for (size_t k = 0; k < ctxs.size(); ++k) {
    vr_context *c = ctxs[k];
    DeviceGuard dk(c->device);
    size_t fb = 0, tb = 0;
    VR_HIP(hipMemGetInfo(&fb, &tb));
    os << "\t\tdevice " << c->device << (k == 0 ? " (primary)" : " (group member)") << ": used (MB) "
       << mb(tb - fb) << " of " << mb(tb) << ", part buffer (MB) " << mb(c->d_part_bytes)
       << ", reusable buffers (MB) " << mb(vr_host::pool_bytes(c->device)) << "\n";
    for (int t = 0; t < T_COUNT; ++t) {
      const BufPtr &b = g_tex.bind[t];
      if (!b) continue;
      const DevBuf *r = nullptr;
      if (k == 0) {
        r = b.get();
      } else if (t == T_LIGHT) {
        r = c->buf[T_LIGHT].get();
      } else {
        auto it = b->replicas.find(c->device);
        if (b->device == c->device && it == b->replicas.end()) r = b.get();
        else if (it != b->replicas.end() && b->replica_of[c->device] == b->version) r = it->second.get();
      }
      os << "\t\t\t" << tex_names[t] << ": ";
      if (r) os << mb(r->bytes) << " MB resident at " << (const void *)r->ptr << (k && t != T_LIGHT ? " (replica)" : "") << "\n";
      else os << "not resident (replicated at the next render)\n";
    }
    float ms = -1.f;
    bool have = c->timed && vr_host::query_done(c->tev[1], "hipEventQuery (mem_info launch timing)");
    if (have) {
      const hipError_t e = hipEventElapsedTime(&ms, c->tev[0], c->tev[1]);
      if (e != hipSuccess) vr_host::consume(e, "hipEventElapsedTime (mem_info launch timing)");
      have = e == hipSuccess;
    }
    if (have)
      os << "\t\t\tlast launch (ms): " << ms << "\n";
    else
      os << "\t\t\tlast launch (ms): n/a\n";
  }
  const std::string s = os.str();
  if (buf && buflen) {
    const size_t n = std::min(buflen - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return VR_OK;
  VR_GUARD_END
}

static int do_sync_volumes(vr_context *h, uint64_t time_last_mem_sync, const vr_volume *emission,
                    const vr_volume *reflection, const vr_volume *absorption, const vr_volume *dx,
                    const vr_volume *dy, const vr_volume *dz) {
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!emission || !reflection || !absorption) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  // render.cpp:105-113 keys on the argument count: 9 takes the gradient volumes (lookup), 6 resets
  // them, 7 or 8 (dx or dx, dy given, the rest NULL) keeps the handle's previous gradient volumes
  // without reading the given ones; setGradientMethod(compute) then MManager::sync re-enters lookup
  // mode if kept gradient volumes exist (mmanager.hxx:193-200).
  const int given = (dx != nullptr) + (dy != nullptr) + (dz != nullptr);
  const bool lookup = given == 3;
  if (!lookup && given && !(dx && (dy || !dz)))
    return fail(VR_ERR_ARGUMENT, "sync_volumes: gradient volumes must be given in order (dx, dy, dz)");
  for (const vr_volume *v : {emission, reflection, absorption, lookup ? dx : nullptr, lookup ? dy : nullptr,
                             lookup ? dz : nullptr}) {
    if (!v) continue;
    const uint64_t n = v->dims[0] * v->dims[1] * v->dims[2];
    if (n && !v->data) return fail(VR_ERR_ARGUMENT, "volume data is NULL");
    if (v->dims[0] > 0x7FFFFFFF || v->dims[1] > 0x7FFFFFFF || v->dims[2] > 0x7FFFFFFF)
      return fail(VR_ERR_UNSUPPORTED, "volume dimension too large");
  }
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  uint64_t required = required_memory(h);  // render.cpp:90 (before the new volumes are recorded)
  h->time_last_mem_sync = time_last_mem_sync;
  h->vol[T_EM] = make_rec(emission);
  h->vol[T_RE] = make_rec(reflection);
  h->vol[T_AB] = make_rec(absorption);
  if (lookup) {
    h->vol[T_DX] = make_rec(dx);
    h->vol[T_DY] = make_rec(dy);
    h->vol[T_DZ] = make_rec(dz);
  } else if (given == 0) {
    reset_gradients(h);
  }
  required += required_memory(h);
  int rc = check_free_device_memory(required);
  if (rc) return rc;
  g_tex.grad_method = lookup ? G_LOOKUP : G_COMPUTE;  // setGradientMethod (render.cpp:121)
  mm_sync(h);  // returns with the volumes resident (vr_host::Uploader); renders in flight keep running
  for (int t = 0; t < T_COUNT; ++t) h->snap_bind[t] = g_tex.bind[t];
  h->snap_idx[0] = g_tex.idx_em;
  h->snap_idx[1] = g_tex.idx_ab;
  h->snap_idx[2] = g_tex.idx_re;
  h->snap_grad = g_tex.grad_method;
  h->has_snap = true;
  return VR_OK;
  VR_GUARD_END
}

int vr_sync_volumes(vr_context *h, uint64_t time_last_mem_sync, const vr_volume *emission,
                    const vr_volume *reflection, const vr_volume *absorption, const vr_volume *dx,
                    const vr_volume *dy, const vr_volume *dz) {
  std::lock_guard<std::mutex> lk(g_mu);
  const int rc = do_sync_volumes(h, time_last_mem_sync, emission, reflection, absorption, dx, dy, dz);
  if (rc || h->children.empty()) return rc;
  VR_GUARD_BEGIN
  group_sync(h);
  return VR_OK;
  VR_GUARD_END
}

// Multi-channel render (vr_render_channels): channel i is what vr_sync_volumes +
// vr_render (or vr_render_stereo) on ch[i] would produce were it the only object -- before its
// sync the texture bindings its handle's last sync left are restored (the reference's textures are
// module globals: with one object per channel an unchanged channel would otherwise render the
// previous channel's volumes); the syncs run in channel order, each channel's frame is prepared
// against the textures its own sync bound, and the frames
// the staged march can take are marched together in one launch per (gradient mode, absorption
// aliasing, slot size, shading) group, their views' parameters in device memory.  The buffers a
// prepared frame reads stay referenced until the call returns; a later channel's sync never
// overwrites them (each handle owns its buffers).
// The fusable views one device collects for its march_views launches.
struct ViewSet {
  std::vector<BufPtr> keep;
  std::vector<vr::RenderParams> views;
  std::vector<std::array<double, 3>> drift;
  std::vector<int> vmode, vab;
  std::vector<vr::DevLight> lights;
  std::vector<size_t> loff;
};

// Launch the collected views of one device on `stream` (the device current): one march_views launch
// per (gradient mode, absorption aliasing, slot size, shading) group, in channel order within a group.
void launch_view_set(ViewSet &VS, int device, hipStream_t stream, vr_context *timer) {
  if (VS.views.empty()) return;
  std::vector<vr::RenderParams> &views = VS.views;
  const size_t nvw = views.size();
  std::vector<size_t> order(nvw);
  for (size_t k = 0; k < nvw; ++k) order[k] = k;
  auto key = [&](size_t k) {
    return ((VS.vmode[k] * 2 + VS.vab[k]) * 2 + views[k].wide_slot) * 2 + views[k].fast_shade;
  };
  std::stable_sort(order.begin(), order.end(), [&](size_t x, size_t y) { return key(x) < key(y); });
  // the views' lights, staged for these launches on their stream (each channel's own list)
  LaunchRec L;
  L.stream = stream;
  L.device = device;
  L.reads = std::move(VS.keep);
  for (const BufPtr &b : L.reads) wait_ready(b, stream);
  const void *dl = nullptr;
  VR_HIP(L.stage(VS.lights.data(), VS.lights.size() * sizeof(vr::DevLight), &dl));
  const vr::DevLight *d_lights = static_cast<const vr::DevLight *>(dl);
  typedef hipError_t (*views_fn)(const vr::RenderViews &, uint32_t, int, bool, hipStream_t);
  static const views_fn vfns[2][3] = {
      {vr::exact::launch_march_views_k1, vr::exact::launch_march_views_k2,
       VR_EXACT_K4(vr::exact::launch_march_views_k4, vr::exact::launch_march_views_k2)},
      {vr::fast::launch_march_views_k1, vr::fast::launch_march_views_k2, vr::fast::launch_march_views_k4}};
  time_mark(timer, 0, stream);
  size_t g0 = 0;
  while (g0 < nvw) {
    size_t g1 = g0;
    while (g1 < nvw && key(order[g1]) == key(order[g0])) ++g1;
    // depth lanes as for one view: the frame's own tail sets them, and K = 2 stays ahead of K = 1
    // per sample even at many waves per slot
    const int K = exact_lanes(std::min(depth_lanes(views[order[g0]]), 4), views[order[g0]].fast_shade);
    vr::RenderViews V;
    std::memset(&V, 0, sizeof V);
    for (size_t k = g0; k < g1; ++k) {
      vr::RenderParams &P = V.p[k - g0];
      P = views[order[k]];
      for (int d = 0; d < 3; ++d) P.tap_off[d] += (float)(chunk_samples(K) * VS.drift[order[k]][d]);
      P.lights = d_lights ? d_lights + VS.loff[order[k]] : nullptr;
    }
    const size_t v0 = order[g0];
    VR_HIP(vfns[views[v0].fast_shade ? 1 : 0][K == 1 ? 0 : (K == 2 ? 1 : 2)](V, (uint32_t)(g1 - g0), VS.vmode[v0],
                                                                              VS.vab[v0] != 0, stream));
    g0 = g1;
  }
  time_mark(timer, 1, stream);
  // a prepared frame's buffer that no handle or binding holds any more is freed when these launches
  // complete (vr_host::free_when_done); the launches stay asynchronous
  VR_HIP(L.finish());
}

// Multi-channel render (vr_render_channels): channel i is what vr_sync_volumes +
// vr_render (or vr_render_stereo) on ch[i] would produce were it the only object -- before its
// sync the texture bindings its handle's last sync left are restored (the reference's textures are
// module globals: with one object per channel an unchanged channel would otherwise render the
// previous channel's volumes); the syncs run in channel order, each channel's frame is prepared
// against the textures its own sync bound, and the frames the staged march can take are marched
// together in one launch per (gradient mode, absorption aliasing, slot size, shading) group, their
// views' parameters in kernel arguments.  The buffers a prepared frame reads stay referenced until
// its launch completes; a later channel's sync never overwrites them (each handle owns its buffers).
// Group handles (vr_new_multi, all channels on the same devices): every device renders its column
// part of every view (the channel's bindings replicated to it, as group_render does), the parts are
// gathered to the primary of channel 0 over xGMI and assembled there, view by view.
static int do_render_channels(const vr_channel *ch, int32_t n, int32_t stereo, float base, float *d_out,
                              hipStream_t stream) {
  if (!ch || n < 1) return fail(VR_ERR_ARGUMENT, "no channels");
  const int nv = stereo ? 2 : 1;
  if (n * nv > VR_VIEWS_MAX) return fail(VR_ERR_ARGUMENT, "too many channels");
  for (int i = 0; i < n; ++i) {
    if (!valid(ch[i].handle)) return fail(VR_ERR_HANDLE, "Handle not valid.");
    if (!ch[i].args) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
    for (int j = 0; j < i; ++j)
      if (ch[j].handle == ch[i].handle) return fail(VR_ERR_ARGUMENT, "channels need distinct handles");
    if (ch[i].args->resolution[0] != ch[0].args->resolution[0] || ch[i].args->resolution[1] != ch[0].args->resolution[1])
      return fail(VR_ERR_ARGUMENT, "channels differ in image resolution");
    if (ch[i].handle->device != ch[0].handle->device) return fail(VR_ERR_ARGUMENT, "channels on different devices");
    if (ch[i].handle->children.size() != ch[0].handle->children.size())
      return fail(VR_ERR_ARGUMENT, "channels on different device groups");
    for (size_t k = 0; k < ch[i].handle->children.size(); ++k)
      if (ch[i].handle->children[k]->device != ch[0].handle->children[k]->device)
        return fail(VR_ERR_ARGUMENT, "channels on different device groups");
  }
  const size_t img = (size_t)ch[0].args->resolution[0] * (size_t)ch[0].args->resolution[1] * 3;
  if (img && !d_out) return fail(VR_ERR_ARGUMENT, "output is NULL");
  const bool fuse = !test_flag("VR_NO_FUSED_CHANNELS");
  vr_context *h0 = ch[0].handle;
  const int ndev = 1 + (int)h0->children.size();
  const int32_t bc = 16;
  const int64_t W = (int64_t)ch[0].args->resolution[1], H = (int64_t)ch[0].args->resolution[0];
  const int64_t maxc = part_columns(W, bc, 0, ndev);
  const size_t part_floats = (size_t)maxc * (size_t)H * 3;
  const bool grouped = ndev > 1 && part_floats > 0;
  const int nviews = n * nv;  // view vi = i * nv + e
  if (grouped) {
    ensure_part_buffers(h0, ndev, part_floats, nviews);
    VR_HIP(hipStreamWaitEvent(stream, h0->gdone, 0));  // the previous frame's assembly read part 0
  }
  // where view vi of device k goes: the caller's image (one device) or the part buffers
  auto out_of = [&](int k, int vi) -> float * {
    if (!grouped) return d_out + (size_t)vi * img;
    if (k == 0) return h0->d_part + ((size_t)vi * ndev) * part_floats;
    return h0->children[k - 1]->d_part + (size_t)vi * part_floats;
  };
  std::vector<ViewSet> sets(grouped ? ndev : 1);
  for (int i = 0; i < n; ++i) {
    vr_context *h = ch[i].handle;
    if (h->has_snap) {  // this channel's own bindings, not the previous channel's
      for (int t = 0; t < T_COUNT; ++t) g_tex.bind[t] = h->snap_bind[t].lock();
      g_tex.idx_em = h->snap_idx[0];
      g_tex.idx_ab = h->snap_idx[1];
      g_tex.idx_re = h->snap_idx[2];
      g_tex.grad_method = h->snap_grad;
    }
    int rc = do_sync_volumes(h, ch[i].time_last_mem_sync, ch[i].emission, ch[i].reflection, ch[i].absorption,
                             ch[i].dx, ch[i].dy, ch[i].dz);
    if (rc) return rc;
    if (grouped) group_sync(h);
    vr_render_args a = *ch[i].args;
    float eye2[3] = {0.f, 0.f, 0.f};
    if (stereo) {  // as vr_render_stereo: left = the frame's eye at -base, right at +base
      a.props[0] = -base;
      const float *r = a.rotation_flipped;
      const float X[3] = {r[2], r[1], r[0]}, Z[3] = {r[8], r[7], r[6]};
      for (int k = 0; k < 3; ++k) eye2[k] = fmaf(-a.props[2], Z[k], base * X[k]);
    }
    BufPtr saved[T_COUNT];
    for (int t = 0; t < T_COUNT; ++t) saved[t] = g_tex.bind[t];
    for (int k = 0; k < (grouped ? ndev : 1) && !rc; ++k) {
      vr_context *ctx = k == 0 ? h : h->children[k - 1];
      DeviceGuard dg(ctx->device);
      hipStream_t s = k == 0 ? stream : h0->children[k - 1]->gstream;
      if (k > 0) bind_replicas(h, ctx, saved);
      vr_partition pk{bc, k, ndev, 0};
      float *dl = out_of(k, i * nv), *dr = stereo ? out_of(k, i * nv + 1) : nullptr;
      Frame F;
      int fz = 0;
      rc = do_render(ctx, &a, grouped ? &pk : nullptr, dl, nullptr, s, F, dr, stereo ? eye2 : nullptr,
                     fuse ? &fz : nullptr);
      if (rc || !fz) continue;  // (rendered by its own launch against the textures bound now)
      ViewSet &VS = sets[k];
      for (const BufPtr &b : g_tex.bind)
        if (b) VS.keep.push_back(b);
      for (int v = 0; v < nv; ++v) {
        vr::RenderParams P = F.P;
        P.views = 1;
        P.out2 = nullptr;
        P.view_blocks = 0;
        P.out = v ? dr : dl;
        if (v)
          for (int d = 0; d < 3; ++d) P.eye[d] = eye2[d];
        VS.views.push_back(P);
        VS.drift.push_back({F.drift1[0], F.drift1[1], F.drift1[2]});
        VS.vmode.push_back(F.mode);
        VS.vab.push_back(F.ab_alias ? 1 : 0);
        VS.loff.push_back(VS.lights.size());
      }
      VS.lights.insert(VS.lights.end(), g_tex.lights.begin(), g_tex.lights.end());
    }
    for (int t = 0; t < T_COUNT; ++t) g_tex.bind[t] = saved[t];
    if (rc) return rc;
  }
  for (int k = 0; k < (int)sets.size(); ++k) {
    vr_context *ctx = k == 0 ? h0 : h0->children[k - 1];
    DeviceGuard dg(ctx->device);
    launch_view_set(sets[k], ctx->device, k == 0 ? stream : ctx->gstream, ctx);
  }
  if (grouped) {
    std::vector<float *> outs(nviews);
    for (int vi = 0; vi < nviews; ++vi) outs[vi] = d_out + (size_t)vi * img;
    group_gather_assemble(h0, nviews, part_floats, W, H, bc, maxc, outs.data(), stream);
  }
  return VR_OK;
}

int vr_render_channels_device(const vr_channel *ch, int32_t n, int32_t stereo, float base, float *d_out,
                              void *stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!ch || n < 1 || !valid(ch[0].handle)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  VR_GUARD_BEGIN
  DeviceGuard dg(ch[0].handle->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  return do_render_channels(ch, n, stereo, base, d_out, (hipStream_t)stream);
  VR_GUARD_END
}

int vr_render_channels(const vr_channel *ch, int32_t n, int32_t stereo, float base, float *out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!ch || n < 1 || !valid(ch[0].handle)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!ch[0].args) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  VR_GUARD_BEGIN
  vr_context *h = ch[0].handle;
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  const size_t img = (size_t)ch[0].args->resolution[0] * (size_t)ch[0].args->resolution[1] * 3;
  if (img && !out) return fail(VR_ERR_ARGUMENT, "output is NULL");
  const size_t bytes = img * sizeof(float) * (size_t)n * (stereo ? 2 : 1);
  if (bytes > h->d_chan_bytes) {
    if (h->d_chan) VR_HIP(hipFree(h->d_chan));
    h->d_chan = nullptr;
    h->d_chan_bytes = 0;
    VR_HIP(hipMalloc(&h->d_chan, bytes));
    h->d_chan_bytes = bytes;
  }
  int rc = do_render_channels(ch, n, stereo, base, h->d_chan, nullptr);
  if (rc) return rc;
  if (bytes) VR_HIP(hipMemcpy(out, h->d_chan, bytes, hipMemcpyDeviceToHost));
  return VR_OK;
  VR_GUARD_END
}

int vr_sum_channels_device(const float *d_in, int32_t n, int32_t views, uint64_t image_floats, float *d_out,
                           void *stream) {
  if (!d_in || !d_out || n < 1 || views < 1) return fail(VR_ERR_ARGUMENT, "invalid channel sum");
  VR_GUARD_BEGIN
  VR_HIP(vr::launch_sum_channels(d_in, (uint32_t)n, (uint32_t)views, image_floats, d_out, (hipStream_t)stream));
  return VR_OK;
  VR_GUARD_END
}

int vr_render(vr_context *h, const vr_render_args *a, float *out) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!a) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  const size_t bytes = (size_t)a->resolution[0] * (size_t)a->resolution[1] * 3 * sizeof(float);
  if (bytes && !out) return fail(VR_ERR_ARGUMENT, "output is NULL");
  if (bytes > h->d_out_bytes) {
    if (h->d_out) VR_HIP(hipFree(h->d_out));
    h->d_out = nullptr;
    h->d_out_bytes = 0;
    VR_HIP(hipMalloc(&h->d_out, bytes));
    h->d_out_bytes = bytes;
  }
  Frame F;
  int rc = h->children.empty() ? do_render(h, a, nullptr, h->d_out, nullptr, nullptr, F)
                               : group_render(h, a, h->d_out, nullptr);
  if (rc) return rc;
  if (bytes) VR_HIP(hipMemcpy(out, h->d_out, bytes, hipMemcpyDeviceToHost));
  return VR_OK;
  VR_GUARD_END
}

int vr_render_stereo(vr_context *h, const vr_render_args *a, float base, float *out_left, float *out_right) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!a) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  const size_t bytes = (size_t)a->resolution[0] * (size_t)a->resolution[1] * 3 * sizeof(float);
  if (bytes && (!out_left || !out_right)) return fail(VR_ERR_ARGUMENT, "output is NULL");
  if (2 * bytes > h->d_out_bytes) {
    if (h->d_out) VR_HIP(hipFree(h->d_out));
    h->d_out = nullptr;
    h->d_out_bytes = 0;
    VR_HIP(hipMalloc(&h->d_out, 2 * bytes));
    h->d_out_bytes = 2 * bytes;
  }
  // left eye: camera x offset -base (the frame's own eye); right eye: +base, formed as build_frame
  // forms it (fma(-dist, Z, xoff * X), render.cpp:211-221 column order)
  vr_render_args al = *a;
  al.props[0] = -base;
  const float *r = a->rotation_flipped;
  const float X[3] = {r[2], r[1], r[0]}, Z[3] = {r[8], r[7], r[6]};
  const float dist = a->props[2];
  float eye2[3];
  for (int i = 0; i < 3; ++i) eye2[i] = fmaf(-dist, Z[i], base * X[i]);
  Frame F;
  float *d_left = h->d_out, *d_right = h->d_out + bytes / sizeof(float);
  int rc = h->children.empty() ? do_render(h, &al, nullptr, d_left, nullptr, nullptr, F, d_right, eye2)
                               : group_render(h, &al, d_left, nullptr, d_right, eye2);  // every device
  if (rc) return rc;
  if (bytes) {
    VR_HIP(hipMemcpy(out_left, d_left, bytes, hipMemcpyDeviceToHost));
    VR_HIP(hipMemcpy(out_right, d_right, bytes, hipMemcpyDeviceToHost));
  }
  return VR_OK;
  VR_GUARD_END
}

int vr_render_stereo_device(vr_context *h, const vr_render_args *a, float base, float *d_left, float *d_right,
                            unsigned long long *d_steps, void *stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!a) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  if (!h->children.empty()) return fail(VR_ERR_UNSUPPORTED, "vr_render_stereo_device: one-device handles only");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();
  if ((size_t)a->resolution[0] * (size_t)a->resolution[1] && (!d_left || !d_right))
    return fail(VR_ERR_ARGUMENT, "output is NULL");
  vr_render_args al = *a;  // as vr_render_stereo: left = -base (the frame's eye), right = +base
  al.props[0] = -base;
  const float *r = a->rotation_flipped;
  const float X[3] = {r[2], r[1], r[0]}, Z[3] = {r[8], r[7], r[6]};
  float eye2[3];
  for (int i = 0; i < 3; ++i) eye2[i] = fmaf(-a->props[2], Z[i], base * X[i]);
  Frame F;
  return do_render(h, &al, nullptr, d_left, d_steps, (hipStream_t)stream, F, d_right, eye2);
  VR_GUARD_END
}

int vr_render_device(vr_context *h, const vr_render_args *a, const vr_partition *part, float *d_out,
                     unsigned long long *d_steps, void *stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!a) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  if (!h->children.empty() && !part && !d_steps) return group_render(h, a, d_out, (hipStream_t)stream);
  Frame F;
  return do_render(h, a, part, d_out, d_steps, (hipStream_t)stream, F);
  VR_GUARD_END
}

int64_t vr_partition_columns(int64_t w, const vr_partition *p) {
  if (!p) return w < 0 ? 0 : w;
  if (p->num_parts < 1 || p->block_cols < 1 || p->part < 0 || p->part >= p->num_parts) return -1;
  return part_columns(w, p->block_cols, p->part, p->num_parts);
}

int vr_assemble_partitions(const float *d_parts, int64_t w, int64_t h, int32_t block_cols, int32_t num_parts,
                           int64_t max_cols, float *d_out, void *stream) {
  if (w < 0 || h < 0 || block_cols < 1 || num_parts < 1) return fail(VR_ERR_ARGUMENT, "invalid partition");
  VR_GUARD_BEGIN
  VR_HIP(vr::launch_assemble(d_parts, w, h, block_cols, num_parts, max_cols, d_out, (hipStream_t)stream));
  return VR_OK;
  VR_GUARD_END
}

int vr_render_slab(vr_context *h, const vr_render_args *a, const vr_slab *slab, const vr_partition *part,
                   const float *d_state_in, float *d_state_out, void *stream) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!valid(h)) return fail(VR_ERR_HANDLE, "Handle not valid.");
  if (!a) return fail(VR_ERR_ARGUMENT, "insufficient parameter!");
  VR_GUARD_BEGIN
  DeviceGuard dg(h->device);
  vr_host::prune_retired();  // buffers whose last launch has completed
  Frame F;
  return do_render_slab(h, a, slab, part, d_state_in, d_state_out, (hipStream_t)stream, F);
  VR_GUARD_END
}

int vr_slab_planes(const uint64_t dims[3], const float element_size_um[3], double z0, double z1, uint64_t *first,
                   uint64_t *count) {
  if (!dims || !element_size_um || !first || !count || dims[0] == 0 || dims[2] == 0)
    return fail(VR_ERR_ARGUMENT, "invalid slab geometry");
  // gradient tap offset along z in texels (volumeRender.cpp:273-275 through initRender's box):
  // gstep_z * bscale_z * D = vw * es_x / (2 * es_z * D), es reversed as render.cpp:195 does
  const double esx = element_size_um[2], esz = element_size_um[0];
  const double D = (double)dims[2];
  const double off = (double)dims[0] * esx / (2.0 * esz * D) + 0.5;
  const double lo = std::isfinite(z0) ? std::floor(z0 - 0.5 - off) - 1.0 : 0.0;
  const double hi = std::isfinite(z1) ? std::floor(z1 - 0.5 + off) + 3.0 : D;
  const double a = std::min(std::max(lo, 0.0), D), b = std::min(std::max(hi, 0.0), D);
  *first = (uint64_t)a;
  *count = b > a ? (uint64_t)(b - a) : 0;
  return VR_OK;
}

int vr_depth_lanes(int64_t part_cols, int64_t height) {
  vr::RenderParams P;
  std::memset(&P, 0, sizeof(P));
  P.part_cols = (int32_t)std::min<int64_t>(part_cols, 0x7fffffff);
  P.height = (int32_t)std::min<int64_t>(height, 0x7fffffff);
  return depth_lanes(P);
}

int vr_depth_lanes_tau(int64_t part_cols, int64_t height, double texels_per_pixel) {
  vr::RenderParams P;
  std::memset(&P, 0, sizeof(P));
  P.part_cols = (int32_t)std::min<int64_t>(part_cols, 0x7fffffff);
  P.height = (int32_t)std::min<int64_t>(height, 0x7fffffff);
  P.tau = (float)texels_per_pixel;
  return depth_lanes(P);
}

int vr_synth_shell_device(float *d_out, uint64_t n, void *stream) {
  VR_GUARD_BEGIN
  VR_HIP(vr::launch_synth_shell(d_out, n, 0, n, (hipStream_t)stream));
  return VR_OK;
  VR_GUARD_END
}

int vr_synth_shell_planes_device(float *d_out, uint64_t n, uint64_t z_first, uint64_t count, void *stream) {
  if (z_first + count > n) return fail(VR_ERR_ARGUMENT, "planes outside the volume");
  VR_GUARD_BEGIN
  VR_HIP(vr::launch_synth_shell(d_out, n, z_first, count, (hipStream_t)stream));
  return VR_OK;
  VR_GUARD_END
}

int vr_gradient_device(const float *d_data, const uint64_t dims[3], float *d_gx, float *d_gy, float *d_gz,
                       void *stream) {
  if (!dims) return fail(VR_ERR_ARGUMENT, "dims is NULL");
  if (dims[0] > 0xFFFFFFFFull || dims[1] > 0xFFFFFFFFull || dims[2] > 0xFFFFFFFFull)
    return fail(VR_ERR_UNSUPPORTED, "dimension above 2^32");
  if (dims[0] * dims[1] * dims[2] && (!d_data || !d_gx || !d_gy || !d_gz)) return fail(VR_ERR_ARGUMENT, "NULL buffer");
  VR_GUARD_BEGIN
  VR_HIP(vr::launch_gradient(d_data, dims, d_gx, d_gy, d_gz, (hipStream_t)stream));
  return VR_OK;
  VR_GUARD_END
}

int vr_debug_slot_transition(const int32_t idx_in[3], int32_t sim_em_ab, int32_t sim_em_re, int32_t sim_ab_re,
                             int32_t req_em, int32_t req_ab, int32_t req_re, int32_t idx_out[3],
                             int32_t unbound_out[3]) {
  DebugState s;
  s.idx_em = idx_in[0];
  s.idx_ab = idx_in[1];
  s.idx_re = idx_in[2];
  sync_decisions(s, sim_em_ab, sim_em_re, sim_ab_re, req_em, req_ab, req_re);
  idx_out[0] = s.idx_em;
  idx_out[1] = s.idx_ab;
  idx_out[2] = s.idx_re;
  for (int i = 0; i < 3; ++i) unbound_out[i] = !s.bound[i];
  return VR_OK;
}

#define HG_PI ((float)3.141592653589793238462643383279502884197169399375105820)

// HenyeyGreenstein on the device: the generator's expression per element on
// the GPU, with the sines / cosines of k*pi/N computed here exactly as the host generator does.
int vr_henyey_greenstein_device(uint32_t n, float g, float *d_out, void *stream) {
  if (g > 1 || g < -1) return fail(VR_ERR_ARGUMENT, "g must be in interval [-1,1]");
  if (n && !d_out) return fail(VR_ERR_ARGUMENT, "output is NULL");
  if (!n) return VR_OK;
  VR_GUARD_BEGIN
  const float frac_half = HG_PI / n;
  std::vector<float> tab(2 * (size_t)n);
  for (uint32_t k = 0; k < n; ++k) {
    const float ang = k * frac_half;
    tab[k] = sinf(ang);
    tab[n + k] = cosf(ang);
  }
  hipStream_t s = (hipStream_t)stream;
  float *d_tab = nullptr;
  VR_HIP(hipMallocAsync(reinterpret_cast<void **>(&d_tab), tab.size() * sizeof(float), s));
  VR_HIP(hipMemcpyAsync(d_tab, tab.data(), tab.size() * sizeof(float), hipMemcpyHostToDevice, s));
  VR_HIP(vr::launch_hg_lut(n, d_tab, d_tab + n, g, powf(g, 2.f), 1.f - powf(g, 2.f), d_out, s));
  VR_HIP(hipFreeAsync(d_tab, s));
  VR_HIP(hipStreamSynchronize(s));  // the host table is borrowed by the copy
  return VR_OK;
  VR_GUARD_END
}

// Volume.normalize(newMin, newMax) on the device (Volume.m:208-220), d_out may equal d_in.
int vr_normalize_device(const float *d_in, uint64_t n, double new_min, double new_max, float *d_out, void *stream) {
  if (n && (!d_in || !d_out)) return fail(VR_ERR_ARGUMENT, "NULL buffer");
  if (!n) return VR_OK;
  VR_GUARD_BEGIN
  hipStream_t s = (hipStream_t)stream;
  uint32_t *mm = nullptr;
  VR_HIP(hipMallocAsync(reinterpret_cast<void **>(&mm), 2 * sizeof(uint32_t), s));
  // MATLAB: (newMax - newMin) in double, then single with the single data; newMin single likewise
  VR_HIP(vr::launch_normalize(d_in, n, mm, (float)(new_max - new_min), (float)new_min, d_out, s));
  VR_HIP(hipFreeAsync(mm, s));
  return VR_OK;
  VR_GUARD_END
}

// Volume.resize(newsize) on the device (Volume.m:93-106 -> imresize3 / imresize): separable cubic
// passes with antialiasing when shrinking, the axes in order of increasing scale (stable), an axis
// whose length does not change skipped (its contributions are the identity).
int vr_resize_device(const float *d_in, const uint64_t in_dims[3], const uint64_t out_dims[3], float *d_out,
                     void *stream) {
  if (!in_dims || !out_dims) return fail(VR_ERR_ARGUMENT, "dims is NULL");
  uint64_t nin = 1, nout = 1;
  for (int i = 0; i < 3; ++i) {
    if (in_dims[i] > 0x7FFFFFFFull || out_dims[i] > 0x7FFFFFFFull) return fail(VR_ERR_UNSUPPORTED, "dimension too large");
    nin *= in_dims[i];
    nout *= out_dims[i];
  }
  if (!nout) return VR_OK;
  if (!nin) return fail(VR_ERR_ARGUMENT, "cannot resize an empty volume");
  if (!d_in || !d_out) return fail(VR_ERR_ARGUMENT, "NULL buffer");
  VR_GUARD_BEGIN
  hipStream_t s = (hipStream_t)stream;
  int order[3] = {0, 1, 2};
  double sc[3];
  for (int i = 0; i < 3; ++i) sc[i] = (double)out_dims[i] / (double)in_dims[i];
  std::stable_sort(order, order + 3, [&](int a, int b) { return sc[a] < sc[b]; });
  std::vector<int> passes;
  for (int k = 0; k < 3; ++k)
    if (out_dims[order[k]] != in_dims[order[k]]) passes.push_back(order[k]);
  if (passes.empty()) {
    VR_HIP(hipMemcpyAsync(d_out, d_in, nin * sizeof(float), hipMemcpyDeviceToDevice, s));
    return VR_OK;
  }
  uint64_t cur[3] = {in_dims[0], in_dims[1], in_dims[2]};
  const float *src = d_in;
  // the device temporaries and the host contributions their copies read: all kept until the stream
  // has drained (the final synchronize, or the guard's on an error part-way)
  struct Temps {
    hipStream_t s;
    std::vector<void *> dev;
    std::vector<std::vector<double>> w;
    std::vector<std::vector<int32_t>> idx;
    ~Temps() {  // stream-ordered frees after the passes, then the host data is released
      hipError_t e = hipSuccess;
      for (void *t : dev) {
        const hipError_t r = hipFreeAsync(t, s);
        if (e == hipSuccess) e = r;
      }
      const hipError_t r = hipStreamSynchronize(s);
      if (e == hipSuccess) e = r;
      // (a destructor: not thrown -- a device fault stays pending for the next entry's check)
      if (e != hipSuccess && !vr_host::device_fault(e)) {
        (void)hipGetLastError();
        vr_host::log_error(e, "handled", "vr_resize_device temporaries", true);
      }
    }
  } temps{s, {}, {}, {}};
  temps.w.reserve(passes.size());
  temps.idx.reserve(passes.size());
  for (size_t k = 0; k < passes.size(); ++k) {
    const int dim = passes[k];
    temps.w.emplace_back();
    temps.idx.emplace_back();
    std::vector<double> &w = temps.w.back();
    std::vector<int32_t> &idx = temps.idx.back();
    int32_t P = 0;
    resize_contributions(cur[dim], out_dims[dim], w, idx, P);
    double *d_w = nullptr;
    int32_t *d_idx = nullptr;
    VR_HIP(hipMallocAsync(reinterpret_cast<void **>(&d_w), w.size() * sizeof(double), s));
    temps.dev.push_back(d_w);
    VR_HIP(hipMallocAsync(reinterpret_cast<void **>(&d_idx), idx.size() * sizeof(int32_t), s));
    temps.dev.push_back(d_idx);
    VR_HIP(hipMemcpyAsync(d_w, w.data(), w.size() * sizeof(double), hipMemcpyHostToDevice, s));
    VR_HIP(hipMemcpyAsync(d_idx, idx.data(), idx.size() * sizeof(int32_t), hipMemcpyHostToDevice, s));
    uint64_t nxt[3] = {cur[0], cur[1], cur[2]};
    nxt[dim] = out_dims[dim];
    float *dst = d_out;
    if (k + 1 < passes.size()) {
      VR_HIP(hipMallocAsync(reinterpret_cast<void **>(&dst), nxt[0] * nxt[1] * nxt[2] * sizeof(float), s));
      temps.dev.push_back(dst);
    }
    VR_HIP(vr::launch_resize_dim(src, cur, dim, out_dims[dim], d_w, d_idx, P, dst, s));
    src = dst;
    for (int i = 0; i < 3; ++i) cur[i] = nxt[i];
  }
  return VR_OK;  // ~Temps: free, then synchronize
  VR_GUARD_END
}

// The contributions of one resize axis, for tests: writes P (taps kept) and, if w / idx are not
// NULL, out_len * P weights and 0-based indices.
int vr_resize_contributions(uint64_t in_len, uint64_t out_len, int32_t *P, double *w, int32_t *idx) {
  if (!P || !in_len || !out_len) return fail(VR_ERR_ARGUMENT, "invalid resize axis");
  std::vector<double> ww;
  std::vector<int32_t> ii;
  resize_contributions(in_len, out_len, ww, ii, *P);
  if (w) std::memcpy(w, ww.data(), ww.size() * sizeof(double));
  if (idx) std::memcpy(idx, ii.data(), ii.size() * sizeof(int32_t));
  return VR_OK;
}

// HenyeyGreenstein.cc:39-91 (g in [-1, 1], value at c*N*N + a*N + b)
int vr_henyey_greenstein(uint32_t n, float g, float *out) {
  if (g > 1 || g < -1) return fail(VR_ERR_ARGUMENT, "g must be in interval [-1,1]");
  if (n && !out) return fail(VR_ERR_ARGUMENT, "output is NULL");
  const float frac_half = HG_PI / n;
  const size_t page = (size_t)n * n;
  const float num = 1.f - powf(g, 2.f);
  const float g2 = powf(g, 2.f);
  for (uint32_t c = 0; c < n; ++c) {
    const float gamma = c * frac_half;
    const float s = sinf(gamma), co = cosf(gamma);
    for (uint32_t a = 0; a < n; ++a) {
      const float alpha = a * frac_half;
      const float lx = sinf(alpha), lz = cosf(alpha);
      // lightOut (sin a, 0, cos a) rotated about X by gamma (float3.h:77-106)
      const float rx = 1.f * lx + 0.f * 0.f + 0.f * lz;
      const float ry = 0.f * lx + co * 0.f + s * lz;
      const float rz = 0.f * lx + -s * 0.f + co * lz;
      for (uint32_t b = 0; b < n; ++b) {
        const float beta = b * frac_half;
        const float ix = sinf(beta), iz = cosf(beta);
        const float cosTheta = rx * ix + ry * 0.f + rz * iz;
        const float den = sqrtf(powf((1.f + g2 - (2.f * g * cosTheta)), 3.f));
        out[(size_t)c * page + (size_t)a * n + b] = 1.f / (4.f * HG_PI) * (num / den);
      }
    }
  }
  return VR_OK;
}

uint64_t vr_timestamp(void) {
  const auto ms = std::chrono::duration_cast<std::chrono::milliseconds>(
                      std::chrono::system_clock::now().time_since_epoch())
                      .count();
  return (uint64_t)(uint32_t)(uint64_t)ms;  // stored through an int* (timestamp.cpp:25,33)
}

const char *vr_last_error(void) { return g_last_error.c_str(); }

int64_t vr_hip_errors(char *buf, size_t buflen) {
  vr_host::ErrLog &L = vr_host::errlog();
  std::lock_guard<std::mutex> g(L.mu);
  if (buf && buflen) {
    std::string s;
    for (const std::string &l : L.lines) s += l + "\n";
    const size_t n = std::min(buflen - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return (int64_t)L.count;
}

int vr_set_option(const char *name, int64_t value) {
  if (name && std::strcmp(name, "test_switches") == 0) {
    g_test_switches.store(value ? 1 : 0);
    return VR_OK;
  }
  return fail(VR_ERR_ARGUMENT, std::string("unknown option ") + (name ? name : "(null)"));
}

int vr_last_march_kernel(char *buf, size_t buflen) {
  std::lock_guard<std::mutex> lk(g_mu);
  const std::string &s = vr::last_march_kernel();
  if (buf && buflen) {
    const size_t n = std::min(buflen - 1, s.size());
    std::memcpy(buf, s.data(), n);
    buf[n] = 0;
  }
  return VR_OK;
}

const char *vr_version(void) { return "libvrhip 0.1 gfx950 (MI355X) volume ray-marcher"; }

}  // extern "C"
