// vr_resources.h -- device-resource lifetime of libvrhip's host driver (included by vr_capi.hip only).
//
// The reference serialises everything on CUDA's legacy default stream: an upload or a texture
// rebind can never overlap a render (volumeRender_kernel.cu:551-722 bind/copy synchronously, the
// mex call returns after cudaDeviceSynchronize).  Here renders may be in flight on caller streams
// (vr_render_device, vr_render_channels_device, vr_render_slab) while the host syncs the next frame's
// volumes, so every launch records an event, and what a launch reads is kept until that event:
//   - Event / record_event: a shared completion marker of one launch (or of an upload);
//   - free_when_done: device memory released only after the last launch that read it (a buffer
//     dropped while in flight is parked in the retired list, pruned at every API entry);
//   - ConstRing: per-launch small constants (the light list) staged through a pinned host ring on
//     the launch's own stream -- never a global buffer rewritten under a running kernel;
//   - Uploader: the upload path: persistent per-device copy and pad streams
//     and a device staging ring; a host volume crosses PCIe in plane chunks, each padded into the
//     apron layout (and its statistics taken) on the device while the next chunks copy.
#pragma once

#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "vr_device.h"

namespace vr {
hipError_t launch_pad_planes(const float *src, int64_t z0, int32_t nx, int32_t ny, int32_t nz, float *dst, int64_t k0,
                             int64_t k1, BufStats *st, hipStream_t s);
}

namespace vr_host {

// ---- HIP errors: reported or logged, never dropped ------------------------------------------------
// The reference's release build ignores every CUDA error (common.h:43-47).  Here every error a HIP
// call of the library returns is either thrown to the API caller (HipError -> VR_ERR_DEVICE with
// the call's text) or, where the library has a fallback for it (an optional buffer, a launch
// schedule, a timing event, an already enabled peer mapping), consumed from the thread's HIP error
// state by consume() and appended to a process-wide log that vr_hip_errors() returns.  An error
// found pending at an API entry (raised outside the library, or an asynchronous device fault) is
// logged and printed; a device fault fails the call that finds it (check_pending).
struct HipError {
  hipError_t e;
  const char *what;
};

struct ErrLog {
  std::mutex mu;
  uint64_t count = 0;
  std::vector<std::string> lines;  // the last MAX entries
  static constexpr size_t MAX = 32;
};
inline ErrLog &errlog() {
  static ErrLog &l = *new ErrLog();  // never destroyed (see g_tex)
  return l;
}
inline void log_error(hipError_t e, const char *kind, const char *site, bool print) {
  char buf[320];
  std::snprintf(buf, sizeof buf, "%s: %s (%d) at %s", kind, hipGetErrorName(e), (int)e, site);
  ErrLog &L = errlog();
  std::lock_guard<std::mutex> g(L.mu);
  ++L.count;
  if (L.lines.size() == ErrLog::MAX) L.lines.erase(L.lines.begin());
  L.lines.emplace_back(buf);
  static const bool verbose = [] {
    const char *ev = std::getenv("VR_TRACE_STALE");
    return ev && ev[0] == '1';
  }();
  if (print || verbose) std::fprintf(stderr, "libvrhip: %s\n", buf);
}

// Errors after which the device (context) is unusable: a kernel fault, an illegal access.
inline bool device_fault(hipError_t e) {
  switch (e) {
    case hipErrorIllegalAddress:
    case hipErrorLaunchFailure:
    case hipErrorLaunchTimeOut:
    case hipErrorAssert:
    case hipErrorContextIsDestroyed:
    case hipErrorECCNotCorrectable:
      return true;
    default:
      return false;
  }
}

// After a call that returned rc != hipSuccess and whose failure the caller handles with a fallback:
// the thread's error state is consumed and logged.  A device fault is not a fallback case: thrown.
inline void consume(hipError_t rc, const char *site) {
  const hipError_t e = hipGetLastError();
  const hipError_t r = rc != hipSuccess ? rc : e;
  if (r == hipSuccess) return;
  if (device_fault(r) || device_fault(e)) throw HipError{device_fault(r) ? r : e, site};
  log_error(r, "handled", site, false);
  if (e != hipSuccess && e != r) log_error(e, "pending", site, true);
}

// hipEventQuery's hipErrorNotReady is a status, not a failure: consumed silently; any other error
// of the query is handled as consume() does.  Returns whether the event has completed.
inline bool query_done(hipEvent_t ev, const char *site) {
  const hipError_t rc = hipEventQuery(ev);
  if (rc == hipSuccess) return true;
  if (rc == hipErrorNotReady) {
    if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();  // a status, not an error
    return false;
  }
  consume(rc, site);
  return true;  // a failed query: nothing better to wait for
}

// At an API entry: an error left in this thread's HIP error state was not raised by the library's
// own calls (those are thrown or consumed where they happen) -- another library's, or an
// asynchronous device fault.  Logged and printed; a device fault fails this call.
inline void check_pending(const char *fn) {
  const hipError_t e = hipGetLastError();
  if (e == hipSuccess || e == hipErrorNotReady) return;
  log_error(e, "pending at entry", fn, true);
  if (device_fault(e)) throw HipError{e, fn};
}

struct Event {
  hipEvent_t e = nullptr;
  ~Event() {
    if (e) (void)hipEventDestroy(e);  // a pending event is released when it completes
  }
};
using EventPtr = std::shared_ptr<Event>;

inline hipError_t record_event(hipStream_t s, EventPtr &out) {
  auto ev = std::make_shared<Event>();
  hipError_t rc = hipEventCreateWithFlags(&ev->e, hipEventDisableTiming);
  if (rc == hipSuccess) rc = hipEventRecord(ev->e, s);
  if (rc == hipSuccess) out = ev;
  return rc;
}

// completed (or never recorded); a query error counts as completed -- nothing better to wait for.
// Never throws (destructors prune readers): a device fault stays in the thread's error state for the
// next API entry's check_pending, other query errors are consumed and logged.
inline bool done(const EventPtr &ev) {
  if (!ev || !ev->e) return true;
  const hipError_t rc = hipEventQuery(ev->e);
  if (rc == hipSuccess) return true;
  if (rc == hipErrorNotReady) {
    if (hipPeekAtLastError() == hipErrorNotReady) (void)hipGetLastError();  // a status, not an error
    return false;
  }
  if (!device_fault(rc)) {
    (void)hipGetLastError();
    log_error(rc, "handled", "hipEventQuery (buffer reader)", false);
  }
  return true;
}

inline void wait(const EventPtr &ev) {
  if (ev && ev->e) (void)hipEventSynchronize(ev->e);
}

// Every pending reader of one buffer (the completion events of the launches and peer copies that
// read it, on any streams).  A buffer is rewritten, pooled for reuse or freed only when all of them
// have completed: launches on different streams finish in any order, so the newest event alone
// says nothing about the older ones.
struct Readers {
  std::vector<EventPtr> evs;
  void prune() {
    size_t k = 0;
    for (size_t i = 0; i < evs.size(); ++i)
      if (!vr_host::done(evs[i])) evs[k++] = evs[i];
    evs.resize(k);
  }
  void add(const EventPtr &ev) {
    prune();
    if (ev && ev->e) evs.push_back(ev);
  }
  bool done() {
    prune();
    return evs.empty();
  }
  void wait() {
    for (const EventPtr &ev : evs) vr_host::wait(ev);
    evs.clear();
  }
  void clear() { evs.clear(); }
};
inline Readers readers_of(const EventPtr &ev) {
  Readers r;
  r.add(ev);
  return r;
}

struct Retired {
  void *ptr;
  int device;
  Readers ev;
  bool pinned;
};

inline std::vector<Retired> &retired() {
  static std::vector<Retired> &r = *new std::vector<Retired>();  // never destroyed (see g_tex)
  return r;
}

inline void release(void *ptr, int device, bool pinned) {
  int cur = 0;
  (void)hipGetDevice(&cur);
  if (cur != device) (void)hipSetDevice(device);
  if (pinned)
    (void)hipHostFree(ptr);
  else
    (void)hipFree(ptr);
  if (cur != device) (void)hipSetDevice(cur);
}

// free now if no launch still reads the allocation, else when all its readers complete
inline void free_when_done(void *ptr, int device, Readers ev, bool pinned = false) {
  if (!ptr) return;
  if (ev.done())
    release(ptr, device, pinned);
  else
    retired().push_back({ptr, device, std::move(ev), pinned});
}

// release what has completed; block = wait for everything first (before a retried allocation)
inline void prune_retired(bool block = false) {
  auto &r = retired();
  size_t k = 0;
  for (size_t i = 0; i < r.size(); ++i) {
    if (block) r[i].ev.wait();
    if (r[i].ev.done())
      release(r[i].ptr, r[i].device, r[i].pinned);
    else
      r[k++] = r[i];
  }
  r.resize(k);
}

// Released volume buffers are kept for reuse by size (hipFree waits for the whole device, so
// freeing the previous frame's buffer would stall the render in flight; a movie whose volume
// changes every frame ping-pongs between two buffers).  Bounded: POOL_MAX bytes per device, the
// oldest completed ones freed beyond that, everything on vr_delete or when an allocation fails.
struct Pooled {
  void *ptr;
  int device;
  size_t bytes;
  Readers ev;
};
constexpr size_t POOL_MIN = 1ull << 20, POOL_MAX = 64ull << 30;

inline std::vector<Pooled> &pool() {
  static std::vector<Pooled> &p = *new std::vector<Pooled>();  // never destroyed (see g_tex)
  return p;
}

inline size_t pool_bytes(int device) {
  size_t t = 0;
  for (const Pooled &q : pool())
    if (q.device == device) t += q.bytes;
  return t;
}

// release pooled buffers (all, or of one device: block = wait for their last launches first)
inline void pool_clear(int device = -1) {
  auto &p = pool();
  size_t k = 0;
  for (size_t i = 0; i < p.size(); ++i) {
    if (device < 0 || p[i].device == device) {
      p[i].ev.wait();
      release(p[i].ptr, p[i].device, false);
    } else {
      p[k++] = p[i];
    }
  }
  p.resize(k);
}

// hipMalloc that first reclaims pooled and retired buffers when the device is full
inline hipError_t device_alloc(void **p, size_t bytes) {
  hipError_t rc = hipMalloc(p, bytes);
  if (rc == hipErrorOutOfMemory || rc == hipErrorMemoryAllocation) {
    consume(rc, "hipMalloc (device full: pool and retired buffers reclaimed, retried)");
    int dev = 0;
    (void)hipGetDevice(&dev);
    pool_clear(dev);
    prune_retired(true);
    rc = hipMalloc(p, bytes);
  }
  return rc;
}

// a volume-sized allocation: a pooled buffer of exactly this size whose last launch completed, or
// a new one
inline hipError_t pooled_alloc(void **p, size_t bytes, int device) {
  auto &q = pool();
  for (size_t i = 0; i < q.size(); ++i) {
    if (q[i].device == device && q[i].bytes == bytes && q[i].ev.done()) {
      *p = q[i].ptr;
      q.erase(q.begin() + (ptrdiff_t)i);
      return hipSuccess;
    }
  }
  return device_alloc(p, bytes);
}

// give a volume buffer back: pooled (it stays allocated) unless small or the pool is full
inline void pooled_free(void *ptr, size_t bytes, int device, Readers ev) {
  if (!ptr) return;
  if (bytes < POOL_MIN || bytes > POOL_MAX) {
    free_when_done(ptr, device, std::move(ev));
    return;
  }
  auto &q = pool();
  q.push_back({ptr, device, bytes, std::move(ev)});
  size_t total = pool_bytes(device);
  for (size_t i = 0; i < q.size() && total > POOL_MAX;) {  // oldest completed first
    if (q[i].device == device && q[i].ptr != ptr && q[i].ev.done()) {
      total -= q[i].bytes;
      release(q[i].ptr, device, false);
      q.erase(q.begin() + (ptrdiff_t)i);
    } else {
      ++i;
    }
  }
}

// Per-launch constants through a pinned ring: slot i is rewritten only after the launch that last
// read it completed (its event), so any number of in-flight launches on any streams each see their
// own copy.  A payload larger than a slot gets a dedicated allocation freed after its launch.
struct ConstRing {
  static constexpr size_t SLOT = 4096;
  static constexpr unsigned N = 256;
  int device = -1;
  char *host = nullptr, *dev = nullptr;
  EventPtr ev[N];
  unsigned next = 0;

  hipError_t init(int d) {
    if (host && dev) return hipSuccess;
    device = d;
    hipError_t rc = hipHostMalloc(reinterpret_cast<void **>(&host), SLOT * N, hipHostMallocDefault);
    if (rc == hipSuccess) rc = device_alloc(reinterpret_cast<void **>(&dev), SLOT * N);
    if (rc != hipSuccess) {  // all or nothing: a later call retries (or keeps returning the error)
      if (host) (void)hipHostFree(host);
      host = nullptr;
      dev = nullptr;
    }
    return rc;
  }
};

inline std::map<int, ConstRing> &rings() {
  static std::map<int, ConstRing> &r = *new std::map<int, ConstRing>();  // never destroyed
  return r;
}

// What one launch reads: its buffers' owners are kept alive, and marked with the launch's event by
// finish(); the staged constants' ring slot is released by the same event.
template <class BufPtrT>
struct LaunchRec {
  hipStream_t stream = nullptr;
  int device = 0;
  std::vector<BufPtrT> reads;
  int slot = -1;
  void *big = nullptr;  // a dedicated constants allocation (payload > SLOT)

  // a device copy of `bytes` of host data, ordered on the launch stream
  hipError_t stage(const void *src, size_t bytes, const void **out) {
    *out = nullptr;
    if (!bytes) return hipSuccess;
    if (bytes > ConstRing::SLOT) {
      hipError_t rc = device_alloc(&big, bytes);
      if (rc == hipSuccess) rc = hipMemcpy(big, src, bytes, hipMemcpyHostToDevice);
      *out = big;
      return rc;
    }
    ConstRing &R = rings()[device];
    hipError_t rc = R.init(device);
    if (rc != hipSuccess) return rc;
    slot = (int)(R.next++ % ConstRing::N);
    wait(R.ev[slot]);  // the launch that used this slot N launches ago
    R.ev[slot].reset();
    std::memcpy(R.host + (size_t)slot * ConstRing::SLOT, src, bytes);
    rc = hipMemcpyAsync(R.dev + (size_t)slot * ConstRing::SLOT, R.host + (size_t)slot * ConstRing::SLOT, bytes,
                        hipMemcpyHostToDevice, stream);
    *out = R.dev + (size_t)slot * ConstRing::SLOT;
    return rc;
  }

  // after the launch(es): everything read is released by their completion
  hipError_t finish() {
    EventPtr ev;
    hipError_t rc = record_event(stream, ev);
    if (rc != hipSuccess) {  // cannot track: fall back to waiting here
      consume(rc, "record_event (launch completion; waited for instead)");
      rc = hipStreamSynchronize(stream);
    }
    for (auto &b : reads)
      if (b) b->readers.add(ev);
    if (slot >= 0) rings()[device].ev[slot] = ev;
    if (big) free_when_done(big, device, readers_of(ev));
    big = nullptr;
    return rc;
  }
};

// The upload path of one device (replaces the per-sync cudaMalloc3DArray +
// cudaMemcpy3D of volumeRender_kernel.cu:659-672).  Host volumes cross PCIe in plane chunks of up
// to CHUNK bytes on a copy stream into a ring of NS device staging slots; each chunk is padded into
// the destination (apron layout, vr_device.h, statistics folded in) on a separate, highest-priority
// pad stream as soon as it has landed, while the copy stream moves on to the next slot (it waits
// only for the pad of the chunk that last used that slot).  So when a render of the previous frame
// holds the CUs and the pads run slowly beside it, the PCIe copies still stream back to back.
// Device volumes are padded straight from the caller's buffer.  The call returns when the volume
// is resident (the caller's pointer is borrowed for the call only, render.cpp:307-342) -- renders
// already in flight on other streams keep running meanwhile.
// Pinned bounce ring for pageable host sources (the copy half of the upload path, SURVEY.md 8f row
// 3; VR_UPLOAD_BOUNCE).  A pageable hipMemcpyAsync is staged by the runtime through its own pinned
// buffers, one thread filling them; here the source crosses in PIECE-sized pieces through a ring of
// NB pinned buffers that a pool of host threads fills in parallel (worker w copies pieces w, w + T,
// ...), while the calling thread issues each filled piece's DMA in order on the copy stream.  A
// buffer is refilled only after the DMA of the piece it last held has completed (its event).
struct Bounce {
  static constexpr size_t PIECE = 16ull << 20;
  static constexpr int NB = 16;
  char *pinned = nullptr;
  hipEvent_t ev[NB] = {};

  hipError_t init() {
    if (pinned) return hipSuccess;
    hipError_t rc = hipHostMalloc(reinterpret_cast<void **>(&pinned), PIECE * NB, hipHostMallocDefault);
    for (int i = 0; i < NB && rc == hipSuccess; ++i) rc = hipEventCreateWithFlags(&ev[i], hipEventDisableTiming);
    if (rc != hipSuccess) {  // all or nothing
      consume(rc, "Bounce::init (pinned bounce ring; the runtime's pageable copy instead)");
      for (hipEvent_t &e : ev)
        if (e) (void)hipEventDestroy(e), e = nullptr;
      if (pinned) (void)hipHostFree(pinned);
      pinned = nullptr;
    }
    return rc;
  }

  static int threads() {
    const char *ev = std::getenv("VR_UPLOAD_THREADS");
    return std::max(1, std::min(ev ? std::atoi(ev) : 8, NB));
  }

  // dst (device) <- src (pageable host), `bytes`, ordered on `stream`.  Returns once every piece's
  // DMA is issued (the last ones may still be running).
  hipError_t copy(void *dst, const void *src, size_t bytes, hipStream_t stream) {
    const size_t np = (bytes + PIECE - 1) / PIECE;
    if (!np) return hipSuccess;
    const int T = (int)std::min<size_t>((size_t)threads(), np);
    std::unique_ptr<std::atomic<int>[]> ready(new std::atomic<int>[np]);
    for (size_t i = 0; i < np; ++i) ready[i].store(0, std::memory_order_relaxed);
    std::atomic<size_t> issued{0};
    std::atomic<bool> stop{false};
    auto fill = [&](int w) {
      for (size_t i = (size_t)w; i < np; i += (size_t)T) {
        const int b = (int)(i % NB);
        if (i >= (size_t)NB)  // the piece that last held buffer b has been issued ...
          while (issued.load(std::memory_order_acquire) <= i - NB) {
            if (stop.load(std::memory_order_relaxed)) return;
            std::this_thread::yield();
          }
        (void)hipEventSynchronize(ev[b]);  // ... and its DMA has completed
        const size_t off = i * PIECE;
        std::memcpy(pinned + (size_t)b * PIECE, static_cast<const char *>(src) + off, std::min(PIECE, bytes - off));
        ready[i].store(1, std::memory_order_release);
      }
    };
    std::vector<std::thread> pool;
    pool.reserve((size_t)T);
    for (int w = 0; w < T; ++w) pool.emplace_back(fill, w);
    hipError_t rc = hipSuccess;
    for (size_t i = 0; i < np; ++i) {
      while (!ready[i].load(std::memory_order_acquire)) std::this_thread::yield();
      const int b = (int)(i % NB);
      const size_t off = i * PIECE;
      rc = hipMemcpyAsync(static_cast<char *>(dst) + off, pinned + (size_t)b * PIECE, std::min(PIECE, bytes - off),
                          hipMemcpyHostToDevice, stream);
      if (rc == hipSuccess) rc = hipEventRecord(ev[b], stream);
      if (rc != hipSuccess) {
        stop.store(true);
        break;
      }
      issued.store(i + 1, std::memory_order_release);
    }
    for (std::thread &t : pool) t.join();
    return rc;
  }
};

struct Uploader {
  static constexpr size_t CHUNK = 1ull << 30, WHOLE = 8ull << 30;
  static constexpr int NS = 4;
  int device = -1;
  hipStream_t stream = nullptr;      // copies
  hipStream_t pad_stream = nullptr;  // pads + statistics
  hipEvent_t copied[NS] = {}, padded[NS] = {};
  float *staging = nullptr;  // nslots slots of slot_floats
  size_t slot_floats = 0, nslots = 0;
  vr::BufStats *d_stats = nullptr, *h_stats = nullptr;
  Bounce bounce;  // VR_UPLOAD_BOUNCE=1: host sources through the pinned ring

  static bool use_bounce() {
    const char *ev = std::getenv("VR_UPLOAD_BOUNCE");
    return ev && ev[0] == '1';
  }

  hipError_t init(int d) {
    if (stream) return hipSuccess;
    device = d;
    int lo = 0, hi = 0;
    hipError_t rc = hipDeviceGetStreamPriorityRange(&lo, &hi);
    if (rc == hipSuccess) rc = hipStreamCreateWithFlags(&stream, hipStreamNonBlocking);
    if (rc == hipSuccess) rc = hipStreamCreateWithPriority(&pad_stream, hipStreamNonBlocking, hi);
    for (int i = 0; i < NS && rc == hipSuccess; ++i) {
      rc = hipEventCreateWithFlags(&copied[i], hipEventDisableTiming);
      if (rc == hipSuccess) rc = hipEventCreateWithFlags(&padded[i], hipEventDisableTiming);
    }
    if (rc == hipSuccess) rc = device_alloc(reinterpret_cast<void **>(&d_stats), sizeof(vr::BufStats));
    if (rc == hipSuccess) rc = hipHostMalloc(reinterpret_cast<void **>(&h_stats), sizeof(vr::BufStats), hipHostMallocDefault);
    return rc;
  }

  hipError_t ensure_staging(size_t floats) {
    if (floats <= slot_floats) return hipSuccess;
    nslots = 0;
    if (staging) (void)hipFree(staging);  // both upload streams are idle between uploads
    staging = nullptr;
    slot_floats = 0;
    const size_t slots = floats * sizeof(float) >= WHOLE / 2 ? 1 : NS;  // whole-volume staging: one slot
    hipError_t rc = device_alloc(reinterpret_cast<void **>(&staging), slots * floats * sizeof(float));
    if (rc == hipSuccess) {
      slot_floats = floats;
      nslots = slots;
    }
    return rc;
  }

  // src (host or device, per `on_device`) -> dst (padded, (nx+2)(ny+2)(nz+2) floats); *st = stats
  static bool timing() {
    static const bool on = [] {
      const char *ev = vr::test_switches_on() ? std::getenv("VR_UPLOAD_TIMING") : nullptr;
      return ev && ev[0] == '1';
    }();
    return on;
  }
  static double now_ms() {
    return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
  }

  hipError_t upload(const float *src, bool on_device, int32_t nx, int32_t ny, int32_t nz, float *dst,
                    vr::BufStats *st) {
    const double t0 = now_ms();
    double t_copied = t0;
    hipError_t rc = hipMemsetAsync(d_stats, 0, sizeof(vr::BufStats), pad_stream);
    const uint64_t plane = (uint64_t)nx * (uint64_t)ny;
    if (rc == hipSuccess && on_device) {
      // device data is read after the work already queued on the null stream (which orders after
      // every blocking stream) -- as the previous null-stream upload was -- e.g. a torch tensor
      // just written on torch's default stream
      EventPtr ev;
      rc = record_event(nullptr, ev);
      if (rc == hipSuccess) rc = hipStreamWaitEvent(pad_stream, ev->e, 0);
      if (rc == hipSuccess) rc = vr::launch_pad_planes(src, 0, nx, ny, nz, dst, 0, (int64_t)nz + 2, d_stats, pad_stream);
    } else if (rc == hipSuccess) {
      // up to WHOLE bytes the volume crosses in one copy and is padded once it has landed: a pad
      // that runs beside a render in flight (the previous frame's) is slow, and between chunks it
      // would hold up the copies (measured: 1024^3 movie 98 ms per frame chunked vs 82 whole)
      const uint64_t bytes = plane * (uint64_t)nz * sizeof(float);
      uint64_t chunk = bytes <= WHOLE ? bytes : CHUNK;
      if (const char *ev = std::getenv("VR_UPLOAD_CHUNK_MB")) chunk = std::max<uint64_t>(1, std::strtoull(ev, nullptr, 10)) << 20;
      const uint64_t per = std::max<uint64_t>(1, chunk / (plane * sizeof(float)));
      const uint64_t chunk_planes = std::min<uint64_t>(per, (uint64_t)nz);
      rc = ensure_staging(chunk_planes * plane);
      for (uint64_t z0 = 0, c = 0; rc == hipSuccess && z0 < (uint64_t)nz; z0 += chunk_planes, ++c) {
        const uint64_t z1 = std::min<uint64_t>((uint64_t)nz, z0 + chunk_planes);
        const int k = (int)(c % nslots);
        float *slot = staging + (size_t)k * slot_floats;
        if (c >= nslots) rc = hipStreamWaitEvent(stream, padded[k], 0);  // the slot's previous chunk is padded
        if (rc == hipSuccess) {
          const size_t nbytes = (z1 - z0) * plane * sizeof(float);
          if (use_bounce() && bounce.init() == hipSuccess) rc = bounce.copy(slot, src + z0 * plane, nbytes, stream);
          else rc = hipMemcpyAsync(slot, src + z0 * plane, nbytes, hipMemcpyHostToDevice, stream);
        }
        if (rc == hipSuccess) rc = hipEventRecord(copied[k], stream);
        if (rc == hipSuccess) rc = hipStreamWaitEvent(pad_stream, copied[k], 0);
        // padded planes: source plane z sits at z + 1; the apron planes 0 and nz + 1 replicate the ends
        const int64_t k0 = z0 == 0 ? 0 : (int64_t)z0 + 1;
        const int64_t k1 = z1 == (uint64_t)nz ? (int64_t)nz + 2 : (int64_t)z1 + 1;
        if (rc == hipSuccess) rc = vr::launch_pad_planes(slot, (int64_t)z0, nx, ny, nz, dst, k0, k1, d_stats, pad_stream);
        if (rc == hipSuccess) rc = hipEventRecord(padded[k], pad_stream);
      }
    }
    if (rc == hipSuccess) rc = hipMemcpyAsync(h_stats, d_stats, sizeof(vr::BufStats), hipMemcpyDeviceToHost, pad_stream);
    if (rc == hipSuccess && timing()) {  // diagnostics: when the copies and the pads ended
      hipEvent_t ce = nullptr;
      if (hipEventCreate(&ce) == hipSuccess && hipEventRecord(ce, stream) == hipSuccess) {
        (void)hipEventSynchronize(ce);
        t_copied = now_ms();
      }
      if (ce) (void)hipEventDestroy(ce);
    }
    if (rc == hipSuccess) rc = hipStreamSynchronize(pad_stream);  // the last pad followed the last copy
    if (rc == hipSuccess) rc = hipStreamSynchronize(stream);
    if (rc == hipSuccess && timing())
      std::fprintf(stderr, "VR_UPLOAD_TIMING bytes %llu copies %.2f ms total %.2f ms\n",
                   (unsigned long long)(plane * (uint64_t)nz * sizeof(float)), t_copied - t0, now_ms() - t0);
    if (rc == hipSuccess) *st = *h_stats;
    return rc;
  }
};

inline std::map<int, Uploader> &uploaders() {
  static std::map<int, Uploader> &u = *new std::map<int, Uploader>();  // never destroyed
  return u;
}

}  // namespace vr_host
