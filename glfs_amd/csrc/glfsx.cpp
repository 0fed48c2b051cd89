// glfsx.cpp -- host runtime behind include/glfsx.h.
//
// C++ mirror of the reference's bigblob write-path interface (the reference is
// Go; with no Go toolchain in this image the host side above the C-ABI is C++,
// see DESIGN.md "Boundary").  All hashing/encryption runs in the gfx950
// kernels of post_kernels.hip; this file only stages bytes, sequences
// launches and keeps the reference's Writer bookkeeping (blob.go:71-206).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <atomic>
#include <condition_variable>
#include <mutex>
#include <cctype>
#include <cerrno>
#include <pthread.h>
#include <sched.h>
#include <sys/prctl.h>
#include <unistd.h>
#include <string>
#include <thread>
#include <vector>

#include "../../include/glfsx.h"
#include "kernels.h"

using namespace glfsx;

// A/B switch (tools/build_variant.sh): a launch of one one-shot post (of
// either size class) passes its descriptor by value (launch_one_v /
// launch_med_v) instead of through the pinned descriptor array.
#ifndef GLFSX_ONE_BYVAL
#define GLFSX_ONE_BYVAL 1
#endif

namespace {

thread_local std::string tls_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  tls_err = buf;
  return code;
}

#define HIP_TRY(expr)                                                     \
  do {                                                                    \
    hipError_t e_ = (expr);                                               \
    if (e_ != hipSuccess)                                                 \
      return fail(GLFSX_E_DEVICE, "%s: %s (%s:%d)", #expr,                \
                  hipGetErrorString(e_), __FILE__, __LINE__);             \
  } while (0)

// Grow-only device / pinned-host buffer.  `dirty`: how far from the start
// the bytes may be non-zero (index-node images, level_prepare); SIZE_MAX =
// unknown.
struct DevBuf {
  void *p = nullptr;
  size_t cap = 0;
  size_t dirty = SIZE_MAX;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    dirty = SIZE_MAX;
    size_t want = std::max<size_t>(n, 4096);
    HIP_TRY(hipMalloc(&p, want));
    cap = want;
    return 0;
  }
  uint8_t *u8() const { return static_cast<uint8_t *>(p); }
};
struct PinBuf {
  void *p = nullptr;
  void *dp = nullptr;  // the same memory as the kernels address it
  size_t cap = 0;
  int ensure(size_t n) {
    if (n <= cap) return 0;
    if (p) (void)hipHostFree(p);
    p = dp = nullptr;
    cap = 0;
    size_t want = std::max<size_t>(n, 4096);
    HIP_TRY(hipHostMalloc(&p, want, hipHostMallocPortable));
    cap = want;
    HIP_TRY(hipHostGetDevicePointer(&dp, p, 0));
    return 0;
  }
  uint8_t *u8() const { return static_cast<uint8_t *>(p); }
  uint8_t *dptr() const { return static_cast<uint8_t *>(dp); }
};

// Per-thread device context: the library is reentrant because every host
// thread gets its own stream and staging (bigblob.Writer is single-goroutine,
// glfs.Machine is used concurrently: SURVEY 8b "Threading").
struct Ctx {
  int dev = -1;
  hipStream_t stream = nullptr;
  DevBuf d_in, d_ct, d_refs, d_lvl_a, d_lvl_b, d_small, d_tree;
  PinBuf h_small, h_root;      // h_root: a root ref written by the kernels
  PinBuf h_oin, h_oct, h_oref;  // glfsx_post's one-shot staging
  PinBuf h_bin, h_bct, h_bref;  // glfsx_post_blobs' one-shot staging
  // glfsx_post_blobs' small blobs from host memory: groups of <= 64 MiB
  // through three pinned slots, upload / hash / download on three streams
  struct BlobSlot {
    PinBuf h_in, h_ct, h_meta, h_refs;  // h_meta: local offsets then lengths
    DevBuf d_in, d_ct, d_meta, d_refs;
    hipEvent_t done = nullptr, up = nullptr, hashed = nullptr;
    uint64_t i0 = 0, i1 = 0;            // the group's blob index range
    std::vector<uint64_t> loff;         // local offset of each blob in the range
    bool busy = false;
  } bslot[3];
  hipStream_t s_up = nullptr, s_down = nullptr;
  // glfsx_post_tree_device: a second stream for the tree blob's posts, its
  // events, and the tree layout on the host
  hipStream_t stream2 = nullptr;
  std::vector<hipEvent_t> events;
  PinBuf h_tree;
  ~Ctx() {
    // Process teardown may already have unloaded the HIP runtime; leak.
  }
};
// One context per device the thread has used (a thread may switch devices,
// e.g. one driving several GPUs; switching back finds its stream and
// buffers again instead of leaking them).  Contexts live as long as the
// thread (see ~Ctx).
thread_local std::vector<Ctx *> tls_ctxs;
thread_local int tls_dev = 0;

int ctx_get(Ctx **out) {
  if (tls_dev >= 0 && size_t(tls_dev) < tls_ctxs.size() && tls_ctxs[tls_dev]) {
    Ctx &c = *tls_ctxs[tls_dev];
    HIP_TRY(hipSetDevice(c.dev));
    *out = &c;
    return 0;
  }
  {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess || n == 0)
      return fail(GLFSX_E_DEVICE,
                  "no HIP device available (%s); the glfsx path has no CPU "
                  "fallback",
                  e != hipSuccess ? hipGetErrorString(e) : "count = 0");
    if (tls_dev >= n)
      return fail(GLFSX_E_DEVICE, "device %d out of range (%d devices)",
                  tls_dev, n);
    HIP_TRY(hipSetDevice(tls_dev));
    auto *c = new Ctx();  // lives as long as the thread's use of the device
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
      delete c;
      return fail(GLFSX_E_DEVICE, "hipStreamCreate on device %d failed", tls_dev);
    }
    c->dev = tls_dev;
    if (tls_ctxs.size() <= size_t(tls_dev)) tls_ctxs.resize(tls_dev + 1, nullptr);
    tls_ctxs[tls_dev] = c;
    *out = c;
    return 0;
  }
}

// Wait for a stream whose results the caller is about to return.  Polls
// for up to kSpinNs first: a blocking hipStreamSynchronize wakes the thread
// tens to hundreds of microseconds after the GPU finishes, which is most of
// the host overhead of a short call (a 1 GiB Create takes ~1.3 ms, config
// 4's one call ~5 ms: at a 2 ms bound it waited its last ~3 ms blocked and
// lost ~0.1 ms to the wake-up); longer waits block.  At most kMaxSpinners
// threads poll at once (glfs.Machine is used concurrently; N pollers would
// pin N host cores); the rest block at once, and a poller yields its core
// between queries.  GLFSX_SPIN_US overrides the poll bound (default 20 ms).
const int64_t kSpinNs = [] {
  const char *e = getenv("GLFSX_SPIN_US");
  return e ? int64_t(strtoll(e, nullptr, 10)) * 1000 : int64_t(20000000);
}();
constexpr int kMaxSpinners = 4;
std::atomic<int> g_spinners{0};
hipError_t stream_wait(hipStream_t s) {
  if (g_spinners.fetch_add(1, std::memory_order_relaxed) >= kMaxSpinners) {
    g_spinners.fetch_sub(1, std::memory_order_relaxed);
    return hipStreamSynchronize(s);
  }
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  for (;;) {
    e = hipStreamQuery(s);
    if (e != hipErrorNotReady) break;
    if (std::chrono::duration_cast<std::chrono::nanoseconds>(
            std::chrono::steady_clock::now() - t0).count() > kSpinNs) {
      e = hipStreamSynchronize(s);
      break;
    }
    sched_yield();
  }
  g_spinners.fetch_sub(1, std::memory_order_relaxed);
  return e;
}

// One-launch split posts (k_pass_dc) report a failed DEK wait through a
// word the host reads after the stream drains (fused_errors_take); the
// calls that sync check it and repeat the work with two launches per post.
// tls_fused = false while repeating; tls_fused_failed marks the failure.
thread_local bool tls_fused = true;
thread_local bool tls_fused_failed = false;

int fused_check(hipStream_t s) {
  if (const uint32_t v = fused_errors_take(s)) {
    tls_fused_failed = true;
    return fail(GLFSX_E_DEVICE,
                "one-launch split post on stream %p: %s; its results were discarded",
                static_cast<void *>(s),
                v == 1 ? "a DEK wait timed out" : "a workgroup found no work item");
  }
  return 0;
}

// Run f(); if it failed because a one-launch split post failed, run it again
// with two launches per post.
template <class F>
int with_fused_retry(F &&f) {
  tls_fused_failed = false;
  int rc = f();
  if (rc && tls_fused_failed) {
    tls_fused_failed = false;
    tls_fused = false;
    rc = f();
    tls_fused = true;
  }
  return rc;
}

hipStream_t pick_stream(Ctx *c, void *stream) {
  return stream ? static_cast<hipStream_t>(stream) : c->stream;
}

// ---- One-shot posts (launch_one) ----
// A post of one message of at most kMaxMedLen bytes from host memory: the
// bytes sit in pinned staging, the kernel reads them there and writes ctext
// and ref straight back into pinned staging, then sets the request's flag
// (pinned, OneDesc::flag) to the launch's sequence number, so a post is one
// launch and a wait on a host word -- no stream query.
// Concurrent callers (glfs.Machine is used from many goroutines) are
// coalesced, group-commit style: a caller that finds the leadership free
// and a free launch lane takes every pending request into one launch (one
// workgroup each) and hands the leadership on at once; every caller then
// waits for its own flag.  A lane is free again once its launch has
// completed (its descriptors and flags are read and written until then):
// up to kOneLanes launches are in flight, each carrying whatever queued
// while the earlier ones ran.
constexpr uint32_t kOneBatch = 1024;
constexpr int kOneLanes = 8;
struct OneLane;
struct OneReq {
  OneDesc d{};
  OneReq *next = nullptr;     // the pending stack
  std::atomic<int> armed{0};  // flag / seq / lane below are set (by the leader)
  std::atomic<int> done{0};   // failed before launch (rc, err)
  const uint32_t *flag = nullptr;
  uint32_t seq = 0;
  OneLane *lane = nullptr;
  int rc = 0;
  std::string err;
};
struct OneLane {
  bool busy = false;          // a launch in flight (read and written by the leader only)
  hipStream_t s = nullptr;
  hipEvent_t ev = nullptr;    // recorded after the launch
  uint32_t seq = 0;           // the last launch's sequence number
  OneDesc *h_desc = nullptr;  // pinned, kOneBatch descriptors
  OneDesc *d_desc = nullptr;  // the kernel's view of h_desc
  // pinned, kOneBatch flags + one nobody waits on (glfsx_debug_one_drop)
  uint32_t *h_flag = nullptr, *d_flag = nullptr;
  // medium posts: device copies of the messages, and per descriptor
  // kMedAuxWords words of CVs / arrival counter / DEK (zeroed when grown;
  // the kernels leave every counter at zero)
  DevBuf med_msg, med_aux;
  size_t aux_zeroed = 0;
};
constexpr uint64_t kMedBatchBytes = 64ull << 20;  // device copies per launch
constexpr size_t kMedAuxWords = 64 * 8 + 8 + 8;   // cvs, dek, cnt (+ pad)
struct OnePoster {
  int dev = -1;
  // requests not yet launched: a lock-free stack (many callers push, the
  // leader takes it whole)
  std::atomic<OneReq *> pending{nullptr};
  std::atomic<bool> leader{false};
  std::atomic<int> spinners{0};  // callers polling their flag without sleeping
  OneLane lane[kOneLanes];
};
// glfsx_one_stats: launches, requests launched, lane-full events
std::atomic<uint64_t> g_one_stats[3];
constexpr int kMaxPosterDevs = 64;
std::mutex g_posters_mu;                               // creation only
std::atomic<OnePoster *> g_posters[kMaxPosterDevs];    // one per device, process lifetime

int poster_get(int dev, OnePoster **out) {
  if (dev < 0 || dev >= kMaxPosterDevs) return fail(GLFSX_E_DEVICE, "device %d", dev);
  if ((*out = g_posters[dev].load(std::memory_order_acquire))) return 0;
  std::lock_guard<std::mutex> lk(g_posters_mu);
  if ((*out = g_posters[dev].load(std::memory_order_acquire))) return 0;
  auto *p = new OnePoster();
  p->dev = dev;
  for (OneLane &l : p->lane) {
    void *h = nullptr, *d = nullptr, *hf = nullptr, *df = nullptr;
    if (hipStreamCreateWithFlags(&l.s, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&l.ev, hipEventDisableTiming) != hipSuccess ||
        hipHostMalloc(&h, sizeof(OneDesc) * kOneBatch, hipHostMallocDefault) != hipSuccess ||
        hipHostGetDevicePointer(&d, h, 0) != hipSuccess ||
        hipHostMalloc(&hf, sizeof(uint32_t) * (kOneBatch + 1), hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer(&df, hf, 0) != hipSuccess) {
      for (OneLane &x : p->lane) {
        if (x.h_desc) (void)hipHostFree(x.h_desc);
        if (x.h_flag) (void)hipHostFree(x.h_flag);
        if (x.s) (void)hipStreamDestroy(x.s);
        if (x.ev) (void)hipEventDestroy(x.ev);
      }
      if (h && h != static_cast<void *>(l.h_desc)) (void)hipHostFree(h);
      if (hf) (void)hipHostFree(hf);
      delete p;
      return fail(GLFSX_E_DEVICE, "one-shot post setup failed on device %d", dev);
    }
    l.h_desc = static_cast<OneDesc *>(h);
    l.d_desc = static_cast<OneDesc *>(d);
    l.h_flag = static_cast<uint32_t *>(hf);
    l.d_flag = static_cast<uint32_t *>(df);
    memset(hf, 0, sizeof(uint32_t) * (kOneBatch + 1));
  }
  g_posters[dev].store(p, std::memory_order_release);
  *out = p;
  return 0;
}

void pending_push(OnePoster *P, OneReq *r) {
  OneReq *h = P->pending.load(std::memory_order_relaxed);
  do {
    r->next = h;
  } while (!P->pending.compare_exchange_weak(h, r, std::memory_order_release,
                                             std::memory_order_relaxed));
}

// Test hook (glfsx_debug_one_drop): the next launch sends request k's
// result flag to the lane's spare word, as a launch that failed on the
// device would leave it: the request's caller must see the error, and no
// caller may return while a request of its call is still queued.
std::atomic<uint32_t> g_one_drop{~0u};

// One launch of k_one over the batch's small messages and one launch_med
// (two kernels) over its medium ones, on the lane's stream; request i's
// flag is lane.h_flag[i], set to `seq` when its results are in place.
int one_launch(OneLane &L, const std::vector<OneReq *> &batch, uint32_t seq) {
  const uint32_t drop = g_one_drop.exchange(~0u, std::memory_order_relaxed);
  uint64_t max_small = 0, max_med = 0, med_bytes = 0;
  size_t ns = 0, nm = 0;
  for (const OneReq *r : batch) {
    if (r->d.len <= kMaxOneLen) {
      ++ns;
      max_small = std::max<uint64_t>(max_small, r->d.len);
    } else {
      ++nm;
      max_med = std::max<uint64_t>(max_med, r->d.len);
      med_bytes += (r->d.len + 255) & ~uint64_t(255);
    }
  }
  if (nm) {
    if (int e = L.med_msg.ensure(med_bytes)) return e;
    if (int e = L.med_aux.ensure(nm * kMedAuxWords * 4)) return e;
    if (L.med_aux.cap > L.aux_zeroed) {  // new buffer: counters must start at zero
      HIP_TRY(hipMemsetAsync(L.med_aux.p, 0, L.med_aux.cap, L.s));
      L.aux_zeroed = L.med_aux.cap;
    }
  }
  size_t is = 0, im = ns;
  uint64_t mo = 0;
  for (size_t k = 0; k < batch.size(); ++k) {
    const OneReq *r = batch[k];
    OneDesc d = r->d;
    d.flag = L.d_flag + (k == drop ? kOneBatch : k);
    d.seq = seq;
    if (r->d.len <= kMaxOneLen) {
      L.h_desc[is++] = d;
      continue;
    }
    uint32_t *aux = reinterpret_cast<uint32_t *>(L.med_aux.p) + (im - ns) * kMedAuxWords;
    d.dmsg = L.med_msg.u8() + mo;
    d.cvs = aux;
    d.dek = aux + 64 * 8;
    d.cnt = aux + 64 * 8 + 8;
    mo += (d.len + 255) & ~uint64_t(255);
    L.h_desc[im++] = d;
  }
  if (ns == 1 && GLFSX_ONE_BYVAL)
    HIP_TRY(launch_one_v(L.h_desc[0], L.s));
  else if (ns)
    HIP_TRY(launch_one(L.d_desc, uint32_t(ns), max_small, L.s));
  if (nm == 1 && GLFSX_ONE_BYVAL)
    HIP_TRY(launch_med_v(L.h_desc[ns], L.s));
  else if (nm)
    HIP_TRY(launch_med(L.d_desc + ns, uint32_t(nm), max_med, L.s));
  HIP_TRY(hipEventRecord(L.ev, L.s));
  return 0;
}

// Request r has its results: its flag reached its launch's sequence number.
bool one_finished(const OneReq *r) {
  if (!r->armed.load(std::memory_order_acquire)) return false;
  const uint32_t v = __atomic_load_n(r->flag, __ATOMIC_ACQUIRE);
  return int32_t(v - r->seq) >= 0;
}

const int kOneSpinners = [] {
  const int h = int(std::thread::hardware_concurrency());
  return std::min(16, std::max(4, h / 2));
}();
constexpr int64_t kOneSpinNs = 300000;
// A sleeping waiter's 10 us sleeps would otherwise end up to the default
// 50 us timer slack late: while a caller's thread sleeps in a one-shot wait
// its slack is 1 us, and the thread's own slack is restored when the wait
// returns (the caller's thread -- a Go runtime M, an application thread --
// is not the library's to retune).
struct SleepSlack {
  long saved = -1;
  void on() {
    if (saved >= 0) return;
    saved = prctl(PR_GET_TIMERSLACK, 0UL, 0UL, 0UL, 0UL);
    if (saved < 0) {
      saved = -2;  // unknown: leave it alone
      return;
    }
    prctl(PR_SET_TIMERSLACK, 1000UL, 0UL, 0UL, 0UL);
  }
  ~SleepSlack() {
    if (saved >= 0) prctl(PR_SET_TIMERSLACK, static_cast<unsigned long>(saved), 0UL, 0UL, 0UL);
  }
};

// Post rs[0..n) on device dev (the calling thread's current device); returns
// when every request's ctext and ref are in its staging.
int one_post_many(int dev, OneReq *const *rs, size_t n) {
  for (size_t i = 0; i < n; ++i)
    if (rs[i]->d.len > kMaxMedLen || (reinterpret_cast<uintptr_t>(rs[i]->d.src) & 15))
      return fail(GLFSX_E_ARG, "one-shot post: bad descriptor");
  OnePoster *P;
  if (int e = poster_get(dev, &P)) return e;
  for (size_t i = 0; i < n; ++i) pending_push(P, rs[i]);
  // Waiting: at most kOneSpinners callers (half the host's threads, 4-16)
  // poll with `pause` (a post is ~45-190 us; up to kOneSpinNs); the others,
  // and a spinner past that bound, sleep between polls.  Yielding instead (round 4) kept
  // every waiting caller runnable: at 64-256 callers on a 16-core share
  // the callers that had work (the leader, a caller whose post finished)
  // waited for a core.
  bool spin = P->spinners.fetch_add(1, std::memory_order_relaxed) < kOneSpinners;
  if (!spin) P->spinners.fetch_sub(1, std::memory_order_relaxed);
  struct Unspin {
    OnePoster *P;
    bool &spin;
    ~Unspin() {
      if (spin) P->spinners.fetch_sub(1, std::memory_order_relaxed);
    }
  } unspin{P, spin};
  SleepSlack slack;
  const auto t0 = std::chrono::steady_clock::now();
  uint32_t sleeps = 0;
  // Once a launch of ours is seen to have failed on the device (frc), the
  // call still returns only when no request of it can be touched again: each
  // is failed before launch, finished, or armed on a lane whose launch has
  // completed.  A request still on the pending stack would otherwise be
  // launched -- its descriptor read, its flag and staging written -- after
  // its caller freed it.
  int frc = 0;
  std::string ferr;
  auto settled = [&frc](const OneReq *r) {
    if (r->done.load(std::memory_order_acquire) || one_finished(r)) return true;
    return frc && r->armed.load(std::memory_order_acquire) &&
           hipEventQuery(r->lane->ev) != hipErrorNotReady;
  };
  size_t ndone = 0;  // rs[0..ndone) are settled
  for (uint32_t spins = 0;; ++spins) {
    while (ndone < n && settled(rs[ndone])) ++ndone;
    if (ndone == n) {
      if (frc) return fail(frc, "%s", ferr.c_str());
      for (size_t i = 0; i < n; ++i)
        if (rs[i]->rc) return fail(rs[i]->rc, "%s", rs[i]->err.c_str());
      return 0;
    }
    // leadership only when there is something to launch and nobody holds it
    // (many waiting callers must not bounce the word between cores)
    bool idle = false;
    if (P->pending.load(std::memory_order_relaxed) &&
        !P->leader.load(std::memory_order_relaxed) &&
        P->leader.compare_exchange_strong(idle, true, std::memory_order_acq_rel)) {
      // a lane whose last launch has completed
      OneLane *L = nullptr;
      int rc = 0;
      for (OneLane &l : P->lane) {
        if (l.busy) {
          const hipError_t q = hipEventQuery(l.ev);
          if (q == hipErrorNotReady) continue;
          if (q != hipSuccess && !rc)
            rc = fail(GLFSX_E_DEVICE, "one-shot post: %s", hipGetErrorString(q));
          l.busy = false;
        }
        L = &l;
        break;
      }
      std::vector<OneReq *> batch;
      if (!L) g_one_stats[2].fetch_add(1, std::memory_order_relaxed);
      if (L) {
        // up to kOneBatch requests, at most kMedBatchBytes of medium ones
        // (always at least one request); the rest goes back on the stack
        OneReq *r = P->pending.exchange(nullptr, std::memory_order_acquire);
        uint64_t mb = 0;
        while (r) {
          OneReq *nx = r->next;
          const uint64_t len = r->d.len;
          const bool fits = batch.size() < kOneBatch &&
                            (len <= kMaxOneLen || batch.empty() || mb + len <= kMedBatchBytes);
          if (fits) {
            if (len > kMaxOneLen) mb += len;
            batch.push_back(r);
          } else {
            pending_push(P, r);
          }
          r = nx;
        }
      }
      if (!batch.empty()) {
        const uint32_t seq = ++L->seq;
        if (!rc) rc = one_launch(*L, batch, seq);
        if (!rc) {
          g_one_stats[0].fetch_add(1, std::memory_order_relaxed);
          g_one_stats[1].fetch_add(batch.size(), std::memory_order_relaxed);
          L->busy = true;
          for (size_t k = 0; k < batch.size(); ++k) {
            batch[k]->flag = L->h_flag + k;
            batch[k]->seq = seq;
            batch[k]->lane = L;
            batch[k]->armed.store(1, std::memory_order_release);
          }
        } else {
          // nothing of this batch runs: its owners get the error (a
          // request's owner may return, and free it, once done is set)
          (void)hipStreamSynchronize(L->s);
          const std::string msg = tls_err;
          for (OneReq *b : batch) {
            b->rc = rc;
            b->err = msg;
            b->done.store(1, std::memory_order_release);
          }
        }
      }
      P->leader.store(false, std::memory_order_release);
      continue;
    }
    if (spin) {
      if ((spins & 31) != 0) {
        for (int k = 0; k < 8; ++k) __builtin_ia32_pause();
        continue;
      }
      // every 32 polls: the core goes to any runnable thread (the HIP
      // runtime's own, a caller with work), and the spin bound is checked
      sched_yield();
      if (std::chrono::duration_cast<std::chrono::nanoseconds>(
              std::chrono::steady_clock::now() - t0).count() < kOneSpinNs)
        continue;
      spin = false;
      P->spinners.fetch_sub(1, std::memory_order_relaxed);
    }
    // sleepers back off 10 -> 40 us: hundreds of them must not wake 100 k
    // times a second each
    slack.on();
    std::this_thread::sleep_for(std::chrono::microseconds(10u << std::min(sleeps, 2u)));
    if (!frc && ++sleeps % 1024 == 0) {
      // a long wait: a launch that failed on the device never sets its flags
      for (size_t i = ndone; i < n; ++i) {
        const OneReq *r = rs[i];
        if (!r->armed.load(std::memory_order_acquire) || one_finished(r)) continue;
        // (the lane's event is ours or a later launch's: either way ours
        // has completed when it has)
        const hipError_t q = hipEventQuery(r->lane->ev);
        if (q == hipErrorNotReady || one_finished(r)) continue;
        frc = GLFSX_E_DEVICE;
        ferr = std::string("one-shot post: ") +
               (q == hipSuccess ? "the launch completed without its result flag"
                                : hipGetErrorString(q));
        break;
      }
    }
  }
}

int one_post(int dev, OneReq *r) { return one_post_many(dev, &r, 1); }

void one_keys(OneDesc &d, const uint8_t salt[32], const uint8_t *cid_key) {
  words_from_key(d.salt, salt);
  if (cid_key) {
    words_from_key(d.cid_key, cid_key);
    d.cid_keyed = 1;
  } else {
    blake3_iv_words(d.cid_key);
    d.cid_keyed = 0;
  }
}

void salt_words(uint32_t w[8], const uint8_t *salt) {
  static const uint8_t zero[32] = {0};
  words_from_key(w, salt ? salt : zero);
}

void cid_words(PostJob &j, const uint8_t *cid_key) {
  if (cid_key) {
    words_from_key(j.cid_key, cid_key);
    j.cid_keyed = true;
  } else {
    blake3_iv_words(j.cid_key);
    j.cid_keyed = false;
  }
}

// DeriveKey on the GPU (ref.go:152-161): keyed BLAKE3 of `in`, 32 bytes.
int derive_key_dev(Ctx *c, uint8_t out[32], const uint8_t salt[32],
                   const void *in, size_t n) {
  if (n > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED, "derive_key input of %zu bytes exceeds %llu",
                n, (unsigned long long)kMaxMsgLen);
  if (int e = c->d_small.ensure(64 + n + 64)) return e;
  if (int e = c->h_small.ensure(64)) return e;
  uint8_t *d_out = c->d_small.u8();
  uint8_t *d_in = c->d_small.u8() + 64;
  if (n) HIP_TRY(hipMemcpyAsync(d_in, in, n, hipMemcpyHostToDevice, c->stream));
  PostJob j{};
  j.src = d_in;
  j.ctext = nullptr;
  j.stride = 0;
  j.msg_len = n;
  j.last_len = n;
  j.n = 1;
  j.out = RefLayout{d_out, ~0ull, 0};
  salt_words(j.salt, salt);
  HIP_TRY(launch_keyed_hash(j, 0, c->stream));
  HIP_TRY(hipMemcpyAsync(c->h_small.p, d_out, 32, hipMemcpyDeviceToHost,
                         c->stream));
  HIP_TRY(stream_wait(c->stream));
  memcpy(out, c->h_small.p, 32);
  return 0;
}

// DeriveKey's full contract (ref.go:152-161): any input length, any output
// length -- the streaming one-workgroup hasher of xof_kernels.hip, input in
// slabs of 256 MiB through device staging.
int derive_key_xof(Ctx *c, uint8_t *out, size_t out_len, const uint8_t salt[32],
                   const void *in, size_t n) {
  constexpr uint64_t kGroup = 256ull << 10, kSlabGroups = 1024;
  if (int e = c->d_small.ensure(sizeof(B3State) + out_len + 64)) return e;
  if (int e = c->d_in.ensure(std::min<uint64_t>(n, kSlabGroups * kGroup) + 64)) return e;
  B3State h{};
  words_from_key(h.key, salt);
  h.base = 16;  // KEYED_HASH (BLAKE3 spec 2.1)
  auto *st = reinterpret_cast<B3State *>(c->d_small.p);
  uint8_t *d_out = c->d_small.u8() + ((sizeof(B3State) + 63) & ~size_t(63));
  HIP_TRY(hipMemcpyAsync(st, &h, sizeof h, hipMemcpyHostToDevice, c->stream));
  const uint8_t *p = static_cast<const uint8_t *>(in);
  // every whole group that does not hold the last byte
  const uint64_t groups = n ? (n - 1) / kGroup : 0;
  for (uint64_t g0 = 0; g0 < groups; g0 += kSlabGroups) {
    const uint64_t k = std::min(kSlabGroups, groups - g0);
    HIP_TRY(hipMemcpyAsync(c->d_in.p, p + g0 * kGroup, k * kGroup, hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(launch_b3_absorb(st, c->d_in.u8(), k, c->stream));
  }
  const uint64_t rem = n - groups * kGroup;
  if (rem)
    HIP_TRY(hipMemcpyAsync(c->d_in.p, p + groups * kGroup, rem, hipMemcpyHostToDevice,
                           c->stream));
  HIP_TRY(launch_b3_final(st, c->d_in.u8(), rem, d_out, out_len, c->stream));
  std::vector<uint8_t> tmp(out_len);
  HIP_TRY(hipMemcpyAsync(tmp.data(), d_out, out_len, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(stream_wait(c->stream));
  memcpy(out, tmp.data(), out_len);
  return 0;
}

int check_block_size(uint64_t bs) {
  if (bs < GLFSX_MIN_BLOCK_SIZE)
    return fail(GLFSX_E_BLOCKSIZE_LT_MIN, "blockSize cannot be < %d",
                GLFSX_MIN_BLOCK_SIZE);
  if (bs > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED,
                "block size %llu above the kernels' limit %llu",
                (unsigned long long)bs, (unsigned long long)kMaxMsgLen);
  return 0;
}

struct Salts {
  uint8_t raw[32], index[32];
};

// blob.go:99-101.  DeriveKey is a pure function, so the (salt -> indexSalt,
// rawSalt) pairs are memoised (process-wide): NewWriter is called once per
// blob by glfs.PostBlob (machine.go:64) and would otherwise cost two launches
// each.
struct SaltCacheEntry {
  uint8_t salt[32];
  Salts s;
};
std::mutex g_salts_mu;
std::vector<SaltCacheEntry> g_salts;

int derive_salts(Ctx *c, const uint8_t *salt, Salts *s) {
  static const uint8_t zero[32] = {0};
  const uint8_t *sl = salt ? salt : zero;
  // the calling thread's last salt first: concurrent PostBlob callers (one
  // salt per type) never touch the process-wide lock
  thread_local SaltCacheEntry last{};
  thread_local bool have_last = false;
  if (have_last && memcmp(last.salt, sl, 32) == 0) {
    *s = last.s;
    return 0;
  }
  {
    std::lock_guard<std::mutex> lk(g_salts_mu);
    for (const auto &e : g_salts)
      if (memcmp(e.salt, sl, 32) == 0) {
        *s = e.s;
        last = e;
        have_last = true;
        return 0;
      }
  }
  if (int e = derive_key_dev(c, s->index, sl, "index", 5)) return e;
  if (int e = derive_key_dev(c, s->raw, sl, "raw", 3)) return e;
  SaltCacheEntry ent;
  memcpy(ent.salt, sl, 32);
  ent.s = *s;
  last = ent;
  have_last = true;
  std::lock_guard<std::mutex> lk(g_salts_mu);
  if (g_salts.size() >= 64) g_salts.erase(g_salts.begin());
  g_salts.push_back(ent);
  return 0;
}

// The zero-padded node images of a level of n refs (index.go:33-38: slot i
// of node k at k*bs + 64i, everything else zero).  With bs a multiple of 64,
// ref j lands at byte 64j, so a level writes exactly [0, 64n): instead of
// zeroing all nodes*bs bytes before every level, only the bytes an earlier
// use may have left non-zero past 64n are cleared (config 2 posts 512 refs
// into a 2 MiB node: a 5.3 us memset per step went).
int level_prepare(DevBuf &b, uint64_t n, uint64_t nodes, uint64_t bs, hipStream_t s) {
  if (int e = b.ensure(nodes * bs)) return e;
  const size_t used = size_t(64) * n;
  if (bs % 64 || b.dirty == SIZE_MAX) {
    HIP_TRY(hipMemsetAsync(b.p, 0, b.cap, s));
    b.dirty = bs % 64 ? SIZE_MAX : used;
    return 0;
  }
  if (b.dirty > used) HIP_TRY(hipMemsetAsync(b.u8() + used, 0, b.dirty - used, s));
  b.dirty = used;
  return 0;
}

// Post `nodes` index nodes (each exactly bs bytes) starting at d_nodes;
// refs go into the next level's node buffer (or dense when out.bf = max).
int post_level(Ctx *c, hipStream_t s, const uint8_t salt[32],
               const uint8_t *cid_key, const uint8_t *d_nodes, uint64_t nodes,
               uint64_t bs, uint8_t *d_ctext, RefLayout out) {
  PostJob j{};
  j.src = d_nodes;
  j.ctext = d_ctext;
  j.stride = bs;
  j.msg_len = bs;
  j.last_len = bs;
  j.n = nodes;
  j.out = out;
  words_from_key(j.salt, salt);
  cid_words(j, cid_key);
  HIP_TRY(launch_post(j, s, tls_fused));
  return 0;
}

// Build the levels above a level whose refs sit in `cur` as `nodes` zero-
// padded index nodes (closed form of blob.go:165-206).
int build_up(Ctx *c, hipStream_t s, const Salts &salts, const uint8_t *cid_key,
             uint64_t bs, uint8_t *cur, uint64_t nodes, DevBuf *spare,
             uint8_t root_ref[64], uint64_t *posts) {
  const uint64_t bf = bs / 64;
  for (;;) {
    if (int e = c->d_ct.ensure(nodes * bs)) return e;
    if (nodes == 1) {
      // the root ref goes straight to pinned host memory (no D2H copy)
      if (int e = c->h_root.ensure(64)) return e;
      if (int e = post_level(c, s, salts.index, cid_key, cur, 1, bs,
                             c->d_ct.u8(), RefLayout{c->h_root.dptr(), ~0ull, 0}))
        return e;
      *posts += 1;
      HIP_TRY(stream_wait(s));
      memcpy(root_ref, c->h_root.p, 64);
      return fused_check(s);
    }
    const uint64_t m = (nodes + bf - 1) / bf;
    if (int e = level_prepare(*spare, nodes, m, bs, s)) return e;
    if (int e = post_level(c, s, salts.index, cid_key, cur, nodes, bs,
                           c->d_ct.u8(), RefLayout{spare->u8(), bf, bs}))
      return e;
    *posts += nodes;
    cur = spare->u8();
    nodes = m;
    spare = (spare == &c->d_lvl_a) ? &c->d_lvl_b : &c->d_lvl_a;
  }
}

}  // namespace

// ------------------------------------------------------------------ Writer
// bigblob/blob.go:71-83.  Complete blocks are staged in pinned batches and
// hashed on the GPU; Post calls and index bookkeeping then replay the
// reference's exact order (postBuf -> addRef -> maybe post index node).
//
// Two batch slots make the host round trip a pipeline: while batch k's H2D
// copy, kernels and D2H copies run on the writer's stream, the caller's
// Write()s fill batch k+1; batch k is completed (Posts delivered) when batch
// k+1 is submitted or at Finish.
struct WSlot {
  PinBuf h_in;   // complete blocks (+ the block being filled while current)
  PinBuf h_ct, h_refs;
  DevBuf d_in, d_ct, d_refs;
  hipEvent_t up = nullptr, hashed = nullptr, done = nullptr;
  uint64_t nblk = 0;  // blocks in flight
  uint64_t seq = 0;   // submission order
  PostJob job{};      // the batch's post (repeated if its fused launch failed)
  int lane = 0;       // writer lane (device + streams) the batch runs on
  bool busy = false;
  bool on_dev = false;  // the staged bytes [0, used) live in d_in, not h_in
                        // (written by glfsx_writer_write_device)
  int dev = -1;       // device of d_* (pool key)
};

// Staging slots outlive writers: glfs.PostBlob opens a Writer per blob
// (machine.go:64), and pinned/device allocation costs far more than hashing a
// small blob.  Freed writers return their slots and streams here.  The pools
// are process-wide (keyed by device), so a writer may be created, used and
// freed on different threads (a goroutine migrating between OS threads).
// Staging of single synchronous posts (index nodes, a writer's tail block).
struct OneBuf {
  DevBuf d_in, d_ct, d_ref;
  PinBuf h_in, h_ct, h_ref;  // h_in: one-shot posts of pageable bytes
  int dev = -1;
};
// Concat's staging (glfsx_writer_write_ctext_blocks): two pinned slabs the
// copy threads gather into, the device copy of a slab, its plaintext and its
// refs.  Pooled per device like the slots: a Concat is one Writer, and
// allocating and pinning ~130 MiB for each one cost more than the hashing.
struct CtextBuf {
  PinBuf h[2];
  hipEvent_t ev[2] = {nullptr, nullptr};
  DevBuf d_ctx, d_ptx, d_rfx;
  int dev = -1;
};
std::mutex g_pool_mu;
std::vector<WSlot> g_slot_pool;
std::vector<OneBuf> g_one_pool;
std::vector<CtextBuf> g_ctext_pool;
struct StreamTriple {
  int dev;
  hipStream_t up, hash, down;
};
std::vector<StreamTriple> g_stream_pool;

void release_slot(WSlot &sl) {
  if (sl.h_in.p) (void)hipHostFree(sl.h_in.p);
  if (sl.h_ct.p) (void)hipHostFree(sl.h_ct.p);
  if (sl.h_refs.p) (void)hipHostFree(sl.h_refs.p);
  if (sl.d_in.p) (void)hipFree(sl.d_in.p);
  if (sl.d_ct.p) (void)hipFree(sl.d_ct.p);
  if (sl.d_refs.p) (void)hipFree(sl.d_refs.p);
  for (hipEvent_t ev : {sl.up, sl.hashed, sl.done})
    if (ev) (void)hipEventDestroy(ev);
  sl = WSlot();
}

// A writer lane: one device with its upload, hash and download streams.
// Batches go round-robin over the lanes (glfsx_writer_set_devices), so one
// Writer fed from one host stream hashes on several GPUs at once, each over
// its own PCIe link, while the Posts still replay in block order.
struct WLane {
  int dev = 0;
  hipStream_t ws = nullptr, s_up = nullptr, s_down = nullptr;
  bool own = false;  // streams of its own (not the writer's home streams)
};

// Pooled writer resources.  take_slot / give_slot_locked / *_locked run
// with g_pool_mu held.
void take_slot(WSlot &x, int dev, int lane) {
  for (size_t i = g_slot_pool.size(); i-- > 0;) {
    if (g_slot_pool[i].dev == dev) {
      x = g_slot_pool[i];
      g_slot_pool.erase(g_slot_pool.begin() + i);
      break;
    }
  }
  x.dev = dev;
  x.lane = lane;
}

void give_slot_locked(WSlot &sl) {
  sl.busy = false;
  sl.nblk = 0;
  sl.on_dev = false;
  if (sl.dev >= 0 && g_slot_pool.size() < 64 * 4)
    g_slot_pool.push_back(sl);  // buffers are reused by the next writer
  else
    release_slot(sl);
  sl = WSlot();
}

int current_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

// A lane's streams of its own: from the pool, or new ones on its device.
int take_streams(WLane &L) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (size_t i = g_stream_pool.size(); i-- > 0;) {
      if (g_stream_pool[i].dev == L.dev) {
        L.s_up = g_stream_pool[i].up;
        L.ws = g_stream_pool[i].hash;
        L.s_down = g_stream_pool[i].down;
        g_stream_pool.erase(g_stream_pool.begin() + i);
        L.own = true;
        return 0;
      }
    }
  }
  const int home = current_device();
  HIP_TRY(hipSetDevice(L.dev));
  hipError_t e = hipStreamCreateWithFlags(&L.ws, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.s_up, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipStreamCreateWithFlags(&L.s_down, hipStreamNonBlocking);
  (void)hipSetDevice(home);
  if (e != hipSuccess) return fail(GLFSX_E_DEVICE, "hipStreamCreate on device %d failed", L.dev);
  L.own = true;
  return 0;
}

void give_streams_locked(WLane &L) {
  if (!L.own) return;
  L.own = false;
  if (g_stream_pool.size() < 64) {
    g_stream_pool.push_back({L.dev, L.s_up, L.ws, L.s_down});
    return;
  }
  const int home = current_device();
  (void)hipSetDevice(L.dev);
  for (hipStream_t st : {L.s_up, L.ws, L.s_down})
    if (st) {
      (void)hipStreamSynchronize(st);
      release_stream_scratch(st);
      (void)hipStreamDestroy(st);
    }
  (void)hipSetDevice(home);
}

void give_streams(WLane &L) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  give_streams_locked(L);
}

// Batch slots: one being filled, one uploading/hashing, one downloading.
// GLFSX_SLOTS (2..4) and GLFSX_BATCH_MIB override the defaults (tuning).
constexpr int kMaxSlots = 4;

// A writer owns everything it touches after creation (streams, batch slots,
// single-post staging, its device id and its last error text), so it does
// not depend on the thread that created it: bigblob.Writer is
// single-goroutine (blob.go:71-83), but a goroutine may run on any OS thread
// between cgo calls.
struct glfsx_writer {
  int dev = 0;  // home device: single posts (index nodes, tail) and device input
  // batch streams: uploads, kernels (also the single posts), downloads, so
  // batch k+1's H2D overlaps batch k's D2H on the full-duplex link
  hipStream_t ws = nullptr, s_up = nullptr, s_down = nullptr;
  uint64_t bs = 0, bf = 0;
  Salts salts{};
  uint8_t cid_key[32]{};
  bool has_cid_key = false;
  glfsx_post_fn post = nullptr;
  void *post_ctx = nullptr;
  std::vector<std::vector<uint8_t>> indexes;  // index.go Index per level
  std::vector<uint64_t> counts;
  uint64_t size = 0;
  OneBuf one;                // single posts (index nodes, the tail block)
  // device input (write_device / write_ctext): events ordering the caller's
  // stream with the upload stream, and write_ctext's staging / temporaries
  hipEvent_t ev_in = nullptr, ev_out = nullptr;
  CtextBuf cx;               // write_ctext's staging (from g_ctext_pool)
  bool has_cx = false;
  std::vector<WLane> lanes;  // lane 0 = the home device and streams by default
  std::vector<WSlot> slot;   // a ring: slot i runs on lane i % lanes.size()
  int nslots = 3;            // slots per lane
  int cur = 0;               // slot being filled
  uint64_t seq = 0;
  uint64_t batch_blocks = 1;
  uint64_t full = 0;         // complete blocks staged in slot[cur]
  uint64_t partial = 0;      // bytes of the block being filled
  uint64_t reserved = 0;     // bytes lent out by glfsx_writer_reserve
  bool strict = false;       // deliver every completed block's Post before
                             // Write returns (blob.go:120-133 error timing)
  int sticky = 0;            // first error; the writer is dead afterwards
  std::string err;           // text of the last failed call on this writer
};

namespace {

const uint8_t *cidk(const glfsx_writer *w) {
  return w->has_cid_key ? w->cid_key : nullptr;
}

// Make `dev` current for a scope and the device that was current before it
// current again at its end (a writer's lanes may live on other devices than
// its home).  The device actually current is read, not assumed: scopes nest
// (submit on lane k completes a batch of lane j, whose replay posts on the
// home device), and a scope that trusted a `home` argument skipped the
// switch while another lane's device was current.
struct DevScope {
  int prev = -1, dev;
  explicit DevScope(int dev_) : dev(dev_) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DevScope() {
    if (prev >= 0 && prev != dev) (void)hipSetDevice(prev);
  }
};

// Grow a pinned buffer keeping its first `keep` bytes.
int pin_grow(PinBuf &b, size_t need, size_t keep) {
  if (need <= b.cap) return 0;
  size_t want = std::max(need, b.cap * 2);
  void *p = nullptr;
  HIP_TRY(hipHostMalloc(&p, want, hipHostMallocPortable));
  void *dp = nullptr;
  if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) {
    (void)hipHostFree(p);
    return fail(GLFSX_E_DEVICE, "hipHostGetDevicePointer failed");
  }
  if (b.p) {
    if (keep) memcpy(p, b.p, keep);
    (void)hipHostFree(b.p);
  }
  b.p = p;
  b.dp = dp;
  b.cap = want;
  return 0;
}

// Host copy into pinned staging; large copies are split over a persistent
// pool of copy threads (the Writer's memcpy into w.buf, blob.go:121-126, is
// its host-side cost: one core copies ≈25 GB/s, a 1 MiB PostBlob spent ≈40
// µs here).  Pieces of >= 256 KiB; the caller copies one piece itself and
// spins until the pool has done the rest.  Workers are started on first use
// (up to 15: the GPU box's share is 16 cores) and live for the process.
struct CopyTask {
  uint8_t *dst;
  const uint8_t *src;
  size_t n;
  std::atomic<int> *left;
  // read_at != nullptr: read n bytes at input offset `off` into dst instead
  // (glfsx_writer_read_at); *got = bytes read, or a negative status
  glfsx_read_at_fn read_at = nullptr;
  void *rctx = nullptr;
  uint64_t off = 0;
  int64_t *got = nullptr;
  // blocks != nullptr: gather nblk blocks (bsz bytes each, the last lastn)
  // into dst back to back instead (par_gather)
  const void *const *blocks = nullptr;
  uint64_t nblk = 0, bsz = 0, lastn = 0;
};
void gather_blocks(uint8_t *dst, const void *const *blocks, uint64_t k, uint64_t bs,
                   uint64_t last) {
  for (uint64_t i = 0; i < k; ++i)
    memcpy(dst + i * bs, blocks[i], i + 1 == k ? last : bs);
}

// Read n bytes at offset off through fn, repeating short reads; stops early
// only at the end of the input (fn returns 0) or on an error (< 0).
int64_t read_full(glfsx_read_at_fn fn, void *ctx, uint8_t *dst, uint64_t n, uint64_t off) {
  uint64_t done = 0;
  while (done < n) {
    const int64_t r = fn(ctx, dst + done, n - done, off + done);
    if (r < 0) return r;
    if (r == 0) break;
    done += uint64_t(r);
  }
  return int64_t(done);
}
struct CopyPool {
  std::mutex mu;
  std::condition_variable cv;
  std::vector<CopyTask> q;
  unsigned workers = 0;
  void run() {
    for (;;) {
      CopyTask t;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !q.empty(); });
        t = q.back();
        q.pop_back();
      }
      if (t.blocks)
        gather_blocks(t.dst, t.blocks, t.nblk, t.bsz, t.lastn);
      else if (t.read_at)
        *t.got = read_full(t.read_at, t.rctx, t.dst, t.n, t.off);
      else
        memcpy(t.dst, t.src, t.n);
      t.left->fetch_sub(1, std::memory_order_release);
    }
  }
};
// The NUMA node device `dev` hangs off (sysfs of its PCI function), or -1.
int device_numa_node(int dev) {
  char bdf[64] = {0};
  if (hipDeviceGetPCIBusId(bdf, int(sizeof bdf) - 1, dev) != hipSuccess) return -1;
  for (char *q = bdf; *q; ++q) *q = char(tolower(*q));
  int node = -1;
  if (FILE *f = fopen((std::string("/sys/bus/pci/devices/") + bdf + "/numa_node").c_str(), "r")) {
    if (fscanf(f, "%d", &node) != 1) node = -1;
    fclose(f);
  }
  return node;
}

// The CPUs of NUMA node `node` within this process's affinity; false if
// unknown or none.
bool node_cpus(int node, cpu_set_t *set) {
  if (node < 0) return false;
  char path[96];
  snprintf(path, sizeof path, "/sys/devices/system/node/node%d/cpulist", node);
  FILE *f = fopen(path, "r");
  if (!f) return false;
  cpu_set_t mine;
  CPU_ZERO(set);
  if (sched_getaffinity(0, sizeof mine, &mine) != 0) {
    fclose(f);
    return false;
  }
  int lo = 0, hi = 0;
  char sep = 0;
  while (fscanf(f, "%d", &lo) == 1) {  // "0-63,128-191"
    hi = lo;
    if (fscanf(f, "%c", &sep) == 1 && sep == '-') {
      if (fscanf(f, "%d", &hi) != 1) break;
      if (fscanf(f, "%c", &sep) != 1) sep = 0;
    }
    for (int c = lo; c <= hi && c < CPU_SETSIZE; ++c)
      if (CPU_ISSET(c, &mine)) CPU_SET(c, set);
    if (sep != ',') break;
  }
  fclose(f);
  return CPU_COUNT(set) > 0;
}

// One copy pool per NUMA node, used for the staging of a device on that
// node: its threads run on the node's CPUs (GLFSX_NUMA=0: one unbound pool
// for every device), so their copies and reads land in pinned staging the
// device's DMA engines read -- a file read from the device's node ran 27-29
// -> 35-38 GiB/s on a two-socket box (bench file_feed).
// A process driving GPUs on both sockets (glfsx_create_devices, a Writer
// over several lanes) gets a pool on each (one process-wide pool
// bound to the first device's node served the other socket's GPUs from the
// wrong node).
bool numa_binding() {
  static const bool on = [] {
    const char *e = getenv("GLFSX_NUMA");
    return !e || atoi(e) != 0;
  }();
  return on;
}

CopyPool &copy_pool(int dev = -1) {
  static std::mutex mu;
  static std::vector<std::pair<int, CopyPool *>> pools;  // (node, pool), process lifetime
  static std::vector<int> dev_node;                      // device -> node (-2: unknown yet)
  if (dev < 0 && hipGetDevice(&dev) != hipSuccess) dev = 0;
  std::lock_guard<std::mutex> lk(mu);
  int node = -1;
  if (numa_binding()) {
    if (size_t(dev) >= dev_node.size()) dev_node.resize(dev + 1, -2);
    if (dev_node[dev] == -2) dev_node[dev] = device_numa_node(dev);
    node = dev_node[dev];
  }
  for (auto &p : pools)
    if (p.first == node) return *p.second;
  auto *cp = new CopyPool();
  const unsigned hw = std::thread::hardware_concurrency();
  cp->workers = std::min(15u, hw > 1 ? hw - 1 : 0u);
  cpu_set_t cpus;
  const bool bind = node_cpus(node, &cpus);
  for (unsigned i = 0; i < cp->workers; ++i)
    std::thread([cp, bind, cpus] {
      if (bind) (void)pthread_setaffinity_np(pthread_self(), sizeof cpus, &cpus);
      cp->run();
    }).detach();
  pools.push_back({node, cp});
  return *cp;
}

// dev: the device whose staging dst is (-1: the current device), which
// picks the copy pool of its NUMA node.
void par_memcpy(uint8_t *dst, const uint8_t *src, size_t n, int dev = -1) {
  constexpr size_t kPiece = 256u << 10;
  if (n < 2 * kPiece) {
    memcpy(dst, src, n);
    return;
  }
  CopyPool &P = copy_pool(dev);
  const size_t parts = std::min<size_t>(P.workers + 1, n / kPiece);
  if (parts <= 1) {
    memcpy(dst, src, n);
    return;
  }
  const size_t per = (n / parts + 4095) & ~size_t(4095);
  std::atomic<int> left{0};
  {
    std::lock_guard<std::mutex> lk(P.mu);
    for (size_t o = per; o < n; o += per) {
      left.fetch_add(1, std::memory_order_relaxed);
      P.q.push_back({dst + o, src + o, std::min(per, n - o), &left});
    }
  }
  P.cv.notify_all();
  memcpy(dst, src, std::min(per, n));
  while (left.load(std::memory_order_acquire) > 0) sched_yield();
}

// k blocks (bs bytes each, the last `last`) from scattered addresses into
// dst back to back, over the copy pool (Concat's ctext straight from the
// store's memory into the Writer's pinned staging).  Blocks of >= 4 MiB go
// one par_memcpy each; smaller ones in runs of consecutive blocks per thread.
void par_gather(uint8_t *dst, const void *const *blocks, uint64_t k, uint64_t bs,
                uint64_t last, int dev = -1) {
  if (k == 0) return;
  if (bs >= (4ull << 20)) {
    for (uint64_t i = 0; i < k; ++i)
      par_memcpy(dst + i * bs, static_cast<const uint8_t *>(blocks[i]), i + 1 == k ? last : bs,
                 dev);
    return;
  }
  const uint64_t total = (k - 1) * bs + last;
  CopyPool &P = copy_pool(dev);
  const uint64_t parts =
      std::min<uint64_t>({uint64_t(P.workers) + 1, k, std::max<uint64_t>(1, total >> 18)});
  if (parts <= 1) {
    gather_blocks(dst, blocks, k, bs, last);
    return;
  }
  const uint64_t per = (k + parts - 1) / parts;
  std::atomic<int> left{0};
  {
    std::lock_guard<std::mutex> lk(P.mu);
    for (uint64_t b = per; b < k; b += per) {
      const uint64_t m = std::min(per, k - b);
      CopyTask t{};
      t.dst = dst + b * bs;
      t.left = &left;
      t.blocks = blocks + b;
      t.nblk = m;
      t.bsz = bs;
      t.lastn = b + m == k ? last : bs;
      left.fetch_add(1, std::memory_order_relaxed);
      P.q.push_back(t);
    }
  }
  P.cv.notify_all();
  gather_blocks(dst, blocks, std::min(per, k), bs, per >= k ? last : bs);
  while (left.load(std::memory_order_acquire) > 0) sched_yield();
}

// The asynchronous form of par_gather (Concat's slabs): every part goes to
// the copy pool and *left counts the parts not yet copied; the caller goes
// on (uploads, decrypts and hashes the previous slab) and waits with
// gather_wait before it reads dst.  Blocks are copied in runs of consecutive
// blocks per task, or -- fewer blocks than threads -- in pieces of >= 1 MiB.
void gather_start(std::atomic<int> *left, uint8_t *dst, const void *const *blocks,
                  uint64_t k, uint64_t bs, uint64_t last, int dev = -1) {
  if (k == 0) return;
  CopyPool &P = copy_pool(dev);
  const uint64_t total = (k - 1) * bs + last;
  if (P.workers == 0) {
    gather_blocks(dst, blocks, k, bs, last);
    return;
  }
  const uint64_t parts = std::max<uint64_t>(1, std::min<uint64_t>(P.workers, total >> 20));
  {
    std::lock_guard<std::mutex> lk(P.mu);
    if (k >= parts) {
      const uint64_t per = (k + parts - 1) / parts;
      for (uint64_t b = 0; b < k; b += per) {
        const uint64_t m = std::min(per, k - b);
        CopyTask t{};
        t.dst = dst + b * bs;
        t.left = left;
        t.blocks = blocks + b;
        t.nblk = m;
        t.bsz = bs;
        t.lastn = b + m == k ? last : bs;
        left->fetch_add(1, std::memory_order_relaxed);
        P.q.push_back(t);
      }
    } else {
      const uint64_t pieces = (parts + k - 1) / k;
      for (uint64_t i = 0; i < k; ++i) {
        const uint64_t n = i + 1 == k ? last : bs;
        const uint64_t per = std::max<uint64_t>(1, ((n / pieces) + 4095) & ~uint64_t(4095));
        for (uint64_t o = 0; o < n; o += per) {
          left->fetch_add(1, std::memory_order_relaxed);
          P.q.push_back({dst + i * bs + o, static_cast<const uint8_t *>(blocks[i]) + o,
                         size_t(std::min(per, n - o)), left});
        }
      }
    }
  }
  P.cv.notify_all();
}

void gather_wait(std::atomic<int> *left) {
  while (left->load(std::memory_order_acquire) > 0) sched_yield();
}

// Read n bytes of input at offset off into dst with the copy pool's threads
// (pieces of >= 4 MiB, the caller reading the first): an io.ReaderAt / a
// file read by several threads at once, as a page-cache copy is one core's
// memcpy.  Returns the bytes of the contiguous prefix read (< n only at the
// end of the input) or the first piece's error (negative).
int64_t par_read_at(glfsx_read_at_fn fn, void *ctx, uint8_t *dst, uint64_t n, uint64_t off,
                    unsigned max_threads, int dev = -1) {
  constexpr uint64_t kPiece = 4ull << 20;
  CopyPool &P = copy_pool(dev);
  const uint64_t parts = std::max<uint64_t>(
      1, std::min<uint64_t>({uint64_t(P.workers) + 1, uint64_t(max_threads), n / kPiece}));
  if (parts <= 1) return read_full(fn, ctx, dst, n, off);
  const uint64_t per = (n / parts + 4095) & ~uint64_t(4095);
  std::vector<int64_t> got((n + per - 1) / per, 0);
  std::atomic<int> left{0};
  {
    std::lock_guard<std::mutex> lk(P.mu);
    for (uint64_t o = per, k = 1; o < n; o += per, ++k) {
      left.fetch_add(1, std::memory_order_relaxed);
      CopyTask t{dst + o, nullptr, size_t(std::min(per, n - o)), &left};
      t.read_at = fn;
      t.rctx = ctx;
      t.off = off + o;
      t.got = &got[k];
      P.q.push_back(t);
    }
  }
  P.cv.notify_all();
  got[0] = read_full(fn, ctx, dst, std::min(per, n), off);
  while (left.load(std::memory_order_acquire) > 0) sched_yield();
  uint64_t total = 0;
  for (uint64_t k = 0; k < got.size(); ++k) {
    if (got[k] < 0) return got[k];
    total += uint64_t(got[k]);
    if (uint64_t(got[k]) < std::min(per, n - k * per)) break;  // end of input
  }
  return int64_t(total);
}

// Post one message from host memory (ref.go:98 post + sink), synchronously,
// with the writer's own staging: messages of at most kMaxOneLen bytes as a
// one-shot post (data read in place when it lies 16-B aligned in the pinned
// buffer `pin`), larger ones on the writer's hash stream.
int post_one(glfsx_writer *w, int kind, const uint8_t salt[32],
             const uint8_t *data, uint64_t n, uint8_t ref[64],
             bool dev_src = false, const PinBuf *pin = nullptr,
             uint64_t present = ~0ull) {
  OneBuf &o = w->one;
  if (!dev_src && n <= kMaxMedLen) {
    if (int e = o.h_ct.ensure(n + 64)) return e;
    if (int e = o.h_ref.ensure(64)) return e;
    const uint64_t have = std::min(n, present);
    OneReq r;
    if (pin && pin->dp && ((data - pin->u8()) & 15) == 0) {
      r.d.src = pin->dptr() + (data - pin->u8());
    } else {
      if (int e = o.h_in.ensure(n + 64)) return e;
      if (have) par_memcpy(o.h_in.u8(), data, have);
      r.d.src = o.h_in.dptr();
    }
    r.d.ctext = w->post ? o.h_ct.dptr() : nullptr;
    r.d.ref = o.h_ref.dptr();
    r.d.len = uint32_t(n);
    r.d.present = uint32_t(have);
    one_keys(r.d, salt, cidk(w));
    if (int e = one_post(w->dev, &r)) return e;
    memcpy(ref, o.h_ref.p, 64);
    if (w->post) {
      int rc = w->post(w->post_ctx, kind, ref, o.h_ct.p, n);
      if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
    }
    return 0;
  }
  if (int e = o.d_in.ensure(n + 64)) return e;
  if (int e = o.d_ct.ensure(n + 64)) return e;
  if (int e = o.d_ref.ensure(64)) return e;
  if (int e = o.h_ct.ensure(n + 64)) return e;
  if (int e = o.h_ref.ensure(64)) return e;
  if (dev_src) {  // data is device memory written on the upload stream
    HIP_TRY(hipEventRecord(w->ev_out, w->s_up));
    HIP_TRY(hipStreamWaitEvent(w->ws, w->ev_out, 0));
  } else if (n) {
    HIP_TRY(hipMemcpyAsync(o.d_in.p, data, n, hipMemcpyHostToDevice, w->ws));
  }
  PostJob j{};
  j.src = dev_src ? data : o.d_in.u8();
  j.ctext = o.d_ct.u8();
  j.stride = 0;
  j.msg_len = n;
  j.last_len = n;
  j.n = 1;
  j.out = RefLayout{o.d_ref.u8(), ~0ull, 0};
  words_from_key(j.salt, salt);
  cid_words(j, cidk(w));
  HIP_TRY(launch_post(j, w->ws, tls_fused));
  if (n)
    HIP_TRY(hipMemcpyAsync(o.h_ct.p, o.d_ct.p, n, hipMemcpyDeviceToHost, w->ws));
  HIP_TRY(hipMemcpyAsync(o.h_ref.p, o.d_ref.p, 64, hipMemcpyDeviceToHost, w->ws));
  HIP_TRY(stream_wait(w->ws));
  memcpy(ref, o.h_ref.p, 64);
  if (w->post) {
    int rc = w->post(w->post_ctx, kind, ref, o.h_ct.p, n);
    if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
  }
  return 0;
}

// blob.go:165-182
// A level's node holds only its refs (64 B each); it is zero padded to bs
// bytes when posted (index.go:33-38), so a one-block blob never touches a
// bs-byte buffer.
int post_node(glfsx_writer *w, size_t i, uint8_t r[64]) {
  std::vector<uint8_t> &v = w->indexes[i];
  int e;
  if (w->bs <= kMaxMedLen) {  // the kernel reads the rest as zero
    e = post_one(w, 1, w->salts.index, v.data(), w->bs, r, false, nullptr, v.size());
  } else {
    v.resize(w->bs, 0);
    e = post_one(w, 1, w->salts.index, v.data(), w->bs, r);
  }
  v.clear();
  return e;
}

int add_ref(glfsx_writer *w, size_t i, const uint8_t ref[64]) {
  if (w->indexes.size() <= i) {
    w->indexes.emplace_back();
    w->counts.push_back(0);
  }
  w->indexes[i].insert(w->indexes[i].end(), ref, ref + 64);
  w->counts[i]++;
  if (w->counts[i] < w->bf) return 0;
  uint8_t r2[64];
  if (int e = post_node(w, i, r2)) return e;
  w->counts[i] = 0;
  return add_ref(w, i + 1, r2);
}

// A one-launch split post on the hash stream failed (fused_check): the
// error word cannot tell which batch's launch it was, so every batch still
// in flight is hashed again with two launches per post, in order.
int rehash_inflight(glfsx_writer *w) {
  for (const WLane &L : w->lanes) {
    DevScope d(L.dev);
    HIP_TRY(hipStreamSynchronize(L.ws));
    HIP_TRY(hipStreamSynchronize(L.s_down));
    (void)fused_errors_take(L.ws);
  }
  for (WSlot &x : w->slot) {
    if (!x.busy) continue;
    const WLane &L = w->lanes[x.lane];
    DevScope d(L.dev);
    HIP_TRY(launch_post(x.job, L.ws, false));
    HIP_TRY(hipMemcpyAsync(x.h_refs.p, x.d_refs.p, x.nblk * 64, hipMemcpyDeviceToHost, L.ws));
    if (w->post)
      HIP_TRY(hipMemcpyAsync(x.h_ct.p, x.d_ct.p, x.nblk * w->bs, hipMemcpyDeviceToHost,
                             L.ws));
  }
  for (const WLane &L : w->lanes) {
    DevScope d(L.dev);
    HIP_TRY(stream_wait(L.ws));
  }
  return 0;
}

// Wait for an in-flight batch and replay postBuf (blob.go:152-163) for each
// of its blocks, in order.
int complete(glfsx_writer *w, WSlot &sl) {
  if (!sl.busy) return 0;
  HIP_TRY(hipEventSynchronize(sl.done));
  bool failed;
  {
    const WLane &L = w->lanes[sl.lane];
    DevScope d(L.dev);
    failed = fused_errors_take(L.ws) != 0;
  }
  // the replay's single posts (index nodes: post_one on the writer's hash
  // stream and staging) run on the home device, whichever lane's device the
  // caller (submit) has current
  DevScope home(w->dev);
  if (failed)
    if (int e = rehash_inflight(w)) return e;
  sl.busy = false;
  for (uint64_t b = 0; b < sl.nblk; ++b) {
    const uint8_t *ref = sl.h_refs.u8() + 64 * b;
    if (w->post) {
      int rc = w->post(w->post_ctx, 0, ref, sl.h_ct.u8() + b * w->bs, w->bs);
      if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
    }
    if (int e = add_ref(w, 0, ref)) return e;
    w->size += w->bs;
  }
  return 0;
}

// Enqueue the current slot's complete blocks (H2D, DEK + ChaCha/CID kernels,
// D2H of refs and ctext), finish the oldest batch still in flight if it
// holds the next slot, and switch slots, carrying the partial block over.
int submit(glfsx_writer *w) {
  if (w->full == 0) return 0;
  WSlot &sl = w->slot[w->cur];
  const int next = (w->cur + 1) % int(w->slot.size());
  WSlot &nx = w->slot[next];
  const WLane &L = w->lanes[sl.lane];
  DevScope dscope(L.dev);
  const uint64_t nbytes = w->full * w->bs;
  if (int e = sl.d_in.ensure(nbytes)) return e;
  if (int e = sl.d_ct.ensure(nbytes)) return e;
  if (int e = sl.d_refs.ensure(w->full * 64)) return e;
  if (w->post)
    if (int e = sl.h_ct.ensure(nbytes + 64)) return e;
  if (int e = sl.h_refs.ensure(w->full * 64)) return e;
  if (!sl.done) {
    HIP_TRY(hipEventCreateWithFlags(&sl.up, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&sl.hashed, hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
  }
  if (!sl.on_dev)  // device-written bytes are already in d_in (s_up order)
    HIP_TRY(hipMemcpyAsync(sl.d_in.p, sl.h_in.p, nbytes, hipMemcpyHostToDevice, L.s_up));
  HIP_TRY(hipEventRecord(sl.up, L.s_up));
  HIP_TRY(hipStreamWaitEvent(L.ws, sl.up, 0));
  PostJob j{};
  j.src = sl.d_in.u8();
  j.ctext = sl.d_ct.u8();
  j.stride = w->bs;
  j.msg_len = w->bs;
  j.last_len = w->bs;
  j.n = w->full;
  j.out = RefLayout{sl.d_refs.u8(), ~0ull, 0};
  words_from_key(j.salt, w->salts.raw);
  cid_words(j, cidk(w));
  sl.job = j;
  HIP_TRY(launch_post(j, L.ws, tls_fused));
  HIP_TRY(hipEventRecord(sl.hashed, L.ws));
  HIP_TRY(hipStreamWaitEvent(L.s_down, sl.hashed, 0));
  HIP_TRY(hipMemcpyAsync(sl.h_refs.p, sl.d_refs.p, w->full * 64,
                         hipMemcpyDeviceToHost, L.s_down));
  if (w->post)
    HIP_TRY(hipMemcpyAsync(sl.h_ct.p, sl.d_ct.p, nbytes, hipMemcpyDeviceToHost,
                           L.s_down));
  HIP_TRY(hipEventRecord(sl.done, L.s_down));
  sl.nblk = w->full;
  sl.seq = ++w->seq;
  sl.busy = true;
  // `nx` is the oldest batch in flight (submitted nslots-1 batches ago):
  // completing it keeps Posts in order
  if (int e = complete(w, nx)) return e;
  if (sl.on_dev) {  // carry the partial block over on the device (one lane)
    if (int e = nx.d_in.ensure(w->batch_blocks * w->bs + 64)) return e;
    if (w->partial)
      HIP_TRY(hipMemcpyAsync(nx.d_in.p, sl.d_in.u8() + nbytes, w->partial,
                             hipMemcpyDeviceToDevice, L.s_up));
    nx.on_dev = true;
  } else {
    if (int e = pin_grow(nx.h_in, std::max<uint64_t>(w->partial, 1), 0)) return e;
    if (w->partial) memcpy(nx.h_in.u8(), sl.h_in.u8() + nbytes, w->partial);
    nx.on_dev = false;
  }
  w->cur = next;
  w->full = 0;
  return 0;
}

// Move the current slot's staged bytes between host and device staging.
int slot_to_device(glfsx_writer *w) {
  WSlot &sl = w->slot[w->cur];
  if (sl.on_dev) return 0;
  const uint64_t used = w->full * w->bs + w->partial;
  if (int e = sl.d_in.ensure(w->batch_blocks * w->bs + 64)) return e;
  if (used)
    HIP_TRY(hipMemcpyAsync(sl.d_in.p, sl.h_in.p, used, hipMemcpyHostToDevice, w->s_up));
  sl.on_dev = true;
  return 0;
}

int slot_to_host(glfsx_writer *w) {
  WSlot &sl = w->slot[w->cur];
  if (!sl.on_dev) return 0;
  const uint64_t used = w->full * w->bs + w->partial;
  if (int e = pin_grow(sl.h_in, std::max<uint64_t>(used, 1), 0)) return e;
  if (used) {
    HIP_TRY(hipMemcpyAsync(sl.h_in.p, sl.d_in.p, used, hipMemcpyDeviceToHost, w->s_up));
    HIP_TRY(hipStreamSynchronize(w->s_up));
  }
  sl.on_dev = false;
  return 0;
}

// Append n device bytes, ordered after everything already on the upload
// stream (blob.go:120-133 block bookkeeping, as glfsx_writer_write).
int write_dev(glfsx_writer *w, const uint8_t *p, uint64_t n) {
  while (n) {
    if (int e = slot_to_device(w)) return e;
    WSlot &sl = w->slot[w->cur];
    const uint64_t used = w->full * w->bs + w->partial;
    const uint64_t cap = w->batch_blocks * w->bs;
    const uint64_t take = std::min<uint64_t>(cap - used, n);
    HIP_TRY(hipMemcpyAsync(sl.d_in.u8() + used, p, take, hipMemcpyDeviceToDevice, w->s_up));
    p += take;
    n -= take;
    w->full = (used + take) / w->bs;
    w->partial = (used + take) % w->bs;
    if (w->full == w->batch_blocks)
      if (int e = submit(w)) return e;
  }
  return 0;
}

// blob.go:184-206
int finish_indexes(glfsx_writer *w, uint8_t out[64]) {
  for (size_t i = 0; i < w->indexes.size(); ++i) {
    if (i + 1 == w->indexes.size()) {
      if (w->counts[i] == 0)
        return post_one(w, 1, w->salts.index, nullptr, 0, out);
      if (w->counts[i] == 1) {
        memcpy(out, w->indexes[i].data(), 64);
        return 0;
      }
    }
    if (w->counts[i] > 0) {
      uint8_t r[64];
      if (int e = post_node(w, i, r)) return e;
      if (int e = add_ref(w, i + 1, r)) return e;
    }
  }
  return fail(GLFSX_E_ARG, "should not happen");
}

}  // namespace

extern "C" {

const char *glfsx_last_error(void) { return tls_err.c_str(); }

const char *glfsx_version(void) { return "glfsx 0.1 gfx950"; }

uint32_t glfsx_set_split_target(uint32_t wgs) { return set_split_target(wgs); }
uint32_t glfsx_set_latency_wgs(uint32_t wgs) { return set_latency_wgs(wgs); }

uint64_t glfsx_debug_fused(uint32_t skip_msg, uint64_t wait_us) {
  fused_debug(skip_msg, wait_us);
  return fused_timeouts();
}

uint64_t glfsx_fused_failures(void) { return fused_timeouts(); }

void glfsx_debug_one_drop(uint32_t k) { g_one_drop.store(k, std::memory_order_relaxed); }

int glfsx_one_stats(int reset, uint64_t out[3]) {
  for (int i = 0; i < 3; ++i) {
    const uint64_t v = reset ? g_one_stats[i].exchange(0, std::memory_order_relaxed)
                             : g_one_stats[i].load(std::memory_order_relaxed);
    if (out) out[i] = v;
  }
  return 0;
}

int glfsx_clock_probe(int reset, uint64_t out[2]) {
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  HIP_TRY(clock_probe(reset, out));
  return 0;
}

#if GLFSX_WGTIME
// diagnostic builds only (tools/build_variant.sh): the bulk passes' phase
// timestamps, 8192 x 16 words
int glfsx_debug_wgtime(uint64_t *out) {
  HIP_TRY(debug_wgtime(out));
  return 0;
}
#endif

int glfsx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int glfsx_set_device(int dev) {
  if (dev < 0) return fail(GLFSX_E_ARG, "negative device");
  tls_dev = dev;
  Ctx *c;
  return ctx_get(&c);
}

int glfsx_derive_key(uint8_t *out, size_t out_len, const uint8_t salt[32],
                     const void *input, size_t n) {
  if ((out_len && !out) || !salt || (n && !input)) return fail(GLFSX_E_ARG, "null argument");
  if (out_len == 0) return 0;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  if (out_len > 32 || n > kMaxMsgLen)
    return derive_key_xof(c, static_cast<uint8_t *>(out), out_len, salt, input, n);
  uint8_t full[32];
  if (int e = derive_key_dev(c, full, salt, input, n)) return e;
  memcpy(out, full, out_len);
  return 0;
}

int glfsx_post_batch_device(const uint8_t salt[32], const void *d_ptext,
                            uint64_t total, uint64_t block_size, void *d_ctext,
                            void *d_refs, const uint8_t *cid_key,
                            void *stream) {
  if (!salt || !d_refs || (total && !d_ptext))
    return fail(GLFSX_E_ARG, "null argument");
  if (block_size == 0 || block_size > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED, "block size %llu unsupported",
                (unsigned long long)block_size);
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  const uint64_t n = (total + block_size - 1) / block_size;
  if (n == 0) return 0;
  PostJob j{};
  j.src = static_cast<const uint8_t *>(d_ptext);
  j.ctext = static_cast<uint8_t *>(d_ctext);
  j.stride = block_size;
  j.msg_len = block_size;
  j.last_len = total - (n - 1) * block_size;
  j.n = n;
  j.out = RefLayout{static_cast<uint8_t *>(d_refs), ~0ull, 0};
  words_from_key(j.salt, salt);
  cid_words(j, cid_key);
  HIP_TRY(launch_post(j, pick_stream(c, stream), false));
  return 0;
}

// Shared setup for the device batch entry points.
static int batch_job(PostJob *j, const void *d_ptext, uint64_t total,
                     uint64_t block_size, void *d_ctext, void *d_refs) {
  if (!d_refs || (total && !d_ptext)) return fail(GLFSX_E_ARG, "null argument");
  if (block_size == 0 || block_size > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED, "block size %llu unsupported",
                (unsigned long long)block_size);
  const uint64_t n = (total + block_size - 1) / block_size;
  *j = PostJob{};
  j->src = static_cast<const uint8_t *>(d_ptext);
  j->ctext = static_cast<uint8_t *>(d_ctext);
  j->stride = block_size;
  j->msg_len = block_size;
  j->last_len = n ? total - (n - 1) * block_size : 0;
  j->n = n;
  j->out = RefLayout{static_cast<uint8_t *>(d_refs), ~0ull, 0};
  return 0;
}

int glfsx_dek_batch_device(const uint8_t salt[32], const void *d_ptext,
                           uint64_t total, uint64_t block_size, void *d_refs,
                           void *stream) {
  if (!salt) return fail(GLFSX_E_ARG, "null salt");
  PostJob j;
  if (int e = batch_job(&j, d_ptext, total, block_size, nullptr, d_refs)) return e;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  words_from_key(j.salt, salt);
  HIP_TRY(launch_keyed_hash(j, 32, pick_stream(c, stream)));
  return 0;
}

int glfsx_cid_batch_device(const void *d_ptext, uint64_t total,
                           uint64_t block_size, void *d_ctext, void *d_refs,
                           const uint8_t *cid_key, void *stream) {
  PostJob j;
  if (int e = batch_job(&j, d_ptext, total, block_size, d_ctext, d_refs)) return e;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  cid_words(j, cid_key);
  HIP_TRY(launch_cid_pass(j, pick_stream(c, stream)));
  return 0;
}

int glfsx_post(const uint8_t salt[32], const void *ptext, uint64_t n,
               void *ctext_out, uint8_t *ref_out, const uint8_t *cid_key) {
  if (!salt || !ref_out || (n && !ptext)) return fail(GLFSX_E_ARG, "null argument");
  if (n > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED, "message of %llu bytes above the kernels' limit %llu",
                (unsigned long long)n, (unsigned long long)kMaxMsgLen);
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  if (n <= kMaxMedLen) {
    if (int e = c->h_oin.ensure(n + 64)) return e;
    if (int e = c->h_oct.ensure(n + 64)) return e;
    if (int e = c->h_oref.ensure(64)) return e;
    if (n) par_memcpy(c->h_oin.u8(), static_cast<const uint8_t *>(ptext), n);
    OneReq r;
    r.d.src = c->h_oin.dptr();
    r.d.ctext = (ctext_out && n) ? c->h_oct.dptr() : nullptr;
    r.d.ref = c->h_oref.dptr();
    r.d.len = uint32_t(n);
    r.d.present = uint32_t(n);
    one_keys(r.d, salt, cid_key);
    if (int e = one_post(c->dev, &r)) return e;
    memcpy(ref_out, c->h_oref.p, 64);
    if (ctext_out && n) memcpy(ctext_out, c->h_oct.p, n);
    return 0;
  }
  if (int e = c->d_in.ensure(n + 64)) return e;
  if (int e = c->d_ct.ensure(n + 64)) return e;
  if (int e = c->d_refs.ensure(64)) return e;
  if (n)
    HIP_TRY(hipMemcpyAsync(c->d_in.p, ptext, n, hipMemcpyHostToDevice, c->stream));
  PostJob j{};  // one message; n == 0 is the empty message (one empty chunk)
  j.src = c->d_in.u8();
  j.ctext = c->d_ct.u8();
  j.stride = 0;
  j.msg_len = n;
  j.last_len = n;
  j.n = 1;
  j.out = RefLayout{c->d_refs.u8(), ~0ull, 0};
  words_from_key(j.salt, salt);
  cid_words(j, cid_key);
  HIP_TRY(launch_post(j, c->stream, tls_fused));
  HIP_TRY(hipMemcpyAsync(ref_out, c->d_refs.p, 64, hipMemcpyDeviceToHost, c->stream));
  if (ctext_out && n)
    HIP_TRY(hipMemcpyAsync(ctext_out, c->d_ct.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(stream_wait(c->stream));
  return 0;
}

int glfsx_post_batch(const uint8_t salt[32], const void *ptext, uint64_t total,
                     uint64_t block_size, void *ctext_out, uint8_t *refs_out,
                     const uint8_t *cid_key) {
  if (!salt || !refs_out || (total && !ptext))
    return fail(GLFSX_E_ARG, "null argument");
  if (block_size == 0 || block_size > kMaxMsgLen)
    return fail(GLFSX_E_UNSUPPORTED, "block size %llu unsupported",
                (unsigned long long)block_size);
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  const uint64_t n = (total + block_size - 1) / block_size;
  if (n == 0) return 0;
  // Stage in slabs of whole blocks (<= 256 MiB) to bound device memory.
  const uint64_t slab_blocks =
      std::max<uint64_t>(1, (256ull << 20) / block_size);
  for (uint64_t b0 = 0; b0 < n; b0 += slab_blocks) {
    const uint64_t nb = std::min(slab_blocks, n - b0);
    const uint64_t off = b0 * block_size;
    const uint64_t bytes = std::min<uint64_t>(nb * block_size, total - off);
    if (int e = c->d_in.ensure(bytes + 64)) return e;
    if (int e = c->d_ct.ensure(bytes + 64)) return e;
    if (int e = c->d_refs.ensure(nb * 64)) return e;
    HIP_TRY(hipMemcpyAsync(c->d_in.p, static_cast<const uint8_t *>(ptext) + off,
                           bytes, hipMemcpyHostToDevice, c->stream));
    PostJob j{};
    j.src = c->d_in.u8();
    j.ctext = c->d_ct.u8();
    j.stride = block_size;
    j.msg_len = block_size;
    j.last_len = bytes - (nb - 1) * block_size;
    j.n = nb;
    j.out = RefLayout{c->d_refs.u8(), ~0ull, 0};
    words_from_key(j.salt, salt);
    cid_words(j, cid_key);
    for (bool fused : {true, false}) {  // again with two launches if the fused one failed
      HIP_TRY(launch_post(j, c->stream, fused));
      HIP_TRY(hipMemcpyAsync(refs_out + 64 * b0, c->d_refs.p, nb * 64,
                             hipMemcpyDeviceToHost, c->stream));
      if (ctext_out)
        HIP_TRY(hipMemcpyAsync(static_cast<uint8_t *>(ctext_out) + off, c->d_ct.p,
                               bytes, hipMemcpyDeviceToHost, c->stream));
      HIP_TRY(stream_wait(c->stream));
      if (!fused_errors_take(c->stream)) break;
    }
  }
  return 0;
}

glfsx_writer *glfsx_writer_new(uint64_t block_size, uint64_t store_max,
                               const uint8_t *salt, const uint8_t *cid_key,
                               glfsx_post_fn post, void *post_ctx, int *err) {
  int dummy;
  if (!err) err = &dummy;
  uint64_t bs = store_max;  // blob.go:86
  if (block_size > 0) bs = block_size;
  if (bs > store_max) {  // blob.go:90-92
    *err = fail(GLFSX_E_BLOCKSIZE_GT_MAX, "blockSize %llu > maxSize %llu",
                (unsigned long long)bs, (unsigned long long)store_max);
    return nullptr;
  }
  if (int e = check_block_size(bs)) {  // blob.go:93-95
    *err = e;
    return nullptr;
  }
  Ctx *c;
  if (int e = ctx_get(&c)) {
    *err = e;
    return nullptr;
  }
  auto *w = new glfsx_writer();
  w->dev = c->dev;
  w->bs = bs;
  w->bf = bs / 64;  // blob.go:107
  if (int e = derive_salts(c, salt, &w->salts)) {
    delete w;
    *err = e;
    return nullptr;
  }
  if (cid_key) {
    memcpy(w->cid_key, cid_key, 32);
    w->has_cid_key = true;
  }
  w->post = post;
  w->post_ctx = post_ctx;
  w->indexes.emplace_back();  // blob.go:111 (refs only, see post_node)
  w->counts.push_back(0);
  uint64_t batch_mib = 64;
  if (const char *e = getenv("GLFSX_BATCH_MIB")) batch_mib = std::max(1ull, strtoull(e, nullptr, 10));
  if (const char *e = getenv("GLFSX_SLOTS")) w->nslots = std::min(kMaxSlots, std::max(2, atoi(e)));
  w->batch_blocks = std::max<uint64_t>(1, (batch_mib << 20) / bs);
  w->slot.resize(w->nslots);
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (WSlot &x : w->slot) take_slot(x, w->dev, 0);
    for (size_t i = g_one_pool.size(); i-- > 0;) {
      if (g_one_pool[i].dev == w->dev) {
        w->one = g_one_pool[i];
        g_one_pool.erase(g_one_pool.begin() + i);
        break;
      }
    }
    w->one.dev = w->dev;
    for (size_t i = g_stream_pool.size(); i-- > 0;) {
      if (g_stream_pool[i].dev == w->dev) {
        w->s_up = g_stream_pool[i].up;
        w->ws = g_stream_pool[i].hash;
        w->s_down = g_stream_pool[i].down;
        g_stream_pool.erase(g_stream_pool.begin() + i);
        break;
      }
    }
  }
  if (!w->ws &&
      (hipStreamCreateWithFlags(&w->ws, hipStreamNonBlocking) != hipSuccess ||
       hipStreamCreateWithFlags(&w->s_up, hipStreamNonBlocking) != hipSuccess ||
       hipStreamCreateWithFlags(&w->s_down, hipStreamNonBlocking) != hipSuccess)) {
    glfsx_writer_free(w);
    *err = fail(GLFSX_E_DEVICE, "hipStreamCreate failed");
    return nullptr;
  }
  w->lanes.push_back(WLane{w->dev, w->ws, w->s_up, w->s_down, false});
  *err = 0;
  return w;
}

int glfsx_writer_set_devices(glfsx_writer *w, const int *devs, int ndev) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  if (!devs || ndev < 1 || ndev > 64) return fail(GLFSX_E_ARG, "need 1..64 devices");
  if (w->seq || w->full || w->partial || w->size || w->sticky || w->ev_in)
    return fail(GLFSX_E_ARG, "glfsx_writer_set_devices: the writer has already been written to");
  const int n = glfsx_device_count();
  for (int k = 0; k < ndev; ++k)
    if (devs[k] < 0 || devs[k] >= n)
      return fail(GLFSX_E_ARG, "device %d out of range (%d devices)", devs[k], n);
  std::vector<WLane> lanes(ndev);
  for (int k = 0; k < ndev; ++k) {
    lanes[k].dev = devs[k];
    if (devs[k] == w->dev) {  // the home streams
      lanes[k] = WLane{w->dev, w->ws, w->s_up, w->s_down, false};
      continue;
    }
    // lanes on one device share its streams: a device's copy engines and
    // hardware queues are the resource (GPU_MAX_HW_QUEUES = 4 per process;
    // more streams on one device alias queues and serialise each other:
    // 4 GiB through lanes [0, 0] 40.8 -> 29 GiB/s with separate streams)
    bool shared = false;
    for (int i = 0; i < k && !shared; ++i)
      if (lanes[i].dev == devs[k]) {
        lanes[k] = WLane{devs[k], lanes[i].ws, lanes[i].s_up, lanes[i].s_down, false};
        shared = true;
      }
    if (shared) continue;
    if (int e = take_streams(lanes[k])) {
      for (int i = 0; i < k; ++i) give_streams(lanes[i]);
      return e;
    }
  }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  for (WLane &L : w->lanes) give_streams_locked(L);
  for (WSlot &x : w->slot) give_slot_locked(x);
  w->lanes = std::move(lanes);
  w->slot.assign(size_t(w->nslots) * ndev, WSlot());
  for (size_t i = 0; i < w->slot.size(); ++i)
    take_slot(w->slot[i], w->lanes[i % ndev].dev, int(i % ndev));
  w->cur = 0;
  return 0;
}

namespace {
// Every writer entry point runs on the writer's device (the calling thread
// may have another one current) and keeps the error text on the writer.
struct WriterCall {
  glfsx_writer *w;
  explicit WriterCall(glfsx_writer *w_) : w(w_) {
    int cur = -1;  // a Write of 32 KiB (io.Copy) costs ~1.7 us: skip the set
    if (hipGetDevice(&cur) != hipSuccess || cur != w->dev) (void)hipSetDevice(w->dev);
  }
  int done(int rc) {
    if (rc) w->err = tls_err;
    return rc;
  }
};

// Drain: submit the staged complete blocks and deliver the Posts of every
// batch in flight, oldest first.
int complete_all(glfsx_writer *w) {
  for (;;) {
    WSlot *o = nullptr;
    for (auto &sl : w->slot)
      if (sl.busy && (!o || sl.seq < o->seq)) o = &sl;
    if (!o) return 0;
    if (int e = complete(w, *o)) return e;
  }
}

int drain(glfsx_writer *w) {
  if (int e = submit(w)) return e;
  return complete_all(w);
}

// A few complete blocks (<= kFewBlocks) staged on the host -- with the tail
// at Finish, or without it in a strict Write -- go out as one coalesced
// one-shot post (a request per block, the kernels reading the pinned
// staging in place) instead of a batch through the three-stream pipeline:
// a PostBlob of a few MiB, or a strict Write that completes a block, is one
// launch pair and one wait.  Posts and addRef replay in block order
// (blob.go:152-163), after every older batch's.  Without the tail, the
// partial block's bytes move to the front of the staging.
constexpr uint64_t kFewBlocks = 8;
int post_few(glfsx_writer *w, bool tail, bool *done) {
  *done = false;
  WSlot &sl = w->slot[w->cur];
  if (sl.on_dev || w->full == 0 || w->full > kFewBlocks ||
      w->bs > kMaxMedLen || (w->bs & 15) || !sl.h_in.dp)
    return 0;
  if (int e = complete_all(w)) return e;
  const uint64_t k = w->full + (tail && w->partial ? 1 : 0);
  OneBuf &o = w->one;
  if (w->post)
    if (int e = o.h_ct.ensure(w->full * w->bs + w->partial + 64)) return e;
  if (int e = o.h_ref.ensure(64 * k)) return e;
  std::vector<OneReq> reqs(k);
  std::vector<OneReq *> rp(k);
  for (uint64_t b = 0; b < k; ++b) {
    const uint64_t off = b * w->bs;
    OneDesc &d = reqs[b].d;
    d.src = sl.h_in.dptr() + off;
    d.ctext = w->post ? o.h_ct.dptr() + off : nullptr;
    d.ref = o.h_ref.dptr() + 64 * b;
    d.len = uint32_t(b < w->full ? w->bs : w->partial);
    d.present = d.len;
    one_keys(d, w->salts.raw, cidk(w));
    rp[b] = &reqs[b];
  }
  if (int e = one_post_many(w->dev, rp.data(), k)) return e;
  // refs out first: an index node posted by add_ref reuses the single-post
  // staging (its ctext lands on block 0's, already delivered)
  std::vector<uint8_t> refs(o.h_ref.u8(), o.h_ref.u8() + 64 * k);
  for (uint64_t b = 0; b < k; ++b) {
    const uint64_t len = reqs[b].d.len;
    if (w->post) {
      int rc = w->post(w->post_ctx, 0, &refs[64 * b], o.h_ct.u8() + b * w->bs, len);
      if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
    }
    if (int e = add_ref(w, 0, &refs[64 * b])) return e;
    w->size += len;
  }
  if (tail)
    w->partial = 0;
  else if (w->partial)
    memmove(sl.h_in.u8(), sl.h_in.u8() + w->full * w->bs, w->partial);
  w->full = 0;
  *done = true;
  return 0;
}

// blob.go:120-133 error timing: deliver the Posts of every block completed
// so far before the Write returns.
int drain_strict(glfsx_writer *w) {
  bool few = false;
  if (int e = post_few(w, false, &few)) return e;
  return few ? complete_all(w) : drain(w);
}
}  // namespace

// blob.go:120-133: a block is complete exactly when buffered + incoming
// reaches bs; complete blocks are hashed a batch at a time.
int glfsx_writer_write(glfsx_writer *w, const void *data, size_t n) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (n && !data) return call.done(fail(GLFSX_E_ARG, "null data"));
  const uint8_t *p = static_cast<const uint8_t *>(data);
  while (n) {
    if (int e = slot_to_host(w)) return call.done(w->sticky = e);
    WSlot &sl = w->slot[w->cur];
    const uint64_t used = w->full * w->bs + w->partial;
    const uint64_t cap = w->batch_blocks * w->bs;  // slot holds up to a batch
    const uint64_t take = std::min<uint64_t>(cap - used, n);
    if (int e = pin_grow(sl.h_in, used + take, used)) return call.done(w->sticky = e);
    par_memcpy(sl.h_in.u8() + used, p, take, w->lanes[sl.lane].dev);
    p += take;
    n -= take;
    w->full = (used + take) / w->bs;
    w->partial = (used + take) % w->bs;
    if (w->full == w->batch_blocks)
      if (int e = submit(w)) return call.done(w->sticky = e);
  }
  if (w->strict)
    if (int e = drain_strict(w)) return call.done(w->sticky = e);
  return 0;
}

int glfsx_writer_reserve(glfsx_writer *w, void **buf, uint64_t *cap) {
  if (!w || !buf || !cap) return fail(GLFSX_E_ARG, "null argument");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (int e = slot_to_host(w)) return call.done(w->sticky = e);
  WSlot &sl = w->slot[w->cur];
  const uint64_t used = w->full * w->bs + w->partial;
  const uint64_t room = w->batch_blocks * w->bs;
  if (int e = pin_grow(sl.h_in, room, used)) return call.done(w->sticky = e);
  *buf = sl.h_in.u8() + used;
  *cap = room - used;  // >= 1: a full batch is submitted as soon as it fills
  w->reserved = room - used;
  return 0;
}

int glfsx_writer_commit(glfsx_writer *w, uint64_t n) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (n > w->reserved)
    return call.done(fail(GLFSX_E_ARG, "commit of %llu bytes, %llu reserved",
                          (unsigned long long)n, (unsigned long long)w->reserved));
  w->reserved = 0;
  const uint64_t used = w->full * w->bs + w->partial + n;
  w->full = used / w->bs;
  w->partial = used % w->bs;
  if (w->full == w->batch_blocks)
    if (int e = submit(w)) return call.done(w->sticky = e);
  if (w->strict && n)
    if (int e = drain_strict(w)) return call.done(w->sticky = e);
  return 0;
}

namespace {
// Reader threads per batch of glfsx_writer_read_at (GLFSX_READ_THREADS;
// capped by the copy pool: the GPU box's share is 16 cores).
unsigned read_threads() {
  static const unsigned v = [] {
    const char *e = getenv("GLFSX_READ_THREADS");
    return e ? std::max(1u, unsigned(strtoul(e, nullptr, 10))) : 16u;
  }();
  return v;
}

int64_t pread_fn(void *ctx, void *buf, uint64_t len, uint64_t off) {
  const int fd = int(reinterpret_cast<intptr_t>(ctx));
  for (;;) {
    const ssize_t r = pread(fd, buf, size_t(std::min<uint64_t>(len, 1ull << 30)), off_t(off));
    if (r >= 0) return r;
    if (errno != EINTR) return -int64_t(errno);
  }
}
}  // namespace

int glfsx_writer_read_at(glfsx_writer *w, glfsx_read_at_fn read_at, void *ctx,
                         uint64_t offset, uint64_t n, uint64_t *got) {
  if (got) *got = 0;
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  if (!read_at) return fail(GLFSX_E_ARG, "null reader");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (w->reserved) return call.done(fail(GLFSX_E_ARG, "staging lent out by glfsx_writer_reserve"));
  uint64_t total = 0;
  int rc = 0;
  while (total < n) {
    if (int e = slot_to_host(w)) return call.done(w->sticky = e);
    WSlot &sl = w->slot[w->cur];  // free: submit completed it before moving on
    const uint64_t used = w->full * w->bs + w->partial;
    const uint64_t room = w->batch_blocks * w->bs;
    if (int e = pin_grow(sl.h_in, room, used)) return call.done(w->sticky = e);
    const uint64_t want = std::min(room - used, n - total);
    const int64_t r = par_read_at(read_at, ctx, sl.h_in.u8() + used, want, offset + total,
                                  read_threads(), w->lanes[sl.lane].dev);
    if (r < 0) {
      rc = fail(GLFSX_E_IO, "read of %llu bytes at input offset %llu failed (%lld)",
                (unsigned long long)want, (unsigned long long)(offset + total), (long long)r);
      break;
    }
    total += uint64_t(r);
    w->full = (used + uint64_t(r)) / w->bs;
    w->partial = (used + uint64_t(r)) % w->bs;
    if (w->full == w->batch_blocks)
      if (int e = submit(w)) return call.done(w->sticky = e);
    if (uint64_t(r) < want) break;  // the end of the input
  }
  if (got) *got = total;
  if (w->strict && total)
    if (int e = drain_strict(w)) return call.done(w->sticky = e);
  return call.done(rc);
}

int glfsx_writer_read_fd(glfsx_writer *w, int fd, uint64_t offset, uint64_t n,
                         uint64_t *got) {
  if (fd < 0) {
    if (got) *got = 0;
    return fail(GLFSX_E_ARG, "bad file descriptor %d", fd);
  }
  return glfsx_writer_read_at(w, pread_fn, reinterpret_cast<void *>(intptr_t(fd)), offset, n,
                              got);
}

int glfsx_writer_copy(glfsx_writer *w, const void *data, uint64_t n, uint64_t piece) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  if (piece == 0) return fail(GLFSX_E_ARG, "piece of 0 bytes");
  const uint8_t *p = static_cast<const uint8_t *>(data);
  for (uint64_t off = 0; off < n; off += piece)
    if (int e = glfsx_writer_write(w, p + off, std::min(piece, n - off))) return e;
  return 0;
}

int glfsx_writer_flush(glfsx_writer *w) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (int e = drain(w)) return call.done(w->sticky = e);
  return 0;
}

int glfsx_writer_write_device(glfsx_writer *w, const void *d_data, size_t n,
                              void *stream) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (n && !d_data) return call.done(fail(GLFSX_E_ARG, "null data"));
  if (n == 0) return 0;
  if (w->lanes.size() != 1)
    return call.done(fail(GLFSX_E_UNSUPPORTED, "device input needs a one-device writer"));
  hipStream_t cs = static_cast<hipStream_t>(stream);
  auto go = [&]() -> int {
    if (!w->ev_in) {
      HIP_TRY(hipEventCreateWithFlags(&w->ev_in, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&w->ev_out, hipEventDisableTiming));
    }
    if (cs) {  // the bytes are ready once the caller's stream gets here
      HIP_TRY(hipEventRecord(w->ev_in, cs));
      HIP_TRY(hipStreamWaitEvent(w->s_up, w->ev_in, 0));
    }
    if (int e = write_dev(w, static_cast<const uint8_t *>(d_data), n)) return e;
    // the caller may reuse d_data once its stream passes this point
    HIP_TRY(hipEventRecord(w->ev_out, w->s_up));
    if (cs)
      HIP_TRY(hipStreamWaitEvent(cs, w->ev_out, 0));
    else
      HIP_TRY(hipEventSynchronize(w->ev_out));
    if (w->strict)
      if (int e = drain(w)) return e;
    return 0;
  };
  if (int e = go()) return call.done(w->sticky = e);
  return 0;
}

int glfsx_writer_write_ctext_blocks(glfsx_writer *w, const void *const *blocks,
                                    uint64_t nblocks, uint64_t total, uint64_t block_size,
                                    const uint8_t *refs) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  if (total == 0) return 0;
  if (!blocks || !refs) return call.done(fail(GLFSX_E_ARG, "null argument"));
  if (w->lanes.size() != 1)
    return call.done(fail(GLFSX_E_UNSUPPORTED, "device input needs a one-device writer"));
  if (block_size == 0 || block_size % 64)
    return call.done(fail(GLFSX_E_UNSUPPORTED, "decrypt needs block_size %% 64 == 0"));
  const uint64_t nb = (total + block_size - 1) / block_size;
  if (nblocks != nb)
    return call.done(fail(GLFSX_E_ARG, "%llu blocks given, %llu bytes need %llu",
                          (unsigned long long)nblocks, (unsigned long long)total,
                          (unsigned long long)nb));
  auto go = [&]() -> int {
    if (!w->ev_in) {
      HIP_TRY(hipEventCreateWithFlags(&w->ev_in, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&w->ev_out, hipEventDisableTiming));
    }
    if (!w->has_cx) {
      std::lock_guard<std::mutex> lk(g_pool_mu);
      for (size_t i = g_ctext_pool.size(); i-- > 0;)
        if (g_ctext_pool[i].dev == w->dev) {
          w->cx = g_ctext_pool[i];
          g_ctext_pool.erase(g_ctext_pool.begin() + i);
          break;
        }
      w->cx.dev = w->dev;
      w->has_cx = true;
    }
    CtextBuf &X = w->cx;
    for (hipEvent_t &ev : X.ev)
      if (!ev) HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    const uint64_t slab = std::max<uint64_t>(1, (64ull << 20) / block_size);
    for (PinBuf &hb : X.h)
      if (int e = hb.ensure(slab * block_size + 64 * slab)) return e;
    if (int e = X.d_ctx.ensure(slab * block_size + 64)) return e;
    if (int e = X.d_ptx.ensure(slab * block_size + 64)) return e;
    if (int e = X.d_rfx.ensure(64 * slab)) return e;
    // Three stages overlap: the copy threads gather slab i + 1 from the
    // store's memory into host buffer (i + 1) & 1 while this thread uploads
    // slab i, decrypts it into the Writer's staging and hands it on (the
    // Writer's own pipeline hashes it and brings the ctext back); buffer
    // (i + 1) & 1 is gathered into once slab i - 1's upload from it is done.
    // Uploads, decrypts and the Writer's copies are in order on s_up (the
    // device temporaries are reused in stream order).  A -DGLFSX_CONCAT_TRACE=1
    // build (tools/build_variant.sh) prints each slab's host timeline to
    // stderr.
    const int dev = w->lanes[0].dev;
    const uint64_t ns = (nb + slab - 1) / slab;
    std::atomic<int> left[2];
    left[0].store(0);
    left[1].store(0);
    struct Settle {  // no gather may still write a buffer, or read the
      std::atomic<int> *l;  // caller's blocks, once this call returns
      ~Settle() {
        gather_wait(&l[0]);
        gather_wait(&l[1]);
      }
    } settle{left};
#if GLFSX_CONCAT_TRACE
    constexpr bool trace = true;
#else
    constexpr bool trace = false;
#endif
    const auto tz = std::chrono::steady_clock::now();
    auto us = [&] {
      return double(std::chrono::duration_cast<std::chrono::nanoseconds>(
                        std::chrono::steady_clock::now() - tz).count()) * 1e-3;
    };
    std::vector<double> tr;
    auto start = [&](uint64_t i) {
      const uint64_t b0 = i * slab, k = std::min(slab, nb - b0);
      const uint64_t bytes = std::min<uint64_t>(k * block_size, total - b0 * block_size);
      gather_start(&left[i & 1], X.h[i & 1].u8(), blocks + b0, k, block_size,
                   bytes - (k - 1) * block_size, dev);
    };
    start(0);
    for (uint64_t i = 0; i < ns; ++i) {
      const uint64_t b0 = i * slab, k = std::min(slab, nb - b0);
      const uint64_t bytes = std::min<uint64_t>(k * block_size, total - b0 * block_size);
      PinBuf &hb = X.h[i & 1];
      const double t_in = trace ? us() : 0;
      gather_wait(&left[i & 1]);
      const double t_gathered = trace ? us() : 0;
      memcpy(hb.u8() + bytes, refs + 64 * b0, 64 * k);
      HIP_TRY(hipMemcpyAsync(X.d_ctx.p, hb.p, bytes, hipMemcpyHostToDevice, w->s_up));
      HIP_TRY(hipMemcpyAsync(X.d_rfx.p, hb.u8() + bytes, 64 * k, hipMemcpyHostToDevice,
                             w->s_up));
      HIP_TRY(hipEventRecord(X.ev[i & 1], w->s_up));
      double t_next = t_gathered;
      if (i + 1 < ns) {
        if (i >= 1) HIP_TRY(hipEventSynchronize(X.ev[(i + 1) & 1]));
        t_next = trace ? us() : 0;
        start(i + 1);
      }
      HIP_TRY(launch_decrypt(X.d_ctx.u8(), X.d_ptx.u8(), k, block_size,
                             bytes - (k - 1) * block_size, X.d_rfx.u8(), w->s_up));
      if (int e = write_dev(w, X.d_ptx.u8(), bytes)) return e;
      if (trace) tr.insert(tr.end(), {t_in, t_gathered, t_next, us()});
    }
    if (trace) {
      for (size_t x = 0; x + 3 < tr.size(); x += 4)
        fprintf(stderr,
                "concat slab %zu: wait-gather %.1f..%.1f us, next gather from %.1f, "
                "handed on %.1f\n",
                x / 4, tr[x], tr[x + 1], tr[x + 2], tr[x + 3]);
    }
    HIP_TRY(hipStreamSynchronize(w->s_up));
    if (w->strict)
      if (int e = drain(w)) return e;
    return 0;
  };
  if (int e = go()) return call.done(w->sticky = e);
  return 0;
}

int glfsx_writer_write_ctext(glfsx_writer *w, const void *ctext, uint64_t total,
                             uint64_t block_size, const uint8_t *refs) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  if (total == 0 || !ctext || block_size == 0 || block_size % 64) {
    // (the same checks and errors; nothing to split into blocks)
    const void *one = ctext;
    return glfsx_writer_write_ctext_blocks(w, ctext ? &one : nullptr, 0, total, block_size,
                                           refs);
  }
  const uint64_t nb = (total + block_size - 1) / block_size;
  std::vector<const void *> blocks(nb);
  for (uint64_t j = 0; j < nb; ++j)
    blocks[j] = static_cast<const uint8_t *>(ctext) + j * block_size;
  return glfsx_writer_write_ctext_blocks(w, blocks.data(), nb, total, block_size, refs);
}

int glfsx_writer_set_strict(glfsx_writer *w, int strict) {
  if (!w) return fail(GLFSX_E_ARG, "null writer");
  w->strict = strict != 0;
  return 0;
}

const char *glfsx_writer_error(const glfsx_writer *w) {
  return w ? w->err.c_str() : "null writer";
}

int glfsx_writer_finish(glfsx_writer *w, glfsx_root *out) {
  if (!w || !out) return fail(GLFSX_E_ARG, "null argument");
  WriterCall call(w);
  if (w->sticky) return call.done(fail(w->sticky, "%s", w->err.c_str()));
  bool few = false;
  if (int e = post_few(w, true, &few)) return call.done(w->sticky = e);
  if (!few)
    if (int e = drain(w)) return call.done(w->sticky = e);
  if (w->partial) {  // blob.go:136-140: the tail block, never padded
    uint8_t ref[64];
    const WSlot &sl = w->slot[w->cur];
    if (int e = post_one(w, 0, w->salts.raw, sl.on_dev ? sl.d_in.u8() : sl.h_in.u8(),
                         w->partial, ref, sl.on_dev, &sl.h_in))
      return call.done(w->sticky = e);
    if (int e = add_ref(w, 0, ref)) return call.done(w->sticky = e);
    w->size += w->partial;
    w->partial = 0;
  }
  uint8_t root[64];
  if (int e = finish_indexes(w, root)) return call.done(w->sticky = e);
  memcpy(out->ref, root, 64);
  out->size = w->size;
  out->block_size = w->bs;
  return 0;
}

void glfsx_writer_free(glfsx_writer *w) {
  if (!w) return;
  (void)hipSetDevice(w->dev);
  // a writer that never submitted a batch nor took device input, and did
  // not fail, has nothing in flight (its single posts waited for themselves)
  if (w->seq || w->ev_in || w->sticky) {
    for (hipStream_t st : {w->s_up, w->ws, w->s_down})
      if (st) (void)hipStreamSynchronize(st);
    for (const WLane &L : w->lanes)
      if (L.own) {
        DevScope d(L.dev);
        for (hipStream_t st : {L.s_up, L.ws, L.s_down}) (void)hipStreamSynchronize(st);
      }
  }
  std::vector<hipStream_t> drop;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    for (auto &sl : w->slot) give_slot_locked(sl);
    for (WLane &L : w->lanes) give_streams_locked(L);
    if (g_one_pool.size() < 16) {
      g_one_pool.push_back(w->one);
    } else {
      OneBuf &o = w->one;
      for (void *p : {o.d_in.p, o.d_ct.p, o.d_ref.p})
        if (p) (void)hipFree(p);
      for (void *p : {o.h_ct.p, o.h_ref.p})
        if (p) (void)hipHostFree(p);
    }
    if (w->ws && g_stream_pool.size() < 64)
      g_stream_pool.push_back({w->dev, w->s_up, w->ws, w->s_down});
    else
      drop = {w->s_up, w->ws, w->s_down};
  }
  for (hipStream_t st : drop)
    if (st) {
      release_stream_scratch(st);
      (void)hipStreamDestroy(st);
    }
  for (hipEvent_t ev : {w->ev_in, w->ev_out})
    if (ev) (void)hipEventDestroy(ev);
  if (w->has_cx) {  // (its streams are drained above: ev_in is set)
    bool kept = false;
    {
      std::lock_guard<std::mutex> lk(g_pool_mu);
      if (g_ctext_pool.size() < 4) {
        g_ctext_pool.push_back(w->cx);
        kept = true;
      }
    }
    if (!kept) {
      for (hipEvent_t ev : w->cx.ev)
        if (ev) (void)hipEventDestroy(ev);
      for (PinBuf &b : w->cx.h)
        if (b.p) (void)hipHostFree(b.p);
      for (void *p : {w->cx.d_ctx.p, w->cx.d_ptx.p, w->cx.d_rfx.p})
        if (p) (void)hipFree(p);
    }
  }
  delete w;
}

namespace {
// glfsx_create of a blob of at most one block of <= kMaxMedLen bytes (a
// glfs.PostBlob of a small file, machine.go:64): its Writer would stage the
// bytes, post them as the tail block at Finish and return that block's ref
// as the root (blob.go:136-140, 190-193) -- or, for the empty blob, post
// the empty index node (blob.go:187-189).  The same single Post, without a
// Writer: the thread's pinned one-shot staging and one coalesced one-shot
// post (no writer pools, locks or streams per call).
int create_one_block(Ctx *c, uint64_t bs, const uint8_t *salt, const uint8_t *cid_key,
                     const void *data, uint64_t size, glfsx_post_fn post, void *post_ctx,
                     glfsx_root *out) {
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  if (int e = c->h_oin.ensure(size + 64)) return e;
  if (int e = c->h_oct.ensure(size + 64)) return e;
  if (int e = c->h_oref.ensure(64)) return e;
  if (size) par_memcpy(c->h_oin.u8(), static_cast<const uint8_t *>(data), size);
  OneReq r;
  r.d.src = c->h_oin.dptr();
  r.d.ctext = post ? c->h_oct.dptr() : nullptr;
  r.d.ref = c->h_oref.dptr();
  r.d.len = uint32_t(size);
  r.d.present = uint32_t(size);
  one_keys(r.d, size ? salts.raw : salts.index, cid_key);
  if (int e = one_post(c->dev, &r)) return e;
  memcpy(out->ref, c->h_oref.p, 64);
  out->size = size;
  out->block_size = bs;
  if (post) {
    const int rc = post(post_ctx, size ? 0 : 1, out->ref, c->h_oct.p, size);
    if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
  }
  return 0;
}
}  // namespace

int glfsx_create(uint64_t block_size, uint64_t store_max, const uint8_t *salt,
                 const uint8_t *cid_key, const void *data, uint64_t size,
                 glfsx_post_fn post, void *post_ctx, glfsx_root *out) {
  const uint64_t bs = block_size ? block_size : store_max;  // blob.go:86-89
  if (out && (size == 0 || data) && bs <= store_max && bs >= GLFSX_MIN_BLOCK_SIZE &&
      bs <= kMaxMsgLen && size <= bs && size <= kMaxMedLen) {
    Ctx *c;
    if (int e = ctx_get(&c)) return e;
    return create_one_block(c, bs, salt, cid_key, data, size, post, post_ctx, out);
  }
  int err = 0;
  glfsx_writer *w =
      glfsx_writer_new(block_size, store_max, salt, cid_key, post, post_ctx, &err);
  if (!w) return err;
  int e = glfsx_writer_write(w, data, size);
  if (!e) e = glfsx_writer_finish(w, out);
  glfsx_writer_free(w);
  return e;
}

namespace {
int create_device_impl(uint64_t block_size, const uint8_t *salt,
                       const uint8_t *cid_key, const void *d_data,
                       uint64_t size, void *d_ctext, glfsx_root *out,
                       uint64_t *n_posts, void *stream);
int shard_device_impl(uint64_t block_size, const uint8_t *salt,
                      const uint8_t *cid_key, const void *d_range,
                      uint64_t size, uint64_t first_block, uint64_t nb,
                      void *d_ctext, uint8_t *level1_out, void *stream);
int root_from_level1_impl(uint64_t block_size, const uint8_t *salt,
                          const uint8_t *cid_key, const uint8_t *level1,
                          uint64_t n1, uint64_t size, glfsx_root *out);
}  // namespace

int glfsx_create_device(uint64_t block_size, const uint8_t *salt,
                        const uint8_t *cid_key, const void *d_data,
                        uint64_t size, void *d_ctext, glfsx_root *out,
                        uint64_t *n_posts, void *stream) {
  return with_fused_retry([&] {
    return create_device_impl(block_size, salt, cid_key, d_data, size, d_ctext, out,
                              n_posts, stream);
  });
}

int glfsx_shard_device(uint64_t block_size, const uint8_t *salt,
                       const uint8_t *cid_key, const void *d_range,
                       uint64_t size, uint64_t first_block, uint64_t nb,
                       void *d_ctext, uint8_t *level1_out, void *stream) {
  return with_fused_retry([&] {
    return shard_device_impl(block_size, salt, cid_key, d_range, size, first_block, nb,
                             d_ctext, level1_out, stream);
  });
}

int glfsx_root_from_level1(uint64_t block_size, const uint8_t *salt,
                           const uint8_t *cid_key, const uint8_t *level1,
                           uint64_t n1, uint64_t size, glfsx_root *out) {
  return with_fused_retry([&] {
    return root_from_level1_impl(block_size, salt, cid_key, level1, n1, size, out);
  });
}

namespace {
// Persistent worker threads of glfsx_create_devices, one per (device,
// index): part k of a call runs on the worker of its device whose index
// counts the earlier parts on the same device.  A worker keeps its thread's
// context (stream, level buffers, scratch) across calls, so a call creates
// no streams or buffers once warm.  Calls are serialised (each takes every
// device it names).
struct PartWorker {
  int dev = 0;
  std::mutex mu;
  std::condition_variable cv;
  std::function<int()> fn;
  bool pending = false, done = false;
  int rc = 0;
  std::string err;
  float ms = -1.f;  // the last part's GPU time (HIP events on its stream)
  hipEvent_t ev[2] = {nullptr, nullptr};
  void loop() {
    tls_dev = dev;
    for (;;) {
      std::function<int()> f;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return pending; });
        f = std::move(fn);
        pending = false;
      }
      // the part's work runs on this thread's context stream (the calls get
      // a null stream): events around it time the device's share of the call
      Ctx *c = nullptr;
      bool timed = ctx_get(&c) == 0;
      if (timed && !ev[0])
        timed = hipEventCreate(&ev[0]) == hipSuccess && hipEventCreate(&ev[1]) == hipSuccess;
      if (timed) timed = hipEventRecord(ev[0], c->stream) == hipSuccess;
      const int r = f();
      std::string e = r ? tls_err : std::string();
      float t = -1.f;
      if (timed && hipEventRecord(ev[1], c->stream) == hipSuccess &&
          hipEventSynchronize(ev[1]) == hipSuccess)
        (void)hipEventElapsedTime(&t, ev[0], ev[1]);
      {
        std::lock_guard<std::mutex> lk(mu);
        rc = r;
        err = std::move(e);
        ms = t;
        done = true;
      }
      cv.notify_all();
    }
  }
  void submit(std::function<int()> f) {
    std::lock_guard<std::mutex> lk(mu);
    fn = std::move(f);
    done = false;
    pending = true;
    cv.notify_all();
  }
  int wait(std::string *e, float *t) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return done; });
    *e = err;
    *t = ms;
    return rc;
  }
};
std::mutex g_parts_mu;  // one glfsx_create_devices call at a time
std::vector<std::pair<std::pair<int, int>, PartWorker *>> g_part_workers;
// per part of the last glfsx_create_devices call: data-block pass GPU ms,
// then the levels above (on devs[0]) as one more entry
std::vector<float> g_parts_ms;

PartWorker *part_worker(int dev, int idx) {
  for (auto &x : g_part_workers)
    if (x.first == std::make_pair(dev, idx)) return x.second;
  auto *pw = new PartWorker();  // lives for the process, like its thread
  pw->dev = dev;
  std::thread([pw] { pw->loop(); }).detach();
  g_part_workers.push_back({{dev, idx}, pw});
  return pw;
}

// Run fns[k] on the worker of (devs[k], its index); the first failure (in
// part order) is returned with its text.
int run_parts(const int *devs, std::vector<std::function<int()>> &fns) {
  std::vector<PartWorker *> ws(fns.size());
  for (size_t k = 0; k < fns.size(); ++k) {
    int idx = 0;
    for (size_t i = 0; i < k; ++i) idx += devs[i] == devs[k];
    ws[k] = part_worker(devs[k], idx);
  }
  for (size_t k = 0; k < fns.size(); ++k) ws[k]->submit(std::move(fns[k]));
  int first = 0;
  std::string msg;
  for (size_t k = 0; k < fns.size(); ++k) {
    std::string e;
    float t = -1.f;
    const int rc = ws[k]->wait(&e, &t);
    g_parts_ms.push_back(t);
    if (rc && !first) {
      first = rc;
      msg = "part " + std::to_string(k) + " (device " + std::to_string(devs[k]) + "): " + e;
    }
  }
  return first ? fail(first, "%s", msg.c_str()) : 0;
}
}  // namespace

int glfsx_create_devices_ms(float *ms, int cap) {
  std::lock_guard<std::mutex> lk(g_parts_mu);
  const int n = int(g_parts_ms.size());
  for (int k = 0; k < std::min(n, cap); ++k) ms[k] = g_parts_ms[k];
  return n;
}

// Create over a blob whose bytes lie on several devices (in one
// process): part k = bytes of blocks [first_k, first_k + nb_k) on devs[k];
// each device posts its data blocks and level-1 nodes concurrently, the
// level-1 refs are gathered on the host and levels >= 2 posted on devs[0].
int glfsx_create_devices(uint64_t block_size, const uint8_t *salt,
                         const uint8_t *cid_key, int nparts, const int *devs,
                         const void *const *d_parts, const uint64_t *part_sizes,
                         void *const *d_ctexts, uint8_t *level1_out,
                         glfsx_root *out, uint64_t *n_posts) {
  if (!out || !devs || !d_parts || !part_sizes || nparts < 1 || nparts > 1024)
    return fail(GLFSX_E_ARG, "bad arguments");
  if (int e = check_block_size(block_size)) return e;
  const int ndev = glfsx_device_count();
  const uint64_t bs = block_size, bf = bs / 64, span = bs * bf;
  uint64_t size = 0;
  for (int k = 0; k < nparts; ++k) {
    if (devs[k] < 0 || devs[k] >= ndev)
      return fail(GLFSX_E_ARG, "device %d out of range (%d devices)", devs[k], ndev);
    if (part_sizes[k] && !d_parts[k]) return fail(GLFSX_E_ARG, "null part %d", k);
    if (k + 1 < nparts && (part_sizes[k] == 0 || part_sizes[k] % span))
      return fail(GLFSX_E_ARG,
                  "part %d: %llu bytes; every part but the last must be a positive "
                  "multiple of block_size * block_size/64 = %llu (whole level-1 nodes)",
                  k, (unsigned long long)part_sizes[k], (unsigned long long)span);
    size += part_sizes[k];
  }
  if (nparts > 1 && part_sizes[nparts - 1] == 0)
    return fail(GLFSX_E_ARG, "the last part is empty");
  std::lock_guard<std::mutex> lk(g_parts_mu);
  g_parts_ms.clear();
  const uint64_t n0 = (size + bs - 1) / bs;
  if (nparts == 1 || n0 <= bf) {  // one part: Create on its device
    std::vector<std::function<int()>> fns{[&] {
      return glfsx_create_device(bs, salt, cid_key, d_parts[0], size,
                                 d_ctexts ? d_ctexts[0] : nullptr, out, n_posts, nullptr);
    }};
    return run_parts(devs, fns);  // level1_out is not written
  }
  const uint64_t n1 = (n0 + bf - 1) / bf;
  std::vector<uint8_t> lvl1(n1 * 64);
  std::vector<std::function<int()>> fns;
  uint64_t first = 0;
  for (int k = 0; k < nparts; ++k) {
    const uint64_t nb = (part_sizes[k] + bs - 1) / bs;
    uint8_t *dst = lvl1.data() + (first / bf) * 64;
    void *ct = d_ctexts ? d_ctexts[k] : nullptr;
    const void *src = d_parts[k];
    fns.push_back([=] {
      return glfsx_shard_device(bs, salt, cid_key, src, size, first, nb, ct, dst, nullptr);
    });
    first += nb;
  }
  if (int e = run_parts(devs, fns)) return e;
  std::vector<std::function<int()>> top{[&] {
    return glfsx_root_from_level1(bs, salt, cid_key, lvl1.data(), n1, size, out);
  }};
  if (int e = run_parts(devs, top)) return e;
  if (level1_out) memcpy(level1_out, lvl1.data(), lvl1.size());
  if (n_posts) {
    uint64_t posts = n0 + n1;
    for (uint64_t r = n1; r > 1;) {
      r = (r + bf - 1) / bf;
      posts += r;
    }
    *n_posts = posts;
  }
  return 0;
}

namespace {
int create_device_impl(uint64_t block_size, const uint8_t *salt,
                       const uint8_t *cid_key, const void *d_data,
                       uint64_t size, void *d_ctext, glfsx_root *out,
                       uint64_t *n_posts, void *stream) {
  if (!out || (size && !d_data)) return fail(GLFSX_E_ARG, "null argument");
  if (int e = check_block_size(block_size)) return e;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  hipStream_t s = pick_stream(c, stream);
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  const uint64_t bs = block_size, bf = bs / 64;
  const uint64_t n0 = (size + bs - 1) / bs;
  uint64_t posts = 0;
  if (n0 <= 1) {
    // n0 == 0: post(indexSalt, nil) (blob.go:187-189); n0 == 1: the only
    // data block's ref is the root (blob.go:190-193).
    if (int e = c->d_refs.ensure(64)) return e;
    if (int e = c->d_small.ensure(64)) return e;
    PostJob j{};
    j.src = n0 ? static_cast<const uint8_t *>(d_data) : c->d_small.u8();
    j.ctext = n0 ? static_cast<uint8_t *>(d_ctext) : nullptr;
    j.stride = 0;
    j.msg_len = size;
    j.last_len = size;
    j.n = 1;
    if (int e = c->h_root.ensure(64)) return e;
    j.out = RefLayout{c->h_root.dptr(), ~0ull, 0};  // written straight to the host
    words_from_key(j.salt, n0 ? salts.raw : salts.index);
    cid_words(j, cid_key);
    HIP_TRY(launch_post(j, s, tls_fused));
    HIP_TRY(stream_wait(s));
    memcpy(out->ref, c->h_root.p, 64);
    posts = 1;
  } else {
    const uint64_t n1 = (n0 + bf - 1) / bf;
    if (int e = level_prepare(c->d_lvl_a, n0, n1, bs, s)) return e;
    PostJob j{};
    j.src = static_cast<const uint8_t *>(d_data);
    j.ctext = static_cast<uint8_t *>(d_ctext);
    j.stride = bs;
    j.msg_len = bs;
    j.last_len = size - (n0 - 1) * bs;
    j.n = n0;
    j.out = RefLayout{c->d_lvl_a.u8(), bf, bs};
    words_from_key(j.salt, salts.raw);
    cid_words(j, cid_key);
    HIP_TRY(launch_post(j, s, tls_fused));
    posts = n0;
    if (int e = build_up(c, s, salts, cid_key, bs, c->d_lvl_a.u8(), n1,
                         &c->d_lvl_b, out->ref, &posts))
      return e;
  }
  out->size = size;
  out->block_size = bs;
  if (n_posts) *n_posts = posts;
  return 0;
}

int shard_device_impl(uint64_t block_size, const uint8_t *salt,
                      const uint8_t *cid_key, const void *d_range,
                      uint64_t size, uint64_t first_block, uint64_t nb,
                      void *d_ctext, uint8_t *level1_out, void *stream) {
  if (!level1_out || (nb && !d_range)) return fail(GLFSX_E_ARG, "null argument");
  if (int e = check_block_size(block_size)) return e;
  const uint64_t bs = block_size, bf = bs / 64;
  const uint64_t n0 = (size + bs - 1) / bs;
  if (first_block % bf)
    return fail(GLFSX_E_ARG, "shard start %llu not a multiple of bf=%llu",
                (unsigned long long)first_block, (unsigned long long)bf);
  if (nb == 0 || first_block + nb > n0 || n0 < 2)
    return fail(GLFSX_E_ARG, "bad shard range");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  hipStream_t s = pick_stream(c, stream);
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  const bool has_last = first_block + nb == n0;
  const uint64_t m = (nb + bf - 1) / bf;
  if (int e = level_prepare(c->d_lvl_a, nb, m, bs, s)) return e;
  if (int e = c->d_ct.ensure(m * bs)) return e;
  if (int e = c->d_refs.ensure(m * 64)) return e;
  PostJob j{};
  j.src = static_cast<const uint8_t *>(d_range);
  j.ctext = static_cast<uint8_t *>(d_ctext);
  j.stride = bs;
  j.msg_len = bs;
  j.last_len = has_last ? size - (n0 - 1) * bs : bs;
  j.n = nb;
  j.out = RefLayout{c->d_lvl_a.u8(), bf, bs};
  words_from_key(j.salt, salts.raw);
  cid_words(j, cid_key);
  HIP_TRY(launch_post(j, s, tls_fused));
  if (int e = post_level(c, s, salts.index, cid_key, c->d_lvl_a.u8(), m, bs,
                         c->d_ct.u8(), RefLayout{c->d_refs.u8(), ~0ull, 0}))
    return e;
  HIP_TRY(hipMemcpyAsync(level1_out, c->d_refs.p, m * 64, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  return fused_check(s);
}

int root_from_level1_impl(uint64_t block_size, const uint8_t *salt,
                          const uint8_t *cid_key, const uint8_t *level1,
                          uint64_t n1, uint64_t size, glfsx_root *out) {
  if (!level1 || !out || n1 == 0) return fail(GLFSX_E_ARG, "null argument");
  if (int e = check_block_size(block_size)) return e;
  const uint64_t bs = block_size, bf = bs / 64;
  const uint64_t n0 = (size + bs - 1) / bs;
  if (n0 < 2 || (n0 + bf - 1) / bf != n1)
    return fail(GLFSX_E_ARG, "level-1 count %llu does not match size",
                (unsigned long long)n1);
  out->size = size;
  out->block_size = bs;
  if (n1 == 1) {
    memcpy(out->ref, level1, 64);
    return 0;
  }
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  const uint64_t m = (n1 + bf - 1) / bf;
  if (int e = level_prepare(c->d_lvl_a, n1, m, bs, c->stream)) return e;
  // scatter the gathered refs into zero-padded nodes (index.go:33-38)
  for (uint64_t k = 0; k < m; ++k) {
    const uint64_t cnt = std::min(bf, n1 - k * bf);
    HIP_TRY(hipMemcpyAsync(c->d_lvl_a.u8() + k * bs, level1 + k * bf * 64,
                           cnt * 64, hipMemcpyHostToDevice, c->stream));
  }
  uint64_t posts = 0;
  return build_up(c, c->stream, salts, cid_key, bs, c->d_lvl_a.u8(), m,
                  &c->d_lvl_b, out->ref, &posts);
}
}  // namespace


int glfsx_chacha20_xor(const uint8_t dek[32], const void *src, void *dst,
                       uint64_t n) {
  if (!dek || (n && (!src || !dst))) return fail(GLFSX_E_ARG, "null argument");
  if (n == 0) return 0;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  if (int e = c->d_in.ensure(n)) return e;
  if (int e = c->d_ct.ensure(n)) return e;
  HIP_TRY(hipMemcpyAsync(c->d_in.p, src, n, hipMemcpyHostToDevice, c->stream));
  uint32_t k[8];
  words_from_key(k, dek);
  HIP_TRY(launch_chacha_xor(k, c->d_in.u8(), c->d_ct.u8(), n, c->stream));
  HIP_TRY(hipMemcpyAsync(dst, c->d_ct.p, n, hipMemcpyDeviceToHost, c->stream));
  HIP_TRY(stream_wait(c->stream));
  return 0;
}

int glfsx_post_blobs_device(uint64_t block_size, const uint8_t *salt,
                            const uint8_t *cid_key, const void *d_data,
                            const uint64_t *d_offsets, const uint64_t *d_lengths,
                            uint64_t n, uint64_t max_len, void *d_ctext,
                            void *d_roots, void *stream) {
  if (n == 0) return 0;
  if (!d_data || !d_offsets || !d_lengths || !d_roots)
    return fail(GLFSX_E_ARG, "null argument");
  if (int e = check_block_size(block_size)) return e;
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  hipStream_t s = pick_stream(c, stream);
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  SmallJob j{};
  j.src = static_cast<const uint8_t *>(d_data);
  j.ctext = static_cast<uint8_t *>(d_ctext);
  j.offs = d_offsets;
  j.lens = d_lengths;
  j.n = n;
  j.max_len = max_len;
  j.refs = static_cast<uint8_t *>(d_roots);
  words_from_key(j.raw_salt, salts.raw);
  words_from_key(j.index_salt, salts.index);
  if (cid_key) {
    words_from_key(j.cid_key, cid_key);
    j.cid_keyed = true;
  } else {
    blake3_iv_words(j.cid_key);
  }
  // blobs of <= min(16 KiB, block_size): one lane each (k_small skips the
  // others; a blob longer than its block size has several blocks)
  const uint64_t small_max = small_max_for(block_size);
  j.small_max = small_max;
  HIP_TRY(launch_post_small(j, s));
  if (max_len <= small_max) return 0;
  // larger blobs (the caller said some may exceed 16 KiB): find them, then
  // one post each (<= one block: the root is post(rawSalt, blob),
  // blob.go:190-193) or a whole Create (several blocks)
  std::vector<uint64_t> offs(n), lens(n);
  HIP_TRY(hipMemcpyAsync(offs.data(), d_offsets, 8 * n, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(lens.data(), d_lengths, 8 * n, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  for (uint64_t i = 0; i < n; ++i) {
    if (lens[i] <= small_max) continue;
    const uint8_t *src = static_cast<const uint8_t *>(d_data) + offs[i];
    uint8_t *ct = d_ctext ? static_cast<uint8_t *>(d_ctext) + offs[i] : nullptr;
    uint8_t *ref = static_cast<uint8_t *>(d_roots) + 64 * i;
    if (lens[i] <= block_size) {
      PostJob pj{};
      pj.src = src;
      pj.ctext = ct;
      pj.stride = 0;
      pj.msg_len = lens[i];
      pj.last_len = lens[i];
      pj.n = 1;
      pj.out = RefLayout{ref, ~0ull, 0};
      words_from_key(pj.salt, salts.raw);
      cid_words(pj, cid_key);
      HIP_TRY(launch_post(pj, s, tls_fused));
    } else {
      glfsx_root r;
      if (int e = glfsx_create_device(block_size, salt, cid_key, src, lens[i], ct, &r,
                                      nullptr, s))
        return e;
      HIP_TRY(hipMemcpyAsync(ref, r.ref, 64, hipMemcpyHostToDevice, s));
      HIP_TRY(stream_wait(s));  // r lives on this frame
    }
  }
  return 0;
}

namespace {
// A store sink that keeps every Post (large blobs of glfsx_post_blobs are
// created first and their Posts replayed in call order).
struct CapturedPost {
  int kind;
  uint8_t ref[64];
  std::vector<uint8_t> ctext;
};
int capture_post(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                 uint64_t len) {
  auto *v = static_cast<std::vector<CapturedPost> *>(ctx);
  v->emplace_back();
  CapturedPost &p = v->back();
  p.kind = kind;
  memcpy(p.ref, ref, 64);
  p.ctext.assign(static_cast<const uint8_t *>(ctext),
                 static_cast<const uint8_t *>(ctext) + len);
  return 0;
}
}  // namespace

namespace {
// glfsx_post_blobs' small blobs (<= small_max bytes), pipelined from host
// memory: the blobs are taken in index order in groups whose bytes fit a
// 64 MiB slot; each group's bytes are packed into pinned staging (runs of
// blobs contiguous in `data` copied at once, by the copy pool), uploaded on
// one stream, hashed one lane per blob (launch_post_small) on the context's
// stream and their roots and ctext downloaded on a third, while the next
// group is packed -- three slots in flight, so the host copy, both PCIe
// directions and the kernels overlap.  A group's Posts are delivered when
// its slot is reused or at the end, in blob order, the larger blobs' captured
// Posts in their places: exactly n sequential PostBlob calls' order.
constexpr uint64_t kGroupBytes = 64ull << 20;

int complete_group(Ctx::BlobSlot &g, const uint64_t *lengths, uint64_t small_max,
                   const std::vector<std::vector<CapturedPost>> &big, glfsx_post_fn post,
                   void *post_ctx, uint8_t *roots_out) {
  if (!g.busy) return 0;
  HIP_TRY(hipEventSynchronize(g.done));
  g.busy = false;
  for (uint64_t i = g.i0; i < g.i1; ++i) {
    if (lengths[i] <= small_max) {
      const uint8_t *ref = g.h_refs.u8() + 64 * (i - g.i0);
      memcpy(roots_out + 64 * i, ref, 64);
      if (post) {
        // a small blob's single Post: a data block, or the empty blob's
        // index node (blob.go:187-189)
        int rc = post(post_ctx, lengths[i] ? 0 : 1, roots_out + 64 * i,
                      g.h_ct.u8() + g.loff[i - g.i0], lengths[i]);
        if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
      }
    } else if (post) {
      for (const CapturedPost &p : big[i]) {
        int rc = post(post_ctx, p.kind, p.ref, p.ctext.data(), p.ctext.size());
        if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
      }
    }
  }
  return 0;
}

int post_small_groups(Ctx *c, uint64_t bs, const uint8_t *salt, const uint8_t *cid_key,
                      const uint8_t *data, const uint64_t *offsets, const uint64_t *lengths,
                      uint64_t n, uint64_t small_max,
                      const std::vector<std::vector<CapturedPost>> &big, glfsx_post_fn post,
                      void *post_ctx, uint8_t *roots_out) {
  Salts salts;
  if (int e = derive_salts(c, salt, &salts)) return e;
  if (!c->s_up) HIP_TRY(hipStreamCreateWithFlags(&c->s_up, hipStreamNonBlocking));
  if (!c->s_down) HIP_TRY(hipStreamCreateWithFlags(&c->s_down, hipStreamNonBlocking));
  for (auto &g : c->bslot)
    if (!g.done) {
      HIP_TRY(hipEventCreateWithFlags(&g.done, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&g.up, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&g.hashed, hipEventDisableTiming));
    }
  // on any failure, nothing may still be writing the slots' pinned staging
  auto drain = [&] {
    for (hipStream_t st : {c->s_up, c->stream, c->s_down}) (void)hipStreamSynchronize(st);
    for (auto &g : c->bslot) g.busy = false;
  };
  int k = 0;
  uint64_t i = 0;
  while (i < n) {
    Ctx::BlobSlot &g = c->bslot[k];
    k = (k + 1) % 3;
    if (int e = complete_group(g, lengths, small_max, big, post, post_ctx, roots_out)) {
      drain();
      return e;
    }
    // the group: blobs [i, i1) whose small bytes fit kGroupBytes (a single
    // blob always fits: small blobs are <= 16 KiB)
    uint64_t i1 = i, bytes = 0, max_len = 0;
    while (i1 < n) {
      const uint64_t len = lengths[i1] <= small_max ? lengths[i1] : 0;
      if (i1 > i && bytes + len > kGroupBytes) break;
      bytes += len;
      max_len = std::max(max_len, len);
      ++i1;
    }
    const uint64_t m = i1 - i;
    auto run = [&]() -> int {
      if (int e = g.h_in.ensure(bytes + 64)) return e;
      if (int e = g.d_in.ensure(bytes + 64)) return e;
      if (int e = g.d_ct.ensure(bytes + 64)) return e;
      if (post)
        if (int e = g.h_ct.ensure(bytes + 64)) return e;
      if (int e = g.h_meta.ensure(16 * m)) return e;
      if (int e = g.d_meta.ensure(16 * m)) return e;
      if (int e = g.h_refs.ensure(64 * m)) return e;
      if (int e = g.d_refs.ensure(64 * m)) return e;
      g.loff.assign(m, 0);
      uint64_t *lo = reinterpret_cast<uint64_t *>(g.h_meta.p), *ll = lo + m;
      // pack, copying each run of blobs that are contiguous in `data` at once
      uint64_t o = 0, run_src = 0, run_dst = 0, run_len = 0;
      for (uint64_t j = 0; j < m; ++j) {
        const uint64_t idx = i + j, len = lengths[idx];
        const bool small = len <= small_max;
        lo[j] = small ? o : 0;
        ll[j] = small ? len : kMaxSmallLen + 1;  // skipped by k_small
        g.loff[j] = lo[j];
        if (!small || len == 0) continue;
        if (run_len && offsets[idx] == run_src + run_len && o == run_dst + run_len) {
          run_len += len;
        } else {
          if (run_len) par_memcpy(g.h_in.u8() + run_dst, data + run_src, run_len);
          run_src = offsets[idx];
          run_dst = o;
          run_len = len;
        }
        o += len;
      }
      if (run_len) par_memcpy(g.h_in.u8() + run_dst, data + run_src, run_len);
      if (bytes) HIP_TRY(hipMemcpyAsync(g.d_in.p, g.h_in.p, bytes, hipMemcpyHostToDevice, c->s_up));
      HIP_TRY(hipMemcpyAsync(g.d_meta.p, g.h_meta.p, 16 * m, hipMemcpyHostToDevice, c->s_up));
      HIP_TRY(hipEventRecord(g.up, c->s_up));
      HIP_TRY(hipStreamWaitEvent(c->stream, g.up, 0));
      SmallJob j{};
      j.src = g.d_in.u8();
      j.ctext = g.d_ct.u8();
      j.offs = reinterpret_cast<const uint64_t *>(g.d_meta.p);
      j.lens = j.offs + m;
      j.n = m;
      j.max_len = max_len;
      j.small_max = small_max;
      j.refs = g.d_refs.u8();
      words_from_key(j.raw_salt, salts.raw);
      words_from_key(j.index_salt, salts.index);
      if (cid_key) {
        words_from_key(j.cid_key, cid_key);
        j.cid_keyed = true;
      } else {
        blake3_iv_words(j.cid_key);
      }
      HIP_TRY(launch_post_small(j, c->stream));
      HIP_TRY(hipEventRecord(g.hashed, c->stream));
      HIP_TRY(hipStreamWaitEvent(c->s_down, g.hashed, 0));
      HIP_TRY(hipMemcpyAsync(g.h_refs.p, g.d_refs.p, 64 * m, hipMemcpyDeviceToHost, c->s_down));
      if (post && bytes)
        HIP_TRY(hipMemcpyAsync(g.h_ct.p, g.d_ct.p, bytes, hipMemcpyDeviceToHost, c->s_down));
      HIP_TRY(hipEventRecord(g.done, c->s_down));
      return 0;
    };
    if (int e = run()) {
      drain();
      return e;
    }
    g.i0 = i;
    g.i1 = i1;
    g.busy = true;
    i = i1;
  }
  // the rest, oldest first
  for (int r = 0; r < 3; ++r) {
    Ctx::BlobSlot &g = c->bslot[(k + r) % 3];
    if (int e = complete_group(g, lengths, small_max, big, post, post_ctx, roots_out)) {
      drain();
      return e;
    }
  }
  return 0;
}
}  // namespace

int glfsx_post_blobs(uint64_t block_size, uint64_t store_max, const uint8_t *salt,
                     const uint8_t *cid_key, const void *data,
                     const uint64_t *offsets, const uint64_t *lengths, uint64_t n,
                     glfsx_post_fn post, void *post_ctx, uint8_t *roots_out) {
  if (n == 0) return 0;
  if (!data || !offsets || !lengths || !roots_out)
    return fail(GLFSX_E_ARG, "null argument");
  const uint64_t bs = block_size ? block_size : store_max;  // blob.go:86-89
  if (bs > store_max)
    return fail(GLFSX_E_BLOCKSIZE_GT_MAX, "blockSize %llu > maxSize %llu",
                (unsigned long long)bs, (unsigned long long)store_max);
  if (int e = check_block_size(bs)) return e;
  // small blobs go through the pipelined device batches (post_small_groups);
  // single-block blobs of up to kMaxMedLen as one-shot posts, kMedBatchBytes
  // at a time (their root is the block's ref, blob.go:190-193); larger ones
  // Created one by one through the Writer.  The Posts of the latter two are
  // captured and delivered in call order with the small blobs'.
  std::vector<uint64_t> med;
  std::vector<std::vector<CapturedPost>> big(n);
  uint64_t n_small = 0;
  const uint64_t small_max = small_max_for(bs);  // one block, <= 16 KiB
  for (uint64_t i = 0; i < n; ++i) {
    if (lengths[i] <= small_max) {
      ++n_small;
    } else if (lengths[i] <= bs && lengths[i] <= kMaxMedLen) {
      med.push_back(i);
    } else {
      glfsx_root r;
      if (int e = glfsx_create(bs, store_max, salt, cid_key,
                               static_cast<const uint8_t *>(data) + offsets[i],
                               lengths[i], capture_post, &big[i], &r))
        return e;
      memcpy(roots_out + 64 * i, r.ref, 64);
    }
  }
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  if (!med.empty()) {
    Salts salts;
    if (int e = derive_salts(c, salt, &salts)) return e;
    for (size_t g0 = 0; g0 < med.size();) {
      size_t g1 = g0;
      uint64_t bytes = 0;
      while (g1 < med.size() && (g1 == g0 || bytes + lengths[med[g1]] <= kMedBatchBytes)) {
        bytes += (lengths[med[g1]] + 63) & ~uint64_t(63);
        ++g1;
      }
      const size_t k = g1 - g0;
      if (int e = c->h_bin.ensure(bytes)) return e;
      if (post)
        if (int e = c->h_bct.ensure(bytes)) return e;
      if (int e = c->h_bref.ensure(64 * k)) return e;
      std::vector<OneReq> reqs(k);
      std::vector<OneReq *> rp(k);
      uint64_t o = 0;
      for (size_t j = 0; j < k; ++j) {
        const uint64_t i = med[g0 + j], len = lengths[i];
        par_memcpy(c->h_bin.u8() + o, static_cast<const uint8_t *>(data) + offsets[i], len);
        OneDesc &d = reqs[j].d;
        d.src = c->h_bin.dptr() + o;
        d.ctext = post ? c->h_bct.dptr() + o : nullptr;
        d.ref = c->h_bref.dptr() + 64 * j;
        d.len = d.present = uint32_t(len);
        one_keys(d, salts.raw, cid_key);
        rp[j] = &reqs[j];
        o += (len + 63) & ~uint64_t(63);
      }
      if (int e = one_post_many(c->dev, rp.data(), k)) return e;
      for (size_t j = 0; j < k; ++j) {
        const uint64_t i = med[g0 + j];
        memcpy(roots_out + 64 * i, c->h_bref.u8() + 64 * j, 64);
        if (post) {
          const uint64_t off = reqs[j].d.ctext - c->h_bct.dptr();
          capture_post(&big[i], 0, roots_out + 64 * i, c->h_bct.u8() + off, lengths[i]);
        }
      }
      g0 = g1;
    }
  }
  if (n_small) {
    if (int e = post_small_groups(c, bs, salt, cid_key, static_cast<const uint8_t *>(data),
                                  offsets, lengths, n, small_max, big, post, post_ctx,
                                  roots_out))
      return e;
  } else if (post) {
    for (uint64_t i = 0; i < n; ++i)
      for (const CapturedPost &p : big[i]) {
        int rc = post(post_ctx, p.kind, p.ref, p.ctext.data(), p.ctext.size());
        if (rc) return fail(GLFSX_E_STORE, "store.Post failed with code %d", rc);
      }
  }
  return 0;
}

int glfsx_fill_splitmix_device(void *d_dst, uint64_t offset, uint64_t n,
                               uint64_t seed, void *stream) {
  if (n && !d_dst) return fail(GLFSX_E_ARG, "null argument");
  if (offset & 7) return fail(GLFSX_E_ARG, "offset must be a multiple of 8");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  HIP_TRY(launch_fill(static_cast<uint8_t *>(d_dst), offset, n, seed,
                      pick_stream(c, stream)));
  return 0;
}

int glfsx_decrypt_batch_device(const void *d_ctext, uint64_t total,
                               uint64_t block_size, const void *d_refs,
                               void *d_ptext, void *stream) {
  if (total == 0) return 0;
  if (!d_ctext || !d_refs || !d_ptext) return fail(GLFSX_E_ARG, "null argument");
  if (block_size == 0 || block_size % 64)
    return fail(GLFSX_E_UNSUPPORTED, "decrypt needs block_size %% 64 == 0");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  const uint64_t n = (total + block_size - 1) / block_size;
  HIP_TRY(launch_decrypt(static_cast<const uint8_t *>(d_ctext),
                         static_cast<uint8_t *>(d_ptext), n, block_size,
                         total - (n - 1) * block_size,
                         static_cast<const uint8_t *>(d_refs), pick_stream(c, stream)));
  return 0;
}

// BASELINE config 4 in one call, device-resident: tree.go:250-320's
// PostTreeMap over n entries whose blobs are glfs.PostBlob'd (machine.go:64)
// -- blob roots (glfsx_post_blobs_device), the tree's JSON lines
// (glfsx_tree_encode_device) and the tree blob's Create
// (glfsx_create_device) -- in one call, every launch queued before the host
// waits:
//   A: the blobs' DEK pass;
//   B (beside it): the lines' layout (lengths, then a one-workgroup prefix
//      that stores the total in a pinned word the host reads) and the lines
//      without their hex digits, at raised wave priority (a hex field is
//      fixed width, so the layout does not depend on the roots' values);
//   A: the blobs' CID pass once the static lines are in, writing each
//      root's hex digits into its line;
//   A: the tree blob's blocks and index levels (glfsx_create_device's
//      closed form) once the host has read the total.
// Same bytes and roots as the three calls in sequence
// (tests/test_gpu_tree_read.py).  Blobs above 16 KiB, a tree block size that
// is not a multiple of 64, or no line buffer take the three calls in
// sequence.
namespace {
int post_tree_device_impl(uint64_t n, uint64_t blob_bs, const uint8_t *blob_salt,
                          const uint8_t *tree_salt, const uint8_t *cid_key,
                          const void *d_data, const uint64_t *d_offsets,
                          const uint64_t *d_lengths, uint64_t max_len, void *d_ctext,
                          void *d_roots, const uint8_t *d_names,
                          const uint64_t *d_name_offs, const uint32_t *d_modes,
                          const uint8_t *d_types, const uint64_t *d_type_offs,
                          const uint64_t *d_block_sizes, uint64_t tree_bs, void *d_lines,
                          uint64_t lines_cap, void *d_tree_ctext, glfsx_root *tree_root,
                          uint64_t *lines_len, void *stream) {
  if (!tree_root || !lines_len) return fail(GLFSX_E_ARG, "null argument");
  if (int e = check_block_size(blob_bs)) return e;
  if (int e = check_block_size(tree_bs)) return e;
  if (n == 0 || max_len > small_max_for(blob_bs) || tree_bs % 64 || !d_lines) {
    if (int e = glfsx_post_blobs_device(blob_bs, blob_salt, cid_key, d_data, d_offsets,
                                        d_lengths, n, max_len, d_ctext, d_roots, stream))
      return e;
    if (int e = glfsx_tree_encode_device(n, d_names, d_name_offs, d_modes, d_types,
                                         d_type_offs, static_cast<const uint8_t *>(d_roots),
                                         d_lengths, d_block_sizes, d_lines, lines_cap,
                                         nullptr, lines_len, stream))
      return e;
    return glfsx_create_device(tree_bs, tree_salt, cid_key, d_lines, *lines_len,
                               d_tree_ctext, tree_root, nullptr, stream);
  }
  if (!d_data || !d_offsets || !d_lengths || !d_roots || !d_name_offs || !d_modes ||
      !d_type_offs || !d_block_sizes)
    return fail(GLFSX_E_ARG, "null argument");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  hipStream_t A = pick_stream(c, stream);
  if (!c->stream2) HIP_TRY(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
  hipStream_t B = c->stream2;
  const uint64_t wgs = (n + kTreeWG - 1) / kTreeWG;
  while (c->events.size() < 3) {
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    c->events.push_back(ev);
  }
  hipEvent_t ev_before = c->events[0], ev_layout = c->events[1], ev_static = c->events[2];
  Salts bsalts, tsalts;
  if (int e = derive_salts(c, blob_salt, &bsalts)) return e;
  if (int e = derive_salts(c, tree_salt, &tsalts)) return e;
  const uint64_t words = n + wgs + 1;
  if (int e = c->d_tree.ensure(8 * (words + n))) return e;
  if (int e = c->h_tree.ensure(8 * (wgs + 1))) return e;
  TreeJob tj{};
  tj.n = n;
  tj.names = d_names;
  tj.name_offs = d_name_offs;
  tj.modes = d_modes;
  tj.types = d_types;
  tj.type_offs = d_type_offs;
  tj.roots = static_cast<const uint8_t *>(d_roots);
  tj.sizes = d_lengths;
  tj.block_sizes = d_block_sizes;
  tj.scratch = reinterpret_cast<uint64_t *>(c->d_tree.p);
  tj.total = tj.scratch + words - 1;
  tj.out = static_cast<uint8_t *>(d_lines);
  tj.cap = lines_cap;
  tj.hex_pos = tj.scratch + words;  // where each root's digits go
  tj.prio = 1;                      // beside the DEK pass: raised issue priority
  // the prefix stores the exclusive prefixes and the total in the pinned
  // words the host reads (a copy kernel behind it on B would wait for a CU
  // beside the DEK pass -- 1.1 ms in the round-4 trace)
  tj.prefix_host = reinterpret_cast<uint64_t *>(c->h_tree.dptr());
  // B's work comes after everything already on A
  HIP_TRY(hipEventRecord(ev_before, A));
  HIP_TRY(hipStreamWaitEvent(B, ev_before, 0));
  SmallJob sj{};
  sj.src = static_cast<const uint8_t *>(d_data);
  sj.ctext = static_cast<uint8_t *>(d_ctext);
  sj.max_len = max_len;
  sj.small_max = small_max_for(blob_bs);
  sj.offs = d_offsets;
  sj.lens = d_lengths;
  sj.n = n;
  sj.refs = static_cast<uint8_t *>(d_roots);
  words_from_key(sj.raw_salt, bsalts.raw);
  words_from_key(sj.index_salt, bsalts.index);
  if (cid_key) {
    words_from_key(sj.cid_key, cid_key);
    sj.cid_keyed = true;
  } else {
    blake3_iv_words(sj.cid_key);
  }
  sj.passes = 1;  // the DEK pass: the critical path, queued first
  HIP_TRY(launch_post_small(sj, A));
  HIP_TRY(launch_tree_layout(tj, B));
  HIP_TRY(hipEventRecord(ev_layout, B));
  HIP_TRY(launch_tree_static(tj, B));
  HIP_TRY(hipEventRecord(ev_static, B));
  sj.passes = 2;  // the CID pass, writing the digits once the static parts are in
  sj.hex_out = static_cast<uint8_t *>(d_lines);
  sj.hex_pos = tj.hex_pos;
  sj.cid_wait = ev_static;
  HIP_TRY(launch_post_small(sj, A));
  // the layout (beside the DEK pass) gives the tree blob's size
  HIP_TRY(hipEventSynchronize(ev_layout));
  const uint64_t total = static_cast<const uint64_t *>(c->h_tree.p)[wgs];
  if (total > lines_cap) {
    HIP_TRY(hipStreamSynchronize(A));
    *lines_len = total;
    return fail(GLFSX_E_ARG, "tree lines need %llu bytes, buffer holds %llu",
                (unsigned long long)total, (unsigned long long)lines_cap);
  }
  // the tree blob, on A after the CID pass (its lines are complete then)
  const uint64_t nblk = (total + tree_bs - 1) / tree_bs;
  const uint64_t n1 = (nblk + tree_bs / 64 - 1) / (tree_bs / 64);
  if (int e = level_prepare(c->d_lvl_a, nblk, n1, tree_bs, A)) return e;
  uint8_t *lvl = c->d_lvl_a.u8();
  PostJob j{};
  j.src = static_cast<const uint8_t *>(d_lines);
  j.ctext = static_cast<uint8_t *>(d_tree_ctext);
  j.stride = tree_bs;
  j.msg_len = tree_bs;
  j.n = nblk;
  j.last_len = total - (nblk - 1) * tree_bs;
  j.out = RefLayout{lvl, ~0ull, 0};  // ref t at byte 64t
  words_from_key(j.salt, tsalts.raw);
  cid_words(j, cid_key);
  HIP_TRY(launch_post(j, A, tls_fused));
  *lines_len = total;
  tree_root->size = total;
  tree_root->block_size = tree_bs;
  if (nblk <= 1) {  // one block: its ref is the root (blob.go:190-193)
    if (int e = c->h_root.ensure(64)) return e;
    HIP_TRY(hipMemcpyAsync(c->h_root.p, lvl, 64, hipMemcpyDeviceToHost, A));
    HIP_TRY(stream_wait(A));  // (B is drained: A waited for its static lines)
    if (int e = fused_check(A)) return e;
    memcpy(tree_root->ref, c->h_root.p, 64);
    return 0;
  }
  uint64_t posts = 0;
  return build_up(c, A, tsalts, cid_key, tree_bs, lvl, n1, &c->d_lvl_b, tree_root->ref, &posts);
}
}  // namespace

int glfsx_post_tree_device(uint64_t n, uint64_t blob_bs, const uint8_t *blob_salt,
                           const uint8_t *tree_salt, const uint8_t *cid_key,
                           const void *d_data, const uint64_t *d_offsets,
                           const uint64_t *d_lengths, uint64_t max_len, void *d_ctext,
                           void *d_roots, const uint8_t *d_names,
                           const uint64_t *d_name_offs, const uint32_t *d_modes,
                           const uint8_t *d_types, const uint64_t *d_type_offs,
                           const uint64_t *d_block_sizes, uint64_t tree_bs, void *d_lines,
                           uint64_t lines_cap, void *d_tree_ctext, glfsx_root *tree_root,
                           uint64_t *lines_len, void *stream) {
  return with_fused_retry([&] {
    return post_tree_device_impl(n, blob_bs, blob_salt, tree_salt, cid_key, d_data, d_offsets,
                                 d_lengths, max_len, d_ctext, d_roots, d_names, d_name_offs,
                                 d_modes, d_types, d_type_offs, d_block_sizes, tree_bs, d_lines,
                                 lines_cap, d_tree_ctext, tree_root, lines_len, stream);
  });
}

int glfsx_tree_encode_device(uint64_t n, const uint8_t *d_names,
                             const uint64_t *d_name_offs, const uint32_t *d_modes,
                             const uint8_t *d_types, const uint64_t *d_type_offs,
                             const uint8_t *d_roots, const uint64_t *d_sizes,
                             const uint64_t *d_block_sizes, void *d_out,
                             uint64_t out_cap, uint64_t *d_line_ends,
                             uint64_t *out_len, void *stream) {
  if (!out_len) return fail(GLFSX_E_ARG, "null out_len");
  *out_len = 0;
  if (n == 0) return 0;
  if (!d_name_offs || !d_modes || !d_type_offs || !d_roots || !d_sizes ||
      !d_block_sizes)
    return fail(GLFSX_E_ARG, "null argument");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  hipStream_t s = pick_stream(c, stream);
  const uint64_t words = n + (n + kTreeWG - 1) / kTreeWG + 1;
  if (int e = c->d_tree.ensure(8 * words)) return e;
  if (int e = c->h_small.ensure(64)) return e;
  TreeJob j{};
  j.n = n;
  j.names = d_names;
  j.name_offs = d_name_offs;
  j.modes = d_modes;
  j.types = d_types;
  j.type_offs = d_type_offs;
  j.roots = d_roots;
  j.sizes = d_sizes;
  j.block_sizes = d_block_sizes;
  j.scratch = reinterpret_cast<uint64_t *>(c->d_tree.p);
  j.total = j.scratch + words - 1;
  j.line_ends = d_line_ends;
  j.out = static_cast<uint8_t *>(d_out);
  j.cap = d_out ? out_cap : 0;
  HIP_TRY(launch_tree_encode(j, s));
  HIP_TRY(hipMemcpyAsync(c->h_small.p, j.total, 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(stream_wait(s));
  memcpy(out_len, c->h_small.p, 8);
  if (d_out && *out_len > out_cap)
    return fail(GLFSX_E_ARG, "tree lines need %llu bytes, buffer holds %llu",
                (unsigned long long)*out_len, (unsigned long long)out_cap);
  return 0;
}

int glfsx_fill_splitmix_blobs_device(void *d_dst, uint64_t n, uint64_t len,
                                     uint64_t seed0, void *stream) {
  if (n && len && !d_dst) return fail(GLFSX_E_ARG, "null argument");
  if (len % 8 || (reinterpret_cast<uintptr_t>(d_dst) & 7))
    return fail(GLFSX_E_ARG, "blob length and pointer must be multiples of 8");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  HIP_TRY(launch_fill_blobs(static_cast<uint8_t *>(d_dst), n, len, seed0,
                            pick_stream(c, stream)));
  return 0;
}

// Batched getF decrypt from host memory: slabs of whole blocks through two
// slots and three streams (upload k+1 / decrypt k / download k-1 overlap).
int glfsx_decrypt_batch(const void *ctext, uint64_t total, uint64_t block_size,
                        const uint8_t *refs, void *ptext) {
  if (total == 0) return 0;
  if (!ctext || !refs || !ptext) return fail(GLFSX_E_ARG, "null argument");
  if (block_size == 0 || block_size % 64)
    return fail(GLFSX_E_UNSUPPORTED, "decrypt needs block_size %% 64 == 0");
  Ctx *c;
  if (int e = ctx_get(&c)) return e;
  const uint64_t n = (total + block_size - 1) / block_size;
  const uint64_t slab_blocks = std::max<uint64_t>(1, (64ull << 20) / block_size);
  struct Slot {
    DevBuf d_in, d_out, d_refs;
    PinBuf h_in, h_out;
    hipEvent_t up = nullptr, done = nullptr;
    uint64_t b0 = 0, nb = 0, bytes = 0;
    bool busy = false;
  };
  static thread_local Slot slots[2];
  static thread_local hipStream_t s_up = nullptr, s_dn = nullptr;
  if (!s_up) {
    HIP_TRY(hipStreamCreateWithFlags(&s_up, hipStreamNonBlocking));
    HIP_TRY(hipStreamCreateWithFlags(&s_dn, hipStreamNonBlocking));
  }
  auto finish = [&](Slot &sl) -> int {
    if (!sl.busy) return 0;
    sl.busy = false;
    HIP_TRY(hipEventSynchronize(sl.done));
    par_memcpy(static_cast<uint8_t *>(ptext) + sl.b0 * block_size, sl.h_out.u8(), sl.bytes);
    return 0;
  };
  int k = 0;
  for (uint64_t b0 = 0; b0 < n; b0 += slab_blocks, k ^= 1) {
    Slot &sl = slots[k];
    if (int e = finish(sl)) return e;
    sl.b0 = b0;
    sl.nb = std::min(slab_blocks, n - b0);
    sl.bytes = std::min<uint64_t>(sl.nb * block_size, total - b0 * block_size);
    if (int e = sl.d_in.ensure(sl.bytes + 64)) return e;
    if (int e = sl.d_out.ensure(sl.bytes + 64)) return e;
    if (int e = sl.d_refs.ensure(64 * sl.nb)) return e;
    if (int e = sl.h_in.ensure(sl.bytes + 64 * sl.nb)) return e;
    if (int e = sl.h_out.ensure(sl.bytes)) return e;
    if (!sl.up) {
      HIP_TRY(hipEventCreateWithFlags(&sl.up, hipEventDisableTiming));
      HIP_TRY(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming));
    }
    par_memcpy(sl.h_in.u8(), static_cast<const uint8_t *>(ctext) + b0 * block_size, sl.bytes);
    memcpy(sl.h_in.u8() + sl.bytes, refs + 64 * b0, 64 * sl.nb);
    HIP_TRY(hipMemcpyAsync(sl.d_in.p, sl.h_in.p, sl.bytes, hipMemcpyHostToDevice, s_up));
    HIP_TRY(hipMemcpyAsync(sl.d_refs.p, sl.h_in.u8() + sl.bytes, 64 * sl.nb,
                           hipMemcpyHostToDevice, s_up));
    HIP_TRY(hipEventRecord(sl.up, s_up));
    HIP_TRY(hipStreamWaitEvent(c->stream, sl.up, 0));
    HIP_TRY(launch_decrypt(sl.d_in.u8(), sl.d_out.u8(), sl.nb, block_size,
                           sl.bytes - (sl.nb - 1) * block_size, sl.d_refs.u8(), c->stream));
    HIP_TRY(hipEventRecord(sl.up, c->stream));
    HIP_TRY(hipStreamWaitEvent(s_dn, sl.up, 0));
    HIP_TRY(hipMemcpyAsync(sl.h_out.p, sl.d_out.p, sl.bytes, hipMemcpyDeviceToHost, s_dn));
    HIP_TRY(hipEventRecord(sl.done, s_dn));
    sl.busy = true;
  }
  for (int i = 0; i < 2; ++i, k ^= 1)
    if (int e = finish(slots[k])) return e;
  return 0;
}

// A store sink that only counts (benchmarks, tests): ctx -> uint64_t[2] =
// {posts, bytes}.  Stands in for a native store's Post at ~zero cost.
int glfsx_sink_count(void *ctx, int kind, const uint8_t *ref, const void *ctext,
                     uint64_t len) {
  (void)kind;
  (void)ref;
  (void)ctext;
  uint64_t *c = static_cast<uint64_t *>(ctx);
  if (c) {
    c[0] += 1;
    c[1] += len;
  }
  return 0;
}

// blob.go:219-268 (pure integer shape math, no hashing)
static uint64_t log2_ceil(uint64_t x) {
  int l = 64 - __builtin_clzll(x);
  if (__builtin_popcountll(x) > 1) l++;
  return uint64_t(l) - 1;
}
static uint64_t div_ceil(uint64_t a, uint64_t b) { return (a + b - 1) / b; }

uint64_t glfsx_branching_factor(uint64_t block_size) { return block_size / 64; }

int glfsx_depth(uint64_t size, uint64_t block_size) {
  if (size == 0) return 0;
  const uint64_t blocks = div_ceil(size, block_size);
  const uint64_t bf = glfsx_branching_factor(block_size);
  return int(div_ceil(log2_ceil(blocks), log2_ceil(bf)));
}

}  // extern "C"
