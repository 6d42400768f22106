// api.cpp -- eegfx C ABI: device context, compute entry points and the OffLineDataProvider.
//
// The data provider mirrors DataTransformation/OffLineDataProvider.java (constructor :78,
// loadData :88-98, handleInput :111-141, processEEGFiles :147-268, loadFilesFromInfoTxt
// :283-319, setFileNames :327-365, getData :370, getDataLabels :377) with local files in place
// of HDFS.  Epochs are cut and baseline-corrected on the GPU and stay resident in HBM; getData()
// copies them back on demand.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <sched.h>
#include <string>
#include <utility>
#include <vector>

#include "common.h"
#include "eegfx_ext.h"
#include "launch.h"
#include "spark_sample.h"

using namespace eegfx;

#define HIP_CHECK(expr)                                                                 \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) fail(EEGFX_EHIP, "%s: %s", #expr, hipGetErrorString(_e));     \
  } while (0)

// Microseconds a small call's waiter spins before it sleeps (A/B builds vary it).
#ifndef EEGFX_SMALL_SPIN_US
#define EEGFX_SMALL_SPIN_US 30
#endif
// A/B only: the small-call admission gate around the launch alone (the wait outside it)
#ifndef EEGFX_GATE_LAUNCH_ONLY
#define EEGFX_GATE_LAUNCH_ONLY 0
#endif
// A/B only: configs[4]'s marker positions uploaded beside the first chunk instead of before it
#ifndef EEGFX_STREAM_POS_AFTER
#define EEGFX_STREAM_POS_AFTER 0
#endif
// A/B only: a small call's waiter past the spin polls its event between 10-us sleeps instead of
// sleeping in the runtime's blocking-sync wait
#ifndef EEGFX_SMALL_SLEEP_POLL
#define EEGFX_SMALL_SLEEP_POLL 0
#endif

namespace {

// Grow-only device allocation owned by a context, stream-ordered on the context's stream (`*sp`):
// every use of the buffer is enqueued there (the streamed path's side streams are drained before
// its call returns), so the old allocation is released behind the work already queued and the new
// one is ready for the work that follows.  Growing never waits for the device -- other contexts
// keep running (a hipDeviceSynchronize + hipFree here stalled every context on the device).
struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  const hipStream_t* sp = nullptr;
  void* get(size_t bytes) {
    if (bytes > cap) {
      if (p) (void)hipFreeAsync(p, *sp);
      p = nullptr;
      cap = 0;
      if (hipMallocAsync(&p, bytes ? bytes : 1, *sp) != hipSuccess) {
        (void)hipGetLastError();
        p = nullptr;
        fail(EEGFX_ENOMEM, "hipMallocAsync(%zu) failed", bytes);
      }
      cap = bytes;
    }
    return p;
  }
  void release() {
    if (p) (void)hipFreeAsync(p, *sp);
    p = nullptr;
    cap = 0;
  }
};

// Pinned host memory is never returned to the runtime while the process runs: hipHostFree (like
// hipFree) synchronises the whole device, which waits for every resident per-epoch server of
// every context (up to its 1 s idle exit) -- a context destroyed or a staging buffer grown on one
// executor thread stalled every other thread's calls for a second (profiles/r06/dropin_threads).
// Buffers go back to this process-wide pool instead and are reused by the next request of at
// least their size with the same flags; the pool holds at most the peak of what was in use.
struct PinnedPool {
  std::mutex mu;
  std::multimap<std::pair<unsigned, size_t>, void*> free;  // (flags, capacity) -> buffer
  void* take(size_t bytes, unsigned flags, size_t* cap) {
    bytes = std::max<size_t>(bytes, 64);
    {
      std::lock_guard<std::mutex> l(mu);
      auto it = free.lower_bound({flags, bytes});
      if (it != free.end() && it->first.first == flags && it->first.second <= 2 * bytes + 65536) {
        void* p = it->second;
        *cap = it->first.second;
        free.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    if (hipHostMalloc(&p, bytes, flags) != hipSuccess) {
      (void)hipGetLastError();
      fail(EEGFX_ENOMEM, "hipHostMalloc(%zu) failed", bytes);
    }
    *cap = bytes;
    return p;
  }
  void give(void* p, size_t cap, unsigned flags) {
    if (!p) return;
    std::lock_guard<std::mutex> l(mu);
    free.emplace(std::make_pair(flags, cap), p);
  }
};
PinnedPool& pinned_pool() {
  static PinnedPool* pool = new PinnedPool();  // never destroyed: buffers live to process exit
  return *pool;
}

// Grow-only pinned host buffer (hipHostMalloc: mapped into the device address space, from
// pinned_pool), for the small-batch IFeatureExtraction path and the streamed path's host staging.
// Only touched by the owning context's calls, which synchronise before they return.
struct PinBuf {
  void* p = nullptr;
  size_t cap = 0;
  void* get(size_t bytes) {
    if (bytes > cap) {
      pinned_pool().give(p, cap, hipHostMallocMapped);
      p = nullptr;
      cap = 0;
      p = pinned_pool().take(bytes, hipHostMallocMapped, &cap);
    }
    return p;
  }
  void* device_ptr() const {
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess)
      fail(EEGFX_EHIP, "hipHostGetDevicePointer failed");
    return d;
  }
  void release() {
    pinned_pool().give(p, cap, hipHostMallocMapped);
    p = nullptr;
    cap = 0;
  }
};

ChanSel make_sel(const int32_t* cols, const float* res, int C, int ct) {
  if (C < 1 || C > kMaxChannels) fail(EEGFX_EINVAL, "C=%d outside [1, %d]", C, kMaxChannels);
  if (!cols || !res) fail(EEGFX_EINVAL, "cols/res must be host arrays");
  ChanSel s;
  memset(&s, 0, sizeof(s));
  for (int c = 0; c < C; ++c) {
    if (cols[c] < 0 || cols[c] >= ct)
      fail(EEGFX_EINVAL, "column %d of selected channel %d outside [0, %d)", cols[c], c, ct);
    s.col[c] = cols[c];
    s.res[c] = res[c];
  }
  return s;
}

void check_positions(const int64_t* pos, int64_t n, int64_t n_frames) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t lo = pos[i] - EEGFX_PRESTIMULUS;
    if (lo < 0 || lo > n_frames)
      fail(EEGFX_ERANGE, "epoch %lld: marker position %lld outside [100, %lld]", (long long)i,
           (long long)pos[i], (long long)n_frames + EEGFX_PRESTIMULUS);
  }
}

void check_fe_params(int C, int name, int epoch_size, int skip, int feature_size) {
  if (C < 1 || C > kMaxChannels) fail(EEGFX_EINVAL, "C=%d outside [1, %d]", C, kMaxChannels);
  if (skip < 0 || epoch_size <= 0 || skip + epoch_size > EEGFX_POSTSTIMULUS)
    fail(EEGFX_ERANGE, "window [%d, %d) outside the %d-sample epoch", skip, skip + epoch_size,
         EEGFX_POSTSTIMULUS);
  if (feature_size <= 0) fail(EEGFX_EINVAL, "feature size %d", feature_size);
  if (name != EEGFX_DWT8_NAME || epoch_size != EEGFX_DWT8_EPOCH_SIZE || feature_size > 16)
    fail(EEGFX_ENOTSUP,
         "no kernel for wavelet %d / epoch size %d / feature size %d (supported: dwt-8, 512, <=16)",
         name, epoch_size, feature_size);
}

}  // namespace

struct eegfx_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t stream = nullptr;
  int numerics = EEGFX_EXACT;
  // Error word of the device-side position checks (fused.hip position_ok): host-mapped pinned
  // memory the kernels store 1 into; eegfx_ctx_synchronize reports and clears it.
  int* err_host = nullptr;
  int* err_dev = nullptr;
  size_t err_cap = 0;  // pinned_pool capacity of err_host
  // the fma window kernel's guard strategy (guard.h EEGFX_TRACK_X), set by baseline_kernel in the
  // same host-mapped block, 8 bytes past the error word
  unsigned int* track_host() const { return (unsigned int*)((char*)err_host + 8); }
  unsigned int* track_dev() const { return (unsigned int*)((char*)err_dev + 8); }
  bool guard_track() const {
    return EEGFX_TRACK_X == 2 ||
           (EEGFX_TRACK_X == 1 && __atomic_load_n(track_host(), __ATOMIC_RELAXED) != 0);
  }
  bool timing = false;
  // HIP event pairs bracketing each timed (dominant) kernel launch on the context stream, plus
  // the algorithmic bytes each launch moved; summed by eegfx_ctx_kernel_stats.
  std::vector<std::pair<hipEvent_t, hipEvent_t>> events;
  std::vector<int64_t> event_bytes;
  size_t n_timed = 0;
  DevBuf raw, pos, out, scratch, fused;
  DevBuf lr_x, lr_y, lr_state, lr_part, lr_mask;  // logistic regression (eegfx_logreg_*)
  PinBuf pin_in, pin_out;                // small-batch extract_features staging (zero-copy)
  PinBuf pin_chunk[2];                   // streamed path: host staging of pageable recordings
  // The fma numerics' conditioning guard (guard.h): device memory holding the flagged-row count
  // of the current window_wide_kernel launch (first 128 B), then the running totals of recomputed
  // rows and of rows that went to the second stage, each spread over kGuardSlots lines; the
  // flagged-row list; guard_checked counts the rows that went through a guarded launch.
  static constexpr size_t kGuardDevBytes = 128 + 2 * kGuardSlotBytes + 128;  // + Guard::adapt
  int* guard_dev = nullptr;
  DevBuf guard_list;
  int64_t guard_checked = 0;
  unsigned long long* guard_recomputed_slots() const {
    return (unsigned long long*)((char*)guard_dev + 128);
  }
  unsigned long long* guard_rechecked_slots() const {
    return (unsigned long long*)((char*)guard_dev + 128 + kGuardSlotBytes);
  }
  unsigned long long* guard_adapt() const {
    return (unsigned long long*)((char*)guard_dev + 128 + 2 * kGuardSlotBytes);
  }
  Guard guard_for(int64_t n) {
    if (numerics == EEGFX_EXACT) return Guard{nullptr, nullptr, nullptr};
    guard_checked += n;
    return Guard{guard_dev, (int64_t*)guard_list.get(sizeof(int64_t) * (size_t)std::max<int64_t>(n, 1)),
                 guard_recomputed_slots(), guard_rechecked_slots(), guard_adapt(), track_dev()};
  }
  void bind_buffers() {
    for (DevBuf* b : {&raw, &pos, &out, &scratch, &fused, &lr_x, &lr_y, &lr_state, &lr_part,
                      &lr_mask, &guard_list})
      b->sp = &stream;
  }
  void release_buffers() {
    for (DevBuf* b : {&raw, &pos, &out, &scratch, &fused, &lr_x, &lr_y, &lr_state, &lr_part,
                      &lr_mask, &guard_list})
      b->release();
    pin_in.release();
    pin_out.release();
    pin_chunk[0].release();
    pin_chunk[1].release();
  }
  // streamed path (eegfx_process_recording_streamed): upload / download streams and the chunk
  // events, created on first use and kept for the context's lifetime
  hipStream_t up = nullptr, down = nullptr;
  std::vector<hipEvent_t> copied, done;  // per device chunk buffer: uploaded / kernels done
  void stream_resources(size_t ring) {
    if (!up) {
      HIP_CHECK(hipStreamCreateWithFlags(&up, hipStreamNonBlocking));
      HIP_CHECK(hipStreamCreateWithFlags(&down, hipStreamNonBlocking));
    }
    while (copied.size() < ring) {
      hipEvent_t a = nullptr, b = nullptr;
      HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableTiming));
      if (hipEventCreateWithFlags(&b, hipEventDisableTiming) != hipSuccess) {
        (void)hipEventDestroy(a);
        fail(EEGFX_EHIP, "hipEventCreateWithFlags");
      }
      copied.push_back(a);
      done.push_back(b);
    }
  }
  // Completion of a small (latency-bound) call: spinning on an event query returns ~0.5 us sooner
  // than hipStreamSynchronize (the drop-in bench's launch floor: 11.6 vs 12.2 us).  Past kSmallSpin
  // the thread sleeps until the event completes (a blocking-sync event: interrupt-driven), so a
  // waiter is not runnable: with more calling threads than cores (Spark local[*] on a CPU quota),
  // runnable waiters kept threads whose work had completed off the cores for scheduler slices
  // (profiles/r06/dropin_gate_ab.log).
  static constexpr auto kSmallSpin = std::chrono::microseconds(EEGFX_SMALL_SPIN_US);
  hipEvent_t small_done = nullptr;
  void record_small() {
    if (!small_done)
      HIP_CHECK(hipEventCreateWithFlags(&small_done, hipEventDisableTiming | hipEventBlockingSync));
    HIP_CHECK(hipEventRecord(small_done, stream));
  }
  void wait_small(bool recorded = false) {
    if (!recorded) record_small();
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t e;
    while ((e = hipEventQuery(small_done)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 > kSmallSpin) {
#if EEGFX_SMALL_SLEEP_POLL
        while ((e = hipEventQuery(small_done)) == hipErrorNotReady)
          std::this_thread::sleep_for(std::chrono::microseconds(10));
        break;
#else
        HIP_CHECK(hipEventSynchronize(small_done));
        return;
#endif
      }
    }
    HIP_CHECK(e);
  }
  // The opt-in resident small-batch server (eegfx_ctx_set_mailbox, features_mailbox_kernel): a
  // host-mapped command block, the kernel's own stream (never the context stream: the kernel
  // stays resident), the request sequence and the time of the last request.  A server needs a
  // hardware queue of its own (a queue runs its packets in order: a second kernel behind a
  // resident one waits for it to idle out), and the highest-priority pool has kMbSlotsPerDevice of
  // them, so at most that many contexts of the process hold a server slot on a device
  // (mb_acquire); the others serve their calls on the launch path, and take a slot when one frees.
  bool mailbox = false;   // enabled by the caller
  bool mb_slot = false;   // holds one of the device's server slots
  hipStream_t mb_stream = nullptr;
  MailboxCmd* mb_host = nullptr;
  MailboxCmd* mb_dev = nullptr;
  size_t mb_cap = 0;  // pinned_pool capacity of mb_host
  uint32_t mb_seq = 0;
  uint32_t mb_gen = 0;      // launch generation (MailboxCmd::alive)
  bool mb_live = false;     // launched and not stopped by the host (it may still have idled out)
  bool mb_started = false;  // the live server has published its generation
  bool mb_stuck = false;    // a server that did not start in time: stopped, not yet returned
  std::chrono::steady_clock::time_point mb_last{};
  static constexpr uint64_t kMbIdleTicks = 100000000;  // 1 s of s_memrealtime (100 MHz)
  void mb_launch() {
    // the staging a server reads is fixed for its lifetime (growing it stops the server first)
    mb_host->rows = pin_in.p ? (const double*)pin_in.device_ptr() : nullptr;
    mb_host->out = pin_out.p ? (double*)pin_out.device_ptr() : nullptr;
    if (++mb_gen == 0) mb_gen = 1;
    HIP_CHECK(launch_features_mailbox(mb_stream, mb_dev, kMbIdleTicks, mb_gen));
    mb_live = true;
    mb_started = false;
  }
  // Stops a live server: `stop` is seen within one poll.  A server that has not returned after
  // 10 s (100 ms if it has not been seen to start: its queue is held by another resident kernel)
  // keeps `stop` set, so it returns as soon as it runs, and is marked stuck; mb_ready clears
  // `stop` once it has returned.
  // Returns whether the kernel has returned.
  bool mb_stop() {
    if (!mb_host || !mb_live) return true;
    __atomic_store_n(&mb_host->stop, 1u, __ATOMIC_RELEASE);
    const auto t0 = std::chrono::steady_clock::now();
    hipError_t q;
    while ((q = hipStreamQuery(mb_stream)) == hipErrorNotReady) {
      if (std::chrono::steady_clock::now() - t0 >
          (mb_started ? std::chrono::milliseconds(10000) : std::chrono::milliseconds(100))) {
        mb_live = false;
        mb_stuck = true;
        return false;
      }
      std::this_thread::yield();
    }
    __atomic_store_n(&mb_host->stop, 0u, __ATOMIC_RELEASE);
    mb_live = false;
    HIP_CHECK(q);
    return true;
  }
  // hipSuccess: the server kernel has returned; hipErrorNotReady: it is running; anything else
  // is an error of the stream and is raised
  bool mb_returned() {
    const hipError_t q = hipStreamQuery(mb_stream);
    if (q == hipErrorNotReady) return false;
    HIP_CHECK(q);
    return true;
  }
  // Whether the resident server takes this call (false: the launch path).  Takes a device slot
  // and sets the server up on first use; restarts a server that may be near its 1 s idle exit
  // (no request for 500 ms) so a request never races that exit; posts nothing until the server
  // has published its generation, and falls back to the launch path (marking the server stuck)
  // if it has not started within kMbStartWait.
  static constexpr auto kMbStartWait = std::chrono::milliseconds(20);
  bool mb_ready();
  // One request: n epochs of packed window rows in pin_in -> rows in pin_out (after mb_ready).
  void mb_serve(int64_t n, int C, int nfeat) {
    MailboxCmd* m = mb_host;
    if (++mb_seq == 0) mb_seq = 1;  // 0 means "no request" to the kernel
    const auto now = std::chrono::steady_clock::now();
    __atomic_store_n(&m->req, mailbox_request(mb_seq, C, nfeat, n), __ATOMIC_RELEASE);
    for (uint64_t spin = 1;; ++spin) {
      if (__atomic_load_n(&m->done, __ATOMIC_ACQUIRE) == mb_seq) break;
      // as wait_small: a waiter past kSmallSpin sleeps between polls instead of staying runnable
      if ((spin & 63) == 0 && std::chrono::steady_clock::now() - now > kSmallSpin)
        std::this_thread::sleep_for(std::chrono::microseconds(10));
      if ((spin & 4095) == 0) {
        // a server that returned with the request pending (an error, or a stop from another
        // path): serve it again on the same stream, after that kernel
        if (mb_returned() && __atomic_load_n(&m->done, __ATOMIC_ACQUIRE) != mb_seq) mb_launch();
        if (std::chrono::steady_clock::now() - now > std::chrono::seconds(30))
          fail(EEGFX_EHIP, "mailbox request %u not served within 30 s", mb_seq);
      }
      __builtin_ia32_pause();
    }
    mb_last = std::chrono::steady_clock::now();
  }
  void release_mailbox();
  void release_stream_resources() {
    release_mailbox();
    if (small_done) (void)hipEventDestroy(small_done);
    small_done = nullptr;
    for (hipEvent_t e : copied) (void)hipEventDestroy(e);
    for (hipEvent_t e : done) (void)hipEventDestroy(e);
    copied.clear();
    done.clear();
    if (up) (void)hipStreamDestroy(up);
    if (down) (void)hipStreamDestroy(down);
    up = down = nullptr;
  }

  void activate() const { HIP_CHECK(hipSetDevice(device)); }
  // Waits for the stream, then reports (and clears) a device-resident marker position that a
  // kernel enqueued on this context since the last check refused: every API call that
  // synchronises does this, so an invalid position surfaces at the first synchronising call
  // after it (at the latest eegfx_ctx_synchronize), never silently.
  void check_positions_flag() {
    if (__atomic_exchange_n(err_host, 0, __ATOMIC_ACQ_REL) != 0)
      fail(EEGFX_ERANGE,
           "a device-resident marker position lies outside [100, n_frames + 100] "
           "(OffLineDataProvider.java:220-225: ArrayIndexOutOfBoundsException); the rows of such "
           "epochs are unspecified");
  }
  void drain() {
    HIP_CHECK(hipStreamSynchronize(stream));
    check_positions_flag();
  }
  void tic() {
    if (!timing) return;
    if (n_timed == events.size()) {
      // timing only (read after the stream drains): no system-scope fence at each record, so
      // the bracketed kernel's neighbours pay no cache writeback / invalidate for the timing
      hipEvent_t a, b;
      HIP_CHECK(hipEventCreateWithFlags(&a, hipEventDisableSystemFence));
      HIP_CHECK(hipEventCreateWithFlags(&b, hipEventDisableSystemFence));
      events.emplace_back(a, b);
      event_bytes.push_back(0);
    }
    HIP_CHECK(hipEventRecord(events[n_timed].first, stream));
  }
  void toc(int64_t bytes) {
    if (!timing) return;
    HIP_CHECK(hipEventRecord(events[n_timed].second, stream));
    event_bytes[n_timed] = bytes;
    ++n_timed;
  }
  void destroy_events() {
    for (auto& e : events) {
      (void)hipEventDestroy(e.first);
      (void)hipEventDestroy(e.second);
    }
    events.clear();
    event_bytes.clear();
    n_timed = 0;
  }
};

namespace {

// Resident-server slots per device (eegfx_ctx::mb_ready): the highest-priority hardware queues
// of the process (4 on the box: a fifth server shares a queue and waits behind another until it
// idles out).
constexpr int kMbSlotsPerDevice = 4;
constexpr int kMbMaxDevices = 64;
std::mutex g_mb_mu;
int g_mb_used[kMbMaxDevices] = {};
bool mb_acquire(int dev) {
  if (dev < 0 || dev >= kMbMaxDevices) return false;
  std::lock_guard<std::mutex> l(g_mb_mu);
  if (g_mb_used[dev] >= kMbSlotsPerDevice) return false;
  ++g_mb_used[dev];
  return true;
}
void mb_release(int dev) {
  std::lock_guard<std::mutex> l(g_mb_mu);
  if (dev >= 0 && dev < kMbMaxDevices && g_mb_used[dev] > 0) --g_mb_used[dev];
}

// Admission of small launched calls (one epoch per call from many threads, no server): at most
// kSmallCallers per device are inside the runtime at once, the others sleep and are admitted in
// arrival order.  Without it 28 threads launching and waiting on one device (Spark local[*] with
// 32 executor threads, 4 of them on servers) convoyed in the runtime: calls of 42-48 ms
// (profiles/r06/dropin_gate_ab.log; A/B builds vary the cap).  A leaving caller hands its place to
// the first waiter and wakes that thread alone (each waiter sleeps on its own condition variable):
// a shared one woke every waiter at every exit, ~24 wakeups per call at 32 threads.
#ifndef EEGFX_SMALL_CALLERS
#define EEGFX_SMALL_CALLERS 8
#endif
constexpr int kSmallCallers = EEGFX_SMALL_CALLERS;
struct SmallWaiter {
  std::condition_variable cv;
  bool admitted = false;
  SmallWaiter* next = nullptr;
};
std::mutex g_small_mu;
int g_small_inside[kMbMaxDevices] = {};
SmallWaiter* g_small_head[kMbMaxDevices] = {};  // FIFO of sleeping callers
SmallWaiter* g_small_tail[kMbMaxDevices] = {};
struct SmallCallGate {
  int dev;
  explicit SmallCallGate(int d) : dev(d >= 0 && d < kMbMaxDevices ? d : -1) {
    if (dev < 0 || kSmallCallers <= 0) return;
    std::unique_lock<std::mutex> l(g_small_mu);
    if (!g_small_head[dev] && g_small_inside[dev] < kSmallCallers) {
      ++g_small_inside[dev];
      return;
    }
    SmallWaiter me;
    (g_small_tail[dev] ? g_small_tail[dev]->next : g_small_head[dev]) = &me;
    g_small_tail[dev] = &me;
    me.cv.wait(l, [&] { return me.admitted; });  // the leaver unlinked us and kept our place
  }
  ~SmallCallGate() {
    if (dev < 0 || kSmallCallers <= 0) return;
    std::lock_guard<std::mutex> l(g_small_mu);
    SmallWaiter* w = g_small_head[dev];
    if (!w) {
      --g_small_inside[dev];
      return;
    }
    g_small_head[dev] = w->next;
    if (!g_small_head[dev]) g_small_tail[dev] = nullptr;
    w->admitted = true;
    w->cv.notify_one();  // under the lock: the waiter's frame outlives this call
  }
  SmallCallGate(const SmallCallGate&) = delete;
  SmallCallGate& operator=(const SmallCallGate&) = delete;
};

}  // namespace

bool eegfx_ctx::mb_ready() {
  if (!mailbox) return false;
  if (mb_stuck) {  // a server that never started: the launch path until it has run and returned
    if (!mb_returned()) return false;
    __atomic_store_n(&mb_host->stop, 0u, __ATOMIC_RELEASE);
    mb_stuck = false;
  }
  if (!mb_slot) {
    if (!mb_acquire(device)) return false;
    mb_slot = true;
  }
  if (!mb_stream) {
    try {
      // A stream of the highest priority: the runtime multiplexes a process's streams of one
      // priority over a few hardware queues, and a queue runs its packets in order, so a
      // normal-priority stream sharing the resident kernel's queue would wait behind it (up to
      // its 1 s idle exit).  The high-priority pool keeps the server on a queue of its own while
      // no more than kMbSlotsPerDevice servers exist.
      int least = 0, greatest = 0;
      HIP_CHECK(hipDeviceGetStreamPriorityRange(&least, &greatest));
      HIP_CHECK(hipStreamCreateWithPriority(&mb_stream, hipStreamNonBlocking, greatest));
      mb_host = (MailboxCmd*)pinned_pool().take(
          sizeof(MailboxCmd), hipHostMallocMapped | hipHostMallocCoherent, &mb_cap);
      memset(mb_host, 0, sizeof(MailboxCmd));
      HIP_CHECK(hipHostGetDevicePointer((void**)&mb_dev, mb_host, 0));
      mb_seq = 0;
    } catch (...) {
      release_mailbox();
      mailbox = true;  // still enabled: later calls retry
      throw;
    }
  }
  const auto now = std::chrono::steady_clock::now();
  // no request for 500 ms: the server may be close to its 1 s idle exit -- restart it, so no
  // request is ever posted to a kernel that is returning
  if (mb_live && now - mb_last > std::chrono::milliseconds(500)) {
    if (!mb_stop()) return false;
  }
  if (!mb_live) {
    mb_launch();
    mb_last = now;
  }
  if (!mb_started) {
    const auto t0 = std::chrono::steady_clock::now();
    while (__atomic_load_n(&mb_host->alive, __ATOMIC_ACQUIRE) != mb_gen) {
      if (std::chrono::steady_clock::now() - t0 > kMbStartWait) {
        // still queued: it returns at once when it runs (stop), the call takes the launch path
        __atomic_store_n(&mb_host->stop, 1u, __ATOMIC_RELEASE);
        mb_live = false;
        mb_stuck = true;
        return false;
      }
      __builtin_ia32_pause();
    }
    mb_started = true;
  }
  return true;
}

void eegfx_ctx::release_mailbox() {
  const bool stopped = mb_stop();
  if (mb_stream && stopped && !mb_stuck) (void)hipStreamDestroy(mb_stream);
  if (mb_host && stopped && !mb_stuck)
    pinned_pool().give(mb_host, mb_cap, hipHostMallocMapped | hipHostMallocCoherent);
  // a stuck server keeps its stream and command block (it still reads `stop` when it runs):
  // leaked rather than freed under a queued kernel
  mb_host = nullptr;
  mb_dev = nullptr;
  mb_stream = nullptr;
  mb_live = mb_started = mb_stuck = false;
  if (mb_slot) mb_release(device);
  mb_slot = false;
  mailbox = false;
}

namespace {

void* stage_in(eegfx_ctx* ctx, DevBuf& buf, const void* src, size_t bytes, int mem) {
  if (mem == EEGFX_MEM_DEVICE) return const_cast<void*>(src);
  void* d = buf.get(bytes);
  if (bytes) HIP_CHECK(hipMemcpyAsync(d, src, bytes, hipMemcpyHostToDevice, ctx->stream));
  return d;
}

// Host copy into pinned staging, split over up to 8 threads (one thread tops out near 6 GB/s,
// far below the ~57 GB/s host link it feeds).
void parallel_memcpy(void* dst, const void* src, size_t bytes) {
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const size_t nt = std::min<size_t>({8, hw, std::max<size_t>(1, bytes >> 23)});
  if (nt <= 1) {
    memcpy(dst, src, bytes);
    return;
  }
  std::vector<std::thread> th;
  const size_t per = (bytes / nt + 63) & ~(size_t)63;
  for (size_t t = 0; t < nt; ++t) {
    const size_t a = t * per;
    if (a >= bytes) break;
    const size_t len = std::min(per, bytes - a);
    th.emplace_back([=] { memcpy((char*)dst + a, (const char*)src + a, len); });
  }
  for (auto& x : th) x.join();
}

// The processors this process may run on, as the JVM's Runtime.availableProcessors() counts them
// (Spark local[*]'s defaultParallelism, SparkInitializer.java:44): the affinity mask, capped by a
// cgroup CPU quota (cgroup v2 cpu.max or v1 cfs_quota_us / cfs_period_us), at least 1.
// std::thread::hardware_concurrency() counts every online CPU of the machine instead.
int available_processors() {
  int n = 0;
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
  if (n < 1) n = (int)std::max(1u, std::thread::hardware_concurrency());
  auto cap = [&](double quota, double period) {
    if (quota > 0 && period > 0) n = std::min(n, std::max(1, (int)std::ceil(quota / period)));
  };
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    char q[32] = {0};
    double period = 0;
    if (fscanf(f, "%31s %lf", q, &period) == 2 && strcmp(q, "max") != 0) cap(atof(q), period);
    fclose(f);
  } else if (FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    double quota = -1, period = 0;
    if (fscanf(fq, "%lf", &quota) != 1) quota = -1;
    fclose(fq);
    if (FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(fp, "%lf", &period) != 1) period = 0;
      fclose(fp);
    }
    cap(quota, period);
  }
  return n;
}

// Joins the threads it holds when it goes out of scope (an exception from emplace_back or from a
// later call leaves no joinable std::thread behind, which would call std::terminate).
struct Joiner {
  std::vector<std::thread> th;
  ~Joiner() {
    for (auto& t : th)
      if (t.joinable()) t.join();
  }
};

// Host batches up to this many window bytes go through the zero-copy path of
// eegfx_extract_features_f64 (about 64 epochs of 3 channels).
constexpr size_t kZeroCopyBytes = (size_t)768 << 10;
// the rows of the largest such batch: 192 window rows of 512 doubles, 16 features each
constexpr size_t kZeroCopyOutBytes =
    kZeroCopyBytes / (sizeof(double) * EEGFX_DWT8_EPOCH_SIZE) * EEGFX_DWT8_FEATURE_SIZE * sizeof(double);

void check_mem(int mem) {
  if (mem != EEGFX_MEM_HOST && mem != EEGFX_MEM_DEVICE) fail(EEGFX_EINVAL, "mem flag %d", mem);
}

// raw -> features on the context stream (device pointers).  Fused kernel when one covers the
// layout, otherwise cut + features through the context scratch buffer.
void run_features_from_raw(eegfx_ctx* ctx, const void* raw, int fmt, int64_t n_frames, int ct,
                           const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                           double* out) {
  const bool fast = ctx->numerics != EEGFX_EXACT;
  // fma: rows that fail the conditioning guard (guard.h) are recomputed under EXACT -- inside the
  // kernel that flags them, or (the generic any-layout kernels) by a follow-up launch over the
  // guard list that launch_window_wide issues; baseline_any_kernel zeroes the list's count
  const Guard g = ctx->guard_for(n);
  if (fused_supported(fmt, ct, C, out)) {
    void* fscratch = ctx->fused.get(fused_scratch_bytes(n, C));
    HIP_CHECK(launch_fused_baseline(ctx->stream, raw, n_frames, ct, sel, C, pos, n, fscratch,
                                    ctx->err_dev, nullptr, fast ? &g : nullptr));
    ctx->tic();  // the dominant kernel (DESIGN.md "Measurement")
    HIP_CHECK(launch_fused_window(ctx->stream, raw, n_frames, ct, sel, C, pos, n, fast, fscratch,
                                  out, g, fast && ctx->guard_track()));
    ctx->toc(n * fused_window_bytes_per_epoch(ct, C));
    return;
  }
  if (wide_supported(fmt, ct, C)) {
    void* fscratch = ctx->fused.get(fused_scratch_bytes(n, C));
    HIP_CHECK(launch_baseline_any(ctx->stream, raw, fmt, n_frames, ct, sel, C, pos, n, fscratch,
                                  ctx->err_dev, g.count, fast ? &g : nullptr));
    ctx->tic();
    HIP_CHECK(launch_window_wide(ctx->stream, raw, fmt, n_frames, ct, sel, C, pos, n, fast,
                                 fscratch, out, g, fast && ctx->guard_track()));
    const int64_t elem = fmt == EEGFX_INT_16 ? 2 : 4;
    ctx->toc(n * (EEGFX_DWT8_EPOCH_SIZE * ct * elem + C * 4 + 8 + C * 16 * 8));
    return;
  }
  double* ep = (double*)ctx->scratch.get(sizeof(double) * (size_t)n * C * EEGFX_POSTSTIMULUS);
  ctx->tic();
  HIP_CHECK(launch_cut_epochs(ctx->stream, raw, fmt, n_frames, ct, sel, C, pos, n, ep,
                              ctx->fused.get(fused_scratch_bytes(n, C)), ctx->err_dev));
  HIP_CHECK(launch_features_from_epochs(ctx->stream, ep, n, C, EEGFX_DWT8_SKIP,
                                        EEGFX_DWT8_FEATURE_SIZE, fast, out, EEGFX_POSTSTIMULUS, g));
  ctx->toc(0);
}

// raw -> epochs + features (device pointers): the one-pass kernels when the layout fits them,
// else the cut pass followed by the batch extract over the rows it wrote.
void run_epochs_and_features(eegfx_ctx* ctx, const void* raw, int fmt, int64_t n_frames, int ct,
                             const ChanSel& sel, int C, const int64_t* pos, int64_t n, double* ep,
                             double* feat) {
  const bool fast = ctx->numerics != EEGFX_EXACT;
  const Guard g = ctx->guard_for(n);
  void* fscratch = ctx->fused.get(fused_scratch_bytes(n, C));
  ctx->tic();
  if (cut_features_supported(fmt, ct, C, raw, ep, feat)) {
    HIP_CHECK(launch_cut_features(ctx->stream, raw, fmt, n_frames, ct, sel, C, pos, n, ep, feat,
                                  fast, fscratch, ctx->err_dev, g));
  } else {
    HIP_CHECK(launch_cut_epochs(ctx->stream, raw, fmt, n_frames, ct, sel, C, pos, n, ep, fscratch,
                                ctx->err_dev));
    HIP_CHECK(launch_features_from_epochs(ctx->stream, ep, n, C, EEGFX_DWT8_SKIP,
                                          EEGFX_DWT8_FEATURE_SIZE, fast, feat, EEGFX_POSTSTIMULUS,
                                          g));
  }
  ctx->toc(0);
}

}  // namespace

// ================================================================================================
// OffLineDataProvider
// ================================================================================================
struct eegfx_odp {
  eegfx_ctx* ctx = nullptr;
  std::vector<std::string> args;
  std::string error;
  // Map<String, Integer> files = new LinkedHashMap<>() (:54): insertion order, put() on an
  // existing key keeps the position and replaces the value.
  std::vector<std::pair<std::string, int32_t>> files;
  std::string file_prefix;
  std::string vhdr_file, vmrk_file, eeg_file;
  int32_t fz_index = 0, cz_index = 0, pz_index = 0;  // fields: persist across files (:49-51)
  int64_t balance = 0;                                // numberOfTargets - numberOfNonTargets
  int64_t epochs_counter = 0;
  std::vector<double> labels;
  std::vector<int64_t> positions;
  std::vector<int32_t> file_of_epoch;
  void* d_epochs = nullptr;  // double[n][3][750], resident (hipMalloc, grown copy-on-grow)
  size_t d_epochs_cap = 0;
  int64_t n_epochs = 0;
  // dwt-8 rows of the epochs, double[n][48], computed in the same pass as the epochs
  // (eegfx_process_recording_epochs) under the numerics of the load; getFeatures() with the
  // reference's parameters (8, 512, 175, 16) under the same numerics is then a copy
  void* d_features = nullptr;
  size_t d_features_cap = 0;
  int features_numerics = -1;  // -1: no resident rows (not all epochs have them)

  void put_file(const std::string& k, int32_t v) {
    for (auto& kv : files)
      if (kv.first == k) {
        kv.second = v;
        return;
      }
    files.emplace_back(k, v);
  }

  static bool ends_with_4(const std::string& s, const char* suf) {
    // fileLocation.substring(fileLocation.length() - 4): StringIndexOutOfBounds below 4 chars.
    if (s.size() < 4) fail(EEGFX_EINVAL, "String index out of range: %d", (int)s.size() - 4);
    return s.compare(s.size() - 4, 4, suf) == 0;
  }

  void handle_input() {  // :111-141
    if (args.empty() || args.size() > 6)
      fail(EEGFX_EINVAL,
           "Please enter the input in one of these formats: 1. <location of info.txt file> "
           "2. <location of a .eeg file> <guessed number>  *<optional values>");
    const std::string& loc = args[0];
    if (ends_with_4(loc, ".eeg")) {
      file_prefix = "";
      if (args.size() < 2) fail(EEGFX_EINVAL, "Index 1 out of bounds for length 1");
      int32_t g;
      if (!java_parse_int(args[1], &g))
        fail(EEGFX_EFORMAT, "For input string: \"%s\"", args[1].c_str());
      put_file(loc, g);
    } else if (ends_with_4(loc, ".txt")) {
      const size_t slash = loc.rfind('/');
      if (slash == std::string::npos) fail(EEGFX_EINVAL, "String index out of range: -1");
      file_prefix = loc.substr(0, slash) + "/";
      load_files_from_info_txt(loc);
    } else {
      fail(EEGFX_EINVAL,
           "Please enter the input in one of these formats: 1. <location of info.txt file> "
           "2. <location of a .eeg file> <target number>  *<optional values>");
    }
  }

  void load_files_from_info_txt(const std::string& loc) {  // :283-319
    FILE* f = fopen(loc.c_str(), "rb");
    if (!f) fail(EEGFX_EIO, "File %s does not exist", loc.c_str());
    std::string text;
    char buf[4096];
    size_t r;
    while ((r = fread(buf, 1, sizeof(buf), f)) > 0) text.append(buf, r);
    fclose(f);
    std::vector<std::string> lines;
    std::string cur;
    for (size_t i = 0; i < text.size(); ++i) {  // BufferedReader.readLine
      const char ch = text[i];
      if (ch == '\n' || ch == '\r') {
        lines.push_back(cur);
        cur.clear();
        if (ch == '\r' && i + 1 < text.size() && text[i + 1] == '\n') ++i;
      } else {
        cur.push_back(ch);
      }
    }
    if (!cur.empty()) lines.push_back(cur);
    for (const std::string& line : lines) {
      if (line.empty() || line[0] == '#') continue;
      std::vector<std::string> parts = java_split_space(line);
      if (parts.size() > 1) {
        int32_t num;
        if (!java_parse_int(parts[1], &num))
          fail(EEGFX_EFORMAT, "Line %s contains an improper number format", line.c_str());
        put_file(parts[0], num);
      }
    }
  }

  // setFileNames (:327-365): false = the reference's caught IllegalArgumentException (skip file).
  bool set_file_names(const std::string& loc, std::string* why) {
    if (loc.size() <= 4) {
      *why = "Incorrect file name, must be at least longer than 4 characters ";
      return false;
    }
    if (loc.compare(loc.size() - 4, 4, ".eeg") != 0) {
      *why = "Invalid .eeg file";
      return false;
    }
    const std::string base = loc.substr(0, loc.rfind('.'));
    const std::string vhdr = base + ".vhdr", vmrk = base + ".vmrk";
    if (!file_exists(vhdr)) {
      *why = "No related .vhdr file found for the original .eeg file " + vhdr;
      return false;
    }
    if (!file_exists(vmrk)) {
      *why = "No related .vmrk file found for the original .eeg file " + vmrk;
      return false;
    }
    if (!file_exists(loc)) {
      *why = "No related .eeg file found for the original .eeg file " + loc;
      return false;
    }
    vhdr_file = vhdr;
    vmrk_file = vmrk;
    eeg_file = loc;
    return true;
  }

  void append_epochs(const Header& h, int64_t n_frames, const void* d_raw,
                     const std::vector<int64_t>& pos, int32_t file_idx,
                     const std::vector<double>& lab) {
    const int64_t k = (int64_t)pos.size();
    if (k == 0) return;
    if (!ctx) {  // planning-only provider: selection, labels and offsets without epochs
      n_epochs += k;
      positions.insert(positions.end(), pos.begin(), pos.end());
      labels.insert(labels.end(), lab.begin(), lab.end());
      file_of_epoch.insert(file_of_epoch.end(), (size_t)k, file_idx);
      return;
    }
    const int ct = h.info.n_channels;
    int32_t cols[3];
    float res[3];
    const int32_t idx[3] = {fz_index, cz_index, pz_index};
    for (int c = 0; c < 3; ++c) {
      cols[c] = idx[c] - 1;
      res[c] = 1.0f;
      for (const auto& ci : h.channels)
        if (ci.number == idx[c]) res[c] = (float)ci.resolution;
    }
    const ChanSel sel = make_sel(cols, res, 3, ct);
    const size_t per = sizeof(double) * 3 * EEGFX_POSTSTIMULUS;
    // grow the resident epoch buffer (copy-on-grow)
    const size_t need = per * (size_t)(n_epochs + k);
    if (need > d_epochs_cap) {
      size_t cap = std::max(need, d_epochs_cap * 2);
      void* np = nullptr;
      HIP_CHECK(hipMallocAsync(&np, cap, ctx->stream));
      if (n_epochs)
        HIP_CHECK(hipMemcpyAsync(np, d_epochs, per * (size_t)n_epochs, hipMemcpyDeviceToDevice,
                                 ctx->stream));
      if (d_epochs) HIP_CHECK(hipFreeAsync(d_epochs, ctx->stream));
      d_epochs = np;
      d_epochs_cap = cap;
    }
    const size_t fper = sizeof(double) * 3 * EEGFX_DWT8_FEATURE_SIZE;
    const size_t fneed = fper * (size_t)(n_epochs + k);
    if (fneed > d_features_cap) {
      size_t cap = std::max(fneed, d_features_cap * 2);
      void* np = nullptr;
      HIP_CHECK(hipMallocAsync(&np, cap, ctx->stream));
      if (n_epochs && features_numerics >= 0)
        HIP_CHECK(hipMemcpyAsync(np, d_features, fper * (size_t)n_epochs, hipMemcpyDeviceToDevice,
                                 ctx->stream));
      if (d_features) HIP_CHECK(hipFreeAsync(d_features, ctx->stream));
      d_features = np;
      d_features_cap = cap;
    }
    int64_t* d_pos = (int64_t*)ctx->pos.get(sizeof(int64_t) * (size_t)k);
    HIP_CHECK(hipMemcpyAsync(d_pos, pos.data(), sizeof(int64_t) * (size_t)k,
                             hipMemcpyHostToDevice, ctx->stream));
    // getData()'s epochs and their dwt-8 rows in one pass over each epoch's frames
    run_epochs_and_features(ctx, d_raw, h.info.binary_format, n_frames, ct, sel, 3, d_pos, k,
                            (double*)((char*)d_epochs + per * (size_t)n_epochs),
                            (double*)((char*)d_features + fper * (size_t)n_epochs));
    if (n_epochs == 0) features_numerics = ctx->numerics;
    else if (features_numerics != ctx->numerics) features_numerics = -1;
    ctx->drain();
    n_epochs += k;
    positions.insert(positions.end(), pos.begin(), pos.end());
    labels.insert(labels.end(), lab.begin(), lab.end());
    file_of_epoch.insert(file_of_epoch.end(), (size_t)k, file_idx);
  }

  void process_eeg_files() {  // :147-268
    int32_t file_idx = -1;
    for (const auto& entry : files) {
      ++file_idx;
      std::string why;
      if (!set_file_names(file_prefix + entry.first, &why)) continue;  // logged + skipped (:157-161)
      const Header h = read_header(vhdr_file);
      for (const auto& ch : h.channels) {  // :172-183
        std::string name = ch.name;
        for (auto& c : name) c = (char)tolower((unsigned char)c);
        if (name == "fz") fz_index = ch.number;
        else if (name == "cz") cz_index = ch.number;
        if (name == "pz") pz_index = ch.number;
      }
      const int32_t sel[3] = {fz_index, cz_index, pz_index};
      for (int c = 0; c < 3; ++c)
        if (sel[c] < 1 || sel[c] > h.info.n_channels)
          fail(EEGFX_EINVAL, "%s: channel %s not found (index %d)", vhdr_file.c_str(),
               c == 0 ? "Fz" : c == 1 ? "Cz" : "Pz", sel[c]);
      const int64_t n_frames = recording_frames(h, eeg_file);
      const size_t raw_bytes =
          (size_t)n_frames * h.info.n_channels * sample_bytes(h.info.binary_format);
      void* d_raw = nullptr;
      if (ctx) {  // planning-only providers (no context) never touch the recording payload
        std::vector<char> host(raw_bytes);
        read_recording(h, eeg_file, host.data(), n_frames);
        d_raw = ctx->raw.get(raw_bytes);
        HIP_CHECK(hipMemcpyAsync(d_raw, host.data(), raw_bytes, hipMemcpyHostToDevice,
                                 ctx->stream));
      }

      const std::vector<eegfx_marker> markers = read_markers(vmrk_file);
      std::vector<int64_t> pos(markers.size());
      std::vector<double> lab(markers.size());
      int64_t k = 0;
      const int rc = eegfx_plan_markers(markers.data(), (int64_t)markers.size(), n_frames,
                                        entry.second, &balance, pos.data(), lab.data(), &k);
      pos.resize((size_t)k);
      lab.resize((size_t)k);
      epochs_counter += k;
      append_epochs(h, n_frames, d_raw, pos, file_idx, lab);  // epochs accepted before an error
      if (rc != EEGFX_OK) fail(rc, "%s", last_error().c_str());
    }
  }
};

namespace eegfx {
int ctx_device(const eegfx_ctx* ctx) { return ctx->device; }
void* ctx_stream(const eegfx_ctx* ctx) { return (void*)ctx->stream; }
}  // namespace eegfx

extern "C" {

const char* eegfx_version(void) { return "eegfx 0.1.0 (gfx950)"; }

int eegfx_device_count(int* count) {
  return guarded([&] {
    if (!count) fail(EEGFX_EINVAL, "null argument");
    HIP_CHECK(hipGetDeviceCount(count));
  });
}

int eegfx_ctx_create(int device, eegfx_ctx** out) {
  return guarded([&] {
    if (!out) fail(EEGFX_EINVAL, "null argument");
    std::unique_ptr<eegfx_ctx> c(new eegfx_ctx());
    c->device = device;
    c->activate();
    HIP_CHECK(hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking));
    c->stream = c->own;
    c->bind_buffers();
    c->err_host = (int*)pinned_pool().take(16, hipHostMallocMapped, &c->err_cap);
    memset(c->err_host, 0, 16);  // the error word, then (+8) the guard strategy word
    HIP_CHECK(hipHostGetDevicePointer((void**)&c->err_dev, c->err_host, 0));
    // stream-ordered: no allocation or free of a context synchronises the device
    HIP_CHECK(hipMallocAsync((void**)&c->guard_dev, eegfx_ctx::kGuardDevBytes, c->own));
    HIP_CHECK(hipMemsetAsync(c->guard_dev, 0, eegfx_ctx::kGuardDevBytes, c->own));
    HIP_CHECK(hipStreamSynchronize(c->own));
    *out = c.release();
  });
}

int eegfx_ctx_set_stream(eegfx_ctx* ctx, void* hip_stream) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    const hipStream_t next = hip_stream ? (hipStream_t)hip_stream : ctx->own;
    if (next == ctx->stream) return;
    // the context's buffers are ordered on its stream: drain the old one before switching
    ctx->activate();
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->stream = next;
  });
}

int eegfx_ctx_stream(eegfx_ctx* ctx, void** hip_stream) {
  return guarded([&] {
    if (!ctx || !hip_stream) fail(EEGFX_EINVAL, "null argument");
    *hip_stream = (void*)ctx->stream;
  });
}

int eegfx_ctx_set_numerics(eegfx_ctx* ctx, int numerics) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    if (numerics != EEGFX_EXACT && numerics != EEGFX_FMA)
      fail(EEGFX_EINVAL, "numerics %d", numerics);
    ctx->numerics = numerics;
  });
}

int eegfx_ctx_set_timing(eegfx_ctx* ctx, int enable) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    ctx->activate();
    HIP_CHECK(hipStreamSynchronize(ctx->stream));
    ctx->timing = enable != 0;
    ctx->n_timed = 0;  // events are reused
  });
}

int eegfx_ctx_set_mailbox(eegfx_ctx* ctx, int enable) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    ctx->activate();
    if (!enable) {
      ctx->release_mailbox();
      return;
    }
    if (ctx->mailbox) return;
    // the small-call staging at its largest before any server is launched on it: a server reads
    // the buffers it was launched with, so growing them on a later call stopped and restarted it
    // (with a pinned allocation: the 3-4 ms first calls of tools/mailbox_threads at 16-32 threads)
    (void)ctx->pin_in.get(kZeroCopyBytes);
    (void)ctx->pin_out.get(kZeroCopyOutBytes);
    ctx->mailbox = true;  // the server starts on the first one-epoch call that gets a slot
    (void)ctx->mb_ready();
  });
}

int eegfx_ctx_get_mailbox(eegfx_ctx* ctx, int32_t* enabled, int32_t* resident) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    if (enabled) *enabled = ctx->mailbox ? 1 : 0;
    if (resident) *resident = ctx->mailbox && ctx->mb_slot && ctx->mb_live && ctx->mb_started ? 1 : 0;
  });
}

int eegfx_ctx_synchronize(eegfx_ctx* ctx) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    ctx->activate();
    ctx->drain();
  });
}

int eegfx_ctx_guard_detail(eegfx_ctx* ctx, int64_t* rows_checked, int64_t* rows_rechecked,
                           int64_t* rows_recomputed, int reset) {
  return guarded([&] {
    if (!ctx || !rows_checked || !rows_recomputed) fail(EEGFX_EINVAL, "null argument");
    ctx->activate();
    // the two slot arrays and, right behind them, Guard::adapt (strategy, rechecked offset, rows)
    std::vector<unsigned long long> slots(2 * kGuardSlots * kGuardSlotWords + 3);
    HIP_CHECK(hipMemcpyAsync(slots.data(), ctx->guard_recomputed_slots(),
                             2 * kGuardSlotBytes + 3 * sizeof(unsigned long long),
                             hipMemcpyDeviceToHost, ctx->stream));
    ctx->drain();
    unsigned long long tot[2] = {0, 0};  // recomputed, rechecked
    for (int k = 0; k < 2; ++k)
      for (int i = 0; i < kGuardSlots; ++i) tot[k] += slots[(size_t)(k * kGuardSlots + i) * kGuardSlotWords];
    *rows_checked = ctx->guard_checked;
    *rows_recomputed = (int64_t)tot[0];
    if (rows_rechecked) *rows_rechecked = (int64_t)tot[1];
    if (reset) {
      // the adaptive strategy's offset moves with the cleared total (fused.hip baseline_kernel)
      const unsigned long long off =
          (unsigned long long)((long long)slots[2 * kGuardSlots * kGuardSlotWords + 1] - (long long)tot[1]);
      HIP_CHECK(hipMemsetAsync(ctx->guard_recomputed_slots(), 0, 2 * kGuardSlotBytes, ctx->stream));
      HIP_CHECK(hipMemcpyAsync(ctx->guard_adapt() + 1, &off, sizeof off, hipMemcpyHostToDevice,
                               ctx->stream));
      ctx->drain();
      ctx->guard_checked = 0;
    }
  });
}

int eegfx_ctx_guard_stats(eegfx_ctx* ctx, int64_t* rows_checked, int64_t* rows_recomputed,
                          int reset) {
  return eegfx_ctx_guard_detail(ctx, rows_checked, nullptr, rows_recomputed, reset);
}

int eegfx_ctx_kernel_stats(eegfx_ctx* ctx, int64_t* launches, double* total_ms,
                           int64_t* total_bytes) {
  return guarded([&] {
    if (!ctx || !launches || !total_ms || !total_bytes) fail(EEGFX_EINVAL, "null argument");
    double ms = 0.0;
    int64_t bytes = 0;
    for (size_t i = 0; i < ctx->n_timed; ++i) {
      float t = 0.0f;
      HIP_CHECK(hipEventSynchronize(ctx->events[i].second));
      HIP_CHECK(hipEventElapsedTime(&t, ctx->events[i].first, ctx->events[i].second));
      ms += t;
      bytes += ctx->event_bytes[i];
    }
    *launches = (int64_t)ctx->n_timed;
    *total_ms = ms;
    *total_bytes = bytes;
  });
}

int eegfx_ctx_destroy(eegfx_ctx* ctx) {
  return guarded([&] {
    if (!ctx) return;
    (void)hipSetDevice(ctx->device);
    ctx->release_mailbox();  // before anything that synchronises the whole device
    (void)hipStreamSynchronize(ctx->stream);
    ctx->release_buffers();
    (void)hipStreamSynchronize(ctx->stream);
    (void)hipStreamSynchronize(ctx->own);
    pinned_pool().give(ctx->err_host, ctx->err_cap, hipHostMallocMapped);
    if (ctx->guard_dev) (void)hipFreeAsync(ctx->guard_dev, ctx->own);
    (void)hipStreamSynchronize(ctx->own);
    ctx->release_stream_resources();
    ctx->destroy_events();
    (void)hipStreamDestroy(ctx->own);
    delete ctx;
  });
}

int eegfx_read_raw(eegfx_ctx* ctx, const char* vhdr_path, const char* eeg_path, void* dst,
                   int64_t capacity_bytes, int mem) {
  return guarded([&] {
    if (!vhdr_path || !eeg_path || !dst) fail(EEGFX_EINVAL, "null argument");
    check_mem(mem);
    const Header h = read_header(vhdr_path);
    const int64_t n = recording_frames(h, eeg_path);
    const int64_t bytes = n * h.info.n_channels * sample_bytes(h.info.binary_format);
    if (bytes > capacity_bytes)
      fail(EEGFX_EINVAL, "capacity %lld < %lld bytes", (long long)capacity_bytes, (long long)bytes);
    if (mem == EEGFX_MEM_HOST) {
      read_recording(h, eeg_path, dst, n);
    } else {
      if (!ctx) fail(EEGFX_EINVAL, "device read needs a context");
      ctx->activate();
      std::vector<char> host((size_t)bytes);
      read_recording(h, eeg_path, host.data(), n);
      HIP_CHECK(hipMemcpyAsync(dst, host.data(), (size_t)bytes, hipMemcpyHostToDevice, ctx->stream));
      ctx->drain();
    }
  });
}

int eegfx_cut_epochs_f64(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                         int32_t ct, const int32_t* cols, const float* res, int32_t C,
                         const int64_t* pos, int64_t n, double* epochs_out, int mem) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    check_mem(mem);
    if (fmt != EEGFX_INT_16 && fmt != EEGFX_IEEE_FLOAT_32) fail(EEGFX_EINVAL, "format %d", fmt);
    if (n_frames < 0 || n < 0 || ct < 1) fail(EEGFX_EINVAL, "negative size");
    if (n > 0 && (!raw || !pos || !epochs_out)) fail(EEGFX_EINVAL, "null buffer");
    const ChanSel sel = make_sel(cols, res, C, ct);
    if (mem == EEGFX_MEM_HOST) check_positions(pos, n, n_frames);
    if (n == 0) return;
    ctx->activate();
    const size_t raw_bytes = (size_t)n_frames * ct * (fmt == EEGFX_INT_16 ? 2 : 4);
    const size_t out_bytes = sizeof(double) * (size_t)n * C * EEGFX_POSTSTIMULUS;
    const void* d_raw = stage_in(ctx, ctx->raw, raw, raw_bytes, mem);
    const int64_t* d_pos = (const int64_t*)stage_in(ctx, ctx->pos, pos, sizeof(int64_t) * n, mem);
    double* d_out = mem == EEGFX_MEM_DEVICE ? epochs_out : (double*)ctx->out.get(out_bytes);
    ctx->tic();
    HIP_CHECK(launch_cut_epochs(ctx->stream, d_raw, fmt, n_frames, ct, sel, C, d_pos, n, d_out,
                                ctx->fused.get(fused_scratch_bytes(n, C)), ctx->err_dev));
    ctx->toc(0);
    if (mem == EEGFX_MEM_HOST) {
      HIP_CHECK(hipMemcpyAsync(epochs_out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
      ctx->drain();
    }
  });
}

int eegfx_extract_features_f64(eegfx_ctx* ctx, const double* epochs, int64_t n, int32_t C,
                               int32_t name, int32_t epoch_size, int32_t skip,
                               int32_t feature_size, double* out, int mem) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    check_mem(mem);
    check_fe_params(C, name, epoch_size, skip, feature_size);
    if (n < 0) fail(EEGFX_EINVAL, "negative count");
    if (n == 0) return;
    if (!epochs || !out) fail(EEGFX_EINVAL, "null buffer");
    ctx->activate();
    const size_t in_bytes = sizeof(double) * (size_t)n * C * EEGFX_POSTSTIMULUS;
    const size_t out_bytes = sizeof(double) * (size_t)n * C * feature_size;
    if (mem == EEGFX_MEM_HOST) {
      // Host epochs (the JNI drop-in, IFeatureExtraction.extractFeatures called once per epoch
      // from Spark map closures, LogisticRegressionClassifier.java:55-61, or serial loops,
      // NeuralNetworkClassifier.java:78-86).  Only the window columns [skip, skip+512) of each row
      // are needed (4,096 of 6,000 bytes).
      const size_t row_w = sizeof(double) * EEGFX_DWT8_EPOCH_SIZE;
      const size_t row_p = sizeof(double) * EEGFX_POSTSTIMULUS;
      const uint8_t* src = (const uint8_t*)epochs + sizeof(double) * (size_t)skip;
      if ((size_t)n * C * row_w <= kZeroCopyBytes && features_small_supported(C)) {
        // Small batches (a single epoch above all): latency, not bandwidth.  The window rows are
        // packed into a pinned, device-mapped buffer by the calling thread and the kernel
        // (features_small_kernel) reads them -- and writes the rows -- across the host link
        // directly: one launch and one stream sync, no DMA transfers (each costs a copy-engine
        // round trip) and no allocation once the context's staging has grown.  The rows are EXACT
        // under both numerics (kernels.hip small_epoch), so the fma guard does not count them.
        // a resident server reads the staging it was launched with: stop it before a growth
        // (the next request restarts it on the new buffers)
        if (ctx->mb_live && ((size_t)n * C * row_w > ctx->pin_in.cap || out_bytes > ctx->pin_out.cap))
          ctx->mb_stop();
        double* hin = (double*)ctx->pin_in.get((size_t)n * C * row_w);
        double* hout = (double*)ctx->pin_out.get(out_bytes);
        for (int64_t r = 0; r < n * C; ++r)
          memcpy((uint8_t*)hin + (size_t)r * row_w, src + (size_t)r * row_p, row_w);
        // The resident server (no launch, no stream sync) takes single epochs: it serves a
        // request's epochs one after another (~7 us each), where a launch runs them on a
        // workgroup each (11 epochs: ~20 us launched against ~80 us served).
        if (n == 1 && ctx->mb_ready()) {
          ctx->mb_serve(n, C, feature_size);
          ctx->check_positions_flag();  // as every synchronising call (the launch path below)
          memcpy(out, hout, out_bytes);
          return;
        }
#if EEGFX_GATE_LAUNCH_ONLY
        {
          SmallCallGate gate(ctx->device);
          ctx->tic();
          HIP_CHECK(launch_features_small(ctx->stream, (const double*)ctx->pin_in.device_ptr(), n,
                                          C, feature_size, (double*)ctx->pin_out.device_ptr()));
          ctx->toc(0);
          ctx->record_small();
        }
        ctx->wait_small(true);
#else
        SmallCallGate gate(ctx->device);
        ctx->tic();
        HIP_CHECK(launch_features_small(ctx->stream, (const double*)ctx->pin_in.device_ptr(), n, C,
                                        feature_size, (double*)ctx->pin_out.device_ptr()));
        ctx->toc(0);
        ctx->wait_small();
#endif
        ctx->check_positions_flag();
        memcpy(out, hout, out_bytes);
        return;
      }
      // Large batches: strided 2D copies of the window columns in chunks, each followed by its
      // kernels on the same stream (the kernels are ~3 % of a chunk's copy).  Measured with 100k
      // epochs: 4.2e6 epochs/s against 3.0e6 for copying the whole 18 KB epochs and a 4.6e6
      // host-link bound; packing the rows with host threads into pinned staging first was slower
      // (2.8e6).
      constexpr int64_t kChunk = 8192;  // epochs per chunk
      const size_t chunk_bytes = (size_t)std::min<int64_t>(n, kChunk) * C * row_w;
      uint8_t* dwin = (uint8_t*)ctx->scratch.get(chunk_bytes);
      double* d_out = (double*)ctx->out.get(out_bytes);
      const Guard g = ctx->guard_for(n);
      ctx->tic();
      for (int64_t e0 = 0; e0 < n; e0 += kChunk) {
        const int64_t m = std::min<int64_t>(kChunk, n - e0);
        HIP_CHECK(hipMemcpy2DAsync(dwin, row_w, src + (size_t)e0 * C * row_p, row_p, row_w,
                                   (size_t)(m * C), hipMemcpyHostToDevice, ctx->stream));
        double* rows = d_out + e0 * C * feature_size;
        HIP_CHECK(launch_features_from_epochs(ctx->stream, (const double*)dwin, m, C, 0,
                                              feature_size, ctx->numerics != EEGFX_EXACT, rows,
                                              EEGFX_DWT8_EPOCH_SIZE, g));
      }
      ctx->toc(0);
      HIP_CHECK(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
      ctx->drain();
      return;
    }
    const double* d_in = (const double*)stage_in(ctx, ctx->scratch, epochs, in_bytes, mem);
    double* d_out = mem == EEGFX_MEM_DEVICE ? out : (double*)ctx->out.get(out_bytes);
    const Guard g = ctx->guard_for(n);
    ctx->tic();
    HIP_CHECK(launch_features_from_epochs(ctx->stream, d_in, n, C, skip, feature_size,
                                          ctx->numerics != EEGFX_EXACT, d_out, EEGFX_POSTSTIMULUS,
                                          g));
    ctx->toc(0);
    if (mem == EEGFX_MEM_HOST) {
      HIP_CHECK(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
      ctx->drain();
    }
  });
}

int eegfx_process_recording(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                            int32_t ct, const int32_t* cols, const float* res, int32_t C,
                            const int64_t* pos, int64_t n, double* features, int mem) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    check_mem(mem);
    if (fmt != EEGFX_INT_16 && fmt != EEGFX_IEEE_FLOAT_32) fail(EEGFX_EINVAL, "format %d", fmt);
    if (n_frames < 0 || n < 0 || ct < 1) fail(EEGFX_EINVAL, "negative size");
    if (n > 0 && (!raw || !pos || !features)) fail(EEGFX_EINVAL, "null buffer");
    const ChanSel sel = make_sel(cols, res, C, ct);
    if (mem == EEGFX_MEM_HOST) check_positions(pos, n, n_frames);
    if (n == 0) return;
    ctx->activate();
    const size_t raw_bytes = (size_t)n_frames * ct * (fmt == EEGFX_INT_16 ? 2 : 4);
    const size_t out_bytes = sizeof(double) * (size_t)n * C * EEGFX_DWT8_FEATURE_SIZE;
    const void* d_raw = stage_in(ctx, ctx->raw, raw, raw_bytes, mem);
    const int64_t* d_pos = (const int64_t*)stage_in(ctx, ctx->pos, pos, sizeof(int64_t) * n, mem);
    double* d_out = mem == EEGFX_MEM_DEVICE ? features : (double*)ctx->out.get(out_bytes);
    run_features_from_raw(ctx, d_raw, fmt, n_frames, ct, sel, C, d_pos, n, d_out);
    if (mem == EEGFX_MEM_HOST) {
      HIP_CHECK(hipMemcpyAsync(features, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
      ctx->drain();
    }
  });
}

int eegfx_process_recording_epochs(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                                   int32_t ct, const int32_t* cols, const float* res, int32_t C,
                                   const int64_t* pos, int64_t n, double* features,
                                   double* epochs_out, int mem) {
  if (!epochs_out)
    return eegfx_process_recording(ctx, raw, fmt, n_frames, ct, cols, res, C, pos, n, features,
                                   mem);
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    check_mem(mem);
    if (fmt != EEGFX_INT_16 && fmt != EEGFX_IEEE_FLOAT_32) fail(EEGFX_EINVAL, "format %d", fmt);
    if (n_frames < 0 || n < 0 || ct < 1) fail(EEGFX_EINVAL, "negative size");
    if (n > 0 && (!raw || !pos || !features)) fail(EEGFX_EINVAL, "null buffer");
    const ChanSel sel = make_sel(cols, res, C, ct);
    if (mem == EEGFX_MEM_HOST) check_positions(pos, n, n_frames);
    if (n == 0) return;
    ctx->activate();
    const size_t raw_bytes = (size_t)n_frames * ct * (fmt == EEGFX_INT_16 ? 2 : 4);
    const size_t ep_bytes = sizeof(double) * (size_t)n * C * EEGFX_POSTSTIMULUS;
    const size_t f_bytes = sizeof(double) * (size_t)n * C * EEGFX_DWT8_FEATURE_SIZE;
    const void* d_raw = stage_in(ctx, ctx->raw, raw, raw_bytes, mem);
    const int64_t* d_pos = (const int64_t*)stage_in(ctx, ctx->pos, pos, sizeof(int64_t) * n, mem);
    double* d_ep = mem == EEGFX_MEM_DEVICE ? epochs_out : (double*)ctx->scratch.get(ep_bytes);
    double* d_f = mem == EEGFX_MEM_DEVICE ? features : (double*)ctx->out.get(f_bytes);
    run_epochs_and_features(ctx, d_raw, fmt, n_frames, ct, sel, C, d_pos, n, d_ep, d_f);
    if (mem == EEGFX_MEM_HOST) {
      HIP_CHECK(hipMemcpyAsync(epochs_out, d_ep, ep_bytes, hipMemcpyDeviceToHost, ctx->stream));
      HIP_CHECK(hipMemcpyAsync(features, d_f, f_bytes, hipMemcpyDeviceToHost, ctx->stream));
      ctx->drain();
    }
  });
}

// Config 5 (BASELINE.json configs[4]): a long recording in host memory, streamed to the device in
// chunks of `chunk_frames` frames.  Epochs are taken in position order; a chunk starts at the
// first unprocessed epoch's baseline frame (pos - 100) and holds every following epoch whose
// frames [pos-100, pos+687) fit (or reach past the recording end, which the kernels zero-pad), so
// consecutive chunks overlap by at most one epoch span (787 frames) -- the halo.  A ring of four
// device chunk buffers and an upload stream let the H2D run up to three chunks ahead of the
// kernels, and each chunk's rows leave on a download stream as soon as its kernels finish (the
// host link runs both directions at once; with two buffers the event hops between streams
// stalled the uploads).  A pageable source is first copied into one of two pinned staging
// buffers by host threads (that copy overlaps the device work), a pinned source (hipHostMalloc /
// registered) is copied directly.
int eegfx_process_recording_streamed(eegfx_ctx* ctx, const void* raw, int32_t fmt,
                                     int64_t n_frames, int32_t ct, const int32_t* cols,
                                     const float* res, int32_t C, const int64_t* pos, int64_t n,
                                     double* features, int64_t chunk_frames) {
  return guarded([&] {
    if (!ctx) fail(EEGFX_EINVAL, "null context");
    if (fmt != EEGFX_INT_16 && fmt != EEGFX_IEEE_FLOAT_32) fail(EEGFX_EINVAL, "format %d", fmt);
    if (n_frames < 0 || n < 0 || ct < 1) fail(EEGFX_EINVAL, "negative size");
    if (n > 0 && (!raw || !pos || !features)) fail(EEGFX_EINVAL, "null buffer");
    constexpr int64_t kSpan = EEGFX_PRESTIMULUS + EEGFX_DWT8_SKIP + EEGFX_DWT8_EPOCH_SIZE;  // 787
    if (chunk_frames < kSpan)
      fail(EEGFX_EINVAL, "chunk_frames %lld < one epoch span (%lld)", (long long)chunk_frames,
           (long long)kSpan);
    const ChanSel sel = make_sel(cols, res, C, ct);
    check_positions(pos, n, n_frames);
    if (n == 0) return;
    ctx->activate();
    const int64_t FB = (int64_t)ct * (fmt == EEGFX_INT_16 ? 2 : 4);
    const int64_t F = (int64_t)C * EEGFX_DWT8_FEATURE_SIZE;
    // positions in order (the usual .vmrk case) are used as they are; otherwise the epochs are
    // processed in position order and the rows are put back at the end
    const bool in_order = std::is_sorted(pos, pos + n);
    std::vector<int64_t> order, sorted_pos;
    const int64_t* spos = pos;
    if (!in_order) {
      order.resize((size_t)n);
      for (int64_t i = 0; i < n; ++i) order[(size_t)i] = i;
      std::stable_sort(order.begin(), order.end(),
                       [&](int64_t a, int64_t b) { return pos[a] < pos[b]; });
      sorted_pos.resize((size_t)n);
      for (int64_t i = 0; i < n; ++i) sorted_pos[(size_t)i] = pos[order[(size_t)i]];
      spos = sorted_pos.data();
    }
    // The positions go up front on the context stream.  Measured slower (profiles/r06/): the
    // kernels writing the rows straight into a pinned caller buffer instead of a download per
    // chunk (8.84 against 7.2 ms per configs[4] step); a pageable position copy per chunk on the
    // upload stream (9.5 ms: each one blocks the host behind every earlier upload); one position
    // copy on the context stream behind the first chunk's frames (7.44-7.48 against 7.13-7.16);
    // each pinned chunk as two halves on two upload streams (7.75-7.81 against 7.14).
    int64_t* d_pos = (int64_t*)ctx->pos.get(sizeof(int64_t) * (size_t)n);
    auto upload_positions = [&] {
      HIP_CHECK(hipMemcpyAsync(d_pos, spos, sizeof(int64_t) * (size_t)n, hipMemcpyHostToDevice,
                               ctx->stream));
    };
    if (!EEGFX_STREAM_POS_AFTER) upload_positions();
    double* d_out = (double*)ctx->out.get(sizeof(double) * (size_t)(n * F));
    (void)ctx->fused.get(fused_scratch_bytes(n, C));  // every chunk's baselines fit: no realloc
    // chunk buffers: 64 B front pad (the kernels round the first quad down by < 16 B) + data
    // (rounded to 256 B so the second buffer is as aligned as the first: the kernels read
    // 16-byte quads relative to `raw`)
    const size_t cbytes = ((size_t)(chunk_frames * FB) + 128 + 255) & ~(size_t)255;
    // Chunk sizes ramp up (c/4, c/2, then c) and down (about half of what remains, not below
    // c/4) so that the first upload and the last download -- the parts of a call that nothing
    // overlaps -- stay short.
    const int64_t last = spos[n - 1] - EEGFX_PRESTIMULUS + kSpan;
    auto chunk_at = [&](int64_t k, int64_t lo) {
      int64_t c = k < 2 ? chunk_frames >> (2 - k) : chunk_frames;
      const int64_t rest = last - lo;
      if (rest < 2 * chunk_frames) c = std::min(c, (rest + 1) / 2);
      return std::min(chunk_frames, std::max(c, std::max(chunk_frames / 4, 2 * kSpan)));
    };
    struct Chunk {
      int64_t i, j, lo, hi;  // epochs [i, j), frames [lo, hi)
    };
    std::vector<Chunk> plan;
    for (int64_t i = 0; i < n;) {
      const int64_t lo = spos[i] - EEGFX_PRESTIMULUS;
      const int64_t hi = std::min(lo + chunk_at((int64_t)plan.size(), lo), n_frames);
      // the epochs whose span [pos-100, pos+687) ends by hi (all of them at the recording end):
      // a prefix of the sorted positions, found by bisection (a linear scan of configs[4]'s 576k
      // positions delayed the first upload by ~150 us)
      const int64_t j =
          hi == n_frames ? n
                         : std::upper_bound(spos + i, spos + n, hi + EEGFX_PRESTIMULUS - kSpan) - spos;
      plan.push_back({i, j, lo, hi});
      i = j;
    }
    // A ring of 4 device chunk buffers (fewer for fewer chunks).  One buffer per chunk (the whole
    // 346 MB recording in HBM, no upload ever waiting for an earlier chunk's kernels) measured the
    // same: 7.16-7.18 against 7.13-7.18 ms (profiles/r06/stream_ring_ab.log).
    const size_t R = std::min<size_t>(plan.size(), 4);
    uint8_t* dbuf = (uint8_t*)ctx->raw.get(R * cbytes);
    hipPointerAttribute_t attr;
    const bool pinned = hipPointerGetAttributes(&attr, raw) == hipSuccess &&
                        attr.type == hipMemoryTypeHost;
    (void)hipGetLastError();  // a pageable pointer can leave an error behind
    void* pin[2] = {nullptr, nullptr};
    ctx->stream_resources(std::max<size_t>(R, 2));
    hipStream_t cs = ctx->up, os = ctx->down;  // upload (H2D) and download (D2H) streams
    hipEvent_t* copied = ctx->copied.data();
    hipEvent_t* done = ctx->done.data();
    try {
      if (!pinned) {  // the context's grow-only staging (pinned_pool: growing it syncs nothing)
        for (int b = 0; b < 2; ++b) pin[b] = ctx->pin_chunk[b].get(cbytes);
      }
      ctx->drain();  // d_pos uploaded; buffers idle
      for (size_t k = 0; k < plan.size(); ++k) {
        const size_t b = k % R;
        const int64_t i = plan[k].i, j = plan[k].j, lo = plan[k].lo, hi = plan[k].hi;
        const int64_t Lb = (lo * FB) & ~(int64_t)15, Hb = hi * FB;
        const size_t bytes = Hb > Lb ? (size_t)(Hb - Lb) : 0;
        uint8_t* dst = dbuf + (size_t)b * cbytes + 64;
        if (k >= R) HIP_CHECK(hipStreamWaitEvent(cs, done[b], 0));  // kernels of chunk k-R done
        const uint8_t* src = (const uint8_t*)raw + Lb;
        if (!pinned) {  // two pinned staging buffers: staging k&1 is free once chunk k-2 uploaded
          if (k >= 2) HIP_CHECK(hipEventSynchronize(copied[(k - 2) % R]));
          if (bytes) parallel_memcpy(pin[k & 1], src, bytes);
          src = (const uint8_t*)pin[k & 1];
        }
        if (bytes) HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, cs));
        HIP_CHECK(hipEventRecord(copied[b], cs));
        if (EEGFX_STREAM_POS_AFTER && k == 0) upload_positions();  // beside the first chunk's
        HIP_CHECK(hipStreamWaitEvent(ctx->stream, copied[b], 0));
        // frame f of the recording lives at raw_dev + f*FB for lo <= f < hi (pointer arithmetic
        // only: nothing below dst is ever read)
        const uint8_t* raw_dev = dst - Lb;
        run_features_from_raw(ctx, raw_dev, fmt, hi, ct, sel, C, d_pos + i, j - i,
                              d_out + i * F);
        HIP_CHECK(hipEventRecord(done[b], ctx->stream));
        if (in_order) {  // rows of this chunk go straight to the caller on the download stream
          HIP_CHECK(hipStreamWaitEvent(os, done[b], 0));
          HIP_CHECK(hipMemcpyAsync(features + i * F, d_out + i * F,
                                   sizeof(double) * (size_t)((j - i) * F), hipMemcpyDeviceToHost,
                                   os));
        }
      }
      if (in_order) {
        HIP_CHECK(hipStreamSynchronize(os));
      } else {
        std::vector<double> sorted((size_t)(n * F));
        HIP_CHECK(hipMemcpyAsync(sorted.data(), d_out, sizeof(double) * sorted.size(),
                                 hipMemcpyDeviceToHost, ctx->stream));
        ctx->drain();
        for (int64_t r = 0; r < n; ++r)
          memcpy(features + order[(size_t)r] * F, sorted.data() + r * F,
                 sizeof(double) * (size_t)F);
      }
      HIP_CHECK(hipStreamSynchronize(cs));
      ctx->drain();
    } catch (...) {
      (void)hipStreamSynchronize(ctx->stream);
      if (cs) (void)hipStreamSynchronize(cs);
      if (os) (void)hipStreamSynchronize(os);
      throw;
    }
  });
}

// the classifier of LogisticRegressionClassifier.java:85-114 on the GPU
// (csrc/logreg.hip): MLlib 1.6.2 LogisticRegressionWithSGD.  miniBatchFraction < 1: iteration i
// trains on data.sample(false, f, 42 + i) of the rows in `num_partitions` ParallelCollectionRDD
// slices (spark_sample.h), drawn on the host (threads over iterations) as one bit mask per
// iteration and uploaded before the iterations that read them.  The hinge loop of
// eegfx_ext.h (SVMWithSGD) stays full-batch (outside the contract, not extended).
static int glm_sgd_train(int grad, eegfx_ctx* ctx, const double* X, const double* y, int64_t n,
                         int32_t d, int32_t num_iterations, double step_size, double reg_param,
                         double mini_batch_fraction, double convergence_tol,
                         int32_t num_partitions, double* weights, int32_t* iterations_run,
                         int mem) {
  return guarded([&] {
    if (!ctx || !weights) fail(EEGFX_EINVAL, "null argument");
    check_mem(mem);
    if (n < 1) fail(EEGFX_EINVAL, "empty training set");  // GeneralizedLinearAlgorithm: first()
    if (!X || !y) fail(EEGFX_EINVAL, "null X / y");
    if (d < 1 || d > kLrMaxFeatures) fail(EEGFX_EINVAL, "d=%d outside [1, %d]", d, kLrMaxFeatures);
    if (num_iterations < 0) fail(EEGFX_EINVAL, "num_iterations %d", num_iterations);
    // RDD.sample's require(fraction >= 0.0), then BernoulliSampler's upper bound 1 up to
    // RandomSampler.roundingEpsilon
    if (!(mini_batch_fraction >= 0.0))
      fail(EEGFX_EINVAL, "Negative fraction value: %g", mini_batch_fraction);
    if (!(mini_batch_fraction <= 1.0 + 1e-6))
      fail(EEGFX_EINVAL, "Sampling fraction (%g) must be on interval [0, 1]", mini_batch_fraction);
    const bool sampled = mini_batch_fraction < 1.0;
    if (sampled && grad != kGradLogistic)
      fail(EEGFX_ENOTSUP, "miniBatchFraction %g: the SVM loop is full-batch only",
           mini_batch_fraction);
    if (sampled && num_partitions < 1) fail(EEGFX_EINVAL, "num_partitions %d", num_partitions);
    ctx->activate();
    const double* dX = X;
    const double* dy = y;
    if (mem == EEGFX_MEM_HOST) {
      double* bx = (double*)ctx->lr_x.get(sizeof(double) * (size_t)(n * d));
      double* by = (double*)ctx->lr_y.get(sizeof(double) * (size_t)n);
      HIP_CHECK(hipMemcpyAsync(bx, X, sizeof(double) * (size_t)(n * d), hipMemcpyHostToDevice,
                               ctx->stream));
      HIP_CHECK(hipMemcpyAsync(by, y, sizeof(double) * (size_t)n, hipMemcpyHostToDevice,
                               ctx->stream));
      dX = bx;
      dy = by;
    }
    const size_t sbytes = sizeof(LrState) + sizeof(double) * (size_t)d;
    std::vector<uint8_t> hs(sbytes, 0);
    LrState* h = (LrState*)hs.data();
    h->converged = num_iterations == 0 ? 1 : 0;
    memcpy(h->w, weights, sizeof(double) * (size_t)d);  // initial weights (zeros in MLlib)
    LrState* st = (LrState*)ctx->lr_state.get(sbytes);
    HIP_CHECK(hipMemcpyAsync(st, hs.data(), sbytes, hipMemcpyHostToDevice, ctx->stream));
    HIP_CHECK(launch_lr_validate(ctx->stream, dy, n, st));
    const int G = lr_grid(n);
    double* part = (double*)ctx->lr_part.get(sizeof(double) * (size_t)G * d);
    if (!sampled) {
      for (int i = 0; i < num_iterations; ++i)
        HIP_CHECK(launch_lr_iteration(ctx->stream, grad, dX, dy, n, d, nullptr, n, st, part, G,
                                      step_size, reg_param, convergence_tol, num_iterations));
    } else {
      // the masks of up to ~256 MB of iterations at a time, drawn by threads over iterations
      const int64_t words = (n + 31) / 32;
      const int chunk = (int)std::max<int64_t>(
          1, std::min<int64_t>(num_iterations, ((int64_t)64 << 20) / words));
      std::vector<uint32_t> masks((size_t)(chunk * words));
      std::vector<int64_t> counts((size_t)chunk);
      uint32_t* dmask = (uint32_t*)ctx->lr_mask.get(sizeof(uint32_t) * masks.size());
      const int T_max = std::min(64, available_processors());
      for (int i0 = 0; i0 < num_iterations; i0 += chunk) {
        const int k = std::min(chunk, num_iterations - i0);
        ctx->drain();  // the previous chunk's upload and iterations are done with both buffers
        if (i0 > 0) {  // converged (or stopped): the remaining iterations would be skipped
          int32_t conv = 0;
          HIP_CHECK(hipMemcpyAsync(&conv, &st->converged, sizeof(conv), hipMemcpyDeviceToHost,
                                   ctx->stream));
          HIP_CHECK(hipStreamSynchronize(ctx->stream));
          if (conv != 0) break;
        }
        const int T = std::max(1, std::min(k, T_max));
        {
          Joiner pool;
          for (int t = 0; t < T; ++t)
            pool.th.emplace_back([&, t] {
              for (int j = t; j < k; j += T)  // GradientDescent's i = i0 + j + 1, seed 42 + i
                counts[j] = spark::sample_mask(n, mini_batch_fraction, num_partitions,
                                               42 + (int64_t)(i0 + j + 1),
                                               &masks[(size_t)j * words]);
            });
        }
        HIP_CHECK(hipMemcpyAsync(dmask, masks.data(), sizeof(uint32_t) * (size_t)(k * words),
                                 hipMemcpyHostToDevice, ctx->stream));
        for (int j = 0; j < k; ++j)
          HIP_CHECK(launch_lr_iteration(ctx->stream, grad, dX, dy, n, d, dmask + (size_t)j * words,
                                        counts[j], st, part, G, step_size, reg_param,
                                        convergence_tol, num_iterations));
      }
    }
    HIP_CHECK(hipMemcpyAsync(hs.data(), st, sbytes, hipMemcpyDeviceToHost, ctx->stream));
    ctx->drain();
    if (h->converged == 2) fail(EEGFX_EINVAL, "Input validation failed: labels must be 0.0 or 1.0");
    memcpy(weights, h->w, sizeof(double) * (size_t)d);
    if (iterations_run) *iterations_run = h->iter;
  });
}

static int glm_predict(int grad, eegfx_ctx* ctx, const double* X, int64_t n, int32_t d,
                       const double* weights, double intercept, double threshold, double* out,
                       int mem) {
  return guarded([&] {
    if (!ctx || !weights) fail(EEGFX_EINVAL, "null argument");
    check_mem(mem);
    if (n < 0 || d < 1 || d > kLrMaxFeatures) fail(EEGFX_EINVAL, "n=%lld d=%d", (long long)n, d);
    if (n == 0) return;
    if (!X || !out) fail(EEGFX_EINVAL, "null X / out");
    ctx->activate();
    const double* dX = X;
    double* dout = out;
    if (mem == EEGFX_MEM_HOST) {
      double* bx = (double*)ctx->lr_x.get(sizeof(double) * (size_t)(n * d));
      HIP_CHECK(hipMemcpyAsync(bx, X, sizeof(double) * (size_t)(n * d), hipMemcpyHostToDevice,
                               ctx->stream));
      dX = bx;
      dout = (double*)ctx->lr_y.get(sizeof(double) * (size_t)n);
    }
    const size_t sbytes = sizeof(LrState) + sizeof(double) * (size_t)d;
    LrState* st = (LrState*)ctx->lr_state.get(sbytes);
    HIP_CHECK(hipMemcpyAsync(st->w, weights, sizeof(double) * (size_t)d, hipMemcpyHostToDevice,
                             ctx->stream));
    const bool use_t = !std::isnan(threshold);  // clearThreshold -> scores / margins
    HIP_CHECK(launch_lr_predict(ctx->stream, grad, dX, n, d, st->w, intercept, threshold,
                                use_t ? 1 : 0, dout));
    if (mem == EEGFX_MEM_HOST)
      HIP_CHECK(hipMemcpyAsync(out, dout, sizeof(double) * (size_t)n, hipMemcpyDeviceToHost,
                               ctx->stream));
    ctx->drain();
  });
}

int eegfx_logreg_sgd_train_partitioned(eegfx_ctx* ctx, const double* X, const double* y,
                                       int64_t n, int32_t d, int32_t num_iterations,
                                       double step_size, double reg_param,
                                       double mini_batch_fraction, double convergence_tol,
                                       int32_t num_partitions, double* weights,
                                       int32_t* iterations_run, int mem) {
  return glm_sgd_train(kGradLogistic, ctx, X, y, n, d, num_iterations, step_size, reg_param,
                       mini_batch_fraction, convergence_tol, num_partitions, weights,
                       iterations_run, mem);
}

int eegfx_logreg_sgd_train(eegfx_ctx* ctx, const double* X, const double* y, int64_t n, int32_t d,
                           int32_t num_iterations, double step_size, double reg_param,
                           double mini_batch_fraction, double convergence_tol, double* weights,
                           int32_t* iterations_run, int mem) {
  // Spark local[*] (SparkInitializer.java:44): defaultParallelism = the processors available
  // to the process (Runtime.availableProcessors(): affinity and cgroup quota honoured)
  const int32_t parts = (int32_t)available_processors();
  return glm_sgd_train(kGradLogistic, ctx, X, y, n, d, num_iterations, step_size, reg_param,
                       mini_batch_fraction, convergence_tol, parts, weights, iterations_run, mem);
}

int eegfx_spark_sample(int64_t n, double fraction, int32_t num_partitions, int64_t seed,
                       uint32_t* mask, int64_t* kept) {
  return guarded([&] {
    if (n < 0 || num_partitions < 1 || !mask || !kept) fail(EEGFX_EINVAL, "bad argument");
    if (!(fraction >= -1e-6 && fraction <= 1.0 + 1e-6))
      fail(EEGFX_EINVAL, "Sampling fraction (%g) must be on interval [0, 1]", fraction);
    *kept = spark::sample_mask(n, fraction, num_partitions, seed, mask);
  });
}

int eegfx_logreg_predict(eegfx_ctx* ctx, const double* X, int64_t n, int32_t d,
                         const double* weights, double intercept, double threshold, double* out,
                         int mem) {
  return glm_predict(kGradLogistic, ctx, X, n, d, weights, intercept, threshold, out, mem);
}

// The classifier of SVMClassifier.java:83-111 (MLlib 1.6.2 SVMWithSGD: HingeGradient, the same
// SquaredL2Updater / GradientDescent loop) and SVMModel.predict (:71, :114-137).
int eegfx_svm_sgd_train(eegfx_ctx* ctx, const double* X, const double* y, int64_t n, int32_t d,
                        int32_t num_iterations, double step_size, double reg_param,
                        double mini_batch_fraction, double convergence_tol, double* weights,
                        int32_t* iterations_run, int mem) {
  return glm_sgd_train(kGradHinge, ctx, X, y, n, d, num_iterations, step_size, reg_param,
                       mini_batch_fraction, convergence_tol, 1, weights, iterations_run, mem);
}

int eegfx_svm_predict(eegfx_ctx* ctx, const double* X, int64_t n, int32_t d, const double* weights,
                      double intercept, double threshold, double* out, int mem) {
  return glm_predict(kGradHinge, ctx, X, n, d, weights, intercept, threshold, out, mem);
}

int eegfx_plan_markers_device(eegfx_ctx* ctx, const int64_t* positions,
                              const int32_t* stimulus_index, int64_t n_markers, int64_t n_frames,
                              int32_t guessed, int64_t* balance, int64_t* pos_out,
                              double* label_out, int64_t* n_selected, int mem) {
  return guarded([&] {
    if (!ctx || !balance || !n_selected) fail(EEGFX_EINVAL, "null argument");
    check_mem(mem);
    if (n_markers < 0) fail(EEGFX_EINVAL, "negative marker count");
    if (*balance < -1 || *balance > 1)
      fail(EEGFX_EINVAL, "balance %lld outside {-1, 0, 1}", (long long)*balance);
    *n_selected = 0;
    if (n_markers == 0) return;
    if (!positions || !stimulus_index) fail(EEGFX_EINVAL, "null markers");
    ctx->activate();
    const int64_t n = n_markers;
    const int64_t* d_pos = (const int64_t*)stage_in(ctx, ctx->pos, positions, sizeof(int64_t) * n,
                                                    mem);
    const int32_t* d_stim = (const int32_t*)stage_in(ctx, ctx->lr_y, stimulus_index,
                                                     sizeof(int32_t) * n, mem);
    int64_t* d_pos_out = pos_out;
    double* d_label = label_out;
    if (mem == EEGFX_MEM_HOST) {
      uint8_t* o = (uint8_t*)ctx->out.get((sizeof(int64_t) + sizeof(double)) * (size_t)n);
      d_pos_out = pos_out ? (int64_t*)o : nullptr;
      d_label = label_out ? (double*)(o + sizeof(int64_t) * (size_t)n) : nullptr;
    }
    void* scratch = ctx->scratch.get(plan_scratch_bytes(n));
    PlanResult r;
    HIP_CHECK(launch_plan_markers(ctx->stream, d_pos, d_stim, n, n_frames, guessed,
                                  (int)*balance, scratch, d_pos_out, d_label, &r));
    if (mem == EEGFX_MEM_HOST && r.selected > 0) {
      if (pos_out)
        HIP_CHECK(hipMemcpyAsync(pos_out, d_pos_out, sizeof(int64_t) * (size_t)r.selected,
                                 hipMemcpyDeviceToHost, ctx->stream));
      if (label_out)
        HIP_CHECK(hipMemcpyAsync(label_out, d_label, sizeof(double) * (size_t)r.selected,
                                 hipMemcpyDeviceToHost, ctx->stream));
    }
    ctx->drain();
    *balance = r.balance;
    *n_selected = r.selected;
    if (r.first_unparsable >= 0)  // Integer.parseInt's NumberFormatException ends the reference loop
      fail(EEGFX_EFORMAT, "marker %lld: unparsable stimulus description",
           (long long)r.first_unparsable);
  });
}

int eegfx_synth_recording(eegfx_ctx* ctx, int16_t* dst, int64_t n_frames, int32_t n_channels,
                          uint64_t seed) {
  return guarded([&] {
    if (!ctx || !dst) fail(EEGFX_EINVAL, "null argument");
    if (n_frames < 0 || n_channels < 1) fail(EEGFX_EINVAL, "bad size");
    ctx->activate();
    HIP_CHECK(launch_synth(ctx->stream, dst, n_frames, n_channels, seed));
  });
}

// ---- OffLineDataProvider ----------------------------------------------------------------------
int eegfx_odp_create(eegfx_ctx* ctx, const char* const* args, int32_t n_args, eegfx_odp** out) {
  return guarded([&] {
    if (!out || (n_args > 0 && !args) || n_args < 0) fail(EEGFX_EINVAL, "null argument");
    std::unique_ptr<eegfx_odp> o(new eegfx_odp());
    o->ctx = ctx;
    for (int i = 0; i < n_args; ++i) o->args.emplace_back(args[i] ? args[i] : "");
    *out = o.release();
  });
}

int eegfx_odp_load_data(eegfx_odp* odp) {
  if (!odp) {
    set_last_error("null provider");
    return EEGFX_EINVAL;
  }
  // loadData (:88-98): every exception is logged as fatal and swallowed; what was loaded stays.
  const int rc = guarded([&] {
    if (odp->ctx) odp->ctx->activate();
    odp->handle_input();
    odp->process_eeg_files();
  });
  odp->error = rc == EEGFX_OK ? "" : last_error();
  return rc;
}

const char* eegfx_odp_error(const eegfx_odp* odp) { return odp ? odp->error.c_str() : "null provider"; }

int64_t eegfx_odp_num_epochs(const eegfx_odp* odp) { return odp ? odp->n_epochs : 0; }

int eegfx_odp_get_data(const eegfx_odp* odp, double* out) {
  return guarded([&] {
    if (!odp || !out) fail(EEGFX_EINVAL, "null argument");
    if (!odp->n_epochs) return;
    if (!odp->ctx) fail(EEGFX_EINVAL, "planning-only provider (no device context) holds no epochs");
    odp->ctx->activate();
    HIP_CHECK(hipMemcpyAsync(out, odp->d_epochs,
                             sizeof(double) * 3 * EEGFX_POSTSTIMULUS * (size_t)odp->n_epochs,
                             hipMemcpyDeviceToHost, odp->ctx->stream));
    odp->ctx->drain();
  });
}

int eegfx_odp_get_labels(const eegfx_odp* odp, double* out) {
  return guarded([&] {
    if (!odp || !out) fail(EEGFX_EINVAL, "null argument");
    std::copy(odp->labels.begin(), odp->labels.end(), out);
  });
}

int eegfx_odp_get_positions(const eegfx_odp* odp, int64_t* pos_out, int32_t* file_out) {
  return guarded([&] {
    if (!odp) fail(EEGFX_EINVAL, "null argument");
    if (pos_out) std::copy(odp->positions.begin(), odp->positions.end(), pos_out);
    if (file_out) std::copy(odp->file_of_epoch.begin(), odp->file_of_epoch.end(), file_out);
  });
}

int eegfx_odp_get_features(eegfx_odp* odp, int32_t name, int32_t epoch_size, int32_t skip,
                           int32_t feature_size, double* out) {
  return guarded([&] {
    if (!odp || !out) fail(EEGFX_EINVAL, "null argument");
    check_fe_params(3, name, epoch_size, skip, feature_size);
    if (!odp->n_epochs) return;
    if (!odp->ctx) fail(EEGFX_EINVAL, "planning-only provider (no device context) holds no epochs");
    eegfx_ctx* ctx = odp->ctx;
    ctx->activate();
    const size_t out_bytes = sizeof(double) * (size_t)odp->n_epochs * 3 * feature_size;
    if (skip == EEGFX_DWT8_SKIP && feature_size == EEGFX_DWT8_FEATURE_SIZE &&
        odp->features_numerics == ctx->numerics && odp->d_features) {
      // the rows computed with the epochs at loadData (the one-pass kernels)
      HIP_CHECK(hipMemcpyAsync(out, odp->d_features, out_bytes, hipMemcpyDeviceToHost,
                               ctx->stream));
      ctx->drain();
      return;
    }
    double* d_out = (double*)ctx->out.get(out_bytes);
    const Guard g = ctx->guard_for(odp->n_epochs);
    HIP_CHECK(launch_features_from_epochs(ctx->stream, (const double*)odp->d_epochs,
                                          odp->n_epochs, 3, skip, feature_size,
                                          ctx->numerics != EEGFX_EXACT, d_out, EEGFX_POSTSTIMULUS,
                                          g));
    HIP_CHECK(hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, ctx->stream));
    ctx->drain();
  });
}

void eegfx_odp_destroy(eegfx_odp* odp) {
  if (!odp) return;
  if (odp->ctx && (odp->d_epochs || odp->d_features)) {
    (void)hipSetDevice(odp->ctx->device);
    if (odp->d_epochs) (void)hipFreeAsync(odp->d_epochs, odp->ctx->stream);
    if (odp->d_features) (void)hipFreeAsync(odp->d_features, odp->ctx->stream);
    (void)hipStreamSynchronize(odp->ctx->stream);
  }
  delete odp;
}

}  // extern "C"
