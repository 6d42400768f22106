// Probe: window_kernel (the fused c3 path) or window_wide_kernel (configs[3]) timed under sustained
// load, for A/B studies of kernel variants.  FUSED_SRC / WIDE_SRC name the kernel source to build
// against (default: the product files); build_probes.sh builds one per tools/probes/ablations/ patch.
//
//   hipcc ... -DFUSED_SRC='"build/v1/fused.hip"' window_probe.hip -o window_probe_v1
//   PROBE_WIDE=1 PROBE_ITERS=2000 PROBE_EXACT=1 ./window_probe_v1
//   PROBE_BASELINE=1: time the baseline kernel alone; PROBE_STEP=1: baseline + window per launch;
//   PROBE_FB=1 (built with -DPROBE_ONE_LAUNCH against history/one_launch_step_fused.patch): the
//   step as one launch (launch_fused_step, window_fb_kernel)
//   PROBE_N=8000000: another epoch count (one marker every 1,000 frames as always)
//
// Phase timestamps (per-workgroup s_memrealtime at each phase boundary):
//   restore_variant.sh phase_timestamps_fused, then -DFUSED_SRC='"<dir>/fused.hip"' -DPROBE_TIMESTAMPS
//
// Inputs are the bench workload: synth_kernel recording (configs[1]: 1M epochs x 3 ch, or
// configs[3]: 250k epochs x 32 ch), one marker every 1,000 frames.  Prints the average launch time
// over PROBE_ITERS launches after 200 warm-up launches (the clock settles under the power cap),
// and a checksum of the feature matrix (sum and sum of squares) for a quick equality check
// between variants.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#ifndef FUSED_SRC
#define FUSED_SRC "../../eeg_dataanalysispackage_amd/csrc/fused.hip"
#endif
#ifndef WIDE_SRC
#define WIDE_SRC "../../eeg_dataanalysispackage_amd/csrc/wide.hip"
#endif
#include FUSED_SRC
#include WIDE_SRC
#include "../../eeg_dataanalysispackage_amd/csrc/kernels.hip"
#include "../../eeg_dataanalysispackage_amd/csrc/guard.hip"

int main() {
  const bool wide = getenv("PROBE_WIDE") != nullptr;
  const bool fast = getenv("PROBE_EXACT") == nullptr;
  const int ct = wide ? 32 : 3;
  const char* en = getenv("PROBE_N");  // epochs (configs[2]'s rank shard: 8000000)
  const int64_t n = en ? atoll(en) : wide ? 250000 : 1000000, nf = 1000 * n + 2000;
  int16_t* raw;
  int64_t* pos;
  float* base;
  double* out;
  (void)hipMalloc(&raw, nf * ct * 2);
  (void)hipMalloc(&pos, n * 8);
  (void)hipMalloc(&base, eegfx::fused_scratch_bytes(n, ct));
  (void)hipMalloc(&out, n * 16 * ct * 8);
  (void)eegfx::launch_synth(0, raw, nf, ct, 0x5EED);
  std::vector<int64_t> hp(n);
  for (int64_t i = 0; i < n; ++i) hp[i] = 1000 + 1000 * i;
  (void)hipMemcpy(pos, hp.data(), n * 8, hipMemcpyHostToDevice);
  eegfx::ChanSel sel{};
  for (int c = 0; c < ct; ++c) { sel.col[c] = c; sel.res[c] = 0.1f; }
  // the product's fma guard state (eegfx_ctx: count, the two slot-spread running totals, list)
  int* gdev;
  int64_t* glist;
  const size_t gbytes = 128 + 2 * eegfx::kGuardSlotBytes;
  (void)hipMalloc(&gdev, gbytes);
  (void)hipMemset(gdev, 0, gbytes);
  (void)hipMalloc(&glist, n * 8);
  const eegfx::Guard g =
      fast ? eegfx::Guard{gdev, glist, (unsigned long long*)((char*)gdev + 128),
                          (unsigned long long*)((char*)gdev + 128 + eegfx::kGuardSlotBytes)}
           : eegfx::Guard{nullptr, nullptr, nullptr};
  auto baseline = [&] {
    if (wide) (void)eegfx::launch_baseline_any(0, raw, 0, nf, ct, sel, ct, pos, n, base, nullptr, g.count);
    else (void)eegfx::launch_fused_baseline(0, raw, nf, ct, sel, ct, pos, n, base, nullptr, nullptr);
  };
  auto window = [&] {
    if (wide) (void)eegfx::launch_window_wide(0, raw, 0, nf, ct, sel, ct, pos, n, fast, base, out, g);
    else (void)eegfx::launch_fused_window(0, raw, nf, ct, sel, ct, pos, n, fast, base, out, g);
  };
  baseline();
  const char* it = getenv("PROBE_ITERS");
  const int iters = it ? atoi(it) : 2000;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const bool time_baseline = getenv("PROBE_BASELINE") != nullptr;
  const bool time_step = getenv("PROBE_STEP") != nullptr;  // baseline + window, as bench.py's step
  // PROBE_FB=1: the step as one launch (window_fb_kernel, baselines folded in; built against
  // history/one_launch_step_fused.patch with -DPROBE_ONE_LAUNCH)
#ifdef PROBE_ONE_LAUNCH
  const bool one_launch = getenv("PROBE_FB") != nullptr && !wide;
  auto fstep = [&] {
    (void)eegfx::launch_fused_step(0, raw, nf, ct, sel, ct, pos, n, fast, out, nullptr, g);
  };
#else
  const bool one_launch = false;
  auto fstep = [&] {};
#endif
  // PROBE_OVERLAP=K: the step in K chunks, baseline chunks on one stream and window chunks on
  // another (chunk i's window waits for its baseline; chunk i's baseline of the next step waits
  // for chunk i's window of this one, whose scratch it reuses), so baselines run under windows
  const char* ov = getenv("PROBE_OVERLAP");
  const int K = ov ? atoi(ov) : 0;
  hipStream_t sb = 0, sw = 0;
  std::vector<hipEvent_t> evb(K > 0 ? K : 1), evw(K > 0 ? K : 1);
  std::vector<int64_t> c0(K + 1, 0);
  std::vector<uint8_t*> cs(K > 0 ? K : 1);
  if (K > 0) {
    (void)hipStreamCreateWithFlags(&sb, hipStreamNonBlocking);
    (void)hipStreamCreateWithFlags(&sw, hipStreamNonBlocking);
    const char* rp = getenv("PROBE_RAMP");  // first chunk = n / (K * ramp), the rest equal
    const int ramp = rp ? atoi(rp) : 1;
    c0[1] = n / ((int64_t)K * ramp);
    for (int i = 2; i <= K; ++i) c0[i] = c0[1] + (n - c0[1]) * (i - 1) / (K - 1);
    if (K == 1) c0[1] = n;
    for (int i = 0; i < K; ++i) {
      (void)hipEventCreateWithFlags(&evb[i], hipEventDisableTiming);
      (void)hipEventCreateWithFlags(&evw[i], hipEventDisableTiming);
      (void)hipMalloc(&cs[i], eegfx::fused_scratch_bytes(c0[i + 1] - c0[i], ct));
      (void)hipEventRecord(evw[i], sw);
    }
    fprintf(stderr, "overlap: %d chunks, first %lld epochs\n", K, (long long)c0[1]);
  }
  const bool strict = getenv("PROBE_STRICT") != nullptr;  // no overlap across steps
  auto ostep = [&] {
    for (int i = 0; i < K; ++i) {
      const int64_t a0 = c0[i], m = c0[i + 1] - c0[i];
      (void)hipStreamWaitEvent(sb, evw[strict && i == 0 ? K - 1 : i], 0);
      (void)eegfx::launch_fused_baseline(sb, raw, nf, ct, sel, ct, pos + a0, m, cs[i], nullptr, nullptr);
      (void)hipEventRecord(evb[i], sb);
      (void)hipStreamWaitEvent(sw, evb[i], 0);
      (void)eegfx::launch_fused_window(sw, raw, nf, ct, sel, ct, pos + a0, m, fast, cs[i],
                                       out + a0 * 16 * ct, g);
      (void)hipEventRecord(evw[i], sw);
    }
  };
  auto one = [&] {
    if (K > 0) ostep();
    else if (one_launch) fstep();
    else if (time_step) { baseline(); window(); }
    else if (time_baseline) baseline();
    else window();
  };
  const char* wu = getenv("PROBE_WARMUP");
  const int warm = wu ? atoi(wu) : 200;
  for (int r = 0; r < warm; ++r) one();
  float ms;
  if (K > 0) {  // two streams: wall clock between device-wide drains
    (void)hipDeviceSynchronize();
    const auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < iters; ++r) one();
    (void)hipDeviceSynchronize();
    ms = std::chrono::duration<float, std::milli>(std::chrono::steady_clock::now() - t0).count();
  } else {
    (void)hipEventRecord(a);
    for (int r = 0; r < iters; ++r) one();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    (void)hipEventElapsedTime(&ms, a, b);
  }
#ifdef PROBE_TIMESTAMPS
  {  // one more launch with per-workgroup phase timestamps
    const size_t nwg = (size_t)((n + 7) / 8);
    unsigned long long* d_ts;
    (void)hipMalloc(&d_ts, nwg * 5 * 8);
    (void)hipMemset(d_ts, 0, nwg * 5 * 8);
    (void)hipMemcpyToSymbol(HIP_SYMBOL(eegfx::dev::g_probe_ts), &d_ts, sizeof(d_ts));
    for (int r = 0; r < 50; ++r) window();  // keep the clock at its loaded state
    window();
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> ts(nwg * 5);
    (void)hipMemcpy(ts.data(), d_ts, ts.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t_min = ~0ull, t_max = 0;
    double ph[4] = {0, 0, 0, 0};
    size_t cnt = 0;
    for (size_t i = 0; i < nwg; ++i) {
      const unsigned long long* t = &ts[5 * i];
      if (!t[0]) continue;
      ++cnt;
      t_min = t[0] < t_min ? t[0] : t_min;
      t_max = t[4] > t_max ? t[4] : t_max;
      for (int k = 0; k < 4; ++k) ph[k] += (double)(t[k + 1] - t[k]);
    }
    const double tick_us = 0.01;  // s_memrealtime: 100 MHz
    printf("ts: %zu workgroups, launch span %.1f us; mean per workgroup (us): windows landed %.2f, "
           "level 1 %.2f, levels 2-6 %.2f, rows + normalise + store %.2f, lifetime %.2f\n", cnt,
           (t_max - t_min) * tick_us, ph[0] / cnt * tick_us, ph[1] / cnt * tick_us,
           ph[2] / cnt * tick_us, ph[3] / cnt * tick_us,
           (ph[0] + ph[1] + ph[2] + ph[3]) / cnt * tick_us);
    unsigned long long* none = nullptr;  // detach before freeing: later launches must not write
    (void)hipMemcpyToSymbol(HIP_SYMBOL(eegfx::dev::g_probe_ts), &none, sizeof(none));
    (void)hipDeviceSynchronize();
    std::vector<double> ends;  // end of each workgroup relative to the first start
    for (size_t i = 0; i < nwg; ++i)
      if (ts[5 * i]) ends.push_back((double)(ts[5 * i + 4] - t_min) * tick_us);
    std::sort(ends.begin(), ends.end());
    if (!ends.empty())
      printf("ts: workgroup end times (us from the first start): min %.1f, median %.1f, p99 %.1f, "
             "max %.1f\n", ends.front(), ends[ends.size() / 2], ends[ends.size() * 99 / 100],
             ends.back());
    (void)hipFree(d_ts);
  }
#endif
  (void)hipMemset(out, 0, n * 16 * ct * 8);
  if (K > 0) { ostep(); (void)hipDeviceSynchronize(); }
  else if (one_launch) fstep();
  else { baseline(); window(); }
  std::vector<double> h(n * 16 * ct);
  (void)hipMemcpy(h.data(), out, h.size() * 8, hipMemcpyDeviceToHost);
  double s = 0, q = 0;
  for (double v : h) { s += v; q += v * v; }
  const hipError_t e = hipGetLastError();
  printf("%s %s %s: %.4f ms per launch (%d launches)  checksum %.17g %.17g  %s\n",
         wide ? "wide c32" : "window c3", fast ? "fma" : "exact",
         K > 0 ? "step-overlap" : one_launch ? "step-1-launch" : time_step ? "step" : time_baseline ? "baseline" : "window", ms / iters, iters, s, q, hipGetErrorString(e));
  return e == hipSuccess ? 0 : 1;
}
