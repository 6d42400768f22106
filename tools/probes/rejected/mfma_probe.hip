// Probe: mfma_window_kernel timing with ablations (EEGFX_MFMA_ABLATION: 0 product, 1 no DMA
// waits, 2 no decode, 3 neither) on the bench workload (1M epochs, 3 ch int16, baselines 0).
// Build: see tools/probes/build_probes.sh.  Prints kernel ms and the implied algorithmic GB/s.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "mfma.hip"

int main() {
  const int64_t n = 1000000, nf = 1000 * n + 2000;
  uint8_t* raw;
  int64_t* pos;
  float* base;
  double *mrows, *out;
  (void)hipMalloc(&raw, nf * 6);
  (void)hipMalloc(&pos, n * 8);
  (void)hipMalloc(&base, n * 12);
  (void)hipMalloc(&mrows, 1024 * 8);
  (void)hipMalloc(&out, n * 48 * 8);
  (void)hipMemset(raw, 3, nf * 6);
  (void)hipMemset(base, 0, n * 12);
  std::vector<int64_t> hp(n);
  for (int64_t i = 0; i < n; ++i) hp[i] = 1000 + 1000 * i;
  (void)hipMemcpy(pos, hp.data(), n * 8, hipMemcpyHostToDevice);
  std::vector<double> rows(1024);
  eegfx::dwt8_operator_rows(rows.data());
  (void)hipMemcpy(mrows, rows.data(), 1024 * 8, hipMemcpyHostToDevice);
  eegfx::ChanSel sel{};
  for (int c = 0; c < 3; ++c) { sel.col[c] = c; sel.res[c] = 0.1f; }
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int r = 0; r < 2; ++r)
    (void)eegfx::launch_mfma_window(0, raw, nf, 3, sel, 3, pos, n, base, mrows, out);
  (void)hipEventRecord(a);
  for (int r = 0; r < 10; ++r)
    (void)eegfx::launch_mfma_window(0, raw, nf, 3, sel, 3, pos, n, base, mrows, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  ms /= 10;
  printf("ablation %d: %.4f ms  %.1f GB/s algorithmic (3476 B/epoch)\n", EEGFX_MFMA_ABLATION, ms,
         3476.0 * n / ms / 1e6);
  return 0;
}
