// Probe: window_kernel (VALU cascade, fma numerics) timing under EEGFX_FUSED_ABLATION (bit 0: no
// window DMA, bit 1: no LDS reads/decode, bit 2: no filter bank) on the bench workload.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../eeg_dataanalysispackage_amd/csrc/fused.hip"

__global__ void fill_random(uint32_t* p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z ^= z >> 27;
    p[i] = (uint32_t)z & 0x0FFF0FFFu;  // two int16 samples in [0, 4096)
  }
}

int main() {
  const int64_t n = 1000000, nf = 1000 * n + 2000;
  uint8_t* raw;
  int64_t* pos;
  float* base;
  double* out;
  (void)hipMalloc(&raw, nf * 6);
  (void)hipMalloc(&pos, n * 8);
  (void)hipMalloc(&base, n * 12);
  (void)hipMalloc(&out, n * 48 * 8);
  if (getenv("PROBE_RANDOM")) fill_random<<<4096, 256>>>((uint32_t*)raw, nf * 6 / 4);
  else (void)hipMemset(raw, 3, nf * 6);
  std::vector<int64_t> hp(n);
  const char* sp = getenv("PROBE_SPACING");  // frames between markers (1000: the bench)
  const int64_t spacing = sp ? atoi(sp) : 1000;
  for (int64_t i = 0; i < n; ++i) hp[i] = 1000 + spacing * i;
  (void)hipMemcpy(pos, hp.data(), n * 8, hipMemcpyHostToDevice);
  eegfx::ChanSel sel{};
  for (int c = 0; c < 3; ++c) { sel.col[c] = c; sel.res[c] = 0.1f; }
  (void)eegfx::launch_fused_baseline(0, raw, nf, 3, sel, 3, pos, n, base);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int r = 0; r < 2; ++r)
    (void)eegfx::launch_fused_window(0, raw, nf, 3, sel, 3, pos, n, !getenv("PROBE_EXACT"), base, out);
  if (getenv("PROBE_BASELINE")) {  // time the baseline kernel instead of the window kernel
    hipEvent_t c, d;
    (void)hipEventCreate(&c);
    (void)hipEventCreate(&d);
    for (int r = 0; r < 50; ++r) (void)eegfx::launch_fused_baseline(0, raw, nf, 3, sel, 3, pos, n, base);
    (void)hipEventRecord(c);
    for (int r = 0; r < 500; ++r) (void)eegfx::launch_fused_baseline(0, raw, nf, 3, sel, 3, pos, n, base);
    (void)hipEventRecord(d);
    (void)hipEventSynchronize(d);
    float bms;
    (void)hipEventElapsedTime(&bms, c, d);
    printf("baseline ablation %d: %.4f ms\n", EEGFX_FUSED_ABLATION, bms / 500);
    return 0;
  }
  const char* it = getenv("PROBE_ITERS");
  const int iters = it ? atoi(it) : 10;
  (void)hipEventRecord(a);
  for (int r = 0; r < iters; ++r)
    (void)eegfx::launch_fused_window(0, raw, nf, 3, sel, 3, pos, n, !getenv("PROBE_EXACT"), base, out);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms;
  (void)hipEventElapsedTime(&ms, a, b);
  printf("window ablation %d: %.4f ms\n", EEGFX_FUSED_ABLATION, ms / iters);
  return 0;
}
