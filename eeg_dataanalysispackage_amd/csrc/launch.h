// launch.h -- host-side launchers of the gfx950 kernels (kernels.hip, fused.hip).
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdint>

#include "guard.h"

namespace eegfx {

constexpr int kMaxChannels = 64;

// Selected channels, passed by value as a kernel argument: 0-based column in the multiplexed
// frame and the .vhdr resolution (narrowed to float, as the reference multiplies in fp32).
struct ChanSel {
  int32_t col[kMaxChannels];
  float res[kMaxChannels];
};

// err: device-visible int (the context's host-mapped error word) set to 1 when a kernel reads a
// marker position the reference would not cut (pos - 100 outside [0, n_frames]); may be null.
// scratch: fused_scratch_bytes(n, C) bytes for the baselines (nullptr: single-kernel fallback)
hipError_t launch_cut_epochs(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                             const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                             double* out, void* scratch, int* err);
// The one-pass getData + features (kernels.hip staged_features): baselines, then one workgroup
// per epoch writes the epoch's rows to `out` (double[n][C][750]) and its normalised dwt-8 row to
// `feat` (double[n][16 C]) from the same LDS-staged frames.  hipErrorNotSupported when the layout
// does not fit (cut_features_supported): the caller cuts, then extracts from the rows.
bool cut_features_supported(int fmt, int ct, int C, const void* raw, const double* out,
                            const double* feat);
hipError_t launch_cut_features(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                               double* out, double* feat, bool fast, void* scratch, int* err,
                               const Guard& guard);
// row_stride: doubles between consecutive (epoch, channel) rows of `ep` (750 for materialised
// epochs, 512 for the window-only rows the host path stages)
// guard (fma numerics): the conditioning guard (guard.h); flagged rows are recomputed under EXACT
// inside the kernel and counted in guard.total.
hipError_t launch_features_from_epochs(hipStream_t st, const double* ep, int64_t n, int C, int skip,
                                       int nfeat, bool fast, double* out, int row_stride,
                                       const Guard& guard);
// Small host batches (kernels.hip features_small_kernel): rows = n x C x 512 packed window rows,
// one workgroup per epoch, C <= 16; rows / out may be device pointers of mapped pinned memory.
bool features_small_supported(int C);
// guard.total counts the rows the kernel recomputed under EXACT (guard.h); count/list unused.
// The resident small-batch server (eegfx_ctx_set_mailbox): a host-mapped command block, written
// by the host except `done` (the device's last completed request).
struct MailboxCmd {
  // The request word, written last by the host (release): sequence number << 32 | (C - 1) << 26 |
  // (nfeat - 1) << 21 | n -- the whole request in one aligned 64-bit load, so the kernel needs no
  // second round trip across the host link for its fields (bit 31 unused: the per-epoch path
  // computes EXACT rows under both numerics).
  uint64_t req;
  uint32_t done;  // the last sequence number whose rows are in `out` (device)
  uint32_t stop;  // 1: the kernel returns
  uint32_t alive;  // the launch generation of the kernel that has started (device, at entry)
  uint32_t pad_;
  // staging, fixed while a server runs (growing it stops the server first); read at kernel start
  const double* rows;  // device-mapped pinned [n][C][512] window doubles
  double* out;         // device-mapped pinned [n][C * nfeat] rows
};
inline uint64_t mailbox_request(uint32_t seq, int C, int nfeat, int64_t n) {
  return (uint64_t)seq << 32 | (uint64_t)(C - 1) << 26 | (uint64_t)(nfeat - 1) << 21 |
         (uint64_t)n;
}
hipError_t launch_features_mailbox(hipStream_t st, MailboxCmd* mb, uint64_t idle_ticks,
                                   uint32_t gen);
hipError_t launch_features_small(hipStream_t st, const double* rows, int64_t n, int C, int nfeat,
                                 double* out);
hipError_t launch_synth(hipStream_t st, int16_t* dst, int64_t n_frames, int ct, uint64_t seed);

// Non-temporal reads pay when the regions neighbouring epochs read do not overlap: the average
// marker spacing n_frames / n is at least min_spacing frames (fused.hip).
bool streaming_reads(int64_t n_frames, int64_t n, int64_t min_spacing);

// Fused raw -> features (fused.hip): baseline_kernel then window_kernel.  `scratch` holds
// fused_scratch_bytes(n, C) bytes of device memory (the per-epoch baselines).  fused_supported
// says whether the 3-channel kernels cover (fmt, ct, C); the any-layout kernels of wide.hip take
// the rest.
bool fused_supported(int fmt, int ct, int C, const double* out);
size_t fused_scratch_bytes(int64_t n, int C);
// guard_count: zeroed by the baseline kernel when not null (the 3-channel window kernel recomputes
// the rows that fail the fma conditioning guard itself and uses guard.total only).
hipError_t launch_fused_baseline(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                                 const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                                 void* scratch, int* err, int* guard_count,
                                 const Guard* guard = nullptr);
hipError_t launch_fused_window(hipStream_t st, const void* raw, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                               const void* scratch, double* out, const Guard& guard,
                               bool track = false);
// Algorithmic HBM bytes per epoch of window_kernel (the dominant kernel): window frames, the
// baseline and marker position it reads, the feature row it writes.
int64_t fused_window_bytes_per_epoch(int ct, int C);

// Any-layout fused path (wide.hip): baseline_any_kernel then window_wide_kernel, same scratch
// contract as the 3-channel kernels.  wide_supported: int16/float32, C <= 64, one epoch's staged
// window + features within 64 KB of LDS (int16: about 60 channels in the file).
bool wide_supported(int fmt, int ct, int C);
bool baseline_any_supported(int fmt, int ct, int C);
hipError_t launch_baseline_any(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                               const ChanSel& sel, int C, const int64_t* pos, int64_t n,
                               void* scratch, int* err, int* guard_count,
                               const Guard* guard = nullptr);
hipError_t launch_window_wide(hipStream_t st, const void* raw, int fmt, int64_t n_frames, int ct,
                              const ChanSel& sel, int C, const int64_t* pos, int64_t n, bool fast,
                              const void* scratch, double* out, const Guard& guard,
                              bool track = false);

// guard.hip: the EXACT recomputation of the rows the generic any-layout kernels flagged (no-op
// when g.count is null; launch_window_wide issues it).  raw: the same recording / positions /
// baselines (scratch) as the fused launch.
hipError_t launch_guard_fixup_raw(hipStream_t st, const void* raw, int fmt, int64_t n_frames,
                                  int ct, const ChanSel& sel, int C, const int64_t* pos,
                                  const void* scratch, const Guard& g, double* out);

// logreg.hip: MLlib LogisticRegressionWithSGD (full batch) on device.  State block: iteration
// count, flag (0 running, 1 converged / done, 2 invalid labels), then the d weights.
struct LrState {
  int32_t iter;       // iterations done (GradientDescent's i - 1)
  int32_t converged;  // 1: converged or done, 2: label validation failed
  int32_t updates;    // iterations that updated the weights (a non-empty mini-batch)
  int32_t pad;
  double w[];
};
constexpr int kLrMaxFeatures = 1024;

// plan.hip: marker planning (a4 + a8) as a scan over 3-state balance maps.
struct PlanResult {
  int64_t selected;          // accepted markers
  int64_t balance;           // final class balance
  int64_t first_unparsable;  // index of the first INT32_MIN stimulus index, -1 if none
};
size_t plan_scratch_bytes(int64_t n);
hipError_t launch_plan_markers(hipStream_t st, const int64_t* pos, const int32_t* stim, int64_t n,
                               int64_t n_frames, int32_t guessed, int d0, void* scratch,
                               int64_t* pos_out, double* label_out, PlanResult* result);
int lr_grid(int64_t n);
hipError_t launch_lr_validate(hipStream_t st, const double* y, int64_t n, LrState* state);
// grad: kGradLogistic (LogisticRegressionWithSGD) or kGradHinge (SVMWithSGD); the predict
// kernel scores with the matching model (sigmoid of the margin / the margin itself).
constexpr int kGradLogistic = 0;
constexpr int kGradHinge = 1;
// mask: iteration's mini-batch sample (bit r of word r / 32 = row r), nullptr = the whole batch;
// count = its rows (the gradient's divisor; 0 = an empty sample: no update)
hipError_t launch_lr_iteration(hipStream_t st, int grad, const double* X, const double* y,
                               int64_t n, int d, const uint32_t* mask, int64_t count,
                               LrState* state, double* partial, int G, double step_size,
                               double reg, double tol, int max_iter);
hipError_t launch_lr_predict(hipStream_t st, int grad, const double* X, int64_t n, int d,
                             const double* w, double intercept, double threshold,
                             int use_threshold, double* out);

}  // namespace eegfx
