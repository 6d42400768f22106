// logreg.hip -- the classifier the reference trains on the feature matrix, on the GPU
// (SURVEY.md 8f rank 4): Spark MLlib 1.6.2 LogisticRegressionWithSGD as called by
// Classification/LogisticRegressionClassifier.java:85-114, i.e. gradient descent with
// LogisticGradient, SquaredL2Updater and GradientDescent's convergence test, no intercept, over
// the whole batch or (miniBatchFraction < 1) over the rows of iteration i's sample, a bit mask
// the host draws with Spark's own sampler (api.cpp spark_sample_mask); and
// LogisticRegressionModel.predict for :117-141.
//
// One iteration = two launches on the context stream, no host round trip:
//   lr_grad_kernel    G workgroups x 4 waves.  Row r goes to wave r mod (4G); a wave's 64 lanes
//                     split the d features (lane k: features k, k+64, ...), so a row is one
//                     coalesced load; margin by a wave butterfly, multiplier = 1/(1+exp(-w.x)) - y,
//                     per-lane gradient accumulators.  The 4 waves of a workgroup are summed in LDS
//                     in wave order and the workgroup's partial gradient stored.
//   lr_update_kernel  one workgroup: partials summed in workgroup order (deterministic), / n, the
//                     SquaredL2Updater step with step/sqrt(i), ||w_prev - w|| < tol*max(||w||, 1)
//                     sets the converged flag (from the second iteration, as GradientDescent).
// Every kernel first reads the flag, so the remaining iterations of a converged run are empty
// launches.  Weights and the iteration state stay in device memory for the whole run.
//
// The same loop with HingeGradient is MLlib 1.6.2 SVMWithSGD (Classification/SVMClassifier.java:
// 83-111: same updater, convergence test and defaults), scored by SVMModel.predict (:71, :114-137):
// the gradient kernels take the gradient as a template parameter (grad_mult).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "launch.h"

namespace eegfx {
namespace dev {

constexpr int kLrWaves = 4;
#ifndef EEGFX_LR_UNROLL
#define EEGFX_LR_UNROLL 4
#endif

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Gradient multiplier of one row (the gradient is mult * x).  GRAD 0 = LogisticGradient (binary):
// 1/(1+exp(-w.x)) - y.  GRAD 1 = HingeGradient (SVMWithSGD): with s = 2y - 1, -s when 1 > s * w.x,
// else 0 (the row adds nothing, as MLlib's axpy is skipped).
template <int GRAD>
__device__ __forceinline__ double grad_mult(double margin, double y) {
  if constexpr (GRAD == 0) {
    return 1.0 / (1.0 + exp(-margin)) - y;
  } else {
    const double s = 2.0 * y - 1.0;
    return 1.0 > s * margin ? -s : 0.0;
  }
}

// Row r of iteration's sample (mask == nullptr: every row).
__device__ __forceinline__ bool sampled(const uint32_t* __restrict__ mask, int64_t r) {
  return !mask || ((mask[r >> 5] >> (r & 31)) & 1u);
}

template <int KD, int GRAD>  // features per lane: d <= 64 * KD
__global__ __launch_bounds__(64 * kLrWaves) void lr_grad_kernel(
    const double* __restrict__ X, const double* __restrict__ y, int64_t n, int d,
    const uint32_t* __restrict__ mask, const LrState* __restrict__ st,
    double* __restrict__ partial) {
  if (st->converged) return;
  __shared__ double acc_s[kLrWaves][64 * KD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const double* wt = st->w;
  double wv[KD], acc[KD];
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int f = lane + 64 * k;
    wv[k] = f < d ? wt[f] : 0.0;
    acc[k] = 0.0;
  }
  const int64_t stride = (int64_t)gridDim.x * kLrWaves;
  for (int64_t r = (int64_t)blockIdx.x * kLrWaves + w; r < n; r += stride) {
    if (!sampled(mask, r)) continue;  // wave-uniform: one row per wave
    const double* row = X + r * d;
    double x[KD];
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < KD; ++k) {
      const int f = lane + 64 * k;
      x[k] = f < d ? row[f] : 0.0;
      dot = __builtin_fma(x[k], wv[k], dot);
    }
    dot = wave_sum(dot);
    const double mult = grad_mult<GRAD>(dot, y[r]);
#pragma unroll
    for (int k = 0; k < KD; ++k) acc[k] = __builtin_fma(mult, x[k], acc[k]);
  }
#pragma unroll
  for (int k = 0; k < KD; ++k) acc_s[w][lane + 64 * k] = acc[k];
  __syncthreads();
  for (int f = threadIdx.x; f < d; f += blockDim.x) {
    double s = acc_s[0][f];
#pragma unroll
    for (int v = 1; v < kLrWaves; ++v) s += acc_s[v][f];
    partial[(int64_t)blockIdx.x * d + f] = s;
  }
}

// Cross-lane move of a double by DPP (two 32-bit halves); all 64 lanes active.
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)u, CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(uint32_t)(u >> 32), CTRL, 0xF, 0xF, false);
  return __builtin_bit_cast(double, ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
}
// Sum over the 16 lanes of a DPP row, result in every lane of the row: quad_perm xor 1, xor 2,
// then row_half_mirror and row_mirror pair the quads and the halves (4 VALU steps, no LDS).
__device__ __forceinline__ double row16_sum(double v) {
  v += dpp_d<0xB1>(v);
  v += dpp_d<0x4E>(v);
  v += dpp_d<0x141>(v);
  v += dpp_d<0x140>(v);
  return v;
}

// d <= 16*FPL: a row is owned by the 16 lanes of one DPP row (lane j: features j, j+16, ...), so
// a wave works on 4 rows at once, two such groups in flight.
template <int FPL, int GRAD>
__global__ __launch_bounds__(64 * kLrWaves) void lr_grad16_kernel(
    const double* __restrict__ X, const double* __restrict__ y, int64_t n, int d,
    const uint32_t* __restrict__ mask, const LrState* __restrict__ st,
    double* __restrict__ partial) {
  if (st->converged) return;
  __shared__ double acc_s[kLrWaves * 4][16 * FPL];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, j = lane & 15;
  double wv[FPL], acc[FPL];
#pragma unroll
  for (int k = 0; k < FPL; ++k) {
    const int f = j + 16 * k;
    wv[k] = f < d ? st->w[f] : 0.0;
    acc[k] = 0.0;
  }
  constexpr int U = EEGFX_LR_UNROLL;  // groups of 4 rows in flight per wave
  const int64_t stride = (int64_t)gridDim.x * kLrWaves * 4 * U;
  for (int64_t r0 = ((int64_t)blockIdx.x * kLrWaves + w) * 4 * U; r0 < n; r0 += stride) {
    double x[U][FPL], dot[U], yy[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional loads from clamped addresses (no exec-mask branch around a load, so all
      // U x FPL loads of the group issue before the first wait).  A row past n re-reads row
      // n-1 and gets multiplier 0 below; a feature slot past d meets weight 0 and is never
      // stored -- real data of the same rows, so non-finite inputs propagate as they would.
      // (Measured per gradient: hinge 0.114 -> 0.082 ms per iteration on 1M x 48; logistic,
      // whose exp the compiler already schedules the guarded loads around, keeps the guarded
      // form: 0.087 vs 0.090 ms.)
      const int64_t r = r0 + 4 * u + q;
      dot[u] = 0.0;
      if constexpr (GRAD == 0) {
        const bool ok = r < n && sampled(mask, r);
        const double* row = X + (ok ? r : 0) * d;
#pragma unroll
        for (int k = 0; k < FPL; ++k) {
          const int f = j + 16 * k;
          x[u][k] = (ok && f < d) ? row[f] : 0.0;
          dot[u] = __builtin_fma(x[u][k], wv[k], dot[u]);
        }
        yy[u] = ok ? y[r] : 0.0;
      } else {
        const double* row = X + (r < n ? r : n - 1) * d;
#pragma unroll
        for (int k = 0; k < FPL; ++k) {
          const int f = j + 16 * k;
          x[u][k] = row[f < d ? f : d - 1];
          dot[u] = __builtin_fma(x[u][k], wv[k], dot[u]);
        }
        yy[u] = y[r < n ? r : n - 1];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double m = row16_sum(dot[u]);
      const bool ok = r0 + 4 * u + q < n && sampled(mask, r0 + 4 * u + q);
      const double mult = ok ? grad_mult<GRAD>(m, yy[u]) : 0.0;
#pragma unroll
      for (int k = 0; k < FPL; ++k) acc[k] = __builtin_fma(mult, x[u][k], acc[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < FPL; ++k) acc_s[w * 4 + q][j + 16 * k] = acc[k];
  __syncthreads();
  for (int f = threadIdx.x; f < d; f += blockDim.x) {
    double s = acc_s[0][f];
#pragma unroll
    for (int v = 1; v < kLrWaves * 4; ++v) s += acc_s[v][f];
    partial[(int64_t)blockIdx.x * d + f] = s;
  }
}

__global__ __launch_bounds__(256) void lr_update_kernel(const double* __restrict__ partial, int G,
                                                        int64_t n, int d, double step_size,
                                                        double reg, double tol, int max_iter,
                                                        LrState* __restrict__ st) {
  if (st->converged) return;
  __shared__ double red[2][256];
  __shared__ double gs[256];
  const int it = st->iter + 1;
  const double step = step_size / sqrt((double)it);
  // partial sums: thread (j, f) adds workgroups b = j, j+K, ... (K groups of d threads), then the
  // K group sums are added in group order -- a fixed order, so runs are bit-reproducible
  const int K = d <= 128 ? (int)blockDim.x / d : 1;
  if (K > 1) {
    const int t = threadIdx.x, jj = t / d, f = t - jj * d;
    if (jj < K) {
      double a0 = 0.0, a1 = 0.0;
      int b = jj;
      for (; b + K < G; b += 2 * K) {
        a0 += partial[(int64_t)b * d + f];
        a1 += partial[(int64_t)(b + K) * d + f];
      }
      if (b < G) a0 += partial[(int64_t)b * d + f];
      gs[t] = a0 + a1;
    }
    __syncthreads();
  }
  double diff2 = 0.0, norm2 = 0.0;
  for (int f = threadIdx.x; f < d; f += blockDim.x) {
    double g = 0.0;
    if (K > 1) {
      for (int jj = 0; jj < K; ++jj) g += gs[jj * d + f];
    } else {
      for (int b = 0; b < G; ++b) g += partial[(int64_t)b * d + f];
    }
    g = g / (double)n;
    const double old = st->w[f];
    double nw = old * (1.0 - step * reg);
    nw = nw + (-step) * g;
    st->w[f] = nw;
    diff2 += (old - nw) * (old - nw);
    norm2 += nw * nw;
  }
  red[0][threadIdx.x] = diff2;
  red[1][threadIdx.x] = norm2;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    st->iter = it;
    const int up = st->updates + 1;
    st->updates = up;
    // GradientDescent.isConverged, checked once two updated iterates exist (with a full batch:
    // from iteration 2; an empty mini-batch updates nothing and tests nothing)
    const double diff = sqrt(red[0][0]), nrm = sqrt(red[1][0]);
    if ((up >= 2 && diff < tol * (nrm > 1.0 ? nrm : 1.0)) || it >= max_iter) st->converged = 1;
  }
}

// An iteration whose mini-batch sample is empty (GradientDescent: "The size of sampled batch is
// zero"): i advances, the weights and the convergence state do not.
__global__ void lr_skip_kernel(int max_iter, LrState* __restrict__ st) {
  if (st->converged || threadIdx.x != 0) return;
  st->iter += 1;
  if (st->iter >= max_iter) st->converged = 1;
}

// KIND 0: LogisticRegressionModel.predictPoint (score = sigmoid(w.x + b)); KIND 1:
// SVMModel.predictPoint (score = the margin w.x + b).  out = score > threshold ? 1 : 0, or the score.
template <int KD, int KIND>
__global__ __launch_bounds__(256) void lr_predict_kernel(const double* __restrict__ X, int64_t n,
                                                         int d, const double* __restrict__ wt,
                                                         double intercept, double threshold,
                                                         int use_threshold,
                                                         double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= n) return;
  double dot = 0.0;
#pragma unroll
  for (int k = 0; k < KD; ++k) {
    const int f = lane + 64 * k;
    if (f < d) dot = __builtin_fma(X[r * d + f], wt[f], dot);
  }
  dot = wave_sum(dot);
  if (lane == 0) {
    const double margin = dot + intercept;
    const double score = KIND == 0 ? 1.0 / (1.0 + exp(-margin)) : margin;
    out[r] = use_threshold ? (score > threshold ? 1.0 : 0.0) : score;
  }
}

// DataValidators.binaryLabelValidator: every label 0.0 or 1.0, else the run fails (flag 2).
__global__ __launch_bounds__(256) void lr_validate_kernel(const double* __restrict__ y, int64_t n,
                                                          LrState* __restrict__ st) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    if (!(y[i] == 0.0 || y[i] == 1.0)) st->converged = 2;
}

}  // namespace dev

hipError_t launch_lr_validate(hipStream_t st, const double* y, int64_t n, LrState* state) {
  const int64_t g = (n + 255) / 256;
  hipLaunchKernelGGL(dev::lr_validate_kernel, dim3((unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g))),
                     dim3(256), 0, st, y, n, state);
  return hipGetLastError();
}

int lr_grid(int64_t n) {
  constexpr int64_t cap = 512;  // 2 workgroups per CU
  const int64_t g = (n + 16 * dev::kLrWaves - 1) / (16 * dev::kLrWaves);  // >= 16 rows per wave
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

#define EEGFX_LR_KD(KD, CALL) \
  case KD:                    \
    CALL;                     \
    break;

template <int GRAD>
static hipError_t lr_iteration(hipStream_t st, const double* X, const double* y, int64_t n, int d,
                               const uint32_t* mask, int64_t count, LrState* state,
                               double* partial, int G, double step_size, double reg, double tol,
                               int max_iter) {
  if (count == 0) {
    hipLaunchKernelGGL(dev::lr_skip_kernel, dim3(1), dim3(64), 0, st, max_iter, state);
    return hipGetLastError();
  }
  if (d <= 128) {
    const int fpl = (d + 15) / 16;
    switch (fpl <= 1 ? 1 : fpl <= 2 ? 2 : fpl <= 3 ? 3 : fpl <= 4 ? 4 : 8) {
      EEGFX_LR_KD(1, hipLaunchKernelGGL((dev::lr_grad16_kernel<1, GRAD>), dim3(G), dim3(256), 0,
                                        st, X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(2, hipLaunchKernelGGL((dev::lr_grad16_kernel<2, GRAD>), dim3(G), dim3(256), 0,
                                        st, X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(3, hipLaunchKernelGGL((dev::lr_grad16_kernel<3, GRAD>), dim3(G), dim3(256), 0,
                                        st, X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(4, hipLaunchKernelGGL((dev::lr_grad16_kernel<4, GRAD>), dim3(G), dim3(256), 0,
                                        st, X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(8, hipLaunchKernelGGL((dev::lr_grad16_kernel<8, GRAD>), dim3(G), dim3(256), 0,
                                        st, X, y, n, d, mask, state, partial))
    }
  } else {
    const int kd = (d + 63) / 64;
    switch (kd <= 1 ? 1 : kd <= 2 ? 2 : kd <= 4 ? 4 : kd <= 8 ? 8 : 16) {
      EEGFX_LR_KD(1, hipLaunchKernelGGL((dev::lr_grad_kernel<1, GRAD>), dim3(G), dim3(256), 0, st,
                                        X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(2, hipLaunchKernelGGL((dev::lr_grad_kernel<2, GRAD>), dim3(G), dim3(256), 0, st,
                                        X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(4, hipLaunchKernelGGL((dev::lr_grad_kernel<4, GRAD>), dim3(G), dim3(256), 0, st,
                                        X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(8, hipLaunchKernelGGL((dev::lr_grad_kernel<8, GRAD>), dim3(G), dim3(256), 0, st,
                                        X, y, n, d, mask, state, partial))
      EEGFX_LR_KD(16, hipLaunchKernelGGL((dev::lr_grad_kernel<16, GRAD>), dim3(G), dim3(256), 0,
                                         st, X, y, n, d, mask, state, partial))
    }
  }
  hipLaunchKernelGGL(dev::lr_update_kernel, dim3(1), dim3(256), 0, st, partial, G, count, d,
                     step_size, reg, tol, max_iter, state);
  return hipGetLastError();
}

hipError_t launch_lr_iteration(hipStream_t st, int grad, const double* X, const double* y,
                               int64_t n, int d, const uint32_t* mask, int64_t count,
                               LrState* state, double* partial, int G, double step_size,
                               double reg, double tol, int max_iter) {
  return grad == kGradHinge ? lr_iteration<1>(st, X, y, n, d, mask, count, state, partial, G,
                                              step_size, reg, tol, max_iter)
                            : lr_iteration<0>(st, X, y, n, d, mask, count, state, partial, G,
                                              step_size, reg, tol, max_iter);
}

template <int KIND>
static hipError_t lr_predict(hipStream_t st, const double* X, int64_t n, int d, const double* w,
                             double intercept, double threshold, int use_threshold, double* out) {
  const dim3 grid((unsigned)((n + 3) / 4));
  const int kd = (d + 63) / 64;
  switch (kd <= 1 ? 1 : kd <= 2 ? 2 : kd <= 4 ? 4 : kd <= 8 ? 8 : 16) {
    EEGFX_LR_KD(1, hipLaunchKernelGGL((dev::lr_predict_kernel<1, KIND>), grid, dim3(256), 0, st, X,
                                      n, d, w, intercept, threshold, use_threshold, out))
    EEGFX_LR_KD(2, hipLaunchKernelGGL((dev::lr_predict_kernel<2, KIND>), grid, dim3(256), 0, st, X,
                                      n, d, w, intercept, threshold, use_threshold, out))
    EEGFX_LR_KD(4, hipLaunchKernelGGL((dev::lr_predict_kernel<4, KIND>), grid, dim3(256), 0, st, X,
                                      n, d, w, intercept, threshold, use_threshold, out))
    EEGFX_LR_KD(8, hipLaunchKernelGGL((dev::lr_predict_kernel<8, KIND>), grid, dim3(256), 0, st, X,
                                      n, d, w, intercept, threshold, use_threshold, out))
    EEGFX_LR_KD(16, hipLaunchKernelGGL((dev::lr_predict_kernel<16, KIND>), grid, dim3(256), 0, st,
                                       X, n, d, w, intercept, threshold, use_threshold, out))
  }
  return hipGetLastError();
}

hipError_t launch_lr_predict(hipStream_t st, int grad, const double* X, int64_t n, int d,
                             const double* w, double intercept, double threshold,
                             int use_threshold, double* out) {
  if (n == 0) return hipSuccess;
  return grad == kGradHinge
             ? lr_predict<1>(st, X, n, d, w, intercept, threshold, use_threshold, out)
             : lr_predict<0>(st, X, n, d, w, intercept, threshold, use_threshold, out);
}
#undef EEGFX_LR_KD

}  // namespace eegfx
