/*
 * eegfx_oracle.c -- CPU restatement of the reference epoch-to-feature path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the
 * `cpu_baseline` leg of bench.py.  Nothing in the product path
 * (eeg_dataanalysispackage_amd/, include/) links, loads or calls it.
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off, no fast-math, so every
 * double/float operation below is one correctly rounded IEEE op in source order).
 *
 * What it restates (all paths relative to the reference checkout):
 *   decode      eegloader-hdfs 2.4 readBinaryData (un-vendored jar, pom.xml:84-88),
 *               behaviour pinned in SURVEY.md Appendix A: v = (float)raw * (float)res.
 *   cut         OffLineDataProvider.java:220-225 Arrays.copyOfRange(ch, pos-100, pos+750)
 *               + DataProviderUtils.java:49-59 toFloatArray (zero pad past the end).
 *   baseline    Utils/Baseline.java:29-42 (sequential fp32 sum of 100, /100f, subtract).
 *   widen       EpochHolder.java:75-91 (double) e[i+100], i < 750.
 *   features    FeatureExtraction/WaveletTransform.java:107-141: per channel copy
 *               epoch[c][175..686], eegdsp 1.0 processSignal (un-vendored jar,
 *               pom.xml:79-83; pinned in SURVEY.md Appendix A: 10-tap Daubechies with
 *               12-decimal literals, periodic extension, pyramid while n >= 10), keep the
 *               first 16 coefficients, then Utils/SignalProcessing.java:38-52 normalize.
 *
 * Pinned against the reference's own goldens (tests/test_oracle_golden.py):
 *   OfflineDataProviderTest.java:81   sum of epochs  == -253772.18676757812
 *   FeatureExtractionTest.java:106    sum of features == -24.861844096031625
 *   /Epochs.csv                       Pz samples, bit-exact
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define PRE 100   /* Const.java:61 PREESTIMULUS_VALUES */
#define POST 750  /* Const.java:62 POSTSTIMULUS_VALUES */
#define CUT (PRE + POST)
#define TAPS 10

/* eegdsp names[8]: SURVEY.md Appendix A (12-decimal literals are load-bearing). */
static const double H[TAPS] = {0.160102397974,  0.603829269797,  0.724308528438,
                               0.138428145901,  -0.242294887066, -0.032244869585,
                               0.077571493840,  -0.006241490213, -0.012580751999,
                               0.003335725285};

static double G[TAPS];
static int g_ready = 0;

static void init_g(void) {
  if (g_ready) return;
  /* g[j] = (-1)^(j+1) * h[9-j]  (quadrature mirror) */
  for (int j = 0; j < TAPS; ++j) G[j] = ((j & 1) ? 1.0 : -1.0) * H[TAPS - 1 - j];
  g_ready = 1;
}

/* a3: decode one sample of a multiplexed recording (fmt 0 = INT_16, 1 = IEEE_FLOAT_32). */
static float decode_sample(const void* raw, int fmt, int64_t frame, int ct, int col, float res) {
  if (fmt == 0) {
    const int16_t* r = (const int16_t*)raw;
    return (float)r[frame * ct + col] * res;
  }
  const float* r = (const float*)raw;
  return r[frame * ct + col] * res;
}

/* a5-a7 for one (epoch, channel): seg[i] = decoded[pos-100+i] (0 past end),
 * fp32 sequential baseline, subtract, widen the 750 post-stimulus samples. */
static void cut_baseline_widen(const void* raw, int fmt, int64_t n_frames, int ct, int col,
                               float res, int64_t pos, double* out750) {
  float seg[CUT];
  int64_t lo = pos - PRE;
  for (int i = 0; i < CUT; ++i) {
    int64_t f = lo + i;
    seg[i] = (f < n_frames) ? decode_sample(raw, fmt, f, ct, col, res) : 0.0f;
  }
  float b = 0.0f;
  for (int i = 0; i < PRE; ++i) b += seg[i];
  b = b / (float)PRE;
  for (int i = 0; i < CUT; ++i) seg[i] -= b;
  for (int i = 0; i < POST; ++i) out750[i] = (double)seg[i + PRE];
}

/* eegdsp DWT, reference-faithful: full pyramid including the unused detail
 * bands, in-place layout [a_L d_L d_{L-1} ... d_1]. */
static void dwt_full(double* x, int n0, double* tmp) {
  for (int n = n0; n >= TAPS; n /= 2) {
    int h = n / 2;
    for (int i = 0; i < h; ++i) {
      double a = 0.0, d = 0.0;
      for (int j = 0; j < TAPS; ++j) {
        int k = (2 * i + j) % n;
        a += x[k] * H[j];
        d += x[k] * G[j];
      }
      tmp[i] = a;
      tmp[i + h] = d;
    }
    memcpy(x, tmp, sizeof(double) * (size_t)(2 * h));
  }
}

/* Minimal cascade: approximations only, details only at the last level.
 * Produces the same first-16 coefficients bit for bit (details never feed back). */
static void dwt_min16(double* x, int n0, double* tmp) {
  int n = n0;
  while (n / 2 >= TAPS) {  /* next level still runs: only approximations needed */
    int h = n / 2;
    for (int i = 0; i < h; ++i) {
      double a = 0.0;
      for (int j = 0; j < TAPS; ++j) a += x[(2 * i + j) % n] * H[j];
      tmp[i] = a;
    }
    memcpy(x, tmp, sizeof(double) * (size_t)h);
    n = h;
  }
  dwt_full(x, n, tmp); /* last level: a and d */
}

/* The minimal cascade covers the first 2*h_last coefficients (a_L ++ d_L) only. */
static int min_cascade_ok(int win, int nfeat) {
  int n = win;
  while (n / 2 >= TAPS) n /= 2;
  return n >= TAPS && nfeat <= 2 * (n / 2);
}

/* WaveletTransform.extractFeatures for one epoch (double[C][750] row-major). */
static void extract_one(const double* epoch, int C, int skip, int win, int nfeat, int faithful,
                        double* out) {
  double* x = (double*)malloc(sizeof(double) * (size_t)win * 2);
  double* tmp = x + win;
  for (int c = 0; c < C; ++c) {
    for (int j = 0; j < win; ++j) x[j] = epoch[(size_t)c * POST + skip + j];
    if (faithful || !min_cascade_ok(win, nfeat)) dwt_full(x, win, tmp);
    else dwt_min16(x, win, tmp);
    for (int j = 0; j < nfeat; ++j) out[c * nfeat + j] = x[j];
  }
  free(x);
  /* SignalProcessing.normalize: sqrt(sum pow(f,2)) in order, then divide. */
  double s = 0.0;
  for (int i = 0; i < C * nfeat; ++i) s += out[i] * out[i];
  s = sqrt(s);
  for (int i = 0; i < C * nfeat; ++i) out[i] = out[i] / s;
}

/* ---------------------------------------------------------------- exports */

void oracle_decode_epochs(const void* raw, int fmt, int64_t n_frames, int ct, const int32_t* cols,
                          const float* res, int C, const int64_t* pos, int64_t n_epochs,
                          double* epochs_out) {
  for (int64_t e = 0; e < n_epochs; ++e)
    for (int c = 0; c < C; ++c)
      cut_baseline_widen(raw, fmt, n_frames, ct, cols[c], res[c], pos[e],
                         epochs_out + ((size_t)e * C + c) * POST);
}

void oracle_extract_features(const double* epochs, int64_t n, int C, int skip, int win, int nfeat,
                             int faithful, double* out) {
  init_g();
  for (int64_t e = 0; e < n; ++e)
    extract_one(epochs + (size_t)e * C * POST, C, skip, win, nfeat, faithful,
                out + (size_t)e * C * nfeat);
}

/* Fused raw -> features for a contiguous epoch range [e0, e1). */
static void process_range(const void* raw, int fmt, int64_t n_frames, int ct, const int32_t* cols,
                          const float* res, int C, const int64_t* pos, int64_t e0, int64_t e1,
                          int skip, int win, int nfeat, int faithful, double* feat) {
  double* ep = (double*)malloc(sizeof(double) * (size_t)C * POST);
  for (int64_t e = e0; e < e1; ++e) {
    for (int c = 0; c < C; ++c)
      cut_baseline_widen(raw, fmt, n_frames, ct, cols[c], res[c], pos[e], ep + (size_t)c * POST);
    extract_one(ep, C, skip, win, nfeat, faithful, feat + (size_t)e * C * nfeat);
  }
  free(ep);
}

typedef struct {
  const void* raw; int fmt; int64_t n_frames; int ct; const int32_t* cols; const float* res;
  int C; const int64_t* pos; int64_t e0, e1; int skip, win, nfeat, faithful; double* feat;
} job_t;

static void* job_main(void* p) {
  job_t* j = (job_t*)p;
  process_range(j->raw, j->fmt, j->n_frames, j->ct, j->cols, j->res, j->C, j->pos, j->e0, j->e1,
                j->skip, j->win, j->nfeat, j->faithful, j->feat);
  return NULL;
}

/* Threads split contiguous epoch ranges (SURVEY.md 8d CPU baseline). */
void oracle_process_recording(const void* raw, int fmt, int64_t n_frames, int ct,
                              const int32_t* cols, const float* res, int C, const int64_t* pos,
                              int64_t n_epochs, int skip, int win, int nfeat, int faithful,
                              int nthreads, double* feat) {
  init_g();
  if (nthreads < 1) nthreads = 1;
  if (nthreads == 1) {
    process_range(raw, fmt, n_frames, ct, cols, res, C, pos, 0, n_epochs, skip, win, nfeat,
                  faithful, feat);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  job_t* jobs = (job_t*)malloc(sizeof(job_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) {
    job_t j = {raw, fmt, n_frames, ct, cols, res, C, pos,
               n_epochs * t / nthreads, n_epochs * (t + 1) / nthreads,
               skip, win, nfeat, faithful, feat};
    jobs[t] = j;
    pthread_create(&th[t], NULL, job_main, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
