/*
 * eegfx_oracle.c -- CPU restatement of the reference epoch-to-feature path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity checker and the
 * `cpu_baseline` leg of bench.py.  Nothing in the product path
 * (eeg_dataanalysispackage_amd/, include/) links, loads or calls it.
 *
 * Build: oracle/Makefile  (gcc -O3 -ffp-contract=off, no fast-math, so every
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

/* ------------------------------------------ optimised CPU baseline (bench only)
 *
 * The same operations as process_range(faithful = 0) in the same order for every epoch, so its
 * features are bit-identical to the faithful path (the unused detail bands never feed back), but
 * organised for a CPU: only the 612 frames that reach the features are decoded (100 baseline +
 * the 512-sample window), the periodic cascade runs on a buffer extended by 8 samples instead of a
 * modulo per tap, nothing is allocated per epoch, and VE epochs advance together with the epoch
 * index innermost so the compiler vectorises across epochs (an AVX2 clone is picked at run time).
 * Used only by bench.py's cpu_baseline leg and the tests that pin it to the faithful path. */
#define VE 4
#define FAST_WIN 512
#define FAST_EXT 8 /* 2i + j <= n + 7 for the last output of a level */

typedef double v4d __attribute__((vector_size(VE * sizeof(double))));

/* unaligned vector load / store (macros: a vector-returning helper trips -Wpsabi) */
#define LD4(dst, p) memcpy(&(dst), (p), sizeof(v4d))
#define ST4(p, v) memcpy((p), &(v), sizeof(v4d))

/* x: [n + 8][VE] samples (epoch innermost), t: scratch of the same size; coef: [16][VE]. */
__attribute__((target_clones("avx2", "default")))
static void fast_cascade(double* x, double* t, int nfeat, double* coef) {
  int n = FAST_WIN;
  while (n / 2 >= TAPS) {
    const int h = n / 2;
    memcpy(x + (size_t)n * VE, x, sizeof(double) * FAST_EXT * VE);
    for (int i = 0; i < h; ++i) {
      v4d a = {0.0, 0.0, 0.0, 0.0};
      for (int j = 0; j < TAPS; ++j) {
        v4d v;
        LD4(v, x + (size_t)(2 * i + j) * VE);
        a += v * H[j];
      }
      ST4(t + (size_t)i * VE, a);
    }
    double* s = x;
    x = t;
    t = s;
    n = h;
  }
  /* last level (n = 16): approximations and details */
  const int h = n / 2;
  memcpy(x + (size_t)n * VE, x, sizeof(double) * FAST_EXT * VE);
  for (int i = 0; i < h; ++i) {
    v4d a = {0.0, 0.0, 0.0, 0.0}, d = {0.0, 0.0, 0.0, 0.0};
    for (int j = 0; j < TAPS; ++j) {
      v4d v;
      LD4(v, x + (size_t)(2 * i + j) * VE);
      a += v * H[j];
      d += v * G[j];
    }
    if (i < nfeat) ST4(coef + (size_t)i * VE, a);
    if (i + h < nfeat) ST4(coef + (size_t)(i + h) * VE, d);
  }
}

static void fast_range(const void* raw, int fmt, int64_t n_frames, int ct, const int32_t* cols,
                       const float* res, int C, const int64_t* pos, int64_t e0, int64_t e1,
                       int skip, int nfeat, double* feat) {
  double* xb = (double*)malloc(sizeof(double) * (size_t)(FAST_WIN + FAST_EXT) * VE * 2);
  double* tb = xb + (size_t)(FAST_WIN + FAST_EXT) * VE;
  double coef[16 * VE];
  for (int64_t g = e0; g < e1; g += VE) {
    const int ne = (int)((e1 - g) < VE ? (e1 - g) : VE);
    for (int c = 0; c < C; ++c) {
      for (int e = 0; e < VE; ++e) {
        if (e >= ne) {
          for (int j = 0; j < FAST_WIN; ++j) xb[(size_t)j * VE + e] = 0.0;
          continue;
        }
        const int64_t lo = pos[g + e] - PRE;
        const int64_t w0 = lo + PRE + skip;
        const float r = res[c];
        float b = 0.0f;
        if (w0 + FAST_WIN <= n_frames && fmt == 0) { /* the whole cut is inside the recording */
          const int16_t* p = (const int16_t*)raw + lo * ct + cols[c];
          for (int i = 0; i < PRE; ++i) b += (float)p[(size_t)i * ct] * r;
          b = b / (float)PRE;
          const int16_t* q = (const int16_t*)raw + w0 * ct + cols[c];
          for (int j = 0; j < FAST_WIN; ++j)
            xb[(size_t)j * VE + e] = (double)((float)q[(size_t)j * ct] * r - b);
          continue;
        }
        for (int i = 0; i < PRE; ++i) {
          const int64_t f = lo + i;
          b += (f < n_frames) ? decode_sample(raw, fmt, f, ct, cols[c], r) : 0.0f;
        }
        b = b / (float)PRE;
        for (int j = 0; j < FAST_WIN; ++j) {
          const int64_t f = w0 + j;
          const float v = (f < n_frames) ? decode_sample(raw, fmt, f, ct, cols[c], r) : 0.0f;
          xb[(size_t)j * VE + e] = (double)(v - b);
        }
      }
      fast_cascade(xb, tb, nfeat, coef);
      for (int e = 0; e < ne; ++e)
        for (int j = 0; j < nfeat; ++j)
          feat[(size_t)(g + e) * C * nfeat + (size_t)c * nfeat + j] = coef[(size_t)j * VE + e];
    }
    for (int e = 0; e < ne; ++e) {
      double* f = feat + (size_t)(g + e) * C * nfeat;
      double s = 0.0;
      for (int i = 0; i < C * nfeat; ++i) s += f[i] * f[i];
      s = sqrt(s);
      for (int i = 0; i < C * nfeat; ++i) f[i] = f[i] / s;
    }
  }
  free(xb);
}

typedef struct {
  const void* raw; int fmt; int64_t n_frames; int ct; const int32_t* cols; const float* res;
  int C; const int64_t* pos; int64_t e0, e1; int skip, nfeat; double* feat;
} fast_job_t;

static void* fast_job_main(void* p) {
  fast_job_t* j = (fast_job_t*)p;
  fast_range(j->raw, j->fmt, j->n_frames, j->ct, j->cols, j->res, j->C, j->pos, j->e0, j->e1,
             j->skip, j->nfeat, j->feat);
  return NULL;
}

/* Returns 0, or -1 when the parameters are outside the optimised layout (win 512, nfeat <= 16,
 * skip + 512 <= 750): callers then use oracle_process_recording. */
int oracle_process_recording_fast(const void* raw, int fmt, int64_t n_frames, int ct,
                                  const int32_t* cols, const float* res, int C,
                                  const int64_t* pos, int64_t n_epochs, int skip, int win,
                                  int nfeat, int nthreads, double* feat) {
  if (win != FAST_WIN || nfeat < 1 || nfeat > 16 || skip < 0 || skip + win > POST) return -1;
  init_g();
  if (nthreads < 1) nthreads = 1;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  fast_job_t* jobs = (fast_job_t*)malloc(sizeof(fast_job_t) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) {
    /* ranges start on VE boundaries so every group but the last is full */
    const int64_t groups = (n_epochs + VE - 1) / VE;
    const int64_t a = groups * t / nthreads * VE, b = groups * (t + 1) / nthreads * VE;
    fast_job_t j = {raw, fmt, n_frames, ct, cols, res, C, pos, a, b < n_epochs ? b : n_epochs,
                    skip, nfeat, feat};
    jobs[t] = j;
    pthread_create(&th[t], NULL, fast_job_main, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}

/* The optimised CPU form of WaveletTransform.extractFeatures on caller epochs (double[n][C][750]):
 * the channels of one epoch share the vector lanes (groups of VE), so a single-epoch call -- the
 * per-epoch drop-in of SURVEY.md 8b -- is vectorised too.  Bit-identical to
 * oracle_extract_features.  Returns -1 outside the optimised layout (see above). */
int oracle_extract_features_fast(const double* epochs, int64_t n, int C, int skip, int win,
                                 int nfeat, double* out) {
  if (win != FAST_WIN || nfeat < 1 || nfeat > 16 || skip < 0 || skip + win > POST) return -1;
  init_g();
  double* xb = (double*)malloc(sizeof(double) * (size_t)(FAST_WIN + FAST_EXT) * VE * 2);
  double* tb = xb + (size_t)(FAST_WIN + FAST_EXT) * VE;
  double coef[16 * VE];
  for (int64_t e = 0; e < n; ++e) {
    const double* ep = epochs + (size_t)e * C * POST;
    double* f = out + (size_t)e * C * nfeat;
    for (int c0 = 0; c0 < C; c0 += VE) {
      for (int j = 0; j < FAST_WIN; ++j)
        for (int l = 0; l < VE; ++l)
          xb[(size_t)j * VE + l] = (c0 + l < C) ? ep[(size_t)(c0 + l) * POST + skip + j] : 0.0;
      fast_cascade(xb, tb, nfeat, coef);
      for (int l = 0; l < VE && c0 + l < C; ++l)
        for (int j = 0; j < nfeat; ++j) f[(c0 + l) * nfeat + j] = coef[(size_t)j * VE + l];
    }
    double s = 0.0;
    for (int i = 0; i < C * nfeat; ++i) s += f[i] * f[i];
    s = sqrt(s);
    for (int i = 0; i < C * nfeat; ++i) f[i] = f[i] / s;
  }
  free(xb);
  return 0;
}
