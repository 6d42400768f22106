/* The Java drop-in's call sequence, run from C through the JNI shim's core (integration/jni/
 * eegfx_shim.c) -- what GpuOffLineDataProvider, GpuWaveletTransform and
 * GpuLogisticRegressionClassifier (integration/java/) do between their JNI boundaries:
 *
 *   new GpuOffLineDataProvider({info.txt}); loadData(); getData(); getDataLabels(); getFeatures()
 *   GpuWaveletTransform.extractFeatures(epoch) from THREADS threads, one context per thread
 *     (the Java ThreadLocal; Spark local[*] executors), one epoch per call, EEGFX_MEM_HOST
 *   GpuWaveletTransform.extractFeaturesBatch(all epochs)
 *   GpuLogisticRegressionClassifier.train (default LogisticRegressionWithSGD) / test
 *
 * argv: <info.txt> [gpu].  Without "gpu" only the planning-only provider (no context: positions,
 * labels) and the host-side shim functions run.  With "gpu" it prints the getFeatures rows and the
 * trained weights as hex floats ("row i: ...", "weights: ..."), which tests/test_gpu_c_abi.py
 * compares with tests/golden/golden_vectors.json and oracle/mllib_logreg.py.  Exit status 0 =
 * every check made here passed. */
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "eegfx_shim.h"

#define CHECK(cond, ...)                     \
  do {                                       \
    if (!(cond)) {                           \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                 \
      exit(1);                               \
    }                                        \
  } while (0)

enum { C = 3, POST = 750, F = 48, THREADS = 4 };

typedef struct {
  int t;
  int64_t n;
  const double* epochs;
  double* rows;
  int mailbox; /* -Deegfx.mailbox=true */
} worker;

static void* extract_per_epoch(void* arg) {  /* one executor thread, its own context */
  worker* w = (worker*)arg;
  const int64_t ctx = eegfx_shim_ctx_create(0);
  CHECK(ctx != 0, "thread %d ctx: %s", w->t, eegfx_last_error());
  if (w->mailbox)
    CHECK(eegfx_shim_ctx_set_mailbox(ctx, 1) == EEGFX_OK, "thread %d mailbox: %s", w->t,
          eegfx_last_error());
  for (int64_t i = w->t; i < w->n; i += THREADS)
    CHECK(eegfx_shim_extract(ctx, w->epochs + i * C * POST, 1, C, 8, 512, 175, 16,
                             w->rows + i * F) == EEGFX_OK,
          "extract epoch %lld: %s", (long long)i, eegfx_last_error());
  CHECK(eegfx_shim_ctx_destroy(ctx) == EEGFX_OK, "ctx_destroy");
  return NULL;
}

int main(int argc, char** argv) {
  CHECK(argc >= 2, "usage: shim_consumer <info.txt> [gpu]");
  const int gpu = argc >= 3 && strcmp(argv[2], "gpu") == 0;
  const char* args[1] = {argv[1]};

  /* host-side shim functions */
  CHECK(eegfx_shim_exception_class(EEGFX_OK) == NULL, "OK maps to no exception");
  CHECK(strcmp(eegfx_shim_exception_class(EEGFX_ERANGE),
               "java/lang/ArrayIndexOutOfBoundsException") == 0, "ERANGE class");
  CHECK(strcmp(eegfx_shim_exception_class(EEGFX_EINVAL), "java/lang/IllegalArgumentException") == 0,
        "EINVAL class");
  {
    const double pred[6] = {1, 0, 1, 1, 0, 0}, lab[6] = {1, 0, 0, 1, 1, 0};
    int32_t s[4];
    CHECK(eegfx_shim_statistics(pred, lab, 6, s) == EEGFX_OK, "statistics");
    /* actual/predicted: (1,1) x2 -> tp; (0,0) x2 -> tn; actual 0 predicted 1 -> the reference's
     * "fn"; actual 1 predicted 0 -> its "fp" (column-major toArray read as tn, fp, fn, tp) */
    CHECK(s[0] == 2 && s[1] == 2 && s[2] == 1 && s[3] == 1, "statistics %d %d %d %d", s[0], s[1],
          s[2], s[3]);
    const double one[2] = {1, 1};
    CHECK(eegfx_shim_statistics(pred, one, 2, s) == EEGFX_ERANGE, "single class -> AIOOBE");
  }

  /* planning-only provider (no device): the selection of OfflineDataProviderTest.java:65-88 */
  {
    int st = 0;
    const int64_t odp = eegfx_shim_odp_create(0, args, 1, &st);
    CHECK(odp != 0 && st == EEGFX_OK, "planning odp_create: %s", eegfx_last_error());
    CHECK(eegfx_shim_odp_load_data(odp) == EEGFX_OK, "planning load: %s", eegfx_shim_odp_error(odp));
    const int64_t n = eegfx_shim_odp_num_epochs(odp);
    double lab[64];
    CHECK(n == 11 && eegfx_shim_odp_get_labels(odp, lab) == EEGFX_OK, "planning: %lld epochs",
          (long long)n);
    double t = 0;
    for (int64_t i = 0; i < n; ++i) t += lab[i];
    CHECK(t == 5.0, "planning: %g targets (golden 5)", t);
    eegfx_shim_odp_destroy(odp);
  }
  if (!gpu) {
    printf("shim_consumer ok (host)\n");
    return 0;
  }

  /* GpuOffLineDataProvider */
  const int64_t ctx = eegfx_shim_ctx_create(0);
  CHECK(ctx != 0, "ctx_create: %s", eegfx_last_error());
  int st = 0;
  const int64_t odp = eegfx_shim_odp_create(ctx, args, 1, &st);
  CHECK(odp != 0, "odp_create: %s", eegfx_last_error());
  CHECK(eegfx_shim_odp_load_data(odp) == EEGFX_OK, "loadData: %s", eegfx_shim_odp_error(odp));
  const int64_t n = eegfx_shim_odp_num_epochs(odp);
  CHECK(n == 11, "%lld epochs (golden 11)", (long long)n);
  double* epochs = (double*)malloc(sizeof(double) * (size_t)n * C * POST);
  double* lab = (double*)malloc(sizeof(double) * (size_t)n);
  double* feat = (double*)malloc(sizeof(double) * (size_t)n * F);
  CHECK(eegfx_shim_odp_get_data(odp, epochs) == EEGFX_OK, "getData: %s", eegfx_last_error());
  CHECK(eegfx_shim_odp_get_labels(odp, lab) == EEGFX_OK, "getDataLabels");
  CHECK(eegfx_shim_odp_get_features(odp, 8, 512, 175, 16, feat) == EEGFX_OK, "getFeatures: %s",
        eegfx_last_error());
  double esum = 0.0; /* OfflineDataProviderTest.java:73-81: per-epoch, per-channel sums */
  for (int64_t i = 0; i < n; ++i)
    for (int c = 0; c < C; ++c) {
      double s = 0.0;
      for (int k = 0; k < POST; ++k) s += epochs[(i * C + c) * POST + k];
      esum += s;
    }
  CHECK(esum == -253772.18676757812, "epoch sum %.17g (golden -253772.18676757812)", esum);

  /* GpuWaveletTransform.extractFeatures, one epoch per call from THREADS threads: launched per
   * call, then with -Deegfx.mailbox=true (each thread's context serves from a resident workgroup) */
  double* rows = (double*)malloc(sizeof(double) * (size_t)n * F);
  for (int mailbox = 0; mailbox < 2; ++mailbox) {
    pthread_t th[THREADS];
    worker w[THREADS];
    memset(rows, 0, sizeof(double) * (size_t)n * F);
    for (int t = 0; t < THREADS; ++t) {
      w[t] = (worker){t, n, epochs, rows, mailbox};
      CHECK(pthread_create(&th[t], NULL, extract_per_epoch, &w[t]) == 0, "pthread_create");
    }
    for (int t = 0; t < THREADS; ++t) pthread_join(th[t], NULL);
    CHECK(memcmp(rows, feat, sizeof(double) * (size_t)n * F) == 0,
          "per-epoch extractFeatures rows (mailbox %d) differ from getFeatures", mailbox);
  }
  /* extractFeaturesBatch */
  CHECK(eegfx_shim_extract(ctx, epochs, (int32_t)n, C, 8, 512, 175, 16, rows) == EEGFX_OK,
        "extractFeaturesBatch: %s", eegfx_last_error());
  CHECK(memcmp(rows, feat, sizeof(double) * (size_t)n * F) == 0,
        "extractFeaturesBatch rows differ from getFeatures");
  for (int64_t i = 0; i < n; ++i) {
    printf("row %lld:", (long long)i);
    for (int j = 0; j < F; ++j) printf(" %a", feat[i * F + j]);
    printf("\n");
  }

  /* GpuLogisticRegressionClassifier: train (the default constructor's parameters) and test */
  double wts[F];
  memset(wts, 0, sizeof wts);
  CHECK(eegfx_shim_lr_train(ctx, feat, lab, (int32_t)n, F, 100, 1.0, 0.01, 1.0, 0.001, 4, wts) ==
            EEGFX_OK,
        "train: %s", eegfx_last_error());
  double* pred = (double*)malloc(sizeof(double) * (size_t)n);
  CHECK(eegfx_shim_lr_predict(ctx, feat, (int32_t)n, F, wts, pred) == EEGFX_OK, "predict: %s",
        eegfx_last_error());
  int32_t s[4];
  CHECK(eegfx_shim_statistics(pred, lab, (int32_t)n, s) == EEGFX_OK, "statistics");
  printf("weights:");
  for (int j = 0; j < F; ++j) printf(" %a", wts[j]);
  printf("\nstatistics: %d %d %d %d\n", s[0], s[1], s[2], s[3]);
  /* the config path with config_mini_batch_fraction = 0.5 (regParam 0.0, :98-108) over 4 slices */
  memset(wts, 0, sizeof wts);
  CHECK(eegfx_shim_lr_train(ctx, feat, lab, (int32_t)n, F, 20, 1.0, 0.0, 0.5, 0.001, 4, wts) ==
            EEGFX_OK,
        "train (mini-batch): %s", eegfx_last_error());
  printf("weights_minibatch:");
  for (int j = 0; j < F; ++j) printf(" %a", wts[j]);
  printf("\n");

  eegfx_shim_odp_destroy(odp);
  CHECK(eegfx_shim_ctx_destroy(ctx) == EEGFX_OK, "ctx_destroy");
  free(epochs);
  free(lab);
  free(feat);
  free(rows);
  free(pred);
  printf("shim_consumer ok (gpu)\n");
  return 0;
}
