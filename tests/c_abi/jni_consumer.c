/* The Java drop-in's JNI natives (integration/jni/eegfx_jni.c) RUN without a JVM: this file is a
 * mock JNI environment (tests/c_abi/jni_mock/jni.h: Java arrays and strings as plain structs) that
 * calls every Java_cz_zcu_kiv_* function the way the Java classes in integration/java/ do.
 *
 *   host: GpuLogisticRegressionClassifier.nativeStatistics (the reference's confusion-matrix
 *         reading, and the single-class ArrayIndexOutOfBoundsException status), the planning-only
 *         provider through GpuOffLineDataProvider's natives with no context (infoTrain.txt: 11
 *         epochs, 5 targets, OfflineDataProviderTest.java:65-88), nativeLastError.
 *   gpu:  GpuOffLineDataProvider: nativeCtxCreate, nativeOdpCreate(String[]{info.txt}),
 *         nativeOdpLoadData, nativeOdpNumEpochs, nativeOdpGetData / GetLabels / GetFeatures;
 *         GpuWaveletTransform: nativeCreate, nativeExtract one epoch per call (launched, then with
 *         nativeSetMailbox) and as a batch, equal to getFeatures bit for bit;
 *         GpuLogisticRegressionClassifier: nativeCtxCreate, nativeTrain, nativePredict,
 *         nativeStatistics; nativeOdpDestroy.  Prints the rows and weights as hex floats for
 *         tests/test_gpu_c_abi.py.
 * The mock also checks the natives' array discipline: every array they read is read whole, every
 * output array is written only on success, and no native leaves a string pinned.
 * argv: <info.txt> [gpu].  Exit status 0 = every check made here passed. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <jni.h>

#include "eegfx.h"

#define CHECK(cond, ...)                     \
  do {                                       \
    if (!(cond)) {                           \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                 \
      exit(1);                               \
    }                                        \
  } while (0)

/* ---- the mock JVM objects ------------------------------------------------------------------ */
enum { K_DOUBLES = 1, K_INTS, K_STRING, K_OBJECTS };
struct _jobject {
  int kind;
  jsize n;
  void* data; /* jdouble[n] / jint[n] / char* / jobject[n] */
  int reads, writes;
};
static int pinned_strings = 0;

static jobject new_doubles(jsize n) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = K_DOUBLES;
  o->n = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(jdouble));
  return o;
}
static jobject new_ints(jsize n) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = K_INTS;
  o->n = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(jint));
  return o;
}
static jobject new_string(const char* s) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = K_STRING;
  const size_t len = strlen(s) + 1;
  o->data = malloc(len);
  memcpy(o->data, s, len);
  return o;
}
static jobject new_objects(jsize n, const jobject* v) {
  jobject o = (jobject)calloc(1, sizeof(struct _jobject));
  o->kind = K_OBJECTS;
  o->n = n;
  o->data = calloc(n > 0 ? (size_t)n : 1, sizeof(jobject));
  memcpy(o->data, v, sizeof(jobject) * (size_t)n);
  return o;
}
static void drop(jobject o) {
  if (!o) return;
  free(o->data);
  free(o);
}
#define D(o) ((jdouble*)(o)->data)

static jsize JNICALL m_GetArrayLength(JNIEnv* env, jarray a) {
  (void)env;
  CHECK(a && a->kind != K_STRING, "GetArrayLength on a non-array");
  return a->n;
}
static void JNICALL m_GetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len,
                                           jdouble* buf) {
  (void)env;
  CHECK(a->kind == K_DOUBLES && start >= 0 && len >= 0 && start + len <= a->n,
        "GetDoubleArrayRegion out of bounds");
  memcpy(buf, D(a) + start, sizeof(jdouble) * (size_t)len);
  if (start == 0 && len == a->n) ++a->reads;
}
static void JNICALL m_SetDoubleArrayRegion(JNIEnv* env, jdoubleArray a, jsize start, jsize len,
                                           const jdouble* buf) {
  (void)env;
  CHECK(a->kind == K_DOUBLES && start >= 0 && len >= 0 && start + len <= a->n,
        "SetDoubleArrayRegion out of bounds");
  memcpy(D(a) + start, buf, sizeof(jdouble) * (size_t)len);
  ++a->writes;
}
static void JNICALL m_SetIntArrayRegion(JNIEnv* env, jintArray a, jsize start, jsize len,
                                        const jint* buf) {
  (void)env;
  CHECK(a->kind == K_INTS && start >= 0 && len >= 0 && start + len <= a->n,
        "SetIntArrayRegion out of bounds");
  memcpy((jint*)a->data + start, buf, sizeof(jint) * (size_t)len);
  ++a->writes;
}
static jobject JNICALL m_GetObjectArrayElement(JNIEnv* env, jobjectArray a, jsize i) {
  (void)env;
  CHECK(a->kind == K_OBJECTS && i >= 0 && i < a->n, "GetObjectArrayElement out of bounds");
  return ((jobject*)a->data)[i];
}
static jstring JNICALL m_NewStringUTF(JNIEnv* env, const char* utf) {
  (void)env;
  return new_string(utf ? utf : "");
}
static const char* JNICALL m_GetStringUTFChars(JNIEnv* env, jstring s, jboolean* is_copy) {
  (void)env;
  CHECK(s->kind == K_STRING, "GetStringUTFChars on a non-string");
  if (is_copy) *is_copy = JNI_FALSE;
  ++pinned_strings;
  return (const char*)s->data;
}
static void JNICALL m_ReleaseStringUTFChars(JNIEnv* env, jstring s, const char* chars) {
  (void)env;
  CHECK(s->kind == K_STRING && chars == s->data, "ReleaseStringUTFChars of another string");
  --pinned_strings;
}
static const struct JNINativeInterface_ table = {
    m_GetArrayLength,         m_GetDoubleArrayRegion, m_SetDoubleArrayRegion,
    m_SetIntArrayRegion,      m_GetObjectArrayElement, m_NewStringUTF,
    m_GetStringUTFChars,      m_ReleaseStringUTFChars};
static JNIEnv env_storage = &table;
static JNIEnv* const env = &env_storage;

/* ---- the natives (integration/jni/eegfx_jni.c) ---------------------------------------------- */
#define WT FeatureExtraction_GpuWaveletTransform
#define ODP DataTransformation_GpuOffLineDataProvider
#define LR Classification_GpuLogisticRegressionClassifier
#define CAT_(a, b) a##_##b
#define CAT(a, b) CAT_(a, b)
#define JN(cls, m) CAT(CAT(Java_cz_zcu_kiv, cls), m)
jlong JN(WT, nativeCreate)(JNIEnv*, jclass, jint);
jint JN(WT, nativeSetMailbox)(JNIEnv*, jclass, jlong, jboolean);
jint JN(WT, nativeExtract)(JNIEnv*, jclass, jlong, jdoubleArray, jint, jint, jint, jint, jint, jint,
                           jdoubleArray);
jstring JN(WT, nativeLastError)(JNIEnv*, jclass);
jlong JN(ODP, nativeCtxCreate)(JNIEnv*, jclass, jint);
jlong JN(ODP, nativeOdpCreate)(JNIEnv*, jclass, jlong, jobjectArray);
jint JN(ODP, nativeOdpLoadData)(JNIEnv*, jclass, jlong);
jstring JN(ODP, nativeOdpError)(JNIEnv*, jclass, jlong);
jlong JN(ODP, nativeOdpNumEpochs)(JNIEnv*, jclass, jlong);
jint JN(ODP, nativeOdpGetData)(JNIEnv*, jclass, jlong, jdoubleArray);
jint JN(ODP, nativeOdpGetLabels)(JNIEnv*, jclass, jlong, jdoubleArray);
jint JN(ODP, nativeOdpGetFeatures)(JNIEnv*, jclass, jlong, jint, jint, jint, jint, jdoubleArray);
void JN(ODP, nativeOdpDestroy)(JNIEnv*, jclass, jlong, jlong);
jstring JN(ODP, nativeLastError)(JNIEnv*, jclass);
jlong JN(LR, nativeCtxCreate)(JNIEnv*, jclass, jint);
jint JN(LR, nativeTrain)(JNIEnv*, jclass, jlong, jdoubleArray, jdoubleArray, jint, jint, jint,
                         jdouble, jdouble, jdouble, jdouble, jint, jdoubleArray);
jint JN(LR, nativePredict)(JNIEnv*, jclass, jlong, jdoubleArray, jint, jint, jdoubleArray,
                           jdoubleArray);
jint JN(LR, nativeStatistics)(JNIEnv*, jclass, jdoubleArray, jdoubleArray, jint, jintArray);
jstring JN(LR, nativeLastError)(JNIEnv*, jclass);

enum { C = 3, POST = 750, F = 48 };

static jobject doubles_of(const double* v, jsize n) {
  jobject o = new_doubles(n);
  memcpy(o->data, v, sizeof(double) * (size_t)n);
  return o;
}

int main(int argc, char** argv) {
  CHECK(argc >= 2, "usage: jni_consumer <info.txt> [gpu]");
  const int gpu = argc >= 3 && strcmp(argv[2], "gpu") == 0;
  jclass k = NULL;

  /* GpuLogisticRegressionClassifier.test's statistics (host only) */
  {
    const double p[6] = {1, 0, 1, 1, 0, 0}, l[6] = {1, 0, 0, 1, 1, 0};
    jobject pred = doubles_of(p, 6), lab = doubles_of(l, 6), out = new_ints(4);
    CHECK(JN(LR, nativeStatistics)(env, k, pred, lab, 6, out) == EEGFX_OK, "nativeStatistics");
    const jint* s = (const jint*)out->data;
    CHECK(s[0] == 2 && s[1] == 2 && s[2] == 1 && s[3] == 1, "statistics %d %d %d %d", s[0], s[1],
          s[2], s[3]);
    CHECK(pred->reads == 1 && lab->reads == 1 && out->writes == 1, "statistics array traffic");
    drop(lab);
    const double one[2] = {1, 1};
    jobject lab1 = doubles_of(one, 2), out1 = new_ints(4);
    CHECK(JN(LR, nativeStatistics)(env, k, pred, lab1, 2, out1) == EEGFX_ERANGE,
          "single class -> ArrayIndexOutOfBoundsException status");
    CHECK(out1->writes == 0, "a failed call must not write its output");
    jstring e = JN(LR, nativeLastError)(env, k);
    CHECK(e && e->kind == K_STRING, "nativeLastError");
    drop(e);
    drop(lab1);
    drop(out1);
    drop(pred);
    drop(out);
  }

  /* GpuOffLineDataProvider's natives on the planning-only provider (no context) */
  jobject info = new_string(argv[1]);
  jobject args = new_objects(1, &info);
  {
    const jlong odp = JN(ODP, nativeOdpCreate)(env, k, 0, args);
    CHECK(odp != 0, "planning nativeOdpCreate: %s", eegfx_last_error());
    CHECK(pinned_strings == 0, "nativeOdpCreate left %d strings pinned", pinned_strings);
    CHECK(JN(ODP, nativeOdpLoadData)(env, k, odp) == EEGFX_OK, "planning loadData");
    const jlong n = JN(ODP, nativeOdpNumEpochs)(env, k, odp);
    CHECK(n == 11, "planning: %lld epochs (golden 11)", (long long)n);
    jobject lab = new_doubles((jsize)n);
    CHECK(JN(ODP, nativeOdpGetLabels)(env, k, odp, lab) == EEGFX_OK, "planning getDataLabels");
    double t = 0;
    for (jlong i = 0; i < n; ++i) t += D(lab)[i];
    CHECK(t == 5.0, "planning: %g targets (golden 5)", t);
    jstring e = JN(ODP, nativeOdpError)(env, k, odp);
    CHECK(e && e->kind == K_STRING, "nativeOdpError");
    drop(e);
    drop(lab);
    JN(ODP, nativeOdpDestroy)(env, k, odp, 0);
  }
  if (!gpu) {
    drop(args);
    drop(info);
    printf("jni_consumer ok (host)\n");
    return 0;
  }

  /* new GpuOffLineDataProvider({info.txt}); loadData(); getData(); getDataLabels(); getFeatures() */
  const jlong ctx = JN(ODP, nativeCtxCreate)(env, k, 0);
  CHECK(ctx != 0, "nativeCtxCreate: %s", eegfx_last_error());
  const jlong odp = JN(ODP, nativeOdpCreate)(env, k, ctx, args);
  CHECK(odp != 0, "nativeOdpCreate: %s", eegfx_last_error());
  CHECK(JN(ODP, nativeOdpLoadData)(env, k, odp) == EEGFX_OK, "loadData");
  const jlong n = JN(ODP, nativeOdpNumEpochs)(env, k, odp);
  CHECK(n == 11, "%lld epochs (golden 11)", (long long)n);
  jobject epochs = new_doubles((jsize)(n * C * POST)), lab = new_doubles((jsize)n),
          feat = new_doubles((jsize)(n * F));
  CHECK(JN(ODP, nativeOdpGetData)(env, k, odp, epochs) == EEGFX_OK, "getData");
  CHECK(JN(ODP, nativeOdpGetLabels)(env, k, odp, lab) == EEGFX_OK, "getDataLabels");
  CHECK(JN(ODP, nativeOdpGetFeatures)(env, k, odp, 8, 512, 175, 16, feat) == EEGFX_OK,
        "getFeatures");
  CHECK(epochs->writes == 1 && lab->writes == 1 && feat->writes == 1, "provider array traffic");
  double esum = 0.0; /* OfflineDataProviderTest.java:73-81 */
  for (jlong i = 0; i < n * C; ++i) {
    double s = 0.0;
    for (int j = 0; j < POST; ++j) s += D(epochs)[i * POST + j];
    esum += s;
  }
  CHECK(esum == -253772.18676757812, "epoch sum %.17g (golden -253772.18676757812)", esum);

  /* GpuWaveletTransform.extractFeatures, one epoch per call (launched, then the resident server),
   * and extractFeaturesBatch */
  const jlong wctx = JN(WT, nativeCreate)(env, k, 0);
  CHECK(wctx != 0, "nativeCreate: %s", eegfx_last_error());
  jobject one = new_doubles(C * POST), row = new_doubles(F);
  for (int mailbox = 0; mailbox < 2; ++mailbox) {
    if (mailbox) CHECK(JN(WT, nativeSetMailbox)(env, k, wctx, JNI_TRUE) == EEGFX_OK, "mailbox");
    for (jlong i = 0; i < n; ++i) {
      memcpy(one->data, D(epochs) + i * C * POST, sizeof(double) * C * POST);
      CHECK(JN(WT, nativeExtract)(env, k, wctx, one, 1, C, 8, 512, 175, 16, row) == EEGFX_OK,
            "extractFeatures epoch %lld", (long long)i);
      CHECK(memcmp(row->data, D(feat) + i * F, sizeof(double) * F) == 0,
            "extractFeatures row %lld (mailbox %d) differs from getFeatures", (long long)i,
            mailbox);
    }
  }
  CHECK(JN(WT, nativeSetMailbox)(env, k, wctx, JNI_FALSE) == EEGFX_OK, "mailbox off");
  jobject rows = new_doubles((jsize)(n * F));
  CHECK(JN(WT, nativeExtract)(env, k, wctx, epochs, (jint)n, C, 8, 512, 175, 16, rows) ==
            EEGFX_OK,
        "extractFeaturesBatch");
  CHECK(memcmp(rows->data, feat->data, sizeof(double) * (size_t)(n * F)) == 0,
        "extractFeaturesBatch rows differ from getFeatures");
  /* an unsupported window is refused and leaves the output untouched */
  const int w0 = rows->writes;
  CHECK(JN(WT, nativeExtract)(env, k, wctx, epochs, (jint)n, C, 8, 256, 175, 16, rows) ==
            EEGFX_ENOTSUP,
        "epoch size 256 must be refused");
  CHECK(rows->writes == w0, "a refused call must not write its output");
  for (jlong i = 0; i < n; ++i) {
    printf("row %lld:", (long long)i);
    for (int j = 0; j < F; ++j) printf(" %a", D(feat)[i * F + j]);
    printf("\n");
  }

  /* GpuLogisticRegressionClassifier.train (defaults) / test */
  const jlong lctx = JN(LR, nativeCtxCreate)(env, k, 0);
  CHECK(lctx != 0, "classifier nativeCtxCreate");
  jobject w = new_doubles(F), pred = new_doubles((jsize)n), st = new_ints(4);
  CHECK(JN(LR, nativeTrain)(env, k, lctx, feat, lab, (jint)n, F, 100, 1.0, 0.01, 1.0, 0.001, 4,
                            w) == EEGFX_OK,
        "nativeTrain: %s", eegfx_last_error());
  CHECK(w->writes == 1, "weights written once");
  CHECK(JN(LR, nativePredict)(env, k, lctx, feat, (jint)n, F, w, pred) == EEGFX_OK,
        "nativePredict");
  CHECK(JN(LR, nativeStatistics)(env, k, pred, lab, (jint)n, st) == EEGFX_OK, "nativeStatistics");
  printf("weights:");
  for (int j = 0; j < F; ++j) printf(" %a", D(w)[j]);
  const jint* s = (const jint*)st->data;
  printf("\nstatistics: %d %d %d %d\n", s[0], s[1], s[2], s[3]);

  JN(ODP, nativeOdpDestroy)(env, k, odp, ctx);
  CHECK(eegfx_ctx_destroy((eegfx_ctx*)(intptr_t)wctx) == EEGFX_OK, "destroy extractor context");
  CHECK(eegfx_ctx_destroy((eegfx_ctx*)(intptr_t)lctx) == EEGFX_OK, "destroy classifier context");
  CHECK(pinned_strings == 0, "%d strings left pinned", pinned_strings);
  drop(epochs); drop(lab); drop(feat); drop(one); drop(row); drop(rows); drop(w); drop(pred);
  drop(st); drop(args); drop(info);
  printf("jni_consumer ok (gpu)\n");
  return 0;
}
