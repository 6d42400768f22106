/* eegfx_jni.c -- libeegfx_jni.so, the JNI side of the Java drop-in (integration/java/).
 * Each native copies its Java input arrays into native buffers (GetDoubleArrayRegion), calls the
 * shim (eegfx_shim.c: the libeegfx call sequence) on those, copies the results back
 * (SetDoubleArrayRegion) and returns the eegfx status; the Java classes raise the reference's
 * exception for a non-zero status (eegfx_shim_exception_class gives the same mapping to native
 * callers).  No JNI critical region is held across device work: a native call may wait on the
 * device for a long time (nativeTrain runs the whole SGD loop, nativeExtract may wait on a busy
 * device), and a critical region blocks the JVM's garbage collector for every thread meanwhile.
 * A buffer that cannot be allocated returns EEGFX_ENOMEM (OutOfMemoryError).
 *   make -C integration jni        (needs JAVA_HOME; see integration/Makefile) */
#include <jni.h>
#include <stdlib.h>

#include "eegfx_shim.h"

/* Native copy of a Java double[] (NULL array -> NULL buffer, *ok stays 1); *ok = 0 when the copy
 * cannot be allocated.  copy = 0 allocates without reading (output arrays). */
static jdouble* take(JNIEnv* env, jdoubleArray arr, int copy, int* ok) {
  if (!arr) return NULL;
  const jsize n = (*env)->GetArrayLength(env, arr);
  jdouble* p = (jdouble*)malloc((n > 0 ? (size_t)n : 1) * sizeof(jdouble));
  if (!p) { *ok = 0; return NULL; }
  if (copy && n > 0) (*env)->GetDoubleArrayRegion(env, arr, 0, n, p);
  return p;
}
/* Writes a native result back into its Java array (when the call succeeded) and frees it. */
static void give(JNIEnv* env, jdoubleArray arr, jdouble* p, int rc) {
  if (!p) return;
  if (rc == EEGFX_OK) (*env)->SetDoubleArrayRegion(env, arr, 0, (*env)->GetArrayLength(env, arr), p);
  free(p);
}

static jstring last_error(JNIEnv* env) { return (*env)->NewStringUTF(env, eegfx_last_error()); }

/* ---- cz.zcu.kiv.FeatureExtraction.GpuWaveletTransform -------------------------------------- */
JNIEXPORT jlong JNICALL
Java_cz_zcu_kiv_FeatureExtraction_GpuWaveletTransform_nativeCreate(JNIEnv* env, jclass k, jint dev) {
  (void)env; (void)k;
  return (jlong)eegfx_shim_ctx_create(dev);
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_FeatureExtraction_GpuWaveletTransform_nativeSetMailbox(JNIEnv* env, jclass k,
                                                                      jlong ctx, jboolean on) {
  (void)env; (void)k;
  return eegfx_shim_ctx_set_mailbox(ctx, on ? 1 : 0);
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_FeatureExtraction_GpuWaveletTransform_nativeExtract(
    JNIEnv* env, jclass k, jlong ctx, jdoubleArray epochs, jint n, jint C, jint name,
    jint epochSize, jint skip, jint featureSize, jdoubleArray out) {
  (void)k;
  int ok = 1;
  jdouble* in = take(env, epochs, 1, &ok);
  jdouble* o = take(env, out, 0, &ok);
  const int rc = ok ? eegfx_shim_extract(ctx, in, n, C, name, epochSize, skip, featureSize, o)
                    : EEGFX_ENOMEM;
  give(env, out, o, rc);
  free(in);
  return rc;
}

JNIEXPORT jstring JNICALL
Java_cz_zcu_kiv_FeatureExtraction_GpuWaveletTransform_nativeLastError(JNIEnv* env, jclass k) {
  (void)k;
  return last_error(env);
}

/* ---- cz.zcu.kiv.DataTransformation.GpuOffLineDataProvider ---------------------------------- */
JNIEXPORT jlong JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeCtxCreate(JNIEnv* env, jclass k,
                                                                          jint dev) {
  (void)env; (void)k;
  return (jlong)eegfx_shim_ctx_create(dev);
}

JNIEXPORT jlong JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpCreate(JNIEnv* env, jclass k,
                                                                          jlong ctx,
                                                                          jobjectArray args) {
  (void)k;
  const jsize n = args ? (*env)->GetArrayLength(env, args) : 0;
  const char** a = (const char**)calloc(n > 0 ? (size_t)n : 1, sizeof(char*));
  jstring* s = (jstring*)calloc(n > 0 ? (size_t)n : 1, sizeof(jstring));
  int ok = a && s;
  for (jsize i = 0; ok && i < n; ++i) {
    s[i] = (jstring)(*env)->GetObjectArrayElement(env, args, i);
    a[i] = s[i] ? (*env)->GetStringUTFChars(env, s[i], NULL) : "";
    if (!a[i]) ok = 0;  /* out of memory (the JVM has an OutOfMemoryError pending) */
  }
  int status = 0;
  const int64_t odp = ok ? eegfx_shim_odp_create(ctx, a, (int32_t)n, &status) : 0;
  for (jsize i = 0; s && a && i < n; ++i)
    if (s[i] && a[i]) (*env)->ReleaseStringUTFChars(env, s[i], a[i]);
  free(s);
  free((void*)a);
  return (jlong)odp;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpLoadData(JNIEnv* env, jclass k,
                                                                            jlong odp) {
  (void)env; (void)k;
  return eegfx_shim_odp_load_data(odp);
}

JNIEXPORT jstring JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpError(JNIEnv* env, jclass k,
                                                                         jlong odp) {
  (void)k;
  return (*env)->NewStringUTF(env, eegfx_shim_odp_error(odp));
}

JNIEXPORT jlong JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpNumEpochs(JNIEnv* env, jclass k,
                                                                             jlong odp) {
  (void)env; (void)k;
  return (jlong)eegfx_shim_odp_num_epochs(odp);
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpGetData(JNIEnv* env, jclass k,
                                                                           jlong odp,
                                                                           jdoubleArray out) {
  (void)k;
  int ok = 1;
  jdouble* o = take(env, out, 0, &ok);
  const int rc = ok ? eegfx_shim_odp_get_data(odp, o) : EEGFX_ENOMEM;
  give(env, out, o, rc);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpGetLabels(JNIEnv* env, jclass k,
                                                                             jlong odp,
                                                                             jdoubleArray out) {
  (void)k;
  int ok = 1;
  jdouble* o = take(env, out, 0, &ok);
  const int rc = ok ? eegfx_shim_odp_get_labels(odp, o) : EEGFX_ENOMEM;
  give(env, out, o, rc);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpGetFeatures(
    JNIEnv* env, jclass k, jlong odp, jint name, jint epochSize, jint skip, jint featureSize,
    jdoubleArray out) {
  (void)k;
  int ok = 1;
  jdouble* o = take(env, out, 0, &ok);
  const int rc = ok ? eegfx_shim_odp_get_features(odp, name, epochSize, skip, featureSize, o) : EEGFX_ENOMEM;
  give(env, out, o, rc);
  return rc;
}

JNIEXPORT void JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpDestroy(JNIEnv* env, jclass k,
                                                                           jlong odp, jlong ctx) {
  (void)env; (void)k;
  eegfx_shim_odp_destroy(odp);
  if (ctx) eegfx_shim_ctx_destroy(ctx);
}

JNIEXPORT jstring JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeLastError(JNIEnv* env, jclass k) {
  (void)k;
  return last_error(env);
}

/* ---- cz.zcu.kiv.Classification.GpuLogisticRegressionClassifier ----------------------------- */
JNIEXPORT jlong JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeCtxCreate(JNIEnv* env,
                                                                               jclass k,
                                                                               jint dev) {
  (void)env; (void)k;
  return (jlong)eegfx_shim_ctx_create(dev);
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeTrain(
    JNIEnv* env, jclass k, jlong ctx, jdoubleArray x, jdoubleArray y, jint n, jint d, jint iters,
    jdouble step, jdouble reg, jdouble frac, jdouble tol, jint partitions, jdoubleArray w) {
  (void)k;
  int ok = 1;
  jdouble* px = take(env, x, 1, &ok);
  jdouble* py = take(env, y, 1, &ok);
  jdouble* pw = take(env, w, 1, &ok);  /* weights in (initial) and out */
  const int rc = ok ? eegfx_shim_lr_train(ctx, px, py, n, d, iters, step, reg, frac, tol,
                                          partitions, pw)
                    : EEGFX_ENOMEM;
  give(env, w, pw, rc);
  free(py);
  free(px);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativePredict(
    JNIEnv* env, jclass k, jlong ctx, jdoubleArray x, jint n, jint d, jdoubleArray w,
    jdoubleArray out) {
  (void)k;
  int ok = 1;
  jdouble* px = take(env, x, 1, &ok);
  jdouble* pw = take(env, w, 1, &ok);
  jdouble* po = take(env, out, 0, &ok);
  const int rc = ok ? eegfx_shim_lr_predict(ctx, px, n, d, pw, po) : EEGFX_ENOMEM;
  give(env, out, po, rc);
  free(pw);
  free(px);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeStatistics(
    JNIEnv* env, jclass k, jdoubleArray pred, jdoubleArray labels, jint n, jintArray out) {
  (void)k;
  jint tmp[4] = {0, 0, 0, 0};
  int ok = 1;
  jdouble* pp = take(env, pred, 1, &ok);
  jdouble* pl = take(env, labels, 1, &ok);
  const int rc = ok ? eegfx_shim_statistics(pp, pl, n, (int32_t*)tmp) : EEGFX_ENOMEM;
  free(pl);
  free(pp);
  if (rc == EEGFX_OK) (*env)->SetIntArrayRegion(env, out, 0, 4, tmp);
  return rc;
}

JNIEXPORT jstring JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeLastError(JNIEnv* env,
                                                                               jclass k) {
  (void)k;
  return last_error(env);
}
