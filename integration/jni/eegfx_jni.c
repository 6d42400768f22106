/* eegfx_jni.c -- libeegfx_jni.so, the JNI side of the Java drop-in (integration/java/).
 * Each native pins its Java arrays (GetPrimitiveArrayCritical: no copies, no JNI calls until they
 * are released), calls the shim (eegfx_shim.c: the libeegfx call sequence), unpins, and returns
 * the eegfx status; the Java classes raise the reference's exception for a non-zero status
 * (eegfx_shim_exception_class gives the same mapping to native callers).
 *   make -C integration jni        (needs JAVA_HOME; see integration/Makefile) */
#include <jni.h>
#include <stdlib.h>

#include "eegfx_shim.h"

#define PIN(arr) ((arr) ? (jdouble*)(*env)->GetPrimitiveArrayCritical(env, (arr), NULL) : NULL)
#define UNPIN(arr, p, mode) \
  do { if (p) (*env)->ReleasePrimitiveArrayCritical(env, (arr), (p), (mode)); } while (0)

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
  jdouble* in = PIN(epochs);
  jdouble* o = PIN(out);
  const int rc = eegfx_shim_extract(ctx, in, n, C, name, epochSize, skip, featureSize, o);
  UNPIN(out, o, 0);
  UNPIN(epochs, in, JNI_ABORT);
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
  for (jsize i = 0; i < n; ++i) {
    s[i] = (jstring)(*env)->GetObjectArrayElement(env, args, i);
    a[i] = s[i] ? (*env)->GetStringUTFChars(env, s[i], NULL) : "";
  }
  int status = 0;
  const int64_t odp = eegfx_shim_odp_create(ctx, a, (int32_t)n, &status);
  for (jsize i = 0; i < n; ++i)
    if (s[i]) (*env)->ReleaseStringUTFChars(env, s[i], a[i]);
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
  jdouble* o = PIN(out);
  const int rc = eegfx_shim_odp_get_data(odp, o);
  UNPIN(out, o, 0);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpGetLabels(JNIEnv* env, jclass k,
                                                                             jlong odp,
                                                                             jdoubleArray out) {
  (void)k;
  jdouble* o = PIN(out);
  const int rc = eegfx_shim_odp_get_labels(odp, o);
  UNPIN(out, o, 0);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_DataTransformation_GpuOffLineDataProvider_nativeOdpGetFeatures(
    JNIEnv* env, jclass k, jlong odp, jint name, jint epochSize, jint skip, jint featureSize,
    jdoubleArray out) {
  (void)k;
  jdouble* o = PIN(out);
  const int rc = eegfx_shim_odp_get_features(odp, name, epochSize, skip, featureSize, o);
  UNPIN(out, o, 0);
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
  jdouble* px = PIN(x);
  jdouble* py = PIN(y);
  jdouble* pw = PIN(w);
  const int rc = eegfx_shim_lr_train(ctx, px, py, n, d, iters, step, reg, frac, tol, partitions,
                                     pw);
  UNPIN(w, pw, 0);
  UNPIN(y, py, JNI_ABORT);
  UNPIN(x, px, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativePredict(
    JNIEnv* env, jclass k, jlong ctx, jdoubleArray x, jint n, jint d, jdoubleArray w,
    jdoubleArray out) {
  (void)k;
  jdouble* px = PIN(x);
  jdouble* pw = PIN(w);
  jdouble* po = PIN(out);
  const int rc = eegfx_shim_lr_predict(ctx, px, n, d, pw, po);
  UNPIN(out, po, 0);
  UNPIN(w, pw, JNI_ABORT);
  UNPIN(x, px, JNI_ABORT);
  return rc;
}

JNIEXPORT jint JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeStatistics(
    JNIEnv* env, jclass k, jdoubleArray pred, jdoubleArray labels, jint n, jintArray out) {
  (void)k;
  jint tmp[4] = {0, 0, 0, 0};
  jdouble* pp = PIN(pred);
  jdouble* pl = PIN(labels);
  const int rc = eegfx_shim_statistics(pp, pl, n, (int32_t*)tmp);
  UNPIN(labels, pl, JNI_ABORT);
  UNPIN(pred, pp, JNI_ABORT);
  if (rc == EEGFX_OK) (*env)->SetIntArrayRegion(env, out, 0, 4, tmp);
  return rc;
}

JNIEXPORT jstring JNICALL
Java_cz_zcu_kiv_Classification_GpuLogisticRegressionClassifier_nativeLastError(JNIEnv* env,
                                                                               jclass k) {
  (void)k;
  return last_error(env);
}
