/* eegfx_shim.h -- the logic of the Java drop-in's JNI shim (integration/jni/eegfx_jni.c) as plain
 * C: everything between pinning the Java arrays and returning a status.  The JNI functions only
 * pin/unpin arrays and convert strings; the calls into libeegfx, their order and their arguments
 * live here, so the exact sequence the Java classes run is built and tested without a JDK
 * (tests/c_abi/shim_consumer.c, tests/test_gpu_c_abi.py).
 *
 * Reference seams:
 *   GpuWaveletTransform        -> IFeatureExtraction (FeatureExtraction/IFeatureExtraction.java:27-35),
 *                                 WaveletTransform(8, 512, 175, 16) (WaveletTransform.java:82-141),
 *                                 registered as fe=dwt-8-gpu next to PipelineBuilder.java:127-139
 *   GpuOffLineDataProvider     -> OffLineDataProvider (DataTransformation/OffLineDataProvider.java:78,
 *                                 88-98, 370-379)
 *   GpuLogisticRegressionClassifier -> LogisticRegressionClassifier.train/test
 *                                 (Classification/LogisticRegressionClassifier.java:85-141) */
#ifndef EEGFX_SHIM_H_
#define EEGFX_SHIM_H_

#include <stdint.h>

#include "eegfx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Java exception class (JNI name) for an eegfx status, the exception the reference throws at the
 * same point; NULL for EEGFX_OK. */
const char* eegfx_shim_exception_class(int status);

/* ---- GpuWaveletTransform ------------------------------------------------------------------ */
/* nativeCreate: one context per calling thread (the Java ThreadLocal; Spark local[*] executor
 * threads reach extractFeatures concurrently, LogisticRegressionClassifier.java:50,90).  Returns
 * 0 on failure (eegfx_last_error has the text). */
int64_t eegfx_shim_ctx_create(int32_t device);
int eegfx_shim_ctx_destroy(int64_t ctx);
/* opt-in resident per-epoch server of the context (eegfx_ctx_set_mailbox); GpuWaveletTransform
 * turns it on for every executor thread's context when -Deegfx.mailbox=true */
int eegfx_shim_ctx_set_mailbox(int64_t ctx, int32_t enable);
/* nativeExtract: n epochs double[n][C][750] (flattened by the Java side from its double[][][]) ->
 * rows double[n][C * feature_size] in host memory (EEGFX_MEM_HOST: one epoch takes the
 * per-epoch latency kernel, batches the chunked-copy path). */
int eegfx_shim_extract(int64_t ctx, const double* epochs, int32_t n, int32_t C, int32_t name,
                       int32_t epoch_size, int32_t skip, int32_t feature_size, double* out);

/* ---- GpuOffLineDataProvider --------------------------------------------------------------- */
/* nativeOdpCreate(ctx, String[] args): returns the provider handle or 0 (status in *status). */
int64_t eegfx_shim_odp_create(int64_t ctx, const char* const* args, int32_t n_args, int* status);
/* nativeOdpLoadData: the reference swallows and logs load errors (:88-98); the status is returned
 * for the Java side to log, the epochs loaded before the error stay. */
int eegfx_shim_odp_load_data(int64_t odp);
const char* eegfx_shim_odp_error(int64_t odp);
int64_t eegfx_shim_odp_num_epochs(int64_t odp);
int eegfx_shim_odp_get_data(int64_t odp, double* out);     /* double[n][3][750] */
int eegfx_shim_odp_get_labels(int64_t odp, double* out);   /* double[n]         */
int eegfx_shim_odp_get_features(int64_t odp, int32_t name, int32_t epoch_size, int32_t skip,
                                int32_t feature_size, double* out);
void eegfx_shim_odp_destroy(int64_t odp);

/* ---- GpuLogisticRegressionClassifier ------------------------------------------------------ */
/* nativeTrain: MLlib LogisticRegressionWithSGD on the device (host arrays); weights in/out.
 * partitions: the training RDD's partition count, which fixes Spark's per-iteration mini-batch
 * sample when fraction < 1 -- parallelize(epochs) under local[*] makes defaultParallelism =
 * Runtime.availableProcessors() slices (LogisticRegressionClassifier.java:87). */
int eegfx_shim_lr_train(int64_t ctx, const double* X, const double* y, int32_t n, int32_t d,
                        int32_t iterations, double step, double reg, double fraction, double tol,
                        int32_t partitions, double* weights);
/* nativePredict: LogisticRegressionModel.predict with the default threshold 0.5. */
int eegfx_shim_lr_predict(int64_t ctx, const double* X, int32_t n, int32_t d,
                          const double* weights, double* out);
/* nativeStatistics: LogisticRegressionClassifier.test :129-137 -- MulticlassMetrics' confusion
 * matrix over the classes of the ACTUAL labels (ascending), flattened column-major by toArray and
 * read as tn, fp, fn, tp = cm[0], cm[1], cm[2], cm[3].  out = {tp, tn, fp, fn}, the
 * ClassificationStatistics constructor's order.  A single actual class gives a 1 x 1 matrix, whose
 * cm[1] the reference reads out of bounds: EEGFX_ERANGE (ArrayIndexOutOfBoundsException). */
int eegfx_shim_statistics(const double* pred, const double* labels, int32_t n, int32_t out[4]);

#ifdef __cplusplus
}
#endif
#endif /* EEGFX_SHIM_H_ */
