/* eegfx_shim.c -- see eegfx_shim.h.  C99, links libeegfx.so only. */
#include "eegfx_shim.h"

#include <stddef.h>
#include <stdlib.h>

const char* eegfx_shim_exception_class(int status) {
  switch (status) {
    case EEGFX_OK: return NULL;
    case EEGFX_EIO: return "java/io/IOException";
    case EEGFX_EFORMAT: return "java/lang/NumberFormatException";
    case EEGFX_ERANGE: return "java/lang/ArrayIndexOutOfBoundsException";
    case EEGFX_ENOMEM: return "java/lang/OutOfMemoryError";
    case EEGFX_EHIP: return "java/lang/IllegalStateException";
    default: return "java/lang/IllegalArgumentException";  /* EINVAL, ENOTSUP */
  }
}

int64_t eegfx_shim_ctx_create(int32_t device) {
  eegfx_ctx* ctx = NULL;
  return eegfx_ctx_create(device, &ctx) == EEGFX_OK ? (int64_t)(intptr_t)ctx : 0;
}

int eegfx_shim_ctx_destroy(int64_t ctx) {
  return eegfx_ctx_destroy((eegfx_ctx*)(intptr_t)ctx);
}

int eegfx_shim_ctx_set_mailbox(int64_t ctx, int32_t enable) {
  return eegfx_ctx_set_mailbox((eegfx_ctx*)(intptr_t)ctx, enable ? 1 : 0);
}

int eegfx_shim_extract(int64_t ctx, const double* epochs, int32_t n, int32_t C, int32_t name,
                       int32_t epoch_size, int32_t skip, int32_t feature_size, double* out) {
  return eegfx_extract_features_f64((eegfx_ctx*)(intptr_t)ctx, epochs, n, C, name, epoch_size,
                                    skip, feature_size, out, EEGFX_MEM_HOST);
}

int64_t eegfx_shim_odp_create(int64_t ctx, const char* const* args, int32_t n_args, int* status) {
  eegfx_odp* odp = NULL;
  const int rc = eegfx_odp_create((eegfx_ctx*)(intptr_t)ctx, args, n_args, &odp);
  if (status) *status = rc;
  return rc == EEGFX_OK ? (int64_t)(intptr_t)odp : 0;
}

int eegfx_shim_odp_load_data(int64_t odp) { return eegfx_odp_load_data((eegfx_odp*)(intptr_t)odp); }

const char* eegfx_shim_odp_error(int64_t odp) {
  return eegfx_odp_error((const eegfx_odp*)(intptr_t)odp);
}

int64_t eegfx_shim_odp_num_epochs(int64_t odp) {
  return eegfx_odp_num_epochs((const eegfx_odp*)(intptr_t)odp);
}

int eegfx_shim_odp_get_data(int64_t odp, double* out) {
  return eegfx_odp_get_data((const eegfx_odp*)(intptr_t)odp, out);
}

int eegfx_shim_odp_get_labels(int64_t odp, double* out) {
  return eegfx_odp_get_labels((const eegfx_odp*)(intptr_t)odp, out);
}

int eegfx_shim_odp_get_features(int64_t odp, int32_t name, int32_t epoch_size, int32_t skip,
                                int32_t feature_size, double* out) {
  return eegfx_odp_get_features((eegfx_odp*)(intptr_t)odp, name, epoch_size, skip, feature_size,
                                out);
}

void eegfx_shim_odp_destroy(int64_t odp) { eegfx_odp_destroy((eegfx_odp*)(intptr_t)odp); }

int eegfx_shim_lr_train(int64_t ctx, const double* X, const double* y, int32_t n, int32_t d,
                        int32_t iterations, double step, double reg, double fraction, double tol,
                        int32_t partitions, double* weights) {
  int32_t run = 0;
  return eegfx_logreg_sgd_train_partitioned((eegfx_ctx*)(intptr_t)ctx, X, y, n, d, iterations,
                                            step, reg, fraction, tol, partitions, weights, &run,
                                            EEGFX_MEM_HOST);
}

int eegfx_shim_lr_predict(int64_t ctx, const double* X, int32_t n, int32_t d,
                          const double* weights, double* out) {
  return eegfx_logreg_predict((eegfx_ctx*)(intptr_t)ctx, X, n, d, weights, 0.0, 0.5, out,
                              EEGFX_MEM_HOST);
}

int eegfx_shim_statistics(const double* pred, const double* labels, int32_t n, int32_t out[4]) {
  if ((n > 0 && (!pred || !labels)) || !out) return EEGFX_EINVAL;
  /* the classes of the actual labels, ascending (MulticlassMetrics.labels in Spark 1.6) */
  double cls[2];
  int k = 0;
  for (int32_t i = 0; i < n; ++i) {
    int seen = 0;
    for (int j = 0; j < k; ++j) seen |= cls[j] == labels[i];
    if (seen) continue;
    if (k == 2) return EEGFX_EINVAL;  /* the reference's classifiers are binary */
    cls[k++] = labels[i];
  }
  if (k == 2 && cls[1] < cls[0]) {
    const double t = cls[0];
    cls[0] = cls[1];
    cls[1] = t;
  }
  if (k < 2) return EEGFX_ERANGE;  /* 1 x 1 matrix: confusionMatrix[1] is out of bounds */
  int32_t cm[2][2] = {{0, 0}, {0, 0}};  /* [actual][predicted] */
  for (int32_t i = 0; i < n; ++i) {
    const int a = labels[i] == cls[1];
    if (pred[i] == cls[0]) ++cm[a][0];
    else if (pred[i] == cls[1]) ++cm[a][1];  /* a prediction outside the classes falls out */
  }
  /* toArray is column-major: {cm[0][0], cm[1][0], cm[0][1], cm[1][1]} = tn, fp, fn, tp */
  const int32_t tn = cm[0][0], fp = cm[1][0], fn = cm[0][1], tp = cm[1][1];
  out[0] = tp;
  out[1] = tn;
  out[2] = fp;
  out[3] = fn;
  return EEGFX_OK;
}
