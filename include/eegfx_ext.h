/* eegfx_ext.h -- extensions of libeegfx OUTSIDE the hot-path drop-in contract of eegfx.h.
 *
 * SURVEY.md section 2 marks the reference's SVM classifier (Classification/SVMClassifier.java)
 * out of scope for the MI355X hot path; the entry points below were built in round 1 on the
 * device loop of eegfx_logreg_sgd_train (HingeGradient instead of LogisticGradient) and are kept,
 * tested and exported, but not extended, and INTEGRATION.md's drop-in does not rely on them.
 */
#ifndef EEGFX_EXT_H_
#define EEGFX_EXT_H_

#include "eegfx.h"

#ifdef __cplusplus
extern "C" {
#endif

/* SVMClassifier.java:83-111 trains MLlib 1.6.2 SVMWithSGD: the loop above with HingeGradient
 * (s = 2y - 1; rows with 1 > s * w.x add -s * x to the gradient) -- the default constructor (step
 * 1.0, 100 iterations, regParam 0.01, fraction 1.0) or, with the config_* keys, the static
 * train(rdd, iterations, step, config_reg_param, fraction).  Same arguments, errors and device
 * loop as eegfx_logreg_sgd_train, full batch only (mini_batch_fraction < 1: EEGFX_ENOTSUP).
 * eegfx_svm_predict: SVMModel.predict (SVMClassifier.java:71) --
 * margin = w.x + b, out = margin > threshold ? 1 : 0 (MLlib's default threshold 0.0), or the
 * margin itself when threshold is NaN (clearThreshold). */
int eegfx_svm_sgd_train(eegfx_ctx* ctx, const double* X, const double* y, int64_t n, int32_t d,
                        int32_t num_iterations, double step_size, double reg_param,
                        double mini_batch_fraction, double convergence_tol, double* weights,
                        int32_t* iterations_run, int mem);
int eegfx_svm_predict(eegfx_ctx* ctx, const double* X, int64_t n, int32_t d, const double* weights,
                      double intercept, double threshold, double* out, int mem);

#ifdef __cplusplus
}
#endif
#endif /* EEGFX_EXT_H_ */
