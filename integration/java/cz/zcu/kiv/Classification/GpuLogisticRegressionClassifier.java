package cz.zcu.kiv.Classification;

import java.io.IOException;
import java.util.HashMap;
import java.util.List;

import cz.zcu.kiv.FeatureExtraction.GpuWaveletTransform;
import cz.zcu.kiv.FeatureExtraction.IFeatureExtraction;
import cz.zcu.kiv.Utils.ClassificationStatistics;

/**
 * train_clf=logreg-gpu: LogisticRegressionClassifier (LogisticRegressionClassifier.java:85-141)
 * with MLlib 1.6.2's LogisticRegressionWithSGD run on the device (eegfx_logreg_sgd_train) and
 * LogisticRegressionModel.predict (eegfx_logreg_predict); the statistics keep the reference's
 * reading of the confusion matrix (:129-137, eegfx_shim_statistics).  The feature extractor must
 * be a GpuWaveletTransform (its batched form feeds the rows).  save/load (Spark model
 * directories) are outside the hot path (SURVEY.md section 2).
 */
public class GpuLogisticRegressionClassifier implements IClassifier {
    static { System.loadLibrary("eegfx_jni"); }

    private static final ThreadLocal<Long> CTX = new ThreadLocal<Long>() {
        @Override protected Long initialValue() { return nativeCtxCreate(0); }
    };

    private IFeatureExtraction fe;
    private HashMap<String, String> config = new HashMap<String, String>(5);
    private double[] weights;

    @Override public void setFeatureExtraction(IFeatureExtraction fe) { this.fe = fe; }
    @Override public IFeatureExtraction getFeatureExtraction() { return fe; }
    @Override public void setConfig(HashMap<String, String> config) { this.config = config; }

    @Override
    public void train(List<double[][]> epochs, List<Double> targets, IFeatureExtraction fe) {
        this.fe = fe;
        double[][] x = features(epochs);
        double[] y = new double[targets.size()];
        for (int i = 0; i < y.length; i++) y[i] = targets.get(i);
        // :98-112 -- the three config keys select the static train(rdd, iterations, step,
        // fraction) (regParam 0.0), otherwise new LogisticRegressionWithSGD().run (step 1.0,
        // 100 iterations, regParam 0.01, fraction 1.0); MLlib's convergence tolerance is 0.001
        boolean cfg = config.containsKey("config_num_iterations")
                && config.containsKey("config_step_size")
                && config.containsKey("config_mini_batch_fraction");
        int iters = cfg ? Integer.parseInt(config.get("config_num_iterations")) : 100;
        double step = cfg ? Double.parseDouble(config.get("config_step_size")) : 1.0;
        double frac = cfg ? Double.parseDouble(config.get("config_mini_batch_fraction")) : 1.0;
        double reg = cfg ? 0.0 : 0.01;
        int d = fe.getFeatureDimension();
        weights = new double[d];
        // :87 parallelize(epochs) under local[*]: one slice per available core, which fixes the
        // per-iteration sample(false, frac, 42 + i) when frac < 1
        int partitions = Runtime.getRuntime().availableProcessors();
        check(nativeTrain(CTX.get(), flatten(x, d), y, x.length, d, iters, step, reg, frac, 0.001,
                          partitions, weights));
    }

    @Override
    public ClassificationStatistics test(List<double[][]> epochs, List<Double> targets) {
        if (weights == null) throw new IllegalStateException("The classifier has not been trained");
        double[][] x = features(epochs);
        double[] pred = new double[x.length];
        check(nativePredict(CTX.get(), flatten(x, weights.length), x.length, weights.length,
                            weights, pred));
        double[] y = new double[targets.size()];
        for (int i = 0; i < y.length; i++) y[i] = targets.get(i);
        int[] s = new int[4];                                    // tp, tn, fp, fn
        check(nativeStatistics(pred, y, y.length, s));
        return new ClassificationStatistics(s[0], s[1], s[2], s[3]);
    }

    @Override public void save(String file) throws IOException {
        throw new UnsupportedOperationException("model directories are outside the GPU hot path");
    }

    @Override public void load(String file) {
        throw new UnsupportedOperationException("model directories are outside the GPU hot path");
    }

    private double[][] features(List<double[][]> epochs) {
        return ((GpuWaveletTransform) fe).extractFeaturesBatch(epochs.toArray(new double[0][][]));
    }

    private static double[] flatten(double[][] x, int d) {
        double[] flat = new double[x.length * d];
        for (int i = 0; i < x.length; i++) System.arraycopy(x[i], 0, flat, i * d, d);
        return flat;
    }

    private static void check(int rc) {
        if (rc == -6) throw new ArrayIndexOutOfBoundsException(nativeLastError());   // EEGFX_ERANGE
        if (rc != 0) throw new IllegalArgumentException(nativeLastError());
    }

    private static native long nativeCtxCreate(int device);
    private static native int nativeTrain(long ctx, double[] x, double[] y, int n, int d, int iters,
                                          double step, double reg, double frac, double tol,
                                          int partitions, double[] weights);
    private static native int nativePredict(long ctx, double[] x, int n, int d, double[] w,
                                            double[] out);
    private static native int nativeStatistics(double[] pred, double[] labels, int n, int[] out);
    private static native String nativeLastError();
}
