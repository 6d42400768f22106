package cz.zcu.kiv.DataTransformation;

import java.util.ArrayList;
import java.util.List;

import org.apache.commons.logging.Log;
import org.apache.commons.logging.LogFactory;

/**
 * OffLineDataProvider (OffLineDataProvider.java:42-380) on an MI355X, as a subclass: a caller that
 * holds the provider as an OffLineDataProvider (PipelineBuilder.java:115-120, the
 * OfflineDataProviderTest cases) changes only its `new`.  The constructor keeps the reference's
 * signature (`throws Exception`, :78); loadData, getData and getDataLabels are overridden (:88,
 * :370, :377), so the base class's HDFS client (:90) is never reached.  getFeatures adds the rows
 * of WaveletTransform(8, 512, 175, 16) for every epoch in getData() order, which loadData computes
 * in the same pass over each epoch's frames (eegfx_odp_load_data ->
 * eegfx_process_recording_epochs), so it is a copy of rows that already exist.  Local files only
 * (the reference's HDFS client is out of scope).
 */
public class GpuOffLineDataProvider extends OffLineDataProvider {
    static { System.loadLibrary("eegfx_jni"); }

    private static final Log logger = LogFactory.getLog(GpuOffLineDataProvider.class);
    private static final int CHANNELS = 3, POSTSTIMULUS = 750, FEATURES = 48;
    private final long ctx, odp;

    public GpuOffLineDataProvider(String[] args) throws Exception { // OffLineDataProvider.java:78
        super(args);
        ctx = nativeCtxCreate(0);                                  // eegfx_ctx_create
        if (ctx == 0) throw new IllegalStateException(nativeLastError());
        odp = nativeOdpCreate(ctx, args);                          // eegfx_odp_create
        if (odp == 0) throw new IllegalArgumentException(nativeLastError());
    }

    /** :88-98 -- a failure is logged and swallowed; the epochs loaded before it stay. */
    @Override
    public void loadData() {
        if (nativeOdpLoadData(odp) != 0) logger.fatal(nativeOdpError(odp));
    }

    @Override
    public List<double[][]> getData() {                            // :370-372
        int n = (int) nativeOdpNumEpochs(odp);
        double[] flat = new double[n * CHANNELS * POSTSTIMULUS];
        check(nativeOdpGetData(odp, flat));                        // eegfx_odp_get_data
        List<double[][]> epochs = new ArrayList<double[][]>(n);
        for (int i = 0; i < n; i++) {
            double[][] e = new double[CHANNELS][POSTSTIMULUS];
            for (int c = 0; c < CHANNELS; c++)
                System.arraycopy(flat, (i * CHANNELS + c) * POSTSTIMULUS, e[c], 0, POSTSTIMULUS);
            epochs.add(e);
        }
        return epochs;
    }

    @Override
    public List<Double> getDataLabels() {                          // :377-379
        int n = (int) nativeOdpNumEpochs(odp);
        double[] lab = new double[n];
        check(nativeOdpGetLabels(odp, lab));                       // eegfx_odp_get_labels
        List<Double> out = new ArrayList<Double>(n);
        for (double v : lab) out.add(v);
        return out;
    }

    /** extractFeatures over getData(), computed by loadData (eegfx_odp_get_features). */
    public double[][] getFeatures() {
        int n = (int) nativeOdpNumEpochs(odp);
        double[] flat = new double[n * FEATURES];
        check(nativeOdpGetFeatures(odp, 8, 512, 175, 16, flat));
        double[][] rows = new double[n][FEATURES];
        for (int i = 0; i < n; i++) System.arraycopy(flat, i * FEATURES, rows[i], 0, FEATURES);
        return rows;
    }

    /** Frees the provider and its device context (the reference has no counterpart: GC). */
    public void close() { nativeOdpDestroy(odp, ctx); }

    private static void check(int rc) {
        if (rc != 0) throw new IllegalArgumentException(nativeLastError());
    }

    private static native long nativeCtxCreate(int device);
    private static native long nativeOdpCreate(long ctx, String[] args);
    private static native int nativeOdpLoadData(long odp);
    private static native String nativeOdpError(long odp);
    private static native long nativeOdpNumEpochs(long odp);
    private static native int nativeOdpGetData(long odp, double[] out);
    private static native int nativeOdpGetLabels(long odp, double[] out);
    private static native int nativeOdpGetFeatures(long odp, int name, int epochSize, int skip,
                                                   int featureSize, double[] out);
    private static native void nativeOdpDestroy(long odp, long ctx);
    private static native String nativeLastError();
}
