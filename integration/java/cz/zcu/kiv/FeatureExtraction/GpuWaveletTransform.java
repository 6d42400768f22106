package cz.zcu.kiv.FeatureExtraction;

/**
 * fe=dwt-8 on an MI355X through libeegfx: a drop-in for WaveletTransform(8, 512, 175, 16)
 * (WaveletTransform.java:82-141) behind IFeatureExtraction (IFeatureExtraction.java:27-35).
 * Registered next to the CPU extractor in PipelineBuilder.java:127-139:
 *     case "dwt-8-gpu": fe = new GpuWaveletTransform(8, 512, 175, 16); break;
 * Java 7/8 (Spark 1.6); natives in integration/jni/eegfx_jni.c (libeegfx_jni.so).
 */
public class GpuWaveletTransform implements IFeatureExtraction {
    static { System.loadLibrary("eegfx_jni"); }

    /** Channels the reference extracts (WaveletTransform.CHANNELS = {1, 2, 3}: Fz, Cz, Pz). */
    private static final int CHANNELS = 3;
    private static final int POSTSTIMULUS = 750;   // Const.POSTSTIMULUS_VALUES

    /** -Deegfx.mailbox=true: every thread's context keeps a resident workgroup serving its
     *  one-epoch calls without a kernel launch each (eegfx_ctx_set_mailbox; DESIGN.md section 9). */
    private static final boolean MAILBOX = Boolean.getBoolean("eegfx.mailbox");

    // One device context per calling thread: extractFeatures is reached concurrently from the
    // Spark local[*] executor threads (LogisticRegressionClassifier.java:50,90), and an eegfx
    // context drives one stream.
    private static final ThreadLocal<Long> CTX = new ThreadLocal<Long>() {
        @Override protected Long initialValue() {
            long c = nativeCreate(0);
            if (c == 0) throw new IllegalStateException(nativeLastError());
            if (MAILBOX && nativeSetMailbox(c, true) != 0)
                throw new IllegalStateException(nativeLastError());
            return c;
        }
    };

    // WaveletTransform's constructors (WaveletTransform.java:78-98): the defaults are 8, 512, 175
    // and 16; the four-argument form assigns without the setters' checks, as the reference's
    // does (an unsupported combination is refused by extractFeatures, EEGFX_ENOTSUP); the one-
    // argument form goes through setWaveletName.
    private int epochSize = 512, skipSamples = 175, featureSize = 16;
    private int name;

    public GpuWaveletTransform() { this.name = 8; }

    public GpuWaveletTransform(int name, int epochSize, int skipSamples, int featureSize) {
        this.name = name;
        this.epochSize = epochSize;
        this.skipSamples = skipSamples;
        this.featureSize = featureSize;
    }

    public GpuWaveletTransform(int name) { setWaveletName(name); }

    @Override
    public double[] extractFeatures(double[][] epoch) {
        return extractFeaturesBatch(new double[][][] { epoch })[0];
    }

    /** The batched form: one call per Spark partition (mapPartitions) instead of one per epoch. */
    public double[][] extractFeaturesBatch(double[][][] epochs) {
        int n = epochs.length;
        double[] flat = new double[n * CHANNELS * POSTSTIMULUS];
        for (int i = 0; i < n; i++)
            for (int c = 0; c < CHANNELS; c++)
                System.arraycopy(epochs[i][c], 0, flat, (i * CHANNELS + c) * POSTSTIMULUS, POSTSTIMULUS);
        double[] out = new double[n * CHANNELS * featureSize];
        int rc = nativeExtract(CTX.get(), flat, n, CHANNELS, name, epochSize, skipSamples,
                               featureSize, out);
        if (rc != 0) throw new IllegalArgumentException(nativeLastError());
        double[][] rows = new double[n][CHANNELS * featureSize];
        for (int i = 0; i < n; i++)
            System.arraycopy(out, i * CHANNELS * featureSize, rows[i], 0, CHANNELS * featureSize);
        return rows;
    }

    @Override
    public int getFeatureDimension() { return featureSize * CHANNELS; }

    // The reference's setters and their argument checks (WaveletTransform.java:160-215)
    public void setWaveletName(int name) {
        if (name < 0 || name > 17) throw new IllegalArgumentException("Wavelet Name must be >= 0 and <= 17");
        this.name = name;
    }

    public void setEpochSize(int epochSize) {
        if (epochSize > 0 && epochSize <= POSTSTIMULUS) this.epochSize = epochSize;
        else throw new IllegalArgumentException("Epoch Size must be > 0 and <= " + POSTSTIMULUS);
    }

    public void setSkipSamples(int skipSamples) {
        if (skipSamples > 0 && skipSamples <= POSTSTIMULUS) this.skipSamples = skipSamples;
        else throw new IllegalArgumentException("Skip Samples must be > 0 and <= " + POSTSTIMULUS);
    }

    public void setFeatureSize(int featureSize) {
        if (featureSize > 0 && featureSize <= 1024) this.featureSize = featureSize;
        else throw new IllegalArgumentException("Feature Size must be > 0 and <= 1024");
    }

    // WaveletTransform.java:214-244: same text, same fields compared, same hash
    @Override
    public String toString() {
        return "DWT: EPOCH_SIZE: " + this.epochSize +
                " FEATURE_SIZE: " + this.featureSize +
                " WAVELETNAME: " + this.name +
                " SKIP_SAMPLES: " + this.skipSamples +
                "\n";
    }

    @Override
    public boolean equals(Object o) {
        if (this == o) return true;
        if (o == null || getClass() != o.getClass()) return false;
        GpuWaveletTransform that = (GpuWaveletTransform) o;
        return epochSize == that.epochSize && skipSamples == that.skipSamples
                && name == that.name && featureSize == that.featureSize;
    }

    @Override
    public int hashCode() {
        int result = epochSize;
        result = 31 * result + skipSamples;
        result = 31 * result + name;
        result = 31 * result + featureSize;
        return result;
    }

    private static native long nativeCreate(int device);
    private static native int nativeSetMailbox(long ctx, boolean on);
    private static native int nativeExtract(long ctx, double[] epochs, int n, int C, int name,
                                            int epochSize, int skip, int featureSize, double[] out);
    private static native String nativeLastError();
}
