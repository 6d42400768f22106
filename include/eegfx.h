/*
 * eegfx.h -- C ABI of the MI355X-native epoch-to-feature path.
 *
 * This is the drop-in boundary for the reference's hot path
 * (NEUROINFORMATICS-GROUP-FAV-KIV-ZCU/EEG_DataAnalysisPackage, paths relative to its checkout):
 *
 *   src/main/java/cz/zcu/kiv/DataTransformation/OffLineDataProvider.java   (processEEGFiles)
 *   src/main/java/cz/zcu/kiv/FeatureExtraction/IFeatureExtraction.java     (extractFeatures)
 *   src/main/java/cz/zcu/kiv/FeatureExtraction/WaveletTransform.java       (fe=dwt-8)
 *
 * Every entry point below names the reference interface it replaces.  The ABI is plain C:
 * no C++ or torch types, caller-owned buffers, int status returns (0 = ok, < 0 = error),
 * error text from eegfx_last_error() (thread-local).  Java binds it through JNI
 * (INTEGRATION.md); Python binds it through ctypes (eeg_dataanalysispackage_amd/_lib.py).
 *
 * Threading: every function is reentrant.  Calls that take an eegfx_ctx serialise on that
 * context's HIP stream; use one context per calling thread (e.g. per Spark executor thread,
 * LogisticRegressionClassifier.java:50,90) for concurrency.
 *
 * Memory: pointer arguments of compute calls are host or device pointers as selected by the
 * `mem` argument (EEGFX_MEM_HOST: the library stages through its own device buffers and
 * returns after the results are back in host memory; EEGFX_MEM_DEVICE: pointers are HIP
 * device pointers, the work is enqueued on the context stream and the call returns without
 * synchronising -- call eegfx_ctx_synchronize()).  Device-resident marker positions are
 * validated by the kernels that read them (OffLineDataProvider.java:220-225: pos-100 must lie
 * in [0, n_frames]); a violation is reported as EEGFX_ERANGE by the next call on that context
 * that synchronises it, which also clears it.  The calls that synchronise are
 * eegfx_ctx_synchronize, eegfx_ctx_guard_stats / _detail, every EEGFX_MEM_HOST compute call,
 * eegfx_read_raw with EEGFX_MEM_DEVICE, eegfx_logreg_sgd_train / eegfx_svm_sgd_train, and
 * eegfx_logreg_predict / eegfx_svm_predict with EEGFX_MEM_DEVICE.  When such a call returns
 * EEGFX_ERANGE for an earlier call's position, its own work has completed and its outputs are
 * valid; the rows of the epochs with the refused positions are unspecified.  Results of
 * EEGFX_MEM_DEVICE calls are unspecified until a synchronising call has returned EEGFX_OK.  Host
 * positions are checked before any work is enqueued and fail the call itself.
 *
 * Numerics: EEGFX_EXACT reproduces the reference's fp64 operation order value for value;
 * EEGFX_FMA runs the fused-multiply-add filter bank and is within 1e-9 of it on every row: a
 * conditioning guard bounds each row's rounding difference from the EXACT row,
 * and the rows it cannot certify (features at rounding level, e.g. a window in the filters' null
 * space) are recomputed under EXACT on the device before the call's results are complete.
 * Small host batches of eegfx_extract_features_f64 (the per-epoch drop-in) are computed under
 * EXACT in both settings (latency-bound; the guard's counters do not count them).
 */
#ifndef EEGFX_H_
#define EEGFX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define EEGFX_ABI_VERSION 1

/* ---- status codes ---------------------------------------------------------------------- */
#define EEGFX_OK 0
#define EEGFX_EINVAL -1    /* bad argument: IllegalArgumentException in the reference      */
#define EEGFX_EIO -2       /* file missing / unreadable: IOException                       */
#define EEGFX_EFORMAT -3   /* malformed .vhdr/.vmrk/info.txt: NumberFormatException & co.  */
#define EEGFX_EHIP -4      /* HIP runtime error                                            */
#define EEGFX_ENOMEM -5    /* allocation failure                                           */
#define EEGFX_ERANGE -6    /* epoch out of range: ArrayIndexOutOfBoundsException           */
#define EEGFX_ENOTSUP -7   /* parameter combination without a kernel                       */

/* ---- constants of the reference (Utils/Const.java:61-71, WaveletTransform.java:47-87) ---- */
#define EEGFX_PRESTIMULUS 100   /* Const.PREESTIMULUS_VALUES  */
#define EEGFX_POSTSTIMULUS 750  /* Const.POSTSTIMULUS_VALUES  */
#define EEGFX_USED_CHANNELS 3   /* Const.USED_CHANNELS        */
#define EEGFX_DWT8_NAME 8       /* fe=dwt-8: WaveletTransform(8, 512, 175, 16), PipelineBuilder.java:131 */
#define EEGFX_DWT8_EPOCH_SIZE 512
#define EEGFX_DWT8_SKIP 175
#define EEGFX_DWT8_FEATURE_SIZE 16

/* sample formats of BrainVision BinaryFormat= */
#define EEGFX_INT_16 0
#define EEGFX_IEEE_FLOAT_32 1

#define EEGFX_MEM_HOST 0
#define EEGFX_MEM_DEVICE 1

/* numerics of the DWT filter bank */
#define EEGFX_EXACT 0   /* separate fp64 mul + add in the reference order: bit-exact to Java */
#define EEGFX_FMA 1     /* fp64 fused multiply-add: within 1e-9 relative, fewer instructions;
                           rows the conditioning guard cannot certify are recomputed EXACT */

typedef struct eegfx_ctx eegfx_ctx;
typedef struct eegfx_odp eegfx_odp;

/* ---- library / context ------------------------------------------------------------------ */
const char* eegfx_version(void);
const char* eegfx_last_error(void);
int eegfx_device_count(int* count);
/* Creates a context on HIP device `device` with its own non-blocking stream. */
int eegfx_ctx_create(int device, eegfx_ctx** out);
/* Makes the context enqueue on `hip_stream` (hipStream_t, e.g. torch's current stream);
 * NULL restores the context's own stream.  The previous stream is drained first (the context's
 * device buffers are allocated and released in its stream's order).  The context keeps using an
 * external stream until told otherwise -- eegfx_ctx_destroy drains and frees on it too -- so call
 * eegfx_ctx_set_stream(ctx, NULL) before the caller destroys that stream. */
int eegfx_ctx_set_stream(eegfx_ctx* ctx, void* hip_stream);
/* The stream the context currently enqueues on (hipStream_t). */
int eegfx_ctx_stream(eegfx_ctx* ctx, void** hip_stream);
int eegfx_ctx_set_numerics(eegfx_ctx* ctx, int numerics); /* EEGFX_EXACT (default) | EEGFX_FMA */
/* Waits for the context's stream; EEGFX_ERANGE if a kernel enqueued since the last call met a
 * device-resident marker position the reference would not cut (the flag is cleared). */
int eegfx_ctx_synchronize(eegfx_ctx* ctx);
/* Kernel timing for the roofline leg of bench.py.  While enabled, every compute call brackets its
 * dominant kernel (window_kernel for the fused path) with a pair of HIP events on the context
 * stream; eegfx_ctx_kernel_stats returns the number of timed launches, their summed duration
 * (ms) and the algorithmic HBM bytes they moved.  Enabling (again) resets the counters. */
int eegfx_ctx_set_timing(eegfx_ctx* ctx, int enable);
int eegfx_ctx_kernel_stats(eegfx_ctx* ctx, int64_t* launches, double* total_ms,
                           int64_t* total_bytes);
/* The fma numerics' conditioning guard: rows that went through a guarded (EEGFX_FMA) feature
 * launch on this context, and rows the guard recomputed under EEGFX_EXACT, since the context was
 * created or last reset (reset != 0 clears both after reading).  Synchronises the context.
 * Guarded launches include the feature rows eegfx_odp_load_data computes for the provider's
 * resident feature matrix (eegfx_odp_get_features copies them), on the context it was given. */
int eegfx_ctx_guard_stats(eegfx_ctx* ctx, int64_t* rows_checked, int64_t* rows_recomputed,
                          int reset);
/* The same counters, with the rows that failed the guard's a-priori test and went to its second
 * stage (the row's measured max |x|): rows_rechecked >= rows_recomputed, and
 * rows_rechecked - rows_recomputed rows were certified by the second stage.  rows_rechecked may be
 * NULL. */
int eegfx_ctx_guard_detail(eegfx_ctx* ctx, int64_t* rows_checked, int64_t* rows_rechecked,
                           int64_t* rows_recomputed, int reset);
/* Opt-in resident server for the per-epoch drop-in (IFeatureExtraction.extractFeatures called
 * once per epoch, LogisticRegressionClassifier.java:55-61): enable != 0 starts one resident
 * workgroup on its own stream that polls a host-mapped command word, so single-epoch
 * EEGFX_MEM_HOST eegfx_extract_features_f64 calls on this context (C <= 16) are served without a
 * kernel launch or a stream synchronisation -- the same device code, the same rows (small
 * batches of more epochs stay on the launch path, which runs them in parallel).  It returns by itself after 1 s without a request (and is restarted by the next one), or
 * when disabled / the context is destroyed.  While it runs, a device-wide synchronisation
 * (hipDeviceSynchronize, hipFree, hipHostFree) waits for it: disable it before such calls (the
 * library makes none: its pinned buffers are pooled for the process, its device buffers are
 * allocated and freed stream-ordered, so creating and destroying contexts never waits).  Its
 * stream has the highest priority, which keeps it on a hardware queue of its own (streams of one
 * priority share a few queues in order).  That pool has 4 queues, so at most 4
 * contexts of a process hold a server on one device at a time: a context enabled beyond that
 * serves its calls on the launch path (same rows) and takes a server once a slot frees.  A
 * server that has not started within 20 ms of its launch (its queue held by other work) is
 * stopped and the call takes the launch path; no request is ever posted to a server that has not
 * started.  Off by default. */
int eegfx_ctx_set_mailbox(eegfx_ctx* ctx, int enable);
/* Whether the resident server is enabled on ctx and whether it currently holds a slot with a
 * started server (either pointer may be NULL). */
int eegfx_ctx_get_mailbox(eegfx_ctx* ctx, int32_t* enabled, int32_t* resident);
int eegfx_ctx_destroy(eegfx_ctx* ctx);

/* ---- BrainVision reader (replaces eegloader-hdfs 2.4 cz.zcu.kiv.signal.*, pom.xml:84-88) - */
typedef struct {
  int32_t number;        /* 1-based channel number (Ch<n>=)            ChannelInfo.getNumber() */
  char name[64];         /* first field, "\1" decoded to ','           ChannelInfo.getName()   */
  char reference[64];
  double resolution;     /* third field; 1.0 when empty                                        */
  char unit[32];         /*                                            ChannelInfo.getUnits()  */
} eegfx_channel_info;

typedef struct {
  int32_t n_channels;          /* NumberOfChannels=                                           */
  int32_t binary_format;       /* EEGFX_INT_16 | EEGFX_IEEE_FLOAT_32                           */
  int32_t multiplexed;         /* DataOrientation=MULTIPLEXED -> 1, VECTORIZED -> 0           */
  double sampling_interval_us; /* SamplingInterval=                                           */
  char data_file[512];
  char marker_file[512];
} eegfx_header_info;

typedef struct {
  int32_t number;         /* Mk<n>                                                           */
  char type[64];          /* e.g. "Stimulus", "New Segment"                                  */
  char description[64];   /* e.g. "S  2"                       EEGMarker.getStimulus()       */
  int64_t position;       /* data point, used verbatim as a 0-based index                    */
  int64_t size;
  int32_t channel;
  int32_t stimulus_index; /* int(digits(description)) - 1, or -1 (OffLineDataProvider.java:207-214) */
} eegfx_marker;

/* DataTransformer.getChannelInfo(vhdr) (OffLineDataProvider.java:167-168). `channels` may be
 * NULL to query; at most max_channels entries are written. */
int eegfx_read_header(const char* vhdr_path, eegfx_header_info* info,
                      eegfx_channel_info* channels, int32_t max_channels);
/* DataTransformer.readMarkerList(vmrk) (OffLineDataProvider.java:196). `markers` may be NULL
 * to query the count. */
int eegfx_read_markers(const char* vmrk_path, eegfx_marker* markers, int64_t max_markers,
                       int64_t* n_markers);
/* Number of frames of a .eeg file given its header (file size / (channels * sample size)). */
int eegfx_recording_frames(const char* vhdr_path, const char* eeg_path, int64_t* n_frames);
/* Reads the raw multiplexed samples of a .eeg file into `dst` (n_frames * n_channels samples of
 * the header's binary format; host or device memory per `mem`).  A DataOrientation=VECTORIZED
 * file (channel after channel) is interleaved into the same multiplexed layout while it is read.
 * The decode itself (a3) is done by the kernels, fused with the epoch cut. */
int eegfx_read_raw(eegfx_ctx* ctx, const char* vhdr_path, const char* eeg_path, void* dst,
                   int64_t capacity_bytes, int mem);

/* ---- marker planning: OffLineDataProvider.java:200-265 (a4 + a8) ----------------------------
 * For each marker in order: skip it (no state change) iff position-100 < 0 or
 * position-100 > n_frames (the AIOOBE of Arrays.copyOfRange, :220-225, caught at :262-264);
 * target iff stimulus_index+1 == guessed (:238-240); class balance (:248-260) with
 * *balance = numberOfTargets - numberOfNonTargets carried across files: accept a target iff
 * *balance <= 0, a non-target iff *balance >= 0.  Writes the accepted positions and labels
 * (1.0 / 0.0) in order.  pos_out/label_out may be NULL to count. */
int eegfx_plan_markers(const eegfx_marker* markers, int64_t n_markers, int64_t n_frames,
                       int32_t guessed, int64_t* balance, int64_t* pos_out, double* label_out,
                       int64_t* n_selected);

/* The same planning on the device, for marker lists of configs[2] size (64M markers): each marker
 * is a map of the balance state {-1, 0, 1} (target: D <= 0 -> D + 1; non-target: D >= 0 -> D - 1;
 * out of range: identity), so the sequential walk is a prefix composition, scanned
 * in parallel, followed by a stream compaction of the accepted markers.  positions /
 * stimulus_index (INT32_MIN = unparsable description: planning stops there with EEGFX_EFORMAT,
 * the accepted prefix kept) and pos_out / label_out per `mem`; *balance must be -1, 0 or 1 (the
 * reference's balance starts at 0 and never leaves that set). */
int eegfx_plan_markers_device(eegfx_ctx* ctx, const int64_t* positions,
                              const int32_t* stimulus_index, int64_t n_markers, int64_t n_frames,
                              int32_t guessed, int64_t* balance, int64_t* pos_out,
                              double* label_out, int64_t* n_selected, int mem);

/* ---- compute ------------------------------------------------------------------------------ */
/* a3 + a5..a7: raw multiplexed recording -> baseline-corrected epochs double[n][C][750]
 * (OffLineDataProvider.java:216-233 + EpochHolder.setFZ/CZ/PZ, the List<double[][]> that
 * getData() returns).  cols[c] = 0-based column of selected channel c, res[c] its resolution
 * (host arrays, C <= 64).  raw/pos/epochs_out per `mem`. */
int eegfx_cut_epochs_f64(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                         int32_t n_channels_total, const int32_t* cols, const float* res,
                         int32_t C, const int64_t* pos, int64_t n_epochs, double* epochs_out,
                         int mem);

/* IFeatureExtraction.extractFeatures (IFeatureExtraction.java:27-35), batched over n epochs:
 * WaveletTransform(name, epoch_size, skip, feature_size).extractFeatures for each
 * epochs[i] = double[C][750] (WaveletTransform.java:107-141).  out = double[n][C*feature_size],
 * each row L2-normalised (SignalProcessing.java:38-52).  Supported: name 8 with epoch_size 512,
 * skip + 512 <= 750 and feature_size <= 16 (the coefficients a6 ++ d6), C <= 64. */
int eegfx_extract_features_f64(eegfx_ctx* ctx, const double* epochs, int64_t n, int32_t C,
                               int32_t name, int32_t epoch_size, int32_t skip,
                               int32_t feature_size, double* out, int mem);

/* The fused hot path: raw multiplexed recording -> dwt-8 feature matrix, without materialising
 * the epochs.  Equals eegfx_cut_epochs_f64 followed by eegfx_extract_features_f64 with
 * (8, 512, 175, 16), bit for bit under EEGFX_EXACT. */
int eegfx_process_recording(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                            int32_t n_channels_total, const int32_t* cols, const float* res,
                            int32_t C, const int64_t* pos, int64_t n_epochs, double* features,
                            int mem);

/* getData() and extractFeatures in one pass (OffLineDataProvider.java:216-233 materialises the
 * epochs, LogisticRegressionClassifier.java:87-90 then maps WaveletTransform.extractFeatures over
 * them): the baseline-corrected epochs double[n][C][750] (epochs_out) and their dwt-8 rows
 * double[n][16 C] (features) from one read of each epoch's frames, the filter bank running on
 * the frames the epoch write staged.  Each output equals its own call (eegfx_cut_epochs_f64 /
 * eegfx_process_recording), bit for bit under EEGFX_EXACT.  epochs_out == NULL: the same as
 * eegfx_process_recording.  Layouts whose epoch span does not fit one workgroup's LDS (more than
 * ~40 int16 / ~20 float32 channels in the file) run the two passes instead. */
int eegfx_process_recording_epochs(eegfx_ctx* ctx, const void* raw, int32_t fmt, int64_t n_frames,
                                   int32_t n_channels_total, const int32_t* cols,
                                   const float* res, int32_t C, const int64_t* pos,
                                   int64_t n_epochs, double* features, double* epochs_out,
                                   int mem);

/* configs[4] -- long recordings streamed from host memory: raw (host, n_frames x
 * n_channels_total samples), pos and features are HOST arrays; the recording is moved to the device
 * in chunks of at most chunk_frames frames (>= 787, the frames one epoch spans) on an upload
 * stream that runs up to three chunks ahead of the kernels (a ring of four device chunk buffers;
 * pageable sources go through two pinned staging buffers that the context keeps for later calls
 * and frees when it is destroyed, pinned sources are copied directly),
 * and the rows of each chunk return on a download stream.  Positions may come in any
 * order; features[i] belongs to pos[i].  Results equal eegfx_process_recording on the whole
 * recording (bit for bit under EEGFX_EXACT).  Replaces the whole-file readBinaryData decode of
 * OffLineDataProvider.java:186-188 for recordings that are not kept resident. */
int eegfx_process_recording_streamed(eegfx_ctx* ctx, const void* raw, int32_t fmt,
                                     int64_t n_frames, int32_t n_channels_total,
                                     const int32_t* cols, const float* res, int32_t C,
                                     const int64_t* pos, int64_t n_epochs, double* features,
                                     int64_t chunk_frames);

/* ---- the downstream classifier ----------------------------------------
 * LogisticRegressionClassifier.java:85-114 trains Spark MLlib 1.6.2 LogisticRegressionWithSGD on
 * the feature rows: the default constructor (step 1.0, 100 iterations, regParam 0.01, fraction
 * 1.0) or, with the config_* keys, the static train(...) with regParam 0.0.  This runs that
 * full-batch gradient descent on the device: LogisticGradient, SquaredL2Updater with
 * step/sqrt(i), GradientDescent's convergence test (||w_prev - w|| < tol * max(||w||, 1), MLlib's
 * tol = 0.001), no intercept.  X is n x d row-major (the feature matrix as produced), y the 0/1
 * labels; `weights` holds the initial weights (zeros in MLlib) on entry and the trained ones on
 * return (host array).  mini_batch_fraction < 1 samples each iteration's mini-batch as MLlib does
 * (eegfx_logreg_sgd_train_partitioned below); labels other than 0/1 give EEGFX_EINVAL ("Input
 * validation failed").  eegfx_logreg_predict: LogisticRegressionModel.predict -- score = 1/(1+exp(-(w.x+b))),
 * out = score > threshold ? 1 : 0, or the score itself when threshold is NaN (clearThreshold). */
int eegfx_logreg_sgd_train(eegfx_ctx* ctx, const double* X, const double* y, int64_t n, int32_t d,
                           int32_t num_iterations, double step_size, double reg_param,
                           double mini_batch_fraction, double convergence_tol, double* weights,
                           int32_t* iterations_run, int mem);
int eegfx_logreg_predict(eegfx_ctx* ctx, const double* X, int64_t n, int32_t d,
                         const double* weights, double intercept, double threshold, double* out,
                         int mem);
/* The same training with the Spark partition count stated.  mini_batch_fraction f in [0, 1)
 * (config_mini_batch_fraction, LogisticRegressionClassifier.java:98-108, README.md:136): iteration
 * i (1-based) trains on MLlib's data.sample(false, f, 42 + i) of the n rows split into
 * num_partitions ParallelCollectionRDD slices (partition p: rows [p n / N, (p + 1) n / N)), the
 * sample drawn on the host with Spark 1.6.2's own sampler (PartitionwiseSampledRDD seeds from
 * java.util.Random, BernoulliSampler / GapSamplingIterator on XORShiftRandom; eegfx_spark_sample)
 * and the gradient divided by the sample size; an empty sample skips the update.  f >= 1: the
 * full batch.  eegfx_logreg_sgd_train is this function with num_partitions = the host's hardware
 * threads (Spark local[*]'s defaultParallelism, SparkInitializer.java:44). */
int eegfx_logreg_sgd_train_partitioned(eegfx_ctx* ctx, const double* X, const double* y,
                                       int64_t n, int32_t d, int32_t num_iterations,
                                       double step_size, double reg_param,
                                       double mini_batch_fraction, double convergence_tol,
                                       int32_t num_partitions, double* weights,
                                       int32_t* iterations_run, int mem);
/* RDD.sample(false, fraction, seed) of n rows in num_partitions slices (pure host function):
 * mask = bit r of word r / 32 set for every kept row ((n + 31) / 32 words), *kept = their count. */
int eegfx_spark_sample(int64_t n, double fraction, int32_t num_partitions, int64_t seed,
                       uint32_t* mask, int64_t* kept);

/* eegfx_svm_* (MLlib SVMWithSGD on the same device loop) is declared in eegfx_ext.h: SURVEY.md
 * section 2 marks the SVM classifier out of the hot-path scope, so it is not part of this contract. */

/* ---- multi-GPU ------------------------------------------------------------
 * Epochs shard by contiguous ranges of the selected-epoch list (eegfx_shard_range: balanced, the
 * first n % world ranks take one more); each rank runs the fused path on its range with no
 * collective; eegfx_gather then assembles the [n_total][cols] feature matrix in rank order (the
 * reference's getData() order, OffLineDataProvider.java:370) on every rank, by one RCCL broadcast
 * per rank inside a group (ragged shards land directly in their rows).  `local` and `out` are
 * device pointers on the communicator's context device; the collective runs on that context's
 * stream.  One communicator per (process, device): rank 0 creates the unique id and ships it to
 * the other ranks out of band (e.g. a Spark broadcast variable); a single process that drives
 * several devices (Spark local[*]) uses eegfx_comm_init_all and brackets its per-device gathers
 * with eegfx_group_start / eegfx_group_end. */
#define EEGFX_COMM_ID_BYTES 128
typedef struct eegfx_comm eegfx_comm;
int eegfx_shard_range(int64_t n, int32_t rank, int32_t world, int64_t* start, int64_t* end);
/* The schedule eegfx_gather runs: for every root r < world, the first row offsets[r] and the row
 * count counts[r] of the broadcast rooted at r (= eegfx_shard_range of r; a root with no rows
 * issues no broadcast).  Pure host function. */
int eegfx_gather_schedule(int64_t n_total, int32_t world, int64_t* offsets, int64_t* counts);
int eegfx_comm_unique_id(void* id /* EEGFX_COMM_ID_BYTES */);
int eegfx_comm_create(eegfx_ctx* ctx, int32_t world, int32_t rank, const void* id,
                      eegfx_comm** out);
int eegfx_comm_init_all(eegfx_ctx* const* ctxs, int32_t n, eegfx_comm** out /* n */);
int eegfx_comm_rank(const eegfx_comm* comm, int32_t* rank, int32_t* world);
int eegfx_gather(eegfx_comm* comm, const double* local, int64_t n_total, int64_t cols,
                 double* out);
/* Rooted gather ("grouped ncclSend/ncclRecv to rank 0"): the [n_total][cols]
 * matrix is assembled on `root` only -- the reference's consumer is one JVM holding one list
 * (OffLineDataProvider.java:370-379 getData(), parallelize on the driver in
 * LogisticRegressionClassifier.java:87-94).  Every other rank sends its shard once, the root
 * receives each ragged shard straight into its rows of `out` (its own shard: a device copy, or
 * nothing when `local` already is those rows), all inside one RCCL group, on the context
 * stream.  `out` is read on the root only (may be NULL elsewhere).  Root inbound traffic is
 * (world-1)/world of the matrix over its world-1 xGMI links, where eegfx_gather moves the whole
 * matrix to every rank. */
int eegfx_gather_root(eegfx_comm* comm, const double* local, int64_t n_total, int64_t cols,
                      int32_t root, double* out);
/* The point-to-point plan eegfx_gather_root issues on `rank` (pure host function): up to `world`
 * operations {kind, peer, first row, rows}; the root receives from every other rank with rows
 * (in rank order) and copies its own shard, every other rank with rows sends once to the root. */
#define EEGFX_GATHER_SEND 0
#define EEGFX_GATHER_RECV 1
#define EEGFX_GATHER_COPY 2
typedef struct {
  int32_t kind;  /* EEGFX_GATHER_SEND | _RECV | _COPY                          */
  int32_t peer;  /* the other rank (the root for a send; the rank itself for a copy) */
  int64_t row;   /* first row of the shard in the [n_total][cols] matrix             */
  int64_t rows;  /* rows moved                                                        */
} eegfx_gather_op;
int eegfx_gather_root_plan(int64_t n_total, int32_t world, int32_t rank, int32_t root,
                           eegfx_gather_op* ops /* world entries */, int32_t* n_ops);
int eegfx_group_start(void);
int eegfx_group_end(void);
int eegfx_comm_destroy(eegfx_comm* comm);

/* Deterministic synthetic multiplexed int16 recording, generated on device:
 * DC -25000 counts + bounded random walk + 10 Hz sinusoid, clipped to int16.  dst is a device
 * pointer of n_frames * n_channels int16. */
int eegfx_synth_recording(eegfx_ctx* ctx, int16_t* dst, int64_t n_frames, int32_t n_channels,
                          uint64_t seed);

/* ---- OffLineDataProvider (OffLineDataProvider.java:42-380) ----------------------------------
 * Same argument conventions as the Java constructor: args = { "<info.txt>" } or
 * { "<file.eeg>", "<guessed>", optional... } (1..6 entries).  Paths are local files (the HDFS
 * client of the reference is out of scope).  load_data never fails: like the reference
 * (:88-98) it stops at the first fatal error and keeps what was loaded; the message is
 * available from eegfx_odp_error(). */
/* ctx may be NULL: a planning-only provider parses, selects and labels (positions, labels,
 * file indices) without reading the sample payload or touching a GPU. */
int eegfx_odp_create(eegfx_ctx* ctx, const char* const* args, int32_t n_args, eegfx_odp** out);
int eegfx_odp_load_data(eegfx_odp* odp);
const char* eegfx_odp_error(const eegfx_odp* odp);       /* "" when loading succeeded */
int64_t eegfx_odp_num_epochs(const eegfx_odp* odp);
/* getData(): double[n][3][750] host copy */
int eegfx_odp_get_data(const eegfx_odp* odp, double* out);
/* getDataLabels(): double[n] */
int eegfx_odp_get_labels(const eegfx_odp* odp, double* out);
/* Selected marker positions (int64[n]) and source file index (int32[n]) of every epoch. */
int eegfx_odp_get_positions(const eegfx_odp* odp, int64_t* pos_out, int32_t* file_out);
/* fe=dwt-8 features of every loaded epoch, computed on the device from the resident epochs. */
int eegfx_odp_get_features(eegfx_odp* odp, int32_t name, int32_t epoch_size, int32_t skip,
                           int32_t feature_size, double* out);
void eegfx_odp_destroy(eegfx_odp* odp);

#ifdef __cplusplus
}
#endif
#endif /* EEGFX_H_ */
