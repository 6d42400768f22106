// dropin_bench -- configs[0]'s per-epoch drop-in through the C ABI, timed natively (what a JNI
// caller of IFeatureExtraction.extractFeatures sees, without Python in the loop).
//
//   dropin_bench <repo> [reps] [numerics: 0 exact | 1 fma]
//
// Loads DoD2015_01 through the ABI (eegfx_read_header / _read_raw / _read_markers /
// _plan_markers / _cut_epochs_f64: the 11 infoTrain epochs), then:
//   single   one thread, one context: eegfx_extract_features_f64 on one host epoch per call
//            (FeatureExtractionTest.java:62-67 and the Spark map closure make exactly this call);
//   threads  T threads, one context each (include/eegfx.h's rule for Spark executor threads),
//            all calling concurrently;
//   cpu      the oracle's C restatement (oracle/liboracle.so, full pyramid) on the same epoch,
//            one thread -- the per-thread rate of the CPU baseline; beside it the optimised CPU
//            form (oracle_extract_features_fast: minimal cascade, channels in AVX2 lanes);
//   sync     the floor of one launch round trip on this box: an empty kernel + hipStreamSynchronize,
//            and the same with a spin on hipEventQuery;
//   mailbox  the same calls served by the context's resident workgroup (eegfx_ctx_set_mailbox):
//            one epoch per call, the 11-epoch batch, and T threads with a server each; every row
//            compared bit for bit with the launch path's.
// Prints one JSON object.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "eegfx.h"

static double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                                    \
  do {                                                                           \
    int _rc = (x);                                                               \
    if (_rc != 0) {                                                              \
      fprintf(stderr, "%s failed: %d %s\n", #x, _rc, eegfx_last_error());        \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

static std::vector<double> g_epochs;  // [11][3][750]
static int g_numerics = 1;

struct Lat {
  double med, p99;
};
static Lat stats(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return {v[v.size() / 2], v[(size_t)(v.size() * 0.99)]};
}

struct Job {
  int reps;
  double per_call;
  int rc;
  int mailbox;
  std::vector<double> lat;  // seconds per call
  std::vector<double> at;   // start of each call (steady clock, s)
  long tid;                 // the worker's kernel thread id (to match a runtime API trace)
  int resident;             // held a started server at the end of its calls
  pthread_barrier_t* bar;   // every thread starts together and holds its context to the end
};
static void* worker(void* arg) {
  Job* j = (Job*)arg;
  eegfx_ctx* ctx = nullptr;
  j->rc = eegfx_ctx_create(0, &ctx);
  if (j->rc) return nullptr;
  eegfx_ctx_set_numerics(ctx, g_numerics);
  if (j->mailbox) j->rc |= eegfx_ctx_set_mailbox(ctx, 1);
  double out[48];
  for (int i = 0; i < 20; ++i)
    eegfx_extract_features_f64(ctx, g_epochs.data(), 1, 3, 8, 512, 175, 16, out, EEGFX_MEM_HOST);
  j->lat.resize((size_t)j->reps);
  j->at.resize((size_t)j->reps);
  j->tid = (long)syscall(SYS_gettid);
  if (j->bar) pthread_barrier_wait(j->bar);
  const double t0 = now_s();
  for (int i = 0; i < j->reps; ++i) {
    const double c0 = now_s();
    j->rc |= eegfx_extract_features_f64(ctx, g_epochs.data() + (size_t)(i % 11) * 2250, 1, 3, 8,
                                        512, 175, 16, out, EEGFX_MEM_HOST);
    j->lat[(size_t)i] = now_s() - c0;
    j->at[(size_t)i] = c0;
  }
  j->per_call = (now_s() - t0) / j->reps;
  int32_t en = 0, res = 0;
  eegfx_ctx_get_mailbox(ctx, &en, &res);
  j->resident = res;
  if (j->bar) pthread_barrier_wait(j->bar);  // resident_servers counts servers held at once
  eegfx_ctx_destroy(ctx);
  return nullptr;
}
// T threads with a context each, started together (barrier) and holding their contexts to the
// end; per-call latency over all calls.  mailbox: every context asks for a server (at most 4 hold
// one, the rest serve on the launch path).  The slowest calls go to stderr.
static void thread_leg(int T, int reps, int mailbox, const char* sep) {
  std::vector<pthread_t> th((size_t)T);
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, nullptr, (unsigned)T);
  std::vector<Job> jobs((size_t)T, Job{reps, 0.0, 0, mailbox, {}, {}, 0, 0, &bar});
  for (int t = 0; t < T; ++t) pthread_create(&th[(size_t)t], nullptr, worker, &jobs[(size_t)t]);
  double agg = 0, mean = 0;
  int rc = 0, resident = 0;
  std::vector<double> all;
  for (int t = 0; t < T; ++t) {
    pthread_join(th[(size_t)t], nullptr);
    agg += 1.0 / jobs[(size_t)t].per_call;
    mean += jobs[(size_t)t].per_call / T;
    rc |= jobs[(size_t)t].rc;
    resident += jobs[(size_t)t].resident;
    all.insert(all.end(), jobs[(size_t)t].lat.begin(), jobs[(size_t)t].lat.end());
  }
  pthread_barrier_destroy(&bar);
  // the slowest calls (stderr): thread, call index, whether that thread held a server
  for (int rank = 0; rank < 3; ++rank) {
    int bt = -1, bi = -1;
    double bv = -1;
    for (int t = 0; t < T; ++t)
      for (size_t i = 0; i < jobs[(size_t)t].lat.size(); ++i)
        if (jobs[(size_t)t].lat[i] > bv) { bv = jobs[(size_t)t].lat[i]; bt = t; bi = (int)i; }
    if (bt < 0) break;
    fprintf(stderr, "%s threads %d slowest #%d: %.1f us (thread %d call %d resident %d tid %ld at_ns %.0f)\n",
            mailbox ? "mailbox" : "launch", T, rank, bv * 1e6, bt, bi, jobs[(size_t)bt].resident,
            jobs[(size_t)bt].tid, jobs[(size_t)bt].at[(size_t)bi] * 1e9);
    jobs[(size_t)bt].lat[(size_t)bi] = -jobs[(size_t)bt].lat[(size_t)bi];
  }
  for (int t = 0; t < T; ++t)
    for (double& v : jobs[(size_t)t].lat) v = v < 0 ? -v : v;
  std::sort(all.begin(), all.end());
  printf("%s\"%d\": {\"per_thread_epochs_per_s\": %.1f, \"aggregate_epochs_per_s\": %.1f, ", sep, T,
         1.0 / mean, agg);
  if (mailbox) printf("\"resident_servers\": %d, ", resident);
  printf("\"median_us\": %.2f, \"p99_us\": %.2f, \"max_us\": %.2f, \"rc\": %d}",
         all[all.size() / 2] * 1e6, all[(size_t)(all.size() * 0.99)] * 1e6, all.back() * 1e6, rc);
}

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1024) *p = 0;
}

int main(int argc, char** argv) {
  const std::string repo = argc > 1 ? argv[1] : ".";
  const int reps = argc > 2 ? atoi(argv[2]) : 2000;
  g_numerics = argc > 3 ? atoi(argv[3]) : 1;
  const std::string base = repo + "/tests/golden/test-data/DoD/DoD2015_01";
  eegfx_header_info hi;
  CK(eegfx_read_header((base + ".vhdr").c_str(), &hi, nullptr, 0));
  int64_t nf = 0;
  CK(eegfx_recording_frames((base + ".vhdr").c_str(), (base + ".eeg").c_str(), &nf));
  std::vector<int16_t> raw((size_t)nf * hi.n_channels);
  CK(eegfx_read_raw(nullptr, (base + ".vhdr").c_str(), (base + ".eeg").c_str(), raw.data(),
                    (int64_t)raw.size() * 2, EEGFX_MEM_HOST));
  int64_t nm = 0;
  CK(eegfx_read_markers((base + ".vmrk").c_str(), nullptr, 0, &nm));
  std::vector<eegfx_marker> mk((size_t)nm);
  CK(eegfx_read_markers((base + ".vmrk").c_str(), mk.data(), nm, &nm));
  std::vector<int64_t> pos((size_t)nm);
  std::vector<double> lab((size_t)nm);
  int64_t bal = 0, k = 0;
  CK(eegfx_plan_markers(mk.data(), nm, nf, 1, &bal, pos.data(), lab.data(), &k));
  eegfx_ctx* ctx = nullptr;
  CK(eegfx_ctx_create(0, &ctx));
  CK(eegfx_ctx_set_numerics(ctx, g_numerics));
  const int32_t cols[3] = {0, 1, 2};
  const float res[3] = {0.1f, 0.1f, 0.1f};
  g_epochs.resize((size_t)k * 3 * 750);
  CK(eegfx_cut_epochs_f64(ctx, raw.data(), EEGFX_INT_16, nf, hi.n_channels, cols, res, 3,
                          pos.data(), k, g_epochs.data(), EEGFX_MEM_HOST));

  // single thread, one epoch per call
  double out[48];
  for (int i = 0; i < 50; ++i)
    CK(eegfx_extract_features_f64(ctx, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                  EEGFX_MEM_HOST));
  std::vector<double> lat;
  for (int i = 0; i < reps; ++i) {
    const double t0 = now_s();
    CK(eegfx_extract_features_f64(ctx, g_epochs.data() + (size_t)(i % k) * 2250, 1, 3, 8, 512,
                                  175, 16, out, EEGFX_MEM_HOST));
    lat.push_back(now_s() - t0);
  }
  const Lat single = stats(lat);
  // the 11 epochs as one batch
  std::vector<double> out11((size_t)k * 48);
  lat.clear();
  for (int i = 0; i < reps / 4; ++i) {
    const double t0 = now_s();
    CK(eegfx_extract_features_f64(ctx, g_epochs.data(), k, 3, 8, 512, 175, 16, out11.data(),
                                  EEGFX_MEM_HOST));
    lat.push_back(now_s() - t0);
  }
  const Lat batch = stats(lat);

  // launch round-trip floors
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipEvent_t ev;
  (void)hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  std::vector<double> ls, le;
  for (int i = 0; i < reps; ++i) {
    double t0 = now_s();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
    (void)hipStreamSynchronize(st);
    ls.push_back(now_s() - t0);
    t0 = now_s();
    hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, st, nullptr);
    (void)hipEventRecord(ev, st);
    while (hipEventQuery(ev) == hipErrorNotReady) {
    }
    le.push_back(now_s() - t0);
  }
  const Lat sync_floor = stats(ls), spin_floor = stats(le);

  // T threads, own contexts
  printf("{\"single_epoch\": {\"median_us\": %.2f, \"p99_us\": %.2f, \"epochs_per_s\": %.1f},\n",
         single.med * 1e6, single.p99 * 1e6, 1.0 / single.med);
  printf(" \"batch_11\": {\"median_us\": %.2f, \"epochs_per_s\": %.1f},\n", batch.med * 1e6,
         k / batch.med);
  printf(" \"launch_floor\": {\"empty_kernel_stream_sync_us\": %.2f, \"empty_kernel_event_spin_us\": %.2f},\n",
         sync_floor.med * 1e6, spin_floor.med * 1e6);
  printf(" \"threads\": {");
  // the launch path alone (no server anywhere), up to Spark local[*] on the box's 16 cores and
  // twice that
  const int Ts[5] = {2, 4, 8, 16, 32};
  for (int ti = 0; ti < 5; ++ti) thread_leg(Ts[ti], reps / 2, 0, ti ? ", " : "");
  printf("},\n");

  // the resident server: the same calls without a launch each, rows compared with the launch path
  {
    std::vector<double> want((size_t)k * 48), got((size_t)k * 48);
    for (int64_t i = 0; i < k; ++i)
      CK(eegfx_extract_features_f64(ctx, g_epochs.data() + (size_t)i * 2250, 1, 3, 8, 512, 175, 16,
                                    want.data() + i * 48, EEGFX_MEM_HOST));
    CK(eegfx_ctx_set_mailbox(ctx, 1));
    for (int i = 0; i < 200; ++i)
      CK(eegfx_extract_features_f64(ctx, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                    EEGFX_MEM_HOST));
    lat.clear();
    for (int i = 0; i < reps; ++i) {
      const double t0 = now_s();
      CK(eegfx_extract_features_f64(ctx, g_epochs.data() + (size_t)(i % k) * 2250, 1, 3, 8, 512,
                                    175, 16, got.data() + (i % k) * 48, EEGFX_MEM_HOST));
      lat.push_back(now_s() - t0);
    }
    const Lat mb = stats(lat);
    bool same = std::equal(want.begin(), want.end(), got.begin(), [](double a, double b) {
      return a == b || (a != a && b != b);
    });
    std::vector<double> got11((size_t)k * 48);
    lat.clear();
    for (int i = 0; i < reps / 4; ++i) {
      const double t0 = now_s();
      CK(eegfx_extract_features_f64(ctx, g_epochs.data(), k, 3, 8, 512, 175, 16, got11.data(),
                                    EEGFX_MEM_HOST));
      lat.push_back(now_s() - t0);
    }
    const Lat mb11 = stats(lat);
    same = same && std::equal(want.begin(), want.end(), got11.begin(), [](double a, double b) {
      return a == b || (a != a && b != b);
    });
    CK(eegfx_ctx_set_mailbox(ctx, 0));
    // where the served context's launched batches lose time: the same launched calls on this
    // context (server stopped) while ANOTHER context keeps a server resident
    eegfx_ctx* ctx2 = nullptr;
    CK(eegfx_ctx_create(0, &ctx2));
    CK(eegfx_ctx_set_mailbox(ctx2, 1));
    for (int i = 0; i < 50; ++i)
      CK(eegfx_extract_features_f64(ctx2, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                    EEGFX_MEM_HOST));
    int32_t en2 = 0, res2 = 0;
    CK(eegfx_ctx_get_mailbox(ctx2, &en2, &res2));
    lat.clear();
    for (int i = 0; i < reps / 4; ++i) {
      const double t0 = now_s();
      CK(eegfx_extract_features_f64(ctx, g_epochs.data(), k, 3, 8, 512, 175, 16, got11.data(),
                                    EEGFX_MEM_HOST));
      lat.push_back(now_s() - t0);
      if (i % 64 == 0)  // keep the other server inside its idle window
        CK(eegfx_extract_features_f64(ctx2, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                      EEGFX_MEM_HOST));
    }
    const Lat other11 = stats(lat);
    lat.clear();
    for (int i = 0; i < reps / 4; ++i) {
      const double t0 = now_s();
      CK(eegfx_extract_features_f64(ctx, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                    EEGFX_MEM_HOST));
      lat.push_back(now_s() - t0);
      if (i % 64 == 0)
        CK(eegfx_extract_features_f64(ctx2, g_epochs.data(), 1, 3, 8, 512, 175, 16, out,
                                      EEGFX_MEM_HOST));
    }
    const Lat other1 = stats(lat);
    CK(eegfx_ctx_destroy(ctx2));
    lat.clear();
    for (int i = 0; i < reps / 4; ++i) {  // and with no server anywhere, again
      const double t0 = now_s();
      CK(eegfx_extract_features_f64(ctx, g_epochs.data(), k, 3, 8, 512, 175, 16, got11.data(),
                                    EEGFX_MEM_HOST));
      lat.push_back(now_s() - t0);
    }
    const Lat none11 = stats(lat);
    printf(" \"launched_beside_a_server\": {\"other_context_resident\": %d, \"batch_11_median_us\": %.2f, "
           "\"single_median_us\": %.2f, \"batch_11_no_server_median_us\": %.2f},\n",
           res2, other11.med * 1e6, other1.med * 1e6, none11.med * 1e6);
    printf(" \"mailbox\": {\"single_epoch\": {\"median_us\": %.2f, \"p99_us\": %.2f, "
           "\"epochs_per_s\": %.1f}, \"batch_11\": {\"median_us\": %.2f, \"epochs_per_s\": %.1f}, "
           "\"rows_identical_to_launch_path\": %s, \"threads\": {",
           mb.med * 1e6, mb.p99 * 1e6, 1.0 / mb.med, mb11.med * 1e6, k / mb11.med,
           same ? "true" : "false");
    // every context asking for a server
    const int Tm[5] = {2, 4, 8, 16, 32};
    for (int ti = 0; ti < 5; ++ti) thread_leg(Tm[ti], reps / 2, 1, ti ? ", " : "");
    printf("}},\n");
  }

  // the C port, one thread
  void* h = dlopen((repo + "/oracle/liboracle.so").c_str(), RTLD_NOW);
  double cpu_med = 0;
  if (h) {
    typedef void (*fe_t)(const double*, int64_t, int32_t, int32_t, int32_t, int32_t, int32_t,
                         double*);
    fe_t fe = (fe_t)dlsym(h, "oracle_extract_features");
    if (fe) {
      for (int i = 0; i < 50; ++i) fe(g_epochs.data(), 1, 3, 175, 512, 16, 1, out);
      lat.clear();
      for (int i = 0; i < reps; ++i) {
        const double t0 = now_s();
        fe(g_epochs.data() + (size_t)(i % k) * 2250, 1, 3, 175, 512, 16, 1, out);
        lat.push_back(now_s() - t0);
      }
      cpu_med = stats(lat).med;
    }
  }
  double opt_med = 0;
  if (h) {
    typedef int (*fef_t)(const double*, int64_t, int32_t, int32_t, int32_t, int32_t, double*);
    fef_t fef = (fef_t)dlsym(h, "oracle_extract_features_fast");
    if (fef) {
      for (int i = 0; i < 50; ++i) fef(g_epochs.data(), 1, 3, 175, 512, 16, out);
      lat.clear();
      for (int i = 0; i < reps; ++i) {
        const double t0 = now_s();
        fef(g_epochs.data() + (size_t)(i % k) * 2250, 1, 3, 175, 512, 16, out);
        lat.push_back(now_s() - t0);
      }
      opt_med = stats(lat).med;
    }
  }
  printf(" \"cpu_port_single_thread\": {\"median_us\": %.2f, \"epochs_per_s\": %.1f},\n",
         cpu_med * 1e6, cpu_med > 0 ? 1.0 / cpu_med : 0.0);
  printf(" \"cpu_optimised_single_thread\": {\"median_us\": %.2f, \"epochs_per_s\": %.1f}}\n",
         opt_med * 1e6, opt_med > 0 ? 1.0 / opt_med : 0.0);
  eegfx_ctx_destroy(ctx);
  return 0;
}
