/* Per-epoch drop-in calls from T threads, one context each with the resident server requested
 * (eegfx_ctx_set_mailbox) -- Spark local[*] with -Deegfx.mailbox=true on a box with T executor
 * threads.  At most 4 contexts of the process hold a started server on the device; the others
 * serve on the launch path.  Every row is compared bit for bit with the rows computed on the
 * launch path before any server existed, and every call is timed.
 *
 *   mailbox_threads <DoD2015_01.vhdr> <T> <calls per thread>
 *
 * Prints "threads T resident R calls N median_us M p99_us P max_us X" and exits 0 when every call
 * succeeded with identical rows and at most 4 contexts were resident at once. */
#define _POSIX_C_SOURCE 200809L
#include <pthread.h>
#include <stdatomic.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "eegfx.h"

#define CHECK(cond, ...)                     \
  do {                                       \
    if (!(cond)) {                           \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");                 \
      exit(1);                               \
    }                                        \
  } while (0)

enum { C = 3, POST = 750, F = 48, MAXE = 64 };

static double* g_epochs;
static double* g_want;
static int64_t g_n;
static int g_calls;
static atomic_int g_resident_max;
static atomic_int g_resident_now;
static pthread_barrier_t g_bar;

static double now_us(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec * 1e6 + t.tv_nsec * 1e-3;
}

typedef struct {
  int t;
  double* lat;
  int resident;
} job;

static void* worker(void* arg) {
  job* j = (job*)arg;
  eegfx_ctx* ctx = NULL;
  CHECK(eegfx_ctx_create(0, &ctx) == EEGFX_OK, "ctx_create: %s", eegfx_last_error());
  CHECK(eegfx_ctx_set_mailbox(ctx, 1) == EEGFX_OK, "set_mailbox: %s", eegfx_last_error());
  double row[F];
  pthread_barrier_wait(&g_bar);
  for (int i = 0; i < g_calls; ++i) {
    const int64_t e = (j->t + i) % g_n;
    const double t0 = now_us();
    CHECK(eegfx_extract_features_f64(ctx, g_epochs + e * C * POST, 1, C, 8, 512, 175, 16, row,
                                     EEGFX_MEM_HOST) == EEGFX_OK,
          "thread %d call %d: %s", j->t, i, eegfx_last_error());
    j->lat[i] = now_us() - t0;
    CHECK(memcmp(row, g_want + e * F, sizeof row) == 0, "thread %d epoch %lld: rows differ", j->t,
          (long long)e);
    int32_t en = 0, res = 0;
    CHECK(eegfx_ctx_get_mailbox(ctx, &en, &res) == EEGFX_OK && en == 1, "get_mailbox");
    if (res && !j->resident) {
      j->resident = 1;
      const int now = atomic_fetch_add(&g_resident_now, 1) + 1;
      int prev = atomic_load(&g_resident_max);
      while (now > prev && !atomic_compare_exchange_weak(&g_resident_max, &prev, now)) {}
    }
  }
  pthread_barrier_wait(&g_bar);  /* every thread still holds its context here */
  CHECK(eegfx_ctx_destroy(ctx) == EEGFX_OK, "ctx_destroy");
  return NULL;
}

static int cmp(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  CHECK(argc >= 4, "usage: mailbox_threads <vhdr> <threads> <calls>");
  const int T = atoi(argv[2]);
  g_calls = atoi(argv[3]);
  /* the recording and its epochs through the ABI (eegfx_odp_* on a one-file argument list) */
  eegfx_ctx* ctx = NULL;
  CHECK(eegfx_ctx_create(0, &ctx) == EEGFX_OK, "ctx_create: %s", eegfx_last_error());
  char eeg[1024];
  snprintf(eeg, sizeof eeg, "%s", argv[1]);
  char* dot = strrchr(eeg, '.');
  CHECK(dot != NULL, "vhdr path");
  strcpy(dot, ".eeg");
  const char* args[2] = {eeg, "2"};
  eegfx_odp* odp = NULL;
  CHECK(eegfx_odp_create(ctx, args, 2, &odp) == EEGFX_OK, "odp_create: %s", eegfx_last_error());
  CHECK(eegfx_odp_load_data(odp) == EEGFX_OK, "load_data: %s", eegfx_last_error());
  g_n = eegfx_odp_num_epochs(odp);
  CHECK(g_n > 0 && g_n <= MAXE, "%lld epochs", (long long)g_n);
  g_epochs = (double*)malloc(sizeof(double) * (size_t)g_n * C * POST);
  g_want = (double*)malloc(sizeof(double) * (size_t)g_n * F);
  CHECK(eegfx_odp_get_data(odp, g_epochs) == EEGFX_OK, "get_data");
  /* the launch path's rows (no server anywhere yet) */
  for (int64_t e = 0; e < g_n; ++e)
    CHECK(eegfx_extract_features_f64(ctx, g_epochs + e * C * POST, 1, C, 8, 512, 175, 16,
                                     g_want + e * F, EEGFX_MEM_HOST) == EEGFX_OK,
          "reference rows: %s", eegfx_last_error());
  eegfx_odp_destroy(odp);
  CHECK(eegfx_ctx_destroy(ctx) == EEGFX_OK, "ctx_destroy");

  pthread_t* th = (pthread_t*)calloc((size_t)T, sizeof(pthread_t));
  job* jobs = (job*)calloc((size_t)T, sizeof(job));
  pthread_barrier_init(&g_bar, NULL, (unsigned)T);
  for (int t = 0; t < T; ++t) {
    jobs[t].t = t;
    jobs[t].lat = (double*)calloc((size_t)g_calls, sizeof(double));
    CHECK(pthread_create(&th[t], NULL, worker, &jobs[t]) == 0, "pthread_create");
  }
  for (int t = 0; t < T; ++t) pthread_join(th[t], NULL);
  const size_t N = (size_t)T * (size_t)g_calls;
  double* all = (double*)malloc(sizeof(double) * N);
  for (int t = 0; t < T; ++t) memcpy(all + (size_t)t * g_calls, jobs[t].lat, sizeof(double) * g_calls);
  qsort(all, N, sizeof(double), cmp);
  const int rmax = atomic_load(&g_resident_max);
  printf("threads %d resident %d calls %zu median_us %.2f p99_us %.2f max_us %.2f\n", T, rmax, N,
         all[N / 2], all[(size_t)(N * 0.99)], all[N - 1]);
  CHECK(rmax >= 1 && rmax <= 4, "%d contexts resident at once (1..4 expected)", rmax);
  return 0;
}
