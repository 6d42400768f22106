/* A plain-C consumer of include/eegfx.h -- what the JNI shim of INTEGRATION.md is: no C++, no
 * torch, only the exported C ABI.  Reads the reference's DoD2015_01 recording (argv[1] = path
 * without extension), plans its markers like OffLineDataProvider (guessed = 1), checks the
 * selection against OfflineDataProviderTest's golden (11 epochs, 5 targets) and the error
 * plumbing; with argv[2] == "gpu" it also runs the fused path on device 0 and checks the
 * FeatureExtractionTest.java:106 golden sum exactly.  Exit status 0 = every check passed. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "eegfx.h"

#define CHECK(cond, ...)                      \
  do {                                        \
    if (!(cond)) {                            \
      fprintf(stderr, "FAIL: " __VA_ARGS__);  \
      fprintf(stderr, "\n");                  \
      return 1;                               \
    }                                         \
  } while (0)

static int lower_eq(const char* a, const char* b) {
  for (; *a && *b; ++a, ++b)
    if ((*a | 32) != (*b | 32)) return 0;
  return *a == *b;
}

int main(int argc, char** argv) {
  CHECK(argc >= 2, "usage: abi_consumer <recording base path> [gpu]");
  char vhdr[1024], vmrk[1024], eeg[1024];
  snprintf(vhdr, sizeof vhdr, "%s.vhdr", argv[1]);
  snprintf(vmrk, sizeof vmrk, "%s.vmrk", argv[1]);
  snprintf(eeg, sizeof eeg, "%s.eeg", argv[1]);
  CHECK(strncmp(eegfx_version(), "eegfx", 5) == 0, "version string %s", eegfx_version());

  eegfx_header_info info;
  eegfx_channel_info ch[64];
  CHECK(eegfx_read_header(vhdr, &info, ch, 64) == EEGFX_OK, "read_header: %s", eegfx_last_error());
  int32_t cols[3] = {-1, -1, -1};
  float res[3];
  const char* want[3] = {"fz", "cz", "pz"};  /* OffLineDataProvider.java:175-182 */
  for (int c = 0; c < 3; ++c)
    for (int i = 0; i < info.n_channels && i < 64; ++i)
      if (lower_eq(ch[i].name, want[c])) {
        cols[c] = ch[i].number - 1;
        res[c] = (float)ch[i].resolution;
      }
  CHECK(cols[0] >= 0 && cols[1] >= 0 && cols[2] >= 0, "Fz/Cz/Pz not found");

  int64_t n_markers = 0, n_frames = 0;
  CHECK(eegfx_read_markers(vmrk, NULL, 0, &n_markers) == EEGFX_OK, "%s", eegfx_last_error());
  eegfx_marker* mk = (eegfx_marker*)calloc((size_t)n_markers, sizeof(eegfx_marker));
  CHECK(eegfx_read_markers(vmrk, mk, n_markers, &n_markers) == EEGFX_OK, "%s", eegfx_last_error());
  CHECK(eegfx_recording_frames(vhdr, eeg, &n_frames) == EEGFX_OK, "%s", eegfx_last_error());
  int64_t* pos = (int64_t*)malloc(sizeof(int64_t) * (size_t)n_markers);
  double* lab = (double*)malloc(sizeof(double) * (size_t)n_markers);
  int64_t balance = 0, n = 0;
  CHECK(eegfx_plan_markers(mk, n_markers, n_frames, 1, &balance, pos, lab, &n) == EEGFX_OK,
        "plan_markers: %s", eegfx_last_error());
  double targets = 0;
  for (int64_t i = 0; i < n; ++i) targets += lab[i];
  CHECK(n == 11 && targets == 5.0, "selection %lld epochs, %g targets (golden: 11, 5)",
        (long long)n, targets);

  int64_t s = 0, e = 0;
  CHECK(eegfx_shard_range(10, 3, 4, &s, &e) == EEGFX_OK && s == 8 && e == 10, "shard_range");
  CHECK(eegfx_shard_range(10, 4, 4, &s, &e) == EEGFX_EINVAL, "shard_range error status");
  CHECK(strlen(eegfx_last_error()) > 0, "last_error text after a failure");
  CHECK(eegfx_process_recording(NULL, NULL, 0, 0, 3, cols, res, 3, NULL, 0, NULL,
                                EEGFX_MEM_HOST) == EEGFX_EINVAL, "null context status");

  if (argc >= 3 && strcmp(argv[2], "gpu") == 0) {
    eegfx_ctx* ctx = NULL;
    CHECK(eegfx_ctx_create(0, &ctx) == EEGFX_OK, "ctx_create: %s", eegfx_last_error());
    const size_t bytes = (size_t)n_frames * (size_t)info.n_channels * 2;
    int16_t* raw = (int16_t*)malloc(bytes);
    CHECK(eegfx_read_raw(ctx, vhdr, eeg, raw, (int64_t)bytes, EEGFX_MEM_HOST) == EEGFX_OK,
          "read_raw: %s", eegfx_last_error());
    double* feat = (double*)malloc(sizeof(double) * (size_t)n * 48);
    CHECK(eegfx_process_recording(ctx, raw, EEGFX_INT_16, n_frames, info.n_channels, cols, res, 3,
                                  pos, n, feat, EEGFX_MEM_HOST) == EEGFX_OK,
          "process_recording: %s", eegfx_last_error());
    double total = 0.0; /* FeatureExtractionTest.java:96-105: per-vector sums, then the total */
    for (int64_t i = 0; i < n; ++i) {
      double v = 0.0;
      for (int j = 0; j < 48; ++j) v += feat[i * 48 + j];
      total += v;
    }
    CHECK(total == -24.861844096031625, "feature sum %.17g (golden -24.861844096031625)", total);
    CHECK(eegfx_ctx_destroy(ctx) == EEGFX_OK, "ctx_destroy");
    free(raw);
    free(feat);
    printf("gpu: 11 x 48 features, golden sum matches\n");
  }
  free(mk);
  free(pos);
  free(lab);
  printf("abi_consumer ok\n");
  return 0;
}
