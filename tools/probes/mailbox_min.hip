// mailbox_min -- the resident-server protocol of features_mailbox_kernel alone (no feature math):
// a one-workgroup kernel polls a host-mapped request word and answers each request, the host
// posts requests and spins on the answer.  Reports each step's time and the kernel's view of the
// clock; a watchdog ends the process at a stalled step.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <thread>
#include <unistd.h>

struct Cmd {
  uint32_t req, done, stop, exits;
  uint64_t t_start, t_end, polls;
};

__global__ void mbox(Cmd* mb, uint64_t idle_ticks, int variant) {
  __shared__ uint32_t cmd[1];
  const int tid = threadIdx.x;
  uint32_t last = __hip_atomic_load(&mb->done, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t_start = wall_clock64();
  uint64_t polls = 0;
  for (;;) {
    if (tid == 0) {
      uint32_t go = 0;
      const uint64_t t0 = wall_clock64();
      for (;;) {
        ++polls;
        const uint32_t r = __hip_atomic_load(&mb->req, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        if (r != last) { go = r; break; }
        if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        if (wall_clock64() - t0 > idle_ticks) break;
        if (variant == 0) __builtin_amdgcn_s_sleep(2);
      }
      cmd[0] = go;
    }
    __syncthreads();
    const uint32_t go = cmd[0];
    if (go == 0) break;
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&mb->done, go, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    last = go;
  }
  if (tid == 0) {
    mb->t_start = t_start;
    mb->t_end = wall_clock64();
    mb->polls = polls;
    __hip_atomic_fetch_add(&mb->exits, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static std::atomic<long> g_t0{0};
static std::atomic<int> g_step{0};
static long now_us() {
  return std::chrono::duration_cast<std::chrono::microseconds>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

int main(int argc, char** argv) {
  const int variant = argc > 1 ? atoi(argv[1]) : 0;
  const unsigned flags = argc > 2 ? (unsigned)atoi(argv[2]) : 0;  // 1: no Coherent flag
  std::thread([] {
    for (;;) {
      std::this_thread::sleep_for(std::chrono::milliseconds(200));
      if (g_step > 0 && now_us() - g_t0 > 8000000) {
        printf("WATCHDOG: step %d stalled\n", g_step.load());
        fflush(stdout);
        _exit(3);
      }
    }
  }).detach();
  Cmd* h = nullptr;
  Cmd* d = nullptr;
  unsigned hf = hipHostMallocMapped | (flags & 1 ? 0 : hipHostMallocCoherent);
  if (hipHostMalloc((void**)&h, sizeof(Cmd), hf) != hipSuccess) return 1;
  memset(h, 0, sizeof(Cmd));
  (void)hipHostGetDevicePointer((void**)&d, h, 0);
  hipStream_t st;
  (void)hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  g_step = 1;
  g_t0 = now_us();
  hipLaunchKernelGGL(mbox, dim3(1), dim3(256), 0, st, d, (uint64_t)200000000, variant);
  printf("launch: %s\n", hipGetErrorString(hipGetLastError()));
  fflush(stdout);
  for (uint32_t k = 1; k <= 2000; ++k) {
    g_step = 1 + (int)k;
    g_t0 = now_us();
    const long t = now_us();
    __atomic_store_n(&h->req, k, __ATOMIC_RELEASE);
    uint64_t spins = 0;
    while (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != k) {
      ++spins;
      __builtin_ia32_pause();
      if ((spins & 0xFFFFF) == 0) {
        printf("  req %u: %lu spins, done=%u exits=%u query=%s\n", k, (unsigned long)spins,
               __atomic_load_n(&h->done, __ATOMIC_ACQUIRE), __atomic_load_n(&h->exits, __ATOMIC_ACQUIRE),
               hipGetErrorString(hipStreamQuery(st)));
        fflush(stdout);
      }
    }
    if (k <= 3 || k % 500 == 0) {
      printf("req %u served in %ld us\n", k, now_us() - t);
      fflush(stdout);
    }
  }
  g_step = 9000;
  g_t0 = now_us();
  __atomic_store_n(&h->stop, 1u, __ATOMIC_RELEASE);
  (void)hipStreamSynchronize(st);
  printf("stopped: exits=%u ticks=%lu polls=%lu\n", h->exits, (unsigned long)(h->t_end - h->t_start),
         (unsigned long)h->polls);
  // the idle exit: relaunch, wait 2.5 s without a request
  h->stop = 0;
  g_step = 9001;
  g_t0 = now_us();
  const long t = now_us();
  hipLaunchKernelGGL(mbox, dim3(1), dim3(256), 0, st, d, (uint64_t)200000000, variant);
  (void)hipStreamSynchronize(st);
  printf("idle exit after %ld us: exits=%u ticks=%lu polls=%lu\n", now_us() - t, h->exits,
         (unsigned long)(h->t_end - h->t_start), (unsigned long)h->polls);
  printf("mailbox_min ok\n");
  return 0;
}
