// push_probe -- can the host push a request's window rows into device memory (so that every
// crossing of the host link in a resident-server request is a posted write), and what does that
// save against the server reading them from pinned host memory?
//
//   push_probe           lists the GPU's memory pools and whether the CPU agent may access them
//   push_probe A|B|C [sys]  one-workgroup server, 2000 requests of 12 KB rows -> 48 doubles:
//     A  rows and request word in pinned host memory (the library's protocol)
//     B  rows in device memory written by the host; request word in pinned host memory
//     C  rows and request word in device memory written by the host
//   The rows are read with 16-byte loads after a system-scope acquire fence, or with
//   system-scope atomic loads ("sys").  Device memory is the fine-grained pool when the CPU may
//   access it, else a coarse-grained one opened to the CPU with hsa_amd_agents_allow_access.
//   Every word of the rows changes per request and all 48 answers are checked.
//   The answer (48 doubles + done word) always goes to pinned host memory.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

constexpr int kWords = 12 * 1024 / 8;  // 3 channels x 512 doubles
constexpr int kOut = 48;

struct Host {
  uint64_t req;
  uint32_t done, stop;
  double out[kOut];
};

__global__ __launch_bounds__(256) void server(Host* h, const uint64_t* req_at, const double* rows,
                                              int sys) {
  __shared__ double xs[kWords];
  __shared__ uint32_t cmd;
  const int tid = threadIdx.x;
  const bool wave0 = __builtin_amdgcn_readfirstlane(tid >> 6) == 0;
  uint32_t last = 0;
  for (;;) {
    if (wave0) {
      uint32_t go = 0;
      const uint64_t t0 = wall_clock64();
      for (;;) {
        const uint64_t r = __hip_atomic_load(req_at, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
        const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)r);
        if (s != last) { go = s; break; }
        if (__builtin_amdgcn_readfirstlane(
                (int)__hip_atomic_load(&h->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)))
          break;
        if (wall_clock64() - t0 > 300000000ull) break;
        __builtin_amdgcn_s_sleep(2);
      }
      if (tid == 0) cmd = go;
    }
    __syncthreads();
    const uint32_t go = (uint32_t)__builtin_amdgcn_readfirstlane((int)cmd);
    if (go == 0) break;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (sys) {
      for (int i = tid; i < kWords; i += 256)
        xs[i] = __hip_atomic_load(&rows[i], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      typedef double f64x2 __attribute__((ext_vector_type(2)));
      f64x2 v[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) v[k] = ((const f64x2*)rows)[tid + 256 * k];
#pragma unroll
      for (int k = 0; k < 3; ++k) ((f64x2*)xs)[tid + 256 * k] = v[k];
    }
    __syncthreads();
    if (tid < kOut) {
      double acc = 0.0;
      for (int k = 0; k < kWords / kOut; ++k) acc += xs[tid * (kWords / kOut) + k];
      h->out[tid] = acc + (double)go;
    }
    __threadfence_system();
    __syncthreads();
    if (tid == 0) __hip_atomic_store(&h->done, go, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    last = go;
  }
}

static hsa_agent_t g_cpu{}, g_gpu{};
static bool g_have_cpu = false, g_have_gpu = false;
static hsa_amd_memory_pool_t g_pool{}, g_coarse{};
static bool g_have_pool = false, g_have_coarse = false;

static hsa_status_t on_agent(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_CPU && !g_have_cpu) g_cpu = a, g_have_cpu = true;
  if (t == HSA_DEVICE_TYPE_GPU && !g_have_gpu) g_gpu = a, g_have_gpu = true;
  return HSA_STATUS_SUCCESS;
}

static hsa_status_t on_pool(hsa_amd_memory_pool_t p, void* list) {
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  hsa_amd_memory_pool_access_t acc;
  hsa_amd_agent_memory_pool_get_info(g_cpu, p, HSA_AMD_AGENT_MEMORY_POOL_INFO_ACCESS, &acc);
  size_t size = 0;
  hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SIZE, &size);
  const bool fine = flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED;
  printf("gpu pool: %s%s size %zu MiB, cpu access %s\n", fine ? "fine-grained" : "coarse-grained",
         flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT ? " kernarg" : "", size >> 20,
         acc == HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED          ? "never"
         : acc == HSA_AMD_MEMORY_POOL_ACCESS_ALLOWED_BY_DEFAULT   ? "by default"
                                                                   : "disallowed by default (allow_access)");
  if (fine && acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED && !g_have_pool)
    g_pool = p, g_have_pool = true;
  if (!fine && acc != HSA_AMD_MEMORY_POOL_ACCESS_NEVER_ALLOWED && !g_have_coarse)
    g_coarse = p, g_have_coarse = true;
  (void)list;
  return HSA_STATUS_SUCCESS;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

// 32-byte non-temporal stores (write-combined on a device mapping), then a store fence
static void push(void* dst, const void* src, size_t bytes) {
  __m256i* d = (__m256i*)dst;
  const __m256i* s = (const __m256i*)src;
  for (size_t i = 0; i < bytes / 32; ++i) _mm256_stream_si256(d + i, _mm256_loadu_si256(s + i));
  _mm_sfence();
}

int main(int argc, char** argv) {
  const char mode = argc > 1 ? argv[1][0] : '-';
  const int sys = argc > 2 && !strcmp(argv[2], "sys");
  hipSetDevice(0);
  if (hsa_init() != HSA_STATUS_SUCCESS) { printf("hsa_init failed\n"); return 1; }
  hsa_iterate_agents(on_agent, nullptr);
  if (!g_have_cpu || !g_have_gpu) { printf("no cpu/gpu agent\n"); return 1; }
  hsa_amd_agent_iterate_memory_pools(g_gpu, on_pool, nullptr);
  if (mode == '-') return 0;

  Host* h = nullptr;
  Host* hd = nullptr;
  hipHostMalloc((void**)&h, sizeof(Host), hipHostMallocMapped | hipHostMallocCoherent);
  memset(h, 0, sizeof(Host));
  hipHostGetDevicePointer((void**)&hd, h, 0);
  double* rows_host = nullptr;  // host view of the rows
  double* rows_dev = nullptr;   // device view
  uint64_t* req_host = &h->req;
  uint64_t* req_dev = &hd->req;
  void* dev_block = nullptr;
  if (mode == 'A') {
    hipHostMalloc((void**)&rows_host, kWords * 8, hipHostMallocMapped | hipHostMallocCoherent);
    hipHostGetDevicePointer((void**)&rows_dev, rows_host, 0);
  } else {
    if (!g_have_pool && !g_have_coarse) { printf("no cpu-accessible gpu pool\n"); return 2; }
    printf("device rows in the %s pool\n", g_have_pool ? "fine-grained" : "coarse-grained");
    if (hsa_amd_memory_pool_allocate(g_have_pool ? g_pool : g_coarse, 64 * 1024, 0, &dev_block) !=
        HSA_STATUS_SUCCESS) {
      printf("pool allocate failed\n");
      return 2;
    }
    const hsa_status_t st = hsa_amd_agents_allow_access(1, &g_cpu, nullptr, dev_block);
    printf("allow_access(cpu): %d\n", (int)st);
    if (st != HSA_STATUS_SUCCESS) return 2;
    hsa_amd_agents_allow_access(1, &g_gpu, nullptr, dev_block);
    rows_host = rows_dev = (double*)dev_block;
    if (mode == 'C') {
      req_host = req_dev = (uint64_t*)((char*)dev_block + 32 * 1024);
      *(volatile uint64_t*)req_host = 0;
    }
  }
  std::vector<double> src(kWords);
  for (int i = 0; i < kWords; ++i) src[i] = (double)(i % 97);
  double t0 = now_us();
  push(rows_host, src.data(), kWords * 8);
  printf("first host push of 12 KB: %.2f us\n", now_us() - t0);

  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  hipLaunchKernelGGL(server, dim3(1), dim3(256), 0, st, hd, req_dev, rows_dev, sys);
  std::vector<double> lat, pushes;
  bool ok = true;
  for (uint32_t k = 1; k <= 2000; ++k) {
    for (int i = 0; i < kWords; ++i) src[i] = (double)(i % 97) + (double)k;
    const double a = now_us();
    push(rows_host, src.data(), kWords * 8);
    const double b = now_us();
    __atomic_store_n(req_host, (uint64_t)k, __ATOMIC_RELEASE);
    if (mode == 'C') _mm_sfence();
    const double w0 = now_us();
    while (__atomic_load_n(&h->done, __ATOMIC_ACQUIRE) != k) {
      _mm_pause();
      if (now_us() - w0 > 2e6) {
        printf("request %u not served\n", k);
        h->stop = 1;
        hipStreamSynchronize(st);
        return 3;
      }
    }
    lat.push_back(now_us() - a);
    pushes.push_back(b - a);
    for (int t = 0; t < kOut; ++t) {  // out[t] = the sum of words [32t, 32t+32) + k
      double want = 0.0;
      for (int i = 0; i < kWords / kOut; ++i) want += src[t * (kWords / kOut) + i];
      if (h->out[t] != want + (double)k) ok = false;
    }
  }
  h->stop = 1;
  hipStreamSynchronize(st);
  std::sort(lat.begin(), lat.end());
  std::sort(pushes.begin(), pushes.end());
  printf("mode %c%s: request median %.2f us p99 %.2f us (host push median %.2f us) answers %s\n", mode,
         sys ? " sys" : "", lat[lat.size() / 2], lat[lat.size() * 99 / 100], pushes[pushes.size() / 2],
         ok ? "correct" : "WRONG");
  if (dev_block) hsa_amd_memory_pool_free(dev_block);
  return ok ? 0 : 4;
}
