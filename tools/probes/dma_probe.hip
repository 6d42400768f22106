// Probe: semantics of __builtin_amdgcn_global_load_lds with 16-byte elements on gfx950.
// Each lane passes its own global source address; we check where each lane's 16 bytes land.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

__global__ void probe(const uint32_t* src, uint32_t* out, int dst_off_dw) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[2048];
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) lds[i] = 0xDEADBEEFu;
  __syncthreads();
  const int lane = threadIdx.x;
  // lane l reads global quad (63 - l): reversed, to see per-lane source addressing
  const uint32_t* g = src + 4 * (63 - lane);
  __builtin_amdgcn_global_load_lds((const void*)g, (__attribute__((address_space(3))) void*)(lds + dst_off_dw), 16, 0, 0);
  __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) & lgkm
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int i = threadIdx.x; i < 2048; i += blockDim.x) out[i] = lds[i];
}

int main() {
  std::vector<uint32_t> h(256);
  for (int i = 0; i < 256; ++i) h[i] = i;
  uint32_t *d, *o;
  hipMalloc(&d, 1024); hipMalloc(&o, 8192);
  hipMemcpy(d, h.data(), 1024, hipMemcpyHostToDevice);
  for (int off : {0, 4, 1, 2}) {
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d, o, off);
    std::vector<uint32_t> r(2048);
    hipMemcpy(r.data(), o, 8192, hipMemcpyDeviceToHost);
    printf("dst_off_dw=%d: ", off);
    for (int i = 0; i < 12; ++i) printf("%x ", r[i]);
    printf("... [%d..]=", off); for (int i = off; i < off + 8; ++i) printf("%u ", r[i]);
    int first = -1; for (int i = 0; i < 2048; ++i) if (r[i] == 252) { first = i; break; }
    int cnt = 0; for (int i = 0; i < 2048; ++i) if (r[i] != 0xDEADBEEFu) ++cnt;
    printf(" | lane0 quad (252..255) at dw %d, written dwords %d\n", first, cnt);
  }
  return 0;
}
