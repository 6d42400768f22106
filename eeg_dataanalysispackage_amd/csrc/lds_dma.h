// lds_dma.h -- LDS-DMA (global_load_lds_dwordx4) in its scalar-base form for gfx950.
//
// One instruction moves 16 bytes per active lane from global memory straight into LDS (no VGPR
// staging): lane l's quad at sbase + voff lands at LDS byte address M0 + 16*l.  The base is one
// SGPR pair (wave-uniform: an epoch's window start) and the offset a per-lane VGPR, so the
// address math of a DMA costs no vector ALU work.  M0 is compiler-reserved, hence the save and
// restore inside the same asm statement; the "memory" clobber keeps the compiler from moving LDS
// or global accesses across it.  Completion is tracked by vmcnt: callers drain with
// `s_waitcnt vmcnt(0)` before the barrier that publishes the data.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace eegfx {
namespace dev {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Cache-policy modifier appended to every DMA (perf study: e.g. " nt" for streaming reads).
#ifndef EEGFX_DMA_POLICY
#define EEGFX_DMA_POLICY ""
#endif

// NT: non-temporal read (`nt`), for windows that no other epoch shares.  Measured on
// window_kernel (tools/probes, 3,000 launches): markers 1,000 frames apart 0.9180 -> 0.9101 ms,
// markers 100 frames apart (each frame in ~6 windows, reused through L2) 0.7774 -> 0.8024 ms.
template <bool NT = false>
__device__ __forceinline__ void dma16_s(const uint8_t* sbase, uint32_t voff, const void* lds_dst) {
  const uint32_t lds = (uint32_t)(uintptr_t)(lds_ptr_t)lds_dst;
  uint32_t saved;
  if constexpr (NT) {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %3 nt\n\t"
        "s_nop 0\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "s"(lds), "v"(voff), "s"(sbase)
        : "memory");
  } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %1\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %2, %3" EEGFX_DMA_POLICY "\n\t"
        "s_nop 0\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(saved)
        : "s"(lds), "v"(voff), "s"(sbase)
        : "memory");
  }
}

__device__ __forceinline__ void dma_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

}  // namespace dev
}  // namespace eegfx
