// dev_common.h -- device helpers shared by the MLP kernels (mlp.hip fp32, mlp_bf.hip bf16 split).
#pragma once
#include "pnr_internal.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

// The weight image is one contiguous stream per kernel; `sp` is this lane's cursor into it
// (stream base + wave*256 + lane*4 floats).  stage() copies the next `nfloats` (multiple of 1024)
// into LDS with global_load_lds_dwordx4 (lane-linear destination) and advances the cursor.
//
// The DMA is issued from inline asm ON PURPOSE: when hipcc sees a global_load_lds it cannot tell
// which LDS bytes it writes, so it waits vmcnt(0) before the next ds_read -- i.e. it waits for
// the PREFETCH of chunk c+1 before computing chunk c, exposing the whole load latency (measured:
// 26% of the kernel).  Hidden from hipcc, the DMA is ordered only by the explicit
// `s_waitcnt vmcnt(N); s_barrier` at the top of each chunk (sync_chunk), N = stores issued
// after the DMA that may stay in flight (activation saves).
__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(gsrc), "s"(lds_byte) : "memory");
}

__device__ __forceinline__ uint32_t lds_addr(const float* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) float*)p;
}

__device__ __forceinline__ void stage(const float*& sp, float* dst, int nfloats) {
  const int w = wave_id();
  const int n = nfloats >> 10;
  const uint32_t base = lds_addr(dst) + (uint32_t)(w * 256 * 4);
  for (int i = 0; i < n; ++i) glds16(sp + i * 1024, base + (uint32_t)(i * 4096));
  sp += nfloats;
}

// Wait for this wave's DMA of the current chunk (all but the N youngest VMEM ops), then meet the
// other waves: after it every wave's DMA into the chunk has landed and every wave has finished
// reading the buffer that the next stage() overwrites.
template <int N>
__device__ __forceinline__ void sync_chunk() {
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

}  // namespace pnr
