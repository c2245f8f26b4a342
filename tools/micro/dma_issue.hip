// Microbenchmark: what the weight stream of the decoder kernels costs per step.  One step = the
// decoder's 8 MFMA groups of 6 v_mfma_f32_32x32x16_f16 (48 MFMAs, A fragments read from the LDS ring
// by ds_read_b128) + one barrier, with 32 KB of weights per step staged into a 4-slot LDS ring
// (8 KB per wave, 8 pieces of 1 KB) from an L2-resident image, in several forms:
//   0 none               (no staging: the MFMA + LDS-read + barrier floor)
//   1 glds burst         8 global_load_lds_dwordx4 back to back after the barrier (k_mlp_fwd16 today)
//   2 glds spread        one piece per MFMA group
//   3 glds multi         the 8 pieces in ONE asm statement (M0 saved / restored once)
//   4 regs + ds_write    8 global_load_dwordx4 into VGPRs, written by ds_write_b128 one step later
//   5 glds spread multi  pieces 2 per statement in 4 groups
// One workgroup of 4 waves per CU, every CU busy; cycles per step (s_memtime) of workgroup 7.
//   hipcc --offload-arch=gfx950 -O3 tools/micro/dma_issue.hip -o /tmp/dma_issue && /tmp/dma_issue
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kSlot = 32768, kNbuf = 4, kSteps = 64;

__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void glds(const void* sbase, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_byte) : "memory");
}
// two pieces 4 KB apart in the source and in LDS
__device__ __forceinline__ void glds2(const char* sbase, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %4\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2\n\t"
               "s_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %3\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(sbase + 4096), "s"(lds_byte) : "memory");
}
__device__ __forceinline__ void glds8(const char* b, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %10\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %2\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %3\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %4\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %5\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %6\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %7\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %8\n\ts_add_u32 m0, m0, 4096\n\ts_nop 0\n\t"
               "global_load_lds_dwordx4 %1, %9\n\t"
               "s_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(b), "s"(b + 4096), "s"(b + 8192), "s"(b + 12288), "s"(b + 16384), "s"(b + 20480),
                 "s"(b + 24576), "s"(b + 28672), "s"(lds_byte)
               : "memory");
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void k(const char* __restrict__ img, float* out, unsigned long long* t) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const f16x8* in = reinterpret_cast<const f16x8*>(img);
  f16x8 b0 = in[lane], b1 = in[lane + 64];
  f32x16 acc[8];
  for (int i = 0; i < 8; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  for (int i = threadIdx.x; i < kNbuf * kSlot / 16; i += 256) reinterpret_cast<f16x8*>(lds)[i] = in[i % 4096];
  __syncthreads();
  f32x4 st[8];
  const uint32_t voff = lane * 16;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int g = 0; g < kSteps; ++g) {
    const char* slot = lds + (g % kNbuf) * kSlot;
    const int dslot = (g + 2) % kNbuf;
    const uint32_t dl = lds_addr(lds + dslot * kSlot) + w * 1024;
    const char* src = img + (size_t)((g * 37) % 24) * kSlot + w * 1024;  // 768 KB image, L2-resident
    asm volatile("s_waitcnt vmcnt(8)\n\ts_barrier" ::: "memory");
    if (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 8; ++i) glds(src + i * 4096, voff, dl + i * 4096);
    }
    if (MODE == 3) glds8(src, voff, dl);
    if (MODE == 4) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {  // last step's loads into this step's slot
        asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
        *reinterpret_cast<f32x4*>(lds + dslot * kSlot + w * 1024 + i * 4096 + lane * 16) = st[i];
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) st[i] = *reinterpret_cast<const f32x4*>(src + i * 4096 + lane * 16);
    }
#pragma unroll
    for (int T = 0; T < 8; ++T) {
      if (MODE == 2) glds(src + T * 4096, voff, dl + T * 4096);
      if (MODE == 5 && (T & 1) == 0) glds2(src + T * 4096, voff, dl + T * 4096);
      const f16x8 x = *reinterpret_cast<const f16x8*>(slot + T * 4096 + lane * 16);
      const f16x8 y = *reinterpret_cast<const f16x8*>(slot + T * 4096 + 1024 + lane * 16);
      const f16x8 z = *reinterpret_cast<const f16x8*>(slot + T * 4096 + 2048 + lane * 16);
      const f16x8 u = *reinterpret_cast<const f16x8*>(slot + T * 4096 + 3072 + lane * 16);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(y, b0, acc[T], 0, 0, 0);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, b1, acc[T], 0, 0, 0);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(x, b0, acc[T], 0, 0, 0);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(u, b0, acc[T], 0, 0, 0);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(z, b1, acc[T], 0, 0, 0);
      acc[T] = __builtin_amdgcn_mfma_f32_32x32x16_f16(z, b0, acc[T], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
  for (int i = 0; i < 8; ++i)
    for (int r = 0; r < 16; ++r) s += acc[i][r];
  if (MODE == 4)
    for (int i = 0; i < 8; ++i) s += st[i][0];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 7) t[MODE] = t1 - t0;
}

template <int MODE>
static void run(const char* img, float* out, unsigned long long* t, int ncu) {
  hipFuncSetAttribute((const void*)k<MODE>, hipFuncAttributeMaxDynamicSharedMemorySize, kNbuf * kSlot);
  for (int rep = 0; rep < 3; ++rep) hipLaunchKernelGGL(k<MODE>, dim3(ncu), dim3(256), kNbuf * kSlot, 0, img, out, t);
  hipDeviceSynchronize();
}

int main() {
  char* img;
  float* out;
  unsigned long long* t;
  int ncu = 0;
  hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipMalloc(&img, 32 << 20);
  hipMemset(img, 0x11, 32 << 20);
  hipMalloc(&out, ncu * 256 * 4);
  hipMalloc(&t, 8 * 8);
  hipMemset(t, 0, 64);
  fprintf(stderr, "start\n");
  run<0>(img, out, t, ncu);
  fprintf(stderr, "mode 0 done\n");
  run<1>(img, out, t, ncu);
  run<2>(img, out, t, ncu);
  run<3>(img, out, t, ncu);
  run<4>(img, out, t, ncu);
  run<5>(img, out, t, ncu);
  unsigned long long th[8] = {0};
  hipMemcpy(th, t, 64, hipMemcpyDeviceToHost);
  const char* names[] = {"none", "glds burst (today)", "glds spread 1/group", "glds multi (1 stmt)",
                         "regs + ds_write_b128", "glds 2/stmt, spread"};
  for (int m = 0; m < 6; ++m)
    printf("mode %d %-24s cycles/step %7.1f  (MFMA floor 48 x 32 = 1536)\n", m, names[m], (double)th[m] / kSteps);
  return 0;
}
