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

// Same DMA with a wave-uniform 64-bit base in SGPRs and the lane's 32-bit byte offset in a VGPR
// (the saddr form): a loop that stages many pieces keeps ONE offset VGPR instead of a 64-bit
// address pair per piece (hoisted out of a persistent tile loop, those pairs spilled).
__device__ __forceinline__ void glds16s(const void* sbase, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(sbase), "s"(lds_byte) : "memory");
}

// f16 hi / lo split of two fp32 values as packed pairs (element 0 in bits 15:0): hi = f16(x) (RNE),
// lo = f16(x - hi) (RNE; x - hi is exact in fp32).  Three VALU per pair -- v_cvt_pk_f16_f32 and one
// v_fma_mixlo / mixhi_f16 per value, which forms fma(hi, -1, x) from the f16 half in fp32 and rounds
// it to f16 in place -- where the scalar form took six conversions and two subtractions (and the
// packing).  Bit-identical to it (tools/micro/split_check.hip).
// lo is formed in x0's register (tied), so a split whose inputs die there costs one new register.
__device__ __forceinline__ void split2(float x0, float x1, uint32_t& hi, uint32_t& lo) {
  uint32_t t = __float_as_uint(x0);
  asm("v_cvt_pk_f16_f32 %0, %1, %2\n\t"
      "v_fma_mixlo_f16 %1, %0, -1.0, %1 op_sel_hi:[1,0,0]\n\t"
      "v_fma_mixhi_f16 %1, %0, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]"
      : "=&v"(hi), "+v"(t)
      : "v"(x1));
  lo = t;
}

// Eight LDS-DMA pieces of 1 KB per wave, 4 KB apart in the source and in LDS (one weight step of the
// MLP kernels), in ONE statement: M0 is saved and restored once and stepped by s_add between the
// pieces, and each source base serves two pieces (lane offsets voff and voff + 4096; the 13-bit
// instruction offset cannot be used: it moves the LDS destination too, and stops at 4095): 18 SALU per
// step where eight glds16s took 40.
__device__ __forceinline__ void glds16s_x8(const char* src, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  const uint32_t voff2 = voff + 4096;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %7\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %4\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %4\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %5\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %5\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %6\n\ts_add_u32 m0, m0, 0x1000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %6\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "v"(voff2), "s"(src), "s"(src + 8192), "s"(src + 16384), "s"(src + 24576), "s"(lds_byte)
      : "memory");
}

// Four LDS-DMA pieces of 1 KB per wave, 8 KB apart in the source and in LDS (one weight step of the
// 16-point-wave forward, mlp16w.h: 8 waves x 4 pieces), in one statement: two source bases, two lane
// offsets (voff, voff + 8 KB), M0 stepped by s_add.
__device__ __forceinline__ void glds16s_x4(const char* src, uint32_t voff, uint32_t lds_byte) {
  unsigned keep;
  const uint32_t voff2 = voff + 8192;
  asm volatile(
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %5\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %3\n\ts_add_u32 m0, m0, 0x2000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %3\n\ts_add_u32 m0, m0, 0x2000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %1, %4\n\ts_add_u32 m0, m0, 0x2000\n\ts_nop 0\n\t"
      "global_load_lds_dwordx4 %2, %4\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "v"(voff2), "s"(src), "s"(src + 16384), "s"(lds_byte)
      : "memory");
}

// 16-B store of a training save (activations, deltas), read back only by a later kernel.
// PNR_SAVE_SC1: write-through (sc1) -- the line is dropped from the XCD's L2 instead of kept
// (MI355X_MICROARCH.md "stores of each flavour"), so the save stream does not evict the weight
// images the LDS-DMA ring re-reads.
__device__ __forceinline__ void save16(float* p, float4 v) {
#if defined(PNR_SAVE_SC1)
  typedef float v4f __attribute__((ext_vector_type(4)));
  const v4f x = {v.x, v.y, v.z, v.w};
  asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(p), "v"(x) : "memory");
#else
  *reinterpret_cast<float4*>(p) = v;
#endif
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
#if defined(PNR_EXP_NOWAIT)  // experiment: barrier without the DMA wait (races on LDS: timing only)
  asm volatile("s_barrier" ::: "memory");
#elif defined(PNR_EXP_NOBAR)  // experiment: the DMA wait without the barrier (races on LDS: timing only)
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#else
  asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
#endif
}

// sin / cos for the Fourier features of the split-precision kernels (decoder.py:26-30).  OCML's
// sinf runs its Payne-Hanek large-argument path for every lane (~113 VALU per call, measured);
// here: k = rint(x 2/pi), r = x - k pi/2 by three fma steps with pi/2 = C1 + C2 + C3 (fp32 parts),
// minimax polynomials on [-pi/4, pi/4], quadrant select: ~20 VALU, max abs error 6.7e-8 on
// |x| < 3000 (= the fp32 libm sinf error; checked in tests/test_host_logic.py).  The fma reduction
// stays exact while k is an exact integer, |x| < 2^22; the Fourier arguments x @ B (scene
// coordinates times B ~ N(0, 25^2), decoder.py:21) are orders of magnitude below.  (A sinf
// fallback branch for large |x| is not used: hipcc if-converts it and runs Payne-Hanek always.)
template <bool COS>
__device__ __forceinline__ float fourier_sc(float x) {
  const float k = __builtin_rintf(x * 0.636619772367581343f);
  float r = __builtin_fmaf(-k, 1.5707963705062866f, x);
  r = __builtin_fmaf(-k, -4.3711388286737929e-08f, r);
  r = __builtin_fmaf(-k, -1.7151245100058819e-15f, r);
  const float z = r * r;
  const float sn = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z,
                                                 -1.6666654611e-1f), z * r, r);
  const float cs = __builtin_fmaf(__builtin_fmaf(__builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, z,
                                                                               -1.388731625493765e-3f), z,
                                                                4.166664568298827e-2f), z, -0.5f), z, 1.f);
  const int q = ((int)k + (COS ? 1 : 0)) & 3;
  const float v = (q & 1) ? cs : sn;
  return (q & 2) ? -v : v;
}

// Power of two s with m s in [2^13, 2^14) (1 for m = 0, inf, NaN): the scale under which a block
// of values with max |x| = m is split into f16 hi + lo parts (in range, 22 bits below the max).
// s is clamped to [2^-100, 2^100]: its products with the weight-image scales (2^-20 .. 2^20, k_wscale)
// and their inverses stay normal fp32 numbers (<= 2^120), and a block down to 2^-86 keeps 22 bits
// (gradients of samples far behind a surface reach 1e-30: the fp32 reference keeps them, so does
// the split path).
constexpr int kScaleExpMax = 100;
__device__ __forceinline__ float pt_scale(float m) {
  if (!(m > 0.f) || !(m < 3.0e38f)) return 1.f;
  int ex;
  (void)frexpf(m, &ex);  // m = f 2^ex, f in [0.5, 1)
  int e = 14 - ex;
  e = e < -kScaleExpMax ? -kScaleExpMax : (e > kScaleExpMax ? kScaleExpMax : e);
  return __int_as_float((e + 127) << 23);
}

}  // namespace pnr
