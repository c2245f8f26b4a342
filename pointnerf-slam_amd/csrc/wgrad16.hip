// wgrad16.hip -- weight-gradient GEMMs of the decoder backward for the split precisions.
//
//   C[256][nb] += A[K][256]^T B[K][WB]     (A, B point-major fp32: row k = one point)
//   bias[256]  += sum_k A[k][:]            (optional)
//
// Used for every precision but PNR_PREC_FP32 (wgrad.hip keeps the fp32-MFMA form) on the shapes of
// src/conv_onet/models/decoder.py:149-159 (and the fc_c branch, :122-125):
//   dW3 = delta4^T h3, dW2 = delta3^T h2, dW1 = delta2^T h1     WB = 256 (8 column tiles)
//   dW0 = delta1^T e                                            WB = 96 (3 column tiles, 93 used)
//   dWc_l = (dL/dh_l)^T c                                       WB = 32 (1 column tile)
// A = deltas / dL/dh stored by k_mlp_bwd16, B = activations / Fourier features stored by
// k_mlp_fwd16 (or the gathered point features), all fp32.  With the feature branch the delta chain
// stores only dL/dh_l (unmasked, for dWc_l); the dW GEMMs then read it as A and apply the forward's
// ReLU mask words themselves (MSK): delta_l = dL/dh_l * [h_l > 0], 1 KB/point less written per layer.
//
// Arithmetic: f16x3, the forward's split.  Each operand x = hi + lo (hi = f16(x), lo = f16(x - hi),
// 22 significant bits); A B ~= Ah Bh + Ah Bl + Al Bh on v_mfma_f32_32x32x16_f16 with fp32
// accumulation (the dropped Al Bl term is 2^-22 relative).  A (gradients: any magnitude) is split
// under a per-wave running power of two sc (max |A| sc < 2^15 on every tile; when a tile needs a
// smaller sc -- the first nonzero one does -- the accumulator is rescaled by the exact ratio).
// B is split unscaled where its range is known (activations < 65504 by the forward's
// PNR_STATUS_F16_RANGE check, |e| <= 1); the point features c (dWc, any magnitude: the reference's
// fine-grid features have std 1e-4, where an unscaled lo part would sit in the f16 subnormals) are
// split under a per-wave running power of two of their own (BSC), like A.  The bias row sums are
// fp32 sums of A.
//
// The GEMM moves 2 x 4 B per point and unit and is HBM-bound (the kernel streams 64 KB per 32-point
// tile at ~3 flops per byte of f16 MFMA work).  K (points) is split over workgroups of 8 waves
// (2 per SIMD, one workgroup per CU); wave w owns output rows [32w, 32w + 32) for the whole K range
// in NTB accumulator tiles and stores them (x 1 / scale) as this workgroup's partial tile, which
// k_part_reduce adds into C in a fixed order (deterministic).
//  - A: each wave reads its own 32 columns straight into registers in MFMA operand order (lane l:
//    column 32w + (l & 31), points 16s + 8(l >> 5) + j): two 128-B lines per load instruction.
//  - B: shared by the 8 waves; the block loads a 32 x WB tile with 16-B loads, splits it and writes
//    the hi and lo planes into LDS as [32-column block T][32 points][64 B];
//    ds_read_b64_tr_b16 returns the MFMA operand (8 consecutive points of one column) transposed.
//  - One register set: tile t+1 is loaded while tile t runs its MFMAs; the LDS planes are double
//    buffered, so one barrier per tile orders both.
#include <cmath>
#include <cstdlib>

#include "mlp16.h"

namespace pnr {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int kTileB = 2112;  // bytes of one [32 points][64 B] block, +64 B pad
// BSC (B = point features, WB = 32): the tile is staged in fp32, rows of kBscRow floats (16-B
// aligned; a wave's 32-lane half reads 32 consecutive columns of one row: conflict-free)
constexpr int kBscRow = 36;

template <int NTB, int WB>
struct Wx3 {
  static constexpr int kThreads = 512;                   // 8 waves, 2 per SIMD
  static constexpr int kPlane = NTB * kTileB;            // one plane (hi or lo) of a B tile
  // the tile's 32 g_out rows (SYN) follow the B image: the two planes, or BSC's fp32 rows
  static constexpr int kGo = 2 * kPlane > 32 * kBscRow * 4 ? 2 * kPlane : 32 * kBscRow * 4;
  static constexpr int kCOff = kGo + 512;                // FC: the tile's c rows (fp32, kBscRow floats)
  static constexpr int kSlot = kCOff + 32 * kBscRow * 4;
  static constexpr int kLds = 2 * kSlot;                 // double-buffered
  static constexpr int kC4 = WB / 4;                     // float4 per B row
  static constexpr int kB4 = 32 * kC4;                   // float4 per B tile
  static constexpr int kBPer = (kB4 + kThreads - 1) / kThreads;
};

// WxArgs: pnr_internal.h (a grouped launch carries one per GEMM)

template <int NTB, int WB>
struct WxRegs {
  float a[16];                                 // A element (k-step s, j) -> a[8s + j]  (SYN: mask words)
  float4 b[Wx3<NTB, WB>::kBPer];               // FOUR: the B row's point x (the values come in stage)
  float4 go;                                   // SYN: g_out row k0 + 32 + tid (threads < 32): the NEXT tile's
  float4 cv;                                   // FC: c piece (row tid / 8, columns 4 (tid % 8)..), threads < 256
  uint32_t mb;                                 // MSK + FC: the ReLU bits of a[0..15] (A itself stays unmasked)
};

// mask-word pointer of unit u = 32 w + (lane & 31) for the 32-point group of k0: the lane's 16
// points 8 hh + 16 s + j sit at word (8 hh + 16 s + j) * 4, bit mask_bit(u) (k_mlp_fwd16 conv1)
__device__ __forceinline__ const uint32_t* mask_words(const uint4* masks, int64_t grp) {
  const int u = 32 * wave_id() + (threadIdx.x & 31);
  return reinterpret_cast<const uint32_t*>(masks + grp * 64 + 32 * ((u >> 2) & 1)) + (u >> 6);
}
__device__ __forceinline__ int mask_bit(int u) { return ((u >> 5) & 1) * 16 + ((u >> 3) & 3) * 4 + (u & 3); }

template <int NTB, int WB, bool SYN, bool FOUR, bool MSK = false, bool FC = false>
__device__ __forceinline__ void wx_load(const WxArgs& a, int64_t k0, WxRegs<NTB, WB>& R) {
  using Cfg = Wx3<NTB, WB>;
  const int tid = threadIdx.x, lane = tid & 63;
  // SYN with WB = 32 (dWc_3): A = dL/dh4 = Wo^T g_out unmasked, so no mask words
  constexpr bool SYN_MASKED = SYN && WB != 32;
  if constexpr (SYN && !SYN_MASKED) {
    if (tid < 32) {
      const int64_t row = k0 + 32 + tid;
      R.go = a.g_out[row < a.K ? row : a.K - 1];
    }
  } else if constexpr (SYN) {
    // mask word of unit u = 32w + (lane & 31) for the lane's 16 points 8 hh + 16 s + j of the
    // 32-point group: uint4 (point + 32 ((u >> 2) & 1)), component u >> 6 (k_mlp_fwd16 conv1)
    const int u = 32 * wave_id() + (lane & 31);
    const uint32_t* mw = reinterpret_cast<const uint32_t*>(a.masks + (a.mgrp0 + k0 / 32) * 64 + 32 * ((u >> 2) & 1)) +
                         (u >> 6);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) R.a[8 * s + j] = __uint_as_float(mw[(8 * (lane >> 5) + 16 * s + j) * 4]);
    if (tid < 32) {  // one tile ahead (staged into the other slot, read after the next barrier)
      const int64_t row = k0 + 32 + tid;
      R.go = a.g_out[row < a.K ? row : a.K - 1];
    }
  } else {
    const float* Ab = a.A + (k0 + 8 * (lane >> 5)) * 256 + 32 * wave_id() + (lane & 31);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int j = 0; j < 8; ++j) R.a[8 * s + j] = Ab[(16 * s + j) * 256];
    if constexpr (MSK && FC) {  // the ReLU bits only: the fc_c GEMM needs A unmasked
      const uint32_t* mw = mask_words(a.amasks, a.mgrp0 + k0 / 32);
      const int bit = mask_bit(32 * wave_id() + (lane & 31));
      uint32_t mb = 0u;
#pragma unroll
      for (int i = 0; i < 16; ++i) mb |= ((mw[(8 * (lane >> 5) + 16 * (i >> 3) + (i & 7)) * 4] >> bit) & 1u) << i;
      R.mb = mb;
    } else if constexpr (MSK) {  // delta = dL/dh where the forward's ReLU passed (bit sign-extended, ANDed)
      const uint32_t* mw = mask_words(a.amasks, a.mgrp0 + k0 / 32);
      const int bit = mask_bit(32 * wave_id() + (lane & 31));
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int m = (int)(mw[(8 * (lane >> 5) + 16 * s + j) * 4] << (31 - bit)) >> 31;
          R.a[8 * s + j] = __int_as_float(__float_as_int(R.a[8 * s + j]) & m);
        }
    }
  }
  if constexpr (FC) {
    if (tid < 256) {
      int64_t row = k0 + (tid >> 3);
      row = row < a.kb_rows ? row : a.kb_rows - 1;
      R.cv = *reinterpret_cast<const float4*>(a.cB + row * kCDim + 4 * (tid & 7));
    }
  }
#pragma unroll
  for (int i = 0; i < Cfg::kBPer; ++i) {
    const int q = tid + Cfg::kThreads * i;
    if (Cfg::kB4 % Cfg::kThreads == 0 || q < Cfg::kB4) {  // wave-uniform
      int64_t row = k0 + q / Cfg::kC4;
      row = row < a.kb_rows ? row : a.kb_rows - 1;
      if constexpr (FOUR) R.b[i] = a.xP[row];
      else R.b[i] = *reinterpret_cast<const float4*>(a.B + row * WB + 4 * (q % Cfg::kC4));
    }
  }
}

// B tile -> hi / lo f16 planes of `slot` (SYN: + the next tile's g_out rows into the other slot;
// BSC: fp32 rows of kBscRow floats)

template <int NTB, int WB, bool SYN, bool FOUR, bool BSC = false, bool PRE = false, bool FC = false>
__device__ __forceinline__ void wx_stage_b(const WxRegs<NTB, WB>& R, char* slot, char* next_slot,
                                           const float (&fbr)[Wx3<NTB, WB>::kBPer][3][4]) {
  using Cfg = Wx3<NTB, WB>;
  const int tid = threadIdx.x;
  if (SYN && tid < 32) reinterpret_cast<float4*>(next_slot + Cfg::kGo)[tid] = R.go;
  if (FC && tid < 256)
    *reinterpret_cast<float4*>(slot + Cfg::kCOff + ((tid >> 3) * kBscRow + 4 * (tid & 7)) * 4) = R.cv;
#pragma unroll
  for (int i = 0; i < Cfg::kBPer; ++i) {
    const int q = tid + Cfg::kThreads * i;
    if (Cfg::kB4 % Cfg::kThreads == 0 || q < Cfg::kB4) {
      const int r = q / Cfg::kC4, c = 4 * (q % Cfg::kC4);
      if constexpr (BSC) {
        *reinterpret_cast<float4*>(slot + (r * kBscRow + c) * 4) = R.b[i];
        continue;
      }
      char* base = slot + (c >> 5) * kTileB + r * 64 + (c & 31) * 2;
      if constexpr (PRE) {  // the forward stored the parts: {hi01, hi23, lo01, lo23} (mlp16w.h kSplitSave)
        const uint4 u = __builtin_bit_cast(uint4, R.b[i]);
        *reinterpret_cast<uint2*>(base) = make_uint2(u.x, u.y);
        *reinterpret_cast<uint2*>(base + Cfg::kPlane) = make_uint2(u.z, u.w);
        continue;
      }
      float v[4] = {R.b[i].x, R.b[i].y, R.b[i].z, R.b[i].w};
      if constexpr (FOUR) {  // e[c + e] = sin(x @ B[:, c + e]), as k_mlp_fwd16's prologue computes it
        const float x0 = R.b[i].x, x1 = R.b[i].y, x2 = R.b[i].z;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float arg;
          {
#pragma clang fp contract(off)
            arg = x0 * fbr[i][0][e];
            arg = __builtin_fmaf(x1, fbr[i][1][e], arg);
            arg = __builtin_fmaf(x2, fbr[i][2][e], arg);
          }
          v[e] = c + e < kFourier ? fourier_sc<false>(arg) : 0.f;
        }
      }
      uint32_t h0, l0, h1, l1;  // packed f16 hi / lo pairs (dev_common.h split2)
      split2(v[0], v[1], h0, l0);
      split2(v[2], v[3], h1, l1);
      *reinterpret_cast<uint2*>(base) = make_uint2(h0, h1);
      *reinterpret_cast<uint2*>(base + Cfg::kPlane) = make_uint2(l0, l1);
    }
  }
}

// MFMA operand of 32-column block T, k-step s: lane l holds column 32T + (l&31), points
// 16s + 8(l>>5) + j, j = 0..7 (two transposed reads; lane 4q+p of 16-lane group g supplies point
// 16s + 8(g>>1) + q (+4), columns 16(g&1) + 4p .. +3)
__device__ __forceinline__ f16x8 tr_frag(const char* img, int T, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const char* base = img + T * kTileB + (16 * s + 8 * (g >> 1) + q) * 64 + 32 * (g & 1) + 8 * p;
  const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
  const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * 64));
  const short e[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  f16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __builtin_bit_cast(_Float16, e[j]);
  return r;
}

// the fp32 B rows of a BSC tile (c: point features, 32 columns) as this lane's operand, split under
// the wave's running B scale sb (lowered, with the accumulator, when this tile needs it), and the
// tile's 6 MFMAs into acc
__device__ __forceinline__ void bsc_tile(const char* rows, const f16x8 (&ah)[2], const f16x8 (&al)[2], f32x16& acc,
                                         float& sb) {
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const float* tb = reinterpret_cast<const float*>(rows) + (lane & 31);
  float bv[16];
  float mb = 0.f;
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bv[8 * s + j] = tb[(16 * s + 8 * hh + j) * kBscRow];
      mb = fmaxf(mb, fabsf(bv[8 * s + j]));
    }
  if (__builtin_amdgcn_ballot_w64(mb * sb >= 32768.f) != 0) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) mb = fmaxf(mb, __shfl_xor(mb, o));
    const float ns = pt_scale(mb);
    const float r = ns / sb;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] *= r;
    sb = ns;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    f16x8 bh, bl;
    split8(bv + 8 * s, sb, bh, bl);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[s], bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[s], bh, acc, 0, 0, 0);
  }
}

// A's 16 values of this lane for one tile -> fp32 row sums, the running scale (accumulators rescaled
// when the tile needs a smaller one) and the hi / lo operands
template <int N>
__device__ __forceinline__ void a_split(const float (&v)[16], float& cs, float& sc, f32x16 (&acc)[N], f16x8 (&ah)[2],
                                        f16x8 (&al)[2]) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    m = fmaxf(m, fabsf(v[i]));
    cs += v[i];
  }
  if (__builtin_amdgcn_ballot_w64(m * sc >= 32768.f) != 0) {  // this tile needs a smaller scale
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    const float ns = pt_scale(m);
    const float r = ns / sc;
#pragma unroll
    for (int y = 0; y < N; ++y)
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[y][i] *= r;
    sc = ns;
  }
#pragma unroll
  for (int s = 0; s < 2; ++s) split8(v + 8 * s, sc, ah[s], al[s]);
}

// workgroup `bid` of one weight-gradient GEMM (k_wgrad16: bid = blockIdx.x; k_wgrad16_group: the
// block's index within its job).  FC (feature branch): the same A tiles also feed the layer's fc_c
// GEMM dWc += A^T c -- A unmasked there (MSK: the ReLU bits are applied for the main GEMM only; SYN:
// dL/dh4 = Wo^T g_out before the h4 mask) -- with its own running scales, accumulator and partials
// (a.part2 / a.part_bias2): the 1 KB / point A stream is read once for both GEMMs.
template <int NTB, int WB, bool SYN, bool FOUR, bool BSC, bool MSK, bool PRE = false, bool FC = false>
__device__ __forceinline__ void wgrad16_body(const WxArgs& a, const int bid, char* lds) {
  static_assert(!PRE || (WB == 256 && !FOUR && !BSC && !MSK), "PRE: B = split h1..h3 (hidden / dW3 GEMMs)");
  static_assert(!MSK || (!SYN && !BSC), "MSK: the hidden / first-layer GEMMs");
  static_assert(!BSC || (NTB == 1 && WB == 32 && !FOUR), "BSC: the fc_c shape");
  static_assert(!SYN || !BSC || !MSK, "SYN + BSC: dWc_3 on A = Wo^T g_out (unmasked)");
  static_assert(!BSC || 32 * kBscRow * 4 <= Wx3<NTB, WB>::kSlot, "BSC tile fits the slot");
  static_assert(!FC || (!BSC && !PRE && (MSK || (SYN && WB == 256))), "FC: on a masked main GEMM");
  using Cfg = Wx3<NTB, WB>;
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int w = wave_id();  // output row block of this wave
  const int64_t kb = (int64_t)bid * a.ks;
  const int64_t ke = kb + a.ks < a.K ? kb + a.ks : a.K;
  const int64_t ntile = (ke - kb) / 32;

  f32x16 acc[NTB];
#pragma unroll
  for (int y = 0; y < NTB; ++y)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[y][r] = 0.f;
  float cs = 0.f;          // fp32 row sums of A (bias) for row 32w + (lane & 31), this lane's points
  float sc = 0x1p100f;     // running scale of A (wave-uniform, <= 2^100 as pt_scale); lowered by a tile
  float sb = 0x1p100f;     // BSC / FC: the same for B = c
  f32x16 accc[1];          // FC: the fc_c tile and its row sums (A scale: sc, shared)
  float csc = 0.f;
  if constexpr (FC) {
#pragma unroll
    for (int r = 0; r < 16; ++r) accc[0][r] = 0.f;
  }
  WxRegs<NTB, WB> R;
  float wo[4];             // SYN: Wo[:, u] of this lane's unit, and its mask bit
  int mbit = 0;
  if constexpr (SYN) {
    const int u = 32 * w + (lane & 31);
#pragma unroll
    for (int i = 0; i < 4; ++i) wo[i] = a.wo[i * kHidden + u];
    mbit = ((u >> 5) & 1) * 16 + ((u >> 3) & 3) * 4 + (u & 3);
  }
  float fbr[Cfg::kBPer][3][4];  // FOUR: Fourier B of this thread's 4 columns (fixed over the tiles)
#pragma unroll
  for (int i = 0; i < Cfg::kBPer; ++i)
#pragma unroll
    for (int d = 0; d < 3; ++d)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        fbr[i][d][e] = FOUR ? a.fb[d * kFourierPad + 4 * ((threadIdx.x + Cfg::kThreads * i) % Cfg::kC4) + e] : 0.f;
  if (ntile > 0) wx_load<NTB, WB, SYN, FOUR, MSK, FC>(a, kb, R);
  if (SYN && ntile > 0) {  // the first tile's g_out rows; later tiles' are staged one tile ahead
    if (threadIdx.x < 32) reinterpret_cast<float4*>(lds + Cfg::kGo)[threadIdx.x] = a.g_out[kb + threadIdx.x];
    __syncthreads();
  }
  for (int64_t t = 0; t < ntile; ++t) {
    char* slot = lds + (t & 1) * Cfg::kSlot;
    // g_out rows of tile t + 1 go to the other slot: their last reader (synth of tile t - 1) ran
    // before the previous barrier
    wx_stage_b<NTB, WB, SYN, FOUR, BSC, PRE, FC>(R, slot, lds + ((t + 1) & 1) * Cfg::kSlot, fbr);
    float au[16];  // FC: A unmasked
    uint32_t keep = 0u;  // FC: the main GEMM's ReLU bits of au[0..15]
    if constexpr (SYN) {
      // delta4 = (Wo^T g_out) masked, fp32 FMAs (the tile's g_out rows from LDS, staged before the
      // previous barrier; broadcast reads)
      const float4* go = reinterpret_cast<const float4*>(slot + Cfg::kGo) + 8 * hh;
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float4 g = go[16 * s + j];
          const float d = __builtin_fmaf(wo[3], g.w, __builtin_fmaf(wo[2], g.z, __builtin_fmaf(wo[1], g.y, wo[0] * g.x)));
          if constexpr (FC) {
            au[8 * s + j] = d;
            keep |= ((__float_as_uint(R.a[8 * s + j]) >> mbit) & 1u) << (8 * s + j);
          } else {
            R.a[8 * s + j] = BSC ? d : (((__float_as_uint(R.a[8 * s + j]) >> mbit) & 1u) ? d : 0.f);
          }
        }
    } else if constexpr (FC) {  // MSK + FC: A arrived unmasked, with its ReLU bits
#pragma unroll
      for (int i = 0; i < 16; ++i) au[i] = R.a[i];
      keep = R.mb;
    }
    f16x8 ah[2], al[2];
    if constexpr (FC) {
      // one running scale for both GEMMs (from A unmasked): the main GEMM's operand is the fc_c one
      // with the masked elements' parts zeroed (split8 of 0 is 0 / 0), so only one split is formed
      // and the two hi / lo sets need not both stay live through the MFMAs
#pragma unroll
      for (int i = 0; i < 16; ++i) cs += ((keep >> i) & 1u) ? au[i] : 0.f;
      float m = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        m = fmaxf(m, fabsf(au[i]));
        csc += au[i];
      }
      if (__builtin_amdgcn_ballot_w64(m * sc >= 32768.f) != 0) {
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
        const float ns = pt_scale(m);
        const float r = ns / sc;
#pragma unroll
        for (int y = 0; y < NTB; ++y)
#pragma unroll
          for (int i = 0; i < 16; ++i) acc[y][i] *= r;
#pragma unroll
        for (int i = 0; i < 16; ++i) accc[0][i] *= r;
        sc = ns;
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) split8(au + 8 * s, sc, ah[s], al[s]);
    } else {
      a_split<NTB>(R.a, cs, sc, acc, ah, al);
    }
    {  // next tile into the (now free) registers; the last tile is re-read (keeps the loop uniform)
      const int64_t tn = t + 1 < ntile ? t + 1 : t;
      wx_load<NTB, WB, SYN, FOUR, MSK, FC>(a, kb + 32 * tn, R);
    }
    __syncthreads();  // planes of tile t written; every wave is done with the slot of tile t - 2
    if constexpr (BSC) {
      bsc_tile(slot, ah, al, acc[0], sb);
    } else {
      const char* ph = slot;
      const char* pl = slot + Cfg::kPlane;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 mh = ah[s], ml = al[s];  // FC: the masked operand
        if constexpr (FC) {
          u32x4 hv = __builtin_bit_cast(u32x4, ah[s]), lv = __builtin_bit_cast(u32x4, al[s]);
#pragma unroll
          for (int d = 0; d < 4; ++d) {
            const uint32_t km = (((keep >> (8 * s + 2 * d)) & 1u) ? 0xFFFFu : 0u) |
                                (((keep >> (8 * s + 2 * d + 1)) & 1u) ? 0xFFFF0000u : 0u);
            hv[d] &= km;
            lv[d] &= km;
          }
          mh = __builtin_bit_cast(f16x8, hv);
          ml = __builtin_bit_cast(f16x8, lv);
        }
#pragma unroll
        for (int y = 0; y < NTB; ++y) {
          const f16x8 bh = tr_frag(ph, y, s), bl = tr_frag(pl, y, s);
          acc[y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(mh, bh, acc[y], 0, 0, 0);
          acc[y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(mh, bl, acc[y], 0, 0, 0);
          acc[y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ml, bh, acc[y], 0, 0, 0);
        }
        if constexpr (FC) __builtin_amdgcn_sched_barrier(0);  // (register pressure: no reads hoisted across)
      }
      if constexpr (FC) bsc_tile(slot + Cfg::kCOff, ah, al, accc[0], sb);
    }
  }
  // two-phase flush: this workgroup's tile with plain stores (each instruction two 128-B row
  // segments), summed in a fixed order by k_part_reduce.  (Float atomics ran at one 256-B
  // wave-instruction per ~50 ns per CU -- a 256 x 256 tile took ~51 us per workgroup -- and left the
  // summation order to the scheduler.)
  // (two multiplies: 1 / (sc sb) can leave the fp32 range where each factor does not)
  const float inv = 1.f / sc, invb = BSC ? 1.f / sb : 1.f;
  float* P = a.part + (int64_t)bid * 256 * (NTB * 32);
#pragma unroll
  for (int y = 0; y < NTB; ++y)
#pragma unroll
    for (int r = 0; r < 16; ++r)
      P[(32 * w + perm(r, hh)) * (NTB * 32) + 32 * y + (lane & 31)] = BSC ? (acc[y][r] * inv) * invb : acc[y][r] * inv;
  cs += __shfl_xor(cs, 32);
  if (a.bias && hh == 0) a.part_bias[(int64_t)bid * 256 + 32 * w + lane] = cs;
  if constexpr (FC) {
    const float invc = 1.f / sc, invs = 1.f / sb;
    float* P2 = a.part2 + (int64_t)bid * 256 * 32;
#pragma unroll
    for (int r = 0; r < 16; ++r) P2[(32 * w + perm(r, hh)) * 32 + (lane & 31)] = (accc[0][r] * invc) * invs;
    csc += __shfl_xor(csc, 32);
    if (a.part_bias2 && hh == 0) a.part_bias2[(int64_t)bid * 256 + 32 * w + lane] = csc;
  }
}

template <int NTB, int WB, bool SYN, bool FOUR, bool BSC, bool MSK, bool PRE = false, bool FC = false>
__global__ __launch_bounds__(512, 1) void k_wgrad16(WxArgs a) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  wgrad16_body<NTB, WB, SYN, FOUR, BSC, MSK, PRE, FC>(a, blockIdx.x, lds);
}

// Skinny weight-gradient GEMMs (fp32 FMAs), bandwidth-bound on B:
//   C[m][n] += sum_k A[k][m] B[k][n]   m < M (<= 4), n < N      (bias[m] += sum_k A[k][m])
// A fp32 rows of 4 (float4: g_out, or x = (x0, x1, x2, inside) with M = 3), B fp32 rows of WB.
//   dWo (4 x 256) = g_out^T h4 (+ dbo)       dB (3 x 93) = x^T g_arg
// A block streams its K range: thread (r, c) = (tid / CPR, tid % CPR) loads 32 B (8 columns) of row
// r and the row's float4 of A, keeping 4 x 8 partial sums; the RPI row groups are then added in
// row-group order through LDS and the block's M x N sums go to the partials (part[block][m N + n],
// pbias[block][m]) that k_part_reduce adds into C / bias in a fixed order.
// (NT threads: 256 as a launch of its own, 512 as a job of the grouped launch; `lds` holds the
// RPI x 4 x WB row-group sums and the RPI x 4 bias sums)
template <int WB, int NT>
struct SkinnyGeo {
  static constexpr int CPR = WB / 8;   // threads per row (32 for 256, 12 for 96)
  static constexpr int RPI = NT / CPR; // rows per iteration (8 / 21 at 256 threads, 16 / 42 at 512)
  static constexpr int kLds = RPI * 4 * WB * 4 + RPI * 4 * 4;
};
template <int WB, int NT>
__device__ __forceinline__ void skinny_body(const float4* __restrict__ A, const float* __restrict__ B, int64_t K,
                                            int64_t ks, int M, int N, float* __restrict__ part,
                                            float* __restrict__ pbias, int bid, char* lds) {
  constexpr int CPR = SkinnyGeo<WB, NT>::CPR;
  constexpr int RPI = SkinnyGeo<WB, NT>::RPI;
  float (*red)[4][WB] = reinterpret_cast<float (*)[4][WB]>(lds);
  float (*redb)[4] = reinterpret_cast<float (*)[4]>(lds + RPI * 4 * WB * 4);
  const int tid = threadIdx.x;
  const int r = tid / CPR, c = tid % CPR;
  const bool act = r < RPI;
  const int64_t kb = (int64_t)bid * ks;
  const int64_t ke = kb + ks < K ? kb + ks : K;
  float acc[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[m][j] = 0.f;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    constexpr int U = 8;  // rows in flight per thread (HBM latency: bytes in flight per CU)
    for (int64_t k = kb + r; k < ke; k += U * RPI) {
      float4 av[U], b0[U], b1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ku = k + u * RPI;
        const int64_t kc = ku < ke ? ku : k;  // rows past the range: re-read row k, weighted 0
        av[u] = A[kc];
        b0[u] = *reinterpret_cast<const float4*>(B + kc * WB + 8 * c);
        b1[u] = *reinterpret_cast<const float4*>(B + kc * WB + 8 * c + 4);
        if (ku >= ke) av[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float a4[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
        const float bv[8] = {b0[u].x, b0[u].y, b0[u].z, b0[u].w, b1[u].x, b1[u].y, b1[u].z, b1[u].w};
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[m][j] = __builtin_fmaf(a4[m], bv[j], acc[m][j]);
        if (c == 0) {
#pragma unroll
          for (int m = 0; m < 4; ++m) bs[m] += a4[m];
        }
      }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[r][m][8 * c + j] = acc[m][j];
    if (c == 0)
#pragma unroll
      for (int m = 0; m < 4; ++m) redb[r][m] = bs[m];
  }
  __syncthreads();
  for (int i = tid; i < M * N; i += NT) {
    const int m = i / N, n = i % N;
    float s = red[0][m][n];
#pragma unroll
    for (int q = 1; q < RPI; ++q) s += red[q][m][n];
    part[(int64_t)bid * M * N + i] = s;
  }
  if (pbias && tid < M) {
    float s = redb[0][tid];
#pragma unroll
    for (int q = 1; q < RPI; ++q) s += redb[q][tid];
    pbias[(int64_t)bid * M + tid] = s;
  }
}
// Every split weight-gradient GEMM of a backward chunk in ONE launch (they are independent): block b
// runs workgroup b - first[q] of job q.  At the Mapper's 1,000-ray batch each GEMM fills ~170 CUs
// for ~30 us and five of them ran back to back; grouped they share the chip, and the launch gaps go.
// Registers and LDS are the largest variant's (all are 512-thread, one-workgroup-per-CU kernels).
struct Wgrad16Group {
  WxArgs a[kMaxGemmJobs];
  int var[kMaxGemmJobs];
  int first[kMaxGemmJobs + 1];
  int n;
};
enum : int { kVarHidden = 0, kVarHiddenM, kVarSyn, kVarFirstX, kVarFirstXM, kVarFc, kVarFcOut, kVarSkinnyOut,
              kVarSkinnyFour, kVarHiddenP, kVarSynP,  // P: B pre-split by the forward (mlp16w.h kSplitSave)
              kVarHiddenMF, kVarFirstXMF, kVarSynF };  // F: + the layer's fc_c GEMM on the same A tiles
// the feature branch's fused jobs (FC) in a kernel of their own: their register pressure (spills) stays
// out of the other jobs' code
__device__ __forceinline__ bool group_skinny(const Wgrad16Group& G, int q, int bid, char* lds) {
  switch (G.var[q]) {
    case kVarSkinnyOut:
      skinny_body<256, 512>(reinterpret_cast<const float4*>(G.a[q].A), G.a[q].B, G.a[q].K, G.a[q].ks, 4, kHidden,
                            G.a[q].part, G.a[q].part_bias, bid, lds);
      return true;
    case kVarSkinnyFour:
      skinny_body<96, 512>(reinterpret_cast<const float4*>(G.a[q].A), G.a[q].B, G.a[q].K, G.a[q].ks, 3, kFourier,
                           G.a[q].part, nullptr, bid, lds);
      return true;
    default: return false;
  }
}
__global__ __launch_bounds__(512, 1) void k_wgrad16_group_fc(Wgrad16Group G) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int q = 0;
  while (q + 1 < G.n && (int)blockIdx.x >= G.first[q + 1]) ++q;
  const int bid = (int)blockIdx.x - G.first[q];
  if (group_skinny(G, q, bid, lds)) return;
  switch (G.var[q]) {
    case kVarHiddenMF: wgrad16_body<8, 256, false, false, false, true, false, true>(G.a[q], bid, lds); break;
    case kVarFirstXMF: wgrad16_body<3, 96, false, true, false, true, false, true>(G.a[q], bid, lds); break;
    default: wgrad16_body<8, 256, true, false, false, false, false, true>(G.a[q], bid, lds); break;  // kVarSynF
  }
}
__global__ __launch_bounds__(512, 1) void k_wgrad16_group(Wgrad16Group G) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  int q = 0;
  while (q + 1 < G.n && (int)blockIdx.x >= G.first[q + 1]) ++q;
  const int bid = (int)blockIdx.x - G.first[q];
  switch (G.var[q]) {
    case kVarHidden: wgrad16_body<8, 256, false, false, false, false>(G.a[q], bid, lds); break;
    case kVarHiddenM: wgrad16_body<8, 256, false, false, false, true>(G.a[q], bid, lds); break;
    case kVarSyn: wgrad16_body<8, 256, true, false, false, false>(G.a[q], bid, lds); break;
    case kVarHiddenP: wgrad16_body<8, 256, false, false, false, false, true>(G.a[q], bid, lds); break;
    case kVarSynP: wgrad16_body<8, 256, true, false, false, false, true>(G.a[q], bid, lds); break;
    case kVarFirstX: wgrad16_body<3, 96, false, true, false, false>(G.a[q], bid, lds); break;
    case kVarFirstXM: wgrad16_body<3, 96, false, true, false, true>(G.a[q], bid, lds); break;
    case kVarFcOut: wgrad16_body<1, 32, true, false, true, false>(G.a[q], bid, lds); break;
    // the skinny fp32 GEMMs (dWo, dB) as jobs of the same launch (skinny_body below; A = float4 rows)
    case kVarSkinnyOut:
      skinny_body<256, 512>(reinterpret_cast<const float4*>(G.a[q].A), G.a[q].B, G.a[q].K, G.a[q].ks, 4, kHidden,
                            G.a[q].part, G.a[q].part_bias, bid, lds);
      break;
    case kVarSkinnyFour:
      skinny_body<96, 512>(reinterpret_cast<const float4*>(G.a[q].A), G.a[q].B, G.a[q].K, G.a[q].ks, 3, kFourier,
                           G.a[q].part, nullptr, bid, lds);
      break;
    default: wgrad16_body<1, 32, false, false, true, false>(G.a[q], bid, lds); break;
  }
}

// Deterministic reduction of per-workgroup partials (every weight-gradient GEMM flushes this way):
//   C[r][c] += sum_{g < nwg} part[g][r pw + c]    (r < nr, c < nb)
//   bias[r] += sum_{g < nwg} pbias[g][r]          (r < nr; bias non-null)
// A block owns 64 consecutive elements; wave v of its 8 sums the partials g = v, v + 8, v + 16, ...
// in that order (two chains, even and odd steps, added at the end), the 8 wave sums are added in
// wave order through LDS and wave 0 updates C with a plain read-modify-write (one owner per
// element).  The summation order is a function of nwg alone: no float atomics, so two runs (eager
// or graph-replayed) give identical bits.
constexpr int kRedWaves = 8;
__global__ __launch_bounds__(64 * kRedWaves) void k_part_reduce(const float* __restrict__ part,
                                                                const float* __restrict__ pbias, int nwg, int nr,
                                                                int pw, int nb, float* __restrict__ C, int64_t ldc,
                                                                float* __restrict__ bias) {
  __shared__ float red[kRedWaves][64];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const int64_t E = (int64_t)nr * pw;
  const int64_t nmain = (E + 63) / 64;
  const bool is_bias = (int64_t)blockIdx.x >= nmain;
  const int64_t e = (is_bias ? (int64_t)blockIdx.x - nmain : (int64_t)blockIdx.x) * 64 + lane;
  const float* src = is_bias ? pbias : part;
  const int64_t stride = is_bias ? nr : E;
  const bool ok = is_bias ? (bias != nullptr && e < nr) : (e < E && (int)(e % pw) < nb);
  float s0 = 0.f, s1 = 0.f;
  if (ok) {
    int g = v;
#pragma unroll 4
    for (; g + kRedWaves < nwg; g += 2 * kRedWaves) {
      s0 += src[(int64_t)g * stride + e];
      s1 += src[(int64_t)(g + kRedWaves) * stride + e];
    }
    if (g < nwg) s0 += src[(int64_t)g * stride + e];
  }
  red[v][lane] = s0 + s1;
  __syncthreads();
  if (v == 0 && ok) {
    float s = red[0][lane];
#pragma unroll
    for (int i = 1; i < kRedWaves; ++i) s += red[i][lane];
    if (is_bias) bias[e] += s;
    else C[(e / pw) * ldc + e % pw] += s;
  }
}

struct ReduceJobs {
  ReduceJob j[kMaxReduceJobs];
  int first[kMaxReduceJobs + 1];  // first block of each job; first[n] = grid
  int vec[kMaxReduceJobs];        // 1: the job's elements go 4 per lane (float4 partial rows)
  int n;
};

// every job of a backward chunk in one launch: block b belongs to the job whose block range holds it,
// then the same fixed-order reduction as k_part_reduce.  A job whose partial rows are whole float4s
// (nr pw and pw multiples of 4, 16-B aligned regions: every GEMM job) runs 4 consecutive elements per
// lane, 256 per block -- the same chains and order per element, a quarter of the blocks and load
// instructions (the partial tiles are the launch's bytes: 55 MB at the room0 batch)
__global__ __launch_bounds__(64 * kRedWaves) void k_part_reduce_multi(ReduceJobs J) {
  __shared__ float4 red[kRedWaves][64];
  int q = 0;
  while (q + 1 < J.n && (int)blockIdx.x >= J.first[q + 1]) ++q;
  const ReduceJob& jb = J.j[q];
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const int64_t E = (int64_t)jb.nr * jb.pw;
  const int64_t blk = (int64_t)blockIdx.x - J.first[q];
  if (J.vec[q]) {
    const int64_t nmain = (E + 255) / 256;
    const bool is_bias = blk >= nmain;
    const int64_t e = (is_bias ? blk - nmain : blk) * 256 + 4 * lane;
    const float* src = is_bias ? jb.pbias : jb.part;
    const int64_t stride = is_bias ? jb.nr : E;
    const bool any = is_bias ? (jb.bias != nullptr && e < jb.nr) : e < E;  // all 4 in range (E, nr: x 4)
    float4 s0 = make_float4(0.f, 0.f, 0.f, 0.f), s1 = s0;
    if (any) {
      int g = v;
#pragma unroll 4
      for (; g + kRedWaves < jb.nwg; g += 2 * kRedWaves) {
        const float4 a = *reinterpret_cast<const float4*>(src + (int64_t)g * stride + e);
        const float4 b = *reinterpret_cast<const float4*>(src + (int64_t)(g + kRedWaves) * stride + e);
        s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
        s1.x += b.x; s1.y += b.y; s1.z += b.z; s1.w += b.w;
      }
      if (g < jb.nwg) {
        const float4 a = *reinterpret_cast<const float4*>(src + (int64_t)g * stride + e);
        s0.x += a.x; s0.y += a.y; s0.z += a.z; s0.w += a.w;
      }
    }
    red[v][lane] = make_float4(s0.x + s1.x, s0.y + s1.y, s0.z + s1.z, s0.w + s1.w);
    __syncthreads();
    if (v == 0 && any) {
      float4 t = red[0][lane];
#pragma unroll
      for (int i = 1; i < kRedWaves; ++i) {
        const float4 u = red[i][lane];
        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
      }
      const float sv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t ek = e + k;
        if (!is_bias && (int)(ek % jb.pw) >= jb.nb) continue;  // padding columns (W0: 93 of 96)
        float* dst = is_bias ? jb.bias + ek : jb.C + (ek / jb.pw) * jb.ldc + ek % jb.pw;
        *dst = (jb.overwrite ? 0.f : *dst) + sv[k];
      }
    }
    return;
  }
  const int64_t nmain = (E + 63) / 64;
  const bool is_bias = blk >= nmain;
  const int64_t e = (is_bias ? blk - nmain : blk) * 64 + lane;
  const float* src = is_bias ? jb.pbias : jb.part;
  const int64_t stride = is_bias ? jb.nr : E;
  const bool ok = is_bias ? (jb.bias != nullptr && e < jb.nr) : (e < E && (int)(e % jb.pw) < jb.nb);
  float s0 = 0.f, s1 = 0.f;
  if (ok) {
    int g = v;
#pragma unroll 4
    for (; g + kRedWaves < jb.nwg; g += 2 * kRedWaves) {
      s0 += src[(int64_t)g * stride + e];
      s1 += src[(int64_t)(g + kRedWaves) * stride + e];
    }
    if (g < jb.nwg) s0 += src[(int64_t)g * stride + e];
  }
  red[v][lane].x = s0 + s1;
  __syncthreads();
  if (v == 0 && ok) {
    float s = red[0][lane].x;
#pragma unroll
    for (int i = 1; i < kRedWaves; ++i) s += red[i][lane].x;
    float* dst = is_bias ? jb.bias + e : jb.C + (e / jb.pw) * jb.ldc + e % jb.pw;
    *dst = (jb.overwrite ? 0.f : *dst) + s;
  }
}

int launch_part_reduce_multi(const ReduceJob* jobs, int n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > kMaxReduceJobs) return PNR_E_ARG;
  static const bool vec_ok = !(getenv("PNR_REDUCE_VEC") && getenv("PNR_REDUCE_VEC")[0] == '0');
  ReduceJobs J{};
  int blocks = 0;
  for (int i = 0; i < n; ++i) {
    const ReduceJob& r = jobs[i];
    J.j[i] = r;
    J.first[i] = blocks;
    const int64_t E = (int64_t)r.nr * r.pw;
    const bool vec = vec_ok && E % 4 == 0 && r.pw % 4 == 0 && r.nr % 4 == 0 &&
                     reinterpret_cast<uintptr_t>(r.part) % 16 == 0 &&
                     (r.bias == nullptr || reinterpret_cast<uintptr_t>(r.pbias) % 16 == 0);
    J.vec[i] = vec ? 1 : 0;
    const int epb = vec ? 256 : 64;
    blocks += (int)((E + epb - 1) / epb + (r.bias ? (r.nr + epb - 1) / epb : 0));
  }
  J.first[n] = blocks;
  J.n = n;
  hipLaunchKernelGGL(k_part_reduce_multi, dim3((unsigned)blocks), dim3(64 * kRedWaves), 0, st, J);
  return hip_status(hipGetLastError());
}

int launch_part_reduce(const float* part, const float* pbias, int nwg, int nr, int pw, int nb, float* C, int64_t ldc,
                       float* bias, hipStream_t st) {
  if (nwg <= 0) return 0;
  const int64_t nmain = ((int64_t)nr * pw + 63) / 64;
  const int64_t nbias = bias ? (nr + 63) / 64 : 0;
  hipLaunchKernelGGL(k_part_reduce, dim3((unsigned)(nmain + nbias)), dim3(64 * kRedWaves), 0, st, part, pbias, nwg,
                     nr, pw, nb, C, ldc, bias);
  return hip_status(hipGetLastError());
}

template <int NTB, int WB, bool SYN = false, bool FOUR = false, bool BSC = false, bool MSK = false>
static int launch_k(const WxArgs& a, hipStream_t st, ReduceJob* defer) {
  using Cfg = Wx3<NTB, WB>;
  auto kern = k_wgrad16<NTB, WB, SYN, FOUR, BSC, MSK>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               Cfg::kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  const int nwg = (int)((a.K + a.ks - 1) / a.ks);
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(Cfg::kThreads), Cfg::kLds, st, a);
  const int rc = hip_status(hipGetLastError());
  if (rc) return rc;
  if (defer) {
    *defer = ReduceJob{a.part, a.part_bias, nwg, 256, NTB * 32, a.nb, a.C, a.ldc, a.bias};
    return 0;
  }
  return launch_part_reduce(a.part, a.part_bias, nwg, 256, NTB * 32, a.nb, a.C, a.ldc, a.bias, st);
}

// kind: kWgradHidden (B [K][256]), kWgradFirst (B [K][96], 93 columns) or kWgradFc (B [K][32]);
// K is rounded up to 32 (the A rows up to it exist and carry zero deltas).  Fills the job's
// arguments, its kernel variant and its reduction (the partials go to the backward's scratch:
// WgradSyn part / part_bias).
// per-tile costs measured with PNR_WGRAD_SPLIT=1 (one job per launch, 28-56 workgroups, 43-85 tiles each):
// dW3 (delta4 rebuilt) 2.79-2.85 us, dW2 / dW1 2.50-2.85, dW0 (e recomputed) 1.74-2.14, dWc 1.00-1.09 per
// tile: relative to a plain hidden GEMM
// (the first-layer weight as a build knob; A/B at the end of round 5, room0 / C3 graph ms: 0.60 -> C3
// 0.863-0.864, 0.85 -> 0.514-0.516 / 0.835-0.837, 0.72 -> 0.516-0.518 / 0.832-0.839: kept)
#ifndef PNR_W_FIRSTX
#define PNR_W_FIRSTX 0.72f
#endif
float wgrad16_job_weight(int kind, bool masked) {
  (void)masked;
  switch (kind) {
    case kWgradOutDelta: return 1.05f;
    case kWgradFirstX: return PNR_W_FIRSTX;
    case kWgradFc: return 0.38f;
    case kWgradFcOut: return 0.40f;
    default: return 1.0f;
  }
}

int wgrad16_prepare(int kind, const float* A, const float* B, int64_t K, int64_t kb_rows, float* C, int64_t ldc,
                    float* bias, const WgradSyn* syn, Wgrad16Job* job, ReduceJob* red, ReduceJob* red2) {
  if (kb_rows <= 0) return PNR_E_ARG;
  K = (K + 31) / 32 * 32;
  // split-K over at most one workgroup per CU, >= 8 tiles per workgroup (the flush of the partial
  // tile no longer dominates)
  if (!syn || !syn->part || !syn->part_bias) return PNR_E_ARG;
  // Tiles (32 points) per workgroup: >= 8, up to 256 workgroups per GEMM.  Every workgroup flushes a
  // whole 256 x 256 partial tile that k_part_reduce_multi re-reads, so a grouped launch whose GEMMs
  // are small (the Mapper's 1,000-ray batch: 2,400 tiles x 4 GEMMs) is sized to fill the chip about
  // once instead (one workgroup per CU: 133 + 18 us of GEMM + reduction there against 166 + 46 us at
  // 8 tiles per workgroup); large GEMMs (S-map) keep the wide grid, which hides latency better
  // (109 ms against 117 ms for the S-map step with one workgroup per CU).
  const int64_t tiles = K / 32;
  int64_t per = 8;
  if (syn->group_jobs > 0) {
    int64_t cus = device_cu_count() - syn->reserve_cus;
    cus = cus < 1 ? 1 : cus;
    const int64_t fill = (tiles * syn->group_jobs + cus - 1) / cus;
    if (fill <= 256) {
      // one round of workgroups: tiles per workgroup so that every job's workgroups take about the same
      // time (the group's summed cost over the CUs, divided by this kind's cost per tile)
      const float w = wgrad16_job_weight(kind, syn->amasks != nullptr) + (syn->fc_c ? kWgradFcFusedWeight : 0.f);
      const float gw = syn->group_weight > 0.f ? syn->group_weight : (float)syn->group_jobs;
      const int64_t wfill = (int64_t)((double)tiles * gw / ((double)cus * w) + 0.999);
      per = wfill > per ? wfill : per;
    }
  }
  int64_t nwg = (tiles + per - 1) / per;
  nwg = nwg < 4 ? 4 : (nwg > kWgrad16MaxWg ? kWgrad16MaxWg : nwg);
  int64_t ks = (K + nwg - 1) / nwg;
  ks = (ks + 31) / 32 * 32;
  nwg = (K + ks - 1) / ks;
  WxArgs a{A, B, 256, K, kb_rows, ks, C, ldc, bias, nullptr, nullptr, 0, nullptr, nullptr, nullptr, nullptr,
           syn->part, syn->part_bias};
  const bool msk = syn->amasks != nullptr;
  if (msk) {
    if (kind != kWgradHidden && kind != kWgradFirstX) return PNR_E_ARG;
    a.amasks = syn->amasks;
    a.mgrp0 = syn->mgrp0;
  }
  int var, ntb;
  if (kind == kWgradHidden) {
    if (msk && syn->bsplit) return PNR_E_ARG;  // the feature-branch forward saves fp32
    var = msk ? kVarHiddenM : (syn->bsplit ? kVarHiddenP : kVarHidden);
    ntb = 8;
  } else if (kind == kWgradOutDelta) {  // dW3 += delta4^T h3, delta4 rebuilt from g_out and the h4 masks
    if (!syn->g_out || !syn->masks || !syn->wo) return PNR_E_ARG;
    a.g_out = syn->g_out;
    a.masks = syn->masks;
    a.mgrp0 = syn->mgrp0;
    a.wo = syn->wo;
    var = syn->bsplit ? kVarSynP : kVarSyn;
    ntb = 8;
  } else if (kind == kWgradFc) {  // dWc_l (256 x 32) += gH_l^T c
    a.nb = kCDim;
    var = kVarFc;
    ntb = 1;
  } else if (kind == kWgradFcOut) {  // dWc_3 (256 x 32) += (Wo^T g_out)^T c: dL/dh4 rebuilt, not read
    if (!syn->g_out || !syn->wo) return PNR_E_ARG;
    a.nb = kCDim;
    a.g_out = syn->g_out;
    a.wo = syn->wo;
    var = kVarFcOut;
    ntb = 1;
  } else if (kind == kWgradFirstX) {  // dW0 (256 x 93) += delta1^T sin(x@B): e recomputed from x
    if (!syn->xP || !syn->fb) return PNR_E_ARG;
    a.nb = kFourier;
    a.xP = syn->xP;
    a.fb = syn->fb;
    var = msk ? kVarFirstXM : kVarFirstX;
    ntb = 3;
  } else {
    return PNR_E_ARG;
  }
  if (syn->fc_c) {  // + the layer's fc_c GEMM on the same A tiles (A unmasked), partials after the main ones
    if (!red2 || !syn->fc_C) return PNR_E_ARG;
    if (var == kVarHiddenM) var = kVarHiddenMF;
    else if (var == kVarFirstXM) var = kVarFirstXMF;
    else if (var == kVarSyn) var = kVarSynF;
    else return PNR_E_ARG;  // FC runs on a masked main GEMM (the feature branch's dW jobs)
    a.cB = syn->fc_c;
    a.part2 = a.part + nwg * 256 * ntb * 32;
    a.part_bias2 = syn->fc_bias ? a.part_bias + nwg * 256 : nullptr;
    *red2 = ReduceJob{a.part2, a.part_bias2, (int)nwg, 256, 32, kCDim, syn->fc_C, kCDim, syn->fc_bias};
  }
  job->a = a;
  job->var = var;
  job->nwg = (int)nwg;
  *red = ReduceJob{a.part, a.part_bias, (int)nwg, 256, ntb * 32, a.nb, a.C, a.ldc, a.bias};
  return 0;
}

int launch_wgrad16_group(const Wgrad16Job* jobs, int n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > kMaxGemmJobs) return PNR_E_ARG;
  constexpr int kLds = Wx3<8, 256>::kLds;  // the largest variant
  static_assert(Wx3<3, 96>::kLds <= kLds && Wx3<1, 32>::kLds <= kLds, "group LDS");
  static_assert(SkinnyGeo<256, 512>::kLds <= kLds && SkinnyGeo<96, 512>::kLds <= kLds, "group LDS (skinny jobs)");
  static const bool attr = hipFuncSetAttribute((const void*)k_wgrad16_group, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               kLds) == hipSuccess &&
                           hipFuncSetAttribute((const void*)k_wgrad16_group_fc,
                                               hipFuncAttributeMaxDynamicSharedMemorySize, kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  Wgrad16Group G{};
  int blocks = 0;
  int64_t macs = 0;  // timing units (pnr_timing_read kind 6): multiply-adds / 65,536
  int nfc = 0, nplain = 0;
  for (int i = 0; i < n; ++i) {
    G.a[i] = jobs[i].a;
    G.var[i] = jobs[i].var;
    G.first[i] = blocks;
    blocks += jobs[i].nwg;
    const bool fc = jobs[i].var == kVarHiddenMF || jobs[i].var == kVarFirstXMF || jobs[i].var == kVarSynF;
    const bool skinny = jobs[i].var == kVarSkinnyOut || jobs[i].var == kVarSkinnyFour;
    nfc += fc ? 1 : 0;
    nplain += (fc || skinny) ? 0 : 1;
    macs += jobs[i].a.K * 256 * (jobs[i].a.nb + (fc ? kCDim : 0));
  }
  if (nfc > 0 && nplain > 0) return PNR_E_ARG;  // FC jobs run in k_wgrad16_group_fc, with the skinny ones only
  G.first[n] = blocks;
  G.n = n;
  TimingScope ts(kTimeWgradGroup, macs / 65536, st);
  if (nfc > 0) hipLaunchKernelGGL(k_wgrad16_group_fc, dim3((unsigned)blocks), dim3(512), kLds, st, G);
  else hipLaunchKernelGGL(k_wgrad16_group, dim3((unsigned)blocks), dim3(512), kLds, st, G);
  return hip_status(hipGetLastError());
}

template <int NTB, int WB, bool SYN = false, bool FOUR = false, bool BSC = false, bool MSK = false, bool PRE = false,
          bool FC = false>
static int launch_k(const WxArgs& a, int nwg, hipStream_t st) {
  using Cfg = Wx3<NTB, WB>;
  auto kern = k_wgrad16<NTB, WB, SYN, FOUR, BSC, MSK, PRE, FC>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               Cfg::kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(Cfg::kThreads), Cfg::kLds, st, a);
  return hip_status(hipGetLastError());
}

// one GEMM on its own kernel variant; its reduction deferred into *defer or launched now
int launch_wgrad16(int kind, const float* A, const float* B, int64_t K, int64_t kb_rows, float* C, int64_t ldc,
                   float* bias, hipStream_t st, const WgradSyn* syn, ReduceJob* defer) {
  if (K <= 0) return 0;
  Wgrad16Job j;
  ReduceJob red;
  int rc = wgrad16_prepare(kind, A, B, K, kb_rows, C, ldc, bias, syn, &j, &red);
  if (rc) return rc;
  TimingScope ts(kTimeWgrad, j.a.K, st);
  switch (j.var) {
    case kVarHidden: rc = launch_k<8, 256>(j.a, j.nwg, st); break;
    case kVarHiddenM: rc = launch_k<8, 256, false, false, false, true>(j.a, j.nwg, st); break;
    case kVarSyn: rc = launch_k<8, 256, true>(j.a, j.nwg, st); break;
    case kVarHiddenP: rc = launch_k<8, 256, false, false, false, false, true>(j.a, j.nwg, st); break;
    case kVarSynP: rc = launch_k<8, 256, true, false, false, false, true>(j.a, j.nwg, st); break;
    case kVarHiddenMF: rc = launch_k<8, 256, false, false, false, true, false, true>(j.a, j.nwg, st); break;
    case kVarFirstXMF: rc = launch_k<3, 96, false, true, false, true, false, true>(j.a, j.nwg, st); break;
    case kVarSynF: rc = launch_k<8, 256, true, false, false, false, false, true>(j.a, j.nwg, st); break;
    case kVarFirstX: rc = launch_k<3, 96, false, true>(j.a, j.nwg, st); break;
    case kVarFirstXM: rc = launch_k<3, 96, false, true, false, true>(j.a, j.nwg, st); break;
    case kVarFcOut: rc = launch_k<1, 32, true, false, true>(j.a, j.nwg, st); break;
    default: rc = launch_k<1, 32, false, false, true>(j.a, j.nwg, st); break;
  }
  if (rc) return rc;
  if (defer) {
    *defer = red;
    return 0;
  }
  return launch_part_reduce(red.part, red.pbias, red.nwg, red.nr, red.pw, red.nb, red.C, red.ldc, red.bias, st);
}

template <int WB>
__global__ __launch_bounds__(256) void k_wgrad_skinny(const float4* __restrict__ A, const float* __restrict__ B,
                                                      int64_t K, int64_t ks, int M, int N, float* __restrict__ part,
                                                      float* __restrict__ pbias) {
  __shared__ __attribute__((aligned(16))) char lds[SkinnyGeo<WB, 256>::kLds];
  skinny_body<WB, 256>(A, B, K, ks, M, N, part, pbias, blockIdx.x, lds);
}

// rows per workgroup: >= 256 (a 256-thread launch) / >= 512 (a grouped job), at most kSkinnyMaxWg groups
static int skinny_blocks(int64_t K, int64_t* ks, int64_t min_rows = 256) {
  *ks = (K + kSkinnyMaxWg - 1) / kSkinnyMaxWg;
  if (*ks < min_rows) *ks = min_rows;
  return (int)((K + *ks - 1) / *ks);
}

// dWo / dB as jobs of a grouped launch (512-thread workgroups of >= 512 rows): arguments in the job's
// WxArgs (A = the float4 rows, B, K, ks, partials), reduction into *red
int wgrad_skinny_prepare(int out, const float* A4, const float* B, int64_t K, float* C, float* bias, float* part,
                         float* part_bias, Wgrad16Job* job, ReduceJob* red) {
  if (K <= 0 || !part || (out && !part_bias)) return PNR_E_ARG;
  int64_t ks;
  const int nb = skinny_blocks(K, &ks, 512);
  WxArgs a{};
  a.A = A4;
  a.B = B;
  a.K = K;
  a.ks = ks;
  a.part = part;
  a.part_bias = out && bias ? part_bias : nullptr;
  job->a = a;
  job->var = out ? kVarSkinnyOut : kVarSkinnyFour;
  job->nwg = nb;
  *red = out ? ReduceJob{part, part_bias, nb, 4, kHidden, kHidden, C, (int64_t)kHidden, bias}
             : ReduceJob{part, nullptr, nb, 3, kFourier, kFourier, C, (int64_t)kFourier, nullptr};
  return 0;
}

// dWo (4 x 256) += g_out^T h4, dbo += colsum(g_out)
int launch_wgrad_out16(const float* g_out, const float* h4, int64_t K, float* C, float* bias, float* part,
                       float* part_bias, hipStream_t st, ReduceJob* defer) {
  if (K <= 0) return 0;
  if (!part || !part_bias) return PNR_E_ARG;
  int64_t ks;
  const int nb = skinny_blocks(K, &ks);
  TimingScope ts(kTimeWgrad, K, st);
  hipLaunchKernelGGL(k_wgrad_skinny<256>, dim3((unsigned)nb), dim3(256), 0, st, reinterpret_cast<const float4*>(g_out),
                     h4, K, ks, 4, kHidden, part, bias ? part_bias : nullptr);
  const int rc = hip_status(hipGetLastError());
  if (rc) return rc;
  if (defer) {
    *defer = ReduceJob{part, part_bias, nb, 4, kHidden, kHidden, C, (int64_t)kHidden, bias};
    return 0;
  }
  return launch_part_reduce(part, part_bias, nb, 4, kHidden, kHidden, C, (int64_t)kHidden, bias, st);
}

// dB (3 x 93) += x^T g_arg: x rows float4 (x0, x1, x2, inside), g_arg fp32 [K][96]
int launch_wgrad_fourier16(const float4* xP, const float* garg, int64_t K, float* C, float* part, hipStream_t st,
                           ReduceJob* defer) {
  if (K <= 0) return 0;
  if (!part) return PNR_E_ARG;
  int64_t ks;
  const int nb = skinny_blocks(K, &ks);
  TimingScope ts(kTimeWgrad, K, st);
  hipLaunchKernelGGL(k_wgrad_skinny<96>, dim3((unsigned)nb), dim3(256), 0, st, xP, garg, K, ks, 3, kFourier, part,
                     nullptr);
  const int rc = hip_status(hipGetLastError());
  if (rc) return rc;
  if (defer) {
    *defer = ReduceJob{part, nullptr, nb, 3, kFourier, kFourier, C, (int64_t)kFourier, nullptr};
    return 0;
  }
  return launch_part_reduce(part, nullptr, nb, 3, kFourier, kFourier, C, (int64_t)kFourier, nullptr, st);
}

}  // namespace pnr
