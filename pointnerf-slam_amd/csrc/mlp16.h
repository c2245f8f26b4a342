// mlp16.h -- decoder forward on the 16-bit matrix cores (v_mfma_f32_32x32x16_{f16,bf16}).
//
// Same math as k_mlp_fwd (mlp.hip; src/conv_onet/models/decoder.py:177-203 plus the bound mask of
// src/utils/Renderer.py:43-57 and the fc_c feature branch of decoder.py:196-197), three precisions
// (PR = PNR_PREC_* code):
//   F16X3  every fp32 operand split x = hi + lo, hi = f16(x), lo = f16(x - hi) (22 significant
//          bits); W x ~= Wh xh + Wh xl + Wl xh accumulated in fp32: ~2^-21 relative per product.
//          The weights are scaled by a per-layer power of two (k_wscale) so that their lo parts
//          stay out of the f16 subnormal range and max |W| s <= 2^14; the accumulator is scaled
//          back exactly (acc * 2^-e) before the bias.
//   BF16X3 the same split in bf16 (16 significant bits, ~2^-16 per product; no range limits).
//   BF16   hi parts only (BASELINE config C3: bf16 MLP on MFMA).
// The split forms run 3 MFMAs per 16-deep k-step at 32 cycles: 5.3x the fp32 MFMA rate (8 MFMAs
// of 64 cycles for the same depth).
//
// Execution model (one workgroup = 4 waves = 128 points, one wave per SIMD, 32 points per wave):
//  - The point index sits on the MFMA column (lane & 31).  A 256-unit layer output is 8 fp32
//    accumulator tiles; register r of tile t in lane half hh is unit 32t + perm(r, hh).
//  - A k-step s (s = 0, 1) of input tile kc takes registers 8s..8s+7 of that tile's accumulator,
//    converted to 16 bits, as the B operand (element j of lane half h <-> unit 32kc + perm(8s+j, h)):
//    the activation never leaves the registers.  The weights (A operand) are pre-split and
//    pre-permuted by k_pack16 into exactly that order.
//  - Weights stream through a ring of kNbuf LDS slots by LDS-DMA (one slot per "step" = one input
//    tile of one layer for all 8 output tiles), kNbuf-1 steps in flight.
//  - Lazy epilogue: two accumulator sets (prev, next layer).  While step kc of layer L+1 runs its
//    MFMAs on input tile kc, the VALU builds tile kc+1 (bias, ReLU, feature branch, split) from
//    the previous layer's accumulators, in pieces placed between the MFMA groups.
//  - Feature branch h_L += Wc_L c + bc_L (decoder.py:196-197): c (32 channels) is one B tile kept
//    in registers; each converted tile adds one 32x32 product (6 MFMAs) whose A fragments ride in
//    a 4 KiB tail of the step's slot (the fc stream is laid out in conversion order).
#pragma once
#include <type_traits>

#include "dev_common.h"

namespace pnr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

template <int PR>
struct Prec {
  static constexpr int NP = PR == PNR_PREC_BF16 ? 1 : 2;  // parts per operand
  static constexpr bool F16 = PR == PNR_PREC_F16X3;
  using E = typename std::conditional<F16, _Float16, __bf16>::type;
  using V8 = typename std::conditional<F16, f16x8, bf16x8>::type;
  static __device__ __forceinline__ f32x16 mfma(const V8& a, const V8& b, const f32x16& c) {
    if constexpr (F16) return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
    else return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
  }
};

// ---- stream geometry (see k_pack16) -----------------------------------------------------------
// steps g: 0..2 layer 0 (Fourier tiles), 3..10 / 11..18 / 19..26 hidden layers 1..3, 27..34 output
constexpr int kBfSteps = 35;
// main image: hidden steps NP*16 KiB [T 8][s 2][part NP][lane 64][8]; output steps 4 KiB
// [s 2][part NP][lane 64][8] (zero-padded).  fc image: 32 entries of 4 KiB, entry e = 8L + t
// holds Wc_L rows of unit tile t as [s 2][part NP][lane 64][8] (zero-padded).
constexpr int64_t bf_main_bytes(int np) { return 27LL * np * 16384 + 8LL * 4096; }
constexpr int64_t kBfFcBytes = 32LL * 4096;
// raw float table (LDS-resident): b0..b3 [4][256], bo [32] (4 used), Fourier B [3][96],
// f16 weight scales: inverse [5] (W0..W3, Wo) and forward [5]
constexpr int kRawB = 0, kRawBo = 1024, kRawFB = 1056, kRawInv = 1344, kRawScl = 1352;
constexpr int64_t kRawBytes = 8192;   // padded to 2 x 4 KiB (two DMA pieces)
// fc raw: bc_0..bc_3 [4][256], then the f16 scales of Wc_0..Wc_3: inverse [4], forward [4]
constexpr int kFcRawInv = 1024, kFcRawScl = 1028;
constexpr int64_t kFcRawBytes = 8192;

// Backward (delta chain) image, bf16x3: steps g = 0: Wo^T (K = 4: one k-step) [T 8][part 2][lane][8];
// 1..24: W3^T, W2^T, W1^T input tiles [T 8][s 2][part 2][lane][8]; 25..32: W0^T (96 output rows)
// [T 3][s 2][part 2][lane][8].  fc backward image: 32 entries of 4 KiB, entry e = 8(3 - l) + t
// holds Wc_l^T over unit tile t as [s 2][part 2][lane][8].
constexpr int kBwdSteps = 33;
__host__ __device__ constexpr int64_t bwd_main_off(int g) {
  return g == 0 ? 0 : (g <= 25 ? 16384LL + (g - 1) * 32768LL : 16384LL + 24 * 32768LL + (g - 25) * 12288LL);
}
constexpr int64_t kBwdBytes = bwd_main_off(kBwdSteps);

// Packed buffer (floats): [fp32 image][BF16X3 main][BF16 main][F16X3 main][BF16X3 bwd][raw]
constexpr int64_t kOffBf2 = kPackedFloats;
constexpr int64_t kOffBf1 = kOffBf2 + bf_main_bytes(2) / 4;
constexpr int64_t kOffH2 = kOffBf1 + bf_main_bytes(1) / 4;
constexpr int64_t kOffBwd = kOffH2 + bf_main_bytes(2) / 4;
constexpr int64_t kOffRaw = kOffBwd + kBwdBytes / 4;
constexpr int64_t kPackedFloatsAll = kOffRaw + kRawBytes / 4;
// fc buffer (floats): [fp32 fc image][BF16X3 fc][BF16 fc][F16X3 fc][BF16X3 fc bwd][raw]
constexpr int64_t kOffFcBf2 = kFcPackedFloats;
constexpr int64_t kOffFcBf1 = kOffFcBf2 + kBfFcBytes / 4;
constexpr int64_t kOffFcH2 = kOffFcBf1 + kBfFcBytes / 4;
constexpr int64_t kOffFcBwd = kOffFcH2 + kBfFcBytes / 4;
constexpr int64_t kOffFcRaw = kOffFcBwd + kBfFcBytes / 4;
constexpr int64_t kFcPackedFloatsAll = kOffFcRaw + kFcRawBytes / 4;

static_assert(kOffBf2 % 4 == 0 && kOffFcBf2 % 4 == 0, "16-B aligned images");

constexpr int64_t main_off_floats(int pr) {
  return pr == PNR_PREC_BF16X3 ? kOffBf2 : pr == PNR_PREC_BF16 ? kOffBf1 : kOffH2;
}
constexpr int64_t fc_off_floats(int pr) {
  return pr == PNR_PREC_BF16X3 ? kOffFcBf2 : pr == PNR_PREC_BF16 ? kOffFcBf1 : kOffFcH2;
}

// ---------------------------------------------------------------------------------------------
// Forward kernel
// ---------------------------------------------------------------------------------------------
// Forward step program: layer and input tile of step g, and the epilogue job placed in it
// (h_CL tile CT; tile 0 of a layer is built in that layer's last step).
__host__ __device__ constexpr int fwd_layer(int g) { return g < 3 ? 0 : (g < 27 ? 1 + (g - 3) / 8 : 4); }
__host__ __device__ constexpr int fwd_kc(int g) { return g < 3 ? g : (g - 3) % 8; }
__host__ __device__ constexpr bool fwd_conv(int g) {
  return !(fwd_layer(g) == 0 && fwd_kc(g) < 2) && !(fwd_layer(g) == 4 && fwd_kc(g) == 7);
}
__host__ __device__ constexpr int fwd_ct(int g) {
  return (fwd_layer(g) == 0 || (fwd_layer(g) <= 3 && fwd_kc(g) == 7)) ? 0 : fwd_kc(g) + 1;
}
// activation-save stores one wave issues in step g (SAVE): 4 h quads + the mask words after tile 7
__host__ __device__ constexpr int fwd_stores(int g) { return fwd_conv(g) ? 4 + (fwd_ct(g) == 7 ? 1 : 0) : 0; }
constexpr int kFwdPrologueStores = 13;  // e tiles (3 x 4 quads) + x

template <int NP, bool HASC, bool SAVE = false>
struct BfGeo {
  static constexpr int kMainH = NP * 16384;                  // bytes of a hidden main piece
  static constexpr int kSlot = kMainH + (HASC ? 4096 : 0);   // LDS slot bytes
  static constexpr int kNbuf = NP == 2 ? 4 : 6;
  static constexpr int kDist = kNbuf - 1;                    // steps in flight
  static constexpr int kRawLds = kRawBytes + (HASC ? kFcRawBytes : 0);
  static constexpr int kLds = kNbuf * kSlot + kRawLds;
  __host__ __device__ static constexpr int main_n(int g) { return g < 27 ? kMainH / 4096 : 1; }
  __host__ __device__ static constexpr int fc_n(int g) { return (HASC && g >= 2 && g <= 33) ? 1 : 0; }
  __host__ __device__ static constexpr int n_glds(int g) { return g < kBfSteps ? main_n(g) + fc_n(g) : 0; }
  // VMEM instructions of this wave issued after step g's DMA (at the top of step g - kDist): the
  // DMAs of the steps still allowed in flight plus, when saving, the activation stores of steps
  // g - kDist .. g - 1 (and the prologue's e / x stores while g < kDist).  Exact, so the wait at
  // the top of step g never drains a store.
  __host__ __device__ static constexpr int younger(int g) {
    int s = 0;
    for (int i = g + 1; i < g + kDist && i < kBfSteps; ++i) s += n_glds(i);
    if (SAVE) {
      for (int i = g - kDist < 0 ? 0 : g - kDist; i < g; ++i) s += fwd_stores(i);
      if (g < kDist) s += kFwdPrologueStores;
    }
    return s;
  }
  __host__ __device__ static constexpr int64_t main_off(int g) {
    return g <= 27 ? (int64_t)g * kMainH : 27LL * kMainH + (int64_t)(g - 27) * 4096;
  }
};
static_assert(BfGeo<2, true>::kLds <= 160 * 1024, "LDS budget");
static_assert(BfGeo<1, true>::kLds <= 160 * 1024, "LDS budget");
static_assert(BfGeo<2, true>::younger(0) + BfGeo<2, true>::n_glds(0) < 64, "vmcnt range");
static_assert(BfGeo<2, true, true>::younger(2) < 64 && BfGeo<2, true, true>::younger(3) < 64, "vmcnt range");

struct BfFwdArgs {
  const char* wmain;   // main 16-bit image of the precision
  const char* raw;     // raw float table (8 KiB)
  const char* wfc;     // fc 16-bit image or null
  const char* fcraw;   // fc raw table (8 KiB) or null
  PointSrc src;
  int64_t P;
  float* raw_out;
  SaveArgs save;
  const float* c;      // (rows, 32) features of the launch's points
};

// Per-wave register state of the forward.
template <int PR>
struct BfState {
  using V8 = typename Prec<PR>::V8;
  static constexpr int NP = Prec<PR>::NP;
  f32x16 acc[2][8];    // h_L lives in set L & 1 (layer outputs alternate between the two sets)
  f32x16 out;
  V8 cur[NP][2];       // B operand of the current input tile ([part][k-step])
  V8 nxt[NP][2];       // the next input tile, being built by the epilogue pieces
  V8 ft[3][NP][2];     // Fourier tiles
  V8 ct[NP][2];        // feature tile
  float v[16];         // epilogue values of the tile being converted
  f32x16 f;            // feature-branch product of that tile
  uint32_t mw[4];      // ReLU bit words of the layer being converted
  int64_t col, mask_word0;
  bool valid, inside;
};

// values 4q..4q+3 of a tile = k-step q>>1, elements 4(q&1)..4(q&1)+3
template <int PR, typename T>
__device__ __forceinline__ void split_quad(const float* v4, int q, T (&t)[Prec<PR>::NP][2]) {
  using E = typename Prec<PR>::E;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = v4[i];
    const E h = (E)x;
    t[0][q >> 1][4 * (q & 1) + i] = h;
    if (Prec<PR>::NP == 2) t[Prec<PR>::NP - 1][q >> 1][4 * (q & 1) + i] = (E)(x - (float)h);
  }
}

template <int PR, typename T>
__device__ __forceinline__ void split_tile(const float (&v)[16], T (&t)[Prec<PR>::NP][2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) split_quad<PR>(v + 4 * q, q, t);
}

// A fragments of one 32-row output tile over one 32-deep input tile: [part][k-step]
template <int PR>
struct Frag {
  typename Prec<PR>::V8 a[Prec<PR>::NP][2];
};

template <int PR, int NS = 2>
__device__ __forceinline__ void load_frag(const char* base, Frag<PR>& f) {
  using V8 = typename Prec<PR>::V8;
  constexpr int NP = Prec<PR>::NP;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int s = 0; s < NS; ++s)
#pragma unroll
    for (int pt = 0; pt < NP; ++pt) f.a[pt][s] = *reinterpret_cast<const V8*>(base + (s * NP + pt) * 1024 + lane * 16);
}

// acc (+)= A . act over one 32-deep input tile: per k-step Al.xh + Ah.xl + Ah.xh (split) or Ah.xh.
// ZERO: the accumulator starts at 0 (first input tile of a layer)
template <int PR, bool ZERO, typename T, int NS = 2>
__device__ __forceinline__ void mfma_frag(const Frag<PR>& F, const T (&act)[Prec<PR>::NP][2], f32x16& acc) {
  f32x16 c = acc;
  if (ZERO) {
#pragma unroll
    for (int r = 0; r < 16; ++r) c[r] = 0.f;
  }
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    if (Prec<PR>::NP == 2) {
      c = Prec<PR>::mfma(F.a[1][s], act[0][s], c);
      c = Prec<PR>::mfma(F.a[0][s], act[1][s], c);
    }
    c = Prec<PR>::mfma(F.a[0][s], act[0][s], c);
  }
  acc = c;
}

template <int PR, bool HASC, bool SAVE>
struct BfFwd {
  static constexpr int NP = Prec<PR>::NP;
  static constexpr bool F16 = Prec<PR>::F16;
  using G = BfGeo<NP, HASC, SAVE>;
  using V8 = typename Prec<PR>::V8;
  using St = BfState<PR>;

  // issue the DMA of step g into its ring slot (wave-uniform, lane-linear 4 KiB pieces)
  template <int g>
  static __device__ __forceinline__ void stage_step(const BfFwdArgs& a, const char* lds) {
    if constexpr (g < kBfSteps) {
      const int w = wave_id(), lane = threadIdx.x & 63;
      const uint32_t slot = lds_addr(reinterpret_cast<const float*>(lds + (g % G::kNbuf) * G::kSlot)) + w * 1024;
      const char* src = a.wmain + G::main_off(g) + w * 1024 + lane * 16;
#pragma unroll
      for (int i = 0; i < G::main_n(g); ++i)
        glds16(reinterpret_cast<const float*>(src + i * 4096), slot + i * 4096);
      if constexpr (G::fc_n(g) > 0)
        glds16(reinterpret_cast<const float*>(a.wfc + (int64_t)(g - 2) * 4096 + w * 1024 + lane * 16),
               slot + G::kMainH);
    }
  }

  static __device__ __forceinline__ const float* raw_lds(const char* lds) {
    return reinterpret_cast<const float*>(lds + G::kNbuf * G::kSlot);
  }

  // Epilogue of h_L tile t (src = its accumulator), in pieces spread over a step's MFMA groups:
  //   phase 1, quad q: v = relu(acc + b) for units 4q..4q+3 of the lane (+ ReLU mask bits)
  //   phase 2, quad q: feature branch v += f + bc, activation save, 16-bit split into S.nxt
  template <int L, int t, int q>
  static __device__ __forceinline__ void conv1(const BfFwdArgs& a, St& S, const f32x16& src, const char* lds) {
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    const float* rawl = raw_lds(lds);
    const float4 b = *reinterpret_cast<const float4*>(rawl + kRawB + L * 256 + 32 * t + 8 * q + 4 * hh);
    const float b4[4] = {b.x, b.y, b.z, b.w};
    const float inv = F16 ? rawl[kRawInv + L] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = (F16 ? src[4 * q + i] * inv : src[4 * q + i]) + b4[i];
      S.v[4 * q + i] = x > 0.f ? x : 0.f;
    }
    if constexpr (SAVE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) S.mw[t >> 1] |= (S.v[4 * q + i] > 0.f ? 1u : 0u) << ((t & 1) * 16 + 4 * q + i);
      if (t == 7 && q == 3) {
        a.save.masks[(int64_t)L * (a.save.ld / 32) * 64 + S.mask_word0 + lane] =
            make_uint4(S.mw[0], S.mw[1], S.mw[2], S.mw[3]);
        S.mw[0] = S.mw[1] = S.mw[2] = S.mw[3] = 0u;
      }
    }
  }
  template <int L, int t, int q>
  static __device__ __forceinline__ void conv2(const BfFwdArgs& a, St& S, const char* lds) {
    const int lane = threadIdx.x & 63, hh = lane >> 5;
    if constexpr (HASC) {
      const float* fr = raw_lds(lds) + kRawBytes / 4;
      const float4 b = *reinterpret_cast<const float4*>(fr + L * 256 + 32 * t + 8 * q + 4 * hh);
      const float b4[4] = {b.x, b.y, b.z, b.w};
      const float inv = F16 ? fr[kFcRawInv + L] : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) S.v[4 * q + i] += (F16 ? S.f[4 * q + i] * inv : S.f[4 * q + i]) + b4[i];
    }
    if constexpr (SAVE)
      *reinterpret_cast<float4*>(a.save.hP + ((int64_t)L * a.save.ld + S.col) * kHidden + 32 * t + 8 * q + 4 * hh) =
          make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]);
    split_quad<PR>(S.v + 4 * q, q, S.nxt);
  }

  // epilogue pieces scheduled after MFMA group T of a step with NT groups
  template <int L, int t, int SET, int SHIFT, int NT, int T>
  static __device__ __forceinline__ void conv_pieces(const BfFwdArgs& a, St& S, const char* lds) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t1 = (q + SHIFT) < NT - 1 ? (q + SHIFT) : NT - 1;
      if (t1 == T) {
        if (q == 0) conv1<L, t, 0>(a, S, S.acc[SET][t], lds);
        if (q == 1) conv1<L, t, 1>(a, S, S.acc[SET][t], lds);
        if (q == 2) conv1<L, t, 2>(a, S, S.acc[SET][t], lds);
        if (q == 3) conv1<L, t, 3>(a, S, S.acc[SET][t], lds);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t2 = (4 + q) < NT - 1 ? (4 + q) : NT - 1;
      if (t2 == T) {
        if (q == 0) conv2<L, t, 0>(a, S, lds);
        if (q == 1) conv2<L, t, 1>(a, S, lds);
        if (q == 2) conv2<L, t, 2>(a, S, lds);
        if (q == 3) conv2<L, t, 3>(a, S, lds);
      }
    }
  }

  // MFMA group T of a step (prefetching the fragments of group T+2), then its epilogue pieces
  template <int NT, int T, int OUTSET, bool ZERO, bool CONV, int CL, int CT, int SET, int SHIFT>
  static __device__ __forceinline__ void group(const BfFwdArgs& a, St& S, const char* lds, const char* slot,
                                               const V8 (&act)[NP][2], Frag<PR> (&F)[3], const Frag<PR>& FC) {
    if constexpr (T < NT) {
      if constexpr (T + 2 < NT) load_frag<PR>(slot + (T + 2) * 2 * NP * 1024, F[(T + 2) % 3]);
      if constexpr (NT == 1) mfma_frag<PR, false>(F[0], act, S.out);
      else mfma_frag<PR, ZERO>(F[T % 3], act, S.acc[OUTSET][T]);
      if constexpr (HASC && CONV && T == 0) mfma_frag<PR, true>(FC, S.ct, S.f);
      if constexpr (CONV) conv_pieces<CL, CT, SET, SHIFT, NT, T>(a, S, lds);
      __builtin_amdgcn_sched_barrier(0);
      group<NT, T + 1, OUTSET, ZERO, CONV, CL, CT, SET, SHIFT>(a, S, lds, slot, act, F, FC);
    }
  }

  template <int g>
  static __device__ __forceinline__ void step(const BfFwdArgs& a, St& S, const char* lds) {
    if constexpr (g < kBfSteps) {
      constexpr int layer = fwd_layer(g);
      constexpr int kc = fwd_kc(g);
      constexpr int NT = layer == 4 ? 1 : 8;
      constexpr int OUTSET = layer & 1;                      // h_layer -> acc[layer & 1]
      constexpr bool ZERO = kc == 0 && layer <= 3;
      // epilogue job of this step: h_CL tile CT (tile 0 of a layer is built in its last step)
      constexpr bool CONV = fwd_conv(g);
      constexpr int CL = layer == 0 ? 0 : (layer == 4 ? 3 : (kc < 7 ? layer - 1 : layer));
      constexpr int CT = fwd_ct(g);
      constexpr int SET = CL & 1;
      constexpr int SHIFT = CT == 0 ? 1 : 0;  // that tile is produced by group 0 of this step
      sync_chunk<G::younger(g)>();
      stage_step<g + G::kDist>(a, lds);
      const char* slot = lds + (g % G::kNbuf) * G::kSlot;
      Frag<PR> F[3], FC;
      load_frag<PR>(slot, F[0]);
      if constexpr (NT > 1) load_frag<PR>(slot + 2 * NP * 1024, F[1]);
      if constexpr (HASC && CONV) load_frag<PR>(slot + G::kMainH, FC);
      if constexpr (layer == 0) {
        group<NT, 0, OUTSET, ZERO, CONV, CL, CT, SET, SHIFT>(a, S, lds, slot, S.ft[kc], F, FC);
      } else {
#pragma unroll
        for (int pt = 0; pt < NP; ++pt)
#pragma unroll
          for (int s = 0; s < 2; ++s) S.cur[pt][s] = S.nxt[pt][s];
        group<NT, 0, OUTSET, ZERO, CONV, CL, CT, SET, SHIFT>(a, S, lds, slot, S.cur, F, FC);
      }
      step<g + 1>(a, S, lds);
    }
  }

  template <int g>
  static __device__ __forceinline__ void prologue(const BfFwdArgs& a, const char* lds) {
    if constexpr (g < G::kDist) {
      stage_step<g>(a, lds);
      prologue<g + 1>(a, lds);
    }
  }
};

template <int PR, bool HASC, bool SAVE>
__global__ __launch_bounds__(256, 1) void k_mlp_fwd16(BfFwdArgs a, int mode) {
  using K = BfFwd<PR, HASC, SAVE>;
  using G = typename K::G;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = (int64_t)blockIdx.x * 128 + wave * 32 + j;

  // raw tables (biases, Fourier B, scales; + fc raw) then the first kDist steps, all by LDS-DMA
  {
    const int w = wave_id();
    const uint32_t rbase = lds_addr(K::raw_lds(lds)) + w * 1024;
#pragma unroll
    for (int i = 0; i < (int)(kRawBytes / 4096); ++i)
      glds16(reinterpret_cast<const float*>(a.raw + i * 4096 + w * 1024 + lane * 16), rbase + i * 4096);
    if (HASC) {
#pragma unroll
      for (int i = 0; i < (int)(kFcRawBytes / 4096); ++i)
        glds16(reinterpret_cast<const float*>(a.fcraw + i * 4096 + w * 1024 + lane * 16),
               rbase + kRawBytes + i * 4096);
    }
  }
  K::template prologue<0>(a, lds);

  BfState<PR> S;
  S.valid = p < a.P;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool inside = false;
  if (S.valid) {  // wave-uniform switch on the point source (one load per lane)
    switch (mode) {
      case kPtsF64: load_point<kPtsF64>(a.src, p, x0, x1, x2, inside); break;
      case kPtsF32: load_point<kPtsF32>(a.src, p, x0, x1, x2, inside); break;
      case kRaysZ64: load_point<kRaysZ64>(a.src, p, x0, x1, x2, inside); break;
      default: load_point<kRaysZ32>(a.src, p, x0, x1, x2, inside); break;
    }
  }
  S.inside = inside;
  S.col = a.save.p0 + p;
  S.mask_word0 = ((a.save.p0 + (int64_t)blockIdx.x * 128) / 32 + wave_id()) * 64;
  S.mw[0] = S.mw[1] = S.mw[2] = S.mw[3] = 0u;
  if (HASC) {
    float cv[16];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int jq = 0; jq < 2; ++jq) {
        float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
        if (S.valid) v = *reinterpret_cast<const float4*>(a.c + p * kCDim + 16 * s + 8 * jq + 4 * hh);
        cv[8 * s + 4 * jq + 0] = v.x; cv[8 * s + 4 * jq + 1] = v.y;
        cv[8 * s + 4 * jq + 2] = v.z; cv[8 * s + 4 * jq + 3] = v.w;
      }
    split_tile<PR>(cv, S.ct);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) S.out[r] = 0.f;

  // Fourier features: the raw tables must have landed (they are older than the step DMAs)
  sync_chunk<G::younger(0) + G::n_glds(0)>();
  {
    const float* FB = K::raw_lds(lds) + kRawFB;
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int k = 32 * t + perm(r, hh);
        float arg;
        {
#pragma clang fp contract(off)
          arg = x0 * FB[k];
          arg = __builtin_fmaf(x1, FB[kFourierPad + k], arg);
          arg = __builtin_fmaf(x2, FB[2 * kFourierPad + k], arg);
        }
        v[r] = k < kFourier ? sinf(arg) : 0.f;
      }
      if constexpr (SAVE) {
        float* row = a.save.eP + S.col * kFourierPad + 32 * t + 4 * hh;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          *reinterpret_cast<float4*>(row + 8 * q) = make_float4(v[4 * q], v[4 * q + 1], v[4 * q + 2], v[4 * q + 3]);
      }
      split_tile<PR>(v, S.ft[t]);
    }
    if (SAVE && hh == 0) a.save.xP[S.col] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
  }
  K::template step<0>(a, S, lds);

  if (S.valid && hh == 0) {
    const float* rawl = K::raw_lds(lds);
    const float* bo = rawl + kRawBo;
    const float inv = Prec<PR>::F16 ? rawl[kRawInv + 4] : 1.f;
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (Prec<PR>::F16 ? S.out[i] * inv : S.out[i]) + bo[i];
    reinterpret_cast<float4*>(a.raw_out)[p] = make_float4(o[0], o[1], o[2], S.inside ? o[3] : 100.f);
  }
}

// per-precision launchers (mlp16_fwd_*.hip), dispatched by launch_mlp_fwd_bf (mlp16_pack.hip)
int launch_fwd16_f16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, bool save);
int launch_fwd16_bf16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, bool save);
int launch_fwd16_bf16(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, bool save);

template <int PR, bool HASC, bool SAVE>
static int launch16s(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a) {
  const size_t lds = BfGeo<Prec<PR>::NP, HASC>::kLds;
  auto kern = k_mlp_fwd16<PR, HASC, SAVE>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, a, mode);
  return hip_status(hipGetLastError());
}
template <int PR>
static int launch16(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, bool save) {
  if (hasc) return save ? launch16s<PR, true, true>(mode, grid, st, a) : launch16s<PR, true, false>(mode, grid, st, a);
  return save ? launch16s<PR, false, true>(mode, grid, st, a) : launch16s<PR, false, false>(mode, grid, st, a);
}

}  // namespace pnr
