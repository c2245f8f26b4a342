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
// Training saves (SAVE) are fp32 in every precision: the weight-gradient GEMMs (wgrad16.hip) split
// them into hi/lo f16 parts themselves, so the backward stays fp32-class.  x and h1..h4 are saved;
// the Fourier features e = sin(x@B) are recomputed by the dW0 GEMM from x.  Every value the forward
// splits into f16 parts (hidden activations, features) is checked against the f16 range: a value
// >= 65504 would turn into inf; the kernel then ORs PNR_STATUS_F16_RANGE into *status (when given).
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
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

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
// then Wo [4][256] fp32: the VALU output layer of the kernels without the feature branch (one
// more 4 KiB piece, loaded only by them: the feature-branch variant has no LDS left for it)
constexpr int kRawWo = 2048;
constexpr int64_t kRawWoBytes = 4096;
constexpr int64_t kRawPackedBytes = kRawBytes + kRawWoBytes;
// hidden steps (layer 0 + the three 256-wide layers); the feature-branch kernels add 8 output steps
constexpr int kHidSteps = 27;
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
constexpr int64_t kPackedFloatsAll = kOffRaw + kRawPackedBytes / 4;
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
constexpr int kFwdPrologueStores = 1;  // x (e is not saved: kWgradFirstX recomputes it)

template <int NP, bool HASC, bool SAVE = false>
struct BfGeo {
  static constexpr int kMainH = NP * 16384;                  // bytes of a hidden main piece
  static constexpr int kSlot = kMainH + (HASC ? 4096 : 0);   // LDS slot bytes
  static constexpr int kNbuf = NP == 2 ? 4 : 6;
  static constexpr int kDist = kNbuf - 1;                    // steps in flight
  static constexpr int kRawLds = kRawBytes + (HASC ? kFcRawBytes : kRawWoBytes);
  static constexpr int kLds = kNbuf * kSlot + kRawLds;
  // steps of the DMA / MFMA program: without the feature branch the output layer runs on the VALU
  // after the hidden steps (BfFwd::out_layer)
  static constexpr int kSteps = HASC ? kBfSteps : kHidSteps;
  __host__ __device__ static constexpr int main_n(int g) { return g < 27 ? kMainH / 4096 : 1; }
  __host__ __device__ static constexpr int fc_n(int g) { return (HASC && g >= 2 && g <= 33) ? 1 : 0; }
  __host__ __device__ static constexpr int n_glds(int g) { return g < kSteps ? main_n(g) + fc_n(g) : 0; }
  __host__ __device__ static constexpr int64_t main_off(int g) {
    return g <= 27 ? (int64_t)g * kMainH : 27LL * kMainH + (int64_t)(g - 27) * 4096;
  }
};
static_assert(BfGeo<2, true>::kLds <= 160 * 1024, "LDS budget");
static_assert(BfGeo<1, true>::kLds <= 160 * 1024, "LDS budget");

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
  uint32_t* status;    // PNR_STATUS_* bits (f16 range) or null
};

// A fragments of one 32-row output tile over one 32-deep input tile: [part][k-step]
template <int PR>
struct Frag {
  typename Prec<PR>::V8 a[Prec<PR>::NP][2];
};

// Fragment ring of the split kernels: R tiles, prefetched R-1 MFMA groups ahead (LDS read latency
// under four streaming waves is ~300 cycles: 2 groups of lead left MFMAs waiting).  The feature
// + save variant keeps R = 3 (R = 4 spills there).

// Per-wave register state of the forward.
template <int PR, int R>
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
  float4 bq[4];        // bias quads of that tile (read from LDS at the top of the step)
  float4 bcq[4];       // fc bias quads (features)
  float inv, finv;     // f16 weight scales of the layer / fc branch (finv: times cinv)
  float cinv;          // 1 / s_c: the wave's feature tile is split as c s_c (f16x3; wave-uniform)
  uint32_t mw[4];      // ReLU bit words of the layer being converted
  Frag<PR> F[R];       // fragment ring (one 32-row output tile of the current / next step each)
  Frag<PR> FC;         // feature-branch fragments of the step's epilogue tile
  float vmax;          // max |value| split into f16 parts so far (f16 range check)
  int sb;              // ring slot of step 0 of this tile (persistent kernels: the ring runs on)
#if defined(PNR_EXP_TIMELINE)
  bool tick;
#endif
  int64_t col, mask_word0;
  bool valid, inside;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// 8 values times s split into f16 hi / lo operands (packed pairs, dev_common.h split2)
__device__ __forceinline__ void split8(const float* x, float s, f16x8& hi, f16x8& lo) {
  uint32_t h[4], l[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) split2(x[2 * j] * s, x[2 * j + 1] * s, h[j], l[j]);
  hi = __builtin_bit_cast(f16x8, u32x4{h[0], h[1], h[2], h[3]});
  lo = __builtin_bit_cast(f16x8, u32x4{l[0], l[1], l[2], l[3]});
}

// values 4q..4q+3 of a tile = k-step q>>1, elements 4(q&1)..4(q&1)+3
// PK: the packed f16 split (the feature-branch kernels, at their register limit, keep the scalar form:
// the packed one's extra live registers spill there)
template <int PR, typename T, bool PK = true>
__device__ __forceinline__ void split_quad(const float* v4, int q, T (&t)[Prec<PR>::NP][2]) {
  using E = typename Prec<PR>::E;
  if constexpr (Prec<PR>::F16 && PK) {
    // f16x3: packed pairs (dev_common.h split2: 6 VALU per quad where the scalar form took ~16),
    // dwords 2(q&1), 2(q&1)+1 of the k-step's operand
    uint32_t h0, l0, h1, l1;
    split2(v4[0], v4[1], h0, l0);
    split2(v4[2], v4[3], h1, l1);
    u32x4 hv = __builtin_bit_cast(u32x4, t[0][q >> 1]);
    u32x4 lv = __builtin_bit_cast(u32x4, t[1][q >> 1]);
    hv[2 * (q & 1)] = h0;
    hv[2 * (q & 1) + 1] = h1;
    lv[2 * (q & 1)] = l0;
    lv[2 * (q & 1) + 1] = l1;
    t[0][q >> 1] = __builtin_bit_cast(T, hv);
    t[1][q >> 1] = __builtin_bit_cast(T, lv);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float x = v4[i];
    const E h = (E)x;
    t[0][q >> 1][4 * (q & 1) + i] = h;
    if constexpr (Prec<PR>::NP == 2) t[1][q >> 1][4 * (q & 1) + i] = (E)(x - (float)h);
  }
}

template <int PR, typename T, bool PK = true>
__device__ __forceinline__ void split_tile(const float (&v)[16], T (&t)[Prec<PR>::NP][2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) split_quad<PR, T, PK>(v + 4 * q, q, t);
}


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
    if constexpr (Prec<PR>::NP == 2) {
      c = Prec<PR>::mfma(F.a[1][s], act[0][s], c);
      c = Prec<PR>::mfma(F.a[0][s], act[1][s], c);
    }
    c = Prec<PR>::mfma(F.a[0][s], act[0][s], c);
  }
  acc = c;
}

#if defined(PNR_EXP_TIMELINE)
// experiment: s_memtime timeline of one steady-state tile (S.tick: workgroup 7, its 6th tile;
// wave 0 .. 3, lane 0)
extern __device__ unsigned long long g_pnr_dbg[4][48];
#define PNR_TICK(i)                                                                     \
  do {                                                                                  \
    if (S.tick && (threadIdx.x & 63) == 0)                                              \
      g_pnr_dbg[threadIdx.x >> 6][(i)] = __builtin_amdgcn_s_memtime();                  \
  } while (0)
#else
#define PNR_TICK(i) \
  do {              \
  } while (0)
#endif

// SV: 0 no saves (eval), 1 masks + inputs + activations (training), 2 masks + inputs only (a
// backward with no weight gradients: the Tracker's camera-only step; PNR_PREC_F16X3 only)
template <int PR, bool HASC, int SV>
struct BfFwd {
  static constexpr bool SAVE = SV != 0;   // ReLU masks + inputs
  static constexpr bool SAVEH = SV == 1;  // + h1..h4
  static constexpr int NP = Prec<PR>::NP;
  static constexpr bool F16 = Prec<PR>::F16;
  using G = BfGeo<NP, HASC, SV != 0>;
  using V8 = typename Prec<PR>::V8;
  static constexpr int kRing = (HASC && SAVE) ? 3 : 4, kPf = kRing - 1;
  // group of a step with nt groups that runs epilogue piece q: phase 1 (conv1) and phase 2 (conv2,
  // the activation save).  The training kernel without the feature branch alternates the phases,
  // one save every other MFMA group (the save stream spread over the step, as in k_mlp_bwd16);
  // otherwise phase 1 runs in groups SHIFT..3+SHIFT and phase 2 in 4..7 (the feature branch's
  // product lands in group 3)
  static constexpr bool ALT = !HASC && SAVEH;
  __host__ __device__ static constexpr int grp1(int q, int shift, int n) {
    const int t = ALT ? 2 * q + shift : q + shift;
    return t < n - 1 ? t : n - 1;
  }
  __host__ __device__ static constexpr int grp2(int q, int shift, int n) {
    const int t = ALT ? 2 * q + 1 + shift : 4 + q;
    return t < n - 1 ? t : n - 1;
  }
  using St = BfState<PR, kRing>;
  // Persistent kernels (no feature branch): a workgroup loops over 128-point tiles and the weight
  // stream runs on across tiles -- the last steps of tile i prefetch the first steps of tile i+1
  // into the ring, so no tile waits for its first weights (the non-persistent kernel paid the
  // DMA latency in every workgroup's first three steps: ~4k cycles each against ~2.7k).  Step g of
  // tile i sits in ring slot (g + sb) % kNbuf, sb = i kSteps % kNbuf (continuous numbering).
  static constexpr bool PST = !HASC;

  // issue the DMA of step g into its ring slot (wave-uniform, lane-linear 4 KiB pieces); in the
  // persistent kernels steps g >= kSteps are the next tile's steps g - kSteps
  template <int g>
  static __device__ __forceinline__ void stage_step(const BfFwdArgs& a, const char* lds, int sb) {
    if constexpr (g < G::kSteps || (PST && g < 2 * G::kSteps)) {
      constexpr int st = g < G::kSteps ? g : g - G::kSteps;
      const int w = wave_id(), lane = threadIdx.x & 63;
      const uint32_t slot =
          lds_addr(reinterpret_cast<const float*>(lds + ((g + sb) % G::kNbuf) * G::kSlot)) + w * 1024;
      const uint32_t voff = lane * 16;
      const char* src = a.wmain + G::main_off(st) + w * 1024;  // wave-uniform (SGPRs)
      if constexpr (G::main_n(st) == 8 && !HASC) {  // (the feature-branch kernels: no SGPRs to spare)
        glds16s_x8(src, voff, slot);
      } else {
#pragma unroll
        for (int i = 0; i < G::main_n(st); ++i) glds16s(src + i * 4096, voff, slot + i * 4096);
      }
      if constexpr (G::fc_n(st) > 0) glds16s(a.wfc + (int64_t)(st - 2) * 4096 + w * 1024, voff, slot + G::kMainH);
    }
  }

  // Spread DMA (eval kernel): the 8 pieces of a hidden step's DMA go out one per MFMA group -- pieces
  // 0..2 after the barrier in groups 5..7 of step g, pieces 3..7 in groups 0..4 of step g+1 -- instead
  // of a burst after the barrier.  Only VMEM ops of the eval kernel are these DMAs, and all 8 pieces
  // of DMA(i+1) are still issued before barrier B_i: the vmcnt counts stay those of the burst.
#if defined(PNR_EXP_DMA_SPREAD)
  static constexpr bool SPREAD = !HASC && SV == 0 && NP == 2;
#else
  static constexpr bool SPREAD = false;
#endif
  template <int g, int i>
  static __device__ __forceinline__ void stage_piece(const BfFwdArgs& a, const char* lds, int sb) {
    if constexpr (g < G::kSteps || (PST && g < 2 * G::kSteps)) {
      constexpr int st = g < G::kSteps ? g : g - G::kSteps;
      static_assert(G::main_n(st) == 8 && G::fc_n(st) == 0, "spread: hidden steps only");
      const int w = wave_id(), lane = threadIdx.x & 63;
      const uint32_t slot =
          lds_addr(reinterpret_cast<const float*>(lds + ((g + sb) % G::kNbuf) * G::kSlot)) + w * 1024;
      const char* src = a.wmain + G::main_off(st) + w * 1024;
      glds16s(src + i * 4096, lane * 16, slot + i * 4096);
    }
  }

  static __device__ __forceinline__ const float* raw_lds(const char* lds) {
    return reinterpret_cast<const float*>(lds + G::kNbuf * G::kSlot);
  }

  // Epilogue of h_L tile t (src = its accumulator), in pieces spread over a step's MFMA groups:
  //   phase 1, quad q: v = relu(acc + b) for units 4q..4q+3 of the lane (+ ReLU mask bits)
  //   phase 2, quad q: feature branch v += f + bc, activation save, 16-bit split into S.nxt
  // Epilogue constants of h_L tile t, read at the top of the step BEFORE the fragment prefetch:
  // LDS reads return in order, so a wait for a constant read later would drain the prefetch too.
  template <int L, int t>
  static __device__ __forceinline__ void preload(St& S, const char* lds) {
    const int hh = (threadIdx.x >> 5) & 1;
    const float* rawl = raw_lds(lds);
#pragma unroll
    for (int q = 0; q < 4; ++q) S.bq[q] = *reinterpret_cast<const float4*>(rawl + kRawB + L * 256 + 32 * t + 8 * q + 4 * hh);
    if (F16) S.inv = rawl[kRawInv + L];
  }
  // feature-branch bias quads of h_L tile t (read early in the step, before that group's fragment
  // prefetch, so their wait never drains it)
  template <int L, int t>
  static __device__ __forceinline__ void preload_fc(St& S, const char* lds) {
    const int hh = (threadIdx.x >> 5) & 1;
    const float* fr = raw_lds(lds) + kRawBytes / 4;
#pragma unroll
    for (int q = 0; q < 4; ++q) S.bcq[q] = *reinterpret_cast<const float4*>(fr + L * 256 + 32 * t + 8 * q + 4 * hh);
    if (F16) S.finv = fr[kFcRawInv + L] * S.cinv;
  }

  template <int L, int t, int q>
  static __device__ __forceinline__ void conv1(const BfFwdArgs& a, St& S, const f32x16& src, const char* lds) {
    const int lane = threadIdx.x & 63;
    const float4 b = S.bq[q];
    const float b4[4] = {b.x, b.y, b.z, b.w};
    const float inv = F16 ? S.inv : 1.f;
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
  // fp32 save address of this lane's unit quad (t, q) of h_L: point-major row S.col
  static __device__ __forceinline__ float* h_save(const BfFwdArgs& a, const St& S, int L, int t, int q) {
    const int lane = threadIdx.x & 63;
#if defined(PNR_EXP_LINSAVE)  // experiment: ideal store shape (1 KB contiguous per instruction), wrong layout
    return a.save.hP + ((int64_t)L * a.save.ld + S.col - (lane & 31)) * kHidden + (t * 4 + q) * 256 + lane * 4;
#else
    return a.save.hP + ((int64_t)L * a.save.ld + S.col) * kHidden + 32 * t + 8 * q + 4 * (lane >> 5);
#endif
  }
  template <int L, int t, int q>
  static __device__ __forceinline__ void conv2(const BfFwdArgs& a, St& S, const char* lds) {
    if constexpr (HASC) {
      const float4 b = S.bcq[q];
      const float b4[4] = {b.x, b.y, b.z, b.w};
      const float inv = F16 ? S.finv : 1.f;
#pragma unroll
      for (int i = 0; i < 4; ++i) S.v[4 * q + i] += (F16 ? S.f[4 * q + i] * inv : S.f[4 * q + i]) + b4[i];
    }
#if !defined(PNR_EXP_NOSTORE)
    if constexpr (SAVEH)  // fp32 activation save (pnr_internal.h SaveArgs)
#else
    if constexpr (false)
#endif
      save16(h_save(a, S, L, t, q), make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]));
    S.vmax = fmaxf(S.vmax, fmaxf(fmaxf(fabsf(S.v[4 * q]), fabsf(S.v[4 * q + 1])),
                                 fmaxf(fabsf(S.v[4 * q + 2]), fabsf(S.v[4 * q + 3]))));
    split_quad<PR, V8, !HASC>(S.v + 4 * q, q, S.nxt);
  }

  // epilogue pieces scheduled after MFMA group T of a step with NT groups
  template <int L, int t, int SET, int SHIFT, int NT, int T>
  static __device__ __forceinline__ void conv_pieces(const BfFwdArgs& a, St& S, const char* lds) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (grp1(q, SHIFT, NT) == T) {
        if (q == 0) conv1<L, t, 0>(a, S, S.acc[SET][t], lds);
        if (q == 1) conv1<L, t, 1>(a, S, S.acc[SET][t], lds);
        if (q == 2) conv1<L, t, 2>(a, S, S.acc[SET][t], lds);
        if (q == 3) conv1<L, t, 3>(a, S, S.acc[SET][t], lds);
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (grp2(q, SHIFT, NT) == T) {
        if (q == 0) conv2<L, t, 0>(a, S, lds);
        if (q == 1) conv2<L, t, 1>(a, S, lds);
        if (q == 2) conv2<L, t, 2>(a, S, lds);
        if (q == 3) conv2<L, t, 3>(a, S, lds);
      }
    }
  }

  // ---- step pipeline ------------------------------------------------------------------------
  // Step g runs NT(g) MFMA groups (one per output tile).  The wait + barrier that make step g+1's
  // ring slot valid sit after group SYNC_T(g) of step g, followed by the DMA of step g+1+kD into the
  // slot step g-1 used; the next step's first two fragment tiles and epilogue constants are then
  // read during step g's last groups, so no step starts with an LDS round trip or a barrier.
  static constexpr int kD = G::kNbuf - 2;  // DMA distance (steps)
  __host__ __device__ static constexpr int nt(int g) { return fwd_layer(g) == 4 ? 1 : 8; }
  __host__ __device__ static constexpr int sync_t(int g) { return nt(g) == 1 ? 0 : 5; }
  __host__ __device__ static constexpr int ring(int g) {
    int b = 0;
    for (int i = 0; i < g; ++i) b += nt(i);
    return b % kRing;
  }
  // group of step g that issues the read of the next step's fragment tile k (after the barrier)
  __host__ __device__ static constexpr int next_grp(int g, int k) {
    const int t = nt(g) - kPf + k;
    const int u = t > sync_t(g) ? t : sync_t(g);
    return u < nt(g) - 1 ? u : nt(g) - 1;
  }
  __host__ __device__ static constexpr int shift(int g) { return fwd_ct(g) == 0 ? 1 : 0; }
  __host__ __device__ static constexpr int clamp_t(int t, int g) { return t < nt(g) - 1 ? t : nt(g) - 1; }
  // activation-save stores the epilogue pieces of step g issue in group T (SAVE)
  __host__ __device__ static constexpr int stores_grp(int g, int T) {
    if (!SAVE || !fwd_conv(g)) return 0;
    int n = 0;
#if !defined(PNR_EXP_NOSTORE)
    if (SAVEH)
      for (int q = 0; q < 4; ++q) n += grp2(q, shift(g), nt(g)) == T ? 1 : 0;
#endif
    if (fwd_ct(g) == 7 && grp1(3, shift(g), nt(g)) == T) ++n;  // the mask words (conv1, tile 7, q 3)
    return n;
  }
  __host__ __device__ static constexpr int stores_rng(int g, int t0, int t1) {  // groups [t0, t1]
    int n = 0;
    for (int T = t0; T <= t1; ++T) n += stores_grp(g, T);
    return n;
  }
  // VMEM ops issued after DMA(i) and before the wait of barrier B_i (i >= 1, in step i-1)
  __host__ __device__ static constexpr int younger_b(int i) {
    int n = 0;
    for (int j = i + 1; j <= i + kD - 1; ++j) n += j < G::kSteps ? G::n_glds(j) : (PST ? G::n_glds(j - G::kSteps) : 0);
    if (SAVE) {
      int first = 0;  // first step whose stores all follow the DMA
      if (i >= kD && i - kD >= 1) {
        const int p = i - kD;  // DMA(i) issued at B_p, after group sync_t(p-1) of step p-1
        n += stores_rng(p - 1, sync_t(p - 1) + 1, nt(p - 1) - 1);
        first = p;
      } else {
        if (i < kD) n += kFwdPrologueStores;  // DMA(i) issued in the prologue, before e / x saves
        first = 0;
      }
      for (int g = first; g <= i - 2; ++g) n += stores_rng(g, 0, nt(g) - 1);
      n += stores_rng(i - 1, 0, sync_t(i - 1));
    }
    return n;
  }
  __host__ __device__ static constexpr int younger_b0() {
    int n = 0;
    for (int j = 1; j < kD; ++j) n += G::n_glds(j);
    return n + (SAVE ? kFwdPrologueStores : 0);
  }

  static __device__ __forceinline__ const char* slot_of(const char* lds, int g, int sb) {
    return lds + ((g + sb) % G::kNbuf) * G::kSlot;
  }

  // next step's fragment tile k (issued after its barrier)
  template <int g, int k>
  static __device__ __forceinline__ void next_frag(St& S, const char* lds) {
    if constexpr (k < nt(g)) load_frag<PR>(slot_of(lds, g, S.sb) + k * 2 * NP * 1024, S.F[(ring(g) + k) % kRing]);
  }
  // next step's epilogue constants
  template <int g>
  static __device__ __forceinline__ void next_consts(St& S, const char* lds) {
    constexpr int layer = fwd_layer(g), kc = fwd_kc(g);
    constexpr int CL = layer == 0 ? 0 : (layer == 4 ? 3 : (kc < 7 ? layer - 1 : layer));
    if constexpr (fwd_conv(g)) preload<CL, fwd_ct(g)>(S, lds);
    (void)CL;
  }

  // MFMA group T of step g (prefetching the fragments of group T+2), its epilogue pieces, and the
  // next step's barrier / DMA / first loads where they fall
  template <int g, int T>
  static __device__ __forceinline__ void group(const BfFwdArgs& a, St& S, const char* lds, const V8 (&act)[NP][2]) {
    constexpr int NT = nt(g);
    if constexpr (T < NT) {
      constexpr int layer = fwd_layer(g);
      constexpr int kc = fwd_kc(g);
      constexpr int OUTSET = layer & 1;                      // h_layer -> acc[layer & 1]
      constexpr bool ZERO = kc == 0 && layer <= 3;
#if defined(PNR_EXP_NOCONV)
      constexpr bool CONV = false;  // experiment: no epilogue work
#else
      constexpr bool CONV = fwd_conv(g);
#endif
      // epilogue job of this step: h_CL tile CT (tile 0 of a layer is built in its last step)
      constexpr int CL = layer == 0 ? 0 : (layer == 4 ? 3 : (kc < 7 ? layer - 1 : layer));
      constexpr int CT = fwd_ct(g);
      constexpr int SET = CL & 1;
      constexpr int SHIFT = shift(g);  // that tile is produced by group 0 of this step
      constexpr int b = ring(g);
      const char* slot = slot_of(lds, g, S.sb);
      if constexpr (HASC && CONV && T == clamp_t(1, g)) load_frag<PR>(slot + G::kMainH, S.FC);
      if constexpr (HASC && CONV && T == clamp_t(3, g)) preload_fc<CL, CT>(S, lds);
      if constexpr (T + kPf < NT) load_frag<PR>(slot + (T + kPf) * 2 * NP * 1024, S.F[(b + T + kPf) % kRing]);
      if constexpr (SPREAD && g >= 1 && T < NT - sync_t(g) + 2 && T + 3 < 8) stage_piece<g + kD, T + 3>(a, lds, S.sb);
      __builtin_amdgcn_sched_barrier(0);  // prefetch first, then the group's MFMAs
      if constexpr (NT == 1) {
        if constexpr (kc == 0) mfma_frag<PR, true>(S.F[b], act, S.out);
        else mfma_frag<PR, false>(S.F[b], act, S.out);
      } else {
        mfma_frag<PR, ZERO>(S.F[(b + T) % kRing], act, S.acc[OUTSET][T]);
        // keep the accumulator in AGPRs: otherwise hipcc shuffles whole tiles between the register
        // files every step (measured: 114 v_accvgpr_read per step where the epilogue needs 16)
        asm volatile("" : "+a"(S.acc[OUTSET][T]));
      }
      // feature-branch product, one group before its consumers (conv2 from group 4 on)
      if constexpr (HASC && CONV && T == clamp_t(3, g)) mfma_frag<PR, true>(S.FC, S.ct, S.f);
      if constexpr (CONV) conv_pieces<CL, CT, SET, SHIFT, NT, T>(a, S, lds);
      if constexpr (g + 1 < G::kSteps) {
        if constexpr (T == sync_t(g)) {
          PNR_TICK(3 + g);
#if defined(PNR_EXP_NODMA)
          sync_chunk<0>();
#else
          sync_chunk<younger_b(g + 1)>();
          if constexpr (!SPREAD) stage_step<g + 1 + kD>(a, lds, S.sb);
#endif
        }
        if constexpr (SPREAD && T >= sync_t(g)) stage_piece<g + 1 + kD, T - sync_t(g)>(a, lds, S.sb);
        if constexpr (T == next_grp(g, 0)) next_frag<g + 1, 0>(S, lds);
        if constexpr (T == next_grp(g, 1)) next_frag<g + 1, 1>(S, lds);
        if constexpr (T == next_grp(g, 2)) next_frag<g + 1, 2>(S, lds);
        if constexpr (T == NT - 1) next_consts<g + 1>(S, lds);
      }
      __builtin_amdgcn_sched_barrier(0);
      group<g, T + 1>(a, S, lds, act);
    }
  }

  template <int g>
  static __device__ __forceinline__ void step(const BfFwdArgs& a, St& S, const char* lds) {
    if constexpr (g < G::kSteps) {
      // both accumulator sets live in the 256 AGPRs for the whole kernel; out / f stay in VGPRs.
      // Step 0 only DEFINES them ("=a"): read there, a persistent kernel's tiles would carry the
      // previous tile's registers around the loop (256 AGPRs live across its tail: spills)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          if constexpr (g == 0) asm volatile("" : "=a"(S.acc[st][t]));
          else asm volatile("" : "+a"(S.acc[st][t]));
        }
      if constexpr (fwd_layer(g) == 0) {
        group<g, 0>(a, S, lds, S.ft[fwd_kc(g)]);
      } else {
#pragma unroll
        for (int pt = 0; pt < NP; ++pt)
#pragma unroll
          for (int s = 0; s < 2; ++s) S.cur[pt][s] = S.nxt[pt][s];
        group<g, 0>(a, S, lds, S.cur);
      }
      step<g + 1>(a, S, lds);
    }
  }

  __host__ __device__ static constexpr int prologue_glds() {
    int n = 0;
    for (int j = 0; j < kD; ++j) n += G::n_glds(j);
    return n;
  }
  // prologue DMAs: steps 0 .. kD-1 (after the raw tables)
  template <int g>
  static __device__ __forceinline__ void prologue(const BfFwdArgs& a, const char* lds) {
    if constexpr (g < kD) {
      stage_step<g>(a, lds, 0);
      prologue<g + 1>(a, lds);
    }
  }
  // barrier B_0: step 0's slot is valid; DMA of step kD; step 0's first loads
  static __device__ __forceinline__ void start(const BfFwdArgs& a, St& S, const char* lds) {
    PNR_TICK(2);
#if defined(PNR_EXP_NODMA)
    sync_chunk<0>();
#else
    sync_chunk<younger_b0()>();
    stage_step<kD>(a, lds, S.sb);
#endif
    next_frag<0, 0>(S, lds);
    next_frag<0, 1>(S, lds);
    next_frag<0, 2>(S, lds);
    next_consts<0>(S, lds);
  }

  // ---- output layer on the VALU (no feature branch) ------------------------------------------
  // out[i] (+)= sum over this lane's 16 units of h4 tile t of Wo[i][u] h4[u] (fp32 FMAs; Wo fp32
  // in LDS after the main raw table).  Units of register r: 32 t + perm(r, hh).
  // wo: this lane's 32-bit LDS address of Wo (see out_layer)
  template <int t>
  static __device__ __forceinline__ void out_dot(const St& S, uint32_t wo, float (&o)[4]) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    using lds_f4 = const __attribute__((address_space(3))) v4f;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const v4f w = *reinterpret_cast<lds_f4*>((uintptr_t)(wo + 4 * (i * kHidden + 32 * t + 8 * q)));
        o[i] = __builtin_fmaf(w.x, S.v[4 * q + 0], o[i]);
        o[i] = __builtin_fmaf(w.y, S.v[4 * q + 1], o[i]);
        o[i] = __builtin_fmaf(w.z, S.v[4 * q + 2], o[i]);
        o[i] = __builtin_fmaf(w.w, S.v[4 * q + 3], o[i]);
      }
  }
  // h4 tile t: bias + ReLU (+ mask bits, f16 save), then its share of the output layer
  template <int t>
  static __device__ __forceinline__ void out_tile(const BfFwdArgs& a, St& S, const char* lds, uint32_t wo,
                                                  float (&o)[4]) {
    if constexpr (t < 8) {
      if constexpr (t > 0) {  // tile 0 was converted by the last hidden step (S.v holds it)
        preload<3, t>(S, lds);
        conv1<3, t, 0>(a, S, S.acc[1][t], lds);
        conv1<3, t, 1>(a, S, S.acc[1][t], lds);
        conv1<3, t, 2>(a, S, S.acc[1][t], lds);
        conv1<3, t, 3>(a, S, S.acc[1][t], lds);
#if !defined(PNR_EXP_NOSTORE)
        if constexpr (SAVEH) {
#else
        if constexpr (false) {
#endif
#pragma unroll
          for (int q = 0; q < 4; ++q)
            save16(h_save(a, S, 3, t, q), make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]));
        }
      }
      out_dot<t>(S, wo, o);
      out_tile<t + 1>(a, S, lds, wo, o);
    }
  }
  static __device__ __forceinline__ void out_layer(const BfFwdArgs& a, St& S, const char* lds, float (&o)[4]) {
    o[0] = o[1] = o[2] = o[3] = 0.f;
    // Wo lies above 64 KiB of LDS, past ds_read's 16-bit offset field: from a generic pointer every
    // read got its own address VGPR, which a persistent kernel hoists out of its tile loop (and
    // spills).  One opaque per-tile base, constant offsets folded into the instructions.
    uint32_t wo = lds_addr(raw_lds(lds) + kRawBytes / 4) + 16 * ((threadIdx.x >> 5) & 1);
    asm volatile("" : "+v"(wo));
    out_tile<0>(a, S, lds, wo, o);
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] += __shfl_xor(o[i], 32);  // the other lane half's 128 units
  }
};

// one 128-point tile of k_mlp_fwd16 (it: the workgroup's tile count so far, sb: its ring slot base)
template <int PR, bool HASC, int SV>
static __device__ __forceinline__ void fwd16_tile(const BfFwdArgs& a, int mode, const char* lds, int64_t tile,
                                                 int it, int sb) {
  using K = BfFwd<PR, HASC, SV>;
  constexpr bool SAVE = K::SAVE;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = tile * 128 + wave * 32 + j;
  typename K::St S;
  S.sb = sb;
#if defined(PNR_EXP_TIMELINE)
  S.tick = blockIdx.x == 7 && it == 5;
#endif
  PNR_TICK(0);
  S.valid = p < a.P;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool inside = false;
  if (S.valid) {  // wave-uniform switch on the point source (one load per lane)
    switch (mode) {
      case kPtsF64: load_point<kPtsF64>(a.src, p, x0, x1, x2, inside); break;
      case kPtsF32: load_point<kPtsF32>(a.src, p, x0, x1, x2, inside); break;
      case kRaysZ64: load_point<kRaysZ64>(a.src, p, x0, x1, x2, inside); break;
      case kPtsX4: load_point<kPtsX4>(a.src, p, x0, x1, x2, inside); break;
      default: load_point<kRaysZ32>(a.src, p, x0, x1, x2, inside); break;
    }
  }
  S.inside = inside;
  S.col = a.save.p0 + p;
  S.mask_word0 = ((a.save.p0 + tile * 128) / 32 + wave_id()) * 64;
  S.mw[0] = S.mw[1] = S.mw[2] = S.mw[3] = 0u;
  S.vmax = 0.f;
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
    // f16x3: the wave's feature tile is split as c s_c, s_c = 2^k putting the wave's max |c| in
    // [2^13, 2^14) (pt_scale), so the lo parts stay out of the f16 subnormals whatever the feature
    // magnitude (the reference's fine-grid features have std 1e-4); the fc product carries s_c and
    // finv = 2^-w / s_c undoes it exactly.  Wave-uniform (an SGPR): the training kernel with the
    // feature branch has no VGPR to spare for a per-point scale
    S.cinv = 1.f;
    if constexpr (Prec<PR>::F16) {
      float m = 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) m = fmaxf(m, fabsf(cv[r]));
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
      const float sc = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, pt_scale(m))));
#pragma unroll
      for (int r = 0; r < 16; ++r) cv[r] *= sc;
      S.cinv = 1.f / sc;
      // the scaled features are split into f16 parts too: pt_scale stops at 2^-100, so a feature
      // above ~2^114 would still overflow -- the range check covers them (PNR_STATUS_F16_RANGE)
      S.vmax = m * sc;
    }
    split_tile<PR, typename K::V8, false>(cv, S.ct);
  }
  // no accumulator zero fill: the first input tile of every layer starts its tiles from 0 (ZERO in
  // mfma_frag), and nothing reads a tile before that (256 v_accvgpr_mov saved per workgroup)

  // Fourier features: the raw tables must have landed (they are older than the step DMAs; later
  // tiles of a persistent workgroup read them long after)
  if (it == 0) sync_chunk<K::prologue_glds()>();
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
        v[r] = k < kFourier ? fourier_sc<false>(arg) : 0.f;
      }
      // no e save: the dW0 GEMM recomputes sin(x@B) from the saved x (wgrad16.hip kWgradFirstX)
      split_tile<PR, typename K::V8, !HASC>(v, S.ft[t]);
    }
    // always issued (the step program's vmcnt counts include it); in the map pass the kPtsX4 input
    // rows are this save, so the store rewrites the value the lane has just read
    if (SAVE && hh == 0) a.save.xP[S.col] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
  }
  PNR_TICK(1);
  static_assert(K::younger_b(1) < 64 && K::younger_b(2) < 64 && K::younger_b(3) < 64 && K::younger_b(20) < 64,
                "vmcnt range");
  K::start(a, S, lds);
  K::template step<0>(a, S, lds);
  float o[4];
  if constexpr (HASC) {  // output layer = the last 8 MFMA steps, scaled accumulator
    const float inv = Prec<PR>::F16 ? K::raw_lds(lds)[kRawInv + 4] : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = Prec<PR>::F16 ? S.out[i] * inv : S.out[i];
  } else {
    K::out_layer(a, S, lds, o);
  }
  PNR_TICK(40);
  // f16 range: a split value >= 65504 became inf (bf16 parts have the fp32 range)
  if (Prec<PR>::F16 && a.status != nullptr && !(S.vmax < 65504.f)) atomicOr(a.status, (uint32_t)PNR_STATUS_F16_RANGE);

  if (S.valid && hh == 0) {
    const float* bo = K::raw_lds(lds) + kRawBo;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] += bo[i];
    reinterpret_cast<float4*>(a.raw_out)[p] = make_float4(o[0], o[1], o[2], S.inside ? o[3] : 100.f);
  }
}

template <int PR, bool HASC, int SV>
__global__ __launch_bounds__(256, 1) void k_mlp_fwd16(BfFwdArgs a, int mode) {
  using K = BfFwd<PR, HASC, SV>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63;

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
    } else {  // Wo for the VALU output layer
      glds16(reinterpret_cast<const float*>(a.raw + kRawBytes + w * 1024 + lane * 16), rbase + kRawBytes);
    }
  }
  K::template prologue<0>(a, lds);
  // persistent kernels loop over tiles (grid <= CUs); the others run one tile per workgroup with no
  // loop at all (a loop, even one that runs once, costs the register allocator ~100 spills here)
  if constexpr (K::PST) {
    const int64_t ntiles = (a.P + 127) / 128;
    int sb = 0, it = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
      fwd16_tile<PR, HASC, SV>(a, mode, lds, tile, it, sb);
      sb = (sb + K::G::kSteps) % K::G::kNbuf;
    }
    // the last tile's prefetch of a next tile (always issued: fixed wait counts) must land in the
    // workgroup's LDS before it exits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    fwd16_tile<PR, HASC, SV>(a, mode, lds, blockIdx.x, 0, 0);
  }
}

// per-precision launchers (mlp16_fwd_*.hip), dispatched by launch_mlp_fwd_bf (mlp16_pack.hip)
int launch_fwd16_f16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save);
int launch_fwd16_bf16x3(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save);
int launch_fwd16_bf16(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save);

template <int PR, bool HASC, int SV>
static int launch16s(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a) {
  const size_t lds = BfGeo<Prec<PR>::NP, HASC>::kLds;
  auto kern = k_mlp_fwd16<PR, HASC, SV>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, grid, dim3(256), lds, st, a, mode);
  return hip_status(hipGetLastError());
}
template <int PR>
static int launch16(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, bool hasc, int save) {
  if (save == 2) {  // masks + inputs only: instantiated for the default precision (capi save_mode)
    if constexpr (PR == PNR_PREC_F16X3)
      return hasc ? launch16s<PR, true, 2>(mode, grid, st, a) : launch16s<PR, false, 2>(mode, grid, st, a);
    return PNR_E_ARG;
  }
  if (hasc) return save ? launch16s<PR, true, 1>(mode, grid, st, a) : launch16s<PR, true, 0>(mode, grid, st, a);
  return save ? launch16s<PR, false, 1>(mode, grid, st, a) : launch16s<PR, false, 0>(mode, grid, st, a);
}

}  // namespace pnr
