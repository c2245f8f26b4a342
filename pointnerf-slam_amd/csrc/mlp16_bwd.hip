// mlp16_bwd.hip -- f16x3 delta chain of the decoder backward (k_mlp_bwd16).
#include <cmath>

#include "mlp16.h"

namespace pnr {
// ---------------------------------------------------------------------------------------------
// Backward delta chain for every non-fp32 precision: the k_mlp_bwd math (mlp.hip) --
//   g_h4 = Wo^T g_out, delta_l = (W_l^T delta_{l+1}) * [h_l > 0], g_e = W0^T delta_1,
//   g_arg = g_e * cos(x@B), g_x = B g_arg; with features dL/dh_l is saved before the mask and
//   dL/dc = sum_l Wc_l^T dL/dh_l
// -- on the forward's machinery: chain c = 0 (Wo^T), 1..3 (W3^T..W1^T), 4 (W0^T) alternate between
// the two accumulator sets, each delta tile is built (mask, save, split) in pieces placed between
// the next chain's MFMA groups, weights stream through the same LDS-DMA ring.
//
// Arithmetic: f16x3 (x = hi + lo in f16, 22 significant bits; Wl xh + Wh xl + Wh xh with fp32
// accumulation), the forward's split.  Gradients span far more than the f16 exponent range, so each
// point's chain input is scaled by its own power of two s_p before the split: the MFMA output
// column p is W^T (delta_p s_p), and s_p (with the per-tensor weight scale 2^w of the image) is
// undone exactly on the fp32 accumulator.  s_p puts the point's max |delta| in [2^13, 2^14): every
// split operand is inside the f16 range and keeps 22 bits relative to its point's largest entry,
// whatever the loss scale.  At a chain boundary the point's max over all 8 output tiles is needed
// before tile 0 can be split, so a boundary step folds each finished tile into a running max
// (between the MFMA groups) and converts tile 0 after its last group.
// The deltas, dL/dh (features) and g_arg go to HBM in fp32 (point-major) for the weight-gradient
// GEMMs of wgrad16.hip, which split them again under their own scales.
// ---------------------------------------------------------------------------------------------
__host__ __device__ constexpr int bwd_chain(int g) { return g == 0 ? 0 : (g <= 24 ? 1 + (g - 1) / 8 : 4); }
__host__ __device__ constexpr int bwd_kc(int g) { return g == 0 ? 0 : (g <= 24 ? (g - 1) % 8 : g - 25); }
__host__ __device__ constexpr bool bwd_conv(int g) { return !(bwd_chain(g) == 4 && bwd_kc(g) == 7); }
__host__ __device__ constexpr int bwd_conv_chain(int g) {
  return g == 0 ? 0 : (bwd_kc(g) < 7 ? bwd_chain(g) - 1 : bwd_chain(g));
}
__host__ __device__ constexpr int bwd_conv_tile(int g) { return g == 0 ? 0 : (bwd_kc(g) < 7 ? bwd_kc(g) + 1 : 0); }

template <bool HASC>
struct BwdGeo {
  static constexpr int kSlot = 32768 + (HASC ? 4096 : 0);
  static constexpr int kNbuf = 4;
  static constexpr int kDist = kNbuf - 1;
  static constexpr int kLds = kNbuf * kSlot;
  __host__ __device__ static constexpr int main_n(int g) { return g == 0 ? 4 : (g <= 24 ? 8 : 3); }
  __host__ __device__ static constexpr int fc_n(int g) { return (HASC && g <= 31) ? 1 : 0; }
  __host__ __device__ static constexpr int n_glds(int g) { return g < kBwdSteps ? main_n(g) + fc_n(g) : 0; }
  // delta (+ dL/dh) quads stored in step g
  __host__ __device__ static constexpr int stores(int g) { return bwd_conv(g) ? (HASC ? 8 : 4) : 0; }
  __host__ __device__ static constexpr int younger(int g) {
    int s = 0;
    for (int i = g + 1; i < g + kDist && i < kBwdSteps; ++i) s += n_glds(i);
    for (int i = g - kDist < 0 ? 0 : g - kDist; i < g; ++i) s += stores(i);
    return s;
  }
};
static_assert(BwdGeo<true>::younger(4) < 64, "vmcnt range");

// max |a| over an accumulator tile.  The AGPRs are read from inline asm: written as plain reads,
// hipcc keeps VGPR copies of whole tiles alive and the feature-branch kernel spills.
__device__ __forceinline__ float tile_absmax(const f32x16& a) {
  float m = 0.f;
#pragma unroll
  for (int r = 0; r < 16; r += 2) {
    float x, y;
    asm volatile("v_accvgpr_read_b32 %0, %2\n\tv_accvgpr_read_b32 %1, %3"
                 : "=&v"(x), "=&v"(y)
                 : "a"(a[r]), "a"(a[r + 1]));
    m = fmaxf(m, fmaxf(fabsf(x), fabsf(y)));
  }
  return m;
}

struct BwdState {
  f32x16 acc[2][8];     // chain c output in set c & 1
  f32x16 gc;            // dL/dc (32 channels), times gcf
  f16x8 cur[2][2];
  f16x8 nxt[2][2];
  f16x8 tmp[2][2];      // split dL/dh tile (feature branch operand)
  float v[16];
  uint4 m[4];           // ReLU bit words of h1..h4 (this lane)
  float kacc;           // true value = acc * kacc for the chain accumulating now (2^-w / s_p)
  float kconv;          // the same for the chain being converted
  float sig;            // s_p of the chain being converted (its deltas enter the next chain times sig)
  float mx;             // running max |acc| over the finished tiles of a boundary step
  float gcf;            // gc = true dL/dc * gcf
  int64_t dcol;
};

template <bool HASC>
struct BfBwd {
  static constexpr int PR = PNR_PREC_F16X3;
  using G = BwdGeo<HASC>;

  template <int g>
  static __device__ __forceinline__ void stage_step(const BwdArgs& a, const char* wmain, const char* wfc,
                                                    const char* lds) {
    if constexpr (g < kBwdSteps) {
      const int w = wave_id(), lane = threadIdx.x & 63;
      const uint32_t slot = lds_addr(reinterpret_cast<const float*>(lds + (g % G::kNbuf) * G::kSlot)) + w * 1024;
      const char* src = wmain + bwd_main_off(g) + w * 1024 + lane * 16;
#pragma unroll
      for (int i = 0; i < G::main_n(g); ++i) glds16(reinterpret_cast<const float*>(src + i * 4096), slot + i * 4096);
      if constexpr (G::fc_n(g) > 0)
        glds16(reinterpret_cast<const float*>(wfc + (int64_t)g * 4096 + w * 1024 + lane * 16), slot + 32768);
    }
  }

  // values of quad q times s, split into the f16 parts of tile operand t
  template <typename T>
  static __device__ __forceinline__ void split_scaled(const float* v4, float s, int q, T (&t)[2][2]) {
    const float u[4] = {v4[0] * s, v4[1] * s, v4[2] * s, v4[3] * s};
    split_quad<PR>(u, q, t);
  }

  // delta of chain CC (li = 3 - CC), tile t: phase 1 = dL/dh (save, split for the feature
  // branch), phase 2 = mask, save delta, split into the next B operand
  template <int CC, int t, int q>
  static __device__ __forceinline__ void conv1(const BwdArgs& a, BwdState& S) {
    const int hh = (threadIdx.x >> 5) & 1;
    constexpr int li = 3 - CC;
#pragma unroll
    for (int i = 0; i < 4; ++i) S.v[4 * q + i] = S.acc[CC & 1][t][4 * q + i] * S.kconv;
    if constexpr (HASC) {  // fp32 dL/dh for dWc = gH^T c (wgrad16.hip)
      *reinterpret_cast<float4*>(a.gH + ((int64_t)li * a.ld_d + S.dcol) * kHidden + 32 * t + 8 * q + 4 * hh) =
          make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]);
      split_scaled(S.v + 4 * q, S.sig, q, S.tmp);
    }
  }
  template <int CC, int t, int q>
  static __device__ __forceinline__ void conv2(const BwdArgs& a, BwdState& S) {
    const int hh = (threadIdx.x >> 5) & 1;
    constexpr int li = 3 - CC;
    const uint32_t wd = t < 2 ? S.m[li].x : t < 4 ? S.m[li].y : t < 6 ? S.m[li].z : S.m[li].w;
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (!((wd >> ((t & 1) * 16 + 4 * q + i)) & 1u)) S.v[4 * q + i] = 0.f;
    // fp32 delta for the weight-gradient GEMMs
    *reinterpret_cast<float4*>(a.dP + ((int64_t)li * a.ld_d + S.dcol) * kHidden + 32 * t + 8 * q + 4 * hh) =
        make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]);
    split_scaled(S.v + 4 * q, S.sig, q, S.nxt);
  }

  template <int CC, int t, int SHIFT, int NT, int T>
  static __device__ __forceinline__ void conv_pieces(const BwdArgs& a, BwdState& S, const Frag<PR>& FC) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t1 = (q + SHIFT) < NT - 1 ? (q + SHIFT) : NT - 1;
      if (t1 == T) {
        if (q == 0) conv1<CC, t, 0>(a, S);
        if (q == 1) conv1<CC, t, 1>(a, S);
        if (q == 2) conv1<CC, t, 2>(a, S);
        if (q == 3) conv1<CC, t, 3>(a, S);
      }
    }
    if constexpr (HASC && T == (5 < NT - 1 ? 5 : NT - 1)) mfma_frag<PR, false>(FC, S.tmp, S.gc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t2 = (4 + q) < NT - 1 ? (4 + q) : NT - 1;
      if (t2 == T) {
        if (q == 0) conv2<CC, t, 0>(a, S);
        if (q == 1) conv2<CC, t, 1>(a, S);
        if (q == 2) conv2<CC, t, 2>(a, S);
        if (q == 3) conv2<CC, t, 3>(a, S);
      }
    }
  }

  // Chain boundary (all output tiles of chain CC finished, S.mx their max |acc| in this lane):
  // fix the point's split scale for chain CC's deltas and the multipliers of both chains.
  template <int CC>
  static __device__ __forceinline__ void boundary(BwdState& S, const float* inv, const float* fscl) {
    float m = fmaxf(S.mx, __shfl_xor(S.mx, 32));  // both lane halves hold the same point
    S.mx = 0.f;
    S.kconv = S.kacc;
    S.sig = pt_scale(m * S.kacc);
    S.kacc = inv[3 - CC] / S.sig;  // chain CC+1 runs on W_{3-CC}^T (inv[4 - c] for chain c)
    if constexpr (HASC) {  // dL/dc: the products of layer li = 3 - CC carry 2^wc_li * sig
      const float f = fscl[3 - CC] * S.sig;
      const float r = f / S.gcf;
#pragma unroll
      for (int i = 0; i < 16; ++i) S.gc[i] *= r;
      S.gcf = f;
    }
  }

  template <int NS, int NT, int T, int OUTSET, bool ZERO, bool CONV, bool BND, int CC, int CT, int SHIFT>
  static __device__ __forceinline__ void group(const BwdArgs& a, BwdState& S, const char* slot,
                                               const f16x8 (&act)[2][2], Frag<PR> (&F)[3], const Frag<PR>& FC,
                                               const float* inv, const float* fscl) {
    if constexpr (T < NT) {
      if constexpr (T + 2 < NT) load_frag<PR, NS>(slot + (T + 2) * NS * 2 * 1024, F[(T + 2) % 3]);
      mfma_frag<PR, ZERO, f16x8, NS>(F[T % 3], act, S.acc[OUTSET][T]);
      asm volatile("" : "+a"(S.acc[OUTSET][T]));
      if constexpr (BND) {
        // boundary step: fold the tile finished one group earlier into the running max; after the
        // last group, the last tile, the point scale, and all of tile 0's conversion
        if constexpr (T >= 1) S.mx = fmaxf(S.mx, tile_absmax(S.acc[OUTSET][T - 1]));
        if constexpr (T == NT - 1) {
          S.mx = fmaxf(S.mx, tile_absmax(S.acc[OUTSET][T]));
          boundary<CC>(S, inv, fscl);
          conv_pieces<CC, 0, 0, 1, 0>(a, S, FC);  // as a one-group step: every piece here
        }
      } else if constexpr (CONV) {
        conv_pieces<CC, CT, SHIFT, NT, T>(a, S, FC);
      }
      __builtin_amdgcn_sched_barrier(0);
      group<NS, NT, T + 1, OUTSET, ZERO, CONV, BND, CC, CT, SHIFT>(a, S, slot, act, F, FC, inv, fscl);
    }
  }

  template <int g>
  static __device__ __forceinline__ void step(const BwdArgs& a, BwdState& S, const char* wmain, const char* wfc,
                                              const char* lds, const float* inv, const float* fscl) {
    if constexpr (g < kBwdSteps) {
      constexpr int c = bwd_chain(g);
      constexpr int kc = bwd_kc(g);
      constexpr int NS = g == 0 ? 1 : 2;
      constexpr int NT = c == 4 ? 3 : 8;
      constexpr int OUTSET = c & 1;
      constexpr bool ZERO = kc == 0;
      constexpr bool CONV = bwd_conv(g);
      constexpr int CC = bwd_conv_chain(g);
      constexpr int CT = bwd_conv_tile(g);
      constexpr bool BND = CONV && CT == 0;  // the step that finishes chain CC (g = 0, 8, 16, 24)
      static_assert(!BND || (NT == 8 && CC == c), "boundary steps finish their own chain");
      constexpr int SHIFT = CT == 0 ? 1 : 0;
      sync_chunk<G::younger(g)>();
      stage_step<g + G::kDist>(a, wmain, wfc, lds);
      const char* slot = lds + (g % G::kNbuf) * G::kSlot;
      // both accumulator sets live in the 256 AGPRs for the whole kernel (see k_mlp_fwd16)
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 8; ++t) asm volatile("" : "+a"(S.acc[st][t]));
      asm volatile("" : "+v"(S.gc));
      Frag<PR> F[3], FC;
      load_frag<PR, NS>(slot, F[0]);
      load_frag<PR, NS>(slot + NS * 2 * 1024, F[1]);
      if constexpr (HASC && CONV) load_frag<PR>(slot + 32768, FC);
      __builtin_amdgcn_sched_barrier(0);
      if constexpr (g > 0) {
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int s = 0; s < 2; ++s) S.cur[pt][s] = S.nxt[pt][s];
      }
      group<NS, NT, 0, OUTSET, ZERO, CONV, BND, CC, CT, SHIFT>(a, S, slot, S.cur, F, FC, inv, fscl);
      step<g + 1>(a, S, wmain, wfc, lds, inv, fscl);
    }
  }

  template <int g>
  static __device__ __forceinline__ void prologue(const BwdArgs& a, const char* wmain, const char* wfc,
                                                  const char* lds) {
    if constexpr (g < G::kDist) {
      stage_step<g>(a, wmain, wfc, lds);
      prologue<g + 1>(a, wmain, wfc, lds);
    }
  }
};

template <bool HASC>
__global__ __launch_bounds__(256, 1) void k_mlp_bwd16(const float* __restrict__ W, BwdArgs a, int64_t P) {
  using K = BfBwd<HASC>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = (int64_t)blockIdx.x * 128 + wave * 32 + j;  // chunk-local point
  const bool valid = p < P;
  const char* wmain = reinterpret_cast<const char*>(W + kOffBwd);
  const char* wfc = HASC ? reinterpret_cast<const char*>(a.fcw + kOffFcBwd) : nullptr;
  K::template prologue<0>(a, wmain, wfc, lds);

  // inverse weight-image scales (W0..W3, Wo) and the forward fc scales (Wc_0..Wc_3): k_wscale
  const float* rawt = W + kOffRaw;
  float inv[5], fscl[4];
#pragma unroll
  for (int i = 0; i < 5; ++i) inv[i] = rawt[kRawInv + i];
#pragma unroll
  for (int i = 0; i < 4; ++i) fscl[i] = HASC ? a.fcw[kOffFcRaw + kFcRawScl + i] : 1.f;

  BwdState S;
  S.dcol = p;
  S.mx = 0.f;
  S.gcf = 1.f;
  const int64_t col = a.p0 + p;
  const int64_t mstride = (a.ld / 32) * 64;
  const uint4* mk = a.masks + ((a.p0 + (int64_t)blockIdx.x * 128) / 32 + wave_id()) * 64;
#pragma unroll
  for (int l = 0; l < 4; ++l) S.m[l] = mk[l * mstride + lane];
  // B operand of the Wo^T step: k = o = 0..3 sit in elements 0..3 of lane half 0 (g_out rows
  // exist for every padded point of the launch: the caller zero-fills them), times the point's scale
  {
    const float4 go = reinterpret_cast<const float4*>(a.g_out)[p];
    const float s0 = pt_scale(fmaxf(fmaxf(fabsf(go.x), fabsf(go.y)), fmaxf(fabsf(go.z), fabsf(go.w))));
    float gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) gv[r] = 0.f;
    if (hh == 0) {
      gv[0] = go.x * s0; gv[1] = go.y * s0; gv[2] = go.z * s0; gv[3] = go.w * s0;
    }
    split_tile<PNR_PREC_F16X3>(gv, S.cur);
    S.kacc = inv[4] / s0;
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) S.gc[r] = 0.f;
  // no accumulator zero fill: each layer's first input tile starts its tiles from 0 (ZERO)
  K::template step<0>(a, S, wmain, wfc, lds, inv, fscl);

  // g_arg = g_e * cos(x@B), g_x = B g_arg (the k_mlp_bwd epilogue on set 0, tiles 0..2)
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  if (valid) {
    const float4 xv = a.xP[col];
    x0 = xv.x; x1 = xv.y; x2 = xv.z;
  }
  const float* FB = W + kOffFB;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
  for (int t = 0; t < 3; ++t) {
    float gv[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = 32 * t + perm(r, hh);
      float g = 0.f;
      if (k < kFourier) {
        float arg;
        {
#pragma clang fp contract(off)
          arg = x0 * FB[k];
          arg = __builtin_fmaf(x1, FB[kFourierPad + k], arg);
          arg = __builtin_fmaf(x2, FB[2 * kFourierPad + k], arg);
        }
        g = (S.acc[0][t][r] * S.kacc) * fourier_sc<true>(arg);
        s0 = __builtin_fmaf(FB[k], g, s0);
        s1 = __builtin_fmaf(FB[kFourierPad + k], g, s1);
        s2 = __builtin_fmaf(FB[2 * kFourierPad + k], g, s2);
      }
      gv[r] = g;
    }
    // fp32 g_arg for the dB GEMM (wgrad16.hip k_wgrad_skinny)
    float* row = a.gargP + p * kFourierPad + 32 * t + 4 * hh;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(row + 8 * q) = make_float4(gv[4 * q], gv[4 * q + 1], gv[4 * q + 2], gv[4 * q + 3]);
  }
  if (HASC && valid) {
    const float gi = 1.f / S.gcf;
    float* row = a.g_c + p * kCDim + 4 * hh;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(row + 8 * q) =
          make_float4(S.gc[4 * q] * gi, S.gc[4 * q + 1] * gi, S.gc[4 * q + 2] * gi, S.gc[4 * q + 3] * gi);
  }
  if (a.g_x != nullptr) {
    s0 += __shfl_xor(s0, 32);
    s1 += __shfl_xor(s1, 32);
    s2 += __shfl_xor(s2, 32);
    if (valid && hh == 0) {
      a.g_x[p * 3 + 0] = s0;
      a.g_x[p * 3 + 1] = s1;
      a.g_x[p * 3 + 2] = s2;
    }
  }
}

template <bool HASC>
static int launch_bwd16(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st) {
  const size_t lds = BwdGeo<HASC>::kLds;
  auto kern = k_mlp_bwd16<HASC>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, dim3((unsigned)((P + 127) / 128)), dim3(256), lds, st, packed, a, P);
  return hip_status(hipGetLastError());
}

int launch_mlp_bwd_bf(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st) {
  if (P <= 0) return 0;
  TimingScope ts(kTimeMlpBwd, P, st);
  return a.fcw ? launch_bwd16<true>(packed, a, P, st) : launch_bwd16<false>(packed, a, P, st);
}

}  // namespace pnr
