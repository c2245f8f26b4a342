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
// The deltas (or, with features, dL/dh: delta_l is dL/dh_l masked) and g_arg go to HBM in fp32
// (point-major) for the weight-gradient GEMMs of wgrad16.hip, which split them again under their
// own scales.
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
#ifndef PNR_BWD_NBUF
#define PNR_BWD_NBUF 4
#endif
  // (a 5-slot ring, 160 KiB, built in round 6 gave wrong f16x3 gradients -- up to 5% of max|g_x| --
  // and no speed: tools/_r06ad.sh; the step program's waits are verified for at most 4 slots)
  static_assert(PNR_BWD_NBUF >= 3 && PNR_BWD_NBUF <= 4, "delta-chain DMA ring: 3 or 4 slots");
  static constexpr int kNbuf = HASC ? 4 : PNR_BWD_NBUF;  // 5 x 36 KiB would not fit
  // PIPE: the forward's step pipeline (barrier + DMA mid-step, the next step's fragments read ahead).
  // The feature variant keeps one barrier + DMA at the top of each step: the pipeline spills 61
  // registers there (12 without), and the neural-point mapping step took 190 ms against 168 ms.
  static constexpr bool PIPE = !HASC;
  // DMA distance (steps): with PIPE step g-1's slot frees mid-step g; without, at the top of step g
  static constexpr int kD = PIPE ? kNbuf - 2 : kNbuf - 1;
  static constexpr int kLds = kNbuf * kSlot;
  // fragment ring (groups prefetched kPf ahead; the feature variant keeps 3: 4 spills there)
  static constexpr int kRing = HASC ? 3 : 4, kPf = kRing - 1;
  __host__ __device__ static constexpr int main_n(int g) { return g == 0 ? 4 : (g <= 24 ? 8 : 3); }
  __host__ __device__ static constexpr int fc_n(int g) { return (HASC && g <= 31) ? 1 : 0; }
  __host__ __device__ static constexpr int n_glds(int g) { return g < kBwdSteps ? main_n(g) + fc_n(g) : 0; }
  // MFMA groups (output tiles) and k-steps per fragment of step g
  __host__ __device__ static constexpr int nt(int g) { return bwd_chain(g) == 4 ? 3 : 8; }
  __host__ __device__ static constexpr int ns(int g) { return g == 0 ? 1 : 2; }
  // group after which step g waits + meets for step g+1's slot and issues the DMA of step g+1+kD
  __host__ __device__ static constexpr int sync_t(int g) { return nt(g) == 8 ? 5 : 0; }
  __host__ __device__ static constexpr int clamp_t(int t, int g) { return t < nt(g) - 1 ? t : nt(g) - 1; }
  __host__ __device__ static constexpr int ring(int g) {
    int b = 0;
    for (int i = 0; i < g; ++i) b += nt(i);
    return b % kRing;
  }
  // group of step g that reads the next step's fragment tile k (after the barrier)
  __host__ __device__ static constexpr int next_grp(int g, int k) {
    const int t = nt(g) - kPf + k;
    return clamp_t(t > sync_t(g) ? t : sync_t(g), g);
  }
  __host__ __device__ static constexpr bool bnd(int g) { return bwd_conv(g) && bwd_conv_tile(g) == 0; }
  // group of a step with nt groups in which conversion piece q runs: phase 1 (conv1) and phase 2
  // (conv2, the delta store).  Without the feature branch the phases alternate (stores in every
  // other group: the save stream is spread over the step); with it phase 1 must finish by the
  // feature-branch product in group 5, so the phases run in groups 0-3 and 4-7
  __host__ __device__ static constexpr int grp1(int q, int shift, int n) {
    const int t = HASC ? q + shift : 2 * q + shift;
    return t < n - 1 ? t : n - 1;
  }
  __host__ __device__ static constexpr int grp2(int q, int shift, int n) {
    const int t = HASC ? 4 + q : 2 * q + 1 + shift;
    return t < n - 1 ? t : n - 1;
  }
  // delta (+ dL/dh) quad stores issued in group T of step g (conv_pieces placement)
  __host__ __device__ static constexpr int stores_grp(int g, int T) {
#if defined(PNR_EXP_NOSTORE)
    return 0;
#endif
    if (!bwd_conv(g)) return 0;
    // conv2 stores no delta4 (chain 0: kWgradOutDelta rebuilds it) and, with the feature branch, no
    // delta at all (the dW GEMMs mask conv1's dL/dh themselves); conv1's dL/dh (features) stays
    const bool d = !HASC && bwd_conv_chain(g) != 0;
    // dL/dh stores (features): not for chain 0's dL/dh4 = Wo^T g_out (the dWc_3 GEMM rebuilds it)
    const bool gh = HASC && bwd_conv_chain(g) != 0;
    if (bnd(g)) return T == nt(g) - 1 ? (gh ? 4 : 0) + (d ? 4 : 0) : 0;
    int n = 0;
    for (int q = 0; q < 4; ++q) n += (gh && grp1(q, 0, nt(g)) == T ? 1 : 0) + (d && grp2(q, 0, nt(g)) == T ? 1 : 0);
    return n;
  }
  __host__ __device__ static constexpr int stores_rng(int g, int t0, int t1) {
    int n = 0;
    for (int T = t0; T <= t1; ++T) n += stores_grp(g, T);
    return n;
  }
  // VMEM ops issued after DMA(i) and before the wait of barrier B_i (in step i-1, after group
  // sync_t(i-1)); DMA(i) was issued at B_{i-kD} (or in the prologue / start for i <= kD).  In the
  // persistent kernel DMAs i >= kBwdSteps are the next tile's.  For the first steps of a later tile
  // the previous tile's tail stores, its epilogue stores and this tile's first loads are younger
  // too: uncounted, so the wait is only stricter.
  __host__ __device__ static constexpr int younger_b(int i, bool pst) {
    int n = 0;
    for (int j = i + 1; j <= i + kD - 1; ++j) n += j < kBwdSteps ? n_glds(j) : (pst ? n_glds(j - kBwdSteps) : 0);
    int first = 0;
    if (i >= kD + 1) {
      const int p = i - kD;
      n += stores_rng(p - 1, sync_t(p - 1) + 1, nt(p - 1) - 1);
      first = p;
    }
    for (int g = first; g <= i - 2; ++g) n += stores_rng(g, 0, nt(g) - 1);
    n += stores_rng(i - 1, 0, sync_t(i - 1));
    return n;
  }
  // per-step structure: VMEM ops issued after DMA(g) (top of step g - kD) and before the wait at the
  // top of step g
  __host__ __device__ static constexpr int younger_s(int g) {
    int n = 0;
    for (int j = g + 1; j <= g + kD - 1; ++j) n += j < kBwdSteps ? n_glds(j) : 0;
    for (int i = g - kD < 0 ? 0 : g - kD; i < g; ++i) n += stores_rng(i, 0, nt(i) - 1);
    return n;
  }
  __host__ __device__ static constexpr int younger_b0() {
    int n = 0;
    for (int j = 1; j < kD; ++j) n += n_glds(j);
    return n;
  }
  __host__ __device__ static constexpr bool vm_ok() {
    for (int i = 1; i < kBwdSteps; ++i)
      if (younger_b(i, !HASC) >= 64 || younger_s(i) >= 64) return false;
    return true;
  }
};
static_assert(BwdGeo<true>::vm_ok() && BwdGeo<false>::vm_ok(), "vmcnt range");

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

template <int R>
struct BwdState {
  f32x16 acc[2][8];     // chain c output in set c & 1
  Frag<PNR_PREC_F16X3> F[R];  // fragment ring (one 32-row output tile of the current / next step each)
  Frag<PNR_PREC_F16X3> FC;    // feature-branch fragments of the step's conversion
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
  int sb;               // ring slot of step 0 of this tile (persistent kernel: the ring runs on)
  int64_t dcol;
};

template <bool HASC>
struct BfBwd {
  static constexpr int PR = PNR_PREC_F16X3;
  using G = BwdGeo<HASC>;
  using St = BwdState<G::kRing>;
  // Persistent kernel (no feature branch, as k_mlp_fwd16): a workgroup loops over 128-point tiles
  // and the weight stream runs on across them -- the last steps of tile i prefetch the first steps
  // of tile i+1, so no tile pays the DMA latency of its first steps.  Step g of a tile sits in ring
  // slot (g + sb) % kNbuf, sb = i kBwdSteps % kNbuf (continuous numbering).
  static constexpr bool PST = !HASC;

  // DMA of step g into its ring slot; in the persistent kernel steps g >= kBwdSteps are the next
  // tile's steps g - kBwdSteps
  template <int g>
  static __device__ __forceinline__ void stage_step(const BwdArgs& a, const char* wmain, const char* wfc,
                                                    const char* lds, int sb) {
    if constexpr (g < kBwdSteps || (PST && g < 2 * kBwdSteps)) {
      constexpr int st = g < kBwdSteps ? g : g - kBwdSteps;
      const int w = wave_id(), lane = threadIdx.x & 63;
      const uint32_t slot =
          lds_addr(reinterpret_cast<const float*>(lds + ((g + sb) % G::kNbuf) * G::kSlot)) + w * 1024;
      // wave-uniform base in SGPRs, the lane's byte offset in one VGPR: per-piece 64-bit VGPR
      // addresses are loop-invariant, get hoisted out of the persistent tile loop and spill
      const uint32_t voff = lane * 16;
      const char* src = wmain + bwd_main_off(st) + w * 1024;
      if constexpr (G::main_n(st) == 8 && !HASC) {  // (the feature-branch kernels: no SGPRs to spare)
        glds16s_x8(src, voff, slot);
      } else {
#pragma unroll
        for (int i = 0; i < G::main_n(st); ++i) glds16s(src + i * 4096, voff, slot + i * 4096);
      }
      if constexpr (G::fc_n(st) > 0) glds16s(wfc + (int64_t)st * 4096 + w * 1024, voff, slot + 32768);
    }
  }

  // values of quad q times s, split into the f16 parts of tile operand t
  template <typename T>
  static __device__ __forceinline__ void split_scaled(const float* v4, float s, int q, T (&t)[2][2]) {
    const float u[4] = {v4[0] * s, v4[1] * s, v4[2] * s, v4[3] * s};
    split_quad<PR, f16x8, !HASC>(u, q, t);
  }

  // fp32 save address of this lane's unit quad (t, q) of layer li: point-major row S.dcol
  static __device__ __forceinline__ float* d_save(float* base, const BwdArgs& a, const St& S, int li, int t, int q) {
    const int lane = threadIdx.x & 63;
#if defined(PNR_EXP_LINSAVE)  // experiment: ideal store shape (1 KB contiguous per instruction), wrong layout
    return base + ((int64_t)li * a.ld_d + S.dcol - (lane & 31)) * kHidden + (t * 4 + q) * 256 + lane * 4;
#else
    return base + ((int64_t)li * a.ld_d + S.dcol) * kHidden + 32 * t + 8 * q + 4 * (lane >> 5);
#endif
  }
  // delta of chain CC (li = 3 - CC), tile t: phase 1 = dL/dh (save, split for the feature
  // branch), phase 2 = mask, save delta, split into the next B operand
  template <int CC, int t, int q>
  static __device__ __forceinline__ void conv1(const BwdArgs& a, St& S) {
    constexpr int li = 3 - CC;
#pragma unroll
    for (int i = 0; i < 4; ++i) S.v[4 * q + i] = S.acc[CC & 1][t][4 * q + i] * S.kconv;
    if constexpr (HASC) {  // fp32 dL/dh for dWc = gH^T c (wgrad16.hip; dL/dh4 of chain 0 is rebuilt there)
      if constexpr (CC != 0)
        save16(d_save(a.gH, a, S, li, t, q), make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]));
      split_scaled(S.v + 4 * q, S.sig, q, S.tmp);
    }
  }
  template <int CC, int t, int q>
  static __device__ __forceinline__ void conv2(const BwdArgs& a, St& S) {
    constexpr int li = 3 - CC;
    const uint32_t wd = t < 2 ? S.m[li].x : t < 4 ? S.m[li].y : t < 6 ? S.m[li].z : S.m[li].w;
    // ReLU derivative: the bit sign-extended to an all-ones / zero word (v_bfe_i32) ANDed into the
    // value -- 2 VALU per value where the bit test + compare + select took 3
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int bit = (t & 1) * 16 + 4 * q + i;
      const int m = (int)(wd << (31 - bit)) >> 31;
      S.v[4 * q + i] = __int_as_float(__float_as_int(S.v[4 * q + i]) & m);
    }
    // fp32 delta for the weight-gradient GEMMs (delta4 = chain 0's: not stored, kWgradOutDelta;
    // with the feature branch none: the GEMMs apply the mask words to conv1's dL/dh, wgrad16.hip MSK)
#if !defined(PNR_EXP_NOSTORE)
    if constexpr (CC != 0 && !HASC)
#else
    if constexpr (false)  // experiment: no delta stores (timing bound only)
#endif
      save16(d_save(a.dP, a, S, li, t, q), make_float4(S.v[4 * q], S.v[4 * q + 1], S.v[4 * q + 2], S.v[4 * q + 3]));
    split_scaled(S.v + 4 * q, S.sig, q, S.nxt);
  }

  template <int CC, int t, int SHIFT, int NT, int T>
  static __device__ __forceinline__ void conv_pieces(const BwdArgs& a, St& S, const Frag<PR>& FC) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      if (G::grp1(q, SHIFT, NT) == T) {
        if (q == 0) conv1<CC, t, 0>(a, S);
        if (q == 1) conv1<CC, t, 1>(a, S);
        if (q == 2) conv1<CC, t, 2>(a, S);
        if (q == 3) conv1<CC, t, 3>(a, S);
      }
      if (!HASC && G::grp2(q, SHIFT, NT) == T) {  // alternating phases: piece q's phase 2 right after
        if (q == 0) conv2<CC, t, 0>(a, S);
        if (q == 1) conv2<CC, t, 1>(a, S);
        if (q == 2) conv2<CC, t, 2>(a, S);
        if (q == 3) conv2<CC, t, 3>(a, S);
      }
    }
    if constexpr (HASC && T == (5 < NT - 1 ? 5 : NT - 1)) mfma_frag<PR, false>(FC, S.tmp, S.gc);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int t2 = G::grp2(q, SHIFT, NT);
      if (HASC && t2 == T) {
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
  static __device__ __forceinline__ void boundary(St& S, const float* inv, const float* fscl) {
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

  static __device__ __forceinline__ const char* slot_of(const char* lds, int g, int sb) {
    return lds + ((g + sb) % G::kNbuf) * G::kSlot;
  }
  // the next step's fragment tile k (issued after its barrier)
  template <int g, int k>
  static __device__ __forceinline__ void next_frag(St& S, const char* lds) {
    if constexpr (g < kBwdSteps && k < G::nt(g))
      load_frag<PR, G::ns(g)>(slot_of(lds, g, S.sb) + k * G::ns(g) * 2 * 1024, S.F[(G::ring(g) + k) % G::kRing]);
  }

  // MFMA group T of step g (prefetching the fragments of group T + kPf), its conversion pieces, and
  // the next step's barrier / DMA / first fragment reads where they fall (the k_mlp_fwd16 pipeline:
  // no step starts with an LDS round trip or a barrier)
  template <int g, int T>
  static __device__ __forceinline__ void group(const BwdArgs& a, St& S, const char* wmain, const char* wfc,
                                               const char* lds, const f16x8 (&act)[2][2], const float* inv,
                                               const float* fscl) {
    constexpr int NT = G::nt(g);
    if constexpr (T < NT) {
      constexpr int NS = G::ns(g);
      constexpr int OUTSET = bwd_chain(g) & 1;
      constexpr bool ZERO = bwd_kc(g) == 0;
      constexpr bool CONV = bwd_conv(g);
      constexpr int CC = bwd_conv_chain(g);
      constexpr int CT = bwd_conv_tile(g);
      constexpr bool BND = G::bnd(g);  // the step that finishes chain CC (g = 0, 8, 16, 24)
      static_assert(!BND || (NT == 8 && CC == bwd_chain(g)), "boundary steps finish their own chain");
      constexpr int SHIFT = CT == 0 ? 1 : 0;
      constexpr int b = G::ring(g);
      const char* slot = slot_of(lds, g, S.sb);
      if constexpr (G::PIPE && HASC && CONV && T == G::clamp_t(1, g)) load_frag<PR>(slot + 32768, S.FC);
      if constexpr (T + G::kPf < NT)
        load_frag<PR, NS>(slot + (T + G::kPf) * NS * 2 * 1024, S.F[(b + T + G::kPf) % G::kRing]);
      __builtin_amdgcn_sched_barrier(0);  // prefetch first, then the group's MFMAs
      mfma_frag<PR, ZERO, f16x8, NS>(S.F[(b + T) % G::kRing], act, S.acc[OUTSET][T]);
      asm volatile("" : "+a"(S.acc[OUTSET][T]));
      if constexpr (BND) {
        // boundary step: fold the tile finished one group earlier into the running max; after the
        // last group, the last tile, the point scale, and all of tile 0's conversion
        if constexpr (T >= 1) S.mx = fmaxf(S.mx, tile_absmax(S.acc[OUTSET][T - 1]));
        if constexpr (T == NT - 1) {
          S.mx = fmaxf(S.mx, tile_absmax(S.acc[OUTSET][T]));
          boundary<CC>(S, inv, fscl);
          conv_pieces<CC, 0, 0, 1, 0>(a, S, S.FC);  // as a one-group step: every piece here
        }
      } else if constexpr (CONV) {
        conv_pieces<CC, CT, SHIFT, NT, T>(a, S, S.FC);
      }
      if constexpr (G::PIPE && g + 1 < kBwdSteps) {
        if constexpr (T == G::sync_t(g)) {
          sync_chunk<G::younger_b(g + 1, PST)>();
          stage_step<g + 1 + G::kD>(a, wmain, wfc, lds, S.sb);
        }
        if constexpr (T == G::next_grp(g, 0)) next_frag<g + 1, 0>(S, lds);
        if constexpr (G::kPf > 1 && T == G::next_grp(g, 1)) next_frag<g + 1, 1>(S, lds);
        if constexpr (G::kPf > 2 && T == G::next_grp(g, 2)) next_frag<g + 1, 2>(S, lds);
      }
      __builtin_amdgcn_sched_barrier(0);
      group<g, T + 1>(a, S, wmain, wfc, lds, act, inv, fscl);
    }
  }

  template <int g>
  static __device__ __forceinline__ void step(const BwdArgs& a, St& S, const char* wmain, const char* wfc,
                                              const char* lds, const float* inv, const float* fscl) {
    if constexpr (g < kBwdSteps) {
      // both accumulator sets live in the 256 AGPRs for the whole kernel (see k_mlp_fwd16); step 0
      // only defines them, so a persistent kernel carries no accumulator around its tile loop
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          if constexpr (g == 0) asm volatile("" : "=a"(S.acc[st][t]));
          else asm volatile("" : "+a"(S.acc[st][t]));
        }
      if constexpr (HASC) asm volatile("" : "+v"(S.gc));
      if constexpr (!G::PIPE) {  // the step's barrier, the DMA kD steps ahead, its first fragments
        sync_chunk<G::younger_s(g)>();
        stage_step<g + G::kD>(a, wmain, wfc, lds, S.sb);
        next_frag<g, 0>(S, lds);
        if constexpr (G::kPf > 1) next_frag<g, 1>(S, lds);
        if constexpr (G::kPf > 2) next_frag<g, 2>(S, lds);
        if constexpr (HASC && bwd_conv(g)) load_frag<PR>(slot_of(lds, g, S.sb) + 32768, S.FC);
        __builtin_amdgcn_sched_barrier(0);
      }
      if constexpr (g > 0) {
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int s = 0; s < 2; ++s) S.cur[pt][s] = S.nxt[pt][s];
      }
      group<g, 0>(a, S, wmain, wfc, lds, S.cur, inv, fscl);
      step<g + 1>(a, S, wmain, wfc, lds, inv, fscl);
    }
  }

  // barrier B_0: step 0's slot is valid; DMA of step kD; step 0's first fragment reads
  static __device__ __forceinline__ void start(const BwdArgs& a, St& S, const char* wmain, const char* wfc,
                                               const char* lds) {
    if constexpr (!G::PIPE) return;  // step 0 opens with its own barrier
    sync_chunk<G::younger_b0()>();
    stage_step<G::kD>(a, wmain, wfc, lds, S.sb);
    next_frag<0, 0>(S, lds);
    if constexpr (G::kPf > 1) next_frag<0, 1>(S, lds);
    if constexpr (G::kPf > 2) next_frag<0, 2>(S, lds);
  }

  template <int g>
  static __device__ __forceinline__ void prologue(const BwdArgs& a, const char* wmain, const char* wfc,
                                                  const char* lds) {
    if constexpr (g < G::kD) {
      stage_step<g>(a, wmain, wfc, lds, 0);
      prologue<g + 1>(a, wmain, wfc, lds);
    }
  }
};

// one 128-point tile of k_mlp_bwd16 (sb: its ring slot base)
template <bool HASC>
static __device__ __forceinline__ void bwd16_tile(const float* __restrict__ W, const BwdArgs& a, int64_t P,
                                                  const char* wmain, const char* wfc, const char* lds,
                                                  const float (&inv)[5], const float (&fscl)[4], int64_t tile, int sb) {
  using K = BfBwd<HASC>;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = tile * 128 + wave * 32 + j;  // chunk-local point
  const bool valid = p < P;
  typename K::St S;
  S.sb = sb;
  S.dcol = p;
  S.mx = 0.f;
  S.gcf = 1.f;
  const int64_t col = a.p0 + p;
  // the saved input is used only after the chain: the persistent kernel reads it now, so its
  // latency stays hidden (the feature-branch kernel has no registers to spare: it reads it there)
  float4 xv = make_float4(0.f, 0.f, 0.f, 0.f);
  if (K::PST && valid) xv = a.xP[col];
  const int64_t mstride = (a.ld / 32) * 64;
  const uint4* mk = a.masks + ((a.p0 + tile * 128) / 32 + wave_id()) * 64;
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
    split_tile<PNR_PREC_F16X3, f16x8, !HASC>(gv, S.cur);
    S.kacc = inv[4] / s0;
  }
  if (HASC) {
#pragma unroll
    for (int r = 0; r < 16; ++r) S.gc[r] = 0.f;
  }
  // no accumulator zero fill: each layer's first input tile starts its tiles from 0 (ZERO)
  K::start(a, S, wmain, wfc, lds);
  K::template step<0>(a, S, wmain, wfc, lds, inv, fscl);

  // g_arg = g_e * cos(x@B), g_x = B g_arg (the k_mlp_bwd epilogue on set 0, tiles 0..2)
  if (!K::PST && valid) xv = a.xP[col];
  const float x0 = xv.x, x1 = xv.y, x2 = xv.z;
  const float* FB = W + kOffRaw + kRawFB;  // the raw table's copy (an f16x3-only pack has no fp32 image)
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
      save16(row + 8 * q, make_float4(gv[4 * q], gv[4 * q + 1], gv[4 * q + 2], gv[4 * q + 3]));
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
__global__ __launch_bounds__(256, 1) void k_mlp_bwd16(const float* __restrict__ W, BwdArgs a, int64_t P) {
  using K = BfBwd<HASC>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
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
  if constexpr (K::PST) {
    const int64_t ntiles = (P + 127) / 128;
    int sb = 0;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      bwd16_tile<HASC>(W, a, P, wmain, wfc, lds, inv, fscl, tile, sb);
      sb = (sb + kBwdSteps) % BwdGeo<HASC>::kNbuf;
    }
    // the last tile's prefetch of a next tile (always issued: fixed wait counts) must land in the
    // workgroup's LDS before it exits
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    bwd16_tile<HASC>(W, a, P, wmain, wfc, lds, inv, fscl, blockIdx.x, 0);
  }
}

template <bool HASC>
static int launch_bwd16(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st) {
  const size_t lds = BwdGeo<HASC>::kLds;
  auto kern = k_mlp_bwd16<HASC>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  // one workgroup per 128-point tile; the persistent kernel (no feature branch) loops over tiles on
  // at most one workgroup per CU
  int64_t nwg = (P + 127) / 128;
  if (BfBwd<HASC>::PST) {
    const int ncu = device_cu_count();
    nwg = nwg < ncu ? nwg : ncu;
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)nwg), dim3(256), lds, st, packed, a, P);
  return hip_status(hipGetLastError());
}

int launch_mlp_bwd_bf(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st) {
  if (P <= 0) return 0;
  TimingScope ts(kTimeMlpBwd, P, st);
  return a.fcw ? launch_bwd16<true>(packed, a, P, st) : launch_bwd16<false>(packed, a, P, st);
}

}  // namespace pnr
