// mlp16u.h -- the f16x3 decoder forward with the output units split over two waves per SIMD
// (k_mlp_fwd16u).
//
// Same math and the same weight image as k_mlp_fwd16<PNR_PREC_F16X3, false, *> (mlp16.h;
// src/conv_onet/models/decoder.py:177-203 with the bound mask of src/utils/Renderer.py:43-57): every
// GEMM operand split x = hi + lo in f16, W x ~= Wl xh + Wh xl + Wh xh on v_mfma_f32_32x32x16_f16 with
// fp32 accumulation, the weights scaled by the per-tensor power of two of k_wscale.
//
// k_mlp_fwd16 runs one 32-point wave per SIMD holding all 256 units of a layer twice (two 8-tile
// accumulator sets: 512 registers), so a layer's epilogue VALU (bias, ReLU, masks, saves, the f16
// split) sits in the MFMA stream of the only wave on the SIMD: without it (PNR_EXP_NOCONV) the kernel
// ran 22% (eval) and 33% (training) faster.  Here a 512-thread workgroup runs the same 128-point tile
// as EIGHT waves, two per SIMD: wave w owns point tile w & 3 (32 points) and unit half w >> 2 (output
// tiles 4 (w >> 2) .. + 3), so the two waves of a SIMD (w, w + 4) are the two halves of one point
// tile, each with 2 sets x 4 tiles x 16 = 128 accumulator registers.  A converted input tile of the
// next layer (32 units x 32 points, hi / lo: 4 KiB) is written to LDS by its owner and read back by
// both halves (an exchange buffer per point tile, double-buffered by tile parity); in any one step
// only the owner of the tile being converted runs the epilogue, so the two waves of a SIMD are never
// in their VALU phase together: one converts while the other issues MFMAs.
// Per step a wave runs 4 MFMA groups (its output tiles) of 6 MFMAs and reads 16 KiB of the weight
// slot (the ds_read traffic of k_mlp_fwd16), and issues 4 of the step's 32 LDS-DMA pieces.
// LDS: a 3-slot weight ring (96 KiB: the DMA runs one step ahead), the raw table with Wo (12 KiB),
// the exchange buffers (32 KiB), the output partials (2 KiB).
// Output layer: fp32 VALU against Wo in LDS, each half over its 128 units, the halves' partial sums
// added through LDS.  Saves (training): x, h1..h4 fp32 point-major rows and the ReLU mask words in
// k_mlp_fwd16's layout (each half writes its 8 bytes of a lane's 16-byte word).
#pragma once
#include "mlp16.h"

namespace pnr {

struct U2Geo {
  static constexpr int kNbuf = 3, kSlot = 32768, kD = kNbuf - 2, kSteps = kHidSteps, kNT = 4;
  static constexpr int kRawOff = kNbuf * kSlot;                    // raw table + Wo fp32 (12 KiB)
  static constexpr int kXOff = kRawOff + (int)kRawPackedBytes;     // exchange [pt 4][buf 2][4 KiB]
  static constexpr int kOutOff = kXOff + 4 * 2 * 4096;             // output partials [pt 4][32] float4
  static constexpr int kLds = kOutOff + 4 * 32 * 16;               // 142 KiB
#ifndef PNR_U2_SYNC
#define PNR_U2_SYNC 1
#endif
  static constexpr int kSync = PNR_U2_SYNC;                        // group of a step that meets the next slot
  static constexpr int kRing = 3, kPf = kRing - 1;                 // fragment ring (groups prefetched ahead)
};
static_assert(U2Geo::kLds <= 160 * 1024, "LDS budget");

__host__ __device__ constexpr int u2_layer(int g) { return g < 3 ? 0 : 1 + (g - 3) / 8; }
__host__ __device__ constexpr int u2_kc(int g) { return g < 3 ? g : (g - 3) % 8; }
// step g converts (and exchanges) input tile u2_ct(g) of h_{u2_cl(g)}: the next step's input tile;
// h4 (the last layer) is converted by the output phase
__host__ __device__ constexpr bool u2_conv(int g) { return !(u2_layer(g) == 0 && u2_kc(g) < 2) && g + 1 < kHidSteps; }
__host__ __device__ constexpr int u2_ct(int g) { return (u2_layer(g) == 0 || u2_kc(g) == 7) ? 0 : u2_kc(g) + 1; }
__host__ __device__ constexpr int u2_cl(int g) {
  return u2_layer(g) == 0 ? 0 : (u2_kc(g) < 7 ? u2_layer(g) - 1 : u2_layer(g));
}

struct U2State {
  using F = Frag<PNR_PREC_F16X3>;
  f32x16 acc[2][4];      // h_L (this half's 4 output tiles) in set L & 1
  f16x8 cur[2][2];       // B operand of the current input tile [part][k-step]
  f16x8 nxt[2][2];       // the next one (a Fourier tile, or read back from the exchange)
  float inv;             // 2^-e of the weight image of the layer being converted
  uint32_t rb;           // this lane's LDS address of the raw table (+ 4 hh floats), opaque per step
  uint32_t mw[2];        // ReLU bit words 2uh, 2uh + 1 of the layer being converted
  F Fr[U2Geo::kRing];    // fragment ring
  float vmax;            // max |value| split into f16 parts (f16 range check)
  float x0, x1, x2;
  int sb, uh, pt;        // ring slot base; unit half; point tile (wave-uniform)
  int64_t col, mask_word0;
  __attribute__((address_space(1))) float* hrow;  // h save row of the lane's point (+ 4 hh), h1's region
  bool valid, inside;
};

// SV: 0 eval, 1 training saves (x, masks, h1..h4), 2 masks + x only
template <int SV>
struct U2Fwd {
  static constexpr bool SAVE = SV != 0, SAVEH = SV == 1;
  using G = U2Geo;
  using St = U2State;
  using V8 = f16x8;
  static constexpr int PR = PNR_PREC_F16X3;
  static constexpr int kSteps = G::kSteps, kD = G::kD, kPf = G::kPf, kRing = G::kRing;

  __host__ __device__ static constexpr int n_glds(int g) { return g < kSteps ? 4 : 0; }
  // stores of step g's epilogue in group T, for a wave of unit half uh (only the owner of the tile
  // converts: conv pieces q0, q1 in group 0, q2, q3 in group 1; the half's mask words after its last tile)
  __host__ __device__ static constexpr int stores_grp(int g, int T, int uh) {
    if (!SAVE || !u2_conv(g) || (u2_ct(g) >> 2) != uh) return 0;
    int n = 0;
    if (SAVEH && (T == 0 || T == 1)) n += 2;
    if ((u2_ct(g) & 3) == 3 && T == 1) ++n;
    return n;
  }
  __host__ __device__ static constexpr int stores_rng(int g, int t0, int t1, int uh) {
    int n = 0;
    for (int T = t0; T <= t1; ++T) n += stores_grp(g, T, uh);
    return n;
  }
  // VMEM ops issued after DMA(i) and before the wait of barrier B_i (after group kSync of step i - 1);
  // DMA(i) goes out at B_{i-kD}.  The smaller count of the two halves (a wait that counts fewer younger
  // ops is stricter); a later tile's first barriers also see the previous tile's output-phase stores
  // as younger: uncounted, so stricter too.
  __host__ __device__ static constexpr int younger_b_uh(int i, int uh) {
    int n = 0;
    for (int j = i + 1; j <= i + kD - 1; ++j) n += j < kSteps ? n_glds(j) : n_glds(j - kSteps);
    if (SAVE) {
      int first = 0;
      if (i >= kD && i - kD >= 1) {
        const int p = i - kD;
        n += stores_rng(p - 1, G::kSync + 1, G::kNT - 1, uh);
        first = p;
      } else {
        if (i < kD) n += 1;
        first = 0;
      }
      for (int g = first; g <= i - 2; ++g) n += stores_rng(g, 0, G::kNT - 1, uh);
      n += stores_rng(i - 1, 0, G::kSync, uh);
    }
    return n;
  }
  __host__ __device__ static constexpr int younger_b(int i) {
    return younger_b_uh(i, 0) < younger_b_uh(i, 1) ? younger_b_uh(i, 0) : younger_b_uh(i, 1);
  }
  __host__ __device__ static constexpr int younger_b0() {
    int n = 0;
    for (int j = 1; j < kD; ++j) n += n_glds(j);
    return n + (SAVE ? 1 : 0);
  }
  __host__ __device__ static constexpr bool vm_ok() {
    for (int i = 1; i < kSteps; ++i)
      if (younger_b(i) >= 64) return false;
    return younger_b0() < 64;
  }
  static __device__ __forceinline__ const char* slot_of(const char* lds, int g, int sb) {
    return lds + ((g + sb) % G::kNbuf) * G::kSlot;
  }
  template <int g>
  static __device__ __forceinline__ void stage_step(const char* wimg, const char* lds, int sb) {
    if constexpr (g < 2 * kSteps) {
      constexpr int st = g < kSteps ? g : g - kSteps;
      const int w = wave_id();
      const uint32_t slot = lds_addr(reinterpret_cast<const float*>(slot_of(lds, g, sb))) + w * 1024;
      const char* base = wimg;  // opaque per call (27 steps' source pairs hoisted out of the tile loop spill)
      asm volatile("" : "+s"(base));
      glds16s_x4(base + (int64_t)st * 32768 + w * 1024, (threadIdx.x & 63) * 16, slot);
    }
  }
  static __device__ __forceinline__ const float* raw_lds(const char* lds) {
    return reinterpret_cast<const float*>(lds + G::kRawOff);
  }
  // wait for this wave's DMA (and its LDS writes: the exchange), then meet the other waves
  template <int N>
  static __device__ __forceinline__ void sync_x() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
  }
  // exchange buffer of point tile pt for input tile t (parity buffers)
  static __device__ __forceinline__ uint32_t xaddr(const char* lds, const St& S, int t) {
    return lds_addr(reinterpret_cast<const float*>(lds + G::kXOff)) + (S.pt * 2 + (t & 1)) * 4096 +
           (threadIdx.x & 63) * 16;
  }
  static __device__ __forceinline__ V8 lds16(uint32_t a) {
    return *reinterpret_cast<const __attribute__((address_space(3))) V8*>((uintptr_t)a);
  }
  static __device__ __forceinline__ void sts16(uint32_t a, const V8& v) {
    *reinterpret_cast<__attribute__((address_space(3))) V8*>((uintptr_t)a) = v;
  }
  // Fourier tile t (units 32t + perm(r, hh)) of the lane's point: k_mlp_fwd16's prologue, into `dst`
  template <int t>
  static __device__ __forceinline__ void fourier_tile(St& S, const char* lds, V8 (&dst)[2][2]) {
    const int hh = (threadIdx.x >> 5) & 1;
    uint32_t fb = lds_addr(raw_lds(lds) + kRawFB) + 16 * hh;  // opaque: constant offsets per element
    asm volatile("" : "+v"(fb));
    float v[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int ko = 32 * t + (r & 3) + 8 * (r >> 2);  // perm(r, hh) - 4 hh
      const int k = ko + 4 * hh;
      const auto rd = [&](int c) {
        return *reinterpret_cast<const __attribute__((address_space(3))) float*>(
            (uintptr_t)(fb + 4 * (c * kFourierPad + ko)));
      };
      float arg;
      {
#pragma clang fp contract(off)
        arg = S.x0 * rd(0);
        arg = __builtin_fmaf(S.x1, rd(1), arg);
        arg = __builtin_fmaf(S.x2, rd(2), arg);
      }
      v[r] = k < kFourier ? fourier_sc<false>(arg) : 0.f;
    }
    split_tile<PR, V8, true>(v, dst);
  }
  template <int L, int t>
  static __device__ __forceinline__ void preload(St& S, const char* lds) {
    const int hh = (threadIdx.x >> 5) & 1;
    S.rb = lds_addr(raw_lds(lds)) + 16 * hh;  // opaque base (per-site addresses hoisted out of the loop spill)
    asm volatile("" : "+v"(S.rb));
    S.inv = raw_lds(lds)[kRawInv + L];
  }
  // epilogue of quad q of h_L tile t (this wave's local tile T = t & 3): bias + ReLU, mask bits, fp32
  // save, f16 range fold and the split into S.xt; values stay in `v`
  // (SPLIT: the hi / lo pairs go straight to the exchange buffer at xa, two 8-byte LDS stores)
  template <int L, int t, int q, bool SPLIT>
  static __device__ __forceinline__ void conv_quad(const BfFwdArgs& a, St& S, float (&v)[4], uint32_t xa = 0) {
    const int lane = threadIdx.x & 63;
    typedef float v4f __attribute__((ext_vector_type(4)));
    const v4f b4 = *reinterpret_cast<const __attribute__((address_space(3))) v4f*>(
        (uintptr_t)(S.rb + 4 * (kRawB + L * 256 + 32 * t + 8 * q)));
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = S.acc[L & 1][t & 3][4 * q + i] * S.inv + b4[i];
      v[i] = x > 0.f ? x : 0.f;
    }
    if constexpr (SAVE) {
#pragma unroll
      for (int i = 0; i < 4; ++i) S.mw[(t >> 1) & 1] |= (v[i] > 0.f ? 1u : 0u) << ((t & 1) * 16 + 4 * q + i);
    }
    (void)lane;
    if constexpr (SAVEH)
      *reinterpret_cast<__attribute__((address_space(1))) v4f*>(S.hrow + (int64_t)L * a.save.ld * kHidden + 32 * t +
                                                                8 * q) = v4f{v[0], v[1], v[2], v[3]};
    if constexpr (SPLIT) {
      S.vmax = fmaxf(S.vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
      asm volatile("" : "+v"(S.vmax));  // here, not sunk to the tile's end (keeps every value alive)
      uint32_t h0, l0, h1, l1;
      split2(v[0], v[1], h0, l0);
      split2(v[2], v[3], h1, l1);
      typedef uint32_t u2v __attribute__((ext_vector_type(2)));
      // B operand [part][k-step q >> 1], elements 4 (q & 1) .. + 3: dwords 2 (q & 1), + 1
      *reinterpret_cast<__attribute__((address_space(3))) u2v*>((uintptr_t)(xa + (q >> 1) * 1024 + 8 * (q & 1))) =
          u2v{h0, h1};
      *reinterpret_cast<__attribute__((address_space(3))) u2v*>((uintptr_t)(xa + (2 + (q >> 1)) * 1024 + 8 * (q & 1))) =
          u2v{l0, l1};
    }
  }
  // the half's mask words of layer L (after its last tile): 8 bytes of the lane's 16-byte word
  template <int L>
  static __device__ __forceinline__ void store_masks(const BfFwdArgs& a, St& S) {
    if constexpr (SAVE) {
      const int lane = threadIdx.x & 63;
      uint2* m = reinterpret_cast<uint2*>(a.save.masks + (int64_t)L * (a.save.ld / 32) * 64 + S.mask_word0 + lane);
      m[S.uh] = make_uint2(S.mw[0], S.mw[1]);
      S.mw[0] = S.mw[1] = 0u;
    }
  }

  // MFMA group T of step g: prefetch, 6 MFMAs on output tile 4 uh + T, the owner's epilogue pieces,
  // and the next step's barrier / DMA / exchange read / first fragments / constants
  template <int g, int T>
  static __device__ __forceinline__ void group(const BfFwdArgs& a, St& S, const char* lds) {
    if constexpr (T < G::kNT) {
      constexpr int layer = u2_layer(g), kc = u2_kc(g);
      constexpr int OUT = layer & 1;
      constexpr bool CONV = u2_conv(g);
      constexpr int CL = u2_cl(g), CT = u2_ct(g);
      constexpr int RB = (G::kNT * g) % kRing;
      static_assert((G::kNT * kSteps) % kRing == 0, "ring aligned at tile boundaries");
      const char* slot = slot_of(lds, g, S.sb) + S.uh * 16384;
      if constexpr (T + kPf < G::kNT) load_frag<PR>(slot + (T + kPf) * 4096, S.Fr[(RB + T + kPf) % kRing]);
      __builtin_amdgcn_sched_barrier(0);
      mfma_frag<PR, kc == 0>(S.Fr[(RB + T) % kRing], S.cur, S.acc[OUT][T]);
      asm volatile("" : "+a"(S.acc[OUT][T]));
      // the next Fourier tile (steps 0, 1: no exchange), computed by every wave under the MFMAs
      if constexpr (g < 2 && T == 1) fourier_tile<g + 1>(S, lds, S.nxt);
      // the owner of tile CT converts it: quads 0, 1 in group 0, quads 2, 3 + the exchange write in group 1
      if constexpr (CONV && (T == 0 || T == 1)) {
        if (S.uh == (CT >> 2)) {
          float v[4];
          const uint32_t xa = xaddr(lds, S, CT);
          conv_quad<CL, CT, 2 * T, true>(a, S, v, xa);
          conv_quad<CL, CT, 2 * T + 1, true>(a, S, v, xa);
          if constexpr (T == 1 && (CT & 3) == 3) store_masks<CL>(a, S);
        }
      }
      if constexpr (g + 1 < kSteps) {
        if constexpr (T == G::kSync) {
          sync_x<younger_b(g + 1)>();
          stage_step<g + 1 + kD>(a.wmain, lds, S.sb);
          if constexpr (CONV) {  // the converted tile, from the exchange (both halves)
            const uint32_t xa = xaddr(lds, S, CT);
#pragma unroll
            for (int pt = 0; pt < 2; ++pt)
#pragma unroll
              for (int s = 0; s < 2; ++s) S.nxt[pt][s] = lds16(xa + (pt * 2 + s) * 1024);
          }
        }
        if constexpr (T >= G::kNT - kPf) {
          constexpr int k = T - (G::kNT - kPf);
          load_frag<PR>(slot_of(lds, g + 1, S.sb) + S.uh * 16384 + k * 4096, S.Fr[(G::kNT * (g + 1) + k) % kRing]);
        }
        if constexpr (T == G::kNT - 1 && u2_conv(g + 1)) preload<u2_cl(g + 1), u2_ct(g + 1)>(S, lds);
      }
      __builtin_amdgcn_sched_barrier(0);
      group<g, T + 1>(a, S, lds);
    }
  }
  template <int g>
  static __device__ __forceinline__ void step(const BfFwdArgs& a, St& S, const char* lds) {
    if constexpr (g < kSteps) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if constexpr (g == 0) asm volatile("" : "=a"(S.acc[st][t]));
          else asm volatile("" : "+a"(S.acc[st][t]));
        }
      if constexpr (g > 0) {
#pragma unroll
        for (int pt = 0; pt < 2; ++pt)
#pragma unroll
          for (int s = 0; s < 2; ++s) S.cur[pt][s] = S.nxt[pt][s];
      }
      group<g, 0>(a, S, lds);
      step<g + 1>(a, S, lds);
    }
  }
  template <int g>
  static __device__ __forceinline__ void prologue(const char* wimg, const char* lds) {
    if constexpr (g < kD) {
      stage_step<g>(wimg, lds, 0);
      prologue<g + 1>(wimg, lds);
    }
  }
  static __device__ __forceinline__ void start(const BfFwdArgs& a, St& S, const char* lds) {
    sync_chunk<younger_b0()>();
    stage_step<kD>(a.wmain, lds, S.sb);
#pragma unroll
    for (int k = 0; k < kPf; ++k) load_frag<PR>(slot_of(lds, 0, S.sb) + S.uh * 16384 + k * 4096, S.Fr[k]);
  }
  // output layer: this half's 4 tiles of h4 (bias, ReLU, masks, saves) against Wo (fp32, LDS)
  template <int T>
  static __device__ __forceinline__ void out_tiles(const BfFwdArgs& a, St& S, const char* lds, uint32_t wo,
                                                   float (&o)[4]) {
    if constexpr (T < 4) {
      if (S.uh == 0) out_tile_g<T>(a, S, lds, wo, o);  // global tile 4 uh + T (uh wave-uniform)
      else out_tile_g<4 + T>(a, S, lds, wo, o);
      out_tiles<T + 1>(a, S, lds, wo, o);
    }
  }
  template <int t, int q>
  static __device__ __forceinline__ void out_quad(const BfFwdArgs& a, St& S, uint32_t wo, float (&o)[4]) {
    typedef float v4f __attribute__((ext_vector_type(4)));
    using lds_f4 = const __attribute__((address_space(3))) v4f;
    if constexpr (q < 4) {
      float v[4];
      conv_quad<3, t, q, false>(a, S, v);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const v4f w = *reinterpret_cast<lds_f4*>((uintptr_t)(wo + 4 * (i * kHidden + 32 * t + 8 * q)));
        o[i] = __builtin_fmaf(w.x, v[0], o[i]);
        o[i] = __builtin_fmaf(w.y, v[1], o[i]);
        o[i] = __builtin_fmaf(w.z, v[2], o[i]);
        o[i] = __builtin_fmaf(w.w, v[3], o[i]);
      }
      out_quad<t, q + 1>(a, S, wo, o);
    }
  }
  template <int t>
  static __device__ __forceinline__ void out_tile_g(const BfFwdArgs& a, St& S, const char* lds, uint32_t wo,
                                                    float (&o)[4]) {
    preload<3, t>(S, lds);
    out_quad<t, 0>(a, S, wo, o);
    if constexpr ((t & 3) == 3) store_masks<3>(a, S);
  }
};

template <int SV>
static __device__ __forceinline__ void fwd16u_tile(const BfFwdArgs& a, int mode, const char* lds, int64_t tile,
                                                  int it, int sb) {
  using K = U2Fwd<SV>;
  using G = U2Geo;
  const int lane = threadIdx.x & 63, w = wave_id(), hh = lane >> 5;
  typename K::St S;
  S.sb = sb;
  S.uh = w >> 2;
  S.pt = w & 3;
  const int64_t p = tile * 128 + S.pt * 32 + (lane & 31);
  S.valid = p < a.P;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool inside = false;
  if (S.valid) {
    switch (mode) {
      case kPtsF64: load_point<kPtsF64>(a.src, p, x0, x1, x2, inside); break;
      case kPtsF32: load_point<kPtsF32>(a.src, p, x0, x1, x2, inside); break;
      case kRaysZ64: load_point<kRaysZ64>(a.src, p, x0, x1, x2, inside); break;
      case kPtsX4: load_point<kPtsX4>(a.src, p, x0, x1, x2, inside); break;
      default: load_point<kRaysZ32>(a.src, p, x0, x1, x2, inside); break;
    }
  }
  S.inside = inside;
  S.x0 = x0;
  S.x1 = x1;
  S.x2 = x2;
  S.col = a.save.p0 + p;
  S.mask_word0 = ((a.save.p0 + tile * 128) / 32 + S.pt) * 64;
  S.mw[0] = S.mw[1] = 0u;
  S.vmax = 0.f;
  // opaque per tile, global address space (through the asm a generic pointer would make the saves flat
  // stores, counted in lgkmcnt too and out of order): 64 save sites' addresses hoisted out of the tile
  // loop spill
  S.hrow = (__attribute__((address_space(1))) float*)(uintptr_t)(SV == 1 ? a.save.hP + S.col * kHidden + 4 * hh
                                                                          : nullptr);
  asm volatile("" : "+v"(S.hrow));
  // the raw table must have landed (prologue order: raw 2 pieces, then step 0's 4)
  if (it == 0) sync_chunk<4 * G::kD>();
  K::template fourier_tile<0>(S, lds, S.cur);
  // both halves store x (the same 16 bytes): every wave issues the store its vmcnt counts assume
  if (SV != 0 && hh == 0) a.save.xP[S.col] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
  static_assert(K::vm_ok(), "vmcnt range");
  K::start(a, S, lds);
  K::template step<0>(a, S, lds);
  // output layer: the two halves' partial sums through LDS
  uint32_t wo = lds_addr(K::raw_lds(lds) + kRawWo) + 16 * hh;
  asm volatile("" : "+v"(wo));
  float o[4] = {0.f, 0.f, 0.f, 0.f};
  K::template out_tiles<0>(a, S, lds, wo, o);
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] += __shfl_xor(o[i], 32);
  typedef float v4f __attribute__((ext_vector_type(4)));
  const uint32_t op = lds_addr(reinterpret_cast<const float*>(lds + G::kOutOff)) + (S.pt * 32 + (lane & 31)) * 16;
  if (S.uh == 1 && hh == 0)
    *reinterpret_cast<__attribute__((address_space(3))) v4f*>((uintptr_t)op) = v4f{o[0], o[1], o[2], o[3]};
  if (a.status != nullptr && !(S.vmax < 65504.f)) atomicOr(a.status, (uint32_t)PNR_STATUS_F16_RANGE);
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  if (S.uh == 0 && hh == 0) {
    const v4f q = *reinterpret_cast<const __attribute__((address_space(3))) v4f*>((uintptr_t)op);
    if (S.valid) {
      const float* rawl = K::raw_lds(lds);
      float r[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) r[i] = (o[i] + q[i]) + rawl[kRawBo + i];
      reinterpret_cast<float4*>(a.raw_out)[p] = make_float4(r[0], r[1], r[2], S.inside ? r[3] : 100.f);
    }
  }
}

template <int SV>
__global__ __launch_bounds__(512, 1) void k_mlp_fwd16u(BfFwdArgs a, int mode) {
  using K = U2Fwd<SV>;
  using G = U2Geo;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, w = wave_id();
  {  // raw table + Wo (12 KiB): pieces w and 8 + (w & 3) (waves 4-7 repeat 8-11: the same bytes, and
     // every wave issues the same count)
    const uint32_t base = lds_addr(reinterpret_cast<const float*>(lds)) + G::kRawOff;
    glds16(reinterpret_cast<const float*>(a.raw + w * 1024 + lane * 16), base + w * 1024);
    glds16(reinterpret_cast<const float*>(a.raw + (8 + (w & 3)) * 1024 + lane * 16), base + (8 + (w & 3)) * 1024);
  }
  K::template prologue<0>(a.wmain, lds);
  const int64_t ntiles = (a.P + 127) / 128;
  int sb = 0, it = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    fwd16u_tile<SV>(a, mode, lds, tile, it, sb);
    sb = (sb + G::kSteps) % G::kNbuf;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int launch_fwd16u(int mode, dim3 grid, hipStream_t st, const BfFwdArgs& a, int save);

}  // namespace pnr
