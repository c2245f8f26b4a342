// mlp16w.h -- the f16x3 decoder forward in 16-point waves, two waves per SIMD (k_mlp_fwd16w).
//
// Same math as k_mlp_fwd16<PNR_PREC_F16X3, false, *> (mlp16.h; src/conv_onet/models/decoder.py:177-203
// with the bound mask of src/utils/Renderer.py:43-57): every GEMM operand split x = hi + lo in f16,
// W x ~= Wl xh + Wh xl + Wh xh with fp32 accumulation, the weights scaled by the per-tensor power of
// two of k_wscale.  What changes is the wave geometry.  k_mlp_fwd16 runs one 32-point wave per SIMD
// with both 256-unit accumulator sets in the AGPRs (512 registers: one wave per SIMD), so the epilogue
// VALU of a layer (bias, ReLU, masks, saves, the f16 split) sits in the MFMA stream of the same wave:
// an ablation without it (PNR_EXP_NOCONV) ran 22% (eval) and 33% (training) faster, i.e. it was not
// hidden.  Here a 512-thread workgroup runs the same 128-point tile as EIGHT 16-point waves, two per
// SIMD, on v_mfma_f32_16x16x32_f16:
//   A (16 output units x 32 k)  lane l: row l & 15, k = 8(l >> 4) + j
//   B (32 k x 16 points)        lane l: k = 8(l >> 4) + j, column (point) l & 15
//   D (16 units x 16 points)    lane l: column l & 15, rows 4(l >> 4) + r
// A wave still owns all 256 units of its points (acc: 2 sets x 16 tiles x 4 = 128 AGPRs), so an
// activation never leaves its lane: lane group G = l >> 4 holds units 16T + 4G + r of output tile T,
// and input tile kc (32 units) of the next layer is output tiles 2kc, 2kc + 1 -- k-slot 8G + j is unit
// 32kc + w16_kmap(8G + j), an order the weight image (k_pack16w) is laid out in.  With 256 registers
// per wave the two waves of a SIMD interleave: one wave's epilogue VALU, LDS reads and DMA issue run
// while the other issues MFMAs.  Per step every wave reads the whole 32 KiB weight slot for 16 points
// (256 KiB of ds_read_b128 per step and CU: 171 B/clk at the MFMA floor, under the 256 B/clk of the
// LDS array) and issues 4 of the step's 32 DMA pieces.
// The output layer runs on the MFMA too: Wo (4 rows, padded to 16) split hi / lo, 16 KiB resident in
// LDS for the kernel's lifetime, 3 MFMAs per h4 input tile; the lanes of group 0 hold the 4 outputs.
// Saves (training): x, h1..h4 fp32 point-major rows (16-B pieces) and the ReLU mask words in the
// layout of k_mlp_fwd16 (the delta chain and the weight-gradient GEMMs read them unchanged): lane
// groups G and G ^ 2 hold complementary bits of one 32-point lane's words (OR over lane ^ 32).
#pragma once
#include "mlp16.h"

namespace pnr {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// k-slot s = 8G + j of a hidden input tile <-> unit w16_kmap(s) within its 32 units
__host__ __device__ constexpr int w16_kmap(int s) { return (s & 7) < 4 ? 4 * (s >> 3) + (s & 7) : 12 + 4 * (s >> 3) + (s & 7); }

// image: 27 hidden steps of [T 16][part 2][lane 64][8] f16 (32 KiB each), then Wo [kc 8][part 2][lane 64][8]
constexpr int kW16Steps = 27;
constexpr int64_t kW16StepBytes = 32768;
constexpr int64_t kW16WoBytes = 8 * 2048;
constexpr int64_t kW16Bytes = kW16Steps * kW16StepBytes + kW16WoBytes;
constexpr int64_t kOffW16 = kPackedFloatsAll;  // floats, after the raw table
constexpr int64_t kPackedFloatsW16 = kOffW16 + kW16Bytes / 4;
static_assert(kOffW16 % 4 == 0, "16-B aligned image");

// PNR_W16_HSPLIT=1 (experiment, not the default): training saves of h1..h3 (L = 0..2) in split form --
// each 16-B group of 4 values holds their f16 parts {hi(v0,v1), hi(v2,v3), lo(v0,v1), lo(v2,v3)}
// (split2, unscaled), the B operand image the weight-gradient GEMMs otherwise form per tile
// (wgrad16.hip PRE); h4 stays fp32 (dWo's fp32 FMAs).  Gradients bitwise equal to the fp32 saves
// (tools/lib_ab.py), the grouped launch's VALU instructions -8.6 %, but its time unchanged at the
// room0 batch (0.161 / 0.162 ms) and -1.4 % at 4.19M points, while this kernel's training variant
// spills 35 registers instead of 15 and runs 3.7 % slower: room0 0.5109-0.5120 ms (fp32 saves)
// against 0.5171-0.5189 (profiles/r06_hsplit_ab.txt).  Not kept.
#ifndef PNR_W16_HSPLIT
#define PNR_W16_HSPLIT 0
#endif
template <int L>
constexpr bool kSplitSave = PNR_W16_HSPLIT != 0 && L < 3;

__host__ __device__ constexpr int w16_layer(int g) { return g < 3 ? 0 : 1 + (g - 3) / 8; }
__host__ __device__ constexpr int w16_kc(int g) { return g < 3 ? g : (g - 3) % 8; }
// step g converts input tile w16_ct(g) of h_{w16_cl(g)} (tile 0 of a layer in its own last step)
__host__ __device__ constexpr bool w16_conv(int g) { return !(w16_layer(g) == 0 && w16_kc(g) < 2); }
__host__ __device__ constexpr int w16_ct(int g) {
  return (w16_layer(g) == 0 || w16_kc(g) == 7) ? 0 : w16_kc(g) + 1;
}
__host__ __device__ constexpr int w16_cl(int g) {
  return w16_layer(g) == 0 ? 0 : (w16_kc(g) < 7 ? w16_layer(g) - 1 : w16_layer(g));
}

struct W16Geo {
  static constexpr int kNbuf = 4, kSlot = 32768, kD = kNbuf - 2, kSteps = kW16Steps, kNT = 16;
  static constexpr int kRawOff = kNbuf * kSlot;             // raw table (8 KiB: biases, Fourier B, scales)
  static constexpr int kWoOff = kRawOff + (int)kRawBytes;   // Wo hi / lo image (16 KiB)
  static constexpr int kLds = kWoOff + (int)kW16WoBytes;    // 152 KiB
// the group that meets the next slot: 11 in the eval kernel, 13 with training saves (A/B at 4.19M
// points, profiles/r06_fwd_variants.txt: eval 4.34 / 4.40 / 4.44 ms and training 6.37 / 5.88 / 6.54 ms at
// 11 / 13 / 14)
#ifndef PNR_W16_SYNC
#define PNR_W16_SYNC 0
#endif
#ifndef PNR_W16_RING
#define PNR_W16_RING 3
#endif
  __host__ __device__ static constexpr int sync(int sv) { return PNR_W16_SYNC ? PNR_W16_SYNC : (sv == 0 ? 11 : 13); }
  static constexpr int kRing = PNR_W16_RING, kPf = kRing - 1;  // fragment ring, groups prefetched ahead
  // epilogue pieces of a converting step: conv1 (bias, ReLU, masks) and conv2 (save, split) of
  // output tile 2 ct + q
  // Phased (PNR_W16_PHASED): the two waves of a SIMD (w and w + 4) place their epilogue in opposite
  // halves of the step -- waves 0-3 in groups 1-7, waves 4-7 in groups 9-15 -- so one wave's VALU burst
  // runs beside the other's MFMAs instead of both bursts at the same point of the lockstep schedule.
#ifndef PNR_W16_PHASED
#define PNR_W16_PHASED 0
#endif
  static constexpr bool kPhased = PNR_W16_PHASED != 0;
  __host__ __device__ static constexpr int c1(int q, int ph = 0) { return kPhased ? 1 + 4 * q + 8 * ph : 2 + 4 * q; }
  __host__ __device__ static constexpr int c2(int q, int ph = 0) { return kPhased ? 3 + 4 * q + 8 * ph : 4 + 4 * q; }
  __host__ __device__ static constexpr int cf(int ph = 0) { return kPhased ? 5 + 8 * ph : 6; }  // next Fourier tile
  static constexpr int kPhases = kPhased ? 2 : 1;
};
static_assert(W16Geo::kLds <= 160 * 1024, "LDS budget");

struct W16Frag {
  f16x8 a[2];  // hi, lo: one 16-unit output tile over one 32-deep input tile
};

struct W16State {
  f32x4 acc[2][16];  // h_L in set L & 1
  f32x4 out;
  f16x8 cur[2], nxt[2];  // B operand of the current / next input tile [part]
  f16x8 ft[3][2];        // Fourier tiles
  float v[8];            // epilogue values of the input tile being converted (2 output tiles x 4)
  float4 bq[2];          // its bias quads
  float inv;             // 2^-e of its layer's weight image
  uint32_t mw[4];        // ReLU bit words of the layer being converted (k_mlp_fwd16 layout)
  W16Frag F[W16Geo::kRing];
  float vmax;            // max |value| split into f16 parts (f16 range check)
  int sb;                // ring slot of step 0 of this tile
  int ph;                // epilogue phase of the wave (wave-uniform: waves 4-7 run theirs half a step later)
  int64_t col, mgrp;     // save row of the lane's point; its 32-point mask group
  __attribute__((address_space(1))) float* hrow;  // h save row of the lane's point (+ its 4 units), h_0's region
  float x0, x1, x2;      // the point (Fourier tiles 1, 2 are formed during steps 0, 1)
  bool valid, inside;
};

// SV: 0 eval, 1 training saves (x, masks, h1..h4), 2 masks + x only (the Tracker's camera step)
// NW: waves per workgroup -- 8 (128-point tiles, two waves per SIMD) or 4 (64-point tiles, one wave per
// SIMD: the small batches whose 128-point tiles would leave most CUs idle, k_mlp_fwd16w's launcher)
template <int SV, int NW = 8>
struct W16Fwd {
  static_assert(NW == 8 || NW == 4, "8 or 4 waves");
  static constexpr int kPer = 8 / NW;  // 4-piece DMA rounds per wave and step
  static constexpr bool SAVE = SV != 0, SAVEH = SV == 1;
  using G = W16Geo;
  static constexpr int kSteps = G::kSteps, kD = G::kD, kPf = G::kPf, kRing = G::kRing;
  static constexpr int kSync = G::sync(SV);

  __host__ __device__ static constexpr int n_glds(int g) { return g < kSteps ? 4 * kPer : 0; }
  // VMEM stores the epilogue of step g issues in group T
  __host__ __device__ static constexpr int stores_grp(int g, int T, int ph) {
    if (!SAVE || !w16_conv(g)) return 0;
    int n = 0;
    if (SAVEH && (T == G::c2(0, ph) || T == G::c2(1, ph))) ++n;
    if (w16_ct(g) == 7 && T == G::c1(1, ph)) ++n;  // the layer's mask words, after its last tile
    return n;
  }
  __host__ __device__ static constexpr int stores_rng(int g, int t0, int t1, int ph) {
    int n = 0;
    for (int T = t0; T <= t1; ++T) n += stores_grp(g, T, ph);
    return n;
  }
  // VMEM ops issued after DMA(i) and before the wait of barrier B_i (i >= 1, after group kSync of step
  // i - 1); DMA(i) goes out at B_{i-kD} (prologue / start for i <= kD).  In the persistent loop DMAs
  // i >= kSteps are the next tile's; a later tile's first barriers also see the previous tile's tail
  // stores as younger: uncounted, so their waits are only stricter.
  // (phased: the smaller count of the two phases -- a wait that counts fewer younger ops is stricter)
  __host__ __device__ static constexpr int younger_b(int i) {
    int m = younger_b_ph(i, 0);
    for (int ph = 1; ph < G::kPhases; ++ph) m = younger_b_ph(i, ph) < m ? younger_b_ph(i, ph) : m;
    return m;
  }
  __host__ __device__ static constexpr int younger_b_ph(int i, int ph) {
    int n = 0;
    for (int j = i + 1; j <= i + kD - 1; ++j) n += j < kSteps ? n_glds(j) : n_glds(j - kSteps);
    if (SAVE) {
      int first = 0;
      if (i >= kD && i - kD >= 1) {
        const int p = i - kD;
        n += stores_rng(p - 1, kSync + 1, G::kNT - 1, ph);
        first = p;
      } else {
        if (i < kD) n += 1;  // DMA(i) issued in the prologue, before the x save
        first = 0;
      }
      for (int g = first; g <= i - 2; ++g) n += stores_rng(g, 0, G::kNT - 1, ph);
      n += stores_rng(i - 1, 0, kSync, ph);
    }
    return n;
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
  // ring slot of step g (continuous numbering over the tiles of a persistent workgroup)
  static __device__ __forceinline__ const char* slot_of(const char* lds, int g, int sb) {
    return lds + ((g + sb) % G::kNbuf) * G::kSlot;
  }
  // DMA of step g (>= kSteps: the next tile's step g - kSteps): wave w copies 1-KiB pieces w + NW i
  template <int g>
  static __device__ __forceinline__ void stage_step(const char* wimg, const char* lds, int sb) {
    if constexpr (g < 2 * kSteps) {
      constexpr int st = g < kSteps ? g : g - kSteps;
      const int w = wave_id();
#pragma unroll
      for (int r = 0; r < kPer; ++r) {
        const uint32_t slot = lds_addr(reinterpret_cast<const float*>(slot_of(lds, g, sb))) + (w + NW * r) * 1024;
        const char* base = wimg;  // opaque per call: 27 steps' source pairs hoisted out of the tile loop spill SGPRs
        asm volatile("" : "+s"(base));
        glds16s_x4(base + st * kW16StepBytes + (w + NW * r) * 1024, (threadIdx.x & 63) * 16, slot);
      }
    }
  }
  // 16 B of LDS at a 32-bit LDS byte address (an opaque base stays an LDS access: ds_read_b128)
  static __device__ __forceinline__ f16x8 lds16(uint32_t addr) {
    return *reinterpret_cast<const __attribute__((address_space(3))) f16x8*>((uintptr_t)addr);
  }
  static __device__ __forceinline__ float lds4(uint32_t addr) {
    return *reinterpret_cast<const __attribute__((address_space(3))) float*>((uintptr_t)addr);
  }
  static __device__ __forceinline__ void load_frag(const char* base, W16Frag& f) {
    const int lane = threadIdx.x & 63;
    f.a[0] = *reinterpret_cast<const f16x8*>(base + lane * 16);
    f.a[1] = *reinterpret_cast<const f16x8*>(base + 1024 + lane * 16);
  }
  // acc (+)= A . act over one 32-deep input tile: Al xh + Ah xl + Ah xh
  template <bool ZERO>
  static __device__ __forceinline__ void mfma3(const W16Frag& F, const f16x8 (&act)[2], f32x4& acc) {
    f32x4 c = acc;
    if (ZERO) c = f32x4{0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(F.a[1], act[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(F.a[0], act[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_16x16x32_f16(F.a[0], act[0], c, 0, 0, 0);
    acc = c;
  }
  static __device__ __forceinline__ const float* raw_lds(const char* lds) {
    return reinterpret_cast<const float*>(lds + G::kRawOff);
  }
  // Fourier tile t of the lane's point: features 32t + 8G + j = sin(x @ B) (k_mlp_fwd16's order of
  // operations), split unscaled (|sin| <= 1).  Tile 0 before step 0, tiles 1 and 2 in steps 0 and 1.
  template <int t>
  static __device__ __forceinline__ void fourier_tile(W16State& S, const char* lds) {
    const int gq = (threadIdx.x >> 4) & 3;
    // one opaque LDS base per tile, constant offsets in the instructions (hoisted per element, the
    // 72 Fourier addresses of a persistent workgroup's tile loop spilled)
    uint32_t fb = lds_addr(raw_lds(lds) + kRawFB) + 32 * gq;
    asm volatile("" : "+v"(fb));
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 32 * t + 8 * gq + j;
      float arg;
      {
#pragma clang fp contract(off)
        arg = S.x0 * lds4(fb + 4 * (32 * t + j));
        arg = __builtin_fmaf(S.x1, lds4(fb + 4 * (kFourierPad + 32 * t + j)), arg);
        arg = __builtin_fmaf(S.x2, lds4(fb + 4 * (2 * kFourierPad + 32 * t + j)), arg);
      }
      v[j] = k < kFourier ? fourier_sc<false>(arg) : 0.f;
    }
    uint32_t h[4], l[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) split2(v[2 * j], v[2 * j + 1], h[j], l[j]);
    S.ft[t][0] = __builtin_bit_cast(f16x8, u32x4{h[0], h[1], h[2], h[3]});
    S.ft[t][1] = __builtin_bit_cast(f16x8, u32x4{l[0], l[1], l[2], l[3]});
  }
  // epilogue constants of input tile ct of h_L (read at the end of the previous step)
  template <int L, int ct>
  static __device__ __forceinline__ void preload(W16State& S, const char* lds) {
    const int gq = (threadIdx.x >> 4) & 3;
    // an opaque LDS base per read site (hoisted per (layer, tile), 64 bias addresses spilled)
    uint32_t rb = lds_addr(raw_lds(lds)) + 16 * gq;
    asm volatile("" : "+v"(rb));
    typedef float v4f __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int q = 0; q < 2; ++q) {
      const v4f b = *reinterpret_cast<const __attribute__((address_space(3))) v4f*>(
          (uintptr_t)(rb + 4 * (kRawB + L * 256 + 16 * (2 * ct + q))));
      S.bq[q] = make_float4(b.x, b.y, b.z, b.w);
    }
    S.inv = raw_lds(lds)[kRawInv + L];
  }
  // conv1: values of output tile T = 2 ct + q of h_L: relu(acc 2^-e + b), their mask bits; after the
  // layer's last tile the mask words go out (k_mlp_fwd16 layout)
  template <int L, int ct, int q>
  static __device__ __forceinline__ void conv1(const BfFwdArgs& a, W16State& S, const f32x4& src) {
    constexpr int T = 2 * ct + q;
    const int lane = threadIdx.x & 63, gq = lane >> 4;
    const float4 b = S.bq[q];
    const float b4[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float x = src[i] * S.inv + b4[i];
      S.v[4 * q + i] = x > 0.f ? x : 0.f;
    }
    if constexpr (SAVE) {
      const int sh = 16 * ((T >> 1) & 1) + 8 * (T & 1) + 4 * (gq >> 1);
      uint32_t m = 0u;
#pragma unroll
      for (int i = 0; i < 4; ++i) m |= (S.v[4 * q + i] > 0.f ? 1u : 0u) << i;
      S.mw[T >> 2] |= m << sh;
      if constexpr (T == 15) {
        uint32_t w4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) w4[k] = S.mw[k] | (uint32_t)__shfl_xor((int)S.mw[k], 32);
        if (lane < 32)
          a.save.masks[(int64_t)L * (a.save.ld / 32) * 64 + S.mgrp * 64 + gq * 32 + 16 * (wave_id() & 1) + (lane & 15)] =
              make_uint4(w4[0], w4[1], w4[2], w4[3]);
        S.mw[0] = S.mw[1] = S.mw[2] = S.mw[3] = 0u;
      }
    }
  }
  // conv2: the fp32 save of output tile 2 ct + q, the f16 range fold and the split into dwords 2q, 2q + 1
  // of the next B operand
  template <int L, int ct, int q>
  static __device__ __forceinline__ void conv2(const BfFwdArgs& a, W16State& S) {
    const int gq = (threadIdx.x >> 4) & 3;
    const float* v = S.v + 4 * q;
    (void)gq;
    typedef float v4f __attribute__((ext_vector_type(4)));
    auto* dst = reinterpret_cast<__attribute__((address_space(1))) v4f*>(S.hrow + (int64_t)L * a.save.ld * kHidden +
                                                                        16 * (2 * ct + q));
    if constexpr (SAVEH && !kSplitSave<L>) *dst = v4f{v[0], v[1], v[2], v[3]};
    S.vmax = fmaxf(S.vmax, fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3]))));
    // here, not sunk to the tile's end (which keeps every saved value alive: 232 spills)
    asm volatile("" : "+v"(S.vmax));
    uint32_t h0, l0, h1, l1;
    split2(v[0], v[1], h0, l0);
    split2(v[2], v[3], h1, l1);
    // h1..h3 are only read again as the B operands of the weight-gradient GEMMs, which split them the
    // same way (unscaled split2): the 16 B of 4 values hold their parts instead, {hi01, hi23, lo01, lo23}
    if constexpr (SAVEH && kSplitSave<L>)
      *reinterpret_cast<__attribute__((address_space(1))) u32x4*>(dst) = u32x4{h0, h1, l0, l1};
    u32x4 hv = __builtin_bit_cast(u32x4, S.nxt[0]);
    u32x4 lv = __builtin_bit_cast(u32x4, S.nxt[1]);
    hv[2 * q] = h0;
    hv[2 * q + 1] = h1;
    lv[2 * q] = l0;
    lv[2 * q + 1] = l1;
    S.nxt[0] = __builtin_bit_cast(f16x8, hv);
    S.nxt[1] = __builtin_bit_cast(f16x8, lv);
  }

  // MFMA group T of step g: prefetch, 3 MFMAs, the epilogue piece placed here, and the next step's
  // barrier / DMA / first fragments / constants
  template <int g, int T>
  static __device__ __forceinline__ void group(const BfFwdArgs& a, W16State& S, const char* lds,
                                               const f16x8 (&act)[2]) {
    if constexpr (T < G::kNT) {
      constexpr int layer = w16_layer(g), kc = w16_kc(g);
      constexpr int OUT = layer & 1;
      constexpr bool CONV = w16_conv(g);
      constexpr int CL = w16_cl(g), CT = w16_ct(g), SET = CL & 1;
      // fragment ring: group T of step g uses entry (16 g + T) mod kRing (continuous over the steps; a
      // tile's 27 x 16 groups are a multiple of kRing), and loads the entry of group T + kPf
      constexpr int RB = (G::kNT * g) % kRing;
      static_assert((G::kNT * kSteps) % kRing == 0, "ring aligned at tile boundaries");
      const char* slot = slot_of(lds, g, S.sb);
      if constexpr (T + kPf < G::kNT) load_frag(slot + (T + kPf) * 2048, S.F[(RB + T + kPf) % kRing]);
      __builtin_amdgcn_sched_barrier(0);
#if defined(PNR_EXP_NOCONV)
      constexpr bool NOCONV = true;  // experiment: no epilogue work (timing only)
#else
      constexpr bool NOCONV = false;
#endif
      mfma3<kc == 0>(S.F[(RB + T) % kRing], act, S.acc[OUT][T]);
      asm volatile("" : "+a"(S.acc[OUT][T]));
      // the next Fourier tile and the epilogue pieces, at this wave's phase (a wave-uniform branch)
#pragma unroll
      for (int ph = 0; ph < G::kPhases; ++ph) {
        if (G::kPhases == 1 || S.ph == ph) {
          if constexpr (g < 2) if (T == G::cf(ph)) fourier_tile<g + 1>(S, lds);
          if constexpr (CONV && !NOCONV) {
            if (T == G::c1(0, ph)) conv1<CL, CT, 0>(a, S, S.acc[SET][2 * CT]);
            if (T == G::c1(1, ph)) conv1<CL, CT, 1>(a, S, S.acc[SET][2 * CT + 1]);
            if (T == G::c2(0, ph)) conv2<CL, CT, 0>(a, S);
            if (T == G::c2(1, ph)) conv2<CL, CT, 1>(a, S);
          }
        }
      }
      if constexpr (g + 1 < kSteps) {
        if constexpr (T == kSync) {
          sync_chunk<younger_b(g + 1)>();
          stage_step<g + 1 + kD>(a.wmain, lds, S.sb);
        }
        if constexpr (T >= G::kNT - kPf) {
          constexpr int k = T - (G::kNT - kPf);
          load_frag(slot_of(lds, g + 1, S.sb) + k * 2048, S.F[(G::kNT * (g + 1) + k) % kRing]);
        }
        if constexpr (T == G::kNT - 1 && w16_conv(g + 1)) preload<w16_cl(g + 1), w16_ct(g + 1)>(S, lds);
      }
      __builtin_amdgcn_sched_barrier(0);
      group<g, T + 1>(a, S, lds, act);
    }
  }
  template <int g>
  static __device__ __forceinline__ void step(const BfFwdArgs& a, W16State& S, const char* lds) {
    if constexpr (g < kSteps) {
#pragma unroll
      for (int st = 0; st < 2; ++st)
#pragma unroll
        for (int t = 0; t < 16; ++t) {
          if constexpr (g == 0) asm volatile("" : "=a"(S.acc[st][t]));
          else asm volatile("" : "+a"(S.acc[st][t]));
        }
      if constexpr (w16_layer(g) == 0) {
        group<g, 0>(a, S, lds, S.ft[w16_kc(g)]);
      } else {
        S.cur[0] = S.nxt[0];
        S.cur[1] = S.nxt[1];
        group<g, 0>(a, S, lds, S.cur);
      }
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
  // barrier B_0: step 0's slot is valid; DMA of step kD; step 0's first fragments
  static __device__ __forceinline__ void start(const BfFwdArgs& a, W16State& S, const char* lds) {
    sync_chunk<younger_b0()>();
    stage_step<kD>(a.wmain, lds, S.sb);
#pragma unroll
    for (int k = 0; k < kPf; ++k) load_frag(slot_of(lds, 0, S.sb) + k * 2048, S.F[k]);
  }
  // output layer: h4 input tile t (tile 0 converted by the last hidden step) times the resident Wo image
  template <int t>
  static __device__ __forceinline__ void out_tile(const BfFwdArgs& a, W16State& S, const char* lds, uint32_t wo) {
    if constexpr (t < 8) {
      if constexpr (t > 0) {
        preload<3, t>(S, lds);
        conv1<3, t, 0>(a, S, S.acc[1][2 * t]);
        conv1<3, t, 1>(a, S, S.acc[1][2 * t + 1]);
        conv2<3, t, 0>(a, S);
        conv2<3, t, 1>(a, S);
      }
      W16Frag F;
      F.a[0] = lds16(wo + t * 2048);
      F.a[1] = lds16(wo + t * 2048 + 1024);
      mfma3<t == 0>(F, S.nxt, S.out);
      out_tile<t + 1>(a, S, lds, wo);
    }
  }
};

// one tile of k_mlp_fwd16w, 16 NW points (it: the workgroup's tile count so far, sb: its ring slot base)
template <int SV, int NW>
static __device__ __forceinline__ void fwd16w_tile(const BfFwdArgs& a, int mode, const char* lds, int64_t tile,
                                                  int it, int sb) {
  using K = W16Fwd<SV, NW>;
  using G = W16Geo;
  const int lane = threadIdx.x & 63, w = wave_id(), gq = lane >> 4;
  const int64_t p = tile * (16 * NW) + w * 16 + (lane & 15);
  W16State S;
  S.sb = sb;
  S.ph = G::kPhased ? (w >> 2) : 0;
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
  S.col = a.save.p0 + p;
  S.mgrp = (a.save.p0 + tile * (16 * NW)) / 32 + (w >> 1);
  // opaque per tile: the save addresses of 64 store sites derive from it (hoisted out of the tile loop
  // as separate 64-bit addresses they would take 128 registers)
  // (a global-address-space pointer: through the asm a generic one would turn the saves into flat
  // stores, which count in lgkmcnt too and complete out of order)
  S.hrow = (__attribute__((address_space(1))) float*)(uintptr_t)(SV == 1 ? a.save.hP + S.col * kHidden + 4 * gq
                                                                          : nullptr);
  asm volatile("" : "+v"(S.hrow));
  S.mw[0] = S.mw[1] = S.mw[2] = S.mw[3] = 0u;
  S.vmax = 0.f;
  // the raw tables must have landed (older than the step DMAs) before the Fourier features
  // (prologue order per wave: raw kPer pieces, Wo 2 kPer, steps 0 .. kD-1 4 kPer each)
  if (it == 0) sync_chunk<2 * K::kPer + 4 * K::kPer * G::kD>();
  S.x0 = x0;
  S.x1 = x1;
  S.x2 = x2;
  K::template fourier_tile<0>(S, lds);
  // always issued (the step program's vmcnt counts include it)
  if (SV != 0 && gq == 0) a.save.xP[S.col] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
  static_assert(K::vm_ok(), "vmcnt range");
  K::start(a, S, lds);
  K::template step<0>(a, S, lds);
  // Wo lies above 64 KiB of LDS: one opaque base, constant offsets in the instructions
  uint32_t wo = lds_addr(reinterpret_cast<const float*>(lds + G::kWoOff)) + lane * 16;
  asm volatile("" : "+v"(wo));
  K::template out_tile<0>(a, S, lds, wo);
  if (a.status != nullptr && !(S.vmax < 65504.f)) atomicOr(a.status, (uint32_t)PNR_STATUS_F16_RANGE);
  if (S.valid && gq == 0) {
    const float* rawl = K::raw_lds(lds);
    const float inv = rawl[kRawInv + 4];
    float o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = S.out[i] * inv + rawl[kRawBo + i];
    reinterpret_cast<float4*>(a.raw_out)[p] = make_float4(o[0], o[1], o[2], S.inside ? o[3] : 100.f);
  }
}

template <int SV, int NW>
__global__ __launch_bounds__(64 * NW, 1) void k_mlp_fwd16w(BfFwdArgs a, int mode, MapRowsArgs mr) {
  using K = W16Fwd<SV, NW>;
  using G = W16Geo;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, w = wave_id();
  const int64_t ntiles = (a.P + 16 * NW - 1) / (16 * NW);
  if (SV == 1 && mode == kMapRows) {  // (training only: launch_fwd16w refuses kMapRows otherwise)
    // the map pass's launch-A rows (map_row_point, k_map_pts's arithmetic) of this workgroup's tiles
    // into the x4 rows (src.pts, the x save), by the lanes that load them below (every lane group
    // writes its point's row: a lane reads back its own store), then the usual kPtsX4 loads.  Done
    // and drained before the first DMA, so the step program's vmcnt counts stay as they are.
    const int gq = lane >> 4;
    for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
      const int64_t p = tile * (16 * NW) + w * 16 + (lane & 15);
      if (p < a.P) {
        float x0, x1, x2;
        bool inside;
        map_row_point(mr, p, gq == 0, x0, x1, x2, inside);
        const_cast<float4*>(reinterpret_cast<const float4*>(a.src.pts))[p] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    mode = kPtsX4;
  }
  // raw table (8 KiB: 1-KiB pieces w + NW r) and the Wo image (16 KiB), then the first kD steps
#pragma unroll
  for (int r = 0; r < K::kPer; ++r) {
    const int pc = w + NW * r;
    const uint32_t base = lds_addr(reinterpret_cast<const float*>(lds)) + pc * 1024;
    glds16(reinterpret_cast<const float*>(a.raw + pc * 1024 + lane * 16), base + G::kRawOff);
  }
#pragma unroll
  for (int r = 0; r < K::kPer; ++r) {
    const int pc = w + NW * r;
    const uint32_t base = lds_addr(reinterpret_cast<const float*>(lds)) + pc * 1024;
    const char* wo = a.wmain + kW16Steps * kW16StepBytes;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      glds16(reinterpret_cast<const float*>(wo + i * 8192 + pc * 1024 + lane * 16), base + G::kWoOff + i * 8192);
  }
  K::template prologue<0>(a.wmain, lds);
  int sb = 0, it = 0;
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x, ++it) {
    fwd16w_tile<SV, NW>(a, mode, lds, tile, it, sb);
    sb = (sb + G::kSteps) % G::kNbuf;
  }
  // the last tile's prefetch of a next tile must land before the workgroup exits
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// picks the grid and NW; mr: the map rows of mode kMapRows (else null)
int launch_fwd16w(int mode, hipStream_t st, const BfFwdArgs& a, int save, const MapRowsArgs* mr);

}  // namespace pnr
