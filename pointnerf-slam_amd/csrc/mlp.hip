// mlp.hip -- fused decoder kernels for gfx950 (MI355X).
//
//   k_pack      : raw state_dict tensors -> MFMA-fragment-ordered weight image (pnr_internal.h)
//   k_mlp_fwd   : point generation (Renderer.py:177-179 / 296-298), bound mask (Renderer.py:43-57),
//                 Fourier features (decoder.py:26-30), 4 hidden layers + output layer
//                 (decoder.py:189-203), optional activation save for the backward pass
//   k_mlp_bwd   : delta chain  g_h4 = Wo^T g_out, delta_l = (W^T delta_{l+1}) * [h_l > 0],
//                 g_arg = (W0^T delta_1) * cos(x@B), optional dL/dx = B g_arg
//
// One workgroup = 4 waves (one per SIMD) = 128 points; each wave keeps its 32 points' hidden
// activations (8 tiles x 16 fp32) in registers and accumulates the next layer in 8 MFMA tiles
// (v_mfma_f32_32x32x2_f32: exact fp32 fma chain).  Weights stream through a double-buffered
// 2 x 32 KiB LDS ring filled by global_load_lds (lane-linear, the image is pre-permuted).
#include "dev_common.h"
#include "pack_fp32.h"

namespace pnr {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

#define PNR_FP_STRICT _Pragma("clang fp contract(off)")

// ---------------------------------------------------------------------------------------------
// Packing
// ---------------------------------------------------------------------------------------------
__global__ void k_pack(RawParams rp, float* __restrict__ out) {
  pack_fp32_at(rp, out, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

int launch_pack(const RawParams& rp, float* packed, hipStream_t st) {
  const int threads = 256;
  const int blocks = (int)((kPackedFloats + threads - 1) / threads);
  hipLaunchKernelGGL(k_pack, dim3(blocks), dim3(threads), 0, st, rp, packed);
  return hip_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Building blocks
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// acc[t] += A(chunk, tile t) * act  over the 16 k-steps of one 32-row input tile.
// A fragments are read from LDS one r-quad ahead (ds_read_b128, conflict-free lane-linear
// image); the sched barriers keep at most two r-quads of A (2 x NT x 4 VGPRs) live.
template <int NT>
__device__ __forceinline__ void load_a(const float* chunk, int rq, float4 (&a)[NT]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < NT; ++t) a[t] = *reinterpret_cast<const float4*>(chunk + ((t * 4 + rq) * 64 + lane) * 4);
}
template <int NT>
__device__ __forceinline__ void mfma_rq(const float4 (&a)[NT], const float (&b)[16], int rq, f32x16 (&acc)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = mfma(a[t].x, b[4 * rq + 0], acc[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = mfma(a[t].y, b[4 * rq + 1], acc[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = mfma(a[t].z, b[4 * rq + 2], acc[t]);
#pragma unroll
  for (int t = 0; t < NT; ++t) acc[t] = mfma(a[t].w, b[4 * rq + 3], acc[t]);
}
template <int NT>
__device__ __forceinline__ void mfma_chunk(const float* chunk, const float (&b)[16], f32x16 (&acc)[NT]) {
  float4 a0[NT], a1[NT];
  load_a<NT>(chunk, 0, a0);
  load_a<NT>(chunk, 1, a1);
  mfma_rq<NT>(a0, b, 0, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_a<NT>(chunk, 2, a0);
  mfma_rq<NT>(a1, b, 1, acc);
  __builtin_amdgcn_sched_barrier(0);
  load_a<NT>(chunk, 3, a1);
  mfma_rq<NT>(a0, b, 2, acc);
  __builtin_amdgcn_sched_barrier(0);
  mfma_rq<NT>(a1, b, 3, acc);
  __builtin_amdgcn_sched_barrier(0);
}

// One layer: NCH input tiles streamed as NCH LDS chunks of `chf` floats from cursor `sp`; the
// chunk after the last one (`nxf` floats from cursor `nsp`, 0 = none) is prefetched during the
// last compute.  `buf` (wave-uniform) is the LDS buffer of the current chunk and is advanced.
// `stores0` (wave-uniform) tells the first chunk's sync that N0 stores were issued after its DMA.
template <int NCH, int NT, int N0>
__device__ __forceinline__ void layer(float* lds, const float*& sp, int chf, const float*& nsp, int nxf, int& buf,
                                      const float (&act)[8][16], f32x16 (&acc)[NT], bool stores0) {
#pragma unroll
  for (int c = 0; c < NCH; ++c) {
    if (c == 0 && stores0) sync_chunk<N0>();
    else sync_chunk<0>();
    float* cur = lds + buf * kChunkFloats;
    float* oth = lds + (buf ^ 1) * kChunkFloats;
    if (c + 1 < NCH) stage(sp, oth, chf);
    else if (nxf > 0) stage(nsp, oth, nxf);
    mfma_chunk<NT>(cur, act[c], acc);
    // Pin the accumulators here: without it hipcc defers half of the MFMA chains past the next
    // s_barrier (MFMAs touch no memory), keeps their A fragments alive and spills ~250 VGPRs.
#pragma unroll
    for (int t = 0; t < NT; ++t) asm volatile("" : "+a"(acc[t]));
    buf ^= 1;
  }
}

// One LDS chunk holding 8 k-tiles of 1024 floats (W^T images of fc_c): acc += sum_kc A_kc act[kc]
template <int N0>
__device__ __forceinline__ void chunk8(float* lds, const float*& nsp, int nxf, int& buf, const float (&act)[8][16],
                                       f32x16 (&acc)[1], bool stores0) {
  if (stores0) sync_chunk<N0>();
  else sync_chunk<0>();
  float* cur = lds + buf * kChunkFloats;
  if (nxf > 0) stage(nsp, lds + (buf ^ 1) * kChunkFloats, nxf);
#pragma unroll
  for (int kc = 0; kc < 8; ++kc) mfma_chunk<1>(cur + kc * kSmallChunkFloats, act[kc], acc);
  asm volatile("" : "+a"(acc[0]));
  buf ^= 1;
}

template <int NT>
__device__ __forceinline__ void zero_acc(f32x16 (&acc)[NT]) {
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
}

// act = relu(acc + bias), bias image [t][rq][lane][4]; one tile of bias live at a time
__device__ __forceinline__ void bias_relu(const f32x16 (&acc)[8], const float* __restrict__ img, float (&act)[8][16]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
      const float4 b = *reinterpret_cast<const float4*>(img + ((t * 4 + rq) * 64 + lane) * 4);
      const float v0 = acc[t][4 * rq + 0] + b.x, v1 = acc[t][4 * rq + 1] + b.y;
      const float v2 = acc[t][4 * rq + 2] + b.z, v3 = acc[t][4 * rq + 3] + b.w;
      act[t][4 * rq + 0] = v0 > 0.f ? v0 : 0.f;
      act[t][4 * rq + 1] = v1 > 0.f ? v1 : 0.f;
      act[t][4 * rq + 2] = v2 > 0.f ? v2 : 0.f;
      act[t][4 * rq + 3] = v3 > 0.f ? v3 : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// act += acc + bias  (feature branch fc_c[i](c) added after the ReLU, decoder.py:196-197)
__device__ __forceinline__ void add_bias_acc(const f32x16 (&acc)[8], const float* __restrict__ img,
                                             float (&act)[8][16]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int t = 0; t < 8; ++t) {
#pragma unroll
    for (int rq = 0; rq < 4; ++rq) {
      const float4 b = *reinterpret_cast<const float4*>(img + ((t * 4 + rq) * 64 + lane) * 4);
      act[t][4 * rq + 0] += acc[t][4 * rq + 0] + b.x;
      act[t][4 * rq + 1] += acc[t][4 * rq + 1] + b.y;
      act[t][4 * rq + 2] += acc[t][4 * rq + 2] + b.z;
      act[t][4 * rq + 3] += acc[t][4 * rq + 3] + b.w;
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// B-operand tile of the 32 feature channels of this lane's point: register r = channel perm(r,hh)
// (4 float4 loads of the point's (32,) row).  Zero for invalid points.
__device__ __forceinline__ void load_c_tile(const float* __restrict__ c, int64_t p, bool valid, float (&ct)[8][16]) {
  const int hh = (threadIdx.x >> 5) & 1;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (valid) v = *reinterpret_cast<const float4*>(c + p * kCDim + 8 * q + 4 * hh);
    ct[0][4 * q + 0] = v.x; ct[0][4 * q + 1] = v.y; ct[0][4 * q + 2] = v.z; ct[0][4 * q + 3] = v.w;
  }
}

// store NT tiles of the register activation into a point-major [rows][W] buffer (row = point):
// registers 4q..4q+3 of tile t are units 32t + 8q + 4hh + {0..3}, one 16-B store each.
template <int NT, int W>
__device__ __forceinline__ void save_tiles(float* __restrict__ row, const float (&act)[8][16]) {
  const int hh = (threadIdx.x >> 5) & 1;
  float* q0 = row + 4 * hh;
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      *reinterpret_cast<float4*>(q0 + 32 * t + 8 * q) =
          make_float4(act[t][4 * q], act[t][4 * q + 1], act[t][4 * q + 2], act[t][4 * q + 3]);
}

// ReLU mask of one lane: bit (t&1)*16 + r of word t>>1 is [act[t][r] > 0]; the wave tile's
// 64 lanes store one uint4 each (1 KiB per 32 points per layer).
__device__ __forceinline__ void save_mask(uint4* __restrict__ words, const float (&act)[8][16]) {
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) w[t >> 1] |= (act[t][r] > 0.f ? 1u : 0u) << ((t & 1) * 16 + r);
  words[threadIdx.x & 63] = make_uint4(w[0], w[1], w[2], w[3]);
}

// ---------------------------------------------------------------------------------------------
// Forward
// ---------------------------------------------------------------------------------------------
struct FwdArgs {
  const float* packed;
  PointSrc src;
  int64_t P;
  float* raw;
  SaveArgs save;
  int do_save;
  FeatArgs feat;
};

// VMEM stores issued between a layer's prefetch DMA and the next layer's first sync (a lower
// bound is safe: it only makes the wait stricter): e + x saves = 13, mask + h saves = 33,
// mask only = 1, delta saves = 32, delta + dL/dh saves = 64.
constexpr int kStoresE = 12, kStoresH = 32, kStoresM = 1, kStoresD = 31, kStoresDG = 62;

// torch CPU computes the K=3 product x @ B as fma(x2,B2, fma(x1,B1, x0*B0)) (verified bitwise)
__device__ __forceinline__ float fourier_arg(const float* __restrict__ FB, int k, float x0, float x1, float x2) {
  PNR_FP_STRICT
  float a = x0 * FB[k];
  a = __builtin_fmaf(x1, FB[kFourierPad + k], a);
  a = __builtin_fmaf(x2, FB[2 * kFourierPad + k], a);
  return a;
}

// Weight streams: the main image in layer order (L0F, L1F, L2F, L3F, OF) and, with features
// (HASC), the fc_c image (CF0..CF3); the chunk sequence is L0 [C0] L1 [C1] L2 [C2] L3 [C3] O.
template <int MODE, bool HASC>
__global__ __launch_bounds__(256, 1) void k_mlp_fwd(FwdArgs a) {
  __shared__ __attribute__((aligned(16))) float lds[2 * kChunkFloats];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = (int64_t)blockIdx.x * 128 + wave * 32 + j;
  const bool valid = p < a.P;
  const float* __restrict__ W = a.packed;
  const int lane_off = wave_id() * 256 + lane * 4;

  const float* sp = W + kOffL0F + lane_off;  // weight stream cursors
  const float* spc = HASC ? a.feat.fcw + kOffCF + lane_off : sp;
  int buf = 0;
  stage(sp, lds, kChunkFloats);  // chunk 0 of layer 0 -> buffer 0

  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool inside = false;
  if (valid) load_point<MODE>(a.src, p, x0, x1, x2, inside);

  float act[8][16];
  const float* FB = W + kOffFB;
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = 32 * t + perm(r, hh);
      act[t][r] = k < kFourier ? sinf(fourier_arg(FB, k, x0, x1, x2)) : 0.f;
    }
  // training saves cover every point of the (128-padded) grid: padded columns get finite
  // activations of x = 0 and a zero gradient later, so the weight GEMMs may include them
  const bool save = a.do_save;
  const int64_t col = a.save.p0 + p;
  // first saved column of this wave (p0 is a multiple of 128) -> its 64 mask slots
  const int64_t mask_word0 = ((a.save.p0 + (int64_t)blockIdx.x * 128) / 32 + wave_id()) * 64;
  if (save) {
    save_tiles<3, kFourierPad>(a.save.eP + col * kFourierPad, act);
    if (hh == 0) a.save.xP[col] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
  }

  f32x16 acc[8];
  // epilogue of hidden layer L: ReLU (+ mask save), feature branch, activation save
  auto finish = [&](int L) {
    bias_relu(acc, W + kOffB0 + (int64_t)L * kBiasFloats, act);
    if (save) save_mask(a.save.masks + (int64_t)L * (a.save.ld / 32) * 64 + mask_word0, act);
    if (HASC) {  // h += fc_c[L](c): one chunk, K = 32 channels
      float ct[8][16];
      load_c_tile(a.feat.c, p, valid, ct);
      zero_acc<8>(acc);
      layer<1, 8, kStoresM>(lds, spc, kChunkFloats, sp, L < 3 ? kChunkFloats : kSmallChunkFloats, buf, ct, acc, save);
      add_bias_acc(acc, a.feat.fcw + kOffCB + (int64_t)L * kBiasFloats, act);
    }
    if (save) save_tiles<8, kHidden>(a.save.hP + ((int64_t)L * a.save.ld + col) * kHidden, act);
  };
  zero_acc<8>(acc);
  layer<3, 8, kStoresE>(lds, sp, kChunkFloats, HASC ? spc : sp, kChunkFloats, buf, act, acc, save);
  finish(0);
  // hidden layers 1..3 (pts_linears.1..3)
  for (int L = 1; L <= 3; ++L) {
    const int nxf = HASC ? kChunkFloats : (L < 3 ? kChunkFloats : kSmallChunkFloats);
    zero_acc<8>(acc);
    layer<8, 8, kStoresH>(lds, sp, kChunkFloats, HASC ? spc : sp, nxf, buf, act, acc, save);
    finish(L);
  }

  f32x16 out[1];
  zero_acc<1>(out);
  layer<8, 1, kStoresH>(lds, sp, kSmallChunkFloats, sp, 0, buf, act, out, save);
  // rows 0..3 of the output tile live in lanes 0..31, registers 0..3
  if (valid && hh == 0) {
    const float4 bo = *reinterpret_cast<const float4*>(W + kOffBO + lane * 4);
    float4 o = make_float4(out[0][0] + bo.x, out[0][1] + bo.y, out[0][2] + bo.z, inside ? out[0][3] + bo.w : 100.f);
    reinterpret_cast<float4*>(a.raw)[p] = o;
  }
}

template <bool HASC>
static void launch_fwd_mode(int mode, dim3 grid, dim3 block, hipStream_t st, const FwdArgs& a) {
  switch (mode) {
    case kPtsF64: hipLaunchKernelGGL((k_mlp_fwd<kPtsF64, HASC>), grid, block, 0, st, a); break;
    case kPtsF32: hipLaunchKernelGGL((k_mlp_fwd<kPtsF32, HASC>), grid, block, 0, st, a); break;
    case kRaysZ64: hipLaunchKernelGGL((k_mlp_fwd<kRaysZ64, HASC>), grid, block, 0, st, a); break;
    case kPtsX4: hipLaunchKernelGGL((k_mlp_fwd<kPtsX4, HASC>), grid, block, 0, st, a); break;
    default: hipLaunchKernelGGL((k_mlp_fwd<kRaysZ32, HASC>), grid, block, 0, st, a); break;
  }
}

int launch_mlp_fwd(const float* packed, const PointSrc& src, int mode, int64_t P, float* raw,
                   const SaveArgs* save, hipStream_t st, const FeatArgs* feat) {
  if (P <= 0) return 0;
  if (mode < kPtsF64 || mode > kPtsX4) return PNR_E_ARG;
  FwdArgs a;
  a.packed = packed;
  a.src = src;
  a.P = P;
  a.raw = raw;
  a.do_save = save != nullptr;
  if (save) a.save = *save;
  else a.save = SaveArgs{nullptr, nullptr, nullptr, nullptr, 0, 0};
  a.feat = feat ? *feat : FeatArgs{nullptr, nullptr};
  const dim3 grid((unsigned)((P + 127) / 128)), block(256);
  TimingScope ts(kTimeMlpFwd, P, st);
  if (a.feat.fcw) launch_fwd_mode<true>(mode, grid, block, st, a);
  else launch_fwd_mode<false>(mode, grid, block, st, a);
  return hip_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Backward delta chain
// ---------------------------------------------------------------------------------------------
// act = acc * [h > 0]; the ReLU mask comes from the forward's per-lane bit words
__device__ __forceinline__ void relu_grad(const f32x16 (&acc)[8], const uint4* __restrict__ words,
                                          float (&act)[8][16]) {
  const uint4 m = words[threadIdx.x & 63];
  const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) act[t][r] = ((w[t >> 1] >> ((t & 1) * 16 + r)) & 1u) ? acc[t][r] : 0.f;
}

// act *= [h > 0] in place
__device__ __forceinline__ void relu_mask(const uint4* __restrict__ words, float (&act)[8][16]) {
  const uint4 m = words[threadIdx.x & 63];
  const uint32_t w[4] = {m.x, m.y, m.z, m.w};
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) act[t][r] = ((w[t >> 1] >> ((t & 1) * 16 + r)) & 1u) ? act[t][r] : 0.f;
}

__device__ __forceinline__ void acc_to_act(const f32x16 (&acc)[8], float (&act)[8][16]) {
#pragma unroll
  for (int t = 0; t < 8; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) act[t][r] = acc[t][r];
}

// Weight streams: transposed images W3^T, W2^T, W1^T (8 chunks each), W0^T (8 chunks of 3072);
// with features (HASC) the fc_c^T images CT3..CT0 (one chunk each) precede W3^T .. W0^T.
template <bool HASC>
__global__ __launch_bounds__(256, 1) void k_mlp_bwd(const float* __restrict__ W, BwdArgs a, int64_t P) {
  __shared__ __attribute__((aligned(16))) float lds[2 * kChunkFloats];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, hh = lane >> 5, j = lane & 31;
  const int64_t p = (int64_t)blockIdx.x * 128 + wave * 32 + j;  // chunk-local point
  const bool valid = p < P;
  const int64_t col = a.p0 + p;   // column in the saved activations
  const int64_t dcol = p;         // column in the delta buffers
  const int64_t mstride = (a.ld / 32) * 64;  // mask slots per layer
  // delta saves are skipped for invalid lanes only; a wave with no valid lane issues no store
  // instruction at all, so the relaxed first-chunk wait is used only when some lane is valid
  const bool valid_any = __builtin_amdgcn_readfirstlane((int)((int64_t)blockIdx.x * 128 + wave_id() * 32 < P));
  const uint4* mk = a.masks + ((a.p0 + (int64_t)blockIdx.x * 128) / 32 + wave_id()) * 64;
  const int lane_off = wave_id() * 256 + lane * 4;

  const float* sp = W + kOffL3T + lane_off;  // weight stream cursors
  const float* spc = HASC ? a.fcw + kOffCT + lane_off : sp;
  int buf = 0;
  if (HASC) stage(spc, lds, kChunkFloats);  // CT3 -> buffer 0
  else stage(sp, lds, kChunkFloats);        // W3^T chunk 0 -> buffer 0 (lands during the Wo^T step)

  // g_h4 = Wo^T g_out  (K = 4: k-steps r = 0..3, lane half 0 carries o = r)
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  if (valid && hh == 0) {
    const float4 go = reinterpret_cast<const float4*>(a.g_out)[p];
    g[0] = go.x; g[1] = go.y; g[2] = go.z; g[3] = go.w;
  }
  f32x16 acc[8];
  zero_acc<8>(acc);
  {
    const float* OT = W + kOffOT;
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const float4 w4 = *reinterpret_cast<const float4*>(OT + (t * 64 + lane) * 4);
      acc[t] = mfma(w4.x, g[0], acc[t]);
      acc[t] = mfma(w4.y, g[1], acc[t]);
      acc[t] = mfma(w4.z, g[2], acc[t]);
      acc[t] = mfma(w4.w, g[3], acc[t]);
    }
  }
  f32x16 gc[1];  // dL/dc = sum_l Wc_l^T dL/dh_l  (32 channels x 32 points)
  zero_acc<1>(gc);
  float act[8][16];
  // acc = dL/dh_l (hl = mask index) -> act = delta_l; with features, dL/dh_l also feeds Wc_l^T
  // and is saved for dWc_l; `nxf` = size of the chunk after CT_l (the next W^T chunk)
  auto to_delta = [&](int hl, int nxf) {
    if (HASC) {
      acc_to_act(acc, act);
      chunk8<0>(lds, sp, nxf, buf, act, gc, false);
      if (valid) save_tiles<8, kHidden>(a.gH + ((int64_t)hl * a.ld_d + dcol) * kHidden, act);
      relu_mask(mk + hl * mstride, act);
    } else {
      relu_grad(acc, mk + hl * mstride, act);
    }
    if (valid) save_tiles<8, kHidden>(a.dP + ((int64_t)hl * a.ld_d + dcol) * kHidden, act);
  };
  to_delta(3, kChunkFloats);  // delta4

  // delta3 = W3^T delta4 * [h3>0]; delta2; delta1  (images L3T, L2T, L1T; 8 chunks each)
  constexpr int NS = HASC ? kStoresDG : kStoresD;
  for (int s = 0; s < 3; ++s) {  // s=0: W3^T -> delta3 (uses h3), s=1: W2^T -> delta2, s=2: W1^T -> delta1
    const int nxw = s < 2 ? kChunkFloats : (int)kL0TChunkFloats;  // next W^T chunk
    zero_acc<8>(acc);
    layer<8, 8, NS>(lds, sp, kChunkFloats, HASC ? spc : sp, HASC ? kChunkFloats : nxw, buf, act, acc, valid_any);
    to_delta(2 - s, nxw);  // h3 -> index 2, h2 -> 1, h1 -> 0
  }

  // g_e = W0^T delta1 : 3 output tiles (96 rows, 93 valid)
  f32x16 ge[3];
  zero_acc<3>(ge);
  layer<8, 3, NS>(lds, sp, (int)kL0TChunkFloats, sp, 0, buf, act, ge, valid_any);

  // g_arg = g_e * cos(x@B); g_x = B g_arg
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  if (valid) {
    const float4 xv = a.xP[col];
    x0 = xv.x; x1 = xv.y; x2 = xv.z;
  }
  const float* FB = W + kOffFB;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f;
  float garg[8][16];  // only tiles 0..2 used (save_tiles layout)
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = 32 * t + perm(r, hh);
      float gv = 0.f;
      if (k < kFourier) {
        gv = ge[t][r] * cosf(fourier_arg(FB, k, x0, x1, x2));
        s0 = __builtin_fmaf(FB[k], gv, s0);
        s1 = __builtin_fmaf(FB[kFourierPad + k], gv, s1);
        s2 = __builtin_fmaf(FB[2 * kFourierPad + k], gv, s2);
      }
      garg[t][r] = gv;
    }
  if (valid) save_tiles<3, kFourierPad>(a.gargP + dcol * kFourierPad, garg);
  if (HASC && valid) {
#pragma unroll
    for (int r = 0; r < 16; ++r) garg[0][r] = gc[0][r];
    save_tiles<1, kCDim>(a.g_c + dcol * kCDim, garg);
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

int launch_mlp_bwd(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st) {
  if (P <= 0) return 0;
  const dim3 grid((unsigned)((P + 127) / 128)), block(256);
  TimingScope ts(kTimeMlpBwd, P, st);
  if (a.fcw) hipLaunchKernelGGL(k_mlp_bwd<true>, grid, block, 0, st, packed, a, P);
  else hipLaunchKernelGGL(k_mlp_bwd<false>, grid, block, 0, st, packed, a, P);
  return hip_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// fc_c image (pnr_internal.h "fc_c image"): fc[2l] = fc_c.l.weight (256,32), fc[2l+1] = bias
// ---------------------------------------------------------------------------------------------
__global__ void k_fc_pack(FcRaw fc, float* __restrict__ out) {
  fc_pack_fp32_at(fc, out, (int64_t)blockIdx.x * blockDim.x + threadIdx.x);
}

int launch_fc_pack(const float* const* fc, float* out, hipStream_t st) {
  FcRaw r;
  for (int i = 0; i < PNR_N_FC_PARAMS; ++i) r.p[i] = fc[i];
  const int threads = 256;
  hipLaunchKernelGGL(k_fc_pack, dim3((unsigned)((kFcPackedFloats + threads - 1) / threads)), dim3(threads), 0, st,
                     r, out);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
