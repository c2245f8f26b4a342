// mlp16_pack.hip -- 16-bit weight images of the split-precision decoder kernels (mlp16.h) and
// the forward dispatch on PNR_PREC_*.
#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <unordered_map>

#include "mlp16.h"
#include "mlp16w.h"
#include "pack_fp32.h"

namespace pnr {

int64_t packed_floats_all() { return kPackedFloatsW16; }
int64_t fc_packed_floats_all() { return kFcPackedFloatsAll; }
// ---------------------------------------------------------------------------------------------
// Packing
// ---------------------------------------------------------------------------------------------
// Per-tensor power-of-two scale of the f16 images: s = 2^e, e = floor(log2(2^14 / max|W|)),
// clamped to [-20, 20]; scl[i] = s, inv[i] = 1/s (both exact).  One 1024-thread block per tensor.
struct ScaleArgs {
  const float* w[5];
  int n[5];
  float* inv;
  float* scl;
};
__device__ __forceinline__ void wscale_block(const ScaleArgs& a, const int b) {
  __shared__ float red[16];
  const float* w = a.w[0];  // a.w[b], a.n[b] without a private copy of the arrays (b is uniform)
  int n = a.n[0];
#pragma unroll
  for (int k = 1; k < 5; ++k) {
    w = b == k ? a.w[k] : w;
    n = b == k ? a.n[k] : n;
  }
  const int nt = blockDim.x, nw = nt >> 6;  // any multiple of 64 up to 1024
  // 32 loads in flight per thread (one pass covers a 256 x 256 tensor at 1024 threads x 2): the
  // reduction is one block per tensor, so its time is the number of dependent load rounds
  float m = 0.f;
  for (int i0 = 0; i0 < n; i0 += 32 * nt) {
    float v[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) {  // clamped, unconditional loads (a repeated element leaves the max
      const int i = i0 + k * nt + (int)threadIdx.x;  // alone): a predicated load waits on its own
      v[k] = fabsf(w[i < n ? i : n - 1]);
    }
#pragma unroll
    for (int k = 0; k < 32; ++k) m = fmaxf(m, v[k]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < nw; ++k) red[0] = fmaxf(red[0], red[k]);
    int e = 20;
    if (red[0] > 0.f) {
      int ex;
      frexpf(16384.f / red[0], &ex);  // 16384/max = f 2^ex, f in [0.5,1)
      e = ex - 1;                     // 2^e <= 16384/max
      e = e < -20 ? -20 : (e > 20 ? 20 : e);
    }
    a.scl[b] = ldexpf(1.f, e);
    a.inv[b] = ldexpf(1.f, -e);
  }
}
__global__ __launch_bounds__(1024) void k_wscale(ScaleArgs a) { wscale_block(a, blockIdx.x); }

template <typename E>
__device__ __forceinline__ uint16_t part_bits(float x, int part) {
  const E h = (E)x;
  const E v = part == 0 ? h : (E)(x - (float)h);
  return __builtin_bit_cast(uint16_t, v);
}

// element (T, s, part, lane, j) of a weight fragment image for a layer with A[row][k]:
// row = 32T + (lane&31), k = 32kc + perm(8s+j, lane>>5).  img 0: BF16X3, 1: BF16, 2: F16X3.
__device__ __forceinline__ void pack16_at(const RawParams& rp, uint16_t* __restrict__ bf2, uint16_t* __restrict__ bf1,
                                          uint16_t* __restrict__ h2, float* __restrict__ raw, const int64_t idx64) {
  constexpr int n2 = (int)(bf_main_bytes(2) / 2), n1 = (int)(bf_main_bytes(1) / 2);
  static_assert(2LL * n2 + n1 < (1LL << 30), "32-bit pack indices");
  if (idx64 < 2 * n2 + n1) {
    const int idx = (int)idx64;  // 32-bit index arithmetic (64-bit divisions dominated the pack)
    const int img = idx < n2 ? 0 : (idx < n2 + n1 ? 1 : 2);
    const int np = img == 1 ? 1 : 2;
    const int e0 = img == 0 ? idx : (img == 1 ? idx - n2 : idx - n2 - n1);
    int e = e0;
    const int hstep = np * 8192;  // 16-bit elements per hidden step
    float v = 0.f;
    int part = 0, tensor = 4;
    if (e < 27 * hstep) {
      const int g = e / hstep;
      int r = e - g * hstep;
      const int j = r & 7; r >>= 3;
      const int lane = r & 63; r >>= 6;
      part = r % np; r /= np;
      const int s = r & 1;
      const int T = r >> 1;
      const int layer = g < 3 ? 0 : 1 + (g - 3) / 8;
      const int kc = g < 3 ? g : (g - 3) % 8;
      const int row = 32 * T + (lane & 31);
      const int k = 32 * kc + perm(8 * s + j, lane >> 5);
      const float* W = rp.at(1 + 2 * layer);
      tensor = layer;
      if (layer == 0) v = k < kFourier ? W[row * kFourier + k] : 0.f;
      else v = W[row * kHidden + k];
    } else {
      e -= 27 * hstep;
      const int kc = e >> 11;
      int r = e & 2047;  // 4 KiB piece = 2048 elements
      if (r < np * 1024) {
        const int j = r & 7; r >>= 3;
        const int lane = r & 63; r >>= 6;
        part = r % np;
        const int s = r / np;
        const int row = lane & 31;
        const int k = 32 * kc + perm(8 * s + j, lane >> 5);
        v = row < 4 ? rp.p[9][row * kHidden + k] : 0.f;
      }
    }
    if (img == 2) h2[e0] = part_bits<_Float16>(v * raw[kRawScl + tensor], part);
    else (img == 0 ? bf2 : bf1)[e0] = part_bits<__bf16>(v, part);
    return;
  }
  const int64_t idx = idx64;
  const int64_t ri = idx - 2 * n2 - n1;
  if (ri >= kRawWo && ri < kRawWo + 4 * kHidden) {  // Wo fp32 (the VALU output layer)
    raw[ri] = rp.p[9][ri - kRawWo];
    return;
  }
  if (ri < kRawInv) {
    float v = 0.f;
    const int i = (int)ri;
    if (i < kRawBo) v = rp.at(2 + 2 * (i / 256))[i % 256];
    else if (i < kRawFB) v = (i - kRawBo) < 4 ? rp.p[10][i - kRawBo] : 0.f;
    else {
      const int c = (i - kRawFB) / kFourierPad, k = (i - kRawFB) % kFourierPad;
      v = k < kFourier ? rp.p[0][c * kFourier + k] : 0.f;
    }
    raw[i] = v;
  }
}

// Transposed f16x3 images of the delta chain (element e of the backward stream), each tensor
// scaled by the forward image's power of two (raw[kRawScl + tensor], k_wscale)
__device__ __forceinline__ void pack16_bwd_at(const RawParams& rp, uint16_t* __restrict__ out,
                                              const float* __restrict__ raw, const int64_t e) {
  if (e >= kBwdBytes / 2) return;
  static_assert(kBwdBytes < (1LL << 31), "32-bit pack indices");
  const int byte = 2 * (int)e;
  static_assert(bwd_main_off(1) == 16384 && bwd_main_off(25) == 16384 + 24 * 32768 && kBwdSteps == 33, "bwd steps");
  // step g of byte (bwd_main_off): 16 KiB for Wo^T, 24 x 32 KiB for W3..W1, 8 x 12 KiB for W0^T
  const int g = byte < 16384 ? 0 : (byte < 16384 + 24 * 32768 ? 1 + ((byte - 16384) >> 15)
                                                                : 25 + (byte - 16384 - 24 * 32768) / 12288);
  int r = (byte - (int)bwd_main_off(g)) >> 1;
  const int j = r & 7; r >>= 3;
  const int lane = r & 63; r >>= 6;
  const int part = r & 1; r >>= 1;
  float v = 0.f;
  int tensor = 4;
  if (g == 0) {  // Wo^T: A[row = unit 32T + i][k = o = perm(j, hh)], k < 4
    const int T = r, row = 32 * T + (lane & 31), k = perm(j, lane >> 5);
    v = k < 4 ? rp.p[9][k * kHidden + row] : 0.f;
  } else {
    const int s = r & 1, T = r >> 1;
    const int row = 32 * T + (lane & 31);
    const int kc = g <= 24 ? (g - 1) % 8 : g - 25;
    const int k = 32 * kc + perm(8 * s + j, lane >> 5);
    if (g <= 24) {
      const int l = 3 - (g - 1) / 8;  // W3, W2, W1
      v = rp.at(1 + 2 * l)[k * kHidden + row];
      tensor = l;
    } else {
      v = row < kFourier ? rp.p[1][k * kFourier + row] : 0.f;
      tensor = 0;
    }
  }
  out[e] = part_bits<_Float16>(v * raw[kRawScl + tensor], part);
}

// The 16-point-wave forward image (mlp16w.h, element e of kW16Bytes / 2): 27 hidden steps of
// A[row = 16T + (lane & 15)][k] over [T 16][part 2][lane 64][j 8], k = 32kc + 8(lane >> 4) + j for the
// Fourier layer and 32kc + w16_kmap(8(lane >> 4) + j) for the hidden ones; then Wo (rows 0..3 of 16) per
// h4 input tile [kc 8][part 2][lane 64][j 8].  f16x3 parts under the forward image's scales.
__device__ __forceinline__ void pack16w_at(const RawParams& rp, uint16_t* __restrict__ out,
                                           const float* __restrict__ raw, const int e) {
  constexpr int hstep = (int)(kW16StepBytes / 2);
  static_assert(kW16Bytes / 2 < (1LL << 31), "32-bit pack indices");
  if (e >= (int)(kW16Bytes / 2)) return;
  float v = 0.f;
  int part, tensor;
  if (e < kW16Steps * hstep) {
    const int g = e / hstep;
    int r = e - g * hstep;
    const int j = r & 7; r >>= 3;
    const int lane = r & 63; r >>= 6;
    part = r & 1;
    const int T = r >> 1;
    const int layer = w16_layer(g), kc = w16_kc(g);
    const int row = 16 * T + (lane & 15), s = 8 * (lane >> 4) + j;
    const float* W = rp.at(1 + 2 * layer);
    tensor = layer;
    if (layer == 0) {
      const int k = 32 * kc + s;
      v = k < kFourier ? W[row * kFourier + k] : 0.f;
    } else {
      v = W[row * kHidden + 32 * kc + w16_kmap(s)];
    }
  } else {
    int r = e - kW16Steps * hstep;
    const int j = r & 7; r >>= 3;
    const int lane = r & 63; r >>= 6;
    part = r & 1;
    const int kc = r >> 1, row = lane & 15;
    v = row < 4 ? rp.p[9][row * kHidden + 32 * kc + w16_kmap(8 * (lane >> 4) + j)] : 0.f;
    tensor = 4;
  }
  out[e] = part_bits<_Float16>(v * raw[kRawScl + tensor], part);
}

// The weight images of every precision in two launches (the Mapper repacks once per iteration, and
// at its 1,000-ray batch each launch costs ~5 us of latency on the step's critical path):
//   stage 1: blocks 0..4 the power-of-two weight scales (k_wscale), the rest the fp32 image (k_pack)
//   stage 2: the transposed f16x3 delta-chain images, then the forward 16-bit images and the raw
//            table (k_pack16_bwd, k_pack16) -- both read stage 1's scales
// (the fp32 image is grid-strided over at most kPack1Blocks blocks: the scale blocks' registers allow
// one 1,024-thread block per CU, so a block per 1,024 elements took two rounds)
// flags (pnr_mlp_pack2 / pnr_fc_pack2): PNR_PACK_F16X3_ONLY -- only the images the f16x3 kernels read
// (stage 1: the scale blocks alone, no fp32 image; stage 2: no bf16 images).
constexpr int kPack1Blocks = 248;
__global__ __launch_bounds__(1024) void k_pack_stage1(ScaleArgs sa, RawParams rp, float* __restrict__ packed,
                                                      int nscale) {
  if ((int)blockIdx.x < nscale) {
    wscale_block(sa, blockIdx.x);
    return;
  }
  const int64_t stride = (int64_t)(gridDim.x - nscale) * 1024;
  for (int64_t i = (int64_t)(blockIdx.x - nscale) * 1024 + threadIdx.x; i < kPackedFloats; i += stride)
    pack_fp32_at(rp, packed, i);
}
__global__ __launch_bounds__(256) void k_pack_stage2(RawParams rp, float* __restrict__ packed, int nb_bwd,
                                                     int nb16, int64_t base16) {
  float* raw = packed + kOffRaw;
  if ((int)blockIdx.x >= nb_bwd + nb16)  // the 16-point-wave forward image (after the raw table)
    pack16w_at(rp, reinterpret_cast<uint16_t*>(packed + kOffW16), raw, ((int)blockIdx.x - nb_bwd - nb16) * 256 + threadIdx.x);
  else if ((int)blockIdx.x < nb_bwd)
    pack16_bwd_at(rp, reinterpret_cast<uint16_t*>(packed + kOffBwd), raw, (int64_t)blockIdx.x * 256 + threadIdx.x);
  else
    pack16_at(rp, reinterpret_cast<uint16_t*>(packed + kOffBf2), reinterpret_cast<uint16_t*>(packed + kOffBf1),
              reinterpret_cast<uint16_t*>(packed + kOffH2), raw,
              base16 + (int64_t)(blockIdx.x - nb_bwd) * 256 + threadIdx.x);
}

int launch_pack_all(const RawParams& rp, float* packed, hipStream_t st, int flags) {
  float* raw = packed + kOffRaw;
  ScaleArgs sa;
  const int nw[5] = {kHidden * kFourier, kHidden * kHidden, kHidden * kHidden, kHidden * kHidden, 4 * kHidden};
  for (int i = 0; i < 5; ++i) {
    sa.w[i] = rp.p[i < 4 ? 1 + 2 * i : 9];
    sa.n[i] = nw[i];
  }
  sa.inv = raw + kRawInv;
  sa.scl = raw + kRawScl;
  const int nscale = 5;
  const int nimg = (flags & PNR_PACK_F16X3_ONLY) ? 0 : (int)std::min<int64_t>(kPack1Blocks, (kPackedFloats + 1023) / 1024);
  hipLaunchKernelGGL(k_pack_stage1, dim3(nscale + nimg), dim3(1024), 0, st, sa, rp, packed, nscale);
  const int nb_bwd = (int)((kBwdBytes / 2 + 255) / 256);
  constexpr int64_t n2 = bf_main_bytes(2) / 2, n1 = bf_main_bytes(1) / 2;
  const int64_t n16 = 2 * n2 + n1 + kRawWo + 4 * kHidden;
  const int64_t base16 = (flags & PNR_PACK_F16X3_ONLY) ? n2 + n1 : 0;  // from the f16x3 main image on
  const int nb16 = (int)((n16 - base16 + 255) / 256);
  const int nbw = (int)((kW16Bytes / 2 + 255) / 256);
  hipLaunchKernelGGL(k_pack_stage2, dim3(nb_bwd + nb16 + nbw), dim3(256), 0, st, rp, packed, nb_bwd, nb16, base16);
  return hip_status(hipGetLastError());
}

struct FcRaw16 {
  const float* p[PNR_N_FC_PARAMS];
  __device__ __forceinline__ const float* at(int i) const {  // see RawParams::at
    const float* r = p[0];
#pragma unroll
    for (int k = 1; k < PNR_N_FC_PARAMS; ++k) r = i == k ? p[k] : r;
    return r;
  }
};

// fc entry e = 8L + t: A[row = unit 32t + (lane&31)][k = channel perm(8s+j, lane>>5)] of Wc_L
__device__ __forceinline__ void fc_pack16_at(const FcRaw16& fc, uint16_t* __restrict__ bf2, uint16_t* __restrict__ bf1,
                                             uint16_t* __restrict__ h2, float* __restrict__ raw, int64_t idx) {
  const int64_t n = kBfFcBytes / 2;  // elements per image
  if (idx < 3 * n) {
    const int img = (int)(idx / n);
    const int np = img == 1 ? 1 : 2;
    const int64_t e = idx % n;
    const int ent = (int)(e / 2048);
    int64_t r = e % 2048;
    float v = 0.f;
    int part = 0;
    const int L = ent / 8, t = ent % 8;
    if (r < (int64_t)np * 1024) {
      const int j = (int)(r % 8); r /= 8;
      const int lane = (int)(r % 64); r /= 64;
      part = (int)(r % np);
      const int s = (int)(r / np);
      const int unit = 32 * t + (lane & 31);
      const int ch = perm(8 * s + j, lane >> 5);
      v = fc.at(2 * L)[unit * kCDim + ch];
    }
    if (img == 2) h2[e] = part_bits<_Float16>(v * raw[kFcRawScl + L], part);
    else (img == 0 ? bf2 : bf1)[e] = part_bits<__bf16>(v, part);
    return;
  }
  const int64_t ri = idx - 3 * n;
  if (ri < kFcRawInv) raw[ri] = fc.at(2 * (int)(ri / 256) + 1)[ri % 256];
}

// fc backward entry e = 8(3 - l) + t: A[row = channel (lane&31)][k = unit 32t + perm(8s+j, lane>>5)]
// = Wc_l[unit][channel], f16x3 scaled like the forward image (raw[kFcRawScl + l])
__device__ __forceinline__ void fc_pack16_bwd_at(const FcRaw16& fc, uint16_t* __restrict__ out,
                                                 const float* __restrict__ raw, int64_t e) {
  if (e >= kBfFcBytes / 2) return;
  const int ent = (int)(e / 2048);
  int64_t r = e % 2048;
  const int j = (int)(r % 8); r /= 8;
  const int lane = (int)(r % 64); r /= 64;
  const int part = (int)(r % 2);
  const int s = (int)(r / 2);
  const int l = 3 - ent / 8, t = ent % 8;
  const int unit = 32 * t + perm(8 * s + j, lane >> 5);
  out[e] = part_bits<_Float16>(fc.at(2 * l)[unit * kCDim + (lane & 31)] * raw[kFcRawScl + l], part);
}

// The fc_c images in two launches, as the main images (launch_pack_all): stage 1 the four fc weight
// scales (blocks 0..3) and the fp32 image, stage 2 the forward 16-bit images with the fc raw table and
// the transposed f16x3 backward image (both read stage 1's scales).  Four launches before: ~10 us of
// latency per Mapper iteration at the neural-point configs' real batches.
constexpr int64_t kFc16N = 3 * (kBfFcBytes / 2) + kFcRawInv;  // stage-2 elements of the forward images
__global__ __launch_bounds__(1024) void k_fc_stage1(ScaleArgs sa, FcRaw fr, float* __restrict__ out, int nscale) {
  if ((int)blockIdx.x < nscale) {
    wscale_block(sa, blockIdx.x);
    return;
  }
  const int64_t stride = (int64_t)(gridDim.x - nscale) * 1024;
  for (int64_t i = (int64_t)(blockIdx.x - nscale) * 1024 + threadIdx.x; i < kFcPackedFloats; i += stride)
    fc_pack_fp32_at(fr, out, i);
}
__global__ __launch_bounds__(256) void k_fc_stage2(FcRaw16 fc, float* __restrict__ out, int64_t base) {
  float* raw = out + kOffFcRaw;
  const int64_t idx = base + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx < kFc16N)
    fc_pack16_at(fc, reinterpret_cast<uint16_t*>(out + kOffFcBf2), reinterpret_cast<uint16_t*>(out + kOffFcBf1),
                 reinterpret_cast<uint16_t*>(out + kOffFcH2), raw, idx);
  else
    fc_pack16_bwd_at(fc, reinterpret_cast<uint16_t*>(out + kOffFcBwd), raw, idx - kFc16N);
}

int launch_fc_pack_all(const float* const* fcp, float* out, hipStream_t st, int flags) {
  FcRaw16 r;
  FcRaw fr;
  for (int i = 0; i < PNR_N_FC_PARAMS; ++i) r.p[i] = fr.p[i] = fcp[i];
  float* raw = out + kOffFcRaw;
  ScaleArgs sa{};
  for (int i = 0; i < 4; ++i) {
    sa.w[i] = fcp[2 * i];
    sa.n[i] = kHidden * kCDim;
  }
  sa.inv = raw + kFcRawInv;
  sa.scl = raw + kFcRawScl;
  const int nscale = 4;
  const int nimg = (flags & PNR_PACK_F16X3_ONLY) ? 0 : (int)std::min<int64_t>(64, (kFcPackedFloats + 1023) / 1024);
  hipLaunchKernelGGL(k_fc_stage1, dim3(nscale + nimg), dim3(1024), 0, st, sa, fr, out, nscale);
  const int64_t n2 = kFc16N + kBfFcBytes / 2;
  const int64_t base = (flags & PNR_PACK_F16X3_ONLY) ? 2 * (kBfFcBytes / 2) : 0;  // from the f16x3 image on
  hipLaunchKernelGGL(k_fc_stage2, dim3((unsigned)((n2 - base + 255) / 256)), dim3(256), 0, st, r, out, base);
  return hip_status(hipGetLastError());
}

// The f16x3 forward without features: k_mlp_fwd16w (16-point waves, two per SIMD, mlp16w.h) by
// default, k_mlp_fwd16 (32-point waves, one per SIMD) with PNR_FWD_VARIANT=0 (environment, read per
// launch: A/B runs).  Measured (tools/w16_ab.py, 4.19M points, one process, interleaved rounds,
// profiles/r06_fwd_variants.txt): eval 4.34 against 4.69 ms, training 5.88 against 6.16 ms.  (The
// output-unit split over two waves per SIMD, k_mlp_fwd16u, measured 5.08-5.16 / 7.20-7.37 ms and was
// removed.)
int fwd16_variant(int save) {
  const char* e = getenv("PNR_FWD_VARIANT");
  (void)save;
  return e ? atoi(e) : 1;
}

// the f16x3 forward without the feature branch runs k_mlp_fwd16w (variant 1), whose saves are split
bool fwd_saves_split(int prec, const FeatArgs* feat) {
  return PNR_W16_HSPLIT != 0 && prec == PNR_PREC_F16X3 && !(feat && feat->fcw) && fwd16_variant(1) == 1;
}

namespace {
std::mutex g_hsave_mu;
std::unordered_map<const float*, bool> g_hsave;
}  // namespace
void hsave_set_split(const float* hP, bool split) {
  std::lock_guard<std::mutex> lk(g_hsave_mu);
  if (g_hsave.size() > 4096) g_hsave.clear();  // stale areas (freed workspaces): every forward re-marks its own
  g_hsave[hP] = split;
}
bool hsave_is_split(const float* hP) {
  std::lock_guard<std::mutex> lk(g_hsave_mu);
  const auto it = g_hsave.find(hP);
  return it != g_hsave.end() && it->second;
}

bool fwd_map_rows_ok(int prec, const FeatArgs* feat) {
  return prec == PNR_PREC_F16X3 && !(feat && feat->fcw) && fwd16_variant(1) == 1;
}

int launch_mlp_fwd_bf(int prec, const float* packed, const PointSrc& src, int mode, int64_t P, float* raw,
                      const SaveArgs* save, hipStream_t st, const FeatArgs* feat, uint32_t* status,
                      const MapRowsArgs* mr) {
  if (P <= 0) return 0;
  if (mode < kPtsF64 || mode > kMapRows) return PNR_E_ARG;
  if (mode == kMapRows && !fwd_map_rows_ok(prec, feat)) return PNR_E_ARG;  // k_mlp_fwd16w only
  if (prec != PNR_PREC_BF16X3 && prec != PNR_PREC_BF16 && prec != PNR_PREC_F16X3) return PNR_E_ARG;
  BfFwdArgs a;
  a.wmain = reinterpret_cast<const char*>(packed + main_off_floats(prec));
  a.raw = reinterpret_cast<const char*>(packed + kOffRaw);
  const bool hasc = feat && feat->fcw;
  a.wfc = hasc ? reinterpret_cast<const char*>(feat->fcw + fc_off_floats(prec)) : nullptr;
  a.fcraw = hasc ? reinterpret_cast<const char*>(feat->fcw + kOffFcRaw) : nullptr;
  a.c = hasc ? feat->c : nullptr;
  a.src = src;
  a.P = P;
  a.raw_out = raw;
  a.status = status;
  // 0 no saves, 1 masks + inputs + activations, 2 masks + inputs (hP NULL: no weight gradients)
  const int sv = save == nullptr ? 0 : (save->hP != nullptr ? 1 : 2);
  if (save) a.save = *save;
  else a.save = SaveArgs{nullptr, nullptr, nullptr, nullptr, 0, 0};
  // one workgroup per 128-point tile; the persistent kernels (no feature branch) loop over tiles
  // on at most one workgroup per CU
  int64_t nwg = (P + 127) / 128;
  if (!hasc) {
    const int ncu = device_cu_count();
    nwg = nwg < ncu ? nwg : ncu;
  }
  const dim3 grid((unsigned)nwg);
  TimingScope ts(kTimeMlpFwd, P, st);
  if (prec == PNR_PREC_F16X3 && !hasc) {
    const int var = fwd16_variant(sv);
    if (var == 1) {  // 16-point waves (mlp16w.h)
      BfFwdArgs b = a;
      b.wmain = reinterpret_cast<const char*>(packed + kOffW16);
      return launch_fwd16w(mode, st, b, sv, mode == kMapRows ? mr : nullptr);
    }
  }
  switch (prec) {
    case PNR_PREC_BF16X3: return launch_fwd16_bf16x3(mode, grid, st, a, hasc, sv);
    case PNR_PREC_BF16: return launch_fwd16_bf16(mode, grid, st, a, hasc, sv);
    default: return launch_fwd16_f16x3(mode, grid, st, a, hasc, sv);
  }
}

int64_t packed_raw_wo_offset() { return kOffRaw + kRawWo; }
int64_t packed_raw_fb_offset() { return kOffRaw + kRawFB; }

}  // namespace pnr
