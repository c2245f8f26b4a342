// wgrad.hip -- weight-gradient GEMMs of the decoder backward.
//
//   C[MA][NB] += A[K][MA]^T * B[K][NB]        (A, B point-major: row k = one point)
//   bias[MA]  += sum_k A[k][MA]               (optional)
//
// K (points) is huge (up to millions) and MA, NB <= 256, so the work is split over K: each
// workgroup owns KS consecutive points and streams them in tiles of 32 points.  A tile of a
// point-major operand is one contiguous block (32 x MA floats), copied linearly into LDS with
// 16-B loads/stores (register double-buffering); the MFMA operand reads of that [k][u] image are
// conflict-free (lanes read consecutive units).  The whole MA x NB partial stays in accumulator
// registers (v_mfma_f32_32x32x2_f32, exact fp32) and is stored as this workgroup's partial tile;
// k_part_reduce (wgrad16.hip) adds the partials into C in a fixed order (deterministic).
//
// Used for (src/conv_onet/models/decoder.py:149-159 parameters):
//   dW3 = delta4^T h3, dW2 = delta3^T h2, dW1 = delta2^T h1     MA = NB = 256
//   dW0 = delta1^T e                                            MA = 256, NB = 96 (93 used)
//   dWo = g_out^T h4                                            MA = 4,   NB = 256
//   dB  = x^T g_arg                                             MA = 4 (3 used), NB = 96 (93 used)
//   dWc_l = (dL/dh_l)^T c  (fc_c, neural-point features)        MA = 256, NB = 32
#include "pnr_internal.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kKT = 32;  // points per LDS tile

template <int MT, int NT, int WA, int WB>
struct WgradCfg {
  static constexpr int TILES = MT * NT;
  // wave w owns row tiles [w*RW, w*RW+RW) x all NT col tiles (MT >= 4), or col tiles
  // [w*CW, w*CW+CW) of the single row tile (MT == 1): per k-step it reads RW A and CW B
  // fragments for RW*CW MFMAs
  static constexpr int RW = MT >= 4 ? MT / 4 : 1;
  static constexpr int CW = MT >= 4 ? NT : (NT + 3) / 4;
  static constexpr int TPW = RW * CW;
  static constexpr int A_FLOATS = kKT * WA;
  static constexpr int B_FLOATS = kKT * WB;
  static constexpr int STAGE = A_FLOATS + B_FLOATS;
  static constexpr int A_V4 = (A_FLOATS / 4 + 255) / 256;  // float4 per thread per tile
  static constexpr int B_V4 = (B_FLOATS / 4 + 255) / 256;
};

struct WgradArgs {
  const float* A;  // [K][WA]
  int ma;          // valid columns of A (rows of C)
  const float* B;  // [K][WB]
  int nb;          // valid columns of B (columns of C)
  int64_t K;
  int64_t ks;      // points per workgroup (multiple of kKT)
  float* part;     // [grid][ma][NT 32] partial tiles
  float* pbias;    // [grid][ma] partial column sums of A (bias non-null)
  bool bias;
};

// load one 32-point tile (rows k0.. of a [K][W] operand) as float4 per thread, zero past ke
template <int W, int NV4>
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int64_t k0, int64_t ke, float4 (&v)[NV4]) {
  constexpr int N4 = kKT * W / 4;
  const int64_t lim = (ke - k0) * W / 4;  // valid float4 of this tile
  const float4* s4 = reinterpret_cast<const float4*>(src + k0 * W);
#pragma unroll
  for (int q = 0; q < NV4; ++q) {
    const int e = q * 256 + threadIdx.x;
    v[q] = (e < N4 && e < lim) ? s4[e] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

template <int W, int NV4>
__device__ __forceinline__ void store_tile(float* lds, const float4 (&v)[NV4]) {
  constexpr int N4 = kKT * W / 4;
#pragma unroll
  for (int q = 0; q < NV4; ++q) {
    const int e = q * 256 + threadIdx.x;
    if (e < N4) reinterpret_cast<float4*>(lds)[e] = v[q];
  }
}

template <int MT, int NT, int WA, int WB>
__global__ __launch_bounds__(256, 1) void k_wgrad(WgradArgs a) {
  using Cfg = WgradCfg<MT, NT, WA, WB>;
  __shared__ __attribute__((aligned(16))) float lds[2 * Cfg::STAGE];
  const int lane = threadIdx.x & 63, hh = lane >> 5, i = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t kb = (int64_t)blockIdx.x * a.ks;
  const int64_t ke = kb + a.ks < a.K ? kb + a.ks : a.K;
  const int tr0 = MT >= 4 ? w * Cfg::RW : 0;
  const int tc0 = MT >= 4 ? 0 : w * Cfg::CW;

  f32x16 acc[Cfg::TPW];
#pragma unroll
  for (int q = 0; q < Cfg::TPW; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  float csum = 0.f;  // bias: thread u < ma sums column u of A

  float4 va[Cfg::A_V4], vb[Cfg::B_V4];
  load_tile<WA, Cfg::A_V4>(a.A, kb, ke, va);
  load_tile<WB, Cfg::B_V4>(a.B, kb, ke, vb);
  int buf = 0;
  for (int64_t k0 = kb; k0 < ke; k0 += kKT) {
    float* la = lds + buf * Cfg::STAGE;
    float* lb = la + Cfg::A_FLOATS;
    store_tile<WA, Cfg::A_V4>(la, va);
    store_tile<WB, Cfg::B_V4>(lb, vb);
    __syncthreads();
    if (k0 + kKT < ke) {  // prefetch the next tile into registers while this one computes
      load_tile<WA, Cfg::A_V4>(a.A, k0 + kKT, ke, va);
      load_tile<WB, Cfg::B_V4>(a.B, k0 + kKT, ke, vb);
    }
    if (a.bias && (int)threadIdx.x < a.ma) {  // column sums, 4 independent chains
      float c0 = 0.f, c1 = 0.f, c2 = 0.f, c3 = 0.f;
#pragma unroll
      for (int k = 0; k < kKT; k += 4) {
        c0 += la[(k + 0) * WA + threadIdx.x];
        c1 += la[(k + 1) * WA + threadIdx.x];
        c2 += la[(k + 2) * WA + threadIdx.x];
        c3 += la[(k + 3) * WA + threadIdx.x];
      }
      csum += (c0 + c1) + (c2 + c3);
    }
#pragma unroll
    for (int kk = 0; kk < kKT / 2; ++kk) {
      const int kr = 2 * kk + hh;
      float av[Cfg::RW], bv[Cfg::CW];
#pragma unroll
      for (int x = 0; x < Cfg::RW; ++x) {
        const int ra = 32 * (tr0 + x) + i;
        av[x] = ra < WA ? la[kr * WA + ra] : 0.f;
      }
#pragma unroll
      for (int y = 0; y < Cfg::CW; ++y) {
        const int rb = 32 * (tc0 + y) + i;
        bv[y] = (tc0 + y < NT && rb < WB) ? lb[kr * WB + rb] : 0.f;
      }
#pragma unroll
      for (int x = 0; x < Cfg::RW; ++x)
#pragma unroll
        for (int y = 0; y < Cfg::CW; ++y)
          acc[x * Cfg::CW + y] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[x], bv[y], acc[x * Cfg::CW + y], 0, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < Cfg::TPW; ++q) asm volatile("" : "+a"(acc[q]));
    buf ^= 1;
  }
  // this workgroup's partial tile: part[blk][row][32 tj + i] (rows < ma)
  float* P = a.part + (int64_t)blockIdx.x * a.ma * (NT * 32);
#pragma unroll
  for (int x = 0; x < Cfg::RW; ++x)
#pragma unroll
    for (int y = 0; y < Cfg::CW; ++y) {
      const int ti = tr0 + x, tj = tc0 + y;
      if (tj >= NT) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * ti + perm(r, hh);
        if (row < a.ma) P[row * (NT * 32) + 32 * tj + i] = acc[x * Cfg::CW + y][r];
      }
    }
  if (a.bias && (int)threadIdx.x < a.ma) a.pbias[(int64_t)blockIdx.x * a.ma + threadIdx.x] = csum;
}

// choose the K split so that the grid covers the chip ~2x (<= kWgradMaxWg partial tiles)
static int64_t pick_ks(int64_t K) {
  int64_t ks = (K + kWgradMaxWg - 1) / kWgradMaxWg;
  ks = (ks + kKT - 1) / kKT * kKT;
  if (ks < 256) ks = 256;
  return ks;
}

int launch_wgrad(int kind, const float* A, int ma, const float* B, int nb, int64_t K, float* C, int64_t ldc,
                 float* bias, float* part, float* part_bias, hipStream_t st) {
  if (K <= 0) return 0;
  if (!part || !part_bias) return PNR_E_ARG;
  WgradArgs a{A, ma, B, nb, K, pick_ks(K), part, part_bias, bias != nullptr};
  const int nwg = (int)((K + a.ks - 1) / a.ks);
  const dim3 grid((unsigned)nwg), block(256);
  TimingScope ts(kTimeWgrad, K, st);
  int nt;
  switch (kind) {
    case kWgradHidden: nt = 8; hipLaunchKernelGGL((k_wgrad<8, 8, 256, 256>), grid, block, 0, st, a); break;
    case kWgradFirst: nt = 3; hipLaunchKernelGGL((k_wgrad<8, 3, 256, 96>), grid, block, 0, st, a); break;
    case kWgradOut: nt = 8; hipLaunchKernelGGL((k_wgrad<1, 8, 4, 256>), grid, block, 0, st, a); break;
    case kWgradFourier: nt = 3; hipLaunchKernelGGL((k_wgrad<1, 3, 4, 96>), grid, block, 0, st, a); break;
    case kWgradFc: nt = 1; hipLaunchKernelGGL((k_wgrad<8, 1, 256, 32>), grid, block, 0, st, a); break;
    default: return PNR_E_ARG;
  }
  const int rc = hip_status(hipGetLastError());
  return rc ? rc : launch_part_reduce(part, part_bias, nwg, ma, 32 * nt, nb, C, ldc, bias, st);
}

}  // namespace pnr
