// wgrad.hip -- weight-gradient GEMMs of the decoder backward (replaces rocBLAS).
//
//   C[MA][NB] += A[MA][K] * B[NB][K]^T        (A, B unit-major: row u holds K points)
//   bias[MA]  += sum_k A[MA][k]               (optional)
//
// The K dimension (points) is huge (up to millions) and MA, NB <= 256, so the work is split
// over K: each workgroup owns KS consecutive points, streams them in tiles of 32 points through
// a double-buffered LDS image laid out point-major ([k][u], conflict-free MFMA operand reads),
// keeps its whole MA x NB partial in accumulator registers (v_mfma_f32_32x32x2_f32, exact fp32)
// and adds it into C with float atomics once at the end.
//
// Used for (src/conv_onet/models/decoder.py:149-159 parameters):
//   dW3 = delta4 . h3^T, dW2 = delta3 . h2^T, dW1 = delta2 . h1^T      MA = NB = 256
//   dW0 = delta1 . e^T                                                  MA = 256, NB = 96 (93 used)
//   dWo = g_out . h4^T                                                  MA = 4,   NB = 256
//   dB  = x . g_arg^T                                                   MA = 3,   NB = 96 (93 used)
#include "pnr_internal.h"

namespace pnr {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kKT = 32;  // points per LDS tile

template <int MT, int NT>
struct WgradCfg {
  static constexpr int MA_PAD = 32 * MT;
  static constexpr int NB_PAD = 32 * NT;
  static constexpr int SA = MA_PAD + 1;  // LDS row stride (floats): +1 makes the transposing
  static constexpr int SB = NB_PAD + 1;  // ds_write_b32 and the operand reads conflict-free
  static constexpr int TILES = MT * NT;
  static constexpr int TPW = (TILES + 3) / 4;  // output tiles per wave (round robin)
  static constexpr int A_FLOATS = kKT * SA;
  static constexpr int B_FLOATS = kKT * SB;
  static constexpr int STAGE = A_FLOATS + B_FLOATS;
};

struct WgradArgs {
  const float* A;
  int64_t lda;
  int ma;          // valid rows of A (<= 32*MT)
  const float* B;
  int64_t ldb;
  int nb;          // valid rows of B (<= 32*NT) -- also the number of C columns written
  int64_t K;       // points
  int64_t ks;      // points per workgroup (multiple of kKT)
  float* C;
  int64_t ldc;
  float* bias;     // optional row sums of A
};

// Tile load: 8 threads share one 32-point row segment (one float4 each), so every wave
// instruction reads 8 whole 128-B lines.  Thread t covers rows rep*32 + t/8, rep < NREP.
template <int NREP>
__device__ __forceinline__ void load_tile(const float* __restrict__ src, int64_t ld, int nrows, int64_t k0,
                                          int64_t ke, float4 (&v)[NREP]) {
  const int t = threadIdx.x, q = t & 7;
  const int64_t k = k0 + 4 * q;
#pragma unroll
  for (int rep = 0; rep < NREP; ++rep) {
    const int row = rep * 32 + (t >> 3);
    if (row < nrows && k + 4 <= ke) {
      v[rep] = *reinterpret_cast<const float4*>(src + (int64_t)row * ld + k);
    } else {
      float e[4] = {0.f, 0.f, 0.f, 0.f};
      if (row < nrows)
#pragma unroll
        for (int c = 0; c < 4; ++c)
          if (k + c < ke) e[c] = src[(int64_t)row * ld + k + c];
      v[rep] = make_float4(e[0], e[1], e[2], e[3]);
    }
  }
}

// transpose into the point-major LDS image: lds[k][row], row stride S
template <int NREP, int S>
__device__ __forceinline__ void store_tile(float* lds, const float4 (&v)[NREP]) {
  const int t = threadIdx.x, q = t & 7;
#pragma unroll
  for (int rep = 0; rep < NREP; ++rep) {
    const int row = rep * 32 + (t >> 3);
    float* d = lds + (4 * q) * S + row;
    d[0] = v[rep].x;
    d[S] = v[rep].y;
    d[2 * S] = v[rep].z;
    d[3 * S] = v[rep].w;
  }
}

template <int MT, int NT>
__global__ __launch_bounds__(256, 1) void k_wgrad(WgradArgs a) {
  using Cfg = WgradCfg<MT, NT>;
  constexpr int RA = MT * 32 / 32, RB = NT * 32 / 32;  // row reps per 256 threads (32 rows each)
  __shared__ __attribute__((aligned(16))) float lds[2 * Cfg::STAGE];
  const int lane = threadIdx.x & 63, hh = lane >> 5, i = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t kb = (int64_t)blockIdx.x * a.ks;
  const int64_t ke = kb + a.ks < a.K ? kb + a.ks : a.K;

  f32x16 acc[Cfg::TPW];
#pragma unroll
  for (int q = 0; q < Cfg::TPW; ++q)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[q][r] = 0.f;
  float rsum[RA];
#pragma unroll
  for (int r = 0; r < RA; ++r) rsum[r] = 0.f;

  float4 va[RA], vb[RB];
  load_tile<RA>(a.A, a.lda, a.ma, kb, ke, va);
  load_tile<RB>(a.B, a.ldb, a.nb, kb, ke, vb);
  int buf = 0;
  for (int64_t k0 = kb; k0 < ke; k0 += kKT) {
    float* la = lds + buf * Cfg::STAGE;
    float* lb = la + Cfg::A_FLOATS;
    store_tile<RA, Cfg::SA>(la, va);
    store_tile<RB, Cfg::SB>(lb, vb);
#pragma unroll
    for (int r = 0; r < RA; ++r) rsum[r] += (va[r].x + va[r].y) + (va[r].z + va[r].w);
    __syncthreads();
    if (k0 + kKT < ke) {  // prefetch the next tile into registers while this one computes
      load_tile<RA>(a.A, a.lda, a.ma, k0 + kKT, ke, va);
      load_tile<RB>(a.B, a.ldb, a.nb, k0 + kKT, ke, vb);
    }
#pragma unroll
    for (int kk = 0; kk < kKT / 2; ++kk) {
      const int kr = 2 * kk + hh;
#pragma unroll
      for (int q = 0; q < Cfg::TPW; ++q) {
        const int id = w + 4 * q;
        if (Cfg::TILES % 4 != 0 && id >= Cfg::TILES) continue;
        const int ti = id / NT, tj = id % NT;
        const float av = la[kr * Cfg::SA + 32 * ti + i];
        const float bv = lb[kr * Cfg::SB + 32 * tj + i];
        acc[q] = __builtin_amdgcn_mfma_f32_32x32x2f32(av, bv, acc[q], 0, 0, 0);
      }
    }
#pragma unroll
    for (int q = 0; q < Cfg::TPW; ++q) asm volatile("" : "+a"(acc[q]));
    buf ^= 1;
  }
  // C[32ti + perm(r,hh)][32tj + i] += acc
#pragma unroll
  for (int q = 0; q < Cfg::TPW; ++q) {
    const int id = w + 4 * q;
    if (id >= Cfg::TILES) continue;
    const int ti = id / NT, tj = id % NT;
    const int col = 32 * tj + i;
    if (col >= a.nb) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * ti + perm(r, hh);
      if (row < a.ma) atomicAdd(a.C + (int64_t)row * a.ldc + col, acc[q][r]);
    }
  }
  if (a.bias) {
#pragma unroll
    for (int r = 0; r < RA; ++r) {
      float v = rsum[r];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      const int row = r * 32 + ((int)threadIdx.x >> 3);
      if ((threadIdx.x & 7) == 0 && row < a.ma) atomicAdd(a.bias + row, v);
    }
  }
}

// choose the K split so that the grid covers the chip ~2x
static int64_t pick_ks(int64_t K) {
  int64_t ks = (K + 511) / 512;
  ks = (ks + kKT - 1) / kKT * kKT;
  if (ks < 256) ks = 256;
  return ks;
}

int launch_wgrad(int MT, int NT, const float* A, int64_t lda, int ma, const float* B, int64_t ldb, int nb, int64_t K,
                 float* C, int64_t ldc, float* bias, hipStream_t st) {
  if (K <= 0) return 0;
  WgradArgs a{A, lda, ma, B, ldb, nb, K, pick_ks(K), C, ldc, bias};
  const dim3 grid((unsigned)((K + a.ks - 1) / a.ks)), block(256);
  if (MT == 8 && NT == 8) hipLaunchKernelGGL((k_wgrad<8, 8>), grid, block, 0, st, a);
  else if (MT == 8 && NT == 3) hipLaunchKernelGGL((k_wgrad<8, 3>), grid, block, 0, st, a);
  else if (MT == 1 && NT == 8) hipLaunchKernelGGL((k_wgrad<1, 8>), grid, block, 0, st, a);
  else if (MT == 1 && NT == 3) hipLaunchKernelGGL((k_wgrad<1, 3>), grid, block, 0, st, a);
  else return PNR_E_ARG;
  return hip_status(hipGetLastError());
}

}  // namespace pnr
