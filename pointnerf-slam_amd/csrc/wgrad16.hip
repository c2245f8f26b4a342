// wgrad16.hip -- weight-gradient GEMMs of the decoder backward for the split precisions.
//
//   C[256][NB] += s^-1 * A[K][256]^T B[K][WB]     (A, B point-major f16: row k = one point)
//   bias[256]  += s^-1 * sum_k A[k][:]            (optional)
//
// Used for every precision but PNR_PREC_FP32 (wgrad.hip keeps the fp32 form) on the two large shapes
// of src/conv_onet/models/decoder.py:149-159:
//   dW3 = delta4^T h3, dW2 = delta3^T h2, dW1 = delta2^T h1     WB = 256 (8 column tiles)
//   dW0 = delta1^T e                                            WB = 96 (3 column tiles, 93 used)
// A = deltas stored by k_mlp_bwd16 as f16 * s (s = 2^e from max |g_out|, delta_scale), B = f16
// activations stored by k_mlp_fwd16.  The products of f16 values are exact in fp32, so the only
// error is the one storage rounding of each operand (<= 2^-12 relative).
//
// The training step is HBM-bound on these operands: the kernel only moves them.  K (points) is
// split over workgroups of 8 waves (2 per SIMD).  Each 32-point tile of A and B goes straight from
// HBM into LDS by global_load_lds (16-B pieces: the LDS side is lane-linear, the source address is
// free, so the DMA itself lays the tile out as [32-column block T][32 points][64 B]); a 4-slot ring
// keeps 3 tiles (~100 KB) in flight per CU.  The MFMA operands need 8 consecutive points of one
// column per lane: ds_read_b64_tr_b16 reads them transposed out of the image (a 16-lane group
// covers 4 rows x 32 B = 64 distinct banks; cdna_hip_programming.md T10).  Wave w owns output rows
// [32w, 32w + 32) x all NB columns in NTB accumulator tiles for the whole K range, added into C with
// one float atomic per element at the end.  The bias row sums come from the A fragments.
// K must be a multiple of 32 and rows in [real K, K) zero in A (padded points: delta = 0).
#include <cmath>
#include "mlp16.h"

namespace pnr {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int kTileB = 2112;  // bytes of one [32 points][64 B] block, +64 B pad (store banks)

template <int NTB, int WB>
struct Wg16 {
  static constexpr int kThreads = 512;                     // 8 waves, 2 per SIMD
  // B blocks staged: a multiple of 4 so every wave issues the same DMA pieces (dW0: 4 with one
  // duplicate, dWc: 4 with three duplicates of the one 32-column block)
  static constexpr int kTB = NTB < 4 ? 4 : NTB;
  static constexpr int kImgA = 8 * kTileB;
  static constexpr int kSlot = kImgA + kTB * kTileB;
  static constexpr int kNbuf = 4, kDist = kNbuf - 1;
  static constexpr int kLds = kNbuf * kSlot;
  // DMA pieces (1 KiB = 16 points x 64 B of one block) per wave per tile: A 16 / 8 waves, B 2 kTB / 8
  static constexpr int kPA = 2, kPB = 2 * kTB / 8;
  static constexpr int kPieces = kPA + kPB;
};

struct Wg16Args {
  const _Float16* A;   // [K][256]
  const _Float16* B;   // [K][WB]
  int nb;              // valid columns of B (columns of C)
  int64_t K;           // multiple of 32
  int64_t ks;          // points per workgroup (multiple of 32)
  float* C;
  int64_t ldc;
  float* bias;
  const uint32_t* gmax;  // scale of A: delta_scale(*gmax)
};

__device__ __forceinline__ void glds16b(const void* gsrc, uint32_t lds_byte) {
  glds16(reinterpret_cast<const float*>(gsrc), lds_byte);
}

// stage 32-point tile k0 into `slot`: piece pc of an operand = (block T = pc >> 1, half h = pc & 1),
// lane L -> point 16h + (L >> 2), 16-B chunk (L & 3) of the block's 64 B
template <int NTB, int WB>
__device__ __forceinline__ void stage_tile(const Wg16Args& a, int64_t k0, uint32_t slot) {
  using Cfg = Wg16<NTB, WB>;
  const int w = wave_id(), L = threadIdx.x & 63;
  const int row = L >> 2, c16 = L & 3;
#pragma unroll
  for (int i = 0; i < Cfg::kPA; ++i) {
    const int pc = w + 8 * i, T = pc >> 1, h = pc & 1;
    const char* src = reinterpret_cast<const char*>(a.A + (k0 + 16 * h + row) * 256) + T * 64 + c16 * 16;
    glds16b(src, slot + T * kTileB + h * 1024);
  }
#pragma unroll
  for (int i = 0; i < Cfg::kPB; ++i) {
    const int pc = w + 8 * i, T = pc >> 1, h = pc & 1;
    const int Ts = T < NTB ? T : 0;  // dW0: the 4th block duplicates block 0 (never read)
    const char* src = reinterpret_cast<const char*>(a.B + (k0 + 16 * h + row) * WB) + Ts * 64 + c16 * 16;
    glds16b(src, slot + Cfg::kImgA + T * kTileB + h * 1024);
  }
}

// MFMA operand of 32-column block T, k-step s: lane l holds column 32T + (l&31), points
// 16s + 8(l>>5) + j, j = 0..7 (two transposed reads; lane 4q+p of 16-lane group g supplies point
// 16s + 8(g>>1) + q (+4), columns 16(g&1) + 4p .. +3)
__device__ __forceinline__ f16x8 tr_frag(const char* img, int T, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, q = (l >> 2) & 3, p = l & 3;
  const char* base = img + T * kTileB + (16 * s + 8 * (g >> 1) + q) * 64 + 32 * (g & 1) + 8 * p;
  const v4i16 x = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)base);
  const v4i16 y = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(base + 4 * 64));
  const short e[8] = {x[0], x[1], x[2], x[3], y[0], y[1], y[2], y[3]};
  f16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __builtin_bit_cast(_Float16, e[j]);
  return r;
}

template <int NTB, int WB>
__global__ __launch_bounds__(512, 1) void k_wgrad16(Wg16Args a) {
  using Cfg = Wg16<NTB, WB>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int lane = threadIdx.x & 63, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // output row block of this wave
  const int64_t kb = (int64_t)blockIdx.x * a.ks;
  const int64_t ke = kb + a.ks < a.K ? kb + a.ks : a.K;
  const int64_t ntile = (ke - kb) / 32;
  const uint32_t lbase = lds_addr(reinterpret_cast<const float*>(lds));

  f32x16 acc[NTB];
#pragma unroll
  for (int y = 0; y < NTB; ++y)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[y][r] = 0.f;
  float cs = 0.f;  // row sums of A (bias) for column 32w + (lane & 31), this lane half's points

  // the ring always issues exactly kDist tiles ahead (the tail re-stages the last tile into the
  // free slot) so that every wait below has the same constant count
#pragma unroll
  for (int t = 0; t < Cfg::kDist; ++t)
    stage_tile<NTB, WB>(a, kb + 32 * (t < ntile ? t : ntile - 1), lbase + t * Cfg::kSlot);
  for (int64_t t = 0; t < ntile; ++t) {
    sync_chunk<(Cfg::kDist - 1) * Cfg::kPieces>();  // this wave's pieces of tile t landed; all waves met
    {
      const int64_t tn = t + Cfg::kDist < ntile ? t + Cfg::kDist : ntile - 1;
      stage_tile<NTB, WB>(a, kb + 32 * tn, lbase + (uint32_t)(((t + Cfg::kDist) % Cfg::kNbuf) * Cfg::kSlot));
    }
    const char* ia = lds + (t % Cfg::kNbuf) * Cfg::kSlot;
    const char* ib = ia + Cfg::kImgA;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const f16x8 af = tr_frag(ia, w, s);
#pragma unroll
      for (int j = 0; j < 8; ++j) cs += (float)af[j];
#pragma unroll
      for (int y = 0; y < NTB; ++y)
        acc[y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(af, tr_frag(ib, y, s), acc[y], 0, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the re-staged tail DMAs
  const float inv = 1.f / delta_scale(*a.gmax);
  // C[32w + perm(r,hh)][32y + (lane&31)] += acc / s
#pragma unroll
  for (int y = 0; y < NTB; ++y) {
    const int col = 32 * y + (lane & 31);
    if (col >= a.nb) continue;
#pragma unroll
    for (int r = 0; r < 16; ++r) atomicAdd(a.C + (int64_t)(32 * w + perm(r, hh)) * a.ldc + col, acc[y][r] * inv);
  }
  cs += __shfl_xor(cs, 32);
  if (a.bias && hh == 0) atomicAdd(a.bias + 32 * w + lane, cs * inv);
}

template <int NTB, int WB>
static int launch_k(const Wg16Args& a, hipStream_t st) {
  using Cfg = Wg16<NTB, WB>;
  auto kern = k_wgrad16<NTB, WB>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               Cfg::kLds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, dim3((unsigned)((a.K + a.ks - 1) / a.ks)), dim3(Cfg::kThreads), Cfg::kLds, st, a);
  return hip_status(hipGetLastError());
}

// kind: kWgradHidden (B [K][256]), kWgradFirst (B [K][96], 93 columns) or kWgradFc (B [K][32]);
// K is rounded up to 32
// (the rows up to it exist and carry zero deltas)
int launch_wgrad16(int kind, const void* A, const void* B, int64_t K, float* C, int64_t ldc, float* bias,
                   const uint32_t* gmax, hipStream_t st) {
  if (K <= 0) return 0;
  K = (K + 31) / 32 * 32;
  // split-K: each workgroup flushes its whole C tile (256 KB of float atomics for a hidden layer,
  // ~0.2 us of the chip's atomic rate) and spends ~0.5 us per 32-point tile, so the time
  // (K / 32 / n) * 0.5 + n * 0.2 is least at n = sqrt(2.5 K / 32); at most one workgroup per CU
  int64_t nwg = (int64_t)sqrt(2.5 * (double)K / 32.0);
  nwg = nwg < 4 ? 4 : (nwg > 256 ? 256 : nwg);
  int64_t ks = (K + nwg - 1) / nwg;
  ks = (ks + 31) / 32 * 32;
  Wg16Args a{static_cast<const _Float16*>(A), static_cast<const _Float16*>(B), 256, K, ks, C, ldc, bias, gmax};
  TimingScope ts(kTimeWgrad, K, st);
  if (kind == kWgradHidden) return launch_k<8, 256>(a, st);
  if (kind == kWgradFc) {  // dWc_l (256 x 32) += gH_l^T c : B = f16 copy of the features [K][32]
    a.nb = kCDim;
    return launch_k<1, 32>(a, st);
  }
  if (kind == kWgradFirst) {
    a.nb = kFourier;
    return launch_k<3, 96>(a, st);
  }
  return PNR_E_ARG;
}

// Skinny weight-gradient GEMMs, bandwidth-bound on B:
//   C[m][n] += inv * sum_k A[k][m] B[k][n]   m < M (<= 4), n < N      (bias[m] += sum_k A[k][m])
// A fp32 rows of 4 (float4: g_out, or x = (x0, x1, x2, inside) with M = 3), B f16 rows of WB.
//   dWo (4 x 256) = g_out^T h4 (+ dbo)       dB (3 x 93) = x^T (g_arg * s)  (inv = 1/s)
// A block streams its K range 16 rows at a time: thread (r, c) = (tid / CPR, tid % CPR) loads 16 B
// (8 columns) of row r and the row's float4 of A, keeping 4 x 8 partial sums; the rows are then
// reduced through LDS and flushed with one atomic per output element per block.
template <int WB>
__global__ __launch_bounds__(256) void k_wgrad_skinny16(const float4* __restrict__ A, const _Float16* __restrict__ B,
                                                        int64_t K, int64_t ks, int M, int N, float* __restrict__ C,
                                                        int64_t ldc, float* __restrict__ bias,
                                                        const uint32_t* __restrict__ gmax) {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  constexpr int CPR = WB / 8;          // threads per row (32 for 256, 12 for 96)
  constexpr int RPI = 256 / CPR;       // rows per iteration (8 or 21)
  __shared__ float red[4][256 + 8];
  const int tid = threadIdx.x;
  const int r = tid / CPR, c = tid % CPR;
  const bool act = r < RPI;
  const int64_t kb = (int64_t)blockIdx.x * ks;
  const int64_t ke = kb + ks < K ? kb + ks : K;
  float acc[4][8];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[m][j] = 0.f;
  float bs[4] = {0.f, 0.f, 0.f, 0.f};
  if (act) {
    constexpr int U = 4;  // rows in flight per thread (HBM latency: bytes in flight per CU)
    for (int64_t k = kb + r; k < ke; k += U * RPI) {
      float4 av[U];
      h8 bv[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t ku = k + u * RPI;
        const int64_t kc = ku < ke ? ku : k;  // rows past the range: re-read row k, weighted 0
        av[u] = A[kc];
        bv[u] = *reinterpret_cast<const h8*>(B + kc * WB + 8 * c);
        if (ku >= ke) av[u] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float a4[4] = {av[u].x, av[u].y, av[u].z, av[u].w};
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float x = (float)bv[u][j];
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[m][j] = __builtin_fmaf(a4[m], x, acc[m][j]);
        }
        if (c == 0) {
#pragma unroll
          for (int m = 0; m < 4; ++m) bs[m] += a4[m];
        }
      }
    }
  }
  const float inv = gmax ? 1.f / delta_scale(*gmax) : 1.f;
  // reduce the RPI row groups: column n = 8c + j
  for (int m = 0; m < 4; ++m) {
    for (int i = tid; i < 256 + 8; i += 256) red[m][i] = 0.f;
  }
  __syncthreads();
  if (act) {
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&red[m][8 * c + j], acc[m][j]);  // LDS atomics
    if (c == 0)
#pragma unroll
      for (int m = 0; m < 4; ++m) atomicAdd(&red[m][256 + 4], bs[m]);
  }
  __syncthreads();
  for (int i = tid; i < 4 * N; i += 256) {
    const int m = i / N, n = i % N;
    if (m < M) atomicAdd(C + (int64_t)m * ldc + n, red[m][n] * inv);
  }
  if (bias && tid < M) atomicAdd(bias + tid, red[tid][256 + 4]);
}

// f16 copy of n floats (the per-point features c, the B operand of dWc)
__global__ void k_to_f16(const float* __restrict__ x, _Float16* __restrict__ y, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    y[i] = (_Float16)x[i];
}
int launch_to_f16(const float* x, void* y, int64_t n, hipStream_t st) {
  if (n <= 0) return 0;
  int64_t blocks = (n + 1023) / 1024;
  if (blocks > 4096) blocks = 4096;
  hipLaunchKernelGGL(k_to_f16, dim3((unsigned)blocks), dim3(256), 0, st, x, static_cast<_Float16*>(y), n);
  return hip_status(hipGetLastError());
}

// dWo (4 x 256) += g_out^T h4 (f16), dbo += colsum(g_out)
int launch_wgrad_out16(const float* g_out, const void* h4, int64_t K, float* C, float* bias, hipStream_t st) {
  if (K <= 0) return 0;
  int64_t ks = (K + 1023) / 1024;
  if (ks < 256) ks = 256;
  TimingScope ts(kTimeWgrad, K, st);
  hipLaunchKernelGGL(k_wgrad_skinny16<256>, dim3((unsigned)((K + ks - 1) / ks)), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(g_out), static_cast<const _Float16*>(h4), K, ks, 4, kHidden, C,
                     (int64_t)kHidden, bias, nullptr);
  return hip_status(hipGetLastError());
}

// dB (3 x 93) += x^T g_arg: x rows float4 (x0, x1, x2, inside), g_arg f16 * s [K][96]
int launch_wgrad_fourier16(const float4* xP, const void* garg, int64_t K, float* C, const uint32_t* gmax,
                           hipStream_t st) {
  if (K <= 0) return 0;
  int64_t ks = (K + 1023) / 1024;
  if (ks < 256) ks = 256;
  TimingScope ts(kTimeWgrad, K, st);
  hipLaunchKernelGGL(k_wgrad_skinny16<96>, dim3((unsigned)((K + ks - 1) / ks)), dim3(256), 0, st, xP,
                     static_cast<const _Float16*>(garg), K, ks, 3, kFourier, C, (int64_t)kFourier, nullptr, gmax);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
