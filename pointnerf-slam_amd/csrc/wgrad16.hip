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
#include "mlp16.h"

namespace pnr {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

constexpr int kTileB = 2112;  // bytes of one [32 points][64 B] block, +64 B pad (store banks)

template <int NTB, int WB>
struct Wg16 {
  static constexpr int kThreads = 512;                     // 8 waves, 2 per SIMD
  static constexpr int kTB = NTB == 3 ? 4 : NTB;           // B blocks staged (dW0: 4, one duplicate)
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

// kind: kWgradHidden (B [K][256]) or kWgradFirst (B [K][96], 93 columns); K is rounded up to 32
// (the rows up to it exist and carry zero deltas)
int launch_wgrad16(int kind, const void* A, const void* B, int64_t K, float* C, int64_t ldc, float* bias,
                   const uint32_t* gmax, hipStream_t st) {
  if (K <= 0) return 0;
  K = (K + 31) / 32 * 32;
  int64_t ks = (K + 255) / 256;  // one workgroup per CU
  ks = (ks + 31) / 32 * 32;
  if (ks < 128) ks = 128;
  Wg16Args a{static_cast<const _Float16*>(A), static_cast<const _Float16*>(B), 256, K, ks, C, ldc, bias, gmax};
  TimingScope ts(kTimeWgrad, K, st);
  if (kind == kWgradHidden) return launch_k<8, 256>(a, st);
  if (kind == kWgradFirst) {
    a.nb = kFourier;
    return launch_k<3, 96>(a, st);
  }
  return PNR_E_ARG;
}

// dWo (4 x 256) += g_out^T h4, dbo += colsum(g_out): g_out fp32 [K][4], h4 f16 [K][256].  Thread u
// of a block owns column u; the block streams its K range (bandwidth-bound on h4).
__global__ __launch_bounds__(256) void k_wgrad_out16(const float4* __restrict__ g, const _Float16* __restrict__ h,
                                                     int64_t K, int64_t ks, float* __restrict__ C,
                                                     float* __restrict__ bias) {
  const int u = threadIdx.x;
  const int64_t kb = (int64_t)blockIdx.x * ks;
  const int64_t ke = kb + ks < K ? kb + ks : K;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f, b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
  for (int64_t k = kb; k < ke; ++k) {
    const float4 gv = g[k];
    const float x = (float)h[k * 256 + u];
    s0 = __builtin_fmaf(gv.x, x, s0);
    s1 = __builtin_fmaf(gv.y, x, s1);
    s2 = __builtin_fmaf(gv.z, x, s2);
    s3 = __builtin_fmaf(gv.w, x, s3);
    if (u == 0) { b0 += gv.x; b1 += gv.y; b2 += gv.z; b3 += gv.w; }
  }
  atomicAdd(C + u, s0);
  atomicAdd(C + 256 + u, s1);
  atomicAdd(C + 512 + u, s2);
  atomicAdd(C + 768 + u, s3);
  if (u == 0 && bias) {
    atomicAdd(bias + 0, b0); atomicAdd(bias + 1, b1); atomicAdd(bias + 2, b2); atomicAdd(bias + 3, b3);
  }
}

int launch_wgrad_out16(const float* g_out, const void* h4, int64_t K, float* C, float* bias, hipStream_t st) {
  if (K <= 0) return 0;
  int64_t ks = (K + 2047) / 2048;
  if (ks < 64) ks = 64;
  TimingScope ts(kTimeWgrad, K, st);
  hipLaunchKernelGGL(k_wgrad_out16, dim3((unsigned)((K + ks - 1) / ks)), dim3(256), 0, st,
                     reinterpret_cast<const float4*>(g_out), static_cast<const _Float16*>(h4), K, ks, C, bias);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
