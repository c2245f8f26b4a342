// wgrad16.hip -- weight-gradient GEMMs of the decoder backward on bf16x3 split MFMA.
//
//   C[256][NB] += A[K][256]^T B[K][WB]        (A, B point-major fp32: row k = one point)
//   bias[256]  += sum_k A[k][:]               (optional)
//
// Used for every precision but PNR_PREC_FP32 (wgrad.hip keeps the fp32 MFMA form) on the two large
// shapes of src/conv_onet/models/decoder.py:149-159:
//   dW3 = delta4^T h3, dW2 = delta3^T h2, dW1 = delta2^T h1     WB = 256 (8 column tiles)
//   dW0 = delta1^T e                                            WB = 96 (3 column tiles, 93 used)
//
// K (points, millions) is split over workgroups.  A workgroup streams 32-point tiles: every thread
// loads its float4s of the next tile into registers while the current tile computes, then splits
// them into bf16 hi / lo parts and writes them to a double-buffered LDS image [part][128-column
// half][32 rows][256 B] whose 16-B chunks are XOR-swizzled by row.  The MFMA operands need 8
// consecutive points of one column per lane: ds_read_b64_tr_b16 reads them transposed out of that
// image (conflict-free with the swizzle; cdna_hip_programming.md T10).  Wave w owns output rows
// [64w, 64w + 64) x all NB columns: 2 x NTB accumulator tiles stay in AGPRs for the whole K range
// and are added into C with one float atomic per element at the end.
// Per product Al.Bh + Ah.Bl + Ah.Bh: ~2^-16 relative, exponent range of fp32.
#include "mlp16.h"

namespace pnr {

typedef short v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4i16 lds_v4i16;

template <int NTB, int WB>
struct Wg16 {
  static constexpr int kHalvesA = 2;
  static constexpr int kHalvesB = (WB + 127) / 128;
  static constexpr int kImgA = 2 * kHalvesA * 32 * 256;  // bytes
  static constexpr int kImgB = 2 * kHalvesB * 32 * 256;
  static constexpr int kBuf = kImgA + kImgB;
  static constexpr int kAV4 = 32 * 256 / 4 / 256;          // float4 of A per thread per tile (8)
  static constexpr int kBV4 = (32 * WB / 4 + 255) / 256;   // float4 of B per thread per tile (8 or 3)
};

struct Wg16Args {
  const float* A;   // [K][256]
  const float* B;   // [K][WB]
  int nb;           // valid columns of B (columns of C)
  int64_t K;
  int64_t ks;       // points per workgroup (multiple of 32)
  float* C;
  int64_t ldc;
  float* bias;
};

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }

// byte offset of 16-bit element (row, col) block start: col multiple of 4, within a [half][32][256 B] image
__device__ __forceinline__ int img_off(int row, int col) {
  const int half = col >> 7, cc = col & 127;
  return (half * 32 + row) * 256 + 16 * ((cc >> 3) ^ swz(row)) + 8 * ((cc >> 2) & 1);
}

// split one float4 (row, cols c..c+3) into the hi / lo images
__device__ __forceinline__ void put4(char* img, int part_bytes, int row, int col, const float4& v) {
  const float x[4] = {v.x, v.y, v.z, v.w};
  v4i16 h, l;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const __bf16 hb = (__bf16)x[i];
    const __bf16 lb = (__bf16)(x[i] - (float)hb);
    h[i] = __builtin_bit_cast(short, hb);
    l[i] = __builtin_bit_cast(short, lb);
  }
  const int o = img_off(row, col);
  *reinterpret_cast<v4i16*>(img + o) = h;
  *reinterpret_cast<v4i16*>(img + part_bytes + o) = l;
}

// MFMA operand of column tile T (32 columns), k-step s of the tile, part image `img`:
// lane l holds column 32T + (l&31), rows 16s + 8(l>>5) + j, j = 0..7 (two transposed reads)
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int T, int s) {
  const int l = threadIdx.x & 63, g = l >> 4, i = l & 15, q = i >> 2, p = i & 3;
  const int col = 32 * T + 16 * (g & 1) + 4 * p;
  const int row0 = 16 * s + 8 * (g >> 1) + q;
  const v4i16 a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + img_off(row0, col)));
  const v4i16 b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4i16*)(img + img_off(row0 + 4, col)));
  const short e[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = __builtin_bit_cast(__bf16, e[j]);
  return r;
}

__device__ __forceinline__ f32x16 mfma3(const bf16x8& ah, const bf16x8& al, const bf16x8& bh, const bf16x8& bl,
                                        f32x16 c) {
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

template <int NTB, int WB>
__global__ __launch_bounds__(256, 1) void k_wgrad16(Wg16Args a) {
  using Cfg = Wg16<NTB, WB>;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int tid = threadIdx.x, lane = tid & 63, hh = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t kb = (int64_t)blockIdx.x * a.ks;
  const int64_t ke = kb + a.ks < a.K ? kb + a.ks : a.K;

  f32x16 acc[2][NTB];
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NTB; ++y)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[x][y][r] = 0.f;
  float cs[4] = {0.f, 0.f, 0.f, 0.f};  // column sums of A (bias): columns 4 (tid & 63) .. +3

  float4 va[Cfg::kAV4], vb[Cfg::kBV4];
  auto load = [&](int64_t k0) {
#pragma unroll
    for (int i = 0; i < Cfg::kAV4; ++i) {
      const int f = tid + 256 * i, row = f >> 6;
      va[i] = k0 + row < ke ? reinterpret_cast<const float4*>(a.A + (k0 + row) * 256)[f & 63]
                            : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int i = 0; i < Cfg::kBV4; ++i) {
      const int f = tid + 256 * i, row = f / (WB / 4), c4 = f % (WB / 4);
      vb[i] = (f < 32 * WB / 4 && k0 + row < ke) ? reinterpret_cast<const float4*>(a.B + (k0 + row) * WB)[c4]
                                                 : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  load(kb);
  int buf = 0;
  for (int64_t k0 = kb; k0 < ke; k0 += 32) {
    char* ia = lds + buf * Cfg::kBuf;
    char* ib = ia + Cfg::kImgA;
#pragma unroll
    for (int i = 0; i < Cfg::kAV4; ++i) {
      const int f = tid + 256 * i;
      put4(ia, Cfg::kImgA / 2, f >> 6, 4 * (f & 63), va[i]);
      cs[0] += va[i].x; cs[1] += va[i].y; cs[2] += va[i].z; cs[3] += va[i].w;
    }
#pragma unroll
    for (int i = 0; i < Cfg::kBV4; ++i) {
      const int f = tid + 256 * i;
      if (f < 32 * WB / 4) put4(ib, Cfg::kImgB / 2, f / (WB / 4), 4 * (f % (WB / 4)), vb[i]);
    }
    __syncthreads();
    if (k0 + 32 < ke) load(k0 + 32);  // next tile in flight during the MFMAs
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8 ah[2], al[2];
#pragma unroll
      for (int x = 0; x < 2; ++x) {
        ah[x] = tr_frag(ia, 2 * w + x, s);
        al[x] = tr_frag(ia + Cfg::kImgA / 2, 2 * w + x, s);
      }
#pragma unroll
      for (int y = 0; y < NTB; ++y) {
        const bf16x8 bh = tr_frag(ib, y, s), bl = tr_frag(ib + Cfg::kImgB / 2, y, s);
#pragma unroll
        for (int x = 0; x < 2; ++x) acc[x][y] = mfma3(ah[x], al[x], bh, bl, acc[x][y]);
      }
    }
#pragma unroll
    for (int x = 0; x < 2; ++x)
#pragma unroll
      for (int y = 0; y < NTB; ++y) asm volatile("" : "+a"(acc[x][y]));
    buf ^= 1;
  }
  // C[32(2w+x) + perm(r,hh)][32y + (lane&31)] += acc
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < NTB; ++y) {
      const int col = 32 * y + (lane & 31);
      if (col >= a.nb) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r)
        atomicAdd(a.C + (int64_t)(32 * (2 * w + x) + perm(r, hh)) * a.ldc + col, acc[x][y][r]);
    }
  if (a.bias) {
#pragma unroll
    for (int j = 0; j < 4; ++j) atomicAdd(a.bias + 4 * (tid & 63) + j, cs[j]);
  }
}

template <int NTB, int WB>
static int launch_k(const Wg16Args& a, hipStream_t st) {
  using Cfg = Wg16<NTB, WB>;
  const size_t lds = 2 * Cfg::kBuf;
  auto kern = k_wgrad16<NTB, WB>;
  static const bool attr = hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                               (int)lds) == hipSuccess;
  if (!attr) return PNR_E_ARG;
  hipLaunchKernelGGL(kern, dim3((unsigned)((a.K + a.ks - 1) / a.ks)), dim3(256), lds, st, a);
  return hip_status(hipGetLastError());
}

// kind: kWgradHidden (B [K][256]) or kWgradFirst (B [K][96], 93 columns)
int launch_wgrad16(int kind, const float* A, const float* B, int64_t K, float* C, int64_t ldc, float* bias,
                   hipStream_t st) {
  if (K <= 0) return 0;
  int64_t ks = (K + 511) / 512;  // ~2 workgroups per CU
  ks = (ks + 31) / 32 * 32;
  if (ks < 256) ks = 256;
  TimingScope ts(kTimeWgrad, K, st);
  if (kind == kWgradHidden) return launch_k<8, 256>(Wg16Args{A, B, 256, K, ks, C, ldc, bias}, st);
  if (kind == kWgradFirst) return launch_k<3, 96>(Wg16Args{A, B, kFourier, K, ks, C, ldc, bias}, st);
  return PNR_E_ARG;
}

}  // namespace pnr
