// points.hip -- neural-point feature gather for gfx950.
//
// The reference has no neural-point stage; its nearest analogue is MLP.sample_grid_feature
// (src/conv_onet/models/decoder.py:168-175, trilinear F.grid_sample on a dense grid).  The stage
// is specified by oracle/ref_points.py and include/pnr.h (pnr_points):
//
//   k_hash_count / scan / k_hash_scatter : spatial hash of the points (cell edge `cell`) into
//        2^bits buckets -> cell_start[T+1] + bucket-sorted float4 (x, y, z, index bits)
//   k_gather   : per sample, probe the 27 cells around it, keep the k nearest (d2, index)
//        inside the neighbourhood (IDW ball / trilinear box), normalised weights, then the
//        feature sum  c = sum_k w_k f_k  with 8 lanes per sample reading 128-B feature rows
//   k_gather_bwd : dL/df_i += w_k dL/dc (float atomics, 8 lanes per sample) and dL/dp through
//        the weights (8-lane dot products g.f_k, g.c)
//
// The search is thread-per-sample: the samples of one wave are consecutive points of the same
// two rays, so they probe the same few buckets and the bucket data stays in L1/L2.
#include "pnr_internal.h"

namespace pnr {

#define PNR_FP_STRICT _Pragma("clang fp contract(off)")

namespace {

struct HashGrid {
  float o0, o1, o2;
  float inv;      // 1 / cell
  uint32_t mask;  // T - 1
};

HashGrid make_grid(const pnr_points& p) {
  HashGrid g;
  g.o0 = p.origin[0];
  g.o1 = p.origin[1];
  g.o2 = p.origin[2];
  g.inv = 1.0f / p.cell;
  g.mask = (uint32_t)((1ll << p.table_bits) - 1);
  return g;
}

__device__ __forceinline__ int cell_coord(float x, float o, float inv) {
  PNR_FP_STRICT
  float f = floorf((x - o) * inv);
  f = fminf(fmaxf(f, -1.0e9f), 1.0e9f);  // far-away / non-finite samples: any cell, never UB
  return (int)f;
}

__device__ __forceinline__ uint32_t cell_hash(int cx, int cy, int cz, uint32_t mask) {
  return (((uint32_t)cx * 73856093u) ^ ((uint32_t)cy * 19349663u) ^ ((uint32_t)cz * 83492791u)) & mask;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Index layout
// ---------------------------------------------------------------------------------------------
static inline size_t a256(size_t x) { return (x + 255) / 256 * 256; }

static int64_t scan_scratch_ints(int64_t n) {
  int64_t tot = 0;
  while (true) {
    const int64_t nb = (n + 1023) / 1024;
    tot += 2 * nb + 1;  // tile sums + their scan (nb + 1), then the next level
    if (nb <= 1) break;
    n = nb;
  }
  return tot + 64;
}

IndexView index_view(void* base, int64_t M, int32_t bits, size_t* bytes) {
  IndexView v{};
  v.T = 1ll << bits;
  char* b = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = b ? b + off : nullptr;
    off += a256(n);
    return p;
  };
  v.start = reinterpret_cast<int32_t*>(take((size_t)(v.T + 1) * 4));
  v.count = reinterpret_cast<int32_t*>(take((size_t)v.T * 4));
  v.bucket = reinterpret_cast<int32_t*>(take((size_t)M * 4));
  v.slot = reinterpret_cast<int32_t*>(take((size_t)M * 4));
  v.partial = reinterpret_cast<int32_t*>(take((size_t)scan_scratch_ints(v.T) * 4));
  v.sorted = reinterpret_cast<float4*>(take((size_t)M * 16));
  if (bytes) *bytes = off;
  return v;
}

// ---------------------------------------------------------------------------------------------
// Build
// ---------------------------------------------------------------------------------------------
__global__ void k_hash_count(const float* __restrict__ xyz, int64_t M, HashGrid g, int32_t* __restrict__ count,
                             int32_t* __restrict__ bucket, int32_t* __restrict__ slot) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const float x = xyz[i * 3 + 0], y = xyz[i * 3 + 1], z = xyz[i * 3 + 2];
  const uint32_t b = cell_hash(cell_coord(x, g.o0, g.inv), cell_coord(y, g.o1, g.inv), cell_coord(z, g.o2, g.inv),
                               g.mask);
  bucket[i] = (int32_t)b;
  slot[i] = atomicAdd(count + b, 1);
}

// exclusive scan of 1024-element tiles (256 threads x 4); tile totals -> sums[tile];
// a single-tile scan also writes out[n] = total
__global__ void k_scan_tile(const int32_t* __restrict__ in, int32_t* __restrict__ out, int64_t n,
                            int32_t* __restrict__ sums) {
  __shared__ int32_t wsum[4];
  const int64_t base = (int64_t)blockIdx.x * 1024 + threadIdx.x * 4;
  int v[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) v[e] = base + e < n ? in[base + e] : 0;
  const int t = v[0] + v[1] + v[2] + v[3];
  // inclusive wave scan of t
  int incl = t;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int o = __shfl_up(incl, d);
    if (lane >= d) incl += o;
  }
  if (lane == 63) wsum[w] = incl;
  __syncthreads();
  int woff = 0;
  for (int k = 0; k < w; ++k) woff += wsum[k];
  int run = woff + incl - t;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    if (base + e < n) out[base + e] = run;
    run += v[e];
  }
  if (threadIdx.x == 255) {
    const int total = woff + incl;
    sums[blockIdx.x] = total;
    if (gridDim.x == 1) out[n] = total;
  }
}

__global__ void k_scan_add(int32_t* __restrict__ out, int64_t n, const int32_t* __restrict__ offs, int64_t nb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] += offs[i / 1024];
  else if (i == n) out[n] = offs[nb];
}

// out[0..n] = exclusive scan of in[0..n), out[n] = total.  scratch: scan_scratch_ints(n) ints.
static int scan_exclusive(const int32_t* in, int32_t* out, int64_t n, int32_t* scratch, hipStream_t st) {
  const int64_t nb = (n + 1023) / 1024;
  int32_t* sums = scratch;
  hipLaunchKernelGGL(k_scan_tile, dim3((unsigned)nb), dim3(256), 0, st, in, out, n, sums);
  if (nb > 1) {
    int32_t* offs = scratch + nb;  // nb + 1 entries
    int rc = scan_exclusive(sums, offs, nb, offs + nb + 1, st);
    if (rc) return rc;
    hipLaunchKernelGGL(k_scan_add, dim3((unsigned)((n + 1 + 255) / 256)), dim3(256), 0, st, out, n, offs, nb);
  }
  return hip_status(hipGetLastError());
}

__global__ void k_hash_scatter(const float* __restrict__ xyz, int64_t M, const int32_t* __restrict__ start,
                               const int32_t* __restrict__ bucket, const int32_t* __restrict__ slot,
                               float4* __restrict__ sorted) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int64_t pos = (int64_t)start[bucket[i]] + slot[i];
  sorted[pos] = make_float4(xyz[i * 3 + 0], xyz[i * 3 + 1], xyz[i * 3 + 2], __int_as_float((int)i));
}

int launch_points_build(const pnr_points& pts, hipStream_t st) {
  const int64_t M = pts.n_points;
  IndexView v = index_view(pts.index, M, pts.table_bits, nullptr);
  if (hipMemsetAsync(v.count, 0, (size_t)v.T * 4, st) != hipSuccess) return (int)hipGetLastError();
  const HashGrid g = make_grid(pts);
  const unsigned nbm = (unsigned)((M + 255) / 256);
  if (M > 0)
    hipLaunchKernelGGL(k_hash_count, dim3(nbm), dim3(256), 0, st, pts.xyz, M, g, v.count, v.bucket, v.slot);
  int rc = scan_exclusive(v.count, v.start, v.T, v.partial, st);
  if (rc) return rc;
  if (M > 0)
    hipLaunchKernelGGL(k_hash_scatter, dim3(nbm), dim3(256), 0, st, pts.xyz, M, v.start, v.bucket, v.slot, v.sorted);
  return hip_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Gather
// ---------------------------------------------------------------------------------------------
struct GatherArgs {
  PointSrc src;
  int64_t P, rows;
  HashGrid g;
  const int32_t* start;
  const float4* sorted;
  const float4* feats4;  // (M, 8) float4
  const float* xyz;      // (M, 3)
  int k;
  float r2, eps;
  float h0, h1, h2;      // trilinear spacing
  float* c;              // (rows, 32)
  int32_t* idx;          // (rows, k) or null
  float* w;              // (rows, k) or null
};

__device__ __forceinline__ bool key_less(float da, int ia, float db, int ib) {
  return da < db || (da == db && ia < ib);
}

template <int SRC, int KER>
__global__ __launch_bounds__(256) void k_gather(GatherArgs a) {
  PNR_FP_STRICT
  __shared__ int32_t s_idx[256 * PNR_MAX_K];
  __shared__ float s_w[256 * PNR_MAX_K];
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;

  float kd[PNR_MAX_K];
  int ki[PNR_MAX_K];
#pragma unroll
  for (int s = 0; s < PNR_MAX_K; ++s) {
    kd[s] = __builtin_inff();
    ki[s] = 0x7fffffff;
  }
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  if (p < a.P) {
    bool inside;
    load_point<SRC>(a.src, p, x0, x1, x2, inside);
    const int cx = cell_coord(x0, a.g.o0, a.g.inv), cy = cell_coord(x1, a.g.o1, a.g.inv),
              cz = cell_coord(x2, a.g.o2, a.g.inv);
#pragma unroll 1
    for (int n = 0; n < 27; ++n) {
      const int qx = cx + n % 3 - 1, qy = cy + (n / 3) % 3 - 1, qz = cz + n / 9 - 1;
      const uint32_t b = cell_hash(qx, qy, qz, a.g.mask);
      const int e = a.start[b + 1];
#pragma unroll 1
      for (int jj = a.start[b]; jj < e; ++jj) {
        const float4 q = a.sorted[jj];
        const float d0 = x0 - q.x, d1 = x1 - q.y, d2 = x2 - q.z;
        const float dd = (d0 * d0 + d1 * d1) + d2 * d2;
        bool ok;
        if (KER == PNR_GATHER_IDW) ok = dd <= a.r2;
        else ok = fabsf(d0) < a.h0 && fabsf(d1) < a.h1 && fabsf(d2) < a.h2;
        if (!ok) continue;
        // a colliding bucket holds points of other cells: count each point only in its own cell
        if (cell_coord(q.x, a.g.o0, a.g.inv) != qx || cell_coord(q.y, a.g.o1, a.g.inv) != qy ||
            cell_coord(q.z, a.g.o2, a.g.inv) != qz)
          continue;
        const int id = __float_as_int(q.w);
        if (!key_less(dd, id, kd[PNR_MAX_K - 1], ki[PNR_MAX_K - 1])) continue;
        kd[PNR_MAX_K - 1] = dd;
        ki[PNR_MAX_K - 1] = id;
#pragma unroll
        for (int s = PNR_MAX_K - 1; s > 0; --s) {
          if (key_less(kd[s], ki[s], kd[s - 1], ki[s - 1])) {
            const float tdd = kd[s]; kd[s] = kd[s - 1]; kd[s - 1] = tdd;
            const int tid = ki[s]; ki[s] = ki[s - 1]; ki[s - 1] = tid;
          }
        }
      }
    }
  }
  // weights of the first k, normalised by their sequential sum (ascending distance)
  float wv[PNR_MAX_K];
  float W = 0.f;
#pragma unroll
  for (int s = 0; s < PNR_MAX_K; ++s) {
    float w = 0.f;
    if (s < a.k && ki[s] != 0x7fffffff) {
      if (KER == PNR_GATHER_IDW) {
        w = 1.0f / fmaxf(sqrtf(kd[s]), a.eps);
      } else {  // per-axis offsets of the kept point (same f32 arithmetic as the search)
        const float* xi = a.xyz + (int64_t)ki[s] * 3;
        const float t0 = 1.0f - fabsf(x0 - xi[0]) / a.h0;
        const float t1 = 1.0f - fabsf(x1 - xi[1]) / a.h1;
        const float t2 = 1.0f - fabsf(x2 - xi[2]) / a.h2;
        w = (t0 * t1) * t2;
      }
    }
    wv[s] = w;
    W = W + w;
  }
  const float Wd = W > 0.f ? W : 1.0f;
#pragma unroll
  for (int s = 0; s < PNR_MAX_K; ++s) {
    const bool v = s < a.k && ki[s] != 0x7fffffff;
    const float wn = v ? wv[s] / Wd : 0.f;
    s_idx[threadIdx.x * PNR_MAX_K + s] = v ? ki[s] : -1;
    s_w[threadIdx.x * PNR_MAX_K + s] = wn;
    if (p < a.rows && s < a.k) {
      if (a.idx) a.idx[p * a.k + s] = v ? ki[s] : -1;
      if (a.w) a.w[p * a.k + s] = wn;
    }
  }
  __syncthreads();
  // feature sum: 8 lanes per sample, lane q owns channels 4q..4q+3 (one 16-B load per neighbour)
  const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6, gq = lane >> 3, q = lane & 7;
#pragma unroll 1
  for (int rr = 0; rr < 8; ++rr) {
    const int s = wv_ * 64 + rr * 8 + gq;
    const int64_t ps = (int64_t)blockIdx.x * 256 + s;
    if (ps >= a.rows) continue;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int kk = 0; kk < PNR_MAX_K; ++kk) {
      const int id = s_idx[s * PNR_MAX_K + kk];
      if (id < 0) continue;
      const float wn = s_w[s * PNR_MAX_K + kk];
      const float4 f = a.feats4[(int64_t)id * 8 + q];
      acc.x = acc.x + wn * f.x;
      acc.y = acc.y + wn * f.y;
      acc.z = acc.z + wn * f.z;
      acc.w = acc.w + wn * f.w;
    }
    reinterpret_cast<float4*>(a.c)[ps * 8 + q] = acc;
  }
}


// ---------------------------------------------------------------------------------------------
// Backward
// ---------------------------------------------------------------------------------------------
struct GatherBwdArgs {
  PointSrc src;
  const float4* xP;      // MLP inputs (fused path) or null (positions from src)
  int64_t P;
  const float* xyz;
  const float4* feats4;
  int k;
  float eps, h0, h1, h2;
  const int32_t* idx;
  const float* w;
  const float* c;
  const float* g_c;
  float* g_feats;        // (M,32) += or null
  float* g_p;            // (P,3) or null
  int gp_accum;
};

template <int SRC, int KER>
__global__ __launch_bounds__(256) void k_gather_bwd(GatherBwdArgs a) {
  PNR_FP_STRICT
  const int lane = threadIdx.x & 63, wv_ = threadIdx.x >> 6, gq = lane >> 3, q = lane & 7;
#pragma unroll 1
  for (int rr = 0; rr < 8; ++rr) {
    const int64_t p = (int64_t)blockIdx.x * 256 + wv_ * 64 + rr * 8 + gq;
    if (p >= a.P) continue;  // groups of 8 lanes share p: the shuffles below stay inside a group
    const float4 g = reinterpret_cast<const float4*>(a.g_c)[p * 8 + q];
    float dots[PNR_MAX_K];
    float gcd = 0.f;
    if (a.g_p) {
      const float4 cv = reinterpret_cast<const float4*>(a.c)[p * 8 + q];
      gcd = g.x * cv.x + g.y * cv.y + g.z * cv.z + g.w * cv.w;
    }
#pragma unroll
    for (int kk = 0; kk < PNR_MAX_K; ++kk) {
      dots[kk] = 0.f;
      if (kk >= a.k) continue;
      const int id = a.idx[p * a.k + kk];
      if (id < 0) continue;
      const float wn = a.w[p * a.k + kk];
      if (a.g_feats) {
        float* gf = a.g_feats + (int64_t)id * 32 + 4 * q;
        unsafeAtomicAdd(gf + 0, wn * g.x);
        unsafeAtomicAdd(gf + 1, wn * g.y);
        unsafeAtomicAdd(gf + 2, wn * g.z);
        unsafeAtomicAdd(gf + 3, wn * g.w);
      }
      if (a.g_p) {
        const float4 f = a.feats4[(int64_t)id * 8 + q];
        dots[kk] = g.x * f.x + g.y * f.y + g.z * f.z + g.w * f.w;
      }
    }
    if (!a.g_p) continue;
#pragma unroll
    for (int m = 1; m < 8; m <<= 1) {
      gcd += __shfl_xor(gcd, m);
#pragma unroll
      for (int kk = 0; kk < PNR_MAX_K; ++kk) dots[kk] += __shfl_xor(dots[kk], m);
    }
    if (q != 0) continue;
    float x0, x1, x2;
    if (a.xP) {
      const float4 xv = a.xP[p];
      x0 = xv.x; x1 = xv.y; x2 = xv.z;
    } else {
      bool inside;
      load_point<SRC>(a.src, p, x0, x1, x2, inside);
    }
    // dL/dp = sum_k wn_k (g.f_k - g.c) (1/w_k) dw_k/dp
    float gp0 = 0.f, gp1 = 0.f, gp2 = 0.f;
#pragma unroll
    for (int kk = 0; kk < PNR_MAX_K; ++kk) {
      if (kk >= a.k) continue;
      const int id = a.idx[p * a.k + kk];
      if (id < 0) continue;
      const float wn = a.w[p * a.k + kk];
      const float* xi = a.xyz + (int64_t)id * 3;
      const float d0 = x0 - xi[0], d1 = x1 - xi[1], d2 = x2 - xi[2];
      const float coef = wn * (dots[kk] - gcd);
      if (KER == PNR_GATHER_IDW) {
        const float dd = (d0 * d0 + d1 * d1) + d2 * d2;
        if (sqrtf(dd) > a.eps) {  // w = 1/|d|: (1/w) dw/dp = -d / |d|^2
          const float f = -coef / dd;
          gp0 += f * d0; gp1 += f * d1; gp2 += f * d2;
        }
      } else {  // w = prod (1 - |d_a|/h_a): (1/w) dw/dp_a = -sign(d_a) / (h_a t_a)
        const float t0 = 1.0f - fabsf(d0) / a.h0, t1 = 1.0f - fabsf(d1) / a.h1, t2 = 1.0f - fabsf(d2) / a.h2;
        const float s0 = d0 > 0.f ? 1.f : (d0 < 0.f ? -1.f : 0.f);
        const float s1 = d1 > 0.f ? 1.f : (d1 < 0.f ? -1.f : 0.f);
        const float s2 = d2 > 0.f ? 1.f : (d2 < 0.f ? -1.f : 0.f);
        gp0 -= coef * s0 / (a.h0 * t0);
        gp1 -= coef * s1 / (a.h1 * t1);
        gp2 -= coef * s2 / (a.h2 * t2);
      }
    }
    float* o = a.g_p + p * 3;
    if (a.gp_accum) {
      o[0] += gp0; o[1] += gp1; o[2] += gp2;
    } else {
      o[0] = gp0; o[1] = gp1; o[2] = gp2;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------------
static bool points_ok(const pnr_points& pts) {
  return pts.n_points >= 0 && pts.k >= 1 && pts.k <= PNR_MAX_K && pts.table_bits >= 10 && pts.table_bits <= 24 &&
         pts.index && (pts.mode == PNR_GATHER_IDW || pts.mode == PNR_GATHER_TRILINEAR) && pts.cell > 0.f &&
         (pts.n_points == 0 || (pts.xyz && pts.feats));
}

template <int KER>
static void gather_mode(int mode, dim3 grid, hipStream_t st, const GatherArgs& a) {
  switch (mode) {
    case kPtsF64: hipLaunchKernelGGL((k_gather<kPtsF64, KER>), grid, dim3(256), 0, st, a); break;
    case kPtsF32: hipLaunchKernelGGL((k_gather<kPtsF32, KER>), grid, dim3(256), 0, st, a); break;
    case kRaysZ64: hipLaunchKernelGGL((k_gather<kRaysZ64, KER>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_gather<kRaysZ32, KER>), grid, dim3(256), 0, st, a); break;
  }
}

int launch_gather(const pnr_points& pts, const PointSrc& src, int mode, int64_t P, int64_t rows, float* c,
                  int32_t* idx, float* w, hipStream_t st) {
  if (!points_ok(pts) || mode < kPtsF64 || mode > kRaysZ32 || P < 0 || rows < P) return PNR_E_ARG;
  if (rows == 0) return PNR_OK;
  IndexView v = index_view(pts.index, pts.n_points, pts.table_bits, nullptr);
  GatherArgs a{};
  a.src = src;
  a.P = P;
  a.rows = rows;
  a.g = make_grid(pts);
  a.start = v.start;
  a.sorted = v.sorted;
  a.feats4 = reinterpret_cast<const float4*>(pts.feats);
  a.xyz = pts.xyz;
  a.k = pts.k;
  a.r2 = pts.radius * pts.radius;
  a.eps = pts.eps;
  a.h0 = pts.spacing[0];
  a.h1 = pts.spacing[1];
  a.h2 = pts.spacing[2];
  a.c = c;
  a.idx = idx;
  a.w = w;
  const dim3 grid((unsigned)((rows + 255) / 256));
  TimingScope ts(kTimeGather, P, st);
  if (pts.mode == PNR_GATHER_IDW) gather_mode<PNR_GATHER_IDW>(mode, grid, st, a);
  else gather_mode<PNR_GATHER_TRILINEAR>(mode, grid, st, a);
  return hip_status(hipGetLastError());
}

template <int KER>
static void gather_bwd_mode(int mode, dim3 grid, hipStream_t st, const GatherBwdArgs& a) {
  switch (mode) {
    case kPtsF64: hipLaunchKernelGGL((k_gather_bwd<kPtsF64, KER>), grid, dim3(256), 0, st, a); break;
    case kPtsF32: hipLaunchKernelGGL((k_gather_bwd<kPtsF32, KER>), grid, dim3(256), 0, st, a); break;
    case kRaysZ64: hipLaunchKernelGGL((k_gather_bwd<kRaysZ64, KER>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_gather_bwd<kRaysZ32, KER>), grid, dim3(256), 0, st, a); break;
  }
}

int launch_gather_bwd(const pnr_points& pts, const PointSrc* src, int mode, const float4* xP, int64_t P,
                      const int32_t* idx, const float* w, const float* c, const float* g_c, float* g_p,
                      bool gp_accum, hipStream_t st) {
  if (!points_ok(pts) || P < 0 || (!src && !xP) || mode < kPtsF64 || mode > kRaysZ32) return PNR_E_ARG;
  if (P == 0 || (!pts.g_feats && !g_p)) return PNR_OK;
  if (!idx || !w || !g_c || (g_p && !c)) return PNR_E_ARG;
  GatherBwdArgs a{};
  if (src) a.src = *src;
  a.xP = xP;
  a.P = P;
  a.xyz = pts.xyz;
  a.feats4 = reinterpret_cast<const float4*>(pts.feats);
  a.k = pts.k;
  a.eps = pts.eps;
  a.h0 = pts.spacing[0];
  a.h1 = pts.spacing[1];
  a.h2 = pts.spacing[2];
  a.idx = idx;
  a.w = w;
  a.c = c;
  a.g_c = g_c;
  a.g_feats = pts.g_feats;
  a.g_p = g_p;
  a.gp_accum = gp_accum ? 1 : 0;
  const dim3 grid((unsigned)((P + 255) / 256));
  TimingScope ts(kTimeGatherBwd, P, st);
  if (pts.mode == PNR_GATHER_IDW) gather_bwd_mode<PNR_GATHER_IDW>(mode, grid, st, a);
  else gather_bwd_mode<PNR_GATHER_TRILINEAR>(mode, grid, st, a);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
