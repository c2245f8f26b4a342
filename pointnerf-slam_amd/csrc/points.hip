// points.hip -- neural-point feature gather for gfx950.
//
// The reference has no neural-point stage; its nearest analogue is MLP.sample_grid_feature
// (src/conv_onet/models/decoder.py:168-175, trilinear F.grid_sample on a dense grid).  The stage
// is specified by oracle/ref_points.py and include/pnr.h (pnr_points).
//
// Index (pnr_points_build): points hashed by cell (edge `cell` >= 2 x reach) into T = 2^bits
// buckets, bucket-sorted float4 (x, y, z, index bits) with each bucket ordered by sub-cell (the
// 2x2x2 half-cells of a cell), one 16-B header per bucket {start, end, packed cell key |
// collision flag}, one 16-B sub-cell end-offset table per bucket, and an occupancy filter (one
// bit per hashed probe-block base cell).
//
// Gather, two passes:
//   k_gather_probe  one thread per sample row: coalesced zero fill of the block's output rows,
//                   occupancy-filter test of the sample's 2x2x2 probe block; samples that may have
//                   neighbours go to a work list (one atomic per wave, 64 sub-lists).  Free space -- most of a
//                   ray -- costs one L2-resident bit load.
//   k_gather_search persistent blocks over the work list (grid = resident blocks), one thread per
//                   sample: 8 bucket headers and sub-cell tables (foreign buckets of a hash collision
//                   are skipped by their key); per probe cell one span from the first to the last
//                   sub-cell (half-cell) the reach box touches, the spans compacted into the
//                   thread's LDS row and scanned by ONE flat candidate loop (uniform exit, next span
//                   read ahead); a branch-free top-k network on packed (d2, index) float64 keys
//                   (v_min/v_max_f64, 2 VALU per stage); normalised weights, then the feature sum
//                   with 8 lanes per sample.
//   k_gather_bwd    dL/df_i += w_k dL/dc (float atomics) and dL/dp through the weights.
#include <mutex>

#include "pnr_internal.h"

namespace pnr {

#define PNR_FP_STRICT _Pragma("clang fp contract(off)")

namespace {

struct HashGrid {
  float o0, o1, o2;
  float inv;       // 1 / cell
  uint32_t mask;   // T - 1
  uint32_t omask;  // occupancy bits - 1
};

int occ_bits_log2(int32_t bits) { return bits + 6 < 26 ? bits + 6 : 26; }

HashGrid make_grid(const pnr_points& p) {
  HashGrid g;
  g.o0 = p.origin[0];
  g.o1 = p.origin[1];
  g.o2 = p.origin[2];
  g.inv = 1.0f / p.cell;
  g.mask = (uint32_t)((1ll << p.table_bits) - 1);
  g.omask = (uint32_t)((1ll << occ_bits_log2(p.table_bits)) - 1);
  return g;
}

__device__ __forceinline__ int cell_coord(float x, float o, float inv) {
  PNR_FP_STRICT
  float f = floorf((x - o) * inv);
  f = fminf(fmaxf(f, -1.0e9f), 1.0e9f);  // far-away / non-finite samples: any cell, never UB
  return (int)f;
}

// half of its cell a coordinate lies in (0 lower, 1 upper), from the same f32 value as cell_coord
__device__ __forceinline__ int sub_bit(float x, float o, float inv) {
  PNR_FP_STRICT
  float t = (x - o) * inv;
  t = fminf(fmaxf(t, -1.0e9f), 1.0e9f);
  return t - floorf(t) >= 0.5f ? 1 : 0;
}
// sub-cell (2x2x2 halves of a cell) of a point, x fastest
__device__ __forceinline__ int sub_index(float x, float y, float z, float o0, float o1, float o2, float inv) {
  return sub_bit(x, o0, inv) | (sub_bit(y, o1, inv) << 1) | (sub_bit(z, o2, inv) << 2);
}

// lower of the two cells per axis that cover [x - reach, x + reach] when cell >= 2 reach
__device__ __forceinline__ void base_cell(float x, float o, float inv, int& b) {
  PNR_FP_STRICT
  float t = (x - o) * inv;
  t = fminf(fmaxf(t, -1.0e9f), 1.0e9f);
  const float f = floorf(t);
  b = (int)f - (t - f < 0.5f ? 1 : 0);
}

__device__ __forceinline__ uint32_t cell_hash(int cx, int cy, int cz, uint32_t mask) {
  return (((uint32_t)cx * 73856093u) ^ ((uint32_t)cy * 19349663u) ^ ((uint32_t)cz * 83492791u)) & mask;
}

// exact cell identity: 3 x 21-bit two's complement (scenes stay far below 2^20 cells per axis)
__device__ __forceinline__ uint64_t cell_key(int cx, int cy, int cz) {
  return (uint64_t)((uint32_t)cx & 0x1FFFFFu) | ((uint64_t)((uint32_t)cy & 0x1FFFFFu) << 21) |
         ((uint64_t)((uint32_t)cz & 0x1FFFFFu) << 42);
}
constexpr uint64_t kCollision = 1ull << 63;

// (d2, index) as one float64 whose order is the lexicographic order: d2 >= 0 has monotone float
// bits; +2^20 on the high word keeps every key a normal double (no denormal flushing)
__device__ __forceinline__ double pack_key(float d2, int id) {
  const uint64_t k = ((uint64_t)((uint32_t)__float_as_int(d2) + 0x00100000u) << 32) | (uint32_t)id;
  return __longlong_as_double((long long)k);
}
__device__ __forceinline__ float key_d2(double k) {
  return __int_as_float((int)((uint32_t)((uint64_t)__double_as_longlong(k) >> 32) - 0x00100000u));
}
__device__ __forceinline__ int key_id(double k) { return (int)(uint32_t)(uint64_t)__double_as_longlong(k); }

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
  v.tmp = reinterpret_cast<float4*>(take((size_t)M * 16));
  v.hdr = reinterpret_cast<int4*>(take((size_t)v.T * 16));
  v.sub = reinterpret_cast<int4*>(take((size_t)v.T * 16));
  v.occ_words = (1ll << occ_bits_log2(bits)) / 32;
  v.occ = reinterpret_cast<uint32_t*>(take((size_t)v.occ_words * 4));
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
  int incl = t;  // inclusive wave scan of t
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

// Order each bucket by sub-cell (counting sort, one thread per bucket; buckets hold a few points)
// and record the 8 sub-cell end offsets as u16.  A bucket of >= 65535 points keeps its order and
// gets 0xFFFF as last offset: the search then scans it whole (the distance test keeps it exact).
__global__ void k_bucket_sub(const int32_t* __restrict__ start, const float4* __restrict__ tmp, int64_t T,
                             HashGrid g, float4* __restrict__ sorted, int4* __restrict__ sub) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= T) return;
  const int s = start[b], e = start[b + 1], n = e - s;
  if (n >= 65535) {
    for (int j = s; j < e; ++j) sorted[j] = tmp[j];
    sub[b] = make_int4(-1, -1, -1, -1);
    return;
  }
  uint32_t c[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int j = s; j < e; ++j) {
    const float4 q = tmp[j];
    const int si = sub_index(q.x, q.y, q.z, g.o0, g.o1, g.o2, g.inv);
#pragma unroll
    for (int k = 0; k < 8; ++k) c[k] += si == k ? 1u : 0u;
  }
  uint32_t end[8], pos[8];
  uint32_t run = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    pos[k] = (uint32_t)s + run;
    run += c[k];
    end[k] = run;
  }
  for (int j = s; j < e; ++j) {
    const float4 q = tmp[j];
    const int si = sub_index(q.x, q.y, q.z, g.o0, g.o1, g.o2, g.inv);
    uint32_t dst = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      dst = si == k ? pos[k] : dst;
      pos[k] += si == k ? 1u : 0u;
    }
    sorted[dst] = q;
  }
  sub[b] = make_int4((int)(end[0] | (end[1] << 16)), (int)(end[2] | (end[3] << 16)), (int)(end[4] | (end[5] << 16)),
                     (int)(end[6] | (end[7] << 16)));
}

// bucket header {start, end, key lo, key hi}: the cell of the bucket's first point, plus the
// collision flag when the bucket also holds points of other cells
__global__ void k_bucket_hdr(const int32_t* __restrict__ start, const float4* __restrict__ sorted, int64_t T,
                             HashGrid g, int4* __restrict__ hdr) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= T) return;
  const int s = start[b], e = start[b + 1];
  uint64_t key = 0;
  if (e > s) {
    const float4 q = sorted[s];
    key = cell_key(cell_coord(q.x, g.o0, g.inv), cell_coord(q.y, g.o1, g.inv), cell_coord(q.z, g.o2, g.inv));
    for (int j = s + 1; j < e; ++j) {
      const float4 r = sorted[j];
      if (cell_key(cell_coord(r.x, g.o0, g.inv), cell_coord(r.y, g.o1, g.inv), cell_coord(r.z, g.o2, g.inv)) != key) {
        key |= kCollision;
        break;
      }
    }
  }
  hdr[b] = make_int4(s, e, (int)(uint32_t)key, (int)(uint32_t)(key >> 32));
}

// Occupancy filter: bit hash(b) is set when the probe block with base cell b (cells b..b+1 per
// axis) holds a point.  A clear bit proves a sample has no candidate (hash collisions only set
// extra bits), so free-space samples skip the bucket headers.
__global__ void k_occ_mark(const float* __restrict__ xyz, int64_t M, HashGrid g, uint32_t* __restrict__ occ) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= M) return;
  const int cx = cell_coord(xyz[i * 3 + 0], g.o0, g.inv), cy = cell_coord(xyz[i * 3 + 1], g.o1, g.inv),
            cz = cell_coord(xyz[i * 3 + 2], g.o2, g.inv);
#pragma unroll
  for (int n = 0; n < 8; ++n) {
    const uint32_t bit = cell_hash(cx - (n & 1), cy - ((n >> 1) & 1), cz - (n >> 2), g.omask);
    atomicOr(occ + (bit >> 5), 1u << (bit & 31u));
  }
}

int launch_points_build(const pnr_points& pts, hipStream_t st) {
  const int64_t M = pts.n_points;
  IndexView v = index_view(pts.index, M, pts.table_bits, nullptr);
  if (hipMemsetAsync(v.count, 0, (size_t)v.T * 4, st) != hipSuccess) return (int)hipGetLastError();
  if (hipMemsetAsync(v.occ, 0, (size_t)v.occ_words * 4, st) != hipSuccess) return (int)hipGetLastError();
  const HashGrid g = make_grid(pts);
  const unsigned nbm = (unsigned)((M + 255) / 256);
  if (M > 0)
    hipLaunchKernelGGL(k_hash_count, dim3(nbm), dim3(256), 0, st, pts.xyz, M, g, v.count, v.bucket, v.slot);
  int rc = scan_exclusive(v.count, v.start, v.T, v.partial, st);
  if (rc) return rc;
  if (M > 0) {
    hipLaunchKernelGGL(k_hash_scatter, dim3(nbm), dim3(256), 0, st, pts.xyz, M, v.start, v.bucket, v.slot, v.tmp);
    hipLaunchKernelGGL(k_occ_mark, dim3(nbm), dim3(256), 0, st, pts.xyz, M, g, v.occ);
  }
  hipLaunchKernelGGL(k_bucket_sub, dim3((unsigned)((v.T + 255) / 256)), dim3(256), 0, st, v.start, v.tmp, v.T, g,
                     v.sorted, v.sub);
  hipLaunchKernelGGL(k_bucket_hdr, dim3((unsigned)((v.T + 255) / 256)), dim3(256), 0, st, v.start, v.sorted, v.T, g,
                     v.hdr);
  return hip_status(hipGetLastError());
}

// ---------------------------------------------------------------------------------------------
// Gather
// ---------------------------------------------------------------------------------------------
// Point features are float32 (M,32), or float16 (M,32) when pnr_points.feat_half (SURVEY.md
// A15: the C5 budget's fp16 features); every sum and weight stays float32.
typedef _Float16 pnr_h4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ float4 load_feat4(const float4* f, int half, int64_t i4) {
  if (!half) return f[i4];
  const pnr_h4 h = reinterpret_cast<const pnr_h4*>(f)[i4];
  return make_float4((float)h.x, (float)h.y, (float)h.z, (float)h.w);
}
__device__ __forceinline__ float load_feat1(const float4* f, int half, int64_t i) {
  return half ? (float)reinterpret_cast<const _Float16*>(f)[i] : reinterpret_cast<const float*>(f)[i];
}
// Streaming (non-temporal) 16-B stores for the probe's zero fill: whole 128-B lines per 8 lanes,
// read by no kernel of this launch.  Measured (profiles/r01f_gather_nt_ablation.txt): the gather
// 1.53 -> 1.39 ms, and 1.36 ms with the search's c rows (8 lanes x 16 B = one 128-B row) streamed
// too.  On partial lines they cost far more: with the search's 4-B idx/w stores streamed the
// gather took 2.05 ms, and the MLP's 8-B activation saves made the training forward 5x slower
// (10.8 -> 51.7 ms), so both keep ordinary stores.
#ifndef PNR_NT_FILL
#define PNR_NT_FILL 1
#endif
template <typename T>
__device__ __forceinline__ void nt_store(T* p, const T& v) {
  if (PNR_NT_FILL) {
    __builtin_nontemporal_store(v.x, &p->x);
    __builtin_nontemporal_store(v.y, &p->y);
    __builtin_nontemporal_store(v.z, &p->z);
    __builtin_nontemporal_store(v.w, &p->w);
  } else {
    *p = v;
  }
}

// Work lists: samples are appended by wave (one atomic per wave) to one of kLists sub-lists, each
// with its own counter on its own 128-B line, dealt round-robin by wave -- a single counter would
// serialise ~10^5 same-address atomics.  Consumers walk (sub-list, 256-item chunk) tasks.
constexpr int kLists = 64;
struct WorkList {
  uint32_t* cnt;   // [kLists * 32], counter r at cnt[32 r]
  float4* items;   // [kLists][cap]
  int64_t cap;     // per sub-list capacity
};

static int64_t wl_cap(int64_t rows) {
  const int64_t waves = (rows + 63) / 64;
  return (waves + kLists - 1) / kLists * 64;
}
static size_t wl_bytes(int64_t rows) { return (size_t)kLists * 32 * 4 + (size_t)kLists * wl_cap(rows) * 16; }
static WorkList wl_view(void* ws, int64_t rows) {
  WorkList w;
  w.cnt = static_cast<uint32_t*>(ws);
  w.items = reinterpret_cast<float4*>(static_cast<char*>(ws) + kLists * 32 * 4);
  w.cap = wl_cap(rows);
  return w;
}

__device__ __forceinline__ void wl_append(const WorkList& wl, bool has, const float4& item) {
  const uint64_t m = __ballot(has);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int r = (int)(((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kLists - 1));
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(wl.cnt + r * 32, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  if (has) wl.items[(int64_t)r * wl.cap + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = item;
}

struct GatherArgs {
  PointSrc src;
  int64_t P, rows;
  HashGrid g;
  const int4* hdr;
  const int4* sub;       // per bucket: sub-cell end offsets (k_bucket_sub)
  const float4* sorted;
  const float4* feats4;  // (M, 8) float4, or (M, 32) f16 when feat_half
  const float* xyz;      // (M, 3)
  const uint32_t* occ;   // occupancy filter
  int feat_half;         // features stored as float16 (pnr_points.feat_half)
  int k;
  float r2, eps;
  float h0, h1, h2;      // trilinear spacing
  float rho0, rho1, rho2;  // neighbourhood reach per axis in cell units, with a 2^-10 margin
  float* c;              // (rows, 32)
  int32_t* idx;          // (rows, k) or null
  float* w;              // (rows, k) or null
  WorkList wl;           // (x, y, z, sample row bits) of the samples that may have neighbours
};

// Pass 1, one thread per sample row: the occupancy bit of each sample's probe block; the hits go
// to the work list, the block zero-fills the other rows of its 256 with coalesced stores.
template <int SRC>
__global__ __launch_bounds__(256) void k_gather_probe(GatherArgs a) {
  PNR_FP_STRICT
  __shared__ uint8_t s_has[256];
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int64_t nrow = a.rows - r0 < 256 ? a.rows - r0 : 256;
  const int64_t p = r0 + threadIdx.x;
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool has = false;
  if (p < a.P) {
    bool inside;
    load_point<SRC>(a.src, p, x0, x1, x2, inside);
    int bx, by, bz;
    base_cell(x0, a.g.o0, a.g.inv, bx);
    base_cell(x1, a.g.o1, a.g.inv, by);
    base_cell(x2, a.g.o2, a.g.inv, bz);
    const uint32_t bit = cell_hash(bx, by, bz, a.g.omask);
    has = (a.occ[bit >> 5] >> (bit & 31u)) & 1u;
  }
  s_has[threadIdx.x] = has ? 1 : 0;
  __syncthreads();
  // coalesced zero fill of the rows the search pass will not write
  {
    float4* c4 = reinterpret_cast<float4*>(a.c) + r0 * 8;
    for (int e = threadIdx.x; e < nrow * 8; e += 256)
      if (!s_has[e >> 3]) nt_store(c4 + e, make_float4(0.f, 0.f, 0.f, 0.f));
    if (a.idx && p < a.rows && !has) {  // this row's k (index, weight) slots
      if (a.k == 8 && ((reinterpret_cast<uintptr_t>(a.idx) | reinterpret_cast<uintptr_t>(a.w)) & 15) == 0) {
        int4* i4 = reinterpret_cast<int4*>(a.idx) + p * 2;
        float4* w4 = reinterpret_cast<float4*>(a.w) + p * 2;
        nt_store(i4, make_int4(-1, -1, -1, -1));
        nt_store(i4 + 1, make_int4(-1, -1, -1, -1));
        nt_store(w4, make_float4(0.f, 0.f, 0.f, 0.f));
        nt_store(w4 + 1, make_float4(0.f, 0.f, 0.f, 0.f));
      } else {
        for (int t = 0; t < a.k; ++t) {
          a.idx[p * a.k + t] = -1;
          a.w[p * a.k + t] = 0.f;
        }
      }
    }
  }
  wl_append(a.wl, has, make_float4(x0, x1, x2, __int_as_float((int)p)));
}

// Pass 2, persistent blocks over the work list, one thread per sample.  A thread's non-empty
// probe ranges (own bucket whole; colliding bucket with a per-point cell test; foreign bucket not
// at all) are compacted into its LDS row, so the candidate loop is ONE flat loop over all of them
// (trip count = the wave's largest candidate total) with the next range read ahead.  Top-k is a
// branch-free insertion network on (d2, index) keys packed into positive doubles (their order is
// the lexicographic one): v_min_f64 / v_max_f64 by inline asm, 2 VALU per stage (the builtins add
// an IEEE canonicalisation per operand).  The feature sum then runs 8 lanes per sample, 4 feature
// rows in flight per lane.
// end offset of sub-cell k (0..7) in a bucket's sub table (8 x u16)
__device__ __forceinline__ int sub_end(const int4& sb, int k) {
  const int w = k < 2 ? sb.x : (k < 4 ? sb.y : (k < 6 ? sb.z : sb.w));
  return (int)(((uint32_t)w >> (16 * (k & 1))) & 0xFFFFu);
}
// per axis: bits 2c+h (c = block cell 0/1, h = half) of the half-cells that [u - rho', u + rho']
// touches, u = (x - o) * inv as in cell_coord and b = the block's first cell
__device__ __forceinline__ uint32_t half_mask(float x, float o, float inv, float rho, int b) {
  PNR_FP_STRICT
  float u = (x - o) * inv;
  u = fminf(fmaxf(u, -1.0e9f), 1.0e9f);
  const float r = rho + fabsf(u) * 6.0e-7f;
  const int lo = (int)floorf(2.0f * (u - r)) - 2 * b, hi = (int)floorf(2.0f * (u + r)) - 2 * b;
  uint32_t m = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) m |= (lo <= k && k <= hi) ? (1u << k) : 0u;
  return m;
}

// one network stage: key <- min(key, kn), return max(key, kn); key is updated in place (a tied
// operand), so the unrolled network carries no register copies around the candidate loop
__device__ __forceinline__ double kstage(double& key, double kn) {
  double hi;
  asm("v_max_f64 %1, %0, %2\n\tv_min_f64 %0, %0, %2" : "+v"(key), "=&v"(hi) : "v"(kn));
  return hi;
}

// One wave per search block: a round's barriers then never hold a finished wave behind the
// block's slowest one.  1.25 -> 1.20 ms per gather against 256-thread blocks (128: 1.22 ms;
// profiles/r01g_gather_occupancy_ablation.txt).
#ifndef PNR_SEARCH_BLOCK
#define PNR_SEARCH_BLOCK 64
#endif
constexpr int kSearchBlock = PNR_SEARCH_BLOCK;
union SearchLds {
  struct {
    int2 rng[8][kSearchBlock];      // [range][thread] (start, end): conflict-free per-thread access
    uint8_t cell[8][kSearchBlock];  // probe cell n | 8 if the bucket collides
  } r;
  struct {
    int32_t idx[kSearchBlock * PNR_MAX_K];
    float w[kSearchBlock * PNR_MAX_K];
    int32_t row[kSearchBlock];
  } f;
};

// One search round of a block: thread tid searches work item `wk` (x, y, z, row bits) when `has`;
// block-uniform call (it holds barriers).
template <int KER>
__device__ __forceinline__ void search_round(const GatherArgs& a, SearchLds& L, const float4 wk, const bool has) {
  PNR_FP_STRICT
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, gq = lane >> 3, q = lane & 7;
  const double kInf = __longlong_as_double(0x7FF0000000000000ll);
  {
    double key[PNR_MAX_K];
#pragma unroll
    for (int t = 0; t < PNR_MAX_K; ++t) key[t] = kInf;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    int row = -1, bx = 0, by = 0, bz = 0, nr = 0;
    __syncthreads();  // the previous task's feature phase is done with the LDS
    if (has) {
      x0 = wk.x; x1 = wk.y; x2 = wk.z;
      row = __float_as_int(wk.w);
      base_cell(x0, a.g.o0, a.g.inv, bx);
      base_cell(x1, a.g.o1, a.g.inv, by);
      base_cell(x2, a.g.o2, a.g.inv, bz);
      // half-cells (block-relative, 0..3 per axis) that the reach box [u - rho, u + rho] touches;
      // the margin (2^-10 of rho + 5 ulp of u) covers the f32 rounding of both sides' coordinates
      const uint32_t am0 = half_mask(x0, a.g.o0, a.g.inv, a.rho0, bx);
      const uint32_t am1 = half_mask(x1, a.g.o1, a.g.inv, a.rho1, by);
      const uint32_t am2 = half_mask(x2, a.g.o2, a.g.inv, a.rho2, bz);
#pragma unroll
      for (int n0 = 0; n0 < 8; n0 += 4) {  // 4 bucket headers + sub-cell tables in flight at a time
        int4 h[4], sb[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int n = n0 + u;
          const uint32_t bk = cell_hash(bx + (n & 1), by + ((n >> 1) & 1), bz + (n >> 2), a.g.mask);
          h[u] = a.hdr[bk];
          sb[u] = a.sub[bk];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int n = n0 + u;
          const int cx = bx + (n & 1), cy = by + ((n >> 1) & 1), cz = bz + (n >> 2);
          const uint64_t hk = (uint64_t)(uint32_t)h[u].z | ((uint64_t)(uint32_t)h[u].w << 32);
          const bool coll = (hk & kCollision) != 0;
          const bool own = (hk & ~kCollision) == cell_key(cx, cy, cz);
          // this cell's wanted sub-cells (x fastest) and the one span from the first to the last
          const uint32_t xm = (am0 >> (2 * (n & 1))) & 3u, ym = (am1 >> (2 * ((n >> 1) & 1))) & 3u,
                         zm = (am2 >> (2 * (n >> 2))) & 3u;
          const uint32_t plane = ((ym & 1u) ? xm : 0u) | ((ym & 2u) ? xm << 2 : 0u);
          const uint32_t m = ((zm & 1u) ? plane : 0u) | ((zm & 2u) ? plane << 4 : 0u);
          int s0 = h[u].x, s1 = h[u].y;
          if (m != 0u && (((uint32_t)sb[u].w >> 16) != 0xFFFFu)) {  // an ordered bucket: the span only
            const int f = __ffs((int)m) - 1, l = 31 - __clz((int)m);
            s0 = h[u].x + (f == 0 ? 0 : sub_end(sb[u], f - 1));
            s1 = h[u].x + sub_end(sb[u], l);
          }
          if ((coll || own) && m != 0u && s1 > s0) {
            L.r.rng[nr][tid] = make_int2(s0, s1);
            L.r.cell[nr][tid] = (uint8_t)(n | (coll ? 8 : 0));
            ++nr;
          }
        }
      }
    }
    // flat candidate loop over the nr ranges; uniform over the wave (finished lanes insert +inf, a
    // no-op), so the key registers are updated in place with no copies at the loop head
    int jj = 0, je = 0, cf = 0, k = 0;
    int2 nx = nr > 0 ? L.r.rng[0][tid] : make_int2(0, 0);
    while (true) {
      const bool act = jj < je || k < nr;
      if (__ballot(act) == 0) break;
      double kn = kInf;
      if (act) {
        if (jj >= je) {
          jj = nx.x;
          je = nx.y;
          cf = L.r.cell[k][tid];
          ++k;
          if (k < nr) nx = L.r.rng[k][tid];  // read ahead
        }
        const float4 qv = a.sorted[jj++];
        const float d0 = x0 - qv.x, d1 = x1 - qv.y, d2 = x2 - qv.z;
        const float dd = (d0 * d0 + d1 * d1) + d2 * d2;
        bool ok;
        if (KER == PNR_GATHER_IDW) ok = dd <= a.r2;
        else ok = fabsf(d0) < a.h0 && fabsf(d1) < a.h1 && fabsf(d2) < a.h2;
        if (cf & 8) {  // colliding bucket: the point must lie in this probe cell
          ok = ok && cell_coord(qv.x, a.g.o0, a.g.inv) == bx + (cf & 1) &&
               cell_coord(qv.y, a.g.o1, a.g.inv) == by + ((cf >> 1) & 1) &&
               cell_coord(qv.z, a.g.o2, a.g.inv) == bz + ((cf >> 2) & 1);
        }
        if (ok) kn = pack_key(dd, __float_as_int(qv.w));
      }
#pragma unroll
      for (int t = 0; t < PNR_MAX_K; ++t) kn = kstage(key[t], kn);
    }
    // weights of the first k, normalised by their sequential sum (ascending distance)
    float wv_[PNR_MAX_K];
    int ki[PNR_MAX_K];
    float W = 0.f;
#pragma unroll
    for (int t = 0; t < PNR_MAX_K; ++t) {
      float w = 0.f;
      const bool v = t < a.k && key[t] != kInf;
      ki[t] = v ? key_id(key[t]) : -1;
      if (v) {
        if (KER == PNR_GATHER_IDW) {
          w = 1.0f / fmaxf(sqrtf(key_d2(key[t])), a.eps);
        } else {  // per-axis offsets of the kept point (same f32 arithmetic as the search)
          const float* xi = a.xyz + (int64_t)ki[t] * 3;
          const float t0 = 1.0f - fabsf(x0 - xi[0]) / a.h0;
          const float t1 = 1.0f - fabsf(x1 - xi[1]) / a.h1;
          const float t2 = 1.0f - fabsf(x2 - xi[2]) / a.h2;
          w = (t0 * t1) * t2;
        }
      }
      wv_[t] = w;
      W = W + w;
    }
    const float Wd = W > 0.f ? W : 1.0f;
    __syncthreads();  // every thread is past its range reads: the LDS becomes the feature lists
    L.f.row[tid] = row;
    float wnv[PNR_MAX_K];
#pragma unroll
    for (int t = 0; t < PNR_MAX_K; ++t) {
      const float wn = ki[t] >= 0 ? wv_[t] / Wd : 0.f;
      wnv[t] = wn;
      L.f.idx[tid * PNR_MAX_K + t] = ki[t];
      L.f.w[tid * PNR_MAX_K + t] = wn;
    }
    if (row >= 0 && a.idx) {
      // k = 8: the row's 8 indices and 8 weights as 16-B stores (1.37 -> 1.31 ms per gather)
      if (PNR_MAX_K == 8 && a.k == 8 && ((reinterpret_cast<uintptr_t>(a.idx) | reinterpret_cast<uintptr_t>(a.w)) & 15) == 0) {
        int4* i4 = reinterpret_cast<int4*>(a.idx) + (int64_t)row * 2;
        float4* w4 = reinterpret_cast<float4*>(a.w) + (int64_t)row * 2;
        i4[0] = make_int4(ki[0], ki[1], ki[2], ki[3]);
        i4[1] = make_int4(ki[4], ki[5], ki[6], ki[7]);
        w4[0] = make_float4(wnv[0], wnv[1], wnv[2], wnv[3]);
        w4[1] = make_float4(wnv[4], wnv[5], wnv[6], wnv[7]);
      } else {
        for (int t = 0; t < a.k; ++t) {
          a.idx[(int64_t)row * a.k + t] = ki[t];
          a.w[(int64_t)row * a.k + t] = wnv[t];
        }
      }
    }
    __syncthreads();
    // feature sum: 8 lanes per sample, lane q owns channels 4q..4q+3
#pragma unroll 1
    for (int rr = 0; rr < 8; ++rr) {
      const int sl = wv * 64 + rr * 8 + gq;
      const int rw = L.f.row[sl];
      if (rw < 0) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t0 = 0; t0 < PNR_MAX_K; t0 += 4) {  // 4 feature rows in flight
        int id[4];
        float4 f[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          id[t] = L.f.idx[sl * PNR_MAX_K + t0 + t];
          f[t] = make_float4(0.f, 0.f, 0.f, 0.f);
          if (id[t] >= 0) f[t] = load_feat4(a.feats4, a.feat_half, (int64_t)id[t] * 8 + q);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (id[t] >= 0) {
            const float wn = L.f.w[sl * PNR_MAX_K + t0 + t];
            acc.x = acc.x + wn * f[t].x;
            acc.y = acc.y + wn * f[t].y;
            acc.z = acc.z + wn * f[t].z;
            acc.w = acc.w + wn * f[t].w;
          }
        }
      }
      nt_store(reinterpret_cast<float4*>(a.c) + (int64_t)rw * 8 + q, acc);  // 8 lanes: one 128-B row
    }
  }
}

// Pass 2: persistent blocks over the probe's work list, one search round per kSearchBlock-item chunk.
template <int KER>
// The search is latency-bound: 7 waves per SIMD (72 VGPRs, one 8-B spill) instead of the 6 its
// free allocation gives: 1.31 -> 1.25 ms per gather.  8 waves (64 VGPRs, 11 spills) measured the
// same as 7; 8 header loads in flight instead of 4 cost 2 waves of occupancy and took 1.49 ms
// (profiles/r01g_gather_occupancy_ablation.txt).
#ifndef PNR_SEARCH_WAVES
#define PNR_SEARCH_WAVES 7
#endif
__global__ __launch_bounds__(kSearchBlock, PNR_SEARCH_WAVES) void k_gather_search(GatherArgs a) {
  __shared__ SearchLds L;
  const int64_t nchunk = (a.wl.cap + kSearchBlock - 1) / kSearchBlock;
  for (int64_t task = blockIdx.x; task < kLists * nchunk; task += gridDim.x) {
    const int r = (int)(task % kLists);
    const int64_t j0 = task / kLists * kSearchBlock;
    const int64_t n_work = (int64_t)a.wl.cnt[r * 32];
    if (j0 >= n_work) continue;  // uniform over the block
    const int64_t i = j0 + threadIdx.x;
    const bool has = i < n_work;
    const float4 wk = has ? a.wl.items[r * a.wl.cap + i] : make_float4(0.f, 0.f, 0.f, 0.f);
    search_round<KER>(a, L, wk, has);
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
  int feat_half;
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
  WorkList wl;           // rows with at least one neighbour
};

// rows with a neighbour (idx[row][0] >= 0: neighbours are stored nearest first) -> work list
__global__ __launch_bounds__(256) void k_gather_bwd_probe(GatherBwdArgs a) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool has = p < a.P && a.idx[p * a.k] >= 0;
  wl_append(a.wl, has, make_float4(0.f, 0.f, 0.f, __int_as_float((int)p)));
}

// Half a wave per row: lane c owns channel c, so the feature-gradient atomics of one neighbour
// are ONE instruction per two rows, each row a whole 128-B line (2 full 64-B atomic requests).
template <int SRC, int KER>
__global__ __launch_bounds__(256) void k_gather_bwd(GatherBwdArgs a) {
  PNR_FP_STRICT
  const int ch = threadIdx.x & 31, half = threadIdx.x >> 5;  // 8 half-waves per block
  const int64_t nchunk = (a.wl.cap + 255) / 256;
  for (int64_t task = blockIdx.x; task < kLists * nchunk; task += gridDim.x) {
    const int rl = (int)(task % kLists);
    const int64_t j0 = task / kLists * 256;
    const int64_t n_work = (int64_t)a.wl.cnt[rl * 32];
    if (j0 >= n_work) continue;  // uniform over the block
    const int64_t jn = n_work - j0 < 256 ? n_work - j0 : 256;
    // half-wave `half` takes 32 consecutive items: rows of one ray, whose neighbour lists overlap.
    // A neighbour shared with the previous row carries its partial sum forward instead of being
    // flushed: the atomic goes out when it leaves the list (or at the end of the run).
    int pid[PNR_MAX_K];
    float pacc[PNR_MAX_K];
#pragma unroll
    for (int kk = 0; kk < PNR_MAX_K; ++kk) {
      pid[kk] = -1;
      pacc[kk] = 0.f;
    }
    const int64_t te = 32 * half + 32 < jn ? 32 * half + 32 : jn;
#pragma unroll 1
    for (int64_t t = 32 * half; t < te; ++t) {  // uniform over each half-wave
      const int64_t p = __float_as_int(a.wl.items[rl * a.wl.cap + j0 + t].w);
      // every load of the row issued at once: g_c / c rows, the k (index, weight) pairs (broadcast
      // within the half-wave), then the k feature rows and atomics predicated, no dependent branches
      const float g = a.g_c[p * 32 + ch];
      const float cc = a.g_p ? a.c[p * 32 + ch] : 0.f;
      int id[PNR_MAX_K];
      float wn[PNR_MAX_K];
#pragma unroll
      for (int kk = 0; kk < PNR_MAX_K; ++kk) {
        id[kk] = kk < a.k ? a.idx[p * a.k + kk] : -1;
        wn[kk] = kk < a.k ? a.w[p * a.k + kk] : 0.f;
      }
      float x0 = 0.f, x1 = 0.f, x2 = 0.f;
      float xi[PNR_MAX_K][3];
      if (a.g_p && ch == 0) {  // the point and its neighbours' positions, in flight during the sums
        if (a.xP) {
          const float4 xv = a.xP[p];
          x0 = xv.x; x1 = xv.y; x2 = xv.z;
        } else {
          bool inside;
          load_point<SRC>(a.src, p, x0, x1, x2, inside);
        }
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) {
          const int64_t j = id[kk] >= 0 ? id[kk] : 0;
          xi[kk][0] = a.xyz[j * 3 + 0];
          xi[kk][1] = a.xyz[j * 3 + 1];
          xi[kk][2] = a.xyz[j * 3 + 2];
        }
      }
      float dots[PNR_MAX_K];
      if (a.g_p) {
        float f[PNR_MAX_K];
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk)
          f[kk] = id[kk] >= 0 ? load_feat1(a.feats4, a.feat_half, (int64_t)id[kk] * 32 + ch) : 0.f;
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) dots[kk] = g * f[kk];
      }
      if (a.g_feats) {
        float cur[PNR_MAX_K];
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) cur[kk] = id[kk] >= 0 ? wn[kk] * g : 0.f;
#pragma unroll
        for (int j = 0; j < PNR_MAX_K; ++j) {  // ids within a row are distinct: at most one match
          bool kept = false;
#pragma unroll
          for (int kk = 0; kk < PNR_MAX_K; ++kk) {
            const bool mt = pid[j] >= 0 && id[kk] == pid[j];
            cur[kk] += mt ? pacc[j] : 0.f;
            kept = kept || mt;
          }
          if (pid[j] >= 0 && !kept) unsafeAtomicAdd(a.g_feats + (int64_t)pid[j] * 32 + ch, pacc[j]);
        }
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) {
          pid[kk] = id[kk];
          pacc[kk] = cur[kk];
        }
      }
      if (!a.g_p) continue;
      float gcd = g * cc;
#pragma unroll
      for (int m = 1; m < 32; m <<= 1) {  // sums over the 32 channels (xor stays inside the half-wave)
        gcd += __shfl_xor(gcd, m);
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) dots[kk] += __shfl_xor(dots[kk], m);
      }
      if (ch != 0) continue;
      // dL/dp = sum_k wn_k (g.f_k - g.c) (1/w_k) dw_k/dp
      float gp0 = 0.f, gp1 = 0.f, gp2 = 0.f;
#pragma unroll
      for (int kk = 0; kk < PNR_MAX_K; ++kk) {
        if (id[kk] < 0) continue;
        const float d0 = x0 - xi[kk][0], d1 = x1 - xi[kk][1], d2 = x2 - xi[kk][2];
        const float coef = wn[kk] * (dots[kk] - gcd);
        if (KER == PNR_GATHER_IDW) {
          const float dd = (d0 * d0 + d1 * d1) + d2 * d2;
          if (sqrtf(dd) > a.eps) {  // w = 1/|d|: (1/w) dw/dp = -d / |d|^2
            const float fq = -coef / dd;
            gp0 += fq * d0; gp1 += fq * d1; gp2 += fq * d2;
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
    if (a.g_feats) {
#pragma unroll
      for (int j = 0; j < PNR_MAX_K; ++j)
        if (pid[j] >= 0) unsafeAtomicAdd(a.g_feats + (int64_t)pid[j] * 32 + ch, pacc[j]);
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------------------
// cell >= 2 reach (1 + 2^-9): the search widens the reach by 2^-10 (+ 5 ulp of the cell coordinate)
// and its half-cell masks only cover the 2x2x2 probe block, so the widened reach must stay <= half a
// cell; at cell == 2 reach a neighbour on the block edge could be dropped by f32 rounding
// (pnr.NeuralPoints applies the same bound)
constexpr float kCellMargin = 1.0f + 1.0f / 512.0f;
static bool points_ok(const pnr_points& pts) {
  const float reach = pts.mode == PNR_GATHER_IDW
                          ? pts.radius
                          : fmaxf(pts.spacing[0], fmaxf(pts.spacing[1], pts.spacing[2]));
  return pts.n_points >= 0 && pts.k >= 1 && pts.k <= PNR_MAX_K && pts.table_bits >= 10 && pts.table_bits <= 24 &&
         pts.index && (pts.mode == PNR_GATHER_IDW || pts.mode == PNR_GATHER_TRILINEAR) && reach > 0.f &&
         pts.cell >= 2.0f * reach * kCellMargin && (pts.n_points == 0 || (pts.xyz && pts.feats));
}

// persistent grid = the blocks of `kern` resident at once (a later wave of blocks would run as a
// tail), at most `tasks`; queried once per (kernel, block size, device): template variants of one
// kernel share a function-pointer type, so the cache is keyed by the pointer itself
template <typename K>
static unsigned resident_grid(K kern, int block, int64_t tasks) {
  struct Entry {
    const void* kern;
    int block, dev, resident;
  };
  static Entry cache[64];
  static int n_cache = 0;
  static std::mutex mu;
  int dev = 0;
  (void)hipGetDevice(&dev);
  int resident = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    for (int i = 0; i < n_cache; ++i)
      if (cache[i].kern == (const void*)kern && cache[i].block == block && cache[i].dev == dev) resident = cache[i].resident;
    if (!resident) {
      int cus = 0, per = 0;
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kern, block, 0);
      resident = (cus > 0 && per > 0) ? cus * per : 2048;
      if (n_cache < 64) cache[n_cache++] = Entry{(const void*)kern, block, dev, resident};
    }
  }
  return (unsigned)(tasks < resident ? tasks : resident);
}

static void gather_probe(int mode, dim3 grid, hipStream_t st, const GatherArgs& a) {
  switch (mode) {
    case kPtsF64: hipLaunchKernelGGL((k_gather_probe<kPtsF64>), grid, dim3(256), 0, st, a); break;
    case kPtsF32: hipLaunchKernelGGL((k_gather_probe<kPtsF32>), grid, dim3(256), 0, st, a); break;
    case kRaysZ64: hipLaunchKernelGGL((k_gather_probe<kRaysZ64>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_gather_probe<kRaysZ32>), grid, dim3(256), 0, st, a); break;
  }
}

size_t gather_workspace_bytes(int64_t P) { return wl_bytes(P > 0 ? P : 0); }

int launch_gather(const pnr_points& pts, const PointSrc& src, int mode, int64_t P, int64_t rows, float* c,
                  int32_t* idx, float* w, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!points_ok(pts) || mode < kPtsF64 || mode > kRaysZ32 || P < 0 || rows < P || P >= (1ll << 31)) return PNR_E_ARG;
  if (rows == 0) return PNR_OK;
  if (!ws || ws_bytes < gather_workspace_bytes(P)) return PNR_E_WORKSPACE;
  IndexView v = index_view(pts.index, pts.n_points, pts.table_bits, nullptr);
  GatherArgs a{};
  a.src = src;
  a.P = P;
  a.rows = rows;
  a.g = make_grid(pts);
  a.hdr = v.hdr;
  a.sub = v.sub;
  a.sorted = v.sorted;
  a.feats4 = reinterpret_cast<const float4*>(pts.feats);
  a.feat_half = pts.feat_half ? 1 : 0;
  a.xyz = pts.xyz;
  a.occ = v.occ;
  a.k = pts.k;
  a.r2 = pts.radius * pts.radius;
  a.eps = pts.eps;
  a.h0 = pts.spacing[0];
  a.h1 = pts.spacing[1];
  a.h2 = pts.spacing[2];
  {
    const float inv = 1.0f / pts.cell, mg = 1.0f + 1.0f / 1024.0f;
    const bool idw = pts.mode == PNR_GATHER_IDW;
    a.rho0 = (idw ? pts.radius : pts.spacing[0]) * inv * mg;
    a.rho1 = (idw ? pts.radius : pts.spacing[1]) * inv * mg;
    a.rho2 = (idw ? pts.radius : pts.spacing[2]) * inv * mg;
  }
  a.c = c;
  a.idx = idx;
  a.w = w;
  a.wl = wl_view(ws, P);
  if (hipMemsetAsync(a.wl.cnt, 0, kLists * 32 * 4, st) != hipSuccess) return (int)hipGetLastError();
  TimingScope ts(kTimeGather, P, st);
  gather_probe(mode, dim3((unsigned)((rows + 255) / 256)), st, a);
  const int64_t tasks = kLists * ((a.wl.cap + kSearchBlock - 1) / kSearchBlock);
  if (pts.mode == PNR_GATHER_IDW) {
    auto kern = k_gather_search<PNR_GATHER_IDW>;
    hipLaunchKernelGGL(kern, dim3(resident_grid(kern, kSearchBlock, tasks)), dim3(kSearchBlock), 0, st, a);
  } else {
    auto kern = k_gather_search<PNR_GATHER_TRILINEAR>;
    hipLaunchKernelGGL(kern, dim3(resident_grid(kern, kSearchBlock, tasks)), dim3(kSearchBlock), 0, st, a);
  }
  return hip_status(hipGetLastError());
}

template <int SRC, int KER>
static void gather_bwd_launch(int64_t tasks, hipStream_t st, const GatherBwdArgs& a) {
  auto kern = k_gather_bwd<SRC, KER>;
  hipLaunchKernelGGL(kern, dim3(resident_grid(kern, 256, tasks)), dim3(256), 0, st, a);
}
template <int KER>
static void gather_bwd_mode(int mode, int64_t tasks, hipStream_t st, const GatherBwdArgs& a) {
  switch (mode) {
    case kPtsF64: gather_bwd_launch<kPtsF64, KER>(tasks, st, a); break;
    case kPtsF32: gather_bwd_launch<kPtsF32, KER>(tasks, st, a); break;
    case kRaysZ64: gather_bwd_launch<kRaysZ64, KER>(tasks, st, a); break;
    default: gather_bwd_launch<kRaysZ32, KER>(tasks, st, a); break;
  }
}

int launch_gather_bwd(const pnr_points& pts, const PointSrc* src, int mode, const float4* xP, int64_t P,
                      const int32_t* idx, const float* w, const float* c, const float* g_c, float* g_p,
                      bool gp_accum, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!points_ok(pts) || P < 0 || (!src && !xP) || mode < kPtsF64 || mode > kRaysZ32 || P >= (1ll << 31))
    return PNR_E_ARG;
  if (P == 0 || (!pts.g_feats && !g_p)) return PNR_OK;
  if (!idx || !w || !g_c || (g_p && !c)) return PNR_E_ARG;
  if (!ws || ws_bytes < gather_workspace_bytes(P)) return PNR_E_WORKSPACE;
  GatherBwdArgs a{};
  if (src) a.src = *src;
  a.xP = xP;
  a.P = P;
  a.xyz = pts.xyz;
  a.feats4 = reinterpret_cast<const float4*>(pts.feats);
  a.feat_half = pts.feat_half ? 1 : 0;
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
  a.wl = wl_view(ws, P);
  if (hipMemsetAsync(a.wl.cnt, 0, kLists * 32 * 4, st) != hipSuccess) return (int)hipGetLastError();
  if (g_p && !gp_accum && hipMemsetAsync(g_p, 0, (size_t)P * 12, st) != hipSuccess) return (int)hipGetLastError();
  TimingScope ts(kTimeGatherBwd, P, st);
  hipLaunchKernelGGL(k_gather_bwd_probe, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, a);
  const int64_t tasks = kLists * ((a.wl.cap + 255) / 256);
  if (pts.mode == PNR_GATHER_IDW) gather_bwd_mode<PNR_GATHER_IDW>(mode, tasks, st, a);
  else gather_bwd_mode<PNR_GATHER_TRILINEAR>(mode, tasks, st, a);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
