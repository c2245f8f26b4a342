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
// Gather (launch_gather), the samples grouped by probe block:
//   k_gather_probe  one thread per sample row: coalesced zero fill of the block's output rows,
//                   occupancy-filter test of the sample's 2x2x2 probe block; a sample that may have
//                   neighbours takes a slot in its block's group (one counter per group-table entry,
//                   the block's base cell hashed) and goes to a work list (one atomic per wave, 64
//                   sub-lists).  Free space -- most of a ray -- costs one L2-resident bit load.
//   k_scan_*        exclusive scan of the group counts -> group start offsets.
//   k_group_scatter work items -> the grouped list (group start + slot): the samples of one probe
//                   block are contiguous.
//   k_gather_search persistent waves over 64-item chunks of the grouped list.  Per probe block in
//                   the chunk (usually one or two): lanes 0..7 load the 8 bucket headers, the wave
//                   stages the block's candidate points into LDS with coalesced loads (one global
//                   round trip per 64 candidates, shared by every sample of the block), then every
//                   lane of the block scans the staged list by broadcast LDS reads; the top-k network
//                   on packed (d2, index) float64 keys (v_min/v_max_f64, 2 VALU per stage) runs only
//                   for candidates that some lane keeps (ballot).  Normalised weights, then the
//                   feature sum with 8 lanes per sample.
//   k_gather_bwd    dL/df_i += w_k dL/dc (float atomics) and dL/dp through the weights.
#include <mutex>

#include <type_traits>

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

// One-block exclusive scan for n <= kScanSmall: thread t sums its run of consecutive elements, the
// block scans the run sums, each thread writes its run (one launch where the tiled scan takes three:
// the gather's group table at the Mapper's 1,000-ray batch has ~4 k entries; larger tables take the tiled scan:
// one block over 16 k entries took 29 us at config C5)
constexpr int64_t kScanSmall = 4096;
__global__ __launch_bounds__(1024) void k_scan_small(const int32_t* __restrict__ in, int32_t* __restrict__ out,
                                                     int64_t n) {
  __shared__ int32_t wsum[16];
  const int per = (int)((n + 1023) / 1024);
  const int64_t b = (int64_t)threadIdx.x * per;
  int t = 0;
  for (int e = 0; e < per; ++e) t += b + e < n ? in[b + e] : 0;
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
  for (int e = 0; e < per; ++e) {
    if (b + e < n) {
      out[b + e] = run;
      run += in[b + e];
    }
  }
  if (threadIdx.x == 1023) out[n] = woff + incl;
}

// out[0..n] = exclusive scan of in[0..n), out[n] = total.  scratch: scan_scratch_ints(n) ints.
static int scan_exclusive(const int32_t* in, int32_t* out, int64_t n, int32_t* scratch, hipStream_t st) {
  if (n > 0 && n <= kScanSmall) {
    hipLaunchKernelGGL(k_scan_small, dim3(1), dim3(1024), 0, st, in, out, n);
    return hip_status(hipGetLastError());
  }
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
  int2* aux;       // [kLists][cap] (group, slot in the group) of each item, or null
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
  w.aux = nullptr;
  return w;
}

// Group table of the forward gather: G = 2^gbits counters, one per hashed probe-block base cell
// (a few blocks may share an entry; the search separates them), sized from the sample count
static int group_bits(int64_t P) {
  int b = 10;
  while (b < 22 && (1ll << b) < P / 32) ++b;
  return b;
}
struct GroupView {
  WorkList wl;       // items + aux
  int32_t* gcnt;     // [G]
  int32_t* gstart;   // [G + 1]
  int32_t* scratch;  // scan scratch
  float4* grouped;   // [P] items in group order
  int gbits;
};
static GroupView group_view(void* ws, int64_t P, size_t* bytes) {
  GroupView v{};
  char* b = static_cast<char*>(ws);
  size_t off = 0;
  auto take = [&](size_t n) {
    char* p = b ? b + off : nullptr;
    off += a256(n);
    return p;
  };
  char* wl = take(wl_bytes(P));
  v.wl = wl_view(wl, P);
  v.wl.aux = reinterpret_cast<int2*>(take((size_t)kLists * v.wl.cap * 8));
  v.gbits = group_bits(P);
  const int64_t G = 1ll << v.gbits;
  v.gcnt = reinterpret_cast<int32_t*>(take((size_t)G * 4));
  v.gstart = reinterpret_cast<int32_t*>(take((size_t)(G + 1) * 4));
  v.scratch = reinterpret_cast<int32_t*>(take((size_t)scan_scratch_ints(G) * 4));
  v.grouped = reinterpret_cast<float4*>(take((size_t)(P > 0 ? P : 1) * 16));
  if (bytes) *bytes = off;
  return v;
}

__device__ __forceinline__ void wl_append(const WorkList& wl, bool has, const float4& item,
                                          int2 aux = make_int2(0, 0)) {
  const uint64_t m = __ballot(has);
  if (m == 0) return;
  const int lane = threadIdx.x & 63;
  const int r = (int)(((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) & (kLists - 1));
  const int leader = __ffsll((unsigned long long)m) - 1;
  uint32_t base = 0;
  if (lane == leader) base = atomicAdd(wl.cnt + r * 32, (uint32_t)__popcll(m));
  base = __shfl(base, leader);
  if (has) {
    const int64_t at = (int64_t)r * wl.cap + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    wl.items[at] = item;
    if (wl.aux) wl.aux[at] = aux;
  }
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
  int32_t* gcnt;         // [G] samples per group (probe block base cell hashed with gmask)
  const int32_t* gstart; // [G + 1] group start offsets in `grouped`; gstart[G] = all items
  float4* grouped;       // the work items in group order
  uint32_t gmask;        // G - 1
  int chunk;             // work items per search chunk (one wave): 64, or fewer for small launches
};

// Pass 1, one thread per sample row: the occupancy bit of each sample's probe block; the hits go
// to the work list, the block zero-fills the other rows of its 256 with coalesced stores.
// zero rows (c, and the k index / weight slots) of a probe block: the rows without a work item, or
// every row (all: the search rewrites the rows of its items)
__device__ __forceinline__ void probe_fill(const GatherArgs& a, int64_t r0, int64_t nrow, int64_t p, bool has,
                                           const uint8_t* s_has, bool all) {
  float4* c4 = reinterpret_cast<float4*>(a.c) + r0 * 8;
  for (int e = threadIdx.x; e < nrow * 8; e += 256)
    if (all || !s_has[e >> 3]) nt_store(c4 + e, make_float4(0.f, 0.f, 0.f, 0.f));
  if (a.idx && p < a.rows && (all || !has)) {  // this row's k (index, weight) slots
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

template <int SRC>
__global__ __launch_bounds__(256) void k_gather_probe(GatherArgs a) {
  PNR_FP_STRICT
  __shared__ uint8_t s_has[256];
  const int64_t r0 = (int64_t)blockIdx.x * 256;
  const int64_t nrow = a.rows - r0 < 256 ? a.rows - r0 : 256;
  const int64_t p = r0 + threadIdx.x;
#if defined(PNR_EXP_FILLALL)  // experiment: every row zero-filled first, with no wait on the test
  probe_fill(a, r0, nrow, p, false, s_has, true);
#endif
  float x0 = 0.f, x1 = 0.f, x2 = 0.f;
  bool has = false;
  int bx = 0, by = 0, bz = 0;
  if (p < a.P) {
    bool inside;
    load_point<SRC>(a.src, p, x0, x1, x2, inside);
    base_cell(x0, a.g.o0, a.g.inv, bx);
    base_cell(x1, a.g.o1, a.g.inv, by);
    base_cell(x2, a.g.o2, a.g.inv, bz);
    const uint32_t bit = cell_hash(bx, by, bz, a.g.omask);
    has = (a.occ[bit >> 5] >> (bit & 31u)) & 1u;
  }
  int2 gs = make_int2(0, 0);  // (group, slot in the group)
  if (has) gs.x = (int)cell_hash(bx, by, bz, a.gmask);
#if !defined(PNR_PROBE_SERIAL)
  // The zero fill goes out first (stores: nothing waits on them), then the work-list atomic and the
  // group atomics are all issued before any of their returns is read, so one wave pays one
  // round trip instead of a chain of them in front of its fill.
  // (each wave filling its own 64 rows from its ballot, with no block barrier, measured no faster:
  // 1.080-1.090 against 1.068-1.083 ms per gather)
  s_has[threadIdx.x] = has ? 1 : 0;
  __syncthreads();
  probe_fill(a, r0, nrow, p, has, s_has, false);
  {
    const int lane = threadIdx.x & 63;
    const uint64_t m = __ballot(has);
    if (m == 0) return;
    const int r = (int)(((int64_t)blockIdx.x * 4 + (threadIdx.x >> 6)) & (kLists - 1));
    const int wl_leader = __ffsll((unsigned long long)m) - 1;
    uint32_t wl_base = 0;
    if (lane == wl_leader) wl_base = atomicAdd(a.wl.cnt + r * 32, (uint32_t)__popcll(m));
    int my_atom = 0, my_leader = 0, my_rank = 0;
    uint64_t todo = m;
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int gl = __builtin_amdgcn_readlane(gs.x, leader);
      const uint64_t peers = __ballot(has && gs.x == gl) & todo;
      if (lane == leader) my_atom = atomicAdd(a.gcnt + gl, (int)__popcll(peers));
      if ((peers >> lane) & 1ull) {
        my_leader = leader;
        my_rank = (int)__popcll(peers & ((1ull << lane) - 1ull));
      }
      todo &= ~peers;
    }
    gs.y = __shfl(my_atom, my_leader) + my_rank;
    wl_base = __shfl(wl_base, wl_leader);
    if (has) {
      const int64_t at = (int64_t)r * a.wl.cap + wl_base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      a.wl.items[at] = make_float4(x0, x1, x2, __int_as_float((int)p));
      a.wl.aux[at] = gs;
    }
  }
#else
  {
    // one atomic per distinct group of the wave: consecutive samples of a ray share probe blocks,
    // and same-address atomics of one instruction serialise in L2 (slots: base + rank among the peers)
    const int lane = threadIdx.x & 63;
    uint64_t todo = __ballot(has);
    while (todo) {
      const int leader = __ffsll((unsigned long long)todo) - 1;
      const int gl = __builtin_amdgcn_readlane(gs.x, leader);
      const uint64_t peers = __ballot(has && gs.x == gl) & todo;
      int base = 0;
      if (lane == leader) base = atomicAdd(a.gcnt + gl, (int)__popcll(peers));
      base = __builtin_amdgcn_readlane(base, leader);
      if ((peers >> lane) & 1ull) gs.y = base + (int)__popcll(peers & ((1ull << lane) - 1ull));
      todo &= ~peers;
    }
  }
  s_has[threadIdx.x] = has ? 1 : 0;
#if !defined(PNR_EXP_FILLALL) && !defined(PNR_EXP_NOFILL)
  __syncthreads();
  probe_fill(a, r0, nrow, p, has, s_has, false);
#endif
  wl_append(a.wl, has, make_float4(x0, x1, x2, __int_as_float((int)p)), gs);
#endif
}

// work items -> the grouped list: grouped[gstart[group] + slot].  A block per 256-item chunk of each
// sub-list's capacity (most of them exit at once): measured against 16 blocks per sub-list striding
// over its filled part (61 us) and that loop unrolled four items deep (66 us), this is the fastest
// (57 us per 3.6M items).
__global__ __launch_bounds__(256) void k_group_scatter(GatherArgs a) {
  const int r = (int)(blockIdx.x % kLists);
  const int64_t i = (int64_t)(blockIdx.x / kLists) * 256 + threadIdx.x;
  if (i >= (int64_t)a.wl.cnt[r * 32]) return;
  const int64_t at = (int64_t)r * a.wl.cap + i;
  const int2 gs = a.wl.aux[at];
  a.grouped[a.gstart[gs.x] + gs.y] = a.wl.items[at];
}

// one network stage: key <- min(key, kn), return max(key, kn); key is updated in place (a tied
// operand), so the unrolled network carries no register copies around the candidate loop
__device__ __forceinline__ double kstage(double& key, double kn) {
  double hi;
  asm("v_max_f64 %1, %0, %2\n\tv_min_f64 %0, %0, %2" : "+v"(key), "=&v"(hi) : "v"(kn));
  return hi;
}

// Pass 2: one wave per block, persistent over 64-item chunks of the grouped list.  The samples of a
// probe block are contiguous there, so a chunk holds one or a few blocks ("segments"): per segment
// the 8 bucket headers are read by lanes 0..7, the block's candidates (the 8 cells' buckets: own
// bucket whole, colliding bucket with a per-point cell test, foreign bucket not at all) are staged
// into LDS kCandBatch at a time by coalesced loads, and every lane of the segment scans them by
// broadcast LDS reads.  Against a thread per sample walking its own candidates through global
// memory, a candidate costs one global load per block instead of one per sample.
constexpr int kCandBatch = 128;
typedef int v4i32 __attribute__((ext_vector_type(4)));
struct SearchLds {
  float4 cand[kCandBatch + 1];   // staged candidate points (x, y, z, index bits) + pair padding
  uint8_t tag[kCandBatch + 1];   // probe cell n | 8 if its bucket collides
  int32_t idx[64 * PNR_MAX_K];
  float w[64 * PNR_MAX_K];
  int32_t row[64];
};

// feature-sum rows per round (k_gather_search) and the waves per SIMD its registers allow
#ifndef PNR_FEAT_ROWS
#define PNR_FEAT_ROWS 2
#endif
#ifndef PNR_SEARCH_WAVES
#define PNR_SEARCH_WAVES (PNR_FEAT_ROWS > 1 ? 5 : 7)
#endif
// HALF: float16 features (pnr_points.feat_half), its own instantiation (a run-time dtype branch in the
// feature rounds added register pressure that spilled)
// PAR (candidate-parallel, small chunks of ncs <= 8 items): lane l works for item l mod ncs and
// visits every (64 / ncs)-th staged candidate, keeping a partial top-k; after the segments the
// partial lists of an item's lanes are merged by a butterfly of bitonic merges.  A segment's serial
// scan then runs over 1 / (64 / ncs) of its candidates (the Mapper's real batches: chunks of 4 items,
// each a segment of its own, whose scan over a dense block dominated the search).  Keys are unique
// (d^2, index) pairs, so the merged list is the oracle's whatever lane visited which candidate.
template <int KER, bool HALF, bool PAR>
__global__ __launch_bounds__(64, PNR_SEARCH_WAVES) void k_gather_search(GatherArgs a) {
  PNR_FP_STRICT
  __shared__ SearchLds L;
  const int lane = threadIdx.x, gq = lane >> 3, q = lane & 7;
  const double kInf = __longlong_as_double(0x7FF0000000000000ll);
  const int64_t n_items = a.gstart[(int64_t)a.gmask + 1];
  const int ncs = PAR ? a.chunk : 64;  // items per chunk
  const int64_t nchunk = (n_items + ncs - 1) / ncs;
  for (int64_t chunk = blockIdx.x; chunk < nchunk; chunk += gridDim.x) {
    const int64_t it = chunk * ncs + (PAR ? (lane & (ncs - 1)) : lane);
    const bool has = (PAR || lane < ncs) && it < n_items;
    float x0 = 0.f, x1 = 0.f, x2 = 0.f;
    int row = -1, bx = 0, by = 0, bz = 0;
    if (has) {
      const float4 wk = a.grouped[it];
      x0 = wk.x; x1 = wk.y; x2 = wk.z;
      row = __float_as_int(wk.w);
      base_cell(x0, a.g.o0, a.g.inv, bx);
      base_cell(x1, a.g.o1, a.g.inv, by);
      base_cell(x2, a.g.o2, a.g.inv, bz);
    }
    double key[PNR_MAX_K];
#pragma unroll
    for (int t = 0; t < PNR_MAX_K; ++t) key[t] = kInf;
    uint64_t pending = __ballot(has);
    while (pending) {  // one segment (= probe block) per trip, wave-uniform
      const int leader = __ffsll((unsigned long long)pending) - 1;
      const int lbx = __builtin_amdgcn_readlane(bx, leader), lby = __builtin_amdgcn_readlane(by, leader),
                lbz = __builtin_amdgcn_readlane(bz, leader);
      const bool member = ((pending >> lane) & 1ull) && bx == lbx && by == lby && bz == lbz;
      pending &= ~__ballot(member);
      int cs[8], ce[8], cb[8], cf[8];  // wave-uniform: list start / end, bucket start, tag per cell
#if !defined(PNR_VECTOR_HDR)
      // the 8 probe cells' bucket headers by SCALAR loads (one s_load_dwordx4 each, one wait): the
      // cell coordinates are wave-uniform, so the headers land in SGPRs and the per-cell ranges, their
      // running sum and the collision tags are scalar arithmetic (no lane loads, scan or readlanes)
      {
        const int4* hp[8];
#pragma unroll
        for (int n = 0; n < 8; ++n)
          hp[n] = a.hdr + cell_hash(lbx + (n & 1), lby + ((n >> 1) & 1), lbz + (n >> 2), a.g.mask);
        v4i32 h[8];
        asm volatile(
            "s_load_dwordx4 %0, %8, 0x0\n\ts_load_dwordx4 %1, %9, 0x0\n\t"
            "s_load_dwordx4 %2, %10, 0x0\n\ts_load_dwordx4 %3, %11, 0x0\n\t"
            "s_load_dwordx4 %4, %12, 0x0\n\ts_load_dwordx4 %5, %13, 0x0\n\t"
            "s_load_dwordx4 %6, %14, 0x0\n\ts_load_dwordx4 %7, %15, 0x0\n\t"
            "s_waitcnt lgkmcnt(0)"
            : "=&s"(h[0]), "=&s"(h[1]), "=&s"(h[2]), "=&s"(h[3]), "=&s"(h[4]), "=&s"(h[5]), "=&s"(h[6]), "=&s"(h[7])
            : "s"(hp[0]), "s"(hp[1]), "s"(hp[2]), "s"(hp[3]), "s"(hp[4]), "s"(hp[5]), "s"(hp[6]), "s"(hp[7])
            : "memory");
        int run = 0;
#pragma unroll
        for (int n = 0; n < 8; ++n) {
          const int cx = lbx + (n & 1), cy = lby + ((n >> 1) & 1), cz = lbz + (n >> 2);
          const uint64_t hk = (uint64_t)(uint32_t)h[n].z | ((uint64_t)(uint32_t)h[n].w << 32);
          const bool coll = (hk & kCollision) != 0;
          const bool own = (hk & ~kCollision) == cell_key(cx, cy, cz);
          const int len = (coll || own) ? h[n].y - h[n].x : 0;
          cb[n] = (coll || own) ? h[n].x : 0;
          cs[n] = run;
          run += len;
          ce[n] = run;
          cf[n] = n | (coll ? 8 : 0);
        }
      }
#else
      // the 8 probe cells' candidate ranges, lane n < 8 for cell n
      int s0 = 0, len = 0, fl = 0;
      if (lane < 8) {
        const int cx = lbx + (lane & 1), cy = lby + ((lane >> 1) & 1), cz = lbz + (lane >> 2);
        const int4 h = a.hdr[cell_hash(cx, cy, cz, a.g.mask)];
        const uint64_t hk = (uint64_t)(uint32_t)h.z | ((uint64_t)(uint32_t)h.w << 32);
        const bool coll = (hk & kCollision) != 0;
        const bool own = (hk & ~kCollision) == cell_key(cx, cy, cz);
        if (coll || own) {
          s0 = h.x;
          len = h.y - h.x;
        }
        fl = lane | (coll ? 8 : 0);
      }
      int incl = len;  // inclusive scan over lanes 0..7
#pragma unroll
      for (int d = 1; d < 8; d <<= 1) {
        const int t = __shfl_up(incl, d);
        if (lane >= d) incl += t;
      }
#pragma unroll
      for (int n = 0; n < 8; ++n) {
        ce[n] = __builtin_amdgcn_readlane(incl, n);
        cs[n] = ce[n] - __builtin_amdgcn_readlane(len, n);
        cb[n] = __builtin_amdgcn_readlane(s0, n);
        cf[n] = __builtin_amdgcn_readlane(fl, n);
      }
#endif
      const int total = ce[7];
      // no colliding bucket among the 8 (the common case): no tag reads, no per-point cell test
      const bool coll_any = ((cf[0] | cf[1] | cf[2] | cf[3] | cf[4] | cf[5] | cf[6] | cf[7]) & 8) != 0;
      auto visit = [&](const float4& qv, int tg, bool coll) {
        const float d0 = x0 - qv.x, d1 = x1 - qv.y, d2 = x2 - qv.z;
        const float dd = (d0 * d0 + d1 * d1) + d2 * d2;
        bool ok;
        if (KER == PNR_GATHER_IDW) ok = dd <= a.r2;
        else ok = fabsf(d0) < a.h0 && fabsf(d1) < a.h1 && fabsf(d2) < a.h2;
        ok = ok && member;
        if (coll && (tg & 8)) {  // colliding bucket: the point must lie in this probe cell
          ok = ok && cell_coord(qv.x, a.g.o0, a.g.inv) == lbx + (tg & 1) &&
               cell_coord(qv.y, a.g.o1, a.g.inv) == lby + ((tg >> 1) & 1) &&
               cell_coord(qv.z, a.g.o2, a.g.inv) == lbz + ((tg >> 2) & 1);
        }
        if (__ballot(ok) == 0) return;  // nobody keeps it: the network would be a no-op
        double kn = ok ? pack_key(dd, __float_as_int(qv.w)) : kInf;
#if defined(PNR_EXP_NONET)  // experiment (wrong results, timing only): one stage instead of the network
        kn = kstage(key[0], kn);
#else
#pragma unroll
        for (int t = 0; t < PNR_MAX_K; ++t) kn = kstage(key[t], kn);
#endif
      };
      for (int base = 0; base < total; base += kCandBatch) {
        const int cnt = total - base < kCandBatch ? total - base : kCandBatch;
#pragma unroll
        for (int j = lane; j < kCandBatch; j += 64) {
          // both of a lane's candidates loaded unconditionally (past the batch: sorted point 0 -- the
          // search runs only when the cloud has points -- not stored), so their round trips overlap
          const int g = base + j;
          int src = 0, tg = 0;
#pragma unroll
          for (int n = 0; n < 8; ++n) {
            const bool in = g >= cs[n] && g < ce[n];
            src = in ? cb[n] + (g - cs[n]) : src;
            tg = in ? cf[n] : tg;
          }
          const float4 v = a.sorted[src];
          if (j < cnt) {
            L.cand[j] = v;
            L.tag[j] = (uint8_t)tg;
          } else if (j == cnt) {  // pair padding: a point no sample reaches (d2 = inf, never kept)
            const float inf = __int_as_float(0x7F800000);
            L.cand[j] = make_float4(inf, inf, inf, 0.f);
            L.tag[j] = 0;
          }
        }
        __syncthreads();
        if constexpr (PAR) {
          const int stride = 64 / ncs;
          if (!coll_any) {
            for (int j = lane / ncs; j < cnt; j += stride) visit(L.cand[j], 0, false);
          } else {
            for (int j = lane / ncs; j < cnt; j += stride) visit(L.cand[j], L.tag[j], true);
          }
        } else {
#if !defined(PNR_SEARCH_SERIAL)
          if (!coll_any) {
            // two candidates per trip: both LDS reads in flight before the first test
            for (int j = 0; j < cnt; j += 2) {
              const float4 q0 = L.cand[j], q1 = L.cand[j + 1];
              visit(q0, 0, false);
              visit(q1, 0, false);
            }
          } else
#endif
          {
            for (int j = 0; j < cnt; ++j) visit(L.cand[j], L.tag[j], true);
          }
        }
        __syncthreads();  // the next batch overwrites the staged list
      }
    }
    if constexpr (PAR) {
      // merge the partial lists of each item's lanes (lanes equal mod ncs): the k smallest of two
      // ascending lists as min(a_i, b_{k-1-i}) (bitonic), sorted by a bitonic merge network
      for (int d = ncs; d < 64; d <<= 1) {
        double r[PNR_MAX_K];
#pragma unroll
        for (int t = 0; t < PNR_MAX_K; ++t) {
          const double pk = __shfl_xor(key[PNR_MAX_K - 1 - t], d);
          r[t] = fmin(key[t], pk);
        }
#pragma unroll
        for (int h = PNR_MAX_K / 2; h >= 1; h >>= 1)
#pragma unroll
          for (int t = 0; t < PNR_MAX_K; ++t)
            if ((t & h) == 0) {
              const double lo = fmin(r[t], r[t + h]), hi = fmax(r[t], r[t + h]);
              r[t] = lo;
              r[t + h] = hi;
            }
#pragma unroll
        for (int t = 0; t < PNR_MAX_K; ++t) key[t] = r[t];
      }
      if (lane >= ncs) row = -1;  // one lane per item carries it on
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
#if !defined(PNR_SEARCH_NOCOMPACT)
    // feature-sum slots: rows with neighbours first, then rows without (a zero c row, no loads),
    // then empty lanes, so the feature rounds that wait on loads are only those of the ~half of the
    // rows that have neighbours; the rest store zeros without a wait
    int slot, n_live;
    {
      const bool hn = row >= 0 && ki[0] >= 0;
      const uint64_t mn = __ballot(hn), mz = __ballot(row >= 0 && !hn);
      n_live = (int)__popcll(mn | mz);
      const uint64_t below = (1ull << lane) - 1ull;
      if (hn) slot = (int)__popcll(mn & below);
      else if (row >= 0) slot = (int)__popcll(mn) + (int)__popcll(mz & below);
      else slot = (int)__popcll(mn) + (int)__popcll(mz) + (int)__popcll(~(mn | mz) & below);
    }
#else
    const int slot = lane, n_live = 64;
#endif
    L.row[slot] = row;
    float wnv[PNR_MAX_K];
#pragma unroll
    for (int t = 0; t < PNR_MAX_K; ++t) {
      const float wn = ki[t] >= 0 ? wv_[t] / Wd : 0.f;
      wnv[t] = wn;
      L.idx[slot * PNR_MAX_K + t] = ki[t];
      L.w[slot * PNR_MAX_K + t] = wn;
    }
    if (row >= 0 && a.idx) {
      // k = 8: the row's 8 indices and 8 weights as 16-B stores
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
#if PNR_FEAT_ROWS > 1
    // PNR_FEAT_ROWS samples per round: their feature loads in flight together (the loads cannot move
    // above the previous round's c stores on their own: the compiler must assume they alias).
    // Measured (tools/gather_bench.py, 13.5M samples): 1 row per round 1.22 ms, 2 rows 1.13 ms.
    // f16 features: every load of a round is issued before any of them is used (the indices read
    // from LDS first, each row loaded raw, converted afterwards).  An f16 load whose conversion sits
    // in its own branch compiled to a vmcnt(0) wait inside it, serialising the round's 16 loads
    // (measured, tools/gather_bench.py --feat-dtype float16: 1.158-1.174 -> 1.084-1.099 ms).  The
    // fp32 form keeps its direct loads (the raw form split them into 8-B halves: 1.08 -> 1.13 ms).
    if constexpr (HALF) {
#pragma unroll 1
      for (int rr = 0; rr < 8; rr += PNR_FEAT_ROWS) {
        if (rr * 8 >= n_live) break;  // the remaining slots are empty lanes
        int rw[PNR_FEAT_ROWS];
        uint2 raw[PNR_FEAT_ROWS][PNR_MAX_K];
#pragma unroll
        for (int u = 0; u < PNR_FEAT_ROWS; ++u) {
          const int sl = (rr + u) * 8 + gq;
          rw[u] = L.row[sl];
#pragma unroll
          for (int t = 0; t < PNR_MAX_K; ++t) {  // missing neighbour / empty slot: point 0, skipped below
            const int id = L.idx[sl * PNR_MAX_K + t];
            const uint32_t off = (uint32_t)(rw[u] >= 0 && id >= 0 ? id : 0) * 8u + (uint32_t)q;  // < 2^32
            raw[u][t] = reinterpret_cast<const uint2*>(a.feats4)[off];
          }
        }
#pragma unroll
        for (int u = 0; u < PNR_FEAT_ROWS; ++u) {
          if (rw[u] < 0) continue;
          const int sl = (rr + u) * 8 + gq;
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int t = 0; t < PNR_MAX_K; ++t) {
            if (L.idx[sl * PNR_MAX_K + t] >= 0) {
              const uint2 r = raw[u][t];
              const float f0 = (float)__builtin_bit_cast(_Float16, (uint16_t)(r.x & 0xffffu));
              const float f1 = (float)__builtin_bit_cast(_Float16, (uint16_t)(r.x >> 16));
              const float f2 = (float)__builtin_bit_cast(_Float16, (uint16_t)(r.y & 0xffffu));
              const float f3 = (float)__builtin_bit_cast(_Float16, (uint16_t)(r.y >> 16));
              const float wn = L.w[sl * PNR_MAX_K + t];
              acc.x = acc.x + wn * f0;
              acc.y = acc.y + wn * f1;
              acc.z = acc.z + wn * f2;
              acc.w = acc.w + wn * f3;
            }
          }
          nt_store(reinterpret_cast<float4*>(a.c) + (int64_t)rw[u] * 8 + q, acc);  // 8 lanes: one 128-B row
        }
      }
    } else {
#pragma unroll 1
      for (int rr = 0; rr < 8; rr += PNR_FEAT_ROWS) {
        if (rr * 8 >= n_live) break;  // the remaining slots are empty lanes
        int rw[PNR_FEAT_ROWS];
        float4 f[PNR_FEAT_ROWS][PNR_MAX_K];
#pragma unroll
        for (int u = 0; u < PNR_FEAT_ROWS; ++u) {
          const int sl = (rr + u) * 8 + gq;
          rw[u] = L.row[sl];
#pragma unroll
          for (int t = 0; t < PNR_MAX_K; ++t) {
            const int id = L.idx[sl * PNR_MAX_K + t];
#if defined(PNR_EXP_F32UNCOND)  // experiment: clamped, unconditional loads (point 0 for a missing one)
            f[u][t] = a.feats4[(uint32_t)(rw[u] >= 0 && id >= 0 ? id : 0) * 8u + (uint32_t)q];
#else
            f[u][t] = make_float4(0.f, 0.f, 0.f, 0.f);
            if (rw[u] >= 0 && id >= 0) f[u][t] = load_feat4(a.feats4, a.feat_half, (int64_t)id * 8 + q);
#endif
          }
        }
#pragma unroll
        for (int u = 0; u < PNR_FEAT_ROWS; ++u) {
          if (rw[u] < 0) continue;
          const int sl = (rr + u) * 8 + gq;
          float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int t = 0; t < PNR_MAX_K; ++t) {
            if (L.idx[sl * PNR_MAX_K + t] >= 0) {
              const float wn = L.w[sl * PNR_MAX_K + t];
              acc.x = acc.x + wn * f[u][t].x;
              acc.y = acc.y + wn * f[u][t].y;
              acc.z = acc.z + wn * f[u][t].z;
              acc.w = acc.w + wn * f[u][t].w;
            }
          }
          nt_store(reinterpret_cast<float4*>(a.c) + (int64_t)rw[u] * 8 + q, acc);  // 8 lanes: one 128-B row
        }
      }
    }
#else
#pragma unroll 1
#if defined(PNR_EXP_NOFEAT)  // experiment (wrong results, timing only): no feature sum
    for (int rr = 0; rr < 0; ++rr) {
#else
    for (int rr = 0; rr < 8; ++rr) {
#endif
      if (rr * 8 >= n_live) break;  // the remaining slots are empty lanes
      const int sl = rr * 8 + gq;
      const int rw = L.row[sl];
      if (rw < 0) continue;
      float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
      for (int t0 = 0; t0 < PNR_MAX_K; t0 += 4) {  // 4 feature rows in flight
        int id[4];
        float4 f[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) {  // unconditional loads (see the PNR_FEAT_ROWS > 1 form)
          id[t] = L.idx[sl * PNR_MAX_K + t0 + t];
          f[t] = load_feat4(a.feats4, a.feat_half, (int64_t)(id[t] >= 0 ? id[t] : 0) * 8 + q);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (id[t] >= 0) {
            const float wn = L.w[sl * PNR_MAX_K + t0 + t];
            acc.x = acc.x + wn * f[t].x;
            acc.y = acc.y + wn * f[t].y;
            acc.z = acc.z + wn * f[t].z;
            acc.w = acc.w + wn * f[t].w;
          }
        }
      }
      nt_store(reinterpret_cast<float4*>(a.c) + (int64_t)rw * 8 + q, acc);  // 8 lanes: one 128-B row
    }
#endif
    __syncthreads();  // the next chunk rewrites the feature lists
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
  // Feature gradients in exact fixed point (order-independent, hence deterministic): every term
  // w dL/dc becomes an int64 multiple of 2^-s, s from max |dL/dc| over the rows and the guard bits
  // (a sum of <= 2^guard terms never overflows); k_gather_bwd_fin converts once into g_feats
  long long* facc;       // [M][32] int64 accumulators: only the rows a work-list row names are used
  uint32_t* touched;     // [M bits] rows of facc in use: set (and the row zeroed) by k_gather_bwd_gmax
  uint32_t* gmax;        // bits of max |dL/dc| over the work list's rows (NaN / inf propagate)
  unsigned long long* n_flush;  // int64 atomic instructions (256 B each) issued, for the roofline
  int guard;
  int run;               // work items per half-wave run (32, fewer for small launches)
};

// rows with a neighbour (idx[row][0] >= 0: neighbours are stored nearest first) -> work list
__global__ __launch_bounds__(256) void k_gather_bwd_probe(GatherBwdArgs a) {
  const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const bool has = p < a.P && a.idx[p * a.k] >= 0;
  wl_append(a.wl, has, make_float4(0.f, 0.f, 0.f, __int_as_float((int)p)));
}

// max |dL/dc| over the rows of the work list (half a wave per row; the integer max of the bits of
// |x| is the float max, and a NaN row wins it: its bits are the largest)
__global__ __launch_bounds__(256) void k_gather_bwd_gmax(GatherBwdArgs a) {
  const int ch = threadIdx.x & 31, half = threadIdx.x >> 5;
  const int64_t nchunk = (a.wl.cap + 255) / 256;
  uint32_t m = 0u;
  for (int64_t task = blockIdx.x; task < kLists * nchunk; task += gridDim.x) {
    const int rl = (int)(task % kLists);
    const int64_t j0 = task / kLists * 256;
    const int64_t n_work = (int64_t)a.wl.cnt[rl * 32];
    if (j0 >= n_work) continue;
    const int64_t jn = n_work - j0 < 256 ? n_work - j0 : 256;
#pragma unroll 4
    for (int64_t t = half; t < jn; t += 8) {
      const int64_t p = __float_as_int(a.wl.items[rl * a.wl.cap + j0 + t].w);
      const uint32_t b = __float_as_uint(a.g_c[p * 32 + ch]) & 0x7FFFFFFFu;
      m = m > b ? m : b;
      // the row's neighbours: the first lane to name a feature row zeroes its accumulators (the
      // accumulating launch runs after this one, so no add can precede the zero fill)
      const int id = a.touched && ch < a.k ? a.idx[p * a.k + ch] : -1;
      if (id >= 0) {
        const uint32_t bit = 1u << (id & 31);
        if (!(atomicOr(a.touched + (id >> 5), bit) & bit)) {
          longlong2* row = reinterpret_cast<longlong2*>(a.facc + (int64_t)id * 32);
#pragma unroll
          for (int e = 0; e < 16; ++e) row[e] = make_longlong2(0, 0);
        }
      }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t v = (uint32_t)__shfl_xor((int)m, o);
    m = m > v ? m : v;
  }
  if ((threadIdx.x & 63) == 0 && m != 0u) atomicMax(a.gmax, m);
}

// 2^s of the fixed-point feature gradients: |term| <= max |dL/dc| < 2^e, so |term| 2^s < 2^(62 - guard)
__device__ __forceinline__ int fx_shift(uint32_t gmax_bits, int guard) {
  if (gmax_bits == 0u || gmax_bits >= 0x7F800000u) return 0;  // all zero, or non-finite (k_gather_bwd_fin)
  int e;
  (void)frexpf(__uint_as_float(gmax_bits), &e);
  return 62 - guard - e;
}
__device__ __forceinline__ long long fx_term(float x, int s) {
  return (long long)rintf(ldexpf(x, s));  // exact power-of-two scale, one rounding to an integer
}

// Half a wave per row: lane c owns channel c, so the feature-gradient atomics of one neighbour
// are ONE instruction per two rows, each row 256 contiguous bytes of int64 (4 full 64-B requests).
template <int SRC, int KER>
__global__ __launch_bounds__(256) void k_gather_bwd(GatherBwdArgs a) {
  PNR_FP_STRICT
  const int ch = threadIdx.x & 31, half = threadIdx.x >> 5;  // 8 half-waves per block
  const int R = a.run, per = 8 * R;  // items per half-wave run / per block task
  const int64_t nchunk = (a.wl.cap + per - 1) / per;
  const int fs = a.g_feats ? fx_shift(*a.gmax, a.guard) : 0;
  unsigned long long* facc = reinterpret_cast<unsigned long long*>(a.facc);
  uint32_t nfl = 0;  // flushes of this half-wave (uniform over it)
  for (int64_t task = blockIdx.x; task < kLists * nchunk; task += gridDim.x) {
    const int rl = (int)(task % kLists);
    const int64_t j0 = task / kLists * per;
    const int64_t n_work = (int64_t)a.wl.cnt[rl * 32];
    if (j0 >= n_work) continue;  // uniform over the block
    const int64_t jn = n_work - j0 < per ? n_work - j0 : per;
    // half-wave `half` takes R consecutive items: rows of one ray, whose neighbour lists overlap.
    // A neighbour shared with the previous row carries its partial sum forward instead of being
    // flushed: the atomic goes out when it leaves the list (or at the end of the run).  Integer
    // sums: the result does not depend on which rows share a run, nor on the atomics' order.
    int pid[PNR_MAX_K];
    long long pacc[PNR_MAX_K];
#pragma unroll
    for (int kk = 0; kk < PNR_MAX_K; ++kk) {
      pid[kk] = -1;
      pacc[kk] = 0;
    }
    const int64_t te = (int64_t)R * half + R < jn ? (int64_t)R * half + R : jn;
#pragma unroll 1
    for (int64_t t = (int64_t)R * half; t < te; ++t) {  // uniform over each half-wave
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
        long long cur[PNR_MAX_K];
#pragma unroll
        for (int kk = 0; kk < PNR_MAX_K; ++kk) cur[kk] = id[kk] >= 0 ? fx_term(wn[kk] * g, fs) : 0;
#pragma unroll
        for (int j = 0; j < PNR_MAX_K; ++j) {  // ids within a row are distinct: at most one match
          bool kept = false;
#pragma unroll
          for (int kk = 0; kk < PNR_MAX_K; ++kk) {
            const bool mt = pid[j] >= 0 && id[kk] == pid[j];
            cur[kk] += mt ? pacc[j] : 0;
            kept = kept || mt;
          }
          if (pid[j] >= 0 && !kept) {
            atomicAdd(facc + (int64_t)pid[j] * 32 + ch, (unsigned long long)pacc[j]);
            ++nfl;
          }
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
        if (pid[j] >= 0) {
          atomicAdd(facc + (int64_t)pid[j] * 32 + ch, (unsigned long long)pacc[j]);
          ++nfl;
        }
    }
  }
  if (a.g_feats && a.n_flush) {  // one count per half-wave (lane 0 of each half), one atomic per wave
    uint32_t n = ch == 0 ? nfl : 0u;
    n += (uint32_t)__shfl_xor((int)n, 32);
    if ((threadIdx.x & 63) == 0 && n) atomicAdd(a.n_flush, (unsigned long long)n);
  }
}

// g_feats += facc 2^-s (4 values per thread) on the rows some sample named (the others received no
// term: left as they are, their accumulators never zeroed); a non-finite max |dL/dc| makes the
// elements of those rows NaN
__global__ __launch_bounds__(256) void k_gather_bwd_fin(const long long* __restrict__ facc, float* __restrict__ g,
                                                       int64_t n, const uint32_t* __restrict__ gmax, int guard,
                                                       const uint32_t* __restrict__ touched) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  const int64_t row = i / 32;
  if (touched && !((touched[row >> 5] >> (row & 31)) & 1u)) return;
  const uint32_t gb = *gmax;
  const int s = fx_shift(gb, guard);
  const bool bad = gb >= 0x7F800000u;
  // g may be a view at any float offset of a flat gradient buffer: 16-B accesses only when aligned
  if (i + 4 <= n && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
    const longlong2 v0 = *reinterpret_cast<const longlong2*>(facc + i);
    const longlong2 v1 = *reinterpret_cast<const longlong2*>(facc + i + 2);
    float4 o = *reinterpret_cast<float4*>(g + i);
    o.x += bad ? __int_as_float(0x7FC00000) : (float)ldexp((double)v0.x, -s);
    o.y += bad ? __int_as_float(0x7FC00000) : (float)ldexp((double)v0.y, -s);
    o.z += bad ? __int_as_float(0x7FC00000) : (float)ldexp((double)v1.x, -s);
    o.w += bad ? __int_as_float(0x7FC00000) : (float)ldexp((double)v1.y, -s);
    *reinterpret_cast<float4*>(g + i) = o;
  } else {
    const int64_t e = i + 4 < n ? i + 4 : n;
    for (int64_t j = i; j < e; ++j) g[j] += bad ? __int_as_float(0x7FC00000) : (float)ldexp((double)facc[j], -s);
  }
}

// Up to four zero fills in one launch (the counters and accumulators a gather / gather backward
// starts from): each hipMemsetAsync is a launch of its own, ~5 us apiece in the Mapper's captured
// iteration at its real batch sizes.  Regions are 4-B aligned; 16-B stores where aligned.
struct ZeroRegions {
  char* p[4];
  int64_t bytes[4];
  int n;
};
__global__ __launch_bounds__(256) void k_zero_regions(ZeroRegions z) {
  const int64_t tid = (int64_t)blockIdx.x * 256 + threadIdx.x, nth = (int64_t)gridDim.x * 256;
  for (int r = 0; r < z.n; ++r) {
    char* p = z.p[r];
    const int64_t nb = z.bytes[r];
    const int64_t head = ((16 - ((uintptr_t)p & 15)) & 15) < nb ? ((16 - ((uintptr_t)p & 15)) & 15) : nb;
    for (int64_t i = tid * 4; i < head; i += nth * 4) *reinterpret_cast<uint32_t*>(p + i) = 0u;
    const int64_t n16 = (nb - head) / 16;
    uint4* q = reinterpret_cast<uint4*>(p + head);
    for (int64_t i = tid; i < n16; i += nth) q[i] = make_uint4(0u, 0u, 0u, 0u);
    for (int64_t i = head + n16 * 16 + tid * 4; i < nb; i += nth * 4) *reinterpret_cast<uint32_t*>(p + i) = 0u;
  }
}
static int zero_regions(const ZeroRegions& z, hipStream_t st) {
  int64_t total = 0;
  for (int r = 0; r < z.n; ++r) total += z.bytes[r];
  if (total <= 0) return PNR_OK;
  const int64_t blocks = (total / 16 + 255) / 256;
  hipLaunchKernelGGL(k_zero_regions, dim3((unsigned)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048)), dim3(256), 0,
                     st, z);
  return hip_status(hipGetLastError());
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
    case kPtsX4: hipLaunchKernelGGL((k_gather_probe<kPtsX4>), grid, dim3(256), 0, st, a); break;
    default: hipLaunchKernelGGL((k_gather_probe<kRaysZ32>), grid, dim3(256), 0, st, a); break;
  }
}

size_t gather_workspace_bytes(int64_t P) {
  size_t b = 0;
  group_view(nullptr, P > 0 ? P : 0, &b);
  return b;
}

// backward workspace: the work list of rows with a neighbour | 256-B control block (max |dL/dc| bits
// at 0, issued atomic instructions at 8) | with feature gradients, the int64 accumulators [M][32]
struct GatherBwdView {
  WorkList wl;
  char* ctl;
  uint32_t* gmax;
  unsigned long long* n_flush;
  long long* facc;
  uint32_t* touched;
};
static GatherBwdView gather_bwd_view(void* ws, int64_t P, int64_t M, bool feats, size_t* bytes = nullptr) {
  GatherBwdView v{};
  char* b = static_cast<char*>(ws);
  size_t off = a256(wl_bytes(P > 0 ? P : 0));
  if (b) v.wl = wl_view(b, P > 0 ? P : 0);
  v.ctl = b ? b + off : nullptr;
  v.gmax = reinterpret_cast<uint32_t*>(v.ctl);
  v.n_flush = reinterpret_cast<unsigned long long*>(v.ctl ? v.ctl + 8 : nullptr);
  off += 256;
  if (feats) {
    v.facc = reinterpret_cast<long long*>(b ? b + off : nullptr);
    off += a256((size_t)(M > 0 ? M : 0) * kCDim * 8);
    v.touched = reinterpret_cast<uint32_t*>(b ? b + off : nullptr);
    off += a256((size_t)((M > 0 ? M : 0) + 31) / 32 * 4);
  }
  if (bytes) *bytes = off;
  return v;
}
size_t gather_bwd_workspace_bytes(int64_t P, int64_t M, bool feats) {
  size_t b = 0;
  gather_bwd_view(nullptr, P, M, feats, &b);
  return b;
}

int launch_gather(const pnr_points& pts, const PointSrc& src, int mode, int64_t P, int64_t rows, float* c,
                  int32_t* idx, float* w, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!points_ok(pts) || mode < kPtsF64 || mode > kPtsX4 || P < 0 || rows < P || P >= (1ll << 31)) return PNR_E_ARG;
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
  GroupView gv = group_view(ws, P, nullptr);
  a.wl = gv.wl;
  a.gcnt = gv.gcnt;
  a.gstart = gv.gstart;
  a.grouped = gv.grouped;
  a.gmask = (uint32_t)((1ll << gv.gbits) - 1);
  const int64_t G = 1ll << gv.gbits;
  {
    ZeroRegions z{};
    z.p[0] = reinterpret_cast<char*>(a.wl.cnt);
    z.bytes[0] = kLists * 32 * 4;
    z.p[1] = reinterpret_cast<char*>(a.gcnt);
    z.bytes[1] = G * 4;
    z.n = 2;
    if (int rc = zero_regions(z, st)) return rc;
  }
  TimingScope ts(kTimeGather, P, st);
  gather_probe(mode, dim3((unsigned)((rows + 255) / 256)), st, a);
  int rc = scan_exclusive(a.gcnt, gv.gstart, G, gv.scratch, st);
  if (rc) return rc;
  hipLaunchKernelGGL(k_group_scatter, dim3((unsigned)(kLists * ((a.wl.cap + 255) / 256))), dim3(256), 0, st, a);
  // Items per chunk: a chunk's segments (probe blocks) run one after another in its wave, each a few
  // dependent round trips.  At the Mapper's real batches (1,000-5,000 rays) the items of a chunk rarely
  // share a block, so 64-item chunks left ~200 waves each walking up to 64 segments in series
  // (config C3: 209 + 320 us per iteration); smaller chunks spread the segments over the machine's
  // ~5,000 wave slots.  The S-map batches (> 2.6M samples: 80 per block) keep 64.
  // (64 items from 2.6M samples up: the S-map batches; below, candidate-parallel chunks of 8 or 4)
  a.chunk = P >= 64 * 5 * 1024 * 8 ? 64 : (P >= 160 * 1024 ? 8 : 4);
  const int64_t tasks = (P + a.chunk - 1) / a.chunk;  // upper bound on the chunks (the kernel reads the real count)
  const bool par = a.chunk <= 8;  // candidate-parallel scan for small chunks
  auto kern = pts.mode == PNR_GATHER_IDW
                  ? (a.feat_half ? (par ? k_gather_search<PNR_GATHER_IDW, true, true>
                                        : k_gather_search<PNR_GATHER_IDW, true, false>)
                                 : (par ? k_gather_search<PNR_GATHER_IDW, false, true>
                                        : k_gather_search<PNR_GATHER_IDW, false, false>))
                  : (a.feat_half ? (par ? k_gather_search<PNR_GATHER_TRILINEAR, true, true>
                                        : k_gather_search<PNR_GATHER_TRILINEAR, true, false>)
                                 : (par ? k_gather_search<PNR_GATHER_TRILINEAR, false, true>
                                        : k_gather_search<PNR_GATHER_TRILINEAR, false, false>));
  hipLaunchKernelGGL(kern, dim3(resident_grid(kern, 64, tasks)), dim3(64), 0, st, a);
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
    case kPtsX4: gather_bwd_launch<kPtsX4, KER>(tasks, st, a); break;
    default: gather_bwd_launch<kRaysZ32, KER>(tasks, st, a); break;
  }
}

int launch_gather_bwd(const pnr_points& pts, const PointSrc* src, int mode, const float4* xP, int64_t P,
                      const int32_t* idx, const float* w, const float* c, const float* g_c, float* g_p,
                      bool gp_accum, void* ws, size_t ws_bytes, hipStream_t st) {
  if (!points_ok(pts) || P < 0 || (!src && !xP) || mode < kPtsF64 || mode > kPtsX4 || P >= (1ll << 31))
    return PNR_E_ARG;
  if (P == 0 || (!pts.g_feats && !g_p)) return PNR_OK;
  if (!idx || !w || !g_c || (g_p && !c)) return PNR_E_ARG;
  const bool feats = pts.g_feats != nullptr;
  if (!ws || ws_bytes < gather_bwd_workspace_bytes(P, pts.n_points, feats)) return PNR_E_WORKSPACE;
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
  GatherBwdView v = gather_bwd_view(ws, P, pts.n_points, feats);
  a.wl = v.wl;
  a.facc = v.facc;
  a.touched = P * (int64_t)pts.k < 4 * pts.n_points ? v.touched : nullptr;  // sparse: touched rows only
  a.gmax = v.gmax;
  a.n_flush = v.n_flush;
  // a sum of at most P terms per element (the ids of a row are distinct): 2^guard > P
  int guard = 1;
  while (guard < 40 && (1ll << guard) <= P) ++guard;
  a.guard = guard;
  // Items per half-wave run: each run's rows are serial (every row a few dependent loads and its
  // atomics); the S-map batches keep 32 (long runs carry shared neighbours between a ray's rows), the
  // Mapper's real batches shorter runs so the rows spread over the machine (config C3: 92 us per
  // backward with 32-row runs over ~600 half-waves)
  a.run = 32;
  while (a.run > 2 && P / a.run < 2 * 5 * 1024 * 8) a.run >>= 1;
  {
    ZeroRegions z{};
    z.p[z.n] = reinterpret_cast<char*>(a.wl.cnt);
    z.bytes[z.n++] = kLists * 32 * 4;
    if (feats) {
      z.p[z.n] = v.ctl;
      z.bytes[z.n++] = 256;
      // Sparse calls (the Mapper's real batches: a few neighbour slots per point of the cloud) zero
      // and convert only the rows their samples name (the touched map, set by the max pass); dense
      // ones (S-map: 15M neighbour slots over 182k points, where marking took 1.1 ms of same-word
      // atomics) zero every accumulator and convert every row
      if (!a.touched) {
        z.p[z.n] = reinterpret_cast<char*>(v.facc);
        z.bytes[z.n++] = pts.n_points * kCDim * 8;
      } else {
        z.p[z.n] = reinterpret_cast<char*>(v.touched);
        z.bytes[z.n++] = (pts.n_points + 31) / 32 * 4;
      }
    }
    if (g_p && !gp_accum) {
      z.p[z.n] = reinterpret_cast<char*>(g_p);
      z.bytes[z.n++] = P * 12;
    }
    if (int rc = zero_regions(z, st)) return rc;
  }
  TimingScope ts(kTimeGatherBwd, P, st);
  hipLaunchKernelGGL(k_gather_bwd_probe, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, a);
  const int64_t tasks = kLists * ((a.wl.cap + 255) / 256);
  if (feats) hipLaunchKernelGGL(k_gather_bwd_gmax, dim3(resident_grid(k_gather_bwd_gmax, 256, tasks)), dim3(256), 0, st, a);
  const int64_t rtasks = kLists * ((a.wl.cap + 8 * a.run - 1) / (8 * a.run));
  if (pts.mode == PNR_GATHER_IDW) gather_bwd_mode<PNR_GATHER_IDW>(mode, rtasks, st, a);
  else gather_bwd_mode<PNR_GATHER_TRILINEAR>(mode, rtasks, st, a);
  if (feats && pts.n_points > 0) {
    const int64_t n = pts.n_points * kCDim;
    hipLaunchKernelGGL(k_gather_bwd_fin, dim3((unsigned)((n / 4 + 255) / 256 + 1)), dim3(256), 0, st, v.facc, pts.g_feats,
                       n, v.gmax, guard, a.touched);
  }
  return hip_status(hipGetLastError());
}

int gather_bwd_atomics(const void* ws, int64_t P, int64_t M, unsigned long long* n, hipStream_t st) {
  GatherBwdView v = gather_bwd_view(const_cast<void*>(ws), P, M, true);
  if (hipMemcpyAsync(n, v.n_flush, 8, hipMemcpyDeviceToHost, st) != hipSuccess) return (int)hipGetLastError();
  return hip_status(hipStreamSynchronize(st));
}

}  // namespace pnr
