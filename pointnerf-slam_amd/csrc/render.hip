// render.hip -- ray-level kernels of the renderer (thread per ray; cheap next to the MLP).
//
//   k_gt_max          max(1.2 * gt_depth) of the batch              Renderer.py:112
//   k_coarse_z        near/far + stratified depths (float64)         Renderer.py:90-116, 157-171
//   k_pdf             coarse compositing weights + inverse-CDF       common.py:204-245, 19-63;
//                     importance depths (float64)                    Renderer.py:186-190
//   k_fine            sort(cat(z, z_samples)) + final compositing    Renderer.py:191-201
//   k_fine_bwd        compositing backward -> dL/draw per point       (autograd of common.py:224-244)
//   k_ray_grads       dL/drays_o, dL/drays_d (tracking)              Renderer.py:177-178, common.py:230
//   k_reg_z           regulation depths (float32, jittered)          Renderer.py:280-294
//   k_get_rays        full-frame / per-pixel rays                    common.py:74-89, 248-266
//   k_window_rays     a mapping iteration's window pixel batch       Mapper.py:560-606, common.py:74-134
//   k_window_sample   the same batch drawn on the device + t_rand + the far clamp (one launch)
//   k_adam            torch.optim.Adam step                          Mapper.py:498-502, 657-662
//
// Arithmetic follows torch's CPU semantics where it is observable: python scalars are applied
// in float32, cumprod / cumsum accumulate in float64 and round per element, x@B for K=3 and
// |d| are fma chains, and no floating-point contraction is allowed elsewhere (fp contract off).
#include <math.h>

#include <algorithm>

#include "pnr_internal.h"

#pragma clang fp contract(off)

namespace pnr {

__device__ __forceinline__ double max_nan(double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); }
__device__ __forceinline__ double min_nan(double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); }
__device__ __forceinline__ float relu(float x) { return x > 0.f ? x : 0.f; }

__device__ __forceinline__ float ray_norm(const float* d) {
  return sqrtf(__builtin_fmaf(d[2], d[2], __builtin_fmaf(d[1], d[1], d[0] * d[0])));
}

// ---------------------------------------------------------------------------------------------
// batch max of 1.2 gt in two launches (one up to 4,096 rays): kGtParts blocks write partial maxima
// to out[1..], then one block reduces them into out[0] (the workspace slot holds 64 floats).  NaN
// propagates (torch.max).
constexpr int kGtParts = 63;
__device__ __forceinline__ float max_nanf(float m, float v) { return (v > m || v != v) ? v : m; }
__device__ __forceinline__ float block_max_256(float m, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) m = max_nanf(m, __shfl_xor(m, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  return max_nanf(max_nanf(red[0], red[1]), max_nanf(red[2], red[3]));
}
__global__ __launch_bounds__(256) void k_gt_max_part(const float* __restrict__ gt, int64_t n, float* __restrict__ out) {
  __shared__ float red[4];
  float m = -INFINITY;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    m = max_nanf(m, gt[i] * 1.2f);
  m = block_max_256(m, red);
  if (threadIdx.x == 0) out[gridDim.x == 1 ? 0 : 1 + blockIdx.x] = m;  // one part: the result itself
}
__global__ __launch_bounds__(256) void k_gt_max(int parts, float* __restrict__ out) {
  __shared__ float red[4];
  const float m = block_max_256((int)threadIdx.x < parts ? out[1 + threadIdx.x] : -INFINITY, red);
  if (threadIdx.x == 0) out[0] = m;
}

// near/far and the stratified z of the first pass.  z: (N, S) float64.
__global__ void k_coarse_z(pnr_render_params prm, const float* __restrict__ ro, const float* __restrict__ rd,
                           const float* __restrict__ gt, const float* __restrict__ gmax, int64_t n_rays,
                           double* __restrict__ z, double* __restrict__ far_out) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_rays) return;
  double fb = 0.0;
  for (int a = 0; a < 3; ++a) {
    const double o = (double)ro[n * 3 + a], d = (double)rd[n * 3 + a];
    const double t0 = (prm.bound[2 * a] - o) / d;
    const double t1 = (prm.bound[2 * a + 1] - o) / d;
    const double mx = max_nan(t0, t1);
    fb = a == 0 ? mx : min_nan(fb, mx);
  }
  fb = fb + 0.01;
  double far = fb;
  float nearf = 0.01f;
  if (gt != nullptr) {
    const double hi = prm.far_mode == 1 ? prm.far_clamp : (double)(*gmax);
    far = fb != fb ? fb : (fb < 0.0 ? 0.0 : fb);  // clamp(min=0)
    far = far != far ? far : (far > hi ? hi : far);
    nearf = gt[n] * 0.01f;
  }
  if (far_out) far_out[n] = far;
  const int S = prm.n_samples;
  for (int s = 0; s < S; ++s) {
    const float t = prm.t_vals[s];
    double zz;
    if (!prm.lindisp) {
      zz = (double)(nearf * (1.f - t)) + far * (double)t;
    } else {
      const float inv_near = gt != nullptr ? 1.f / nearf : 100.f;
      zz = 1.0 / ((double)(inv_near * (1.f - t)) + (1.0 / far) * (double)t);
    }
    z[n * S + s] = zz;
  }
}

// Map pass (pnr_map_fwd): the rows of MLP launch A, one thread per row, points and bound tests in
// the reference's dtypes (the arithmetic of k_reg_z + load_point<kRaysZ32> and of k_coarse_z +
// load_point<kRaysZ64>, expression for expression):
//   rows [0, n S)        regulation samples (Renderer.py:280-298): float32 z in [0, 0.85 gt] jittered,
//                        float32 points and bound test;
//   rows [pr, pr + n S)  the render's coarse samples (Renderer.py:90-116, 157-182): near/far with the
//                        batch far clamp, float64 stratified z (also written to zc for k_pdf / k_fine),
//                        float64 points and bound test;
//   other rows < rows    padding: (0, 0, 0, outside).
// x4 row = (x, y, z, inside ? 1 : 0) float32: the MLP input (kPtsX4) and its saved copy at once.
__global__ void k_map_pts(MapRowsArgs m, int64_t rows, float4* __restrict__ x4) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= rows) return;
  float x0, x1, x2;
  bool inside;
  map_row_point(m, e, true, x0, x1, x2, inside);
  x4[e] = make_float4(x0, x1, x2, inside ? 1.f : 0.f);
}

// ---------------------------------------------------------------------------------------------
// coarse weights -> sample_pdf -> z_samples (N, I) float64
// The ray kernels below run one thread per ray; at the Mapper's batch (1,000 rays: 16 waves) every
// one of them is latency-bound on its per-sample loads.  SS / II > 0 specialise them for the
// config's sample counts (32 + 12): the loops unroll, so a ray's loads are all in flight at once
// (with runtime counts they went out one sample at a time).  The arithmetic and its order are the
// same in both forms.
// Map pass extras (MapPts, null outside pnr_map_fwd): the importance samples' kPtsX4 rows (float64
// points and bound test, load_point<kRaysZ64>), the regulation rows' densities copied out of the MLP
// launch (Renderer.py:299-300: sigma = raw[..., -1]), and the importance segment's padding rows zeroed.
struct MapPts {
  const float* ro;
  float4* x4i;          // importance rows
  int64_t x4i_pad;      // padding rows after the n I importance rows
  const float4* rawr;   // regulation rows of launch A
  float* sigma;         // (n, S) regulation densities
};
template <int SS, int II>
__global__ __launch_bounds__(64) void k_pdf(pnr_render_params prm, const float* __restrict__ rd,
                                            const double* __restrict__ zc, const float4* __restrict__ rawc,
                                            int64_t n_rays, double* __restrict__ zi, MapPts mp) {
  __shared__ float wl[PNR_MAX_SAMPLES][64];
  __shared__ float cdf[PNR_MAX_SAMPLES][64];
  const int tid = threadIdx.x;
  const int64_t ray0 = (int64_t)blockIdx.x * 64, n = ray0 + tid;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance;
  if (mp.x4i) {  // the importance launch's padding rows: outside points at x = 0
    for (int64_t i = n; i < mp.x4i_pad; i += (int64_t)gridDim.x * 64)
      mp.x4i[n_rays * I + i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (mp.sigma) {  // the regulation densities of the block's rays: coalesced copy
    const int nr = (int)(n_rays - ray0 < 64 ? n_rays - ray0 : 64);
    for (int e = tid; e < nr * S; e += 64) mp.sigma[ray0 * S + e] = mp.rawr[ray0 * S + e].w;
  }
  if (n >= n_rays) return;
  const double* z = zc + n * S;
  const float4* raw = rawc + n * S;
  auto zq = [&](int q) -> double { return z[q]; };
  auto sq = [&](int q) -> float { return raw[q].w; };
  const float nrm = ray_norm(rd + n * 3);
  double T = 1.0;
#pragma unroll
  for (int q = 0; q < S; ++q) {
    const float dz = q < S - 1 ? (float)(zq(q + 1) - zq(q)) : 1e10f;
    const float delta = dz * nrm;
    const float a = 1.f - expf(-relu(sq(q)) * delta);
    wl[q][tid] = a * (float)T;
    T *= (double)(1.f - a + 1e-10f);
  }
  // sample_pdf(bins = mid(z) (S-1), weights[1:-1] (S-2))
  const int M = S - 2;
  float sum = 0.f;
  for (int m = 0; m < M; ++m) sum += wl[m + 1][tid] + 1e-5f;
  double acc = 0.0;
  cdf[0][tid] = 0.f;
  for (int m = 0; m < M; ++m) {
    acc += (double)((wl[m + 1][tid] + 1e-5f) / sum);
    cdf[m + 1][tid] = (float)acc;
  }
#pragma unroll 4
  for (int k = 0; k < I; ++k) {
    const float u = prm.u_vals[k];
    // searchsorted(cdf, u, right=True): first index with cdf > u (binary search over M+1 entries)
    int lo = 0, hi = M + 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cdf[mid][tid] <= u) lo = mid + 1; else hi = mid;
    }
    const int below = lo - 1 > 0 ? lo - 1 : 0;
    const int above = lo < M ? lo : M;
    const float c0 = cdf[below][tid], c1 = cdf[above][tid];
    float denom = c1 - c0;
    if (denom < 1e-5f) denom = 1.f;
    const float t = (u - c0) / denom;
    const double b0 = .5 * (zq(below + 1) + zq(below));
    const double b1 = .5 * (zq(above + 1) + zq(above));
    const double zz = b0 + (double)t * (b1 - b0);
    zi[n * I + k] = zz;
    if (mp.x4i) {  // load_point<kRaysZ64> of the importance sample
      const double q0 = (double)mp.ro[n * 3 + 0] + (double)rd[n * 3 + 0] * zz;
      const double q1 = (double)mp.ro[n * 3 + 1] + (double)rd[n * 3 + 1] * zz;
      const double q2 = (double)mp.ro[n * 3 + 2] + (double)rd[n * 3 + 2] * zz;
      const bool inside = (q0 < prm.bound[1]) && (q0 > prm.bound[0]) && (q1 < prm.bound[3]) && (q1 > prm.bound[2]) &&
                          (q2 < prm.bound[5]) && (q2 > prm.bound[4]);
      mp.x4i[n * I + k] = make_float4((float)q0, (float)q1, (float)q2, inside ? 1.f : 0.f);
    }
  }
}

// NaN-aware strict order used for torch.sort (NaN sorts last)
__device__ __forceinline__ bool lt_nan(double a, double b) { return (a < b) || (a == a && b != b); }
__device__ __forceinline__ bool eq_nan(double a, double b) { return (a == b) || (a != a && b != b); }

// Sort the S+I depths of ray n into ascending order; ord[q] = source index (< S: coarse).
// torch.sort's order here is the stable one (coarse before importance on ties, NaN last).  The
// coarse depths (near..far linspace) and the importance depths (inverse-cdf of increasing u) are
// each non-decreasing unless far < near or a value is NaN: then a stable merge gives exactly that
// order in O(S+I); otherwise the rank sort below does.
template <int SS, int II>
__device__ __forceinline__ void sort_ray(double (*zl)[64], int S, int I, uint8_t (*ord)[64], int tid) {
  if (SS > 0) S = SS;
  if (II > 0) I = II;
  const int M = S + I;
  // zl[m][tid]: the ray's depths in natural order (coarse 0..S-1, importance S..M-1), staged
  bool sorted = true;
  double prev = zl[0][tid];
  sorted = prev == prev;
#pragma unroll
  for (int m = 1; m < S; ++m) {
    const double v = zl[m][tid];
    sorted = sorted && prev <= v;  // false for NaN
    prev = v;
  }
  if (I > 0) {
    prev = zl[S][tid];
    sorted = sorted && prev == prev;
#pragma unroll
    for (int k = 1; k < I; ++k) {
      const double v = zl[S + k][tid];
      sorted = sorted && prev <= v;
      prev = v;
    }
  }
  if (sorted) {
    int i = 0, k = 0;
    for (int q = 0; q < M; ++q) {
      const bool coarse = k >= I || (i < S && zl[i][tid] <= zl[S + k][tid]);
      ord[q][tid] = (uint8_t)(coarse ? i : S + k);
      i += coarse ? 1 : 0;
      k += coarse ? 0 : 1;
    }
    return;
  }
  for (int i = 0; i < M; ++i) {
    const double v = zl[i][tid];
    int r = 0;
    for (int m = 0; m < M; ++m) {
      const double w = zl[m][tid];
      r += (lt_nan(w, v) || (eq_nan(w, v) && m < i)) ? 1 : 0;
    }
    ord[r][tid] = (uint8_t)i;
  }
}

// final pass: depth/var (float64), rgb (float32); saves the sort order for the backward
template <int SS, int II>
__global__ __launch_bounds__(64) void k_fine(pnr_render_params prm, const float* __restrict__ rd,
                                             const double* __restrict__ zc, const double* __restrict__ zi,
                                             const float4* __restrict__ rawc, const float4* __restrict__ rawi,
                                             int64_t n_rays, double* __restrict__ depth, double* __restrict__ var,
                                             float* __restrict__ rgb, uint8_t* __restrict__ ord_out) {
  __shared__ double zl[PNR_MAX_SAMPLES][64];
  __shared__ uint8_t ord[PNR_MAX_SAMPLES][64];
  __shared__ float wl[PNR_MAX_SAMPLES][64];
  const int tid = threadIdx.x;
  const int64_t n = (int64_t)blockIdx.x * 64 + tid;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance, M = S + I;
  if (n >= n_rays) return;
  // the ray's depths, natural order
#pragma unroll
  for (int m = 0; m < S; ++m) zl[m][tid] = zc[n * S + m];
#pragma unroll
  for (int k = 0; k < I; ++k) zl[S + k][tid] = zi[n * I + k];
  sort_ray<SS, II>(zl, S, I, ord, tid);
  const float nrm = ray_norm(rd + n * 3);
  double T = 1.0, D = 0.0;
  float r0 = 0.f, r1 = 0.f, r2 = 0.f;
#pragma unroll
  for (int q = 0; q < M; ++q) {
    const int s = ord[q][tid];
    const double zq = zl[s][tid];
    const float dz = q < M - 1 ? (float)(zl[ord[q + 1][tid]][tid] - zq) : 1e10f;
    const float4 c = s < S ? rawc[n * S + s] : rawi[n * I + (s - S)];
    const float a = 1.f - expf(-relu(c.w) * (dz * nrm));
    const float w = a * (float)T;
    T *= (double)(1.f - a + 1e-10f);
    wl[q][tid] = w;
    r0 += w * c.x; r1 += w * c.y; r2 += w * c.z;
    D += (double)w * zq;
  }
  double V = 0.0;
#pragma unroll
  for (int q = 0; q < M; ++q) {
    const double dd = zl[ord[q][tid]][tid] - D;
    V += (double)wl[q][tid] * dd * dd;
  }
  depth[n] = D;
  var[n] = V;
  rgb[n * 3 + 0] = r0; rgb[n * 3 + 1] = r1; rgb[n * 3 + 2] = r2;
  if (ord_out) {  // 4 bytes per store
    uint32_t* o = reinterpret_cast<uint32_t*>(ord_out + n * PNR_MAX_SAMPLES);
#pragma unroll
    for (int q = 0; q < M; q += 4) {
      uint32_t v = 0;
#pragma unroll
      for (int b = 0; b < 4; ++b) v |= (q + b < M ? (uint32_t)ord[q + b][tid] : 0u) << (8 * b);
      o[q >> 2] = v;
    }
  }
}

// Map pass extras of k_fine_bwd (pnr_map_bwd): the regulation rows and a third padding range
struct MapBwd {
  const float* g_sigma;   // (n, S) dL/dsigma of the regulation samples, or null
  const float4* insr;     // their kPtsX4 rows (inside flags)
  float4* gor;            // their dL/draw rows
  float4* pad2;
  int np2;
};

// Backward of the final compositing: writes dL/draw (float4) for every coarse and importance
// point, sigma channel zeroed where the point was outside the bound (Renderer.py:57 assigns
// the density, so no gradient reaches the MLP there); g_nrm[n] = dL/d|rays_d|.
template <int SS, int II>
__global__ __launch_bounds__(64) void k_fine_bwd(pnr_render_params prm, const float* __restrict__ rd,
                                                 const double* __restrict__ zc, const double* __restrict__ zi,
                                                 const float4* __restrict__ rawc, const float4* __restrict__ rawi,
                                                 const float4* __restrict__ insc, const float4* __restrict__ insi,
                                                 const uint8_t* __restrict__ ord_in, int64_t n_rays,
                                                 const double* __restrict__ g_depth, const double* __restrict__ g_var,
                                                 const float* __restrict__ g_rgb, float4* __restrict__ goc,
                                                 float4* __restrict__ goi, float* __restrict__ g_nrm,
                                                 float4* __restrict__ pad0, int np0, float4* __restrict__ pad1, int np1,
                                                 MapBwd mb) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int64_t n = (int64_t)blockIdx.x * 64 + tid;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance, M = S + I;
  // [M][64] per-ray columns: z (sorted), alpha and T; w = alpha * T and dz are recomputed from
  // them bit-for-bit, which keeps the LDS per block at 16 B per sample (3 blocks per CU at M = 44)
  double* zs = reinterpret_cast<double*>(smem);
  float* al = reinterpret_cast<float*>(zs + M * 64);
  float* Tl = al + M * 64;
  const int64_t ray0 = (int64_t)blockIdx.x * 64;
  {  // the padding rows of the MLP launches get dL/draw = 0 (the MLP backward reads every row)
    const int64_t gi = (int64_t)blockIdx.x * 64 + tid, gs = (int64_t)gridDim.x * 64;
    for (int64_t i = gi; i < np0; i += gs) pad0[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < np1; i += gs) pad1[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < mb.np2; i += gs) mb.pad2[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (mb.g_sigma) {  // map pass: the regulation rows' dL/draw (k_gout_sigma): sigma only, 0 outside the bound
    const int S0 = SS > 0 ? SS : prm.n_samples;
    const int nr = (int)(n_rays - ray0 < 64 ? n_rays - ray0 : 64);
    for (int e = tid; e < nr * S0; e += 64) {  // the block's rows, coalesced
      const int64_t r = ray0 * S0 + e;
      mb.gor[r] = make_float4(0.f, 0.f, 0.f, mb.insr[r].w != 0.f ? mb.g_sigma[r] : 0.f);
    }
  }
  if (n >= n_rays) return;
  const uint8_t* ord = ord_in + n * PNR_MAX_SAMPLES;
  // specialised: the ray's sort order in registers (16-B loads of the 64-B row), so the sample
  // loads below depend on no other load
  constexpr int kOw = SS > 0 ? (SS + II + 15) / 16 * 4 : 1;
  uint32_t ow[kOw];
  if constexpr (SS > 0) {
#pragma unroll
    for (int i = 0; i < kOw / 4; ++i) {
      const uint4 v = reinterpret_cast<const uint4*>(ord)[i];
      ow[4 * i] = v.x; ow[4 * i + 1] = v.y; ow[4 * i + 2] = v.z; ow[4 * i + 3] = v.w;
    }
  }
  auto ordq = [&](int q) -> int { return SS > 0 ? (int)((ow[q >> 2] >> (8 * (q & 3))) & 0xffu) : (int)ord[q]; };
  const float* dvec = rd + n * 3;
  const float nrm = ray_norm(dvec);
  auto zsrc = [&](int s) { return s < S ? zc[n * S + s] : zi[n * I + (s - S)]; };
  auto rsrc = [&](int s) { return s < S ? rawc[n * S + s] : rawi[n * I + (s - S)]; };
  double T = 1.0, D = 0.0;
#pragma unroll
  for (int q = 0; q < M; ++q) zs[q * 64 + tid] = zsrc(ordq(q));
#pragma unroll
  for (int q = 0; q < M; ++q) {
    const double zq = zs[q * 64 + tid];
    const float dz = q < M - 1 ? (float)(zs[(q + 1) * 64 + tid] - zq) : 1e10f;
    const float4 c = rsrc(ordq(q));
    const float a = 1.f - expf(-relu(c.w) * (dz * nrm));
    const float w = a * (float)T;
    Tl[q * 64 + tid] = (float)T;
    T *= (double)(1.f - a + 1e-10f);
    al[q * 64 + tid] = a;
    D += (double)w * zq;
  }
  const double gd = g_depth ? g_depth[n] : 0.0;
  const double gv = g_var ? g_var[n] : 0.0;
  const float gr0 = g_rgb ? g_rgb[n * 3 + 0] : 0.f;
  const float gr1 = g_rgb ? g_rgb[n * 3 + 1] : 0.f;
  const float gr2 = g_rgb ? g_rgb[n * 3 + 2] : 0.f;
  double sdev = 0.0;
#pragma unroll
  for (int q = 0; q < M; ++q) sdev += (double)(al[q * 64 + tid] * Tl[q * 64 + tid]) * (zs[q * 64 + tid] - D);
  const double gD = gd - 2.0 * gv * sdev;  // d var / d depth = -2 sum w (z - depth)
  float R = 0.f, gn = 0.f;
#pragma unroll
  for (int q = M - 1; q >= 0; --q) {
    const int s = ordq(q);
    const float4 c = rsrc(s);
    const double zq = zs[q * 64 + tid];
    const double dd = zq - D;
    const float a = al[q * 64 + tid];
    const float w = a * Tl[q * 64 + tid];
    const float gw = (gr0 * c.x + gr1 * c.y + gr2 * c.z) + (float)(gD * zq) + (float)(gv * dd * dd);
    const float ga = Tl[q * 64 + tid] * (gw - R);
    R = gw * a + (1.f - a + 1e-10f) * R;
    const float dz = q < M - 1 ? (float)(zs[(q + 1) * 64 + tid] - zq) : 1e10f;
    const float delta = dz * nrm;
    const float sr = relu(c.w);
    const float ex = expf(-sr * delta);
    float gs = c.w > 0.f ? ga * ex * delta : 0.f;
    const bool inside = s < S ? insc[n * S + s].w != 0.f : insi[n * I + (s - S)].w != 0.f;
    if (!inside) gs = 0.f;
    gn += (ga * ex * sr) * dz;
    const float4 go = make_float4(gr0 * w, gr1 * w, gr2 * w, gs);
    if (s < S) goc[n * S + s] = go; else goi[n * I + (s - S)] = go;
  }
  if (g_nrm) g_nrm[n] = gn;
}

// ---------------------------------------------------------------------------------------------
// Wave-per-ray forms of k_pdf / k_fine / k_fine_bwd for small batches (the Mapper's 1,000 rays: 16
// waves of the thread-per-ray kernels on 1,024 SIMDs, each a ~13 k-instruction serial chain).  Lane
// l of a 64-lane workgroup holds sample l: the per-sample work (loads, expf, alpha, the gradient
// terms, the stores) runs across the lanes, and only the accumulations the reference performs in
// order -- cumprod T (float64), the float / float64 sums, the backward recurrence R -- run as
// serial chains over v_readlane in the same order with the same roundings, so the results are the
// thread-per-ray kernels' bit for bit (tests/test_gpu_render_small.py).
__device__ __forceinline__ float rlf(float v, int l) {
  return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ double rld(double v, int l) {
  const uint64_t b = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)b, l);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(b >> 32), l);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}
// exclusive float64 cumprod of f over lanes 0..M-1 (T_0 = 1; torch.cumprod order): lane l gets T_l
__device__ __forceinline__ double excl_cumprod(double f, int M, int l) {
  double T = 1.0, Tl = 1.0;
  for (int q = 0; q < M; ++q) {
    Tl = l == q ? T : Tl;
    T *= rld(f, q);
  }
  return Tl;
}

template <int SS, int II>
__global__ __launch_bounds__(64) void k_pdf_w(pnr_render_params prm, const float* __restrict__ rd,
                                              const double* __restrict__ zc, const float4* __restrict__ rawc,
                                              int64_t n_rays, double* __restrict__ zi, MapPts mp) {
  __shared__ float cdf[PNR_MAX_SAMPLES];
  __shared__ double zs[PNR_MAX_SAMPLES + 1];
  const int l = threadIdx.x;
  const int64_t n = blockIdx.x;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance;
  if (mp.x4i) {
    for (int64_t i = n * 64 + l; i < mp.x4i_pad; i += (int64_t)gridDim.x * 64)
      mp.x4i[n_rays * I + i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (mp.sigma && l < S) mp.sigma[n * S + l] = mp.rawr[n * S + l].w;
  const int lq = l < S ? l : S - 1;  // clamped, unconditional loads (lanes >= S are never read)
  const double z = zc[n * S + lq];
  const float sg = rawc[n * S + lq].w;
  // the ray's own rows in the same round trip (after the barrier they would wait alone)
  const float nrm = ray_norm(rd + n * 3);
  double ro3[3] = {0.0, 0.0, 0.0}, rd3[3] = {0.0, 0.0, 0.0};
  if (mp.x4i) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      ro3[k] = (double)mp.ro[n * 3 + k];
      rd3[k] = (double)rd[n * 3 + k];
    }
  }
  zs[l] = z;
  __syncthreads();
  const float dz = l < S - 1 ? (float)(zs[l + 1] - z) : 1e10f;
  const float delta = dz * nrm;
  const float a = 1.f - expf(-relu(sg) * delta);
  const double Tl = excl_cumprod((double)(1.f - a + 1e-10f), S, l);
  const float w = a * (float)Tl;  // weights[q] (k_pdf's wl)
  // sample_pdf(bins = mid(z) (S-1), weights[1:-1] (S-2)): the float sum, then the float64 cdf
  const int M = S - 2;
  const float wt = w + 1e-5f;
  float sum = 0.f;
  for (int m = 0; m < M; ++m) sum += rlf(wt, m + 1);
  const float term = wt / sum;  // lane m + 1: term m
  double acc = 0.0;
  float c = 0.f;
  for (int m = 0; m < M; ++m) {
    acc += (double)rlf(term, m + 1);
    c = l == m + 1 ? (float)acc : c;
  }
  if (l <= M) cdf[l] = c;  // cdf[0] = 0
  float u = 0.f;  // u_vals[l] (uniform loads; no per-lane index into the kernel arguments)
  for (int k = 0; k < I; ++k) u = l == k ? prm.u_vals[k] : u;
  __syncthreads();
  if (l >= I) return;
  int lo = 0, hi = M + 1;  // searchsorted(cdf, u, right=True), as k_pdf
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (cdf[mid] <= u) lo = mid + 1; else hi = mid;
  }
  const int below = lo - 1 > 0 ? lo - 1 : 0;
  const int above = lo < M ? lo : M;
  const float c0 = cdf[below], c1 = cdf[above];
  float denom = c1 - c0;
  if (denom < 1e-5f) denom = 1.f;
  const float t = (u - c0) / denom;
  const double b0 = .5 * (zs[below + 1] + zs[below]);
  const double b1 = .5 * (zs[above + 1] + zs[above]);
  const double zz = b0 + (double)t * (b1 - b0);
  zi[n * I + l] = zz;
  if (mp.x4i) {
    const double q0 = ro3[0] + rd3[0] * zz;
    const double q1 = ro3[1] + rd3[1] * zz;
    const double q2 = ro3[2] + rd3[2] * zz;
    const bool inside = (q0 < prm.bound[1]) && (q0 > prm.bound[0]) && (q1 < prm.bound[3]) && (q1 > prm.bound[2]) &&
                        (q2 < prm.bound[5]) && (q2 > prm.bound[4]);
    mp.x4i[n * I + l] = make_float4((float)q0, (float)q1, (float)q2, inside ? 1.f : 0.f);
  }
}

template <int SS, int II>
__global__ __launch_bounds__(64) void k_fine_w(pnr_render_params prm, const float* __restrict__ rd,
                                               const double* __restrict__ zc, const double* __restrict__ zi,
                                               const float4* __restrict__ rawc, const float4* __restrict__ rawi,
                                               int64_t n_rays, double* __restrict__ depth, double* __restrict__ var,
                                               float* __restrict__ rgb, uint8_t* __restrict__ ord_out) {
  __shared__ double zn[PNR_MAX_SAMPLES];
  __shared__ uint8_t os[PNR_MAX_SAMPLES + 4];
  const int l = threadIdx.x;
  const int64_t n = blockIdx.x;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance, M = S + I;
  const int lq = l < M ? l : M - 1;  // clamped, unconditional loads (lanes >= M are never ranked)
  const double zl = *(lq < S ? zc + n * S + lq : zi + n * I + (lq - S));
  zn[l] = zl;
  os[l] = 0;
  if (l < 4) os[64 + l] = 0;
  __syncthreads();
  if (l < M) {  // stable rank (torch.sort, NaN last): sort_ray's order for any input
    int r = 0;
    for (int m = 0; m < M; ++m) {
      const double v = zn[m];
      r += (lt_nan(v, zl) || (eq_nan(v, zl) && m < l)) ? 1 : 0;
    }
    os[r] = (uint8_t)l;
  }
  __syncthreads();
  const int s = os[l];
  const double zq = zn[s];
  const double znx = l + 1 < M ? zn[os[l + 1]] : 0.0;
  const float4 c = *(s < S ? rawc + n * S + s : rawi + n * I + (s - S));  // lanes >= M: s = 0, never read
  const float nrm = ray_norm(rd + n * 3);
  const float dz = l < M - 1 ? (float)(znx - zq) : 1e10f;
  const float a = 1.f - expf(-relu(c.w) * (dz * nrm));
  const double Tl = excl_cumprod((double)(1.f - a + 1e-10f), M, l);
  const float w = a * (float)Tl;
  const float p0 = w * c.x, p1 = w * c.y, p2 = w * c.z;
  const double pD = (double)w * zq;
  float r0 = 0.f, r1 = 0.f, r2 = 0.f;
  double D = 0.0;
  for (int q = 0; q < M; ++q) {
    r0 += rlf(p0, q); r1 += rlf(p1, q); r2 += rlf(p2, q);
    D += rld(pD, q);
  }
  const double dd = zq - D;
  const double pV = (double)w * dd * dd;
  double V = 0.0;
  for (int q = 0; q < M; ++q) V += rld(pV, q);
  if (l == 0) {
    depth[n] = D;
    var[n] = V;
    rgb[n * 3 + 0] = r0; rgb[n * 3 + 1] = r1; rgb[n * 3 + 2] = r2;
  }
  if (ord_out && (l & 3) == 0 && l < M) {  // 4 bytes per store, zero past M (as k_fine)
    uint32_t v = 0;
#pragma unroll
    for (int b = 0; b < 4; ++b) v |= (l + b < M ? (uint32_t)os[l + b] : 0u) << (8 * b);
    reinterpret_cast<uint32_t*>(ord_out + n * PNR_MAX_SAMPLES)[l >> 2] = v;
  }
}

template <int SS, int II>
__global__ __launch_bounds__(64) void k_fine_bwd_w(pnr_render_params prm, const float* __restrict__ rd,
                                                   const double* __restrict__ zc, const double* __restrict__ zi,
                                                   const float4* __restrict__ rawc, const float4* __restrict__ rawi,
                                                   const float4* __restrict__ insc, const float4* __restrict__ insi,
                                                   const uint8_t* __restrict__ ord_in, int64_t n_rays,
                                                   const double* __restrict__ g_depth, const double* __restrict__ g_var,
                                                   const float* __restrict__ g_rgb, float4* __restrict__ goc,
                                                   float4* __restrict__ goi, float* __restrict__ g_nrm,
                                                   float4* __restrict__ pad0, int np0, float4* __restrict__ pad1,
                                                   int np1, MapBwd mb) {
  const int l = threadIdx.x;
  const int64_t n = blockIdx.x;
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance, M = S + I;
  {
    const int64_t gi = n * 64 + l, gs = (int64_t)gridDim.x * 64;
    for (int64_t i = gi; i < np0; i += gs) pad0[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < np1; i += gs) pad1[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < mb.np2; i += gs) mb.pad2[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  if (mb.g_sigma && l < S) {
    const int64_t r = n * S + l;
    mb.gor[r] = make_float4(0.f, 0.f, 0.f, mb.insr[r].w != 0.f ? mb.g_sigma[r] : 0.f);
  }
  const bool act = l < M;
  // clamped, unconditional loads (a predicated load waits on its own); lanes >= M are never read
  const int s = ord_in[n * PNR_MAX_SAMPLES + (act ? l : M - 1)];
  const double zq = *(s < S ? zc + n * S + s : zi + n * I + (s - S));
  const float4 c = *(s < S ? rawc + n * S + s : rawi + n * I + (s - S));
  const bool inside = act && (s < S ? insc + n * S + s : insi + n * I + (s - S))->w != 0.f;
  const double gd = g_depth ? g_depth[n] : 0.0;
  const double gv = g_var ? g_var[n] : 0.0;
  const float gr0 = g_rgb ? g_rgb[n * 3 + 0] : 0.f;
  const float gr1 = g_rgb ? g_rgb[n * 3 + 1] : 0.f;
  const float gr2 = g_rgb ? g_rgb[n * 3 + 2] : 0.f;
  const double znx = __shfl_down(zq, 1);
  const float nrm = ray_norm(rd + n * 3);
  const float dz = l < M - 1 ? (float)(znx - zq) : 1e10f;
  const float delta = dz * nrm;
  const float sr = relu(c.w);
  const float ex = expf(-sr * delta);
  const float a = 1.f - ex;
  const float Tf = (float)excl_cumprod((double)(1.f - a + 1e-10f), M, l);
  const float w = a * Tf;
  const double pD = (double)w * zq;
  double D = 0.0;
  for (int q = 0; q < M; ++q) D += rld(pD, q);
  const double pS = (double)(a * Tf) * (zq - D);
  double sdev = 0.0;
  for (int q = 0; q < M; ++q) sdev += rld(pS, q);
  const double gD = gd - 2.0 * gv * sdev;  // d var / d depth = -2 sum w (z - depth)
  const double dd = zq - D;
  const float gw = (gr0 * c.x + gr1 * c.y + gr2 * c.z) + (float)(gD * zq) + (float)(gv * dd * dd);
  // R before sample q (samples q+1..M-1 folded in, k_fine_bwd's reverse loop)
  const float pa = gw * a, g1 = 1.f - a + 1e-10f;
  float R = 0.f, Rl = 0.f;
  for (int q = M - 1; q >= 0; --q) {
    Rl = l == q ? R : Rl;
    R = rlf(pa, q) + rlf(g1, q) * R;
  }
  const float ga = Tf * (gw - Rl);
  float gs = c.w > 0.f ? ga * ex * delta : 0.f;
  if (!inside) gs = 0.f;
  const float pg = (ga * ex * sr) * dz;
  float gn = 0.f;
  for (int q = M - 1; q >= 0; --q) gn += rlf(pg, q);
  if (act) {
    const float4 go = make_float4(gr0 * w, gr1 * w, gr2 * w, gs);
    if (s < S) goc[n * S + s] = go; else goi[n * I + (s - S)] = go;
  }
  if (g_nrm && l == 0) g_nrm[n] = gn;
}

// dL/drays_o = sum_s dL/dx_s ; dL/drays_d = sum_s dL/dx_s * z_s + g_nrm * d/|d|
template <typename ZT>
__global__ void k_ray_grads(const float* __restrict__ rd, const ZT* __restrict__ za, int sa, const ZT* __restrict__ zb,
                            int sb, const float* __restrict__ gxa, const float* __restrict__ gxb,
                            const float* __restrict__ g_nrm, int64_t n_rays, float* __restrict__ g_o,
                            float* __restrict__ g_d) {
  const int64_t n = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (n >= n_rays) return;
  double o[3] = {0, 0, 0}, d[3] = {0, 0, 0};
  for (int s = 0; s < sa; ++s)
    for (int c = 0; c < 3; ++c) {
      const double g = gxa[(n * sa + s) * 3 + c];
      o[c] += g;
      d[c] += g * (double)za[n * sa + s];
    }
  for (int s = 0; s < sb; ++s)
    for (int c = 0; c < 3; ++c) {
      const double g = gxb[(n * sb + s) * 3 + c];
      o[c] += g;
      d[c] += g * (double)zb[n * sb + s];
    }
  const float* dv = rd + n * 3;
  float gn = g_nrm ? g_nrm[n] : 0.f;
  const float nrm = ray_norm(dv);
  for (int c = 0; c < 3; ++c) {
    g_o[n * 3 + c] = (float)o[c];
    const float extra = (g_nrm && nrm > 0.f) ? gn * dv[c] / nrm : 0.f;
    g_d[n * 3 + c] = (float)d[c] + extra;
  }
}

// ---------------------------------------------------------------------------------------------
// regulation (Renderer.py:280-294): float32 z in [0, 0.85*gt], jittered by t_rand
// one thread per (ray, sample): coalesced t_rand reads and z writes
__global__ void k_reg_z(pnr_render_params prm, const float* __restrict__ gt, const float* __restrict__ t_rand,
                        int64_t n_rays, float* __restrict__ z) {
  const int S = prm.n_samples;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n_rays * S) return;
  const int64_t n = e / S;
  const int s = (int)(e - n * S);
  const float far = gt[n] * 0.85f;
  auto z0 = [&](int k) { return (0.0f * (1.f - prm.t_vals[k])) + far * prm.t_vals[k]; };
  const float zs = z0(s);
  const float lower = s > 0 ? .5f * (zs + z0(s - 1)) : zs;
  const float upper = s < S - 1 ? .5f * (z0(s + 1) + zs) : zs;
  z[e] = lower + (upper - lower) * t_rand[e];
}

__global__ void k_extract_sigma(const float4* __restrict__ raw, int64_t P, float* __restrict__ sigma) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) sigma[p] = raw[p].w;
}

// rows [P, ld) are the MLP launch's padding: dL/draw = 0
__global__ void k_gout_sigma(const float* __restrict__ g_sigma, const float4* __restrict__ xP, int64_t P, int64_t ld,
                             float4* __restrict__ g_out) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (p < P) g_out[p] = make_float4(0.f, 0.f, 0.f, xP[p].w != 0.f ? g_sigma[p] : 0.f);
  else if (p < ld) g_out[p] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// ---------------------------------------------------------------------------------------------
// Mapper loss (src/Mapper.py:628-655) and its gradient, fused: one pass over the rays / regulation
// samples writes the gradients and a per-block partial sum, one block adds the partials in a fixed
// order (deterministic).  Per ray: [gt > 0] |gt - depth| (float64, gt promoted) + w_color
// sum_c |gt_c - c|; per regulation sample: w_reg |sigma|.  Gradients (torch abs: sign(x) with
// sign(0) = 0): g_depth = -sign(gt - depth) [gt > 0], g_color = -w_color sign(gt_c - c), g_sigma =
// w_reg sign(sigma).
constexpr int kLossParts = 256;
__device__ __forceinline__ double sgn(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }
__device__ __forceinline__ float sgnf(float x) { return x > 0.f ? 1.f : (x < 0.f ? -1.f : 0.f); }
__global__ __launch_bounds__(256) void k_map_loss(const float* __restrict__ gt, const double* __restrict__ depth,
                                                  const float* __restrict__ gtc, const float* __restrict__ col,
                                                  int64_t n, float w_color, const float* __restrict__ sigma,
                                                  int64_t ns, float w_reg, double* __restrict__ part,
                                                  double* __restrict__ g_depth, float* __restrict__ g_color,
                                                  float* __restrict__ g_sigma, uint32_t* __restrict__ ticket,
                                                  double* __restrict__ out) {
  __shared__ double red[4];
  double acc = 0.0;
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
    const float g = gt[i];
    const double e = (double)g - depth[i];
    const bool m = g > 0.f;
    acc += m ? fabs(e) : 0.0;
    g_depth[i] = m ? -sgn(e) : 0.0;
    float cs = 0.f;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float ec = gtc[i * 3 + c] - col[i * 3 + c];
      cs += fabsf(ec);
      g_color[i * 3 + c] = -w_color * sgnf(ec);
    }
    acc += (double)(w_color * cs);
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < ns; i += stride) {
    const float s = sigma[i];
    acc += (double)(w_reg * fabsf(s));
    g_sigma[i] = w_reg * sgnf(s);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  // the block's partial, then a ticket: the block that takes the last one adds every partial in a
  // fixed order (one launch; the sum is the same whichever block finishes last).  Hand-off per
  // MI355X_MICROARCH.md (Valid forms): the partial as an 8-B agent atomic, vmcnt(0), ticket atomic;
  // the last block reads the partials by 8-B agent atomics (no per-block L2 write-back, which a
  // release fence costs)
  __shared__ uint32_t last;
  if (threadIdx.x == 0) {
    atomicExch(reinterpret_cast<unsigned long long*>(part) + blockIdx.x,
               (unsigned long long)__double_as_longlong((red[0] + red[1]) + (red[2] + red[3])));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = atomicAdd(ticket, 1u);
    last = t == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  double v = (int)threadIdx.x < (int)gridDim.x
                 ? __longlong_as_double((long long)atomicAdd(reinterpret_cast<unsigned long long*>(part) + threadIdx.x, 0ull))
                 : 0.0;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = (red[0] + red[1]) + (red[2] + red[3]);
    *ticket = 0u;  // zero again for the next call on this workspace
  }
}

// ---------------------------------------------------------------------------------------------
// The tail of a Mapper iteration at wave-per-ray batches (pnr_map_step), fused: k_fine_w's final
// compositing, k_map_loss's loss terms and gradients (render rays and the ray's regulation samples)
// and k_fine_bwd_w's compositing backward in ONE launch, a wave per ray and four rays per block.
// Every value is formed by the same expressions as in those three kernels (the backward reuses the
// forward's weights and sums instead of recomputing them from the stored order: the same bits), so
// the dL/draw rows are identical to the three-launch sequence; only the loss's summation order
// differs (per ray, the four rays of a block, then the blocks in order, added by the block that takes
// the last ticket).  Two launch boundaries and the compositing recompute leave the critical path.
struct FineLoss {
  const float* gt;      // (n) gt depth
  const float* gtc;     // (n, 3) gt colour
  float w_color, w_reg;
  const float4* rawr;   // regulation rows of launch A (sigma = .w)
  const float4* insr;   // their kPtsX4 rows (inside flags)
  float4* gor;          // their dL/draw rows
  float4* pad2;         // importance padding rows
  int np2;
  double* part;         // [gridDim.x] block partial losses
  uint32_t* ticket;     // zero on entry, left zero
  double* loss;
};
template <int SS, int II>
__global__ __launch_bounds__(256) void k_fine_loss_w(pnr_render_params prm, const float* __restrict__ rd,
                                                     const double* __restrict__ zc, const double* __restrict__ zi,
                                                     const float4* __restrict__ rawc, const float4* __restrict__ rawi,
                                                     const float4* __restrict__ insc, const float4* __restrict__ insi,
                                                     int64_t n_rays, float4* __restrict__ goc, float4* __restrict__ goi,
                                                     float* __restrict__ g_nrm, float4* __restrict__ pad0, int np0,
                                                     float4* __restrict__ pad1, int np1, FineLoss fl) {
  __shared__ double zn_[4][PNR_MAX_SAMPLES];
  __shared__ float4 cr_[4][PNR_MAX_SAMPLES];   // raw of each sample, by its unsorted index
  __shared__ float ci_[4][PNR_MAX_SAMPLES];    // its inside flag
  __shared__ uint8_t os_[4][PNR_MAX_SAMPLES + 4];
  __shared__ double red[4];
  __shared__ uint32_t last;
  const int l = threadIdx.x & 63, wv = threadIdx.x >> 6;
  {  // the segments' padding rows: dL/draw = 0 (as k_fine_bwd_w)
    const int64_t gi = (int64_t)blockIdx.x * 256 + threadIdx.x, gs = (int64_t)gridDim.x * 256;
    for (int64_t i = gi; i < np0; i += gs) pad0[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < np1; i += gs) pad1[i] = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t i = gi; i < fl.np2; i += gs) fl.pad2[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // a wave past the batch works on the last ray and stores nothing (the block barriers stay uniform)
  const bool live = (int64_t)blockIdx.x * 4 + wv < n_rays;
  const int64_t n = live ? (int64_t)blockIdx.x * 4 + wv : n_rays - 1;
  double* zn = zn_[wv];
  uint8_t* os = os_[wv];
  const int S = SS > 0 ? SS : prm.n_samples, I = II > 0 ? II : prm.n_importance, M = S + I;
  // every global input of the ray in ONE round trip: the depths, the raw outputs and inside flags by
  // unsorted sample (read through LDS by rank below, instead of two dependent loads after the sort),
  // the ray's gt depth / colour and its regulation rows
  const int lq = l < M ? l : M - 1;
  const double zl = *(lq < S ? zc + n * S + lq : zi + n * I + (lq - S));
  const float4 cl = *(lq < S ? rawc + n * S + lq : rawi + n * I + (lq - S));
  const float il = (lq < S ? insc + n * S + lq : insi + n * I + (lq - S))->w;
  const float g = fl.gt[n];
  const float gtc0 = fl.gtc[n * 3 + 0], gtc1 = fl.gtc[n * 3 + 1], gtc2 = fl.gtc[n * 3 + 2];
  const int64_t rr = n * S + (l < S ? l : S - 1);
  const float sg = fl.rawr[rr].w;
  const float ir = fl.insr[rr].w;
  const float nrm = ray_norm(rd + n * 3);  // (in this round trip: after the barriers below it would wait alone)
  zn[l] = zl;
  cr_[wv][l] = cl;
  ci_[wv][l] = il;
  os[l] = 0;
  if (l < 4) os[64 + l] = 0;
  __syncthreads();
  if (l < M) {
    int r = 0;
    for (int m = 0; m < M; ++m) {
      const double v = zn[m];
      r += (lt_nan(v, zl) || (eq_nan(v, zl) && m < l)) ? 1 : 0;
    }
    os[r] = (uint8_t)l;
  }
  __syncthreads();
  const int s = os[l];
  const double zq = zn[s];
  const double znx = l + 1 < M ? zn[os[l + 1]] : 0.0;
  const float4 c = cr_[wv][s];  // lanes >= M: s = 0, never read
  const float dz = l < M - 1 ? (float)(znx - zq) : 1e10f;
  const float delta = dz * nrm;
  const float sr = relu(c.w);
  const float ex = expf(-sr * delta);
  const float a = 1.f - ex;
  const float Tf = (float)excl_cumprod((double)(1.f - a + 1e-10f), M, l);
  const float w = a * Tf;
  const float p0 = w * c.x, p1 = w * c.y, p2 = w * c.z;
  const double pD = (double)w * zq;
  float r0 = 0.f, r1 = 0.f, r2 = 0.f;
  double D = 0.0;
  for (int q = 0; q < M; ++q) {
    r0 += rlf(p0, q); r1 += rlf(p1, q); r2 += rlf(p2, q);
    D += rld(pD, q);
  }
  // ---- k_map_loss: this ray's terms and the upstream gradients (wave-uniform)
  const double e = (double)g - D;
  const bool msk = g > 0.f;
  double Lr = msk ? fabs(e) : 0.0;
  const double gd = msk ? -sgn(e) : 0.0;
  const float col[3] = {r0, r1, r2}, gtc[3] = {gtc0, gtc1, gtc2};
  float gr[3];
  float cs = 0.f;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float ec = gtc[k] - col[k];
    cs += fabsf(ec);
    gr[k] = -fl.w_color * sgnf(ec);
  }
  Lr += (double)(fl.w_color * cs);
  {  // the ray's regulation samples: w_reg |sigma| and dL/draw = (0, 0, 0, w_reg sign(sigma) [inside])
    const float gsg = fl.w_reg * sgnf(sg);
    if (live && l < S) fl.gor[rr] = make_float4(0.f, 0.f, 0.f, ir != 0.f ? gsg : 0.f);
    const double ls = (double)(fl.w_reg * fabsf(sg));
    for (int q = 0; q < S; ++q) Lr += rld(ls, q);
  }
  // ---- the loss hand-off, issued now so its round trips run under the compositing backward: the
  // block partial as an 8-B agent atomic, read back by 8-B agent atomics (MI355X_MICROARCH.md, valid
  // hand-off forms: no L2 write-back per block, which a release fence would cost), then the ticket;
  // the block that takes the last ticket adds the partials in order at the end
  if (l == 0) red[wv] = live ? Lr : 0.0;
  __syncthreads();
  uint32_t tk = 0u;
  if (threadIdx.x == 0) {
    const double pb = ((red[0] + red[1]) + red[2]) + red[3];
    atomicExch(reinterpret_cast<unsigned long long*>(fl.part) + blockIdx.x, __double_as_longlong(pb));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    tk = atomicAdd(fl.ticket, 1u);
  }
  // ---- k_fine_bwd_w with g_var = 0, from the forward's values
  const bool act = l < M;
  const bool inside = act && ci_[wv][s] != 0.f;
  const double gv = 0.0;
  const float gr0 = gr[0], gr1 = gr[1], gr2 = gr[2];
  const double pS = (double)(a * Tf) * (zq - D);
  double sdev = 0.0;
  for (int q = 0; q < M; ++q) sdev += rld(pS, q);
  const double gD = gd - 2.0 * gv * sdev;
  const double dd = zq - D;
  const float gw = (gr0 * c.x + gr1 * c.y + gr2 * c.z) + (float)(gD * zq) + (float)(gv * dd * dd);
  const float pa = gw * a, g1 = 1.f - a + 1e-10f;
  float R = 0.f, Rl = 0.f;
  for (int q = M - 1; q >= 0; --q) {
    Rl = l == q ? R : Rl;
    R = rlf(pa, q) + rlf(g1, q) * R;
  }
  const float ga = Tf * (gw - Rl);
  float gs = c.w > 0.f ? ga * ex * delta : 0.f;
  if (!inside) gs = 0.f;
  const float pg = (ga * ex * sr) * dz;
  float gn = 0.f;
  for (int q = M - 1; q >= 0; --q) gn += rlf(pg, q);
  if (live && act) {
    const float4 go = make_float4(gr0 * w, gr1 * w, gr2 * w, gs);
    if (s < S) goc[n * S + s] = go; else goi[n * I + (s - S)] = go;
  }
  if (live && g_nrm && l == 0) g_nrm[n] = gn;
  // ---- the loss: the last block adds the partials in order (k_map_loss's hand-off)
  if (threadIdx.x == 0) last = tk == gridDim.x - 1 ? 1u : 0u;
  __syncthreads();
  if (!last) return;
  double v = 0.0;
  for (int i = (int)threadIdx.x; i < (int)gridDim.x; i += 256)
    v += __longlong_as_double(atomicAdd(reinterpret_cast<unsigned long long*>(fl.part) + i, 0ull));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  __syncthreads();
  if (l == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) {
    fl.loss[0] = (red[0] + red[1]) + (red[2] + red[3]);
    *fl.ticket = 0u;
  }
}

// ---------------------------------------------------------------------------------------------
// rays: dirs = [(i-cx)/fx, -(j-cy)/fy, -1]; rays_d = sum(dirs * c2w[:3,:3], -1); rays_o = c2w[:3,3]
__device__ __forceinline__ void make_ray(float i, float j, float fx, float fy, float cx, float cy,
                                         const float* __restrict__ c2w, int ld, float* o, float* d) {
  const float dx = (i - cx) / fx, dy = -((j - cy) / fy), dzv = -1.f;
  for (int r = 0; r < 3; ++r) {
    // torch.sum over the last dim of 3 products: ((a0 + a1) + a2), products rounded
    const float p0 = dx * c2w[r * ld + 0], p1 = dy * c2w[r * ld + 1], p2 = dzv * c2w[r * ld + 2];
    d[r] = (p0 + p1) + p2;
    o[r] = c2w[r * ld + 3];
  }
}

__global__ void k_get_rays(int H, int W, float fx, float fy, float cx, float cy, const float* __restrict__ c2w,
                           float* __restrict__ ro, float* __restrict__ rd) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= (int64_t)H * W) return;
  const int row = (int)(k / W), col = (int)(k % W);
  make_ray((float)col, (float)row, fx, fy, cx, cy, c2w, 4, ro + k * 3, rd + k * 3);
}

__global__ void k_rays_from_uv(const float* __restrict__ ii, const float* __restrict__ jj, int64_t n, float fx,
                               float fy, float cx, float cy, const float* __restrict__ c2w, float* __restrict__ ro,
                               float* __restrict__ rd) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  make_ray(ii[k], jj[k], fx, fy, cx, cy, c2w, 4, ro + k * 3, rd + k * 3);
}

// One Mapper iteration's pixel batch over its keyframe window in one launch (src/Mapper.py:560-606
// per frame: get_samples -> get_sample_uv / select_uv / get_rays_from_uv, src/common.py:74-134):
// ray r belongs to frame r / per_frame, its pixel is idx[r] (uniform over the H x W image, row-major),
// i = idx % W (column), j = idx / W (row); the ray as k_rays_from_uv, gt depth / colour gathered from
// the frame.  c2w: (F, 4, 4); depth (F, H, W); color (F, H, W, 3).
__global__ void k_window_rays(const int64_t* __restrict__ idx, int64_t n, int64_t per_frame, int64_t hw, int W,
                              float fx, float fy, float cx, float cy, const float* __restrict__ c2w,
                              const float* __restrict__ depth, const float* __restrict__ color,
                              float* __restrict__ ro, float* __restrict__ rd, float* __restrict__ gd,
                              float* __restrict__ gc) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n) return;
  const int64_t f = k / per_frame;
  int64_t pix = idx[k];
  pix = pix < 0 ? 0 : (pix >= hw ? hw - 1 : pix);  // select_uv's clamp (common.py:99-100) + stay in the frame
  const float i = (float)(pix % W), j = (float)(pix / W);
  make_ray(i, j, fx, fy, cx, cy, c2w + f * 16, 4, ro + k * 3, rd + k * 3);
  const int64_t q = f * hw + pix;
  gd[k] = depth[q];
  gc[k * 3 + 0] = color[q * 3 + 0];
  gc[k * 3 + 1] = color[q * 3 + 1];
  gc[k * 3 + 2] = color[q * 3 + 2];
}

// A mapping iteration's whole window batch in ONE launch, drawn on the device: the uniform pixels
// (torch.randint(H*W) per ray in Mapper.py:560-606's get_samples), the regulation jitter t_rand
// (torch.rand, Renderer.py:293), the rays and gt of k_window_rays, and the batch far clamp
// max(1.2 gt) (k_gt_max, Renderer.py:112) -- in place of randint + rand (+ the two seed / offset
// fills torch's RNG records in a captured graph) + the gt max.  The draws are a counter-based hash
// (splitmix64 finaliser of seed, batch and draw index), not torch's Philox stream: the same
// distribution, a different sequence.  The state holds the batch counter (advanced by the block
// that takes the last ticket, so a captured graph draws a fresh batch per replay), the ticket and
// the per-block maxima.
constexpr int kSampleParts = 64;
struct SampleState {
  int64_t batch;
  uint32_t ticket;
  uint32_t pad;
  uint64_t part[kSampleParts];  // per-block gt maxima (float bits), written and read by 8-B atomics
};
static_assert(sizeof(SampleState) == 16 + 8 * kSampleParts, "sampler state layout");
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__global__ __launch_bounds__(256) void k_window_sample(uint64_t seed, SampleState* __restrict__ stt, int64_t n,
                                                       int64_t per_frame, int64_t hw, int W, float fx, float fy,
                                                       float cx, float cy, const float* __restrict__ c2w,
                                                       const float* __restrict__ depth,
                                                       const float* __restrict__ color, int S, float* __restrict__ ro,
                                                       float* __restrict__ rd, float* __restrict__ gd,
                                                       float* __restrict__ gc, float* __restrict__ t_rand,
                                                       int64_t* __restrict__ idx_out, float* __restrict__ far_out) {
  __shared__ float red[4];
  __shared__ uint32_t last;
  const int64_t batch = stt->batch;
  const uint64_t base = mix64(seed + (uint64_t)batch * 0x9E3779B97F4A7C15ull);
  // blocks [0, nbr) draw the rays (and their gt maxima, part[0..nbr)); the others draw the jitter,
  // one value per thread (a thread per ray drawing its 32 values serially was the launch's latency)
  const int nbr = (int)(n < (int64_t)kSampleParts * 256 ? (n + 255) / 256 : kSampleParts);
  float m = -INFINITY;
  if ((int)blockIdx.x < nbr) {
    for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < n; k += (int64_t)nbr * 256) {
      const int64_t f = k / per_frame;
      const uint64_t r = mix64(base + (uint64_t)k * 0xD1B54A32D192ED03ull);
      const int64_t pix = (int64_t)(((r >> 32) * (uint64_t)hw) >> 32);  // uniform in [0, hw) (hw < 2^32)
      if (idx_out) idx_out[k] = pix;
      make_ray((float)(pix % W), (float)(pix / W), fx, fy, cx, cy, c2w + f * 16, 4, ro + k * 3, rd + k * 3);
      const int64_t q = f * hw + pix;
      const float d = depth[q];
      gd[k] = d;
      gc[k * 3 + 0] = color[q * 3 + 0];
      gc[k * 3 + 1] = color[q * 3 + 1];
      gc[k * 3 + 2] = color[q * 3 + 2];
      m = max_nanf(m, d * 1.2f);
    }
  } else {
    const int64_t ns = n * S, stride = (int64_t)(gridDim.x - nbr) * 256;
    for (int64_t e = (int64_t)(blockIdx.x - nbr) * 256 + threadIdx.x; e < ns; e += stride) {
      // 24-bit uniforms in [0, 1), like torch.rand's float32: value (k, s) is draw n + k S + s
      const uint64_t u = mix64(base + (uint64_t)(n + e) * 0xD1B54A32D192ED03ull);
      t_rand[e] = (float)(uint32_t)(u >> 40) * 0x1p-24f;
    }
  }
  m = block_max_256(m, red);
  // ticket hand-off as k_map_loss (8-B agent atomics both sides); the last block reduces the maxima
  // and advances the batch
  if (threadIdx.x == 0) {
    if ((int)blockIdx.x < nbr) atomicExch(stt->part + blockIdx.x, (unsigned long long)__float_as_uint(m));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const uint32_t t = atomicAdd(&stt->ticket, 1u);
    last = t == gridDim.x - 1 ? 1u : 0u;
  }
  __syncthreads();
  if (!last) return;
  __shared__ float red2[4];
  const float v = block_max_256(
      (int)threadIdx.x < nbr ? __uint_as_float((uint32_t)atomicAdd(stt->part + threadIdx.x, 0ull)) : -INFINITY, red2);
  if (threadIdx.x == 0) {
    if (far_out) far_out[0] = v;
    stt->batch = batch + 1;
    stt->ticket = 0u;
  }
}

// torch.optim.Adam (amsgrad=False, weight_decay=0), single-tensor semantics
__global__ void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                       float* __restrict__ v, int64_t n, float beta1, float beta2, float eps, float step_size,
                       float bc2_sqrt) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float gi = g[i];
  float mi = m[i];
  mi = mi + (1.f - beta1) * (gi - mi);           // exp_avg.lerp_(grad, 1-beta1)
  float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;  // exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] + (-step_size) * (mi / denom);
}

// the same with the step read on the device (*step_count + 1); the bias corrections follow
// pnr_adam_step's host arithmetic (double pow, then float)
__global__ void k_adam_dev(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                           float* __restrict__ v, int64_t n, float lr, float beta1, float beta2, float eps,
                           const int32_t* __restrict__ step_count) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const double t = (double)(*step_count + 1);
  const double bc1 = 1.0 - pow((double)beta1, t), bc2 = 1.0 - pow((double)beta2, t);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  const float gi = g[i];
  float mi = m[i];
  mi = mi + (1.f - beta1) * (gi - mi);
  float vi = v[i] * beta2 + (1.f - beta2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float denom = sqrtf(vi) / bc2_sqrt + eps;
  p[i] = p[i] + (-step_size) * (mi / denom);
}
// Adam over up to kAdamSegs learning-rate segments of one flat buffer in ONE launch (block ranges per
// segment), the step read on the device (step2[0] + 1) and advanced by the block that takes the last
// ticket (step2[1], zero between launches): every block has read the step before its ticket.
constexpr int kAdamSegs = 4;
struct AdamSegs {
  int64_t off[kAdamSegs], n[kAdamSegs];
  float* m[kAdamSegs];
  float* v[kAdamSegs];
  float lr[kAdamSegs];
  uint16_t* h[kAdamSegs];    // ABI 12: float16 copy of the updated segment (the gather's f16 features) or null
  int first[kAdamSegs + 1];  // first block of each segment
  int nseg;
};
__global__ __launch_bounds__(256) void k_adam_multi(float* __restrict__ p, const float* __restrict__ g, AdamSegs S,
                                                    float beta1, float beta2, float eps, int32_t* __restrict__ step2) {
  int q = 0;
  while (q + 1 < S.nseg && (int)blockIdx.x >= S.first[q + 1]) ++q;
  const int64_t i0 = (int64_t)((int)blockIdx.x - S.first[q]) * 256 + threadIdx.x;
  const int64_t stride = (int64_t)(S.first[q + 1] - S.first[q]) * 256;
  const int32_t step = step2[0];
  const double t = (double)(step + 1);
  const double bc1 = 1.0 - pow((double)beta1, t), bc2 = 1.0 - pow((double)beta2, t);
  const float step_size = (float)((double)S.lr[q] / bc1);
  const float bc2_sqrt = (float)sqrt(bc2);
  // four elements in flight per thread (loads first), so the grid stays small without a serial
  // chain of dependent loads per thread
  const int64_t nq = S.n[q], off = S.off[q];
  float* __restrict__ mq = S.m[q];
  float* __restrict__ vq = S.v[q];
  uint16_t* __restrict__ hq = S.h[q];
  for (int64_t b = i0; b < nq; b += 4 * stride) {
    float gi[4], mi[4], vi[4], pi[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {  // clamped, unconditional loads (a predicated load waits on its own)
      const int64_t i = b + u * stride < nq ? b + u * stride : nq - 1;
      gi[u] = g[off + i];
      mi[u] = mq[i];
      vi[u] = vq[i];
      pi[u] = p[off + i];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = b + u * stride;
      if (i < nq) {
        const float mn = mi[u] + (1.f - beta1) * (gi[u] - mi[u]);
        const float vn = vi[u] * beta2 + (1.f - beta2) * gi[u] * gi[u];
        mq[i] = mn;
        vq[i] = vn;
        const float denom = sqrtf(vn) / bc2_sqrt + eps;
        const float pn = pi[u] + (-step_size) * (mn / denom);
        p[off + i] = pn;
        if (hq) hq[i] = __builtin_bit_cast(uint16_t, (_Float16)pn);  // RNE, as torch's float16 copy
      }
    }
  }
  __syncthreads();  // the block's step reads come before its ticket
  if (threadIdx.x == 0) {
    const uint32_t t = atomicAdd(reinterpret_cast<uint32_t*>(step2 + 1), 1u);
    if (t == gridDim.x - 1) {
      step2[0] = step + 1;
      step2[1] = 0;
    }
  }
}

__global__ void k_step_advance(int32_t* step_count) {
  if (threadIdx.x == 0) atomicAdd(step_count, 1);
}

// ---------------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------------
static inline unsigned nblk(int64_t n, int b) { return (unsigned)((n + b - 1) / b); }

int launch_gt_max(const float* gt, int64_t n, float* out, hipStream_t st) {
  const int parts = (int)std::min<int64_t>(kGtParts, std::max<int64_t>(1, (n + 4095) / 4096));
  hipLaunchKernelGGL(k_gt_max_part, dim3(parts), dim3(256), 0, st, gt, n, out);
  if (parts > 1) hipLaunchKernelGGL(k_gt_max, dim3(1), dim3(256), 0, st, parts, out);  // (<= 4,096 rays: one launch)
  return hip_status(hipGetLastError());
}
int launch_coarse_z(const pnr_render_params& prm, const float* ro, const float* rd, const float* gt,
                    const float* gmax, int64_t n, double* z, double* far_out, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_coarse_z, dim3(nblk(n, 128)), dim3(128), 0, st, prm, ro, rd, gt, gmax, n, z, far_out);
  return hip_status(hipGetLastError());
}
// batches up to this many rays run the wave-per-ray compositing kernels (k_pdf_w / k_fine_w /
// k_fine_bwd_w): below it the thread-per-ray kernels leave most SIMDs idle
constexpr int64_t kWaveRays = 32768;
int launch_pdf(const pnr_render_params& prm, const float* rd, const double* zc, const float* rawc, int64_t n,
               double* zi, hipStream_t st, const float* ro = nullptr, float* x4i = nullptr, int64_t x4i_pad = 0,
               const float* rawr = nullptr, float* sigma = nullptr) {
  if (n <= 0) return 0;
  const MapPts mp{ro, reinterpret_cast<float4*>(x4i), x4i_pad, reinterpret_cast<const float4*>(rawr), sigma};
  if (n <= kWaveRays) {
    if (prm.n_samples == 32 && prm.n_importance == 12)
      hipLaunchKernelGGL((k_pdf_w<32, 12>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, (const float4*)rawc, n, zi,
                         mp);
    else
      hipLaunchKernelGGL((k_pdf_w<0, 0>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, (const float4*)rawc, n, zi,
                         mp);
    return hip_status(hipGetLastError());
  }
  if (prm.n_samples == 32 && prm.n_importance == 12)  // the config's counts (configs/pointNeRF_slam.yaml)
    hipLaunchKernelGGL((k_pdf<32, 12>), dim3(nblk(n, 64)), dim3(64), 0, st, prm, rd, zc, (const float4*)rawc, n, zi, mp);
  else
    hipLaunchKernelGGL((k_pdf<0, 0>), dim3(nblk(n, 64)), dim3(64), 0, st, prm, rd, zc, (const float4*)rawc, n, zi, mp);
  return hip_status(hipGetLastError());
}
MapRowsArgs map_rows_args(const pnr_render_params& prm, const float* ro, const float* rd, const float* gt,
                          const float* t_rand, const float* gmax, int64_t n, int64_t pr, double* zc, double* far_out) {
  MapRowsArgs m{};
  m.ro = ro;
  m.rd = rd;
  m.gt = gt;
  m.t_rand = t_rand;
  m.gmax = gmax;
  m.n_rays = n;
  m.pr = pr;
  m.zc = zc;
  m.far_out = far_out;
  for (int i = 0; i < 6; ++i) m.bound[i] = prm.bound[i];
  m.far_clamp = prm.far_clamp;
  m.far_mode = prm.far_mode;
  m.lindisp = prm.lindisp;
  m.n_samples = prm.n_samples;
  for (int i = 0; i < PNR_MAX_SAMPLES; ++i) m.t_vals[i] = prm.t_vals[i];
  return m;
}
int launch_map_pts(const pnr_render_params& prm, const float* ro, const float* rd, const float* gt, const float* t_rand,
                   const float* gmax, int64_t n, int64_t pr, int64_t rows, double* zc, double* far_out, float* x4,
                   hipStream_t st) {
  if (rows <= 0) return 0;
  const MapRowsArgs m = map_rows_args(prm, ro, rd, gt, t_rand, gmax, n, pr, zc, far_out);
  hipLaunchKernelGGL(k_map_pts, dim3(nblk(rows, 256)), dim3(256), 0, st, m, rows, (float4*)x4);
  return hip_status(hipGetLastError());
}
int launch_fine(const pnr_render_params& prm, const float* rd, const double* zc, const double* zi,
                const float* rawc, const float* rawi, int64_t n, double* depth, double* var, float* rgb,
                uint8_t* ord, hipStream_t st) {
  if (n <= 0) return 0;
  if (n <= kWaveRays) {
    if (prm.n_samples == 32 && prm.n_importance == 12)
      hipLaunchKernelGGL((k_fine_w<32, 12>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                         (const float4*)rawi, n, depth, var, rgb, ord);
    else
      hipLaunchKernelGGL((k_fine_w<0, 0>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                         (const float4*)rawi, n, depth, var, rgb, ord);
    return hip_status(hipGetLastError());
  }
  if (prm.n_samples == 32 && prm.n_importance == 12)
    hipLaunchKernelGGL((k_fine<32, 12>), dim3(nblk(n, 64)), dim3(64), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, n, depth, var, rgb, ord);
  else
    hipLaunchKernelGGL((k_fine<0, 0>), dim3(nblk(n, 64)), dim3(64), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, n, depth, var, rgb, ord);
  return hip_status(hipGetLastError());
}
int launch_fine_bwd(const pnr_render_params& prm, const float* rd, const double* zc, const double* zi,
                    const float* rawc, const float* rawi, const float4* insc, const float4* insi,
                    const uint8_t* ord, int64_t n, const double* gd, const double* gv, const float* grgb,
                    float* goc, float* goi, float* g_nrm, float* pad0, int np0, float* pad1, int np1,
                    hipStream_t st, const float* g_sigma = nullptr, const float4* insr = nullptr,
                    float* gor = nullptr, float* pad2 = nullptr, int np2 = 0) {
  if (n <= 0) return 0;
  const int M = prm.n_samples + prm.n_importance;
  const size_t sh = (size_t)M * 64 * (8 + 2 * 4);
  const MapBwd mb{g_sigma, insr, reinterpret_cast<float4*>(gor), reinterpret_cast<float4*>(pad2), np2};
  if (n <= kWaveRays) {
    if (prm.n_samples == 32 && prm.n_importance == 12)
      hipLaunchKernelGGL((k_fine_bwd_w<32, 12>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, zi,
                         (const float4*)rawc, (const float4*)rawi, insc, insi, ord, n, gd, gv, grgb, (float4*)goc,
                         (float4*)goi, g_nrm, (float4*)pad0, np0, (float4*)pad1, np1, mb);
    else
      hipLaunchKernelGGL((k_fine_bwd_w<0, 0>), dim3((unsigned)n), dim3(64), 0, st, prm, rd, zc, zi,
                         (const float4*)rawc, (const float4*)rawi, insc, insi, ord, n, gd, gv, grgb, (float4*)goc,
                         (float4*)goi, g_nrm, (float4*)pad0, np0, (float4*)pad1, np1, mb);
    return hip_status(hipGetLastError());
  }
  if (prm.n_samples == 32 && prm.n_importance == 12)
    hipLaunchKernelGGL((k_fine_bwd<32, 12>), dim3(nblk(n, 64)), dim3(64), sh, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, insc, insi, ord, n, gd, gv, grgb, (float4*)goc, (float4*)goi, g_nrm,
                       (float4*)pad0, np0, (float4*)pad1, np1, mb);
  else
    hipLaunchKernelGGL((k_fine_bwd<0, 0>), dim3(nblk(n, 64)), dim3(64), sh, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, insc, insi, ord, n, gd, gv, grgb, (float4*)goc, (float4*)goi, g_nrm,
                       (float4*)pad0, np0, (float4*)pad1, np1, mb);
  return hip_status(hipGetLastError());
}
// the fused compositing + loss + compositing backward (k_fine_loss_w); n <= fine_loss_max_rays()
int64_t fine_loss_max_rays() { return kWaveRays; }
int64_t fine_loss_parts(int64_t n) { return (n + 3) / 4; }
int launch_fine_loss(const pnr_render_params& prm, const float* rd, const double* zc, const double* zi,
                     const float* rawc, const float* rawi, const float4* insc, const float4* insi, int64_t n,
                     const float* gt, const float* gtc, float w_color, float w_reg, const float* rawr,
                     const float4* insr, float* gor, float* goc, float* goi, float* g_nrm, float* pad0, int np0,
                     float* pad1, int np1, float* pad2, int np2, double* part, uint32_t* ticket, double* loss,
                     hipStream_t st) {
  if (n <= 0 || n > kWaveRays) return PNR_E_ARG;
  const FineLoss fl{gt, gtc, w_color, w_reg, reinterpret_cast<const float4*>(rawr), insr,
                    reinterpret_cast<float4*>(gor), reinterpret_cast<float4*>(pad2), np2, part, ticket, loss};
  const unsigned nb = (unsigned)fine_loss_parts(n);
  if (prm.n_samples == 32 && prm.n_importance == 12)
    hipLaunchKernelGGL((k_fine_loss_w<32, 12>), dim3(nb), dim3(256), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, insc, insi, n, (float4*)goc, (float4*)goi, g_nrm, (float4*)pad0, np0,
                       (float4*)pad1, np1, fl);
  else
    hipLaunchKernelGGL((k_fine_loss_w<0, 0>), dim3(nb), dim3(256), 0, st, prm, rd, zc, zi, (const float4*)rawc,
                       (const float4*)rawi, insc, insi, n, (float4*)goc, (float4*)goi, g_nrm, (float4*)pad0, np0,
                       (float4*)pad1, np1, fl);
  return hip_status(hipGetLastError());
}
int launch_ray_grads_f64(const float* rd, const double* za, int sa, const double* zb, int sb, const float* gxa,
                         const float* gxb, const float* g_nrm, int64_t n, float* g_o, float* g_d, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_ray_grads<double>, dim3(nblk(n, 128)), dim3(128), 0, st, rd, za, sa, zb, sb, gxa, gxb, g_nrm,
                     n, g_o, g_d);
  return hip_status(hipGetLastError());
}
int launch_ray_grads_f32(const float* rd, const float* za, int sa, const float* gxa, int64_t n, float* g_o,
                         float* g_d, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_ray_grads<float>, dim3(nblk(n, 128)), dim3(128), 0, st, rd, za, sa, (const float*)nullptr, 0,
                     gxa, (const float*)nullptr, (const float*)nullptr, n, g_o, g_d);
  return hip_status(hipGetLastError());
}
int launch_reg_z(const pnr_render_params& prm, const float* gt, const float* t_rand, int64_t n, float* z,
                 hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_reg_z, dim3(nblk(n * prm.n_samples, 256)), dim3(256), 0, st, prm, gt, t_rand, n, z);
  return hip_status(hipGetLastError());
}
int launch_map_loss(const float* gt, const double* depth, const float* gtc, const float* col, int64_t n,
                    float w_color, const float* sigma, int64_t ns, float w_reg, double* part, double* loss,
                    double* g_depth, float* g_color, float* g_sigma, hipStream_t st) {
  const int64_t m = n > ns ? n : ns;
  int parts = (int)((m + 1023) / 1024);
  parts = parts < 1 ? 1 : (parts > kLossParts ? kLossParts : parts);
  // ticket word after the kLossParts partials (the workspace holds kLossParts + 8 doubles, zeroed
  // by the caller before its first use; the kernel leaves it zero)
  hipLaunchKernelGGL(k_map_loss, dim3(parts), dim3(256), 0, st, gt, depth, gtc, col, n, w_color, sigma, ns, w_reg,
                     part, g_depth, g_color, g_sigma, reinterpret_cast<uint32_t*>(part + kLossParts), loss);
  return hip_status(hipGetLastError());
}
int launch_extract_sigma(const float* raw, int64_t P, float* sigma, hipStream_t st) {
  if (P <= 0) return 0;
  hipLaunchKernelGGL(k_extract_sigma, dim3(nblk(P, 256)), dim3(256), 0, st, (const float4*)raw, P, sigma);
  return hip_status(hipGetLastError());
}
int launch_gout_sigma(const float* g_sigma, const float4* inside, int64_t P, int64_t ld, float* g_out, hipStream_t st) {
  if (ld <= 0) return 0;
  hipLaunchKernelGGL(k_gout_sigma, dim3(nblk(ld, 256)), dim3(256), 0, st, g_sigma, inside, P, ld, (float4*)g_out);
  return hip_status(hipGetLastError());
}
int launch_get_rays(int H, int W, float fx, float fy, float cx, float cy, const float* c2w, float* ro, float* rd,
                    hipStream_t st) {
  const int64_t n = (int64_t)H * W;
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_get_rays, dim3(nblk(n, 256)), dim3(256), 0, st, H, W, fx, fy, cx, cy, c2w, ro, rd);
  return hip_status(hipGetLastError());
}
int launch_rays_from_uv(const float* i, const float* j, int64_t n, float fx, float fy, float cx, float cy,
                        const float* c2w, float* ro, float* rd, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_rays_from_uv, dim3(nblk(n, 256)), dim3(256), 0, st, i, j, n, fx, fy, cx, cy, c2w, ro, rd);
  return hip_status(hipGetLastError());
}
int launch_window_rays(const int64_t* idx, int64_t n, int64_t per_frame, int H, int W, float fx, float fy, float cx,
                       float cy, const float* c2w, const float* depth, const float* color, float* ro, float* rd,
                       float* gd, float* gc, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_window_rays, dim3(nblk(n, 256)), dim3(256), 0, st, idx, n, per_frame, (int64_t)H * W, W, fx, fy,
                     cx, cy, c2w, depth, color, ro, rd, gd, gc);
  return hip_status(hipGetLastError());
}
int64_t window_sample_state_bytes() { return (int64_t)sizeof(SampleState); }
int launch_window_sample(uint64_t seed, void* state, int64_t n, int64_t per_frame, int H, int W, float fx, float fy,
                         float cx, float cy, const float* c2w, const float* depth, const float* color, int S,
                         float* ro, float* rd, float* gd, float* gc, float* t_rand, int64_t* idx, float* far_out,
                         hipStream_t st) {
  if (n <= 0) return 0;
  const int64_t nbr = std::min<int64_t>(kSampleParts, nblk(n, 256));                  // ray blocks
  const int64_t nbj = std::min<int64_t>(192, nblk(n * (S > 0 ? S : 0), 1024));      // jitter blocks (4 per thread)
  const int64_t nb = nbr + nbj;
  hipLaunchKernelGGL(k_window_sample, dim3((unsigned)nb), dim3(256), 0, st, seed, (SampleState*)state, n, per_frame,
                     (int64_t)H * W, W, fx, fy, cx, cy, c2w, depth, color, S, ro, rd, gd, gc, t_rand, idx, far_out);
  return hip_status(hipGetLastError());
}
int launch_adam_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                    float eps, const int32_t* step_count, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_adam_dev, dim3(nblk(n, 256)), dim3(256), 0, st, p, g, m, v, n, lr, beta1, beta2, eps,
                     step_count);
  return hip_status(hipGetLastError());
}
int launch_adam_multi(float* p, const float* g, int nseg, const int64_t* off, const int64_t* n, float* const* m,
                      float* const* v, const float* lr, float beta1, float beta2, float eps, int32_t* step2,
                      hipStream_t st, uint16_t* const* half) {
  if (nseg < 1 || nseg > kAdamSegs) return PNR_E_ARG;
  AdamSegs S{};
  int blocks = 0;
  for (int q = 0; q < nseg; ++q) {
    S.off[q] = off[q];
    S.n[q] = n[q];
    S.m[q] = m[q];
    S.v[q] = v[q];
    S.lr[q] = lr[q];
    S.h[q] = half ? half[q] : nullptr;
    S.first[q] = blocks;
    // a block per 1,024 elements (one pass of four loads per thread), at most 1,024 blocks per segment:
    // every block takes one ticket (a ticket per 256 elements -- 870 for the decoder -- queued on one
    // address for ~10 us), and 128 blocks left the 6.4M point features of config C3 latency-bound
    // (49 dependent passes per thread: 88 us)
    const int64_t nb = nblk(n[q] > 0 ? n[q] : 1, 1024);
    blocks += (int)(nb < 1024 ? nb : 1024);
  }
  S.first[nseg] = blocks;
  S.nseg = nseg;
  hipLaunchKernelGGL(k_adam_multi, dim3((unsigned)blocks), dim3(256), 0, st, p, g, S, beta1, beta2, eps, step2);
  return hip_status(hipGetLastError());
}
int launch_step_advance(int32_t* step_count, hipStream_t st) {
  hipLaunchKernelGGL(k_step_advance, dim3(1), dim3(64), 0, st, step_count);
  return hip_status(hipGetLastError());
}
int launch_adam(float* p, const float* g, float* m, float* v, int64_t n, float beta1, float beta2, float eps,
                float step_size, float bc2_sqrt, hipStream_t st) {
  if (n <= 0) return 0;
  hipLaunchKernelGGL(k_adam, dim3(nblk(n, 256)), dim3(256), 0, st, p, g, m, v, n, beta1, beta2, eps, step_size,
                     bc2_sqrt);
  return hip_status(hipGetLastError());
}

}  // namespace pnr
