// pnr_internal.h -- shared constants, packed-weight layout and launch helpers of libpnr.so.
//
// MLP = the iMAP* decoder of src/conv_onet/models/decoder.py:91-203 under
// src/conv_onet/config.py:29-31: Fourier(3->93, sin) -> 93->256 -> 3x(256->256) -> 256->4,
// ReLU after every hidden layer, no skips, no output activation.
//
// Execution model of the MLP kernels (see DESIGN.md "MLP kernel"): one wave owns 32 points,
// the point index sits on the MFMA column (lane & 31), the hidden units sit in registers.
// A hidden activation h (256 x 32 points) is 8 accumulator tiles of v_mfma_f32_32x32x2_f32:
//   lane l = 32*hh + j holds, in tile t, register r:  unit 32*t + perm(r,hh), point j
//   perm(r,hh) = (r&3) + 8*(r>>2) + 4*hh                       (gfx950 32x32 C/D layout)
// The NEXT layer consumes that accumulator directly as its B operand (k-step r of tile t uses
// register r: lane half hh supplies k = 32t + perm(r,hh)), so activations never leave the
// registers.  The weights (A operand) are pre-permuted on the device into exactly the lane
// order each MFMA needs and streamed through LDS in 32 KiB chunks by global_load_lds.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/pnr.h"

namespace pnr {

constexpr int kHidden = 256;
constexpr int kFourier = 93;     // decoder.py:129
constexpr int kFourierPad = 96;  // 3 tiles of 32
constexpr int kTiles = kHidden / 32;
constexpr int kChunkFloats = 8192;       // one 32 KiB LDS chunk = 8 tiles x 16 k-steps x 64 lanes
constexpr int kSmallChunkFloats = 1024;  // output layer: 1 tile x 16 k-steps x 64 lanes

// ---- packed image offsets (floats) -------------------------------------------------------
// forward A images: [chunk kc][tile t][rq][lane][4]
constexpr int64_t kOffL0F = 0;                                   // 3 chunks
constexpr int64_t kOffL1F = kOffL0F + 3 * kChunkFloats;          // 8 chunks each
constexpr int64_t kOffL2F = kOffL1F + 8 * kChunkFloats;
constexpr int64_t kOffL3F = kOffL2F + 8 * kChunkFloats;
constexpr int64_t kOffOF = kOffL3F + 8 * kChunkFloats;           // 8 small chunks
// bias images: [tile][rq][lane][4]
constexpr int64_t kBiasFloats = kTiles * 4 * 64 * 4;             // 8192
constexpr int64_t kOffB0 = kOffOF + 8 * kSmallChunkFloats;
constexpr int64_t kOffB1 = kOffB0 + kBiasFloats;
constexpr int64_t kOffB2 = kOffB1 + kBiasFloats;
constexpr int64_t kOffB3 = kOffB2 + kBiasFloats;
constexpr int64_t kOffBO = kOffB3 + kBiasFloats;                 // [rq][lane][4] 1024
constexpr int64_t kOffFB = kOffBO + 1024;                        // Fourier B padded [3][96]
// backward (transposed) A images
constexpr int64_t kOffOT = kOffFB + 3 * kFourierPad;             // Wo^T: [tile][lane][4] 2048
constexpr int64_t kOffL3T = kOffOT + 2048;                       // W3^T: 8 chunks
constexpr int64_t kOffL2T = kOffL3T + 8 * kChunkFloats;
constexpr int64_t kOffL1T = kOffL2T + 8 * kChunkFloats;
constexpr int64_t kL0TChunkFloats = 3 * 4 * 64 * 4;              // 3 out tiles: 3072
constexpr int64_t kOffL0T = kOffL1T + 8 * kChunkFloats;          // W0^T: 8 chunks of 3072
constexpr int64_t kPackedFloats = kOffL0T + 8 * kL0TChunkFloats;

// ---- fc_c image (neural-point feature injection, decoder.py:122-125,196-197), separate buffer --
// forward  CF_l: [t][rq][lane][4], 8 out tiles x one 32-channel input tile (one LDS chunk)
// bias     CB_l: [t][rq][lane][4] (like the hidden bias images)
// backward CT_l: [kc][rq][lane][4], Wc_l^T: one 32-channel out tile x 8 unit tiles (one LDS chunk)
constexpr int kCDim = PNR_C_DIM;
constexpr int64_t kOffCF = 0;
constexpr int64_t kOffCB = 4 * kChunkFloats;
constexpr int64_t kOffCT = 8 * kChunkFloats;
constexpr int64_t kFcPackedFloats = 12 * kChunkFloats;

__host__ __device__ inline int perm(int r, int hh) { return (r & 3) + 8 * (r >> 2) + 4 * hh; }

// Device views of the 11 reference tensors (src/conv_onet/models/decoder.py state_dict order).
struct RawParams {
  const float* p[PNR_N_PARAMS];
  // p[i] for a per-thread i without the private-memory copy of the array a dynamic index makes
  __host__ __device__ __forceinline__ const float* at(int i) const {
    const float* r = p[0];
#pragma unroll
    for (int k = 1; k < PNR_N_PARAMS; ++k) r = i == k ? p[k] : r;
    return r;
  }
};

// Where the MLP reads its points from.
enum PointMode : int {
  kPtsF64 = 0,      // explicit float64 points (eval_points)
  kPtsF32 = 1,      // explicit float32 points (MLP.forward on f32 / masked in f32)
  kRaysZ64 = 2,     // p = o + d * z, z float64 (render_batch_ray)
  kRaysZ32 = 3,     // p = o + d * z, z float32 (regulation)
  kPtsX4 = 4,       // float4 (x, y, z, inside) rows written by the ray kernels of the map pass (k_map_pts,
                    // k_pdf): the point and its bound test already evaluated in the reference's dtype
  kMapRows = 5,     // the map pass's launch-A rows formed in the forward itself (map_row_point; k_mlp_fwd16w
                    // only): k_map_pts fused into the MLP launch
};

// Launch A of the map pass (pnr_map_fwd / pnr_map_step): row e < n S is regulation sample e % S of ray
// e / S (Renderer.regulation, Renderer.py:284-298: float32 z in [0, 0.85 gt], jittered), rows
// [pr, pr + n S) the coarse samples (Renderer.py:86-116, 157-179: near = 0.01 gt, far = the ray's box
// exit + 0.01 clamped to [0, far clamp], float64 z and points), every other row the zero point outside
// the bound.  k_map_pts evaluates it per row into the kPtsX4 rows; with kMapRows the forward does.
struct MapRowsArgs {
  const float* ro;
  const float* rd;
  const float* gt;
  const float* t_rand;  // (n, S) regulation jitter
  const float* gmax;    // far clamp (device), used unless far_mode == 1
  int64_t n_rays, pr;
  double* zc;           // (n, S) coarse z out
  double* far_out;      // (n) per-ray far out, or null
  double bound[6];
  double far_clamp;
  int far_mode, lindisp, n_samples;
  float t_vals[PNR_MAX_SAMPLES];
};
__device__ __forceinline__ void map_row_point(const MapRowsArgs& m, int64_t e, bool write, float& x0, float& x1,
                                              float& x2, bool& inside) {
#pragma clang fp contract(off)  // (render.hip's rule: the reference's unfused float / double arithmetic)
  auto mx = [](double a, double b) { return (a != a || b != b) ? NAN : (a > b ? a : b); };
  auto mn = [](double a, double b) { return (a != a || b != b) ? NAN : (a < b ? a : b); };
  const int S = m.n_samples;
  x0 = x1 = x2 = 0.f;
  inside = false;
  if (e < m.n_rays * S) {  // regulation (k_reg_z, load_point<kRaysZ32>)
    const int64_t n = e / S;
    const int s = (int)(e - n * S);
    const float far = m.gt[n] * 0.85f;
    auto z0 = [&](int k) { return (0.0f * (1.f - m.t_vals[k])) + far * m.t_vals[k]; };
    const float zs = z0(s);
    const float lower = s > 0 ? .5f * (zs + z0(s - 1)) : zs;
    const float upper = s < S - 1 ? .5f * (z0(s + 1) + zs) : zs;
    const float z = lower + (upper - lower) * m.t_rand[e];
    x0 = m.ro[n * 3 + 0] + m.rd[n * 3 + 0] * z;
    x1 = m.ro[n * 3 + 1] + m.rd[n * 3 + 1] * z;
    x2 = m.ro[n * 3 + 2] + m.rd[n * 3 + 2] * z;
    inside = (x0 < (float)m.bound[1]) && (x0 > (float)m.bound[0]) && (x1 < (float)m.bound[3]) &&
             (x1 > (float)m.bound[2]) && (x2 < (float)m.bound[5]) && (x2 > (float)m.bound[4]);
  } else if (e >= m.pr && e < m.pr + m.n_rays * S) {  // render coarse (k_coarse_z, load_point<kRaysZ64>)
    const int64_t q = e - m.pr;
    const int64_t n = q / S;
    const int s = (int)(q - n * S);
    double fb = 0.0;
    for (int a = 0; a < 3; ++a) {
      const double o = (double)m.ro[n * 3 + a], d = (double)m.rd[n * 3 + a];
      const double t0 = (m.bound[2 * a] - o) / d;
      const double t1 = (m.bound[2 * a + 1] - o) / d;
      const double tm = mx(t0, t1);
      fb = a == 0 ? tm : mn(fb, tm);
    }
    fb = fb + 0.01;
    const double hi = m.far_mode == 1 ? m.far_clamp : (double)(*m.gmax);
    double far = fb != fb ? fb : (fb < 0.0 ? 0.0 : fb);  // clamp(min=0)
    far = far != far ? far : (far > hi ? hi : far);
    const float nearf = m.gt[n] * 0.01f;
    if (write && s == 0 && m.far_out) m.far_out[n] = far;
    const float t = m.t_vals[s];
    double zz;
    if (!m.lindisp) {
      zz = (double)(nearf * (1.f - t)) + far * (double)t;
    } else {
      zz = 1.0 / ((double)((1.f / nearf) * (1.f - t)) + (1.0 / far) * (double)t);
    }
    if (write) m.zc[q] = zz;
    const double q0 = (double)m.ro[n * 3 + 0] + (double)m.rd[n * 3 + 0] * zz;
    const double q1 = (double)m.ro[n * 3 + 1] + (double)m.rd[n * 3 + 1] * zz;
    const double q2 = (double)m.ro[n * 3 + 2] + (double)m.rd[n * 3 + 2] * zz;
    inside = (q0 < m.bound[1]) && (q0 > m.bound[0]) && (q1 < m.bound[3]) && (q1 > m.bound[2]) && (q2 < m.bound[5]) &&
             (q2 > m.bound[4]);
    x0 = (float)q0;
    x1 = (float)q1;
    x2 = (float)q2;
  }
}
MapRowsArgs map_rows_args(const pnr_render_params& prm, const float* ro, const float* rd, const float* gt,
                          const float* t_rand, const float* gmax, int64_t n, int64_t pr, double* zc, double* far_out);

struct PointSrc {
  const void* pts;      // kPtsF64/kPtsF32: (P,3)
  const float* rays_o;  // ray modes: (N,3)
  const float* rays_d;
  const void* z;        // ray modes: (N, spr) float64 or float32, point p -> ray p / spr
  int32_t spr;          // samples per ray
  int32_t use_bound;
  double bound[6];
};

// Point p of a launch as the float32 MLP input (x0,x1,x2) plus the bound test.  Reference:
// pts = o + d * z in float64 (Renderer.py:177-179) or float32 (regulation, :296-298); strict
// bound mask (Renderer.py:43-46) in the points' dtype; MLP input p.float() (decoder.py:189).
template <int MODE>
__device__ __forceinline__ void load_point(const PointSrc& s, int64_t p, float& x0, float& x1, float& x2,
                                           bool& inside) {
#pragma clang fp contract(off)
  if (MODE == kPtsF64 || MODE == kRaysZ64) {
    double q0, q1, q2;
    if (MODE == kPtsF64) {
      const double* pp = reinterpret_cast<const double*>(s.pts) + p * 3;
      q0 = pp[0]; q1 = pp[1]; q2 = pp[2];
    } else {
      const int64_t ray = p / s.spr;
      const double z = reinterpret_cast<const double*>(s.z)[p];
      // torch: rays_o[...,None,:] + rays_d[...,None,:] * z[...,:,None], promoted to float64
      q0 = (double)s.rays_o[ray * 3 + 0] + (double)s.rays_d[ray * 3 + 0] * z;
      q1 = (double)s.rays_o[ray * 3 + 1] + (double)s.rays_d[ray * 3 + 1] * z;
      q2 = (double)s.rays_o[ray * 3 + 2] + (double)s.rays_d[ray * 3 + 2] * z;
    }
    inside = true;
    if (s.use_bound)
      inside = (q0 < s.bound[1]) && (q0 > s.bound[0]) && (q1 < s.bound[3]) && (q1 > s.bound[2]) &&
               (q2 < s.bound[5]) && (q2 > s.bound[4]);
    x0 = (float)q0; x1 = (float)q1; x2 = (float)q2;
  } else if (MODE == kPtsX4) {
    const float4 v = reinterpret_cast<const float4*>(s.pts)[p];
    x0 = v.x; x1 = v.y; x2 = v.z;
    inside = v.w != 0.f;
  } else {
    if (MODE == kPtsF32) {
      const float* pp = reinterpret_cast<const float*>(s.pts) + p * 3;
      x0 = pp[0]; x1 = pp[1]; x2 = pp[2];
    } else {
      const int64_t ray = p / s.spr;
      const float z = reinterpret_cast<const float*>(s.z)[p];
      x0 = s.rays_o[ray * 3 + 0] + s.rays_d[ray * 3 + 0] * z;
      x1 = s.rays_o[ray * 3 + 1] + s.rays_d[ray * 3 + 1] * z;
      x2 = s.rays_o[ray * 3 + 2] + s.rays_d[ray * 3 + 2] * z;
    }
    inside = true;
    if (s.use_bound)  // a float32 tensor compared with a 0-dim float64 tensor compares in float32
      inside = (x0 < (float)s.bound[1]) && (x0 > (float)s.bound[0]) && (x1 < (float)s.bound[3]) &&
               (x1 > (float)s.bound[2]) && (x2 < (float)s.bound[5]) && (x2 > (float)s.bound[4]);
  }
}

// Activation save area for training, POINT-major (row p = one point), ld = total points
// (multiple of 128; padded points hold finite activations of x = 0 and get zero gradient).
// fp32, except h1..h3 of the 16-point-wave f16x3 forward (f16 hi / lo parts: hsave_is_split below).
struct SaveArgs {
  float* eP;       // [ld][96]        Fourier features sin(x@B)
  float* hP;       // [4][ld][256]    h1..h4
  float4* xP;      // [ld]            (x0, x1, x2, inside ? 1 : 0), f32 MLP input
  uint4* masks;    // [4][ld/32][64 lanes] ReLU bit words of h1..h4 (mlp.hip save_mask)
  int64_t ld;
  int64_t p0;      // first point (row) of this launch (multiple of 128)
};

// Neural-point feature injection for the MLP kernels (nullptr fcw = reference decoder).
struct FeatArgs {
  const float* fcw;  // fc_c image (kFcPackedFloats)
  const float* c;    // forward: (rows,32) features, row p of the launch = point p
};
int launch_mlp_fwd(const float* packed, const PointSrc& src, int mode, int64_t P, float* raw,
                   const SaveArgs* save, hipStream_t st, const FeatArgs* feat = nullptr);

struct BwdArgs {
  const float* g_out;  // (P,4) dL/draw, sigma channel already zeroed where masked
  const uint4* masks;  // [4][ld/32][64]
  const float4* xP;    // [ld] saved MLP inputs
  float* dP;           // [4][ld_d][256]  delta1..delta4, point-major, chunk-local rows
  float* gargP;        // [ld_d][96]      dL/d(x@B) (pre-sin argument)
  float* g_x;          // (P,3) dL/dx or nullptr
  int64_t ld;          // rows of the saved activations
  int64_t p0;          // first saved row handled by this launch
  int64_t ld_d;        // rows of the delta buffers (chunk size)
  // feature injection (fcw != nullptr): dL/dh_l before the ReLU mask (for dWc_l = gH_l^T c) and
  // dL/dc = sum_l Wc_l^T dL/dh_l
  const float* fcw;
  float* gH;           // [4][ld_d][256]
  float* g_c;          // [C][32] chunk-local rows
};
int launch_mlp_bwd(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st);
// f16x3 delta chain (mlp16_bwd.hip, per-point scaled): same arguments; every precision but
// PNR_PREC_FP32
int launch_mlp_bwd_bf(const float* packed, const BwdArgs& a, int64_t P, hipStream_t st);

int launch_pack(const RawParams& rp, float* packed, hipStream_t st);
// every image (fp32, 16-bit forward, delta chain, raw table) in two launches (mlp16_pack.hip)
int launch_pack_all(const RawParams& rp, float* packed, hipStream_t st, int flags = 0);  // PNR_PACK_* flags
// float offset of Wo [4][256] fp32 in the packed buffer (the raw table's copy, mlp16.h kRawWo)
int64_t packed_raw_wo_offset();
int64_t packed_raw_fb_offset();  // the raw table's Fourier B [3][96] (f16x3 path: no fp32 image)
int launch_fc_pack(const float* const* fc, float* out, hipStream_t st);

// bf16 split forward (mlp_bf.hip): images appended to the fp32 images in the same buffers
int64_t packed_floats_all();
int64_t fc_packed_floats_all();

int launch_fc_pack_all(const float* const* fc, float* out, hipStream_t st, int flags = 0);  // fp32 + 16-bit images, 2 launches
// prec = PNR_PREC_BF16X3 / PNR_PREC_BF16 / PNR_PREC_F16X3
// status: PNR_STATUS_* bits ORed in on the device (f16 range check of F16X3), or null
int launch_mlp_fwd_bf(int prec, const float* packed, const PointSrc& src, int mode, int64_t P, float* raw,
                      const SaveArgs* save, hipStream_t st, const FeatArgs* feat = nullptr,
                      uint32_t* status = nullptr, const MapRowsArgs* mr = nullptr);
// mode kMapRows is served (the forward runs k_mlp_fwd16w): f16x3 without the feature branch
bool fwd_map_rows_ok(int prec, const FeatArgs* feat);
// Format of a save area's h1..h3 (host-side record keyed by SaveArgs::hP, set by every forward that
// saves activations): fp32, or the f16 hi / lo parts the 16-point-wave forward stores (mlp16w.h
// kSplitSave) -- the backward picks its weight-gradient B staging from it and refuses a split save
// area on the fp32 path.  (Host order = stream order, also under graph capture.)
bool fwd_saves_split(int prec, const FeatArgs* feat);  // mlp16_pack.hip: the dispatch's own rule
void hsave_set_split(const float* hP, bool split);
bool hsave_is_split(const float* hP);
// forward dispatch on PNR_PREC_*
inline int mlp_fwd(int prec, const float* packed, const PointSrc& src, int mode, int64_t P, float* raw,
                   const SaveArgs* save, hipStream_t st, const FeatArgs* feat = nullptr,
                   uint32_t* status = nullptr, const MapRowsArgs* mr = nullptr) {
  if (save && save->hP) hsave_set_split(save->hP, prec != PNR_PREC_FP32 && fwd_saves_split(prec, feat));
  if (prec == PNR_PREC_FP32) return mode == kMapRows ? PNR_E_ARG : launch_mlp_fwd(packed, src, mode, P, raw, save, st, feat);
  return launch_mlp_fwd_bf(prec, packed, src, mode, P, raw, save, st, feat, status, mr);
}

// ---- neural-point gather (points.hip) --------------------------------------------------------
// index buffer layout (pnr_points_index_bytes): cell_start[T+1] | count[T] | bucket[M] | slot[M]
// | scan partials | sorted float4[M] (x, y, z, original index bits) | hdr int4[T] | occupancy bits
struct IndexView {
  int32_t* start;
  int32_t* count;
  int32_t* bucket;
  int32_t* slot;
  int32_t* partial;
  float4* sorted;  // bucket-sorted points, each bucket ordered by half-cell (sub-cell) index
  float4* tmp;     // bucket-scattered points before the sub-cell order (build scratch)
  int4* hdr;       // [T] {start, end, cell key lo, key hi | collision bit}
  int4* sub;       // [T] 8 x u16: end offsets of sub-cells 0..7 in the bucket (0xFFFF last: unordered)
  uint32_t* occ;   // occupancy filter (points.hip k_occ_mark)
  int64_t occ_words;
  int64_t T;
};
IndexView index_view(void* base, int64_t M, int32_t bits, size_t* bytes);
int launch_points_build(const pnr_points& pts, hipStream_t st);
// c rows [0, rows): points [0, P) gathered, rows [P, rows) zeroed
// ws: gather_workspace_bytes(P) (work list of the two-pass gather)
size_t gather_workspace_bytes(int64_t P);
int launch_gather(const pnr_points& pts, const PointSrc& src, int mode, int64_t P, int64_t rows, float* c,
                  int32_t* idx, float* w, void* ws, size_t ws_bytes, hipStream_t st);
// g_c (P,32) -> g_feats (+=), g_p (P,3): `gp_accum` adds into g_p instead of writing it;
// positions come from xP (float4 rows, MLP inputs) when non-null, else from src
int launch_gather_bwd(const pnr_points& pts, const PointSrc* src, int mode, const float4* xP, int64_t P,
                      const int32_t* idx, const float* w, const float* c, const float* g_c, float* g_p,
                      bool gp_accum, void* ws, size_t ws_bytes, hipStream_t st);
// backward workspace: work list + control block + (feats) int64 feature accumulators [M][32]
size_t gather_bwd_workspace_bytes(int64_t P, int64_t M, bool feats);
// 64-bit atomic instructions issued by the last backward on `ws` (synchronises st)
int gather_bwd_atomics(const void* ws, int64_t P, int64_t M, unsigned long long* n, hipStream_t st);

// weight-gradient GEMM shapes (wgrad.hip): C[MA][NB] += A[K][WA]^T B[K][WB]
enum WgradKind : int {
  kWgradHidden = 0, kWgradFirst = 1, kWgradOut = 2, kWgradFourier = 3, kWgradFc = 4,
  kWgradOutDelta = 5,  // split precisions: dW3 = delta4^T h3 with delta4 rebuilt from g_out (WgradSyn)
  kWgradFirstX = 6,    // split precisions: dW0 = delta1^T e with e = sin(x@B) recomputed (WgradSyn xP, fb)
  kWgradFcOut = 7      // split precisions: dWc_3 = (dL/dh4)^T c with dL/dh4 = Wo^T g_out rebuilt (WgradSyn g_out, wo)
};
// kWgradOutDelta: delta4 = (Wo^T g_out) * [h4 > 0] is not stored by the delta chain; the GEMM
// rebuilds it per element from the chunk's g_out rows, the forward's h4 mask words and Wo
struct WgradSyn {
  const float4* g_out;  // [K] chunk-local
  const uint4* masks;   // layer-4 mask words (SaveArgs::masks + 3 x ld / 32 x 64)
  int64_t mgrp0;        // saved row of A row 0, / 32
  const float* wo;      // Wo [4][256] fp32
  const float4* xP;     // kWgradFirstX: saved inputs of the chunk rows
  const float* fb;      // kWgradFirstX: Fourier B padded [3][96] (the raw table copy, packed_raw_fb_offset)
  // every kind: per-workgroup partial tiles (wgrad_part_floats + wgrad_part_bias_floats of scratch),
  // added into C / bias in a fixed order by k_part_reduce -- no float atomics, deterministic
  float* part;
  float* part_bias;
  // kWgradHidden / kWgradFirstX with the feature branch: A is the UNMASKED dL/dh_l (the delta chain
  // stores no delta there) and the GEMM applies the forward's ReLU mask words of that layer itself
  const uint4* amasks;  // mask words of h_l's layer (SaveArgs::masks + (l - 1) x ld / 32 x 64) or null
  // GEMMs that will share one grouped launch (launch_wgrad16_group), 0 = a launch of its own (see
  // wgrad16_prepare's grid rule)
  int group_jobs;
  // the group's summed per-tile cost weights (wgrad16_job_weight): a GEMM kind that costs less per
  // tile gets more tiles per workgroup, so the grouped launch's workgroups finish together
  // CUs left to the grouped launch's skinny jobs (dWo / dB) when the GEMMs are sized to fill the chip once
  int reserve_cus;
  float group_weight;
  // kWgradHidden / kWgradOutDelta: B (h1..h3) saved as f16 hi / lo parts (hsave_is_split)
  int bsplit;
  // non-null c: the job also runs the fc_c GEMM of its layer on its A tiles (FC): dWc += A^T c,
  // dbc += colsum(A), A = dL/dh_l unmasked; its reduction goes to wgrad16_prepare's *red2
  const float* fc_c;
  float* fc_C;
  float* fc_bias;
};
// relative cost per 32-point tile of a split weight-gradient GEMM kind in a grouped launch (measured
// one job per launch at its grouped grid, PNR_WGRAD_SPLIT=1: room0 and C3 batches)
float wgrad16_job_weight(int kind, bool masked);
// Arguments of one split weight-gradient GEMM (wgrad16.hip k_wgrad16)
struct WxArgs {
  const float* A;      // [K][256]
  const float* B;      // [kb_rows][WB]
  int nb;              // valid columns of B (columns of C)
  int64_t K;           // multiple of 32 (rows [real K, K) of A exist and are zero)
  int64_t kb_rows;     // rows of B that exist (reads clamp to the last one: A is zero there)
  int64_t ks;          // points per workgroup (multiple of 32)
  float* C;
  int64_t ldc;
  float* bias;
  // SYN (dW3 = delta4^T h3): A is not read but rebuilt per element from the rank-4 product
  // delta4 = (Wo^T g_out) * [h4 > 0] -- the forward's ReLU mask words of h4 and the tile's g_out
  const float4* g_out;   // [K] chunk-local rows (zero past the real points)
  const uint4* masks;    // layer-4 mask words [ld / 32][64] (k_mlp_fwd16 layout)
  int64_t mgrp0;         // mask group of A row 0 (saved row / 32)
  const uint4* amasks;   // MSK: mask words of A's layer (same layout as masks)
  const float* wo;       // Wo [4][256] fp32
  // FOUR (dW0 = delta1^T e): B = e = sin(x@B) is not read but recomputed from the saved inputs, by
  // the forward's own arithmetic (bit-identical e)
  const float4* xP;      // [K] saved MLP inputs (x0, x1, x2, inside), chunk rows
  const float* fb;       // Fourier B padded [3][96]
  float* part;           // non-null: [grid][256][NTB 32] partial tiles + part_bias [grid][256]
  float* part_bias;      //   (plain stores; k_wgrad_reduce sums them into C / bias)
  // FC (feature branch, wgrad16.hip): the fc_c GEMM dWc_l = (dL/dh_l)^T c on the same A tiles -- A
  // unmasked there -- into a second partial region ([grid][256][32] + [grid][256])
  const float* cB;       // c rows [K][32], chunk-local
  float* part2;
  float* part_bias2;
};

// a prepared GEMM of a grouped launch (wgrad16_prepare -> launch_wgrad16_group)
struct Wgrad16Job {
  WxArgs a;
  int var;   // kernel variant (wgrad16.hip kVar*)
  int nwg;   // workgroups (split-K)
};
constexpr int kMaxGemmJobs = 10;  // 4 hidden + 4 fc_c GEMMs + the skinny dWo / dB
// per-tile cost of a fused fc_c GEMM (FC) relative to a hidden GEMM: its A stream comes with the main
// GEMM's (wgrad16_prepare's grid sizing)
constexpr float kWgradFcFusedWeight = 0.22f;
constexpr int kWgradMaxWg = 512;    // fp32 k_wgrad grid cap
constexpr int kWgrad16MaxWg = 256;  // split k_wgrad16 grid cap
constexpr int kSkinnyMaxWg = 1024;  // k_wgrad_skinny grid cap
// split backward: every GEMM of a chunk keeps its own partial region until ONE reduce launch adds them
// all (W3 / W2 / W1 256 x 256, W0 256 x 96, fc_c 4 x 256 x 32, Wo 4 x 256, B 3 x 93)
// Workgroup counts of one chunk of C points (upper bounds of the grids wgrad16_prepare, skinny_blocks
// and wgrad.hip pick_ks choose for K = C), from which the partial scratch is sized
__host__ __device__ constexpr int64_t wgrad16_nwg_max(int64_t C) {
  return ((C + 31) / 32 + 7) / 8 < 4 ? 4 : (((C + 31) / 32 + 7) / 8 > kWgrad16MaxWg ? kWgrad16MaxWg : ((C + 31) / 32 + 7) / 8);
}
__host__ __device__ constexpr int64_t skinny_nwg_max(int64_t C) {
  return (C + 255) / 256 < kSkinnyMaxWg ? (C + 255) / 256 : kSkinnyMaxWg;
}
__host__ __device__ constexpr int64_t wgrad32_nwg_max(int64_t C) {
  return (C + 255) / 256 < kWgradMaxWg ? (C + 255) / 256 : kWgradMaxWg;
}
constexpr int64_t wgrad_part_floats(int64_t C) {
  return wgrad16_nwg_max(C) * 256 * (3 * 256 + 96 + 4 * 32) + skinny_nwg_max(C) * (4 * 256 + 3 * 93) >
                 wgrad32_nwg_max(C) * 256 * 256
             ? wgrad16_nwg_max(C) * 256 * (3 * 256 + 96 + 4 * 32) + skinny_nwg_max(C) * (4 * 256 + 3 * 93)
             : wgrad32_nwg_max(C) * 256 * 256;
}
constexpr int64_t wgrad_part_bias_floats(int64_t C) {
  return wgrad16_nwg_max(C) * 256 * 8 + skinny_nwg_max(C) * 4 > wgrad32_nwg_max(C) * 256
             ? wgrad16_nwg_max(C) * 256 * 8 + skinny_nwg_max(C) * 4
             : wgrad32_nwg_max(C) * 256;
}
// C[r][c] += sum_g part[g][r pw + c] (r < nr, c < nb), bias[r] += sum_g pbias[g][r]: fixed order
int launch_part_reduce(const float* part, const float* pbias, int nwg, int nr, int pw, int nb, float* C, int64_t ldc,
                       float* bias, hipStream_t st);
// a deferred reduction (the GEMM launchers fill it instead of launching k_part_reduce when given one)
struct ReduceJob {
  const float* part;
  const float* pbias;
  int nwg, nr, pw, nb;
  float* C;
  int64_t ldc;
  float* bias;
  int overwrite = 0;  // 1: C / bias = the sum (+ 0, as into zeroed gradients) instead of += the sum
  int64_t part_floats() const { return (int64_t)nwg * nr * pw; }
  int64_t bias_floats() const { return (int64_t)nwg * nr; }
};
constexpr int kMaxReduceJobs = 12;
// every job's reduction in ONE launch (blocks of a job follow the previous job's)
int launch_part_reduce_multi(const ReduceJob* jobs, int n, hipStream_t st);
int launch_wgrad(int kind, const float* A, int ma, const float* B, int nb, int64_t K, float* C, int64_t ldc,
                 float* bias, float* part, float* part_bias, hipStream_t st);
// split precisions (wgrad16.hip): kWgradHidden / kWgradFirst / kWgradFc as f16x3 GEMMs on fp32
// operands (A = deltas or dL/dh [K][256], B = activations / Fourier features / point features
// [K][WB]; B rows >= kb_rows are not read), dWo and dB as fp32 FMA reductions
// defer: non-null = fill the reduction job instead of launching it (launch_part_reduce_multi later)
int launch_wgrad16(int kind, const float* A, const float* B, int64_t K, int64_t kb_rows, float* C, int64_t ldc,
                   float* bias, hipStream_t st, const WgradSyn* syn = nullptr, ReduceJob* defer = nullptr);
// syn->fc_c non-null (kWgradHidden / kWgradFirstX with syn->amasks, or kWgradOutDelta): the job also
// runs its layer's fc_c GEMM (FC); that GEMM's reduction goes to *red2 (partials after the main ones)
int wgrad16_prepare(int kind, const float* A, const float* B, int64_t K, int64_t kb_rows, float* C, int64_t ldc,
                    float* bias, const WgradSyn* syn, Wgrad16Job* job, ReduceJob* red, ReduceJob* red2 = nullptr);
int launch_wgrad16_group(const Wgrad16Job* jobs, int n, hipStream_t st);
// the skinny dWo (out = 1: A = g_out rows, B = h4, + dbo) / dB (out = 0: A = x rows, B = g_arg) as a job
// of a grouped launch
int wgrad_skinny_prepare(int out, const float* A4, const float* B, int64_t K, float* C, float* bias, float* part,
                         float* part_bias, Wgrad16Job* job, ReduceJob* red);
int launch_wgrad_out16(const float* g_out, const float* h4, int64_t K, float* C, float* bias, float* part,
                       float* part_bias, hipStream_t st, ReduceJob* defer = nullptr);
int launch_wgrad_fourier16(const float4* xP, const float* garg, int64_t K, float* C, float* part, hipStream_t st,
                           ReduceJob* defer = nullptr);

inline int hip_status(hipError_t e) { return e == hipSuccess ? 0 : (int)e; }

// compute units of the current device (cached per device; 256 if the query fails): the grid cap of
// the persistent kernels
int device_cu_count();


// Diagnostics: bracket a launch with hipEvents when pnr_timing_enable(1) (capi.cpp).
enum TimedKernel : int {
  kTimeMlpFwd = 0, kTimeMlpBwd = 1, kTimeRay = 2, kTimeWgrad = 3, kTimeGather = 4, kTimeGatherBwd = 5,
  kTimeWgradGroup = 6, kTimeKinds = 7
};
struct TimingScope {
  hipEvent_t a = nullptr, b = nullptr;
  hipStream_t st;
  int kind;
  int64_t units;
  TimingScope(int kind, int64_t units, hipStream_t st);
  ~TimingScope();
};

}  // namespace pnr
