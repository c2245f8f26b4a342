// capi.cpp -- extern "C" entry points of libpnr.so (declared in include/pnr.h).
//
// Orchestrates the kernels of mlp.hip / render.hip for one render_batch_ray call
// (src/utils/Renderer.py:63-203):
//   gt_max -> coarse_z -> MLP(coarse points) -> pdf (importance z) -> MLP(importance points)
//   -> fine (sort + compositing)
// The first pass's 32 points are NOT re-evaluated in the second pass (the reference does,
// Renderer.py:193-196): the same float64 depth gives the same float32 MLP input and the same
// output, so the fine pass gathers them from the coarse results through the sort order.
//
// Backward: compositing backward -> per point dL/draw -> (chunks of <= kBwdChunk points)
// delta chain kernel (mlp.hip) -> split-K weight-gradient MFMA GEMMs (wgrad.hip / wgrad16.hip,
// per-workgroup partial tiles summed in a fixed order: deterministic) -> optional ray gradients.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "pnr_internal.h"

namespace pnr {
int launch_gt_max(const float*, int64_t, float*, hipStream_t);
int launch_coarse_z(const pnr_render_params&, const float*, const float*, const float*, const float*, int64_t,
                    double*, double*, hipStream_t);
int launch_pdf(const pnr_render_params&, const float*, const double*, const float*, int64_t, double*, hipStream_t,
               const float* ro = nullptr, float* x4i = nullptr, int64_t x4i_pad = 0, const float* rawr = nullptr,
               float* sigma = nullptr);
int launch_map_pts(const pnr_render_params&, const float*, const float*, const float*, const float*, const float*,
                   int64_t, int64_t, int64_t, double*, double*, float*, hipStream_t);
int launch_fine(const pnr_render_params&, const float*, const double*, const double*, const float*, const float*,
                int64_t, double*, double*, float*, uint8_t*, hipStream_t);
int launch_fine_bwd(const pnr_render_params&, const float*, const double*, const double*, const float*,
                    const float*, const float4*, const float4*, const uint8_t*, int64_t, const double*,
                    const double*, const float*, float*, float*, float*, float*, int, float*, int, hipStream_t,
                    const float* g_sigma = nullptr, const float4* insr = nullptr, float* gor = nullptr,
                    float* pad2 = nullptr, int np2 = 0);
int launch_ray_grads_f64(const float*, const double*, int, const double*, int, const float*, const float*,
                         const float*, int64_t, float*, float*, hipStream_t);
int launch_ray_grads_f32(const float*, const float*, int, const float*, int64_t, float*, float*, hipStream_t);
int launch_reg_z(const pnr_render_params&, const float*, const float*, int64_t, float*, hipStream_t);
int launch_extract_sigma(const float*, int64_t, float*, hipStream_t);
int launch_gout_sigma(const float*, const float4*, int64_t, int64_t, float*, hipStream_t);
int launch_get_rays(int, int, float, float, float, float, const float*, float*, float*, hipStream_t);
int launch_rays_from_uv(const float*, const float*, int64_t, float, float, float, float, const float*, float*,
                        float*, hipStream_t);
int64_t window_sample_state_bytes();
int launch_window_sample(uint64_t, void*, int64_t, int64_t, int, int, float, float, float, float, const float*,
                         const float*, const float*, int, float*, float*, float*, float*, float*, int64_t*, float*,
                         hipStream_t);
int launch_window_rays(const int64_t*, int64_t, int64_t, int, int, float, float, float, float, const float*,
                       const float*, const float*, float*, float*, float*, float*, hipStream_t);
int launch_adam(float*, const float*, float*, float*, int64_t, float, float, float, float, float, hipStream_t);
int launch_adam_dev(float*, const float*, float*, float*, int64_t, float, float, float, float, const int32_t*,
                    hipStream_t);
int launch_step_advance(int32_t*, hipStream_t);
int launch_adam_multi(float*, const float*, int, const int64_t*, const int64_t*, float* const*, float* const*,
                      const float*, float, float, float, int32_t*, hipStream_t, uint16_t* const* half = nullptr);
int launch_map_loss(const float*, const double*, const float*, const float*, int64_t, float, const float*, int64_t,
                    float, double*, double*, double*, float*, float*, hipStream_t);
int64_t fine_loss_max_rays();
int64_t fine_loss_parts(int64_t n);
int launch_fine_loss(const pnr_render_params&, const float*, const double*, const double*, const float*, const float*,
                     const float4*, const float4*, int64_t, const float*, const float*, float, float, const float*,
                     const float4*, float*, float*, float*, float*, float*, int, float*, int, float*, int, double*,
                     uint32_t*, double*, hipStream_t);

}  // namespace pnr

using namespace pnr;

// CUs left to the skinny dWo / dB jobs of a grouped weight-gradient launch that fills the chip once: 1/16
// (A/B, room0 / C3 graph ms: 1/8 0.521-0.523 / 0.854-0.859, 1/16 0.518-0.519 / 0.833-0.842, 1/32 and
// 1/64 the same as 1/16 within noise, 1/4 0.526)
#ifndef PNR_SKINNY_CU_DIV
#define PNR_SKINNY_CU_DIV 16
#endif
static_assert(PNR_SKINNY_CU_DIV >= 2, "the skinny jobs' CU share leaves the GEMMs at least half the chip");

// ---- diagnostics: kernel timing --------------------------------------------------------------
namespace {
struct TimedLaunch {
  hipEvent_t a, b;
  int64_t units;
};
std::mutex g_tmu;
bool g_timing = false;
std::vector<TimedLaunch> g_tl[kTimeKinds];
}  // namespace

namespace pnr {
int device_cu_count() {
  static std::mutex mu;
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  const int slot = dev < 64 ? dev : 63;
  std::lock_guard<std::mutex> g(mu);
  if (cached[slot] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[slot] = n;
  }
  return cached[slot];
}

TimingScope::TimingScope(int k, int64_t u, hipStream_t s) : st(s), kind(k), units(u) {
  bool on;
  {
    std::lock_guard<std::mutex> g(g_tmu);
    on = g_timing;
  }
  if (!on) return;
  if (hipEventCreate(&a) != hipSuccess || hipEventCreate(&b) != hipSuccess) {
    a = b = nullptr;
    return;
  }
  (void)hipEventRecord(a, st);
}
TimingScope::~TimingScope() {
  if (!a) return;
  (void)hipEventRecord(b, st);
  std::lock_guard<std::mutex> g(g_tmu);
  g_tl[kind].push_back({a, b, units});
}
}  // namespace pnr

namespace {

constexpr size_t kAlign = 256;
constexpr int64_t kBwdChunk = 1 << 22;  // points per delta-chain / GEMM chunk (4.5 KB each)

inline size_t align_up(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }
inline int64_t pad128(int64_t x) { return (x + 127) / 128 * 128; }

// Linear carve of a caller-provided workspace.
struct Carver {
  char* base;
  size_t off = 0;
  explicit Carver(void* b) : base(static_cast<char*>(b)) {}
  template <typename T>
  T* take(size_t count) {
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += align_up(count * sizeof(T));
    return p;
  }
};

bool valid_prm(const pnr_render_params* p) {
  return p && p->n_samples >= 2 && p->n_importance >= 0 && p->n_samples + p->n_importance <= PNR_MAX_SAMPLES &&
         p->far_mode >= 0 && p->far_mode <= 2 && (p->far_mode != 2 || p->far_clamp_dev != nullptr);
}

// Forward workspace of render_batch_ray.
struct RenderWS {
  float* gmax;
  double* z;       // [N*S coarse | N*I importance]
  float* raw;      // float4 per point, same order
  uint8_t* ord;    // [N][64]
  double* far;     // [N]
  int64_t pc_pad;  // first saved column of the importance segment (coarse points padded to 128)
  int64_t ld;      // pc_pad + importance points padded to 128
  SaveArgs save;   // when save_for_backward; columns [0,pc_pad) coarse, [pc_pad, ld) importance
  // neural-point features (prm->points): rows like the save columns
  float* c;        // [ld][32]
  int32_t* nidx;   // [ld][k]
  float* nw;       // [ld][k]
  void* gws;       // gather work list (coarse and importance passes reuse it)
  size_t gws_bytes;
};

// What the forward keeps for the backward: 0 nothing, 1 every activation, 2 the ReLU masks and the
// inputs only (save_for_backward 2: no weight gradients will be asked for; implemented for the
// default PNR_PREC_F16X3 -- the other precisions save everything)
int save_mode(const pnr_render_params* prm) {
  if (!prm->save_for_backward) return 0;
  return (prm->save_for_backward == 2 && prm->precision == PNR_PREC_F16X3) ? 2 : 1;
}

SaveArgs carve_save(Carver& c, int64_t ld, int prec, bool acts = true) {
  SaveArgs s{};
  s.ld = ld;
  s.p0 = 0;
  // mode 2: hP = eP = NULL, which tells the split forward to store masks and inputs only.  e is
  // written by the fp32 forward only (the split dW0 GEMM recomputes it from x), but its region is
  // carved in every precision so that the layout does not depend on the precision: a forward and a
  // backward called with different precisions still find hP / xP / masks at the same offsets
  (void)prec;
  s.eP = acts ? c.take<float>(kFourierPad * ld) : nullptr;
  s.hP = acts ? c.take<float>((size_t)4 * kHidden * ld) : nullptr;
  s.xP = c.take<float4>(ld);
  s.masks = c.take<uint4>((size_t)4 * (ld / 32) * 64);
  return s;
}

RenderWS carve_render(const pnr_render_params* prm, int64_t n, void* ws, size_t* bytes) {
  Carver c(ws);
  RenderWS w{};
  const int64_t P = n * (prm->n_samples + prm->n_importance);
  w.gmax = c.take<float>(1);
  w.z = c.take<double>(P);
  w.raw = c.take<float>(P * 4);
  w.ord = c.take<uint8_t>(n * PNR_MAX_SAMPLES);
  w.far = c.take<double>(n);
  w.pc_pad = pad128(n * prm->n_samples);
  w.ld = w.pc_pad + pad128(n * prm->n_importance);
  if (prm->save_for_backward) w.save = carve_save(c, w.ld, prm->precision, save_mode(prm) == 1);
  if (prm->points) {
    w.c = c.take<float>((size_t)w.ld * kCDim);
    w.nidx = c.take<int32_t>((size_t)w.ld * prm->points->k);
    w.nw = c.take<float>((size_t)w.ld * prm->points->k);
    const int64_t pmax = n * (prm->n_samples > prm->n_importance ? prm->n_samples : prm->n_importance);
    w.gws_bytes = gather_workspace_bytes(pmax);
    w.gws = c.take<char>(w.gws_bytes);
  }
  if (bytes) *bytes = c.off;
  return w;
}

// Backward scratch shared by render and regulation.
struct BwdWS {
  float* g_out;   // [P] float4
  float* g_x;     // [P][3]
  float* g_nrm;   // [N]
  float* dP;      // [4][C][256]
  float* gargP;   // [C][96]
  float* gH;      // [4][C][256]  features only: dL/dh_l
  float* g_c;     // [P][32]      features only: dL/dc
  float* part;    // weight-gradient partial tiles (wgrad16.hip two-phase flush)
  float* part_bias;
  void* gws;      // features only: gather-backward work list
  size_t gws_bytes;
  int64_t C;
};

// wgrad: weight gradients may be asked for (the partial tiles of the weight-gradient GEMMs)
// M: neural points of the call (the gather backward's int64 feature accumulators), 0 without
BwdWS carve_bwd(int64_t P, int64_t n, void* ws, size_t* bytes, bool feat, bool wgrad, int64_t M = 0) {
  Carver c(ws);
  BwdWS b{};
  b.C = P < kBwdChunk ? ((P + 127) / 128) * 128 : kBwdChunk;
  if (b.C < 128) b.C = 128;
  b.g_out = c.take<float>(P * 4);
  b.g_x = c.take<float>(P * 3);
  b.g_nrm = c.take<float>(n);
  b.dP = c.take<float>((size_t)4 * kHidden * b.C);
  b.gargP = c.take<float>(kFourierPad * b.C);
  if (wgrad) {  // sized from the chunk: the GEMM grids of a small backward are small
    b.part = c.take<float>(wgrad_part_floats(b.C));
    b.part_bias = c.take<float>(wgrad_part_bias_floats(b.C));
  }
  if (feat) {
    b.gH = c.take<float>((size_t)4 * kHidden * b.C);
    b.g_c = c.take<float>((size_t)P * kCDim);
    b.gws_bytes = gather_bwd_workspace_bytes(P, M, true);
    b.gws = c.take<char>(b.gws_bytes);
  }
  if (bytes) *bytes = c.off;
  return b;
}
// neural points whose feature gradients the backward accumulates (the gather backward's int64
// accumulators are sized from it): none when no g_feats is asked for (e.g. a camera-only backward)
int64_t n_pts(const pnr_render_params* prm) {
  return prm->points && prm->points->g_feats ? prm->points->n_points : 0;
}

// fc_c side of the backward: image, per-row features and the 8 accumulated fc_c grads
struct FeatBwd {
  const float* fcw;
  const float* c;        // [rows][32], same rows as the saved activations
  float* const* g_fc;    // 8 device pointers or null
};

__global__ void k_fill(float* p, int64_t n, float v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// Store semantics (grads_overwrite) with nothing to store: the weight gradients of an empty batch
// are zero, exactly as autograd's would be (an early return would leave the previous step's values).
int zero_weight_grads(float* const* grads, float* const* g_fc, hipStream_t st) {
  static const int64_t dec_n[PNR_N_PARAMS] = {3 * kFourier, kHidden * kFourier, kHidden, kHidden * kHidden, kHidden,
                                              kHidden * kHidden, kHidden, kHidden * kHidden, kHidden, 4 * kHidden, 4};
  for (int i = 0; grads && i < PNR_N_PARAMS; ++i)
    if (int rc = hip_status(hipMemsetAsync(grads[i], 0, dec_n[i] * sizeof(float), st))) return rc;
  for (int i = 0; g_fc && i < PNR_N_FC_PARAMS; ++i)
    if (int rc = hip_status(hipMemsetAsync(g_fc[i], 0, (i % 2 ? kHidden : kHidden * kCDim) * sizeof(float), st)))
      return rc;
  return PNR_OK;
}

// Shared backward core over P points with saved activations `sv` and dL/draw in b.g_out.
int mlp_backward_core(int prec, const float* packed, const SaveArgs& sv, int64_t P, BwdWS& b, float* const* grads,
                      bool want_gx, hipStream_t st, const FeatBwd* fb = nullptr, bool overwrite = false) {
  const bool split = prec != PNR_PREC_FP32;  // f16x3 delta chain + f16x3 weight-gradient GEMMs
  if (overwrite && (!split || P == 0)) {  // the fp32 GEMMs add into C: store = add into zeroed gradients
    if (int rc = zero_weight_grads(grads, fb ? fb->g_fc : nullptr, st)) return rc;
    overwrite = false;
  }
  for (int64_t p0 = 0; p0 < P; p0 += b.C) {
    const int64_t C = (P - p0) < b.C ? (P - p0) : b.C;
    BwdArgs a;
    a.g_out = b.g_out + p0 * 4;
    a.masks = sv.masks;
    a.xP = sv.xP;
    a.dP = b.dP;
    a.gargP = b.gargP;
    a.g_x = want_gx ? b.g_x + p0 * 3 : nullptr;
    a.ld = sv.ld;
    a.p0 = p0;
    a.ld_d = b.C;
    a.fcw = fb ? fb->fcw : nullptr;
    a.gH = b.gH;
    a.g_c = fb ? b.g_c + p0 * kCDim : nullptr;
    const int64_t hstride = sv.ld * kHidden;  // h_l rows of this chunk: h + l_idx * ld * 256 + p0 * 256
    const int64_t dstride = b.C * kHidden;
    // split precisions: every GEMM of the chunk writes its own partial region, and ONE reduce launch
    // (fixed order per element) adds them all into the gradients
    ReduceJob jobs[kMaxReduceJobs];
    int nj = 0;
    Wgrad16Job gjobs[kMaxGemmJobs];
    int ng = 0;
    float* pp = b.part;
    float* pb = b.part_bias;
    auto took = [&]() {
      pp += jobs[nj].part_floats();
      pb += jobs[nj].bias_floats();
      ++nj;
    };
    const bool want_fc = fb && fb->g_fc;
    int rc = 0;
    // The skinny fp32 GEMMs of the split precisions -- dWo (4x256) += g_out^T h4, dbo += colsum(g_out)
    // and dB (3x93) += x^T g_arg -- are jobs of the grouped weight-gradient launch: its GEMMs are sized to
    // leave them 1/16 of the CUs (PNR_SKINNY_CU_DIV) when they fill the chip once (the Mapper's 1,000-ray batch), so the two
    // bandwidth-bound streams run beside the GEMMs instead of as launches of their own (dWo ahead of the
    // delta chain, dB behind the GEMMs: 30 us of the iteration's critical path).
    const bool skinny_in_group = split && grads;
    // the delta chain: exact fp32 MFMA for PNR_PREC_FP32, f16x3 split MFMA otherwise
    rc = prec == PNR_PREC_FP32 ? launch_mlp_bwd(packed, a, C, st) : launch_mlp_bwd_bf(packed, a, C, st);
    if (rc) return rc;
    if (!grads && !want_fc) {  // no weight gradients (the Tracker's camera-only backward)
    } else if (split) {  // f16x3 GEMMs on the fp32 saves (h / e by k_mlp_fwd16, deltas by k_mlp_bwd16)
      const float* hp = sv.hP + p0 * kHidden;
      // hidden layers: dW_l += delta_{l+1}^T h_l  (W3: delta4.h3, W2: delta3.h2, W1: delta2.h1); delta4
      // is not stored by k_mlp_bwd16 (rank 4: rebuilt from g_out and the h4 masks inside the GEMM).
      // These GEMMs (and the fc_c ones below) are independent: prepared here, launched as one group.
      // PNR_WGRAD_FC_FUSE=1 (experiment, off by default): with both the decoder's and the feature
      // branch's gradients, each layer's fc_c GEMM runs inside the dW GEMM that reads the same dL/dh_l
      // tiles (FC jobs, k_wgrad16_group_fc: the A stream read once).  The fused 256-column jobs do not fit
      // the 256 registers a wave has at two waves per SIMD (36-40 spilled, 76 in the group kernel): the grouped launch took
      // 1.89 ms against 1.00 at C5, C5 3.81-3.85 against 3.02 ms, the neural-point S-map 185 against
      // 154-156 ms (profiles/r06_fc_fuse_ab.txt)
      static const bool fc_fuse_env = getenv("PNR_WGRAD_FC_FUSE") && getenv("PNR_WGRAD_FC_FUSE")[0] == '1';
      const bool fc_fuse = fc_fuse_env && grads && want_fc;
      WgradSyn syn{reinterpret_cast<const float4*>(b.g_out + p0 * 4), sv.masks + 3 * (sv.ld / 32) * 64, p0 / 32,
                   packed + packed_raw_wo_offset(), sv.xP + p0, packed + packed_raw_fb_offset(), pp, pb, nullptr,
                   (grads ? 4 : 0) + (want_fc && !fc_fuse ? 4 : 0),
                   skinny_in_group ? device_cu_count() / PNR_SKINNY_CU_DIV : 0, 0.f};
      syn.bsplit = hsave_is_split(sv.hP) ? 1 : 0;  // h1..h3 as f16 parts (the 16-point-wave forward)
      if (grads)
        syn.group_weight += wgrad16_job_weight(kWgradOutDelta, false) + 2 * wgrad16_job_weight(kWgradHidden, false) +
                            wgrad16_job_weight(kWgradFirstX, false);
      if (fc_fuse) syn.group_weight += 4 * kWgradFcFusedWeight;
      else if (want_fc)
        syn.group_weight += 3 * wgrad16_job_weight(kWgradFc, false) + wgrad16_job_weight(kWgradFcOut, false);
      // with the feature branch k_mlp_bwd16 stores dL/dh_l only: delta_l = dL/dh_l masked in the GEMM
      const bool fmask = fb != nullptr;
      const int64_t mstride = (sv.ld / 32) * 64;
      const float* dsrc = fmask ? b.gH : b.dP;
      // fcl >= 0: fuse the fc_c GEMM of layer fcl (dWc_l += (dL/dh_l)^T c, dbc_l += colsum) into this job
      auto prep = [&](int kind, const float* A, const float* B, float* Cw, int64_t ldc, float* bias,
                      const uint4* amasks, int fcl = -1) {
        if (rc) return;
        syn.part = pp;
        syn.part_bias = pb;
        syn.amasks = amasks;
        syn.fc_c = fcl >= 0 ? fb->c + p0 * kCDim : nullptr;
        syn.fc_C = fcl >= 0 ? fb->g_fc[2 * fcl] : nullptr;
        syn.fc_bias = fcl >= 0 ? fb->g_fc[2 * fcl + 1] : nullptr;
        rc = wgrad16_prepare(kind, A, B, C, C, Cw, ldc, bias, &syn, &gjobs[ng], &jobs[nj], &jobs[nj + 1]);
        syn.amasks = nullptr;
        syn.fc_c = nullptr;
        if (rc == 0) {
          ++ng;
          took();
          if (fcl >= 0) took();
        }
      };
      if (grads) {
        prep(kWgradOutDelta, nullptr, hp + 2 * hstride, grads[7], kHidden, grads[8], nullptr, fc_fuse ? 3 : -1);
        for (int l = 2; l >= 1; --l)
          prep(kWgradHidden, dsrc + l * dstride, hp + (l - 1) * hstride, grads[1 + 2 * l], kHidden,
               grads[2 + 2 * l], fmask ? sv.masks + l * mstride : nullptr, fc_fuse ? l : -1);
        // first layer: dW0 (256x93) += delta1^T e ; db0 -- e = sin(x@B) recomputed from the saved x
        // (k_mlp_fwd16 saves no e)
        prep(kWgradFirstX, dsrc, nullptr, grads[1], kFourier, grads[2], fmask ? sv.masks : nullptr, fc_fuse ? 0 : -1);
      }
      // feature branch: dWc_l (256x32) += (dL/dh_l)^T c ; dbc_l += colsum(dL/dh_l)
      // (dL/dh4 = Wo^T g_out is rank 4: k_mlp_bwd16 does not store it, the dWc_3 GEMM rebuilds it)
      if (want_fc && !fc_fuse)
        for (int l = 0; l < 4; ++l)
          prep(l == 3 ? kWgradFcOut : kWgradFc, b.gH + l * dstride, fb->c + p0 * kCDim, fb->g_fc[2 * l], kCDim,
               fb->g_fc[2 * l + 1], nullptr);
      // the skinny jobs last in the grid: their workgroups take the CUs the GEMMs leave
      if (rc == 0 && skinny_in_group) {
        rc = wgrad_skinny_prepare(1, b.g_out + p0 * 4, hp + 3 * hstride, C, grads[9], grads[10], pp, pb, &gjobs[ng],
                                  &jobs[nj]);
        if (rc == 0) {
          ++ng;
          took();
          rc = wgrad_skinny_prepare(0, reinterpret_cast<const float*>(sv.xP + p0), b.gargP, C, grads[0], nullptr,
                                    pp, pb, &gjobs[ng], &jobs[nj]);
        }
        if (rc == 0) {
          ++ng;
          took();
        }
      }
      // diagnostics (PNR_WGRAD_SPLIT=1): each job as a launch of its own, so a kernel trace times every
      // GEMM kind at its grouped grid (the per-kind costs behind wgrad16_prepare's sizing weights)
      static const bool split_jobs = getenv("PNR_WGRAD_SPLIT") && getenv("PNR_WGRAD_SPLIT")[0] == '1';
      if (rc == 0 && split_jobs) {
        for (int i = 0; i < ng && rc == 0; ++i) rc = launch_wgrad16_group(gjobs + i, 1, st);
      } else if (rc == 0) {
        rc = launch_wgrad16_group(gjobs, ng, st);
      }
    } else if (grads) {
      if (hsave_is_split(sv.hP)) return PNR_E_ARG;  // saved by the f16x3 forward: not fp32 activations
      const float* hp = sv.hP + p0 * kHidden;
      rc = launch_wgrad(kWgradOut, b.g_out + p0 * 4, 4, hp + 3 * hstride, kHidden, C, grads[9], kHidden, grads[10],
                        b.part, b.part_bias, st);
      for (int l = 3; l >= 1 && rc == 0; --l)
        rc = launch_wgrad(kWgradHidden, b.dP + l * dstride, kHidden, hp + (l - 1) * hstride, kHidden, C,
                          grads[1 + 2 * l], kHidden, grads[2 + 2 * l], b.part, b.part_bias, st);
      if (rc == 0)
        rc = launch_wgrad(kWgradFirst, b.dP, kHidden, sv.eP + p0 * kFourierPad, kFourier, C, grads[1], kFourier,
                          grads[2], b.part, b.part_bias, st);
      // Fourier: dB (3x93) += x^T g_arg   (x rows are float4 (x0,x1,x2,inside): 3 of 4 used)
      if (rc == 0)
        rc = launch_wgrad(kWgradFourier, reinterpret_cast<const float*>(sv.xP + p0), 3, b.gargP, kFourier, C,
                          grads[0], kFourier, nullptr, b.part, b.part_bias, st);
    }
    if (rc) return rc;
    // feature branch (fp32 mode; the split mode's fc_c GEMMs ran in the group above)
    if (fb && fb->g_fc && !split) {
      for (int l = 0; l < 4 && rc == 0; ++l)
        rc = launch_wgrad(kWgradFc, b.gH + l * dstride, kHidden, fb->c + p0 * kCDim, kCDim, C, fb->g_fc[2 * l], kCDim,
                          fb->g_fc[2 * l + 1], b.part, b.part_bias, st);
    }
    if (overwrite && p0 == 0)  // the first chunk stores its sums; the later chunks add to them
      for (int i = 0; i < nj; ++i) jobs[i].overwrite = 1;
    if (rc == 0) rc = launch_part_reduce_multi(jobs, nj, st);
    if (rc) return rc;
  }
  return hip_status(hipGetLastError());
}

bool check_params(const float* const* params) {
  if (!params) return false;
  for (int i = 0; i < PNR_N_PARAMS; ++i)
    if (!params[i]) return false;
  return true;
}

}  // namespace

extern "C" {

// the ctypes mirror (pnr/_lib.py) and tests/test_capi.py assume these offsets
static_assert(offsetof(pnr_points, feat_half) == 104 && sizeof(pnr_points) == 112, "pnr_points layout (ABI 6)");
static_assert(offsetof(pnr_render_params, status) == 608 && sizeof(pnr_render_params) == 624 &&
                  offsetof(pnr_render_params, grads_overwrite) == 604,
              "pnr_render_params layout (ABI 7; ABI 11 grads_overwrite in the padding after precision)");
int pnr_abi_version(void) { return PNR_ABI_VERSION; }

int pnr_timing_enable(int on) {
  std::lock_guard<std::mutex> g(g_tmu);
  g_timing = on != 0;
  return PNR_OK;
}

int pnr_timing_read(int kernel, int64_t* launches, double* ms, int64_t* units) {
  if (kernel < 0 || kernel >= kTimeKinds || !launches || !ms || !units) return PNR_E_ARG;
  std::vector<TimedLaunch> v;
  {
    std::lock_guard<std::mutex> g(g_tmu);
    v.swap(g_tl[kernel]);
  }
  double tot = 0.0;
  int64_t u = 0;
  for (auto& t : v) {
    float e = 0.f;
    (void)hipEventSynchronize(t.b);
    if (hipEventElapsedTime(&e, t.a, t.b) == hipSuccess) tot += e;
    u += t.units;
    (void)hipEventDestroy(t.a);
    (void)hipEventDestroy(t.b);
  }
  *launches = (int64_t)v.size();
  *ms = tot;
  *units = u;
  return PNR_OK;
}

const char* pnr_build_info(void) {
  return "libpnr gfx950: fused decoder on fp32 v_mfma_f32_32x32x2_f32 or bf16x3 / bf16 v_mfma_f32_32x32x16_bf16, "
         "LDS-DMA-streamed weights; "
         "thread-per-ray compositing; split-K MFMA weight-gradient GEMMs; spatial-hash neural-point gather";
}

size_t pnr_mlp_packed_floats(void) { return (size_t)packed_floats_all(); }

int pnr_mlp_pack(const float* const* params, float* packed, void* stream) {
  if (!check_params(params) || !packed) return PNR_E_ARG;
  RawParams rp;
  for (int i = 0; i < PNR_N_PARAMS; ++i) rp.p[i] = params[i];
  return launch_pack_all(rp, packed, (hipStream_t)stream);
}

int pnr_mlp_pack2(const float* const* params, float* packed, int32_t flags, void* stream) {
  if (!check_params(params) || !packed || (flags & ~PNR_PACK_F16X3_ONLY)) return PNR_E_ARG;
  RawParams rp;
  for (int i = 0; i < PNR_N_PARAMS; ++i) rp.p[i] = params[i];
  return launch_pack_all(rp, packed, (hipStream_t)stream, flags);
}

int pnr_eval_points(const float* packed, const double* p, int64_t P, const double* bound6, float* raw_out,
                    int32_t precision, void* stream) {
  if (!packed || P < 0 || (P > 0 && (!p || !raw_out))) return PNR_E_ARG;
  PointSrc s{};
  s.pts = p;
  s.use_bound = bound6 != nullptr;
  if (bound6) memcpy(s.bound, bound6, sizeof(s.bound));
  return mlp_fwd(precision, packed, s, kPtsF64, P, raw_out, nullptr, (hipStream_t)stream);
}

int pnr_eval_points_f32(const float* packed, const float* p, int64_t P, const double* bound6, float* raw_out,
                        int32_t precision, void* stream) {
  if (!packed || P < 0 || (P > 0 && (!p || !raw_out))) return PNR_E_ARG;
  PointSrc s{};
  s.pts = p;
  s.use_bound = bound6 != nullptr;
  if (bound6) memcpy(s.bound, bound6, sizeof(s.bound));
  return mlp_fwd(precision, packed, s, kPtsF32, P, raw_out, nullptr, (hipStream_t)stream);
}

size_t pnr_mlp_train_workspace_bytes(int64_t P) {
  if (P < 0) return 0;
  Carver c(nullptr);
  carve_save(c, pad128(P), PNR_PREC_FP32);
  return c.off;
}

int pnr_mlp_fwd_train(const float* packed, const float* p, int64_t P, float* raw_out, void* ws, size_t ws_bytes,
                      int32_t precision, void* stream) {
  if (!packed || P < 0 || (P > 0 && (!p || !raw_out || !ws))) return PNR_E_ARG;
  if (P == 0) return PNR_OK;
  Carver c(ws);
  SaveArgs sv = carve_save(c, pad128(P), precision);
  if (ws_bytes < c.off) return PNR_E_WORKSPACE;
  PointSrc s{};
  s.pts = p;
  s.use_bound = 0;
  return mlp_fwd(precision, packed, s, kPtsF32, P, raw_out, &sv, (hipStream_t)stream);
}

size_t pnr_mlp_bwd_workspace_bytes(int64_t P) {
  if (P < 0) return 0;
  size_t b = 0;
  carve_bwd(pad128(P), 1, nullptr, &b, false, true);
  return b;
}

int pnr_mlp_bwd(const float* packed, int64_t P, const float* g_raw, float* const* grads, float* g_p, void* ws,
                size_t ws_bytes, void* bwd_ws, size_t bwd_bytes, int32_t precision, void* stream) {
  if (!packed || P < 0 || (P > 0 && (!g_raw || !grads || !ws || !bwd_ws))) return PNR_E_ARG;
  if (P == 0) return PNR_OK;
  for (int i = 0; i < PNR_N_PARAMS; ++i)
    if (!grads[i]) return PNR_E_ARG;
  Carver c(ws);
  SaveArgs sv = carve_save(c, pad128(P), precision);
  size_t bneed = 0;
  BwdWS b = carve_bwd(sv.ld, 1, bwd_ws, &bneed, false, true);
  if (ws_bytes < c.off || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(b.g_out, 0, (size_t)sv.ld * 16, st) != hipSuccess) return (int)hipGetLastError();
  if (hipMemcpyAsync(b.g_out, g_raw, (size_t)P * 16, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  int rc = mlp_backward_core(precision, packed, sv, sv.ld, b, grads, g_p != nullptr, st);
  if (rc) return rc;
  if (g_p && hipMemcpyAsync(g_p, b.g_x, (size_t)P * 12, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  return PNR_OK;
}

size_t pnr_render_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_prm(prm) || n_rays < 0) return 0;
  size_t b = 0;
  carve_render(prm, n_rays, nullptr, &b);
  return b;
}

int pnr_render_fwd(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                   const float* gt_depth, int64_t n, double* depth, double* var, float* rgb, void* workspace,
                   size_t ws_bytes, void* stream) {
  if (!valid_prm(prm) || !packed || n < 0) return PNR_E_ARG;
  if (n == 0) return PNR_OK;
  if (!rays_o || !rays_d || !depth || !var || !rgb || !workspace) return PNR_E_ARG;
  if (prm->points && !prm->points->fc_packed) return PNR_E_ARG;
  if (prm->n_importance > 0 && prm->n_samples < 3) return PNR_E_ARG;
  size_t need = 0;
  RenderWS w = carve_render(prm, n, workspace, &need);
  if (ws_bytes < need) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const int S = prm->n_samples, I = prm->n_importance;
  int rc = 0;
  if (gt_depth && prm->far_mode == 0) rc = launch_gt_max(gt_depth, n, w.gmax, st);
  if (rc) return rc;
  // far_mode 2: the clamp is a device value (k_coarse_z reads it like the batch max of mode 0)
  rc = launch_coarse_z(*prm, rays_o, rays_d, gt_depth, prm->far_mode == 2 ? prm->far_clamp_dev : w.gmax, n, w.z,
                       w.far, st);
  if (rc) return rc;
  PointSrc src{};
  src.rays_o = rays_o;
  src.rays_d = rays_d;
  src.use_bound = 1;
  memcpy(src.bound, prm->bound, sizeof(src.bound));
  src.z = w.z;
  src.spr = S;
  const SaveArgs* sv = prm->save_for_backward ? &w.save : nullptr;
  const pnr_points* pts = prm->points;
  FeatArgs fa{pts ? pts->fc_packed : nullptr, w.c};
  const int K = pts ? pts->k : 0;
  if (pts) {
    rc = launch_gather(*pts, src, kRaysZ64, n * S, w.pc_pad, w.c, sv ? w.nidx : nullptr, sv ? w.nw : nullptr, w.gws,
                       w.gws_bytes, st);
    if (rc) return rc;
  }
  uint32_t* status = reinterpret_cast<uint32_t*>(prm->status);
  rc = mlp_fwd(prm->precision, packed, src, kRaysZ64, n * S, w.raw, sv, st, pts ? &fa : nullptr, status);
  if (rc) return rc;
  double* zi = w.z + n * S;
  float* rawi = w.raw + n * S * 4;
  if (I > 0) {
    rc = launch_pdf(*prm, rays_d, w.z, w.raw, n, zi, st);
    if (rc) return rc;
    src.z = zi;
    src.spr = I;
    SaveArgs s2{};
    if (sv) {
      s2 = *sv;
      s2.p0 = w.pc_pad;
      sv = &s2;
    }
    if (pts) {
      const int64_t o = w.pc_pad;
      rc = launch_gather(*pts, src, kRaysZ64, n * I, w.ld - o, w.c + o * kCDim, sv ? w.nidx + o * K : nullptr,
                         sv ? w.nw + o * K : nullptr, w.gws, w.gws_bytes, st);
      if (rc) return rc;
      fa.c = w.c + o * kCDim;
    }
    rc = mlp_fwd(prm->precision, packed, src, kRaysZ64, n * I, rawi, sv, st, pts ? &fa : nullptr, status);
    if (rc) return rc;
  }
  return launch_fine(*prm, rays_d, w.z, zi, w.raw, rawi, n, depth, var, rgb, w.ord, st);
}

size_t pnr_render_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_prm(prm) || n_rays < 0) return 0;
  size_t b = 0;
  carve_bwd(pad128(n_rays * prm->n_samples) + pad128(n_rays * prm->n_importance), n_rays, nullptr, &b,
            prm->points != nullptr, save_mode(prm) != 2, n_pts(prm));
  return b;
}

int pnr_render_bwd(const pnr_render_params* prm, const float* packed, const float* const* params,
                   const float* rays_o, const float* rays_d, int64_t n, const double* g_depth, const double* g_var,
                   const float* g_rgb, float* const* grads, float* g_rays_o, float* g_rays_d, void* workspace,
                   size_t ws_bytes, void* bwd_ws, size_t bwd_bytes, void* stream) {
  (void)params;
  (void)rays_o;
  if (!valid_prm(prm) || !packed || n < 0 || !prm->save_for_backward) return PNR_E_ARG;
  if (n == 0) {  // store semantics: an empty batch's weight gradients are zero
    if (!prm->grads_overwrite) return PNR_OK;
    if (grads)
      for (int i = 0; i < PNR_N_PARAMS; ++i)
        if (!grads[i]) return PNR_E_ARG;
    return zero_weight_grads(grads, prm->points ? prm->points->g_fc : nullptr, (hipStream_t)stream);
  }
  if (!workspace || !bwd_ws || !rays_d) return PNR_E_ARG;
  if (grads)  // NULL: no decoder weight gradients
    for (int i = 0; i < PNR_N_PARAMS; ++i)
      if (!grads[i]) return PNR_E_ARG;
  // a masks-only forward (save_for_backward 2) kept no activations to form weight gradients from
  if (save_mode(prm) == 2 && (grads || (prm->points && prm->points->g_fc))) return PNR_E_ARG;
  if (prm->need_ray_grads && (!g_rays_o || !g_rays_d)) return PNR_E_ARG;
  size_t need = 0, bneed = 0;
  RenderWS w = carve_render(prm, n, workspace, &need);
  const int S = prm->n_samples, I = prm->n_importance;
  const int64_t ld = w.save.ld;
  const pnr_points* pts = prm->points;
  BwdWS b = carve_bwd(ld, n, bwd_ws, &bneed, pts != nullptr, save_mode(prm) != 2, n_pts(prm));
  if (ws_bytes < need || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  const double* zi = w.z + n * S;
  const float* rawi = w.raw + n * S * 4;
  const int64_t pc = w.pc_pad;
  // dL/draw of every MLP row: the samples' from the compositing backward, zeros on the padding rows
  // [n S, pc) and [pc + n I, ld) (written by the same launch)
  int rc = launch_fine_bwd(*prm, rays_d, w.z, zi, w.raw, rawi, w.save.xP, w.save.xP + pc, w.ord, n,
                           g_depth, g_var, g_rgb, b.g_out, b.g_out + pc * 4, b.g_nrm, b.g_out + n * S * 4,
                           (int)(pc - n * S), b.g_out + (pc + n * I) * 4, (int)(ld - pc - n * I), st);
  if (rc) return rc;
  FeatBwd fb{pts ? pts->fc_packed : nullptr, w.c, pts ? pts->g_fc : nullptr};
  rc = mlp_backward_core(prm->precision, packed, w.save, ld, b, grads, prm->need_ray_grads != 0, st,
                         pts ? &fb : nullptr, prm->grads_overwrite != 0);
  if (rc) return rc;
  if (pts) {  // neural-point features and dL/dp through the gather weights
    rc = launch_gather_bwd(*pts, nullptr, kRaysZ64, w.save.xP, ld, w.nidx, w.nw, w.c, b.g_c,
                           prm->need_ray_grads ? b.g_x : nullptr, true, b.gws, b.gws_bytes, st);
    if (rc) return rc;
  }
  if (prm->need_ray_grads)
    rc = launch_ray_grads_f64(rays_d, w.z, S, zi, I, b.g_x, b.g_x + pc * 3, b.g_nrm, n, g_rays_o, g_rays_d, st);
  return rc;
}

// ---- regulation ---------------------------------------------------------------------------
namespace {
struct RegWS {
  float* z;
  float* raw;
  SaveArgs save;
  float* c;
  int32_t* nidx;
  float* nw;
  void* gws;
  size_t gws_bytes;
};
RegWS carve_reg(const pnr_render_params* prm, int64_t n, void* ws, size_t* bytes) {
  Carver c(ws);
  RegWS w{};
  const int64_t P = n * prm->n_samples;
  w.z = c.take<float>(P);
  w.raw = c.take<float>(P * 4);
  if (prm->save_for_backward) w.save = carve_save(c, pad128(P), prm->precision, save_mode(prm) == 1);
  if (prm->points) {
    w.c = c.take<float>((size_t)pad128(P) * kCDim);
    w.nidx = c.take<int32_t>((size_t)pad128(P) * prm->points->k);
    w.nw = c.take<float>((size_t)pad128(P) * prm->points->k);
    w.gws_bytes = gather_workspace_bytes(P);
    w.gws = c.take<char>(w.gws_bytes);
  }
  if (bytes) *bytes = c.off;
  return w;
}
}  // namespace

size_t pnr_regulation_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_prm(prm) || n_rays < 0) return 0;
  size_t b = 0;
  carve_reg(prm, n_rays, nullptr, &b);
  return b;
}

int pnr_regulation_fwd(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                       const float* gt_depth, const float* t_rand, int64_t n, float* sigma, void* workspace,
                       size_t ws_bytes, void* stream) {
  if (!valid_prm(prm) || !packed || n < 0) return PNR_E_ARG;
  if (n == 0) return PNR_OK;
  if (!rays_o || !rays_d || !gt_depth || !t_rand || !sigma || !workspace) return PNR_E_ARG;
  if (prm->points && !prm->points->fc_packed) return PNR_E_ARG;
  size_t need = 0;
  RegWS w = carve_reg(prm, n, workspace, &need);
  if (ws_bytes < need) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  int rc = launch_reg_z(*prm, gt_depth, t_rand, n, w.z, st);
  if (rc) return rc;
  PointSrc src{};
  src.rays_o = rays_o;
  src.rays_d = rays_d;
  src.use_bound = 1;
  memcpy(src.bound, prm->bound, sizeof(src.bound));
  src.z = w.z;
  src.spr = prm->n_samples;
  const int64_t P = n * prm->n_samples;
  const bool sv = prm->save_for_backward != 0;
  FeatArgs fa{prm->points ? prm->points->fc_packed : nullptr, w.c};
  if (prm->points) {
    rc = launch_gather(*prm->points, src, kRaysZ32, P, pad128(P), w.c, sv ? w.nidx : nullptr, sv ? w.nw : nullptr,
                       w.gws, w.gws_bytes, st);
    if (rc) return rc;
  }
  rc = mlp_fwd(prm->precision, packed, src, kRaysZ32, P, w.raw, sv ? &w.save : nullptr, st,
               prm->points ? &fa : nullptr, reinterpret_cast<uint32_t*>(prm->status));
  if (rc) return rc;
  return launch_extract_sigma(w.raw, P, sigma, st);
}

size_t pnr_regulation_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_prm(prm) || n_rays < 0) return 0;
  size_t b = 0;
  carve_bwd(pad128(n_rays * prm->n_samples), n_rays, nullptr, &b, prm->points != nullptr, save_mode(prm) != 2,
            n_pts(prm));
  return b;
}

int pnr_regulation_bwd(const pnr_render_params* prm, const float* packed, const float* const* params,
                       const float* rays_o, const float* rays_d, int64_t n, const float* g_sigma,
                       float* const* grads, float* g_rays_o, float* g_rays_d, void* workspace, size_t ws_bytes,
                       void* bwd_ws, size_t bwd_bytes, void* stream) {
  (void)params;
  (void)rays_o;
  if (!valid_prm(prm) || !packed || n < 0 || !prm->save_for_backward) return PNR_E_ARG;
  if (n == 0) {  // store semantics: an empty batch's weight gradients are zero
    if (!prm->grads_overwrite) return PNR_OK;
    if (grads)
      for (int i = 0; i < PNR_N_PARAMS; ++i)
        if (!grads[i]) return PNR_E_ARG;
    return zero_weight_grads(grads, prm->points ? prm->points->g_fc : nullptr, (hipStream_t)stream);
  }
  if (!workspace || !bwd_ws || !g_sigma) return PNR_E_ARG;
  if (grads)  // NULL: no decoder weight gradients
    for (int i = 0; i < PNR_N_PARAMS; ++i)
      if (!grads[i]) return PNR_E_ARG;
  // a masks-only forward (save_for_backward 2) kept no activations to form weight gradients from
  if (save_mode(prm) == 2 && (grads || (prm->points && prm->points->g_fc))) return PNR_E_ARG;
  if (prm->need_ray_grads && (!g_rays_o || !g_rays_d || !rays_d)) return PNR_E_ARG;
  size_t need = 0, bneed = 0;
  RegWS w = carve_reg(prm, n, workspace, &need);
  const int64_t P = n * prm->n_samples;
  const int64_t ld = w.save.ld;
  const pnr_points* pts = prm->points;
  BwdWS b = carve_bwd(ld, n, bwd_ws, &bneed, pts != nullptr, save_mode(prm) != 2, n_pts(prm));
  if (ws_bytes < need || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  int rc = launch_gout_sigma(g_sigma, w.save.xP, P, ld, b.g_out, st);  // (zeros on the padding rows)
  if (rc) return rc;
  FeatBwd fb{pts ? pts->fc_packed : nullptr, w.c, pts ? pts->g_fc : nullptr};
  rc = mlp_backward_core(prm->precision, packed, w.save, ld, b, grads, prm->need_ray_grads != 0, st,
                         pts ? &fb : nullptr, prm->grads_overwrite != 0);
  if (rc) return rc;
  if (pts) {
    rc = launch_gather_bwd(*pts, nullptr, kRaysZ32, w.save.xP, ld, w.nidx, w.nw, w.c, b.g_c,
                           prm->need_ray_grads ? b.g_x : nullptr, true, b.gws, b.gws_bytes, st);
    if (rc) return rc;
  }
  if (prm->need_ray_grads) rc = launch_ray_grads_f32(rays_d, w.z, prm->n_samples, b.g_x, n, g_rays_o, g_rays_d, st);
  return rc;
}

// ---- map pass: render + regulation of one Mapper iteration as ONE decoder pass --------------------
namespace {
// Rows of the map pass: regulation [0, pr) | coarse [pr, r1) | importance [r1, ld), each segment's
// real rows first, then padding to a multiple of 128.  `save.xP` holds the kPtsX4 input rows.
struct MapWS {
  float* gmax;
  double* z;     // [n S coarse | n I importance] float64
  double* far;
  float* raw;    // [ld] float4
  uint8_t* ord;  // [n][64]
  int64_t pr, r1, ld;
  SaveArgs save;
  float* c;      // neural points: [ld][32], [ld][k], [ld][k], gather work list
  int32_t* nidx;
  float* nw;
  void* gws;
  size_t gws_bytes;
};
MapWS carve_map(const pnr_render_params* prm, int64_t n, void* ws, size_t* bytes) {
  Carver c(ws);
  MapWS w{};
  const int64_t S = prm->n_samples, I = prm->n_importance;
  w.pr = pad128(n * S);
  w.r1 = w.pr + pad128(n * S);
  w.ld = w.r1 + pad128(n * I);
  w.gmax = c.take<float>(64);
  w.z = c.take<double>(n * (S + I));
  w.far = c.take<double>(n);
  w.raw = c.take<float>((size_t)w.ld * 4);
  w.ord = c.take<uint8_t>(n * PNR_MAX_SAMPLES);
  w.save = carve_save(c, w.ld, prm->precision);
  if (prm->points) {
    w.c = c.take<float>((size_t)w.ld * kCDim);
    w.nidx = c.take<int32_t>((size_t)w.ld * prm->points->k);
    w.nw = c.take<float>((size_t)w.ld * prm->points->k);
    // launch A gathers the r1 regulation + coarse rows, launch B the ld - r1 importance rows (more
    // than r1 when n_importance > 2 n_samples): one workspace serves both
    w.gws_bytes = gather_workspace_bytes(w.r1 > w.ld - w.r1 ? w.r1 : w.ld - w.r1);
    w.gws = c.take<char>(w.gws_bytes);
  }
  if (bytes) *bytes = c.off;
  return w;
}
bool valid_map_prm(const pnr_render_params* prm) {
  return valid_prm(prm) && prm->n_samples >= 3 && prm->n_importance > 0 && prm->precision >= PNR_PREC_FP32 &&
         prm->precision <= PNR_PREC_F16X3;
}
}  // namespace

size_t pnr_map_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_map_prm(prm) || n_rays < 0) return 0;
  size_t b = 0;
  carve_map(prm, n_rays, nullptr, &b);
  return b;
}

namespace {
// The map pass's forward on a carved workspace: launches A and B with the pdf between them, then the
// final compositing into depth / var / rgb unless `fine` is false (pnr_map_step's fused tail runs it)
int map_fwd_core(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                 const float* gt_depth, const float* t_rand, int64_t n, const MapWS& w, double* depth, double* var,
                 float* rgb, float* sigma, bool fine, hipStream_t st) {
  const int S = prm->n_samples, I = prm->n_importance;
  int rc = 0;
  if (prm->far_mode == 0) rc = launch_gt_max(gt_depth, n, w.gmax, st);
  if (rc) return rc;
  float* x4 = reinterpret_cast<float*>(w.save.xP);
  const pnr_points* pts = prm->points;
  const float* gmax = prm->far_mode == 2 ? prm->far_clamp_dev : w.gmax;
  // Launch A's rows (regulation + coarse samples) are formed by k_map_pts into the x4 rows, which the
  // gather and the forward read; without the feature branch the 16-point-wave forward forms them itself
  // (kMapRows: the same arithmetic, map_row_point, its x save is the x4 row) and the launch and its
  // boundary go (PNR_MAP_ROWS_FUSE=0: always k_map_pts)
  static const bool fuse_env = !(getenv("PNR_MAP_ROWS_FUSE") && getenv("PNR_MAP_ROWS_FUSE")[0] == '0');
  const bool fuse = fuse_env && !pts && fwd_map_rows_ok(prm->precision, nullptr);
  if (!fuse) {
    rc = launch_map_pts(*prm, rays_o, rays_d, gt_depth, t_rand, gmax, n, w.pr, w.r1, w.z, w.far, x4, st);
    if (rc) return rc;
  }
  PointSrc src{};
  src.pts = x4;
  FeatArgs fa{pts ? pts->fc_packed : nullptr, w.c};
  const int K = pts ? pts->k : 0;
  uint32_t* status = reinterpret_cast<uint32_t*>(prm->status);
  // launch A: regulation + coarse rows
  if (pts) {
    rc = launch_gather(*pts, src, kPtsX4, w.r1, w.r1, w.c, w.nidx, w.nw, w.gws, w.gws_bytes, st);
    if (rc) return rc;
  }
  if (fuse) {
    const MapRowsArgs mr = map_rows_args(*prm, rays_o, rays_d, gt_depth, t_rand, gmax, n, w.pr, w.z, w.far);
    rc = mlp_fwd(prm->precision, packed, src, kMapRows, w.r1, w.raw, &w.save, st, nullptr, status, &mr);
  } else {
    rc = mlp_fwd(prm->precision, packed, src, kPtsX4, w.r1, w.raw, &w.save, st, pts ? &fa : nullptr, status);
  }
  if (rc) return rc;
  // importance depths and points from the coarse weights; the regulation densities out of launch A
  double* zi = w.z + n * S;
  rc = launch_pdf(*prm, rays_d, w.z, w.raw + w.pr * 4, n, zi, st, rays_o, x4 + w.r1 * 4, w.ld - w.r1 - n * I, w.raw,
                  sigma);
  if (rc) return rc;
  // launch B: importance rows
  PointSrc src2{};
  src2.pts = x4 + w.r1 * 4;
  SaveArgs s2 = w.save;
  s2.p0 = w.r1;
  if (pts) {
    rc = launch_gather(*pts, src2, kPtsX4, n * I, w.ld - w.r1, w.c + w.r1 * kCDim, w.nidx + w.r1 * K,
                       w.nw + w.r1 * K, w.gws, w.gws_bytes, st);
    if (rc) return rc;
    fa.c = w.c + w.r1 * kCDim;
  }
  rc = mlp_fwd(prm->precision, packed, src2, kPtsX4, n * I, w.raw + w.r1 * 4, &s2, st, pts ? &fa : nullptr, status);
  if (rc || !fine) return rc;
  return launch_fine(*prm, rays_d, w.z, zi, w.raw + w.pr * 4, w.raw + w.r1 * 4, n, depth, var, rgb, w.ord, st);
}

// The map pass's backward on carved workspaces: the compositing backward into b.g_out (unless the
// fused tail already wrote it: `fine_done`), the delta chain / weight gradients and the gather backward
int map_bwd_core(const pnr_render_params* prm, const float* packed, const float* rays_d, int64_t n, const MapWS& w,
                 BwdWS& b, const double* g_depth, const float* g_rgb, const float* g_sigma, float* const* grads,
                 bool fine_done, hipStream_t st) {
  const int S = prm->n_samples, I = prm->n_importance;
  const double* zi = w.z + n * S;
  const float4* x4 = w.save.xP;
  const pnr_points* pts = prm->points;
  int rc = 0;
  if (!fine_done) {
    // dL/draw of every row: render rows from the compositing backward, regulation rows from dL/dsigma,
    // zeros on the three segments' padding rows -- one launch
    rc = launch_fine_bwd(*prm, rays_d, w.z, zi, w.raw + w.pr * 4, w.raw + w.r1 * 4, x4 + w.pr, x4 + w.r1, w.ord, n,
                         g_depth, nullptr, g_rgb, b.g_out + w.pr * 4, b.g_out + w.r1 * 4, b.g_nrm,
                         b.g_out + (n * S) * 4, (int)(w.pr - n * S), b.g_out + (w.pr + n * S) * 4,
                         (int)(w.r1 - w.pr - n * S), st, g_sigma, x4, b.g_out, b.g_out + (w.r1 + n * I) * 4,
                         (int)(w.ld - w.r1 - n * I));
    if (rc) return rc;
  }
  FeatBwd fb{pts ? pts->fc_packed : nullptr, w.c, pts ? pts->g_fc : nullptr};
  rc = mlp_backward_core(prm->precision, packed, w.save, w.ld, b, grads, false, st, pts ? &fb : nullptr,
                         prm->grads_overwrite != 0);
  if (rc) return rc;
  if (pts)
    rc = launch_gather_bwd(*pts, nullptr, kPtsX4, x4, w.ld, w.nidx, w.nw, w.c, b.g_c, nullptr, true, b.gws, b.gws_bytes,
                           st);
  return rc;
}

// pnr_map_step's per-ray scratch after the map workspace: the unfused tail's depth / var / rgb /
// sigma and upstream gradients, and the fused tail's block partial losses
struct StepWS {
  double *depth, *var, *g_depth, *part;
  float *rgb, *sigma, *g_rgb, *g_sigma;
};
StepWS carve_step(const pnr_render_params* prm, int64_t n, Carver& c) {
  StepWS s{};
  const int64_t S = prm->n_samples;
  s.depth = c.take<double>(n);
  s.var = c.take<double>(n);
  s.g_depth = c.take<double>(n);
  s.part = c.take<double>(fine_loss_parts(n) > 0 ? fine_loss_parts(n) : 1);
  s.rgb = c.take<float>(n * 3);
  s.sigma = c.take<float>(n * S);
  s.g_rgb = c.take<float>(n * 3);
  s.g_sigma = c.take<float>(n * S);
  return s;
}
}  // namespace

int pnr_map_fwd(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                const float* gt_depth, const float* t_rand, int64_t n, double* depth, double* var, float* rgb,
                float* sigma, void* workspace, size_t ws_bytes, void* stream) {
  if (!valid_map_prm(prm) || !packed || n < 0) return PNR_E_ARG;
  if (n == 0) return PNR_OK;
  if (!rays_o || !rays_d || !gt_depth || !t_rand || !depth || !var || !rgb || !sigma || !workspace) return PNR_E_ARG;
  if (prm->points && !prm->points->fc_packed) return PNR_E_ARG;
  size_t need = 0;
  MapWS w = carve_map(prm, n, workspace, &need);
  if (ws_bytes < need) return PNR_E_WORKSPACE;
  return map_fwd_core(prm, packed, rays_o, rays_d, gt_depth, t_rand, n, w, depth, var, rgb, sigma, true,
                      (hipStream_t)stream);
}

size_t pnr_map_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_map_prm(prm) || n_rays < 0) return 0;
  MapWS w = carve_map(prm, n_rays, nullptr, nullptr);
  size_t b = 0;
  carve_bwd(w.ld, n_rays, nullptr, &b, prm->points != nullptr, true, n_pts(prm));
  return b;
}

int pnr_map_bwd(const pnr_render_params* prm, const float* packed, const float* rays_d, int64_t n,
                const double* g_depth, const float* g_rgb, const float* g_sigma, float* const* grads, void* workspace,
                size_t ws_bytes, void* bwd_ws, size_t bwd_bytes, void* stream) {
  if (!valid_map_prm(prm) || !packed || n < 0) return PNR_E_ARG;
  if (n == 0) {  // store semantics: an empty batch's weight gradients are zero
    if (!prm->grads_overwrite) return PNR_OK;
    if (grads)
      for (int i = 0; i < PNR_N_PARAMS; ++i)
        if (!grads[i]) return PNR_E_ARG;
    return zero_weight_grads(grads, prm->points ? prm->points->g_fc : nullptr, (hipStream_t)stream);
  }
  if (!workspace || !bwd_ws || !rays_d || !g_depth || !g_rgb || !g_sigma) return PNR_E_ARG;
  if (grads)
    for (int i = 0; i < PNR_N_PARAMS; ++i)
      if (!grads[i]) return PNR_E_ARG;
  size_t need = 0, bneed = 0;
  MapWS w = carve_map(prm, n, workspace, &need);
  const pnr_points* pts = prm->points;
  BwdWS b = carve_bwd(w.ld, n, bwd_ws, &bneed, pts != nullptr, true, n_pts(prm));
  if (ws_bytes < need || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  return map_bwd_core(prm, packed, rays_d, n, w, b, g_depth, g_rgb, g_sigma, grads, false, (hipStream_t)stream);
}

size_t pnr_map_step_workspace_bytes(const pnr_render_params* prm, int64_t n_rays) {
  if (!valid_map_prm(prm) || n_rays < 0) return 0;
  Carver c(nullptr);
  carve_map(prm, n_rays, nullptr, &c.off);
  carve_step(prm, n_rays, c);
  return c.off;
}

int pnr_map_step(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                 const float* gt_depth, const float* gt_color, const float* t_rand, int64_t n, float w_color,
                 float w_reg, double* loss, float* const* grads, void* workspace, size_t ws_bytes, void* bwd_ws,
                 size_t bwd_bytes, void* loss_ws, void* stream) {
  if (!valid_map_prm(prm) || !packed || n < 0 || !loss || !loss_ws) return PNR_E_ARG;
  hipStream_t st = (hipStream_t)stream;
  if (grads)
    for (int i = 0; i < PNR_N_PARAMS; ++i)
      if (!grads[i]) return PNR_E_ARG;
  if (n == 0) {  // no rays: loss 0 and (store semantics) zero weight gradients
    if (int rc = hip_status(hipMemsetAsync(loss, 0, sizeof(double), st))) return rc;
    if (!prm->grads_overwrite) return PNR_OK;
    return zero_weight_grads(grads, prm->points ? prm->points->g_fc : nullptr, st);
  }
  if (!rays_o || !rays_d || !gt_depth || !gt_color || !t_rand || !workspace || !bwd_ws) return PNR_E_ARG;
  if (prm->points && !prm->points->fc_packed) return PNR_E_ARG;
  size_t need = 0, bneed = 0;
  MapWS w = carve_map(prm, n, workspace, &need);
  Carver c(workspace);
  c.off = need;
  StepWS sw = carve_step(prm, n, c);
  const pnr_points* pts = prm->points;
  BwdWS b = carve_bwd(w.ld, n, bwd_ws, &bneed, pts != nullptr, true, n_pts(prm));
  if (ws_bytes < c.off || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  const bool fuse = n <= fine_loss_max_rays();
  int rc = map_fwd_core(prm, packed, rays_o, rays_d, gt_depth, t_rand, n, w, sw.depth, sw.var, sw.rgb,
                        fuse ? nullptr : sw.sigma, !fuse, st);
  if (rc) return rc;
  const int64_t S = prm->n_samples, I = prm->n_importance;
  double* lws = static_cast<double*>(loss_ws);
  if (fuse) {
    const float4* x4 = w.save.xP;
    rc = launch_fine_loss(*prm, rays_d, w.z, w.z + n * S, w.raw + w.pr * 4, w.raw + w.r1 * 4, x4 + w.pr, x4 + w.r1, n,
                          gt_depth, gt_color, w_color, w_reg, w.raw, x4, b.g_out, b.g_out + w.pr * 4,
                          b.g_out + w.r1 * 4, b.g_nrm, b.g_out + (n * S) * 4, (int)(w.pr - n * S),
                          b.g_out + (w.pr + n * S) * 4, (int)(w.r1 - w.pr - n * S), b.g_out + (w.r1 + n * I) * 4,
                          (int)(w.ld - w.r1 - n * I), sw.part, reinterpret_cast<uint32_t*>(lws + 256), loss, st);
  } else {
    rc = launch_map_loss(gt_depth, sw.depth, gt_color, sw.rgb, n, w_color, sw.sigma, n * S, w_reg, lws, loss,
                         sw.g_depth, sw.g_rgb, sw.g_sigma, st);
  }
  if (rc) return rc;
  return map_bwd_core(prm, packed, rays_d, n, w, b, sw.g_depth, sw.g_rgb, sw.g_sigma, grads, fuse, st);
}

// ---- neural points ---------------------------------------------------------------------------
size_t pnr_points_index_bytes(int64_t n_points, int32_t table_bits) {
  if (n_points < 0 || table_bits < 10 || table_bits > 24) return 0;
  size_t b = 0;
  index_view(nullptr, n_points, table_bits, &b);
  return b;
}

int pnr_points_build(const pnr_points* pts, void* stream) {
  if (!pts || pts->n_points < 0 || !pts->index || pts->table_bits < 10 || pts->table_bits > 24 || !(pts->cell > 0.f) ||
      (pts->n_points > 0 && !pts->xyz))
    return PNR_E_ARG;
  return launch_points_build(*pts, (hipStream_t)stream);
}

size_t pnr_point_gather_workspace_bytes(int64_t P) { return P < 0 ? 0 : gather_workspace_bytes(P); }

int pnr_point_gather(const pnr_points* pts, const double* p, int64_t P, float* c, int32_t* idx, float* w, void* ws,
                     size_t ws_bytes, void* stream) {
  if (!pts || P < 0 || (P > 0 && (!p || !c)) || (!idx) != (!w)) return PNR_E_ARG;
  PointSrc s{};
  s.pts = p;
  return launch_gather(*pts, s, kPtsF64, P, P, c, idx, w, ws, ws_bytes, (hipStream_t)stream);
}

size_t pnr_point_gather_bwd_workspace_bytes(const pnr_points* pts, int64_t P) {
  if (!pts || P < 0 || pts->n_points < 0) return 0;
  return gather_bwd_workspace_bytes(P, pts->n_points, true);
}

int pnr_point_gather_bwd_atomics(const pnr_points* pts, const void* ws, int64_t P, int64_t* n_instr, void* stream) {
  if (!pts || !ws || P < 0 || !n_instr) return PNR_E_ARG;
  unsigned long long n = 0;
  const int rc = gather_bwd_atomics(ws, P, pts->n_points, &n, (hipStream_t)stream);
  *n_instr = (int64_t)n;
  return rc;
}

int pnr_point_gather_bwd(const pnr_points* pts, const double* p, int64_t P, const int32_t* idx, const float* w,
                         const float* c, const float* g_c, float* g_p, void* ws, size_t ws_bytes, void* stream) {
  if (!pts || P < 0 || (P > 0 && !p)) return PNR_E_ARG;
  PointSrc s{};
  s.pts = p;
  return launch_gather_bwd(*pts, &s, kPtsF64, nullptr, P, idx, w, c, g_c, g_p, false, ws, ws_bytes,
                           (hipStream_t)stream);
}

size_t pnr_fc_packed_floats(void) { return (size_t)fc_packed_floats_all(); }

int pnr_fc_pack(const float* const* fc_params, float* fc_packed, void* stream) {
  if (!fc_params || !fc_packed) return PNR_E_ARG;
  for (int i = 0; i < PNR_N_FC_PARAMS; ++i)
    if (!fc_params[i]) return PNR_E_ARG;
  return launch_fc_pack_all(fc_params, fc_packed, (hipStream_t)stream);
}

int pnr_fc_pack2(const float* const* fc_params, float* fc_packed, int32_t flags, void* stream) {
  if (!fc_params || !fc_packed || (flags & ~PNR_PACK_F16X3_ONLY)) return PNR_E_ARG;
  for (int i = 0; i < PNR_N_FC_PARAMS; ++i)
    if (!fc_params[i]) return PNR_E_ARG;
  return launch_fc_pack_all(fc_params, fc_packed, (hipStream_t)stream, flags);
}

int pnr_eval_points_c(const float* packed, const float* fc_packed, const double* p, const float* c, int64_t P,
                      const double* bound6, float* raw_out, int32_t precision, void* stream) {
  if (!packed || !fc_packed || P < 0 || (P > 0 && (!p || !c || !raw_out))) return PNR_E_ARG;
  PointSrc s{};
  s.pts = p;
  s.use_bound = bound6 != nullptr;
  if (bound6) memcpy(s.bound, bound6, sizeof(s.bound));
  FeatArgs fa{fc_packed, c};
  return mlp_fwd(precision, packed, s, kPtsF64, P, raw_out, nullptr, (hipStream_t)stream, &fa);
}

int pnr_mlp_fwd_train_c(const float* packed, const float* fc_packed, const float* p, const float* c, int64_t P,
                        float* raw_out, void* ws, size_t ws_bytes, int32_t precision, void* stream) {
  if (!packed || !fc_packed || P < 0 || (P > 0 && (!p || !c || !raw_out || !ws))) return PNR_E_ARG;
  if (P == 0) return PNR_OK;
  Carver cv(ws);
  SaveArgs sv = carve_save(cv, pad128(P), precision);
  if (ws_bytes < cv.off) return PNR_E_WORKSPACE;
  PointSrc s{};
  s.pts = p;
  FeatArgs fa{fc_packed, c};
  return mlp_fwd(precision, packed, s, kPtsF32, P, raw_out, &sv, (hipStream_t)stream, &fa);
}

size_t pnr_mlp_bwd_workspace_bytes_c(int64_t P) {
  if (P < 0) return 0;
  size_t b = 0;
  carve_bwd(pad128(P), 1, nullptr, &b, true, true);
  return b;
}

int pnr_mlp_bwd_c(const float* packed, const float* fc_packed, const float* c, int64_t P, const float* g_raw,
                  float* const* grads, float* const* g_fc, float* g_c, float* g_p, void* ws, size_t ws_bytes,
                  void* bwd_ws, size_t bwd_bytes, int32_t precision, void* stream) {
  if (!packed || !fc_packed || P < 0 || (P > 0 && (!c || !g_raw || !grads || !g_fc || !ws || !bwd_ws))) return PNR_E_ARG;
  if (P == 0) return PNR_OK;
  for (int i = 0; i < PNR_N_PARAMS; ++i)
    if (!grads[i]) return PNR_E_ARG;
  for (int i = 0; i < PNR_N_FC_PARAMS; ++i)
    if (!g_fc[i]) return PNR_E_ARG;
  Carver cv(ws);
  SaveArgs sv = carve_save(cv, pad128(P), precision);
  size_t bneed = 0;
  BwdWS b = carve_bwd(sv.ld, 1, bwd_ws, &bneed, true, true);
  if (ws_bytes < cv.off || bwd_bytes < bneed) return PNR_E_WORKSPACE;
  hipStream_t st = (hipStream_t)stream;
  if (hipMemsetAsync(b.g_out, 0, (size_t)sv.ld * 16, st) != hipSuccess) return (int)hipGetLastError();
  if (hipMemcpyAsync(b.g_out, g_raw, (size_t)P * 16, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  // the fc_c GEMMs read c rows up to the padded row count: run them over the real rows only
  FeatBwd fb{fc_packed, c, g_fc};
  int rc = mlp_backward_core(precision, packed, sv, P, b, grads, g_p != nullptr, st, &fb);
  if (rc) return rc;
  if (g_c && hipMemcpyAsync(g_c, b.g_c, (size_t)P * kCDim * 4, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  if (g_p && hipMemcpyAsync(g_p, b.g_x, (size_t)P * 12, hipMemcpyDeviceToDevice, st) != hipSuccess)
    return (int)hipGetLastError();
  return PNR_OK;
}

// ---- rays / optimizer ------------------------------------------------------------------------
int pnr_get_rays(int32_t H, int32_t W, float fx, float fy, float cx, float cy, const float* c2w, float* rays_o,
                 float* rays_d, void* stream) {
  if (H < 0 || W < 0 || !c2w || !rays_o || !rays_d) return PNR_E_ARG;
  return launch_get_rays(H, W, fx, fy, cx, cy, c2w, rays_o, rays_d, (hipStream_t)stream);
}

int pnr_rays_from_uv(const float* i, const float* j, int64_t n, float fx, float fy, float cx, float cy,
                     const float* c2w, float* rays_o, float* rays_d, void* stream) {
  if (n < 0 || (n > 0 && (!i || !j || !c2w || !rays_o || !rays_d))) return PNR_E_ARG;
  return launch_rays_from_uv(i, j, n, fx, fy, cx, cy, c2w, rays_o, rays_d, (hipStream_t)stream);
}

int pnr_window_rays(const int64_t* idx, int64_t n, int64_t n_per_frame, int32_t H, int32_t W, float fx, float fy,
                    float cx, float cy, const float* c2w, const float* depth, const float* color, float* rays_o,
                    float* rays_d, float* gt_depth, float* gt_color, void* stream) {
  if (n < 0 || H <= 0 || W <= 0 || n_per_frame <= 0) return PNR_E_ARG;
  if (n > 0 && (!idx || !c2w || !depth || !color || !rays_o || !rays_d || !gt_depth || !gt_color)) return PNR_E_ARG;
  return launch_window_rays(idx, n, n_per_frame, H, W, fx, fy, cx, cy, c2w, depth, color, rays_o, rays_d, gt_depth,
                            gt_color, (hipStream_t)stream);
}

size_t pnr_window_sample_state_bytes(void) { return (size_t)window_sample_state_bytes(); }

int pnr_window_sample(uint64_t seed, void* state, int64_t n, int64_t n_per_frame, int32_t H, int32_t W, float fx,
                      float fy, float cx, float cy, const float* c2w, const float* depth, const float* color,
                      int32_t n_samples, float* rays_o, float* rays_d, float* gt_depth, float* gt_color,
                      float* t_rand, int64_t* idx, float* far_clamp, void* stream) {
  if (n < 0 || H <= 0 || W <= 0 || n_per_frame <= 0 || n_samples < 0) return PNR_E_ARG;
  if ((int64_t)H * W >= (1LL << 32)) return PNR_E_ARG;
  if (n > 0 && (!state || !c2w || !depth || !color || !rays_o || !rays_d || !gt_depth || !gt_color ||
                (n_samples > 0 && !t_rand)))
    return PNR_E_ARG;
  return launch_window_sample(seed, state, n, n_per_frame, H, W, fx, fy, cx, cy, c2w, depth, color, n_samples, rays_o,
                              rays_d, gt_depth, gt_color, t_rand, idx, far_clamp, (hipStream_t)stream);
}

int pnr_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                  float eps, int64_t step, void* stream) {
  if (n < 0 || step < 1 || (n > 0 && (!p || !g || !m || !v))) return PNR_E_ARG;
  const double bc1 = 1.0 - std::pow((double)beta1, (double)step);
  const double bc2 = 1.0 - std::pow((double)beta2, (double)step);
  const float step_size = (float)((double)lr / bc1);
  const float bc2_sqrt = (float)std::sqrt(bc2);
  return launch_adam(p, g, m, v, n, beta1, beta2, eps, step_size, bc2_sqrt, (hipStream_t)stream);
}

int pnr_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2,
                      float eps, const int32_t* step_count, void* stream) {
  if (n < 0 || !step_count || (n > 0 && (!p || !g || !m || !v))) return PNR_E_ARG;
  return launch_adam_dev(p, g, m, v, n, lr, beta1, beta2, eps, step_count, (hipStream_t)stream);
}

size_t pnr_map_loss_workspace_bytes(void) { return (256 + 8) * sizeof(double); }

int pnr_map_loss(const float* gt_depth, const double* depth, const float* gt_color, const float* color, int64_t n,
                 float w_color, const float* sigma, int64_t n_sigma, float w_reg, double* loss, double* g_depth,
                 float* g_color, float* g_sigma, void* workspace, void* stream) {
  if (n < 0 || n_sigma < 0 || !loss || !workspace) return PNR_E_ARG;
  if (n > 0 && (!gt_depth || !depth || !gt_color || !color || !g_depth || !g_color)) return PNR_E_ARG;
  if (n_sigma > 0 && (!sigma || !g_sigma)) return PNR_E_ARG;
  return launch_map_loss(gt_depth, depth, gt_color, color, n, w_color, sigma, n_sigma, w_reg,
                         static_cast<double*>(workspace), loss, g_depth, g_color, g_sigma, (hipStream_t)stream);
}

int pnr_adam_multi_dev(float* p, const float* g, int32_t n_seg, const int64_t* seg_offset, const int64_t* seg_n,
                       float* const* m, float* const* v, const float* seg_lr, float beta1, float beta2, float eps,
                       int32_t* step2, void* stream) {
  if (!p || !g || !seg_offset || !seg_n || !m || !v || !seg_lr || !step2 || n_seg < 1 || n_seg > 4) return PNR_E_ARG;
  for (int q = 0; q < n_seg; ++q)
    if (seg_n[q] < 0 || seg_offset[q] < 0 || (seg_n[q] > 0 && (!m[q] || !v[q]))) return PNR_E_ARG;
  return launch_adam_multi(p, g, n_seg, seg_offset, seg_n, m, v, seg_lr, beta1, beta2, eps, step2,
                           (hipStream_t)stream);
}

int pnr_adam_multi_dev_h(float* p, const float* g, int32_t n_seg, const int64_t* seg_offset, const int64_t* seg_n,
                         float* const* m, float* const* v, const float* seg_lr, float beta1, float beta2, float eps,
                         uint16_t* const* half_copy, int32_t* step2, void* stream) {
  if (!p || !g || !seg_offset || !seg_n || !m || !v || !seg_lr || !step2 || n_seg < 1 || n_seg > 4) return PNR_E_ARG;
  for (int q = 0; q < n_seg; ++q)
    if (seg_n[q] < 0 || seg_offset[q] < 0 || (seg_n[q] > 0 && (!m[q] || !v[q]))) return PNR_E_ARG;
  return launch_adam_multi(p, g, n_seg, seg_offset, seg_n, m, v, seg_lr, beta1, beta2, eps, step2,
                           (hipStream_t)stream, half_copy);
}

int pnr_step_advance(int32_t* step_count, void* stream) {
  if (!step_count) return PNR_E_ARG;
  return launch_step_advance(step_count, (hipStream_t)stream);
}

}  // extern "C"
