/*
 * pnr.h -- C ABI of the MI355X (gfx950) neural volume renderer `libpnr.so`.
 *
 * Drop-in boundary for the `render_batch_ray` hot path of thua919/pointNeRF-SLAM
 * (src/utils/Renderer.py + src/common.py + src/conv_onet/models/decoder.py).  The Python
 * host mirror `pnr` (pointnerf-slam_amd/pnr/) binds these symbols with ctypes; any other
 * FFI (cgo, JNI, N-API) can bind them the same way -- see INTEGRATION.md.
 *
 * Conventions
 *  - Every pointer argument is a DEVICE pointer owned by the caller, except `pnr_render_params`
 *    and the `const float* const*` parameter-table arrays, which are HOST structs holding device
 *    pointers.  The library allocates no device memory and keeps no per-call state; scratch comes
 *    from the caller's workspace (size from the matching *_workspace_bytes query).
 *  - `stream` is a hipStream_t passed as void* (0 = legacy default stream).  All calls are
 *    asynchronous and stream-ordered; they are re-entrant (the only global state is the opt-in
 *    kernel-timing record of pnr_timing_enable).
 *  - Return value: 0 on success, a negative PNR_E* code on argument errors, or a positive
 *    hipError_t when a launch fails.  No exception ever crosses the ABI.
 *  - Dtypes follow the reference exactly: sample depths z / points / depth / variance are
 *    float64, rays / colours / densities / MLP weights are float32.
 *
 * Decoder parameter table (`params[11]`), the reference state_dict order
 * (src/conv_onet/models/decoder.py:128-159; src/conv_onet/config.py:29-31):
 *    0 embedder._B            (3,93)      1 pts_linears.0.weight (256,93)   2 pts_linears.0.bias (256)
 *    3 pts_linears.1.weight   (256,256)   4 pts_linears.1.bias   (256)
 *    5 pts_linears.2.weight   (256,256)   6 pts_linears.2.bias   (256)
 *    7 pts_linears.3.weight   (256,256)   8 pts_linears.3.bias   (256)
 *    9 output_linear.weight   (4,256)    10 output_linear.bias   (4)
 * all contiguous row-major float32.
 */
#ifndef PNR_H_
#define PNR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PNR_ABI_VERSION 14
#define PNR_N_PARAMS 11
#define PNR_MAX_SAMPLES 64      /* N_samples + N_importance per ray */
#define PNR_C_DIM 32            /* neural-point feature width (decoder.py:122-125 fc_c input) */
#define PNR_MAX_K 8             /* neighbours per sample of the point gather */
#define PNR_N_FC_PARAMS 8       /* fc_c.{0..3}.weight (256,32), fc_c.{0..3}.bias (256), interleaved */

enum {
  PNR_OK = 0,
  PNR_E_ARG = -1,        /* bad argument (null pointer, negative size, unsupported config) */
  PNR_E_WORKSPACE = -2,  /* workspace smaller than *_workspace_bytes */
  PNR_E_BLAS = -3,       /* reserved (no BLAS library is used) */
};

/* ---- neural points (build-defined, no reference counterpart) --------
 * Feature of a sample p: the (up to) k neighbours x_i with the smallest (|p-x_i|^2, i) among
 *   PNR_GATHER_IDW:       |p - x_i| <= radius,           weight w_i = 1 / max(|p - x_i|, eps)
 *   PNR_GATHER_TRILINEAR: |p_a - x_i,a| < spacing_a (all a), w_i = prod_a (1 - |p_a - x_i,a| / spacing_a)
 * c(p) = sum_k (w_k / sum w) f_k, 0 without neighbours (oracle/ref_points.py is the spec).  With
 * points on a lattice, TRILINEAR reproduces MLP.sample_grid_feature's F.grid_sample
 * (src/conv_onet/models/decoder.py:168-175) on interior samples.  The decoder then injects c
 * into every hidden layer: h = relu(W h + b) + fc_c[i](c) (decoder.py:196-197).
 * Search structure: a spatial hash of cubic cells (edge `cell`, corner `origin`) into
 * 2^table_bits buckets, bucket-sorted copies of the positions; built on the device by
 * pnr_points_build into the caller's `index` buffer.  `cell` must be >= 2 * radius * (1 + 2^-9)
 * (IDW) or >= 2 * max(spacing) * (1 + 2^-9) (TRILINEAR): the search visits the 2x2x2 cells
 * covering [p - reach, p + reach], and the margin absorbs the f32 rounding of cell coordinates. */
enum { PNR_GATHER_IDW = 0, PNR_GATHER_TRILINEAR = 1 };

/* Arithmetic of the decoder matmuls (build-defined; the reference runs torch fp32 matmuls).
 *   PNR_PREC_FP32:   v_mfma_f32_32x32x2_f32, an exact fp32 fma chain (bitwise the CPU order per
 *                    product; only the summation order differs from torch CPU).
 *   PNR_PREC_F16X3:  (default) every fp32 operand split x = hi + lo into two f16 parts (22
 *                    significant bits), W x computed as Wh xh + Wh xl + Wl xh on
 *                    v_mfma_f32_32x32x16_f16 with fp32 accumulation (~2^-21 relative per product),
 *                    5.3x the fp32 MFMA rate.  The packer scales each weight tensor by a power of two
 *                    (max |W| s <= 2^14) and the kernel scales the accumulator back exactly.  The
 *                    forward needs |activations| < 65504 (f16 range): a larger value sets
 *                    PNR_STATUS_F16_RANGE in *prm->status.
 *   PNR_PREC_BF16X3: the same split in bf16 parts (16 significant bits, no range limit).
 *   PNR_PREC_BF16:   plain bf16 forward operands, fp32 accumulation (BASELINE config C3).
 * Fourier features, bias, ReLU, compositing and all float64 work stay fp32 / fp64 in every mode.
 * Backward of every mode but PNR_PREC_FP32 (which runs fp32 MFMA throughout): the delta chain is
 * f16x3 with an exact per-point power-of-two scale (any gradient magnitude), and the weight-gradient
 * GEMMs dW0..dW3, dWc are f16x3 on fp32-stored activations and deltas (per-wave power-of-two scale of
 * the deltas; delta4 = (Wo^T g_out) masked is not stored but rebuilt in fp32 FMAs inside the dW3
 * GEMM); dWo and dB are fp32 FMA reductions.  Point features (the fc_c operand) are split under a
 * power-of-two scale of their own in both directions (forward: per wave; dWc: per-wave running
 * scale), so they keep 22 bits whatever their magnitude (the reference's fine-grid features have
 * std 1e-4).  Hidden activations and the Fourier features are split unscaled (|e| <= 1, activations
 * checked < 65504): 22 bits for values >= 2^-3 and an absolute error <= 2^-25 below.  In a
 * weight-gradient element dW[i][j] = sum_p delta_i h_j that bounds each term's error by
 * |delta_i| 2^-25: an element whose unit j stays below ~3e-5 at every point carries more than 1e-3
 * relative error, but is itself < 1e-6 of a typical element.  (A per-point scale of the activation
 * rows, measured this round, cost 32% of the weight-gradient time.)  Every GEMM accumulates in fp32. */
enum { PNR_PREC_FP32 = 0, PNR_PREC_BF16X3 = 1, PNR_PREC_BF16 = 2, PNR_PREC_F16X3 = 3 };

/* Status bits (ABI 7) the kernels OR into the caller's device word pnr_render_params.status:
 *   PNR_STATUS_F16_RANGE  an F16X3 forward met a value >= 65504 to split into f16 parts (the result
 *                         of that call is not fp32-faithful; re-run it in PNR_PREC_FP32). */
enum { PNR_STATUS_F16_RANGE = 1 };

typedef struct pnr_points {
  const float* xyz;         /* (M,3) float32 point positions                                  */
  const float* feats;       /* (M,32) float32 point features                                  */
  int64_t n_points;         /* M                                                              */
  int32_t mode;             /* PNR_GATHER_IDW / PNR_GATHER_TRILINEAR                          */
  int32_t k;                /* neighbours kept, 1..PNR_MAX_K                                  */
  float radius;             /* IDW ball radius                                                */
  float eps;                /* IDW distance floor                                             */
  float spacing[3];         /* TRILINEAR lattice spacing per axis                             */
  float cell;               /* hash cell edge                                                 */
  float origin[3];          /* hash cell origin                                               */
  int32_t table_bits;       /* 10..24                                                         */
  void* index;              /* device buffer of pnr_points_index_bytes() bytes                */
  const float* fc_packed;   /* fc_c weight image (pnr_fc_pack) for the decoder; may be NULL for
                               the standalone gather                                           */
  float* g_feats;           /* backward: dL/dfeats (M,32) ACCUMULATED, or NULL                */
  float* const* g_fc;       /* backward: host array of 8 device ptrs accumulating dL/dfc_c, or NULL */
  int32_t feat_half;        /* ABI 6: 1 = `feats` holds (M,32) float16 (read-only copy of an fp32
                               master; sums, weights and g_feats stay float32), 0 = float32     */
} pnr_points;

/* Renderer configuration: the cfg keys Renderer.__init__ reads (src/utils/Renderer.py:6-21)
 * plus host-computed torch.linspace tables (Renderer.py:157, common.py:33). */
typedef struct pnr_render_params {
  int32_t n_samples;        /* cfg['rendering']['N_samples']  (<= 64)            */
  int32_t n_importance;     /* cfg['rendering']['N_importance'] (n_samples+n_importance <= 64) */
  int32_t lindisp;          /* cfg['rendering']['lindisp']                       */
  int32_t far_mode;         /* 0: clamp far to max(1.2*gt) of THIS batch (Renderer.py:112);
                               1: clamp to `far_clamp` (global max supplied by a sharded caller);
                               2: clamp to *far_clamp_dev (a device float32, e.g. the all-reduced
                                  max of a sharded batch: no host round trip, graph-capturable) */
  double bound[6];          /* slam.bound (3,2) float64 row-major: x0,x1,y0,y1,z0,z1   */
  double far_clamp;         /* used when far_mode == 1                                 */
  float t_vals[PNR_MAX_SAMPLES];   /* torch.linspace(0,1,n_samples) float32           */
  float u_vals[PNR_MAX_SAMPLES];   /* torch.linspace(0,1,n_importance) float32        */
  int32_t save_for_backward;       /* 1: keep MLP activations in the workspace for pnr_render_bwd;
                                      2 (ABI 8): keep only the ReLU masks and inputs -- the backward
                                      then computes NO decoder / fc_c weight gradients (grads and
                                      g_fc must be NULL: the Tracker's camera-only backward); the
                                      split precisions skip the 4 KB/point activation stores
                                      (PNR_PREC_FP32 saves everything either way) */
  int32_t need_ray_grads;          /* backward also produces dL/drays_o, dL/drays_d (tracking) */
  const pnr_points* points;        /* neural-point features, NULL = the reference decoder (c_dim=0) */
  int32_t precision;               /* PNR_PREC_* of the decoder matmuls                           */
  int32_t grads_overwrite;         /* ABI 11, backward: 0 = add the decoder / fc_c weight gradients
                                      into `grads` / `g_fc` (autograd's accumulation), 1 = store them
                                      (the caller need not zero them first; point-feature gradients
                                      always accumulate)                                          */
  int32_t* status;                 /* ABI 7: device int32 receiving PNR_STATUS_* bits (ORed), or NULL */
  const float* far_clamp_dev;      /* ABI 7: device float32 far clamp of far_mode 2                */
} pnr_render_params;

/* ---- library identity -------------------------------------------------------------------- */
int pnr_abi_version(void);
const char* pnr_build_info(void);

/* ---- decoder: MLP.forward / eval_points -------------------------------------------------- */
/* Number of float32 words of the packed (MFMA-fragment-ordered) weight image: the fp32 fragment
 * images plus the bf16 split images of the PNR_PREC_BF16X3 / PNR_PREC_BF16 kernels. */
size_t pnr_mlp_packed_floats(void);
/* Builds the packed image from the 11 reference tensors (params: host array of device ptrs).
 * Must be re-run after every optimizer step (the image is a pure function of the weights). */
int pnr_mlp_pack(const float* const* params, float* packed, void* stream);
/* ABI 14: pnr_mlp_pack with flags.  PNR_PACK_F16X3_ONLY: only the images the PNR_PREC_F16X3 kernels
 * read (the weight scales, the forward and delta-chain images and the raw table; the fp32 and bf16
 * images are left as they were) -- a Mapper iteration's repack after its Adam step, on the critical
 * path.  Those images are bit for bit those of pnr_mlp_pack.  flags 0 = pnr_mlp_pack. */
#define PNR_PACK_F16X3_ONLY 2
int pnr_mlp_pack2(const float* const* params, float* packed, int32_t flags, void* stream);

/* Renderer.eval_points (src/utils/Renderer.py:23-61): raw[P,4] = MLP(p) with raw[:,3] := 100
 * where p is not strictly inside `bound6`.  p float64 (P,3).  `precision`: PNR_PREC_*. */
int pnr_eval_points(const float* packed, const double* p, int64_t P, const double* bound6,
                    float* raw_out, int32_t precision, void* stream);
/* Same for float32 points (MLP.forward on f32 input, decoder.py:177-203); bound6 may be NULL
 * (then no masking).  The mask comparison is done in float32 as torch does for f32 points. */
int pnr_eval_points_f32(const float* packed, const float* p, int64_t P, const double* bound6,
                        float* raw_out, int32_t precision, void* stream);

/* MLP.forward with autograd (decoder.py:177-203 on float32 points, no bound mask): the forward
 * keeps activations in `ws` (size pnr_mlp_train_workspace_bytes(P)); pnr_mlp_bwd consumes them.
 * g_raw (P,4) float32; grads accumulated (+=); g_p (P,3) written when non-NULL. */
size_t pnr_mlp_train_workspace_bytes(int64_t P);
int pnr_mlp_fwd_train(const float* packed, const float* p, int64_t P, float* raw_out, void* ws, size_t ws_bytes,
                      int32_t precision, void* stream);
size_t pnr_mlp_bwd_workspace_bytes(int64_t P);
int pnr_mlp_bwd(const float* packed, int64_t P, const float* g_raw, float* const* grads, float* g_p, void* ws,
                size_t ws_bytes, void* bwd_ws, size_t bwd_bytes, int32_t precision, void* stream);

/* ---- map pass (ABI 10): one Mapper iteration's two decoder passes as ONE pass --------------------
 * src/Mapper.py:623-655 renders the window batch with gt depth (render_batch_ray: N_samples coarse +
 * N_importance importance samples, Renderer.py:63-203) and queries the density at N_samples jittered
 * depths per ray (regulation, Renderer.py:263-301).  pnr_map_fwd runs both with shared MLP launches:
 * launch A over the regulation + coarse samples, launch B over the importance samples; the points and
 * their bound tests are formed by the ray kernels in the reference's dtypes (float32 regulation,
 * float64 render).  Outputs: depth, var (n) float64, rgb (n,3), sigma (n, N_samples) float32 -- bit for
 * bit those of pnr_render_fwd + pnr_regulation_fwd with the same t_rand (tests/test_gpu_mapping.py).
 * pnr_map_bwd takes dL/ddepth, dL/drgb, dL/dsigma and runs ONE delta chain / weight-gradient pass over
 * every sample (grads accumulated, +=; neural points as in pnr_render_bwd); no ray gradients.
 * prm: save_for_backward / need_ray_grads ignored (the pass always trains the decoder); n_importance > 0;
 * far_mode as pnr_render_fwd; t_rand (n, N_samples) float32 in [0,1). */
size_t pnr_map_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_map_fwd(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                const float* gt_depth, const float* t_rand, int64_t n, double* depth, double* var, float* rgb,
                float* sigma, void* workspace, size_t ws_bytes, void* stream);
size_t pnr_map_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_map_bwd(const pnr_render_params* prm, const float* packed, const float* rays_d, int64_t n,
                const double* g_depth, const float* g_rgb, const float* g_sigma, float* const* grads, void* workspace,
                size_t ws_bytes, void* bwd_ws, size_t bwd_bytes, void* stream);

/* ---- neural points ------------------------------------------------------------------------ */
size_t pnr_points_index_bytes(int64_t n_points, int32_t table_bits);
/* (Re)builds pts->index from pts->xyz (after any change of positions / cell / origin). */
int pnr_points_build(const pnr_points* pts, void* stream);
/* Standalone gather: c (P,32) float32 for float64 points p (P,3).  idx (P,k) int32 (-1 = none)
 * and w (P,k) float32 normalised weights are written when non-NULL (needed by the backward).
 * ws: pnr_point_gather_workspace_bytes(P) bytes (work list of samples with candidates). */
size_t pnr_point_gather_workspace_bytes(int64_t P);
int pnr_point_gather(const pnr_points* pts, const double* p, int64_t P, float* c, int32_t* idx, float* w,
                     void* ws, size_t ws_bytes, void* stream);
/* Backward of pnr_point_gather: g_c (P,32) -> pts->g_feats (+=, when non-NULL) and g_p (P,3)
 * (written, when non-NULL: dL/dp through the weights).  ws: pnr_point_gather_bwd_workspace_bytes
 * (ABI 10).  The feature gradient is DETERMINISTIC (ABI 10): every term w_k dL/dc is rounded once to
 * an int64 multiple of 2^-s (s from max |dL/dc| of the call and the guard bits ceil(log2(P+1)), so
 * no sum overflows), the terms are added exactly with 64-bit integer atomics, and the sum is
 * converted once into g_feats.  Any order of the additions gives the same bits.  The absolute error
 * of an element is at most (its term count) x 2^-(63 - guard) x max |dL/dc|: fp32-class for any
 * element above ~2^-14 of the largest term.  A non-finite dL/dc makes every element of the feature
 * rows the call's samples name NaN; rows no sample names are left untouched (ABI 12). */
size_t pnr_point_gather_bwd_workspace_bytes(const pnr_points* pts, int64_t P);
int pnr_point_gather_bwd(const pnr_points* pts, const double* p, int64_t P, const int32_t* idx, const float* w,
                         const float* c, const float* g_c, float* g_p, void* ws, size_t ws_bytes, void* stream);
/* Diagnostics (ABI 10): the 64-bit atomic add instructions (32 lanes x 8 B = 256 B each) the last
 * pnr_point_gather_bwd with workspace `ws` issued (synchronises `stream`). */
int pnr_point_gather_bwd_atomics(const pnr_points* pts, const void* ws, int64_t P, int64_t* n_instr, void* stream);
/* fc_c weight image of the decoder (MLP(c_dim=32)): fc_params = host array of the 8 tensors
 * fc_c.0.weight, fc_c.0.bias, ..., fc_c.3.bias (contiguous float32). */
size_t pnr_fc_packed_floats(void);
int pnr_fc_pack(const float* const* fc_params, float* fc_packed, void* stream);
/* ABI 14: pnr_fc_pack with the pnr_mlp_pack2 flags. */
int pnr_fc_pack2(const float* const* fc_params, float* fc_packed, int32_t flags, void* stream);
/* MLP.forward with per-point features c (P,32): eval (bound6 may be NULL) and training
 * variants.  pnr_mlp_bwd_c also writes g_c (P,32) and accumulates the 8 fc_c grads. */
int pnr_eval_points_c(const float* packed, const float* fc_packed, const double* p, const float* c, int64_t P,
                      const double* bound6, float* raw_out, int32_t precision, void* stream);
int pnr_mlp_fwd_train_c(const float* packed, const float* fc_packed, const float* p, const float* c, int64_t P,
                        float* raw_out, void* ws, size_t ws_bytes, int32_t precision, void* stream);
size_t pnr_mlp_bwd_workspace_bytes_c(int64_t P);
int pnr_mlp_bwd_c(const float* packed, const float* fc_packed, const float* c, int64_t P, const float* g_raw,
                  float* const* grads, float* const* g_fc, float* g_c, float* g_p, void* ws, size_t ws_bytes,
                  void* bwd_ws, size_t bwd_bytes, int32_t precision, void* stream);

/* ---- render_batch_ray (src/utils/Renderer.py:63-203) ------------------------------------- */
size_t pnr_render_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
/* Forward.  depth, var: float64 (N); rgb float32 (N,3).  gt_depth may be NULL (gt_depth=None).
 * The workspace must stay untouched between this call and pnr_render_bwd. */
int pnr_render_fwd(const pnr_render_params* prm, const float* packed,
                   const float* rays_o, const float* rays_d, const float* gt_depth, int64_t n_rays,
                   double* depth, double* var, float* rgb,
                   void* workspace, size_t ws_bytes, void* stream);
/* Backward of the final (44-sample) pass.  Inputs are dL/ddepth, dL/dvar (float64, may be NULL
 * = zero), dL/drgb (float32, may be NULL).  Outputs: `grads` = host array of 11 device pointers
 * receiving dL/dparam (ACCUMULATED: +=, reference layout), or NULL for no decoder weight gradients
 * (ABI 5: the Tracker's camera-only backward skips every weight-gradient launch), g_rays_o / g_rays_d (N,3) float32
 * written (not accumulated) when prm->need_ray_grads, else ignored (may be NULL).
 * `params` = the same 11 raw tensors (needed for the transposed weight images). */
size_t pnr_render_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_render_bwd(const pnr_render_params* prm, const float* packed, const float* const* params,
                   const float* rays_o, const float* rays_d, int64_t n_rays,
                   const double* g_depth, const double* g_var, const float* g_rgb,
                   float* const* grads, float* g_rays_o, float* g_rays_d,
                   void* workspace, size_t ws_bytes,
                   void* bwd_workspace, size_t bwd_ws_bytes, void* stream);

/* ---- Renderer.regulation (src/utils/Renderer.py:263-301) --------------------------------- */
/* sigma[N*n_samples] = density at z = lower + (upper-lower)*t_rand in [0, 0.85*gt], float32 z.
 * t_rand (N, n_samples) float32 replaces the reference's torch.rand draw (Renderer.py:293). */
size_t pnr_regulation_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_regulation_fwd(const pnr_render_params* prm, const float* packed,
                       const float* rays_o, const float* rays_d, const float* gt_depth,
                       const float* t_rand, int64_t n_rays, float* sigma,
                       void* workspace, size_t ws_bytes, void* stream);
size_t pnr_regulation_bwd_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_regulation_bwd(const pnr_render_params* prm, const float* packed, const float* const* params,
                       const float* rays_o, const float* rays_d, int64_t n_rays,
                       const float* g_sigma, float* const* grads, float* g_rays_o, float* g_rays_d,
                       void* workspace, size_t ws_bytes,
                       void* bwd_workspace, size_t bwd_ws_bytes, void* stream);

/* ---- rays (src/common.py:74-89, 248-266) ------------------------------------------------- */
/* Full-frame rays, row-major (H,W,3) float32; c2w (3,4) or (4,4) float32 row-major on device. */
int pnr_get_rays(int32_t H, int32_t W, float fx, float fy, float cx, float cy, const float* c2w,
                 float* rays_o, float* rays_d, void* stream);
/* Rays for pixel coordinates i (column), j (row), float32 (n). */
int pnr_rays_from_uv(const float* i, const float* j, int64_t n, float fx, float fy, float cx, float cy,
                     const float* c2w, float* rays_o, float* rays_d, void* stream);
/* ABI 10: a Mapper iteration's pixel batch over its keyframe window in one launch (src/Mapper.py:560-606:
 * per window frame get_samples(0, H, 0, W, pixs_per_image, ...), src/common.py:110-134).  Ray r uses
 * frame f = r / n_per_frame and pixel idx[r] (int64, uniform over the H x W image, row-major: column
 * idx % W, row idx / W; clamped into the image as select_uv clamps); c2w (F,4,4) float32, depth
 * (F,H,W) float32, color (F,H,W,3) float32.  Writes rays_o, rays_d (n,3), gt_depth (n), gt_color (n,3):
 * the same values as pnr_rays_from_uv + the reference's depth / colour gathers. */
int pnr_window_rays(const int64_t* idx, int64_t n, int64_t n_per_frame, int32_t H, int32_t W, float fx, float fy,
                    float cx, float cy, const float* c2w, const float* depth, const float* color, float* rays_o,
                    float* rays_d, float* gt_depth, float* gt_color, void* stream);

/* ABI 11: the same batch with its draws made on the device, plus the regulation jitter and the far
 * clamp, in ONE launch (a captured Mapper iteration replays it without torch's RNG launches):
 * pixel r ~ uniform over [0, H*W) (get_samples' torch.randint), t_rand (n, n_samples) ~ uniform
 * [0,1) with 24-bit resolution (Renderer.py:293's torch.rand), far_clamp[0] = max(1.2 * gt_depth)
 * (Renderer.py:112; pass it as far_clamp_dev, far_mode 2).  The draws are a counter-based hash of
 * (seed, batch, draw index) -- the reference's distribution, not torch's Philox sequence.  `state`
 * (pnr_window_sample_state_bytes(), zero-filled before the first call, not shared by concurrent
 * calls) holds the batch counter, advanced by each call on the device.  idx (n, int64) receives the
 * drawn pixels and may be NULL; far_clamp may be NULL.  Rays and gt equal pnr_window_rays on idx. */
size_t pnr_window_sample_state_bytes(void);
int pnr_window_sample(uint64_t seed, void* state, int64_t n, int64_t n_per_frame, int32_t H, int32_t W, float fx,
                      float fy, float cx, float cy, const float* c2w, const float* depth, const float* color,
                      int32_t n_samples, float* rays_o, float* rays_d, float* gt_depth, float* gt_color,
                      float* t_rand, int64_t* idx, float* far_clamp, void* stream);

/* ---- optimizer (src/Mapper.py:498-502, 657-662: torch.optim.Adam, default betas/eps) ----- */
/* One Adam step over `n` float32 words: p -= lr * mhat / (sqrt(vhat) + eps).  step >= 1. */
int pnr_adam_step(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                  float beta2, float eps, int64_t step, void* stream);
/* The same step with the step number read on the device: step = *step_count + 1, where
 * step_count (int32, device) counts completed steps and is advanced by pnr_step_advance after the
 * step's last Adam launch.  Host-free, so a captured graph (hipGraph / torch.cuda.CUDAGraph) of a
 * whole mapping iteration replays with the right bias corrections. */
int pnr_adam_step_dev(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1,
                      float beta2, float eps, const int32_t* step_count, void* stream);
int pnr_step_advance(int32_t* step_count, void* stream);
/* ABI 10: Adam over n_seg (1..4) learning-rate segments of one flat parameter buffer -- segment q is
 * p[seg_offset[q] .. + seg_n[q]) with its own moments m[q], v[q] (device pointers, host array) and
 * lr seg_lr[q] -- AND the step advance, in ONE launch: step2 (int32[2], device) = {completed steps,
 * 0}; every element uses step = step2[0] + 1, and the launch leaves {step2[0] + 1, 0}.  Same
 * arithmetic as pnr_adam_step_dev per segment followed by pnr_step_advance. */
int pnr_adam_multi_dev(float* p, const float* g, int32_t n_seg, const int64_t* seg_offset, const int64_t* seg_n,
                       float* const* m, float* const* v, const float* seg_lr, float beta1, float beta2, float eps,
                       int32_t* step2, void* stream);
/* ABI 12: pnr_adam_multi_dev that also writes float16(p) of every updated element of segment q into
 * half_copy[q][0 .. seg_n[q]) when half_copy (host array of n_seg device pointers) and half_copy[q]
 * are non-NULL: the float16 feature copy the gather reads (pnr_points.feat_half), refreshed in the
 * same pass instead of a separate conversion of the whole table (round to nearest even, as torch's
 * float16 copy). */
int pnr_adam_multi_dev_h(float* p, const float* g, int32_t n_seg, const int64_t* seg_offset, const int64_t* seg_n,
                         float* const* m, float* const* v, const float* seg_lr, float beta1, float beta2, float eps,
                         uint16_t* const* half_copy, int32_t* step2, void* stream);

/* Mapper loss terms and their gradients (src/Mapper.py:628-655, the loss of Mapper.optimize_map
 * built from render_batch_ray's depth / colour and regulation's sigma), in one pass (ABI 9):
 *   *loss   = sum_{i<n, gt_depth_i > 0} |gt_depth_i - depth_i| + w_color sum_{i<n} |gt_color_i - color_i|_1
 *           + w_reg sum_{j<n_sigma} |sigma_j|                                          (float64)
 *   g_depth = -sign(gt_depth - depth) [gt_depth > 0]  (float64, n)
 *   g_color = -w_color sign(gt_color - color)         (float32, n x 3)
 *   g_sigma = w_reg sign(sigma)                       (float32, n_sigma)
 * sign(0) = 0 as torch's abs backward.  Either part may be empty (n = 0 or n_sigma = 0, its
 * pointers NULL).  The sum has a fixed order (deterministic).  workspace:
 * pnr_map_loss_workspace_bytes() bytes of device scratch, ZERO-FILLED before its first use (ABI 10: it
 * holds a ticket word that lets the last block add the partial sums, one launch; each call leaves it
 * zero-filled again, so a caller reuses one workspace for the calls of one stream).  Replaces the ~20
 * elementwise / reduction launches the torch form of the loss and its autograd backward cost. */
size_t pnr_map_loss_workspace_bytes(void);
int pnr_map_loss(const float* gt_depth, const double* depth, const float* gt_color, const float* color, int64_t n,
                 float w_color, const float* sigma, int64_t n_sigma, float w_reg, double* loss, double* g_depth,
                 float* g_color, float* g_sigma, void* workspace, void* stream);

/* One Mapper iteration's loss and decoder / fc_c / point-feature gradients in ONE call (ABI 13;
 * src/Mapper.py:623-655): pnr_map_fwd, pnr_map_loss and pnr_map_bwd on the same inputs.  Up to
 * 32,768 rays the final compositing, the loss terms and the compositing backward run as ONE fused
 * wave-per-ray launch (k_fine_loss_w): the gradients are bit for bit those of the three-call form,
 * the loss differs from pnr_map_loss's only in summation order (fixed: deterministic).  Larger
 * batches run the three calls' kernels.  No depth / colour / sigma outputs.
 *   workspace: pnr_map_step_workspace_bytes(prm, n); bwd_ws: pnr_map_bwd_workspace_bytes(prm, n);
 *   loss_ws: a pnr_map_loss workspace (zero-filled before its first use, left zero-filled);
 *   grads / prm->grads_overwrite / prm->points as pnr_map_bwd; *loss float64 on the device.
 * n = 0: *loss = 0 and (grads_overwrite) zero decoder / fc_c gradients. */
size_t pnr_map_step_workspace_bytes(const pnr_render_params* prm, int64_t n_rays);
int pnr_map_step(const pnr_render_params* prm, const float* packed, const float* rays_o, const float* rays_d,
                 const float* gt_depth, const float* gt_color, const float* t_rand, int64_t n, float w_color,
                 float w_reg, double* loss, float* const* grads, void* workspace, size_t ws_bytes, void* bwd_ws,
                 size_t bwd_bytes, void* loss_ws, void* stream);

/* ---- diagnostics (not on the reference API) ----------------------------------------------- */
/* Kernel timing: while enabled, every launch of the timed kernels is bracketed by hipEvents on
 * its own stream.  pnr_timing_read synchronises those events and returns, for `kernel`
 *   0 = fused MLP forward (k_mlp_fwd / k_mlp_fwd16), units = points
 *   1 = MLP delta chain (k_mlp_bwd / k_mlp_bwd16), units = points
 *   2 = ray kernels, units = rays
 *   3 = weight-gradient GEMMs (k_wgrad / k_wgrad16 / k_wgrad_skinny, each with its fixed-order
 *       partial reduction k_part_reduce), units = points of the K dimension
 *   4 = neural-point gather (pnr_point_gather and the render's gathers: probe, group scan /
 *       scatter and search as one bracket), units = samples
 *   5 = neural-point gather backward (k_gather_bwd_probe + k_gather_bwd), units = samples
 *   6 = the grouped split weight-gradient launch (k_wgrad16_group: every f16x3 GEMM of a backward
 *       chunk but dWo / dB), units = multiply-adds / 65,536 (one 256 x 256 layer over one point = 1)
 *       -- kind 3 then holds the dWo / dB launches and the fp32-mode GEMMs
 * the launch count, the summed device milliseconds and the summed units, then clears that
 * kernel's record.  Process-global, mutex-protected; off by default. */
int pnr_timing_enable(int on);
int pnr_timing_read(int kernel, int64_t* launches, double* ms, int64_t* units);

#ifdef __cplusplus
}
#endif
#endif /* PNR_H_ */
