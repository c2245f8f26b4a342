"""CPU restatement of the reference `render_batch_ray` hot path -- TEST INFRASTRUCTURE ONLY.

This module is the parity oracle for the HIP renderer in `pointnerf-slam_amd/`.  Only
`tests/`, `__graft_entry__.smoke()` and the `cpu_baseline` leg of `bench.py` may import it,
and only as the checker / the timed CPU baseline: the product path never routes through it
(the HIP library fails loudly when it is missing).

It restates, in plain PyTorch on the CPU, the reference's algorithm with the reference's dtype
quirks (float64 z / points / depth / variance, float32 MLP / alpha / weights / colour).  Each
function cites the reference file:line it follows (paths relative to thua919/pointNeRF-SLAM).
It is pinned against golden vectors produced by importing the reference itself
(`tests/golden/make_golden.py` -> `tests/golden/*.npz`, checked by
`tests/test_oracle_golden.py`).

Decoder parameters are passed as a dict keyed like the reference `state_dict`
(`embedder._B`, `pts_linears.{0..3}.{weight,bias}`, `output_linear.{weight,bias}`).
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]

N_LAYERS = 4           # pts_linears.0..3   (src/conv_onet/config.py:29-31: n_blocks=4, skips=[])
HIDDEN = 256           # hidden_size=256    (src/conv_onet/config.py:30)
N_FOURIER = 93         # mapping_size       (src/conv_onet/models/decoder.py:129)
OUT_OF_BOUND_SIGMA = 100.0   # src/utils/Renderer.py:57


# --------------------------------------------------------------------------------------------
# Scene bound, rays, poses
# --------------------------------------------------------------------------------------------
def scaled_bound(bound_cfg, scale: float, bound_divisible: float) -> torch.Tensor:
    """src/NICE_SLAM.py:208-213 -- scale the yaml bound, round the upper edge up to a multiple
    of `bound_divisible` above the lower edge.  Returns a (3,2) float64 tensor."""
    b = torch.from_numpy(np.array(bound_cfg) * scale)
    b[:, 1] = (((b[:, 1] - b[:, 0]) / bound_divisible).int() + 1) * bound_divisible + b[:, 0]
    return b


def camera_dirs(i: torch.Tensor, j: torch.Tensor, fx, fy, cx, cy) -> torch.Tensor:
    """Pinhole direction [(i-cx)/fx, -(j-cy)/fy, -1] (src/common.py:82-83, 259-260)."""
    return torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)


def rays_from_uv(i, j, c2w, fx, fy, cx, cy) -> Tuple[torch.Tensor, torch.Tensor]:
    """src/common.py:74-89: world rays for pixel coordinates (i=column, j=row)."""
    if isinstance(c2w, np.ndarray):
        c2w = torch.from_numpy(c2w)
    d = camera_dirs(i, j, fx, fy, cx, cy).reshape(-1, 1, 3)
    rays_d = torch.sum(d * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def full_frame_rays(H, W, fx, fy, cx, cy, c2w) -> Tuple[torch.Tensor, torch.Tensor]:
    """src/common.py:248-266: (H,W,3) rays for every pixel, row-major."""
    if isinstance(c2w, np.ndarray):
        c2w = torch.from_numpy(c2w)
    col, row = torch.meshgrid(torch.linspace(0, W - 1, W), torch.linspace(0, H - 1, H), indexing='ij')
    d = camera_dirs(col.t(), row.t(), fx, fy, cx, cy).reshape(H, W, 1, 3)
    rays_d = torch.sum(d * c2w[:3, :3], -1)
    rays_o = c2w[:3, -1].expand(rays_d.shape)
    return rays_o, rays_d


def quat_to_rotation(q: torch.Tensor) -> torch.Tensor:
    """src/common.py:137-160, restated device-agnostic (the reference's `.to(get_device())`
    fails on CPU tensors).  q = (qr, qi, qj, qk), batched (B,4) -> (B,3,3)."""
    qr, qi, qj, qk = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    s = 2.0 / (q * q).sum(-1)
    rows = [
        1 - s * (qj ** 2 + qk ** 2), s * (qi * qj - qk * qr), s * (qi * qk + qj * qr),
        s * (qi * qj + qk * qr), 1 - s * (qi ** 2 + qk ** 2), s * (qj * qk - qi * qr),
        s * (qi * qk - qj * qr), s * (qj * qk + qi * qr), 1 - s * (qi ** 2 + qj ** 2),
    ]
    return torch.stack(rows, -1).reshape(-1, 3, 3)


def camera_from_tensor(t: torch.Tensor) -> torch.Tensor:
    """src/common.py:163-176: 7-vector (qw,qx,qy,qz,tx,ty,tz) -> (3,4) [R|t]."""
    single = t.dim() == 1
    if single:
        t = t.unsqueeze(0)
    R = quat_to_rotation(t[:, :4])
    RT = torch.cat([R, t[:, 4:, None]], 2)
    return RT[0] if single else RT


def tensor_from_camera(RT) -> torch.Tensor:
    """src/common.py:179-201 without `mathutils`: rotation -> unit quaternion (w,x,y,z) by the
    standard trace branch (Blender's Matrix.to_quaternion), then translation."""
    RT = np.asarray(RT.detach().cpu() if isinstance(RT, torch.Tensor) else RT, dtype=np.float64)
    R, T = RT[:3, :3], RT[:3, 3]
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    return torch.from_numpy(np.concatenate([q, T])).float()


# --------------------------------------------------------------------------------------------
# Decoder (iMAP* MLP, c_dim = 0)
# --------------------------------------------------------------------------------------------
def init_params(seed: int = 0) -> Params:
    """Random init with the reference's distributions: B ~ N(0,1)*25 (decoder.py:21-22),
    xavier_uniform with relu / linear gain and zero bias (decoder.py:75-79)."""
    g = torch.Generator().manual_seed(seed)
    p: Params = {'embedder._B': torch.randn((3, N_FOURIER), generator=g) * 25}
    dims = [(N_FOURIER, HIDDEN)] + [(HIDDEN, HIDDEN)] * (N_LAYERS - 1)
    for li, (fi, fo) in enumerate(dims):
        bound = math.sqrt(2.0) * math.sqrt(6.0 / (fi + fo))
        p[f'pts_linears.{li}.weight'] = (torch.rand((fo, fi), generator=g) * 2 - 1) * bound
        p[f'pts_linears.{li}.bias'] = torch.zeros(fo)
    bound = math.sqrt(6.0 / (HIDDEN + 4))
    p['output_linear.weight'] = (torch.rand((4, HIDDEN), generator=g) * 2 - 1) * bound
    p['output_linear.bias'] = torch.zeros(4)
    return p


def mlp_forward(params: Params, p: torch.Tensor) -> torch.Tensor:
    """src/conv_onet/models/decoder.py:177-203 (c_dim=0, skips=[], color=True) with the Fourier
    embedding of decoder.py:26-30.  p: (P,3) any float dtype -> raw (P,4) float32."""
    x = p.reshape(-1, 3).float()
    h = torch.sin(x @ params['embedder._B'])
    for li in range(N_LAYERS):
        h = F.relu(F.linear(h, params[f'pts_linears.{li}.weight'], params[f'pts_linears.{li}.bias']))
    return F.linear(h, params['output_linear.weight'], params['output_linear.bias'])


class _RoundF32(torch.autograd.Function):
    """float64 -> float32 rounding with the gradient rounded the same way on the way back."""

    @staticmethod
    def forward(ctx, x):
        return x.float()

    @staticmethod
    def backward(ctx, g):
        return g.double()


class _FourierArgCR(torch.autograd.Function):
    """x @ B in the reference's float32 arithmetic (decoder.py:26-30: the same float32 argument as
    the reference), with the backward's two GEMMs -- dL/dB = x^T g over all points and dL/dx =
    g B^T -- summed in float64 and rounded to float32 (correctly rounded, like every other GEMM of
    mlp_forward_cr)."""

    @staticmethod
    def forward(ctx, x, B):
        ctx.save_for_backward(x, B)
        return x @ B

    @staticmethod
    def backward(ctx, g):
        x, B = ctx.saved_tensors
        gd = g.double()
        return (gd @ B.double().t()).float(), (x.double().t() @ gd).float()


def fourier_arg_cr(x: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    return _FourierArgCR.apply(x, B)


def mlp_forward_cr(params: Params, p: torch.Tensor) -> torch.Tensor:
    """mlp_forward with every GEMM CORRECTLY ROUNDED: the hidden and output layers sum in float64
    and round each layer's output (and, in the backward, each layer's input gradient) to float32;
    the Fourier argument x @ B stays the reference's float32 product (decoder.py:26-30), its
    backward GEMMs (dL/dB, dL/dx) are correctly rounded too (fourier_arg_cr).  Not the
    reference's arithmetic -- its float32 sums carry their own rounding -- but the same function
    without summation-order noise: the yardstick for fp32-class gradients
    (tests/golden/make_grads_cr.py)."""
    x = p.reshape(-1, 3).float()
    h = torch.sin(fourier_arg_cr(x, params['embedder._B']))
    for li in range(N_LAYERS):
        h = _RoundF32.apply(F.relu(F.linear(h.double(), params[f'pts_linears.{li}.weight'].double(),
                                            params[f'pts_linears.{li}.bias'].double())))
    return _RoundF32.apply(F.linear(h.double(), params['output_linear.weight'].double(),
                                    params['output_linear.bias'].double()))


def eval_points_cr(params: Params, p: torch.Tensor, bound: torch.Tensor) -> torch.Tensor:
    """eval_points on mlp_forward_cr (bound mask and sigma := 100 as the reference)."""
    ret = mlp_forward_cr(params, p).clone()
    ret[~inside_bound(p, bound), 3] = OUT_OF_BOUND_SIGMA
    return ret


def inside_bound(p: torch.Tensor, bound: torch.Tensor) -> torch.Tensor:
    """src/utils/Renderer.py:43-46: strict inequalities, evaluated in p's dtype (float64)."""
    m = torch.ones(p.shape[0], dtype=torch.bool)
    for a in range(3):
        m &= (p[:, a] < bound[a][1]) & (p[:, a] > bound[a][0])
    return m


def eval_points(params: Params, p: torch.Tensor, bound: torch.Tensor,
                points_batch_size: int = 500000) -> torch.Tensor:
    """src/utils/Renderer.py:23-61: chunked MLP query; density := 100 outside the bound (no grad)."""
    outs = []
    for chunk in torch.split(p, points_batch_size):
        ret = mlp_forward(params, chunk)
        mask = inside_bound(chunk, bound)
        ret = ret.clone()
        ret[~mask, 3] = OUT_OF_BOUND_SIGMA
        outs.append(ret)
    return torch.cat(outs, 0)


# --------------------------------------------------------------------------------------------
# Volume rendering
# --------------------------------------------------------------------------------------------
def composite(raw: torch.Tensor, z: torch.Tensor, rays_d: torch.Tensor):
    """src/common.py:204-245 (occupancy=False): NeRF alpha compositing.
    raw (N,S,4) f32, z (N,S) f64, rays_d (N,3) f32 -> depth f64, var f64, rgb f32, weights f32."""
    dists = (z[..., 1:] - z[..., :-1]).float()
    dists = torch.cat([dists, torch.full_like(dists[..., :1], 1e10)], -1)
    dists = dists * torch.norm(rays_d[..., None, :], dim=-1)
    alpha = 1. - torch.exp(-F.relu(raw[..., -1]) * dists)
    trans = torch.cumprod(torch.cat([torch.ones_like(alpha[:, :1]), 1. - alpha + 1e-10], -1), -1)[:, :-1]
    w = alpha * trans
    rgb = torch.sum(w[..., None] * raw[..., :-1], -2)
    depth = torch.sum(w * z, -1)
    dz = z - depth.unsqueeze(-1)
    var = torch.sum(w * dz * dz, dim=1)
    return depth, var, rgb, w


def sample_pdf(bins: torch.Tensor, weights: torch.Tensor, n: int, det: bool = True,
               u: Optional[torch.Tensor] = None) -> torch.Tensor:
    """src/common.py:19-63: inverse-CDF sampling.  bins (N,M+1) f64, weights (N,M) f32.
    `u` may be passed in explicitly (det=False case), else linspace(0,1,n) f32."""
    w = weights + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    if u is None:
        u = torch.linspace(0., 1., steps=n) if det else torch.rand(list(cdf.shape[:-1]) + [n])
        u = u.expand(list(cdf.shape[:-1]) + [n])
    u = u.contiguous()
    idx = torch.searchsorted(cdf, u, right=True)
    lo = torch.clamp(idx - 1, min=0)
    hi = torch.clamp(idx, max=cdf.shape[-1] - 1)
    ig = torch.stack([lo, hi], -1)
    shape = [ig.shape[0], ig.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(shape), 2, ig)
    bins_g = torch.gather(bins.unsqueeze(1).expand(shape), 2, ig)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    return bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])


def near_far(rays_o, rays_d, bound: torch.Tensor, n_samples: int, gt_depth=None, far_clamp=None):
    """src/utils/Renderer.py:90-116.  near: 0.01 (python float) or 0.01*gt (N,S) f32;
    far: (N,1) f64 box exit + 0.01, clamped to [0, max(1.2*gt)] (batch-global) when gt given.
    `far_clamp` replaces that batch max (the sharded-batch extension of pnr.Renderer)."""
    with torch.no_grad():
        t = (bound.unsqueeze(0) - rays_o.detach().unsqueeze(-1)) / rays_d.detach().unsqueeze(-1)
        far_bb = torch.min(torch.max(t, dim=2)[0], dim=1)[0].unsqueeze(-1) + 0.01
    if gt_depth is None:
        return 0.01, far_bb
    g = gt_depth.reshape(-1, 1)
    near = g.repeat(1, n_samples) * 0.01
    hi = (g * 1.2).max() if far_clamp is None else torch.tensor(far_clamp, dtype=torch.float64)
    far = torch.clamp(far_bb, 0, hi)
    return near, far


def render_batch_ray(params: Params, rays_d, rays_o, bound, n_samples=32, n_importance=12,
                     gt_depth=None, perturb=0.0, lindisp=False, t_rand=None,
                     return_extras=False, points_batch_size=500000, far_clamp=None, eval_fn=None):
    """src/utils/Renderer.py:63-203 (N_surface=0 path; occupancy=False).
    Returns (depth f64 (N,), uncertainty f64 (N,), color f32 (N,3)) [, extras].
    `eval_fn(p) -> raw` replaces the decoder query (e.g. ref_points.eval_points_c for the
    neural-point decoder); default: the reference MLP through `eval_points`."""
    if eval_fn is None:
        eval_fn = lambda q: eval_points(params, q, bound, points_batch_size)  # noqa: E731
    near, far = near_far(rays_o, rays_d, bound, n_samples, gt_depth, far_clamp)
    t_vals = torch.linspace(0., 1., steps=n_samples)
    if not lindisp:
        z = near * (1. - t_vals) + far * t_vals
    else:
        z = 1. / (1. / near * (1. - t_vals) + 1. / far * t_vals)
    if perturb > 0.:
        mids = .5 * (z[..., 1:] + z[..., :-1])
        upper = torch.cat([mids, z[..., -1:]], -1)
        lower = torch.cat([z[..., :1], mids], -1)
        if t_rand is None:
            t_rand = torch.rand(z.shape)
        z = lower + (upper - lower) * t_rand
    N = rays_o.shape[0]
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
    raw = eval_fn(pts.reshape(-1, 3)).reshape(N, z.shape[1], -1)
    depth, var, rgb, w = composite(raw, z, rays_d)
    extras = {'near': near, 'far': far, 'z_coarse': z, 'raw_coarse': raw, 'w_coarse': w}
    if n_importance > 0:
        z_mid = .5 * (z[..., 1:] + z[..., :-1])
        z_s = sample_pdf(z_mid, w[..., 1:-1], n_importance, det=(perturb == 0.)).detach()
        z, _ = torch.sort(torch.cat([z, z_s], -1), -1)
        pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
        raw = eval_fn(pts.reshape(-1, 3)).reshape(N, z.shape[1], -1)
        depth, var, rgb, w = composite(raw, z, rays_d)
        extras.update({'z_samples': z_s, 'z_fine': z, 'raw_fine': raw, 'w_fine': w})
    if return_extras:
        return depth, var, rgb, extras
    return depth, var, rgb


def regulation(params: Params, rays_d, rays_o, gt_depth, bound, n_samples=32, t_rand=None, eval_fn=None):
    """src/utils/Renderer.py:263-301: density at 32 jittered samples in [0, 0.85*gt] (f32 z).
    `t_rand` (N,n_samples) f32 replaces the reference's torch.rand draw at :293."""
    if eval_fn is None:
        eval_fn = lambda q: eval_points(params, q, bound)  # noqa: E731
    g = gt_depth.reshape(-1, 1).repeat(1, n_samples)
    t_vals = torch.linspace(0., 1., steps=n_samples)
    z = 0.0 * (1. - t_vals) + (g * 0.85) * t_vals
    mids = .5 * (z[..., 1:] + z[..., :-1])
    upper = torch.cat([mids, z[..., -1:]], -1)
    lower = torch.cat([z[..., :1], mids], -1)
    if t_rand is None:
        t_rand = torch.rand(z.shape)
    z = lower + (upper - lower) * t_rand
    pts = rays_o[..., None, :] + rays_d[..., None, :] * z[..., :, None]
    return eval_fn(pts.reshape(-1, 3))[:, -1]


def render_img(params: Params, c2w, bound, H, W, fx, fy, cx, cy, gt_depth=None,
               n_samples=32, n_importance=12, ray_batch_size=100000):
    """src/utils/Renderer.py:205-260: full-frame chunked render (no grad)."""
    with torch.no_grad():
        ro, rd = full_frame_rays(H, W, fx, fy, cx, cy, c2w)
        ro, rd = ro.reshape(-1, 3), rd.reshape(-1, 3)
        gt = None if gt_depth is None else gt_depth.reshape(-1)
        ds, vs, cs = [], [], []
        for s in range(0, rd.shape[0], ray_batch_size):
            g = None if gt is None else gt[s:s + ray_batch_size]
            d, v, c = render_batch_ray(params, rd[s:s + ray_batch_size], ro[s:s + ray_batch_size],
                                       bound, n_samples, n_importance, gt_depth=g)
            ds.append(d.double()); vs.append(v.double()); cs.append(c)
        return (torch.cat(ds).reshape(H, W), torch.cat(vs).reshape(H, W), torch.cat(cs).reshape(H, W, 3))


# --------------------------------------------------------------------------------------------
# Caller losses (A14)
# --------------------------------------------------------------------------------------------
def mapping_loss(depth, color, gt_depth, gt_color, sigma_reg, w_color=0.05, w_reg=0.0005):
    """src/Mapper.py:641-655 (depth_supervision=True, occupancy=False): summed L1 losses."""
    m = gt_depth > 0
    loss = torch.abs(gt_depth[m] - depth[m]).sum()
    loss = loss + w_color * torch.abs(gt_color - color).sum()
    return loss + w_reg * torch.abs(sigma_reg).sum()


def tracking_loss(depth, var, color, gt_depth, gt_color, w_color=0.5):
    """src/Tracker.py:306-330 (handle_dynamic=False, depth_supervision=True)."""
    m = gt_depth > 0
    var = var.detach()
    loss = (torch.abs(gt_depth - depth) / torch.sqrt(var + 1e-10))[m].sum()
    return loss + w_color * torch.abs(gt_color - color)[m].sum()


def psnr(a: torch.Tensor, b: torch.Tensor, mask: Optional[torch.Tensor] = None) -> float:
    """-10 log10(MSE) on RGB in [0,1] (no PSNR exists in the reference)."""
    d = (a.double() - b.double()) ** 2
    if mask is not None:
        d = d[mask]
    mse = float(d.mean())
    return float('inf') if mse == 0 else -10.0 * math.log10(mse)
