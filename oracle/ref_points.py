"""CPU restatement of the neural-point feature stage -- TEST INFRASTRUCTURE ONLY.

SURVEY.md §8 row A15.  The reference has no neural-point gather (its `run.py` decoder has
c_dim=0); the stage is build-defined, and this module is its specification:

  * neural points x_i (M,3) f32 with features f_i (M,C) f32;
  * for a sample p (cast to f32 first, like `p.float()` at src/conv_onet/models/decoder.py:189):
      delta_i = p - x_i (f32), d2_i = (dx*dx + dy*dy) + dz*dz (f32, no fma);
  * neighbourhood  'idw':       d2_i <= radius^2                      (Euclidean ball)
                   'trilinear': |delta_i,a| < spacing_a on every axis (the 8 corners of the
                                grid cell holding p when the points sit on a lattice);
  * the (up to) K neighbours with the smallest (d2_i, i), in that order;
  * weights        'idw':       w_i = 1 / max(sqrt(d2_i), eps)
                   'trilinear': w_i = (1-|dx|/hx) * (1-|dy|/hy) * (1-|dz|/hz);
  * c(p) = sum_k (w_k / W) f_k with W = w_0 + w_1 + ... (sequential, ascending distance);
    c(p) = 0 when p has no neighbour;
  * the decoder then injects c into every hidden layer, h = relu(W_i h + b_i) + fc_c[i](c)
    (decoder.py:191-197, fc_c built at :122-125).

With the points on the vertices of a feature grid and the trilinear kernel, c(p) equals the
reference's `MLP.sample_grid_feature` (decoder.py:168-175, `F.grid_sample`, align_corners=True)
on interior samples: that pin, and the full MLP(c_dim=32) forward/backward around it, are checked
against reference outputs in tests/golden/points_c32.npz (tests/golden/make_golden_points.py).
The IDW weighting has no reference counterpart; it is pinned only by this restatement.

Brute force over all points (no spatial hash: the hash is an acceleration structure and does not
change the result), in torch so that autograd gives the backward.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .ref_render import N_LAYERS, OUT_OF_BOUND_SIGMA, inside_bound

Params = Dict[str, torch.Tensor]
C_DIM = 32

# ---- summation magnitudes (test yardstick) ---------------------------------------------------
# Every gradient of the decoder parameters and of the point features is a sum over samples, g =
# sum_p t_p.  Rounded in any order, float32 arithmetic leaves an error of order u sum_p |t_p|
# (u = 2^-24), which a relative bound on g alone cannot express where the sum cancels (|g| <<
# sum_p |t_p|).  While `magnitudes()` is active, mlp_forward_c and point_gather record, per
# gradient element, M = sum_p |t_p| (|delta|^T |h| for a weight, sum |delta| for a bias, sum |w_k|
# |dL/dc| for a feature row) by tensor hooks on the float32 oracle's graph; the GPU parity tests add
# a floor of a few ulps of M to their elementwise tolerance.
_MAG: Optional[Dict[str, torch.Tensor]] = None


class magnitudes:
    """Context manager: `with magnitudes() as m:` -- after the backward, m[name] holds M for the
    parameter `name` (and m['feats'] for the point features), summed over every call."""

    def __enter__(self):
        global _MAG
        _MAG = {}
        return _MAG

    def __exit__(self, *exc):
        global _MAG
        _MAG = None
        return False


def _mag_add(name: str, v: torch.Tensor) -> None:
    m = _MAG
    if m is None:
        return
    v = v.detach().double()
    m[name] = m[name] + v if name in m else v


def _mag_linear(out: torch.Tensor, inp: torch.Tensor, wname: str, bname: Optional[str]) -> None:
    """out = inp W^T + b: |dL/dout|^T |inp| for W, sum |dL/dout| for b."""
    if _MAG is None or not out.requires_grad:
        return
    a = inp.detach().abs().double()

    def hook(g):
        ga = g.detach().abs().double()
        _mag_add(wname, ga.t() @ a)
        if bname is not None:
            _mag_add(bname, ga.sum(0))
    out.register_hook(hook)


def init_fc_c(params: Params, seed: int = 1, c_dim: int = C_DIM, hidden: int = 256) -> Params:
    """Add `fc_c.{i}` (nn.Linear(c_dim, hidden), decoder.py:122-125) with torch's default Linear
    init: weight and bias ~ U(-1/sqrt(c_dim), 1/sqrt(c_dim))."""
    g = torch.Generator().manual_seed(seed)
    b = 1.0 / math.sqrt(c_dim)
    out = dict(params)
    for i in range(N_LAYERS):
        out[f'fc_c.{i}.weight'] = (torch.rand((hidden, c_dim), generator=g) * 2 - 1) * b
        out[f'fc_c.{i}.bias'] = (torch.rand((hidden,), generator=g) * 2 - 1) * b
    return out


def grid_vertices(bound: torch.Tensor, D: int, H: int, W: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Positions (D*H*W, 3) f32 of the vertices of a `align_corners=True` grid over `bound`, in the
    flattening order of grid[0, :, d, h, w] (x <-> w, y <-> h, z <-> d), and the per-axis
    spacing (3,) f32."""
    lo, hi = bound[:, 0].double(), bound[:, 1].double()
    n = torch.tensor([W - 1, H - 1, D - 1], dtype=torch.float64)
    sp = (hi - lo) / n
    d, h, w = torch.meshgrid(torch.arange(D), torch.arange(H), torch.arange(W), indexing='ij')
    idx = torch.stack([w, h, d], -1).reshape(-1, 3).double()
    return (lo + idx * sp).float(), sp.float()


def grid_features(grid: torch.Tensor) -> torch.Tensor:
    """(1,C,D,H,W) -> (D*H*W, C), rows in `grid_vertices` order."""
    C = grid.shape[1]
    return grid[0].reshape(C, -1).t()


def select_neighbours(p: torch.Tensor, xyz: torch.Tensor, mode: str = 'idw', radius: float = 0.0,
                      spacing=None, k: int = 8, chunk: int = 1024):
    """Neighbour search (no grad).  Returns idx (P,K) int64 (-1 = none), in ascending (d2, i)."""
    pf = p.detach().reshape(-1, 3).float()
    x = xyz.detach().float()
    P = pf.shape[0]
    idx = torch.full((P, k), -1, dtype=torch.int64)
    r2 = torch.tensor(radius, dtype=torch.float32) * torch.tensor(radius, dtype=torch.float32)
    if spacing is not None:
        spacing = torch.as_tensor(spacing, dtype=torch.float32)
    for s in range(0, P, chunk):
        q = pf[s:s + chunk]
        dl = q[:, None, :] - x[None, :, :]                       # (c, M, 3) f32
        d2 = (dl[..., 0] * dl[..., 0] + dl[..., 1] * dl[..., 1]) + dl[..., 2] * dl[..., 2]
        if mode == 'idw':
            ok = d2 <= r2
        elif mode == 'trilinear':
            ok = (dl.abs() < spacing).all(-1)
        else:
            raise ValueError(mode)
        key = torch.where(ok, d2, torch.full_like(d2, float('inf')))
        srt, order = torch.sort(key, dim=1, stable=True)
        kk = min(k, order.shape[1])
        sel = order[:, :kk]
        sel = torch.where(torch.isfinite(srt[:, :kk]), sel, torch.full_like(sel, -1))
        idx[s:s + chunk, :kk] = sel
    return idx


def neighbour_weights(p: torch.Tensor, xyz: torch.Tensor, idx: torch.Tensor, mode: str = 'idw',
                      spacing=None, eps: float = 1e-6) -> torch.Tensor:
    """Normalised weights (P,K) f32, differentiable w.r.t. p (f32 arithmetic, no fma)."""
    pf = p.reshape(-1, 3).float()
    valid = idx >= 0
    xi = xyz.float()[idx.clamp(min=0)]                           # (P,K,3)
    dl = pf[:, None, :] - xi
    if mode == 'idw':
        d2 = (dl[..., 0] * dl[..., 0] + dl[..., 1] * dl[..., 1]) + dl[..., 2] * dl[..., 2]
        # sqrt has an infinite derivative at 0; the clamp makes it irrelevant there
        d = torch.sqrt(torch.clamp(d2, min=eps * eps * 0.25))
        w = 1.0 / torch.clamp(d, min=eps)
    else:
        sp = torch.as_tensor(spacing, dtype=torch.float32)
        t = 1.0 - dl.abs() / sp
        w = (t[..., 0] * t[..., 1]) * t[..., 2]
    w = torch.where(valid, w, torch.zeros_like(w))
    # sequential sum in neighbour order
    W = torch.zeros(w.shape[0], dtype=torch.float32)
    for j in range(w.shape[1]):
        W = W + w[:, j]
    W = torch.where(W > 0, W, torch.ones_like(W))
    return w / W[:, None]


def point_gather(p: torch.Tensor, xyz: torch.Tensor, feats: torch.Tensor, mode: str = 'idw',
                 radius: float = 0.0, spacing=None, k: int = 8, eps: float = 1e-6,
                 return_idx: bool = False):
    """c(p) (P,C) f32 -- see the module docstring.  Differentiable w.r.t. p and feats."""
    idx = select_neighbours(p, xyz, mode, radius, spacing, k)
    wn = neighbour_weights(p, xyz, idx, mode, spacing, eps)
    fk = feats.float()[idx.clamp(min=0)]                         # (P,K,C)
    c = torch.zeros(fk.shape[0], fk.shape[2], dtype=torch.float32)
    for j in range(idx.shape[1]):                                # sequential, ascending distance
        c = c + wn[:, j:j + 1] * fk[:, j]
    if _MAG is not None and c.requires_grad:
        wa = torch.where(idx >= 0, wn.detach().abs(), torch.zeros_like(wn)).double()
        ic = idx.clamp(min=0).reshape(-1)
        M = feats.shape[0]

        def hook(g):  # M_feats[i] += |w_k| |dL/dc| over the samples whose neighbour k is point i
            t = (wa[:, :, None] * g.detach().abs().double()[:, None, :]).reshape(-1, g.shape[1])
            _mag_add('feats', torch.zeros((M, g.shape[1]), dtype=torch.float64).index_add_(0, ic, t))
        c.register_hook(hook)
    if return_idx:
        return c, idx, wn
    return c


def mlp_forward_c(params: Params, p: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """decoder.py:177-203 with c_dim != 0, skips=[], color=True: h = relu(W h + b) + fc_c[i](c)."""
    x = p.reshape(-1, 3).float()
    arg = x @ params['embedder._B']
    _mag_linear(arg, x, 'embedder._B.T', None)
    h = torch.sin(arg)
    for li in range(N_LAYERS):
        z = F.linear(h, params[f'pts_linears.{li}.weight'], params[f'pts_linears.{li}.bias'])
        _mag_linear(z, h, f'pts_linears.{li}.weight', f'pts_linears.{li}.bias')
        zc = F.linear(c, params[f'fc_c.{li}.weight'], params[f'fc_c.{li}.bias'])
        _mag_linear(zc, c, f'fc_c.{li}.weight', f'fc_c.{li}.bias')
        h = F.relu(z) + zc
    out = F.linear(h, params['output_linear.weight'], params['output_linear.bias'])
    _mag_linear(out, h, 'output_linear.weight', 'output_linear.bias')
    return out


def mlp_forward_c_cr(params: Params, p: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """mlp_forward_c with every hidden, fc_c and output GEMM CORRECTLY ROUNDED (float64 sums, each
    layer's output rounded to float32; in the backward each layer's input gradient, and dL/dc =
    sum_l Wc_l^T dL/dh_l, rounded likewise).  The yardstick for fp32-class feature-branch gradients
    (tests/golden/make_grads_cr.py), like ref_render.mlp_forward_cr for the c_dim = 0 decoder."""
    from .ref_render import _RoundF32, fourier_arg_cr
    x = p.reshape(-1, 3).float()
    h = torch.sin(fourier_arg_cr(x, params['embedder._B']))
    cd = c.double()
    for li in range(N_LAYERS):
        a = F.relu(F.linear(h.double(), params[f'pts_linears.{li}.weight'].double(),
                            params[f'pts_linears.{li}.bias'].double()))
        a = a + F.linear(cd, params[f'fc_c.{li}.weight'].double(), params[f'fc_c.{li}.bias'].double())
        h = _RoundF32.apply(a)
    return _RoundF32.apply(F.linear(h.double(), params['output_linear.weight'].double(),
                                    params['output_linear.bias'].double()))


def magnitude_of(m: Dict[str, torch.Tensor], name: str) -> torch.Tensor:
    """M for parameter `name` in its own shape (embedder._B is recorded transposed)."""
    if name == 'embedder._B':
        return m['embedder._B.T'].t()
    return m[name]


def eval_points_c(params: Params, p: torch.Tensor, bound: torch.Tensor, points: dict, cr: bool = False) -> torch.Tensor:
    """src/utils/Renderer.py:23-61 with the neural-point features: raw (P,4) f32, density := 100
    outside the bound.  `points` = dict(xyz, feats, mode, radius, spacing, k, eps).  cr: the decoder
    GEMMs correctly rounded (mlp_forward_c_cr; test yardstick)."""
    c = point_gather(p, points['xyz'], points['feats'], points.get('mode', 'idw'),
                     points.get('radius', 0.0), points.get('spacing'), points.get('k', 8),
                     points.get('eps', 1e-6))
    ret = (mlp_forward_c_cr if cr else mlp_forward_c)(params, p, c).clone()
    mask = inside_bound(p.reshape(-1, 3), bound)
    ret[~mask, 3] = OUT_OF_BOUND_SIGMA
    return ret
