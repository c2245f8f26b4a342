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
    if return_idx:
        return c, idx, wn
    return c


def mlp_forward_c(params: Params, p: torch.Tensor, c: torch.Tensor) -> torch.Tensor:
    """decoder.py:177-203 with c_dim != 0, skips=[], color=True: h = relu(W h + b) + fc_c[i](c)."""
    x = p.reshape(-1, 3).float()
    h = torch.sin(x @ params['embedder._B'])
    for li in range(N_LAYERS):
        h = F.relu(F.linear(h, params[f'pts_linears.{li}.weight'], params[f'pts_linears.{li}.bias']))
        h = h + F.linear(c, params[f'fc_c.{li}.weight'], params[f'fc_c.{li}.bias'])
    return F.linear(h, params['output_linear.weight'], params['output_linear.bias'])


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
