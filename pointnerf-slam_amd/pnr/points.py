"""Neural points: positions + learnable features, gathered per sample on the HIP path.

SURVEY.md §8 row A15 (build-defined; the reference has no neural-point stage).  The decoder's
feature input c(p) is aggregated from the k nearest points around p (include/pnr.h `pnr_points`,
oracle/ref_points.py is the spec):

  mode='idw'        points within `radius`, weights 1/max(|p-x|, eps)
  mode='trilinear'  points within one lattice `spacing` per axis, weights prod(1-|dp|/h) --
                    with points on the vertices of a feature grid this is the reference's
                    MLP.sample_grid_feature (src/conv_onet/models/decoder.py:168-175)

A `NeuralPoints` rides in the Renderer's `c` dict under 'points_<decoder name>' (an empty dict
keeps the reference behaviour).  Features are an nn.Parameter; gradients reach them (and the
sample positions, for tracking) through the gather backward.  The spatial hash (pnr_points_build)
is rebuilt on the device whenever the positions change.
"""
from __future__ import annotations

import ctypes
import math

import torch
import torch.nn as nn

from . import _lib

_MODES = {'idw': _lib.GATHER_IDW, 'trilinear': _lib.GATHER_TRILINEAR}


class NeuralPoints(nn.Module):
    def __init__(self, xyz: torch.Tensor, feats: torch.Tensor = None, c_dim: int = 32, mode: str = 'idw',
                 k: int = 8, radius: float = 0.02, eps: float = 1e-6, spacing=None, cell: float = None,
                 origin=None, table_bits: int = None, feat_dtype: str = 'float32'):
        super().__init__()
        if feat_dtype not in ('float32', 'float16'):
            raise ValueError("pnr.NeuralPoints: feat_dtype must be 'float32' or 'float16'")
        if c_dim != _lib.C_DIM:
            raise NotImplementedError(f'pnr.NeuralPoints: c_dim must be {_lib.C_DIM}')
        if mode not in _MODES:
            raise ValueError(f'pnr.NeuralPoints: mode must be one of {sorted(_MODES)}')
        if not 1 <= k <= _lib.MAX_K:
            raise ValueError(f'pnr.NeuralPoints: 1 <= k <= {_lib.MAX_K}')
        xyz = xyz.detach().float().reshape(-1, 3).contiguous()
        M = xyz.shape[0]
        self.register_buffer('xyz', xyz)
        if feats is None:
            feats = torch.zeros((M, c_dim), device=xyz.device)
        self.feats = nn.Parameter(feats.detach().float().reshape(M, c_dim).contiguous().clone())
        self.mode = mode
        self.k = int(k)
        self.radius = float(radius)
        self.eps = float(eps)
        self.spacing = [float(v) for v in (spacing if spacing is not None else (radius, radius, radius))]
        reach = self.radius if mode == 'idw' else max(self.spacing)
        # the search probes the 2x2x2 cells covering [p - reach, p + reach]: cell >= 2 reach, with a
        # margin so that float rounding of the cell coordinates never misses a neighbour
        # (points.hip kCellMargin: the search's widened reach must stay within half a cell)
        self.cell = float(cell) if cell is not None else 2.0 * reach * (1.0 + 4e-3)
        if self.cell < 2.0 * reach * (1.0 + 2.0 ** -9):
            raise ValueError('pnr.NeuralPoints: cell must be >= 2 x the neighbourhood reach x (1 + 2^-9)')
        if origin is None:
            origin = (xyz.min(0).values - self.cell).tolist() if M > 0 else [0.0, 0.0, 0.0]
        self.origin = [float(v) for v in origin]
        if table_bits is None:  # ~2 buckets per occupied cell (a surface cell holds ~4-16 points)
            table_bits = min(24, max(10, int(math.ceil(math.log2(max(M // 2, 1))))))
        self.table_bits = int(table_bits)
        self._index = None
        self._index_key = None
        # float16 features (the C5 budget): the gather reads an f16 copy of the fp32
        # master `feats` (the optimiser's parameter); the copy is refreshed when feats changed
        self.feat_dtype = feat_dtype
        self._feats_h = None
        self._feats_h_key = None

    def invalidate_feats(self):
        """Mark the f16 copy stale (after an in-place update torch does not version, e.g. the
        pnr Adam kernel writing through a raw pointer)."""
        self._feats_h_key = None

    def mark_feats_fresh(self):
        """The f16 copy holds float16(feats) again (written by pnr_adam_multi_dev_h with the master)."""
        if self._feats_h is not None:
            self._feats_h_key = (self.feats.data_ptr(), self.feats._version)

    def _feats_for_gather(self):
        if self.feat_dtype == 'float32':
            return self.feats
        f = self.feats
        key = (f.data_ptr(), f._version)
        if self._feats_h is None or self._feats_h.shape != f.shape or self._feats_h.device != f.device:
            self._feats_h = torch.empty(f.shape, dtype=torch.float16, device=f.device)
            self._feats_h_key = None
        if self._feats_h_key != key:
            with torch.no_grad():
                self._feats_h.copy_(f)
            self._feats_h_key = key
        return self._feats_h

    @classmethod
    def from_grid(cls, grid: torch.Tensor, bound: torch.Tensor, **kw):
        """Points on the vertices of an align_corners=True feature grid (1,C,D,H,W) over `bound`
        (x <-> W, y <-> H, z <-> D), trilinear weights: reproduces F.grid_sample on interior samples."""
        _, C, D, H, W = grid.shape
        b = torch.as_tensor(bound, dtype=torch.float64).reshape(3, 2).cpu()
        lo, hi = b[:, 0], b[:, 1]
        sp = (hi - lo) / torch.tensor([W - 1, H - 1, D - 1], dtype=torch.float64)
        d, h, w = torch.meshgrid(torch.arange(D), torch.arange(H), torch.arange(W), indexing='ij')
        ijk = torch.stack([w, h, d], -1).reshape(-1, 3).double()
        xyz = (lo + ijk * sp).float().to(grid.device)
        feats = grid[0].reshape(C, -1).t().contiguous()
        return cls(xyz, feats, c_dim=C, mode='trilinear', spacing=sp.float().tolist(), **kw)

    # -- device index -----------------------------------------------------------------------------
    def _struct(self) -> _lib.Points:
        s = _lib.Points()
        s.xyz = self.xyz.data_ptr()
        s.feats = self._feats_for_gather().data_ptr()
        s.feat_half = 1 if self.feat_dtype == 'float16' else 0
        s.n_points = self.xyz.shape[0]
        s.mode = _MODES[self.mode]
        s.k = self.k
        s.radius = self.radius
        s.eps = self.eps
        for i in range(3):
            s.spacing[i] = self.spacing[i]
            s.origin[i] = self.origin[i]
        s.cell = self.cell
        s.table_bits = self.table_bits
        return s

    def index(self) -> torch.Tensor:
        """The spatial hash (device bytes), rebuilt when positions or the hash layout changed."""
        _lib.require_cuda(self.xyz)
        key = (self.xyz.data_ptr(), self.xyz._version, self.cell, tuple(self.origin), self.table_bits)
        if self._index is not None and key == self._index_key:
            return self._index
        lib = _lib.load()
        nbytes = lib.pnr_points_index_bytes(self.xyz.shape[0], self.table_bits)
        if self._index is None or self._index.numel() < nbytes or self._index.device != self.xyz.device:
            self._index = torch.empty(nbytes, dtype=torch.uint8, device=self.xyz.device)
        s = self._struct()
        s.index = self._index.data_ptr()
        _lib.check(lib.pnr_points_build(ctypes.byref(s), _lib.stream_of(self.xyz.device)), 'points_build')
        self._index_key = key
        return self._index

    def descriptor(self, fc_packed=None, g_feats=None, g_fc=None):
        """(pnr_points struct, keep-alive list) for one C call."""
        s = self._struct()
        s.index = self.index().data_ptr()
        keep = []
        if fc_packed is not None:
            s.fc_packed = fc_packed.data_ptr()
        if g_feats is not None:
            s.g_feats = g_feats.data_ptr()
        if g_fc is not None:
            arr = _lib.FcPtrArray(*[t.data_ptr() for t in g_fc])
            keep.append(arr)
            s.g_fc = ctypes.cast(arr, ctypes.c_void_p).value
        return s, keep

    def gather(self, p: torch.Tensor) -> torch.Tensor:
        """c(p) (P,32) float32 for points p (P,3); differentiable w.r.t. p and `feats`."""
        p = p.reshape(-1, 3)
        _lib.require_cuda(p)
        return _GatherFn.apply(p.double().contiguous(), self, self.feats)

    def __getstate__(self):
        st = self.__dict__.copy()
        st['_index'] = None  # device caches never cross pickling / deepcopy
        st['_index_key'] = None
        st['_feats_h'] = None
        st['_feats_h_key'] = None
        return st


class _GatherFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, p, pts, feats):
        lib = _lib.load()
        P = p.shape[0]
        dev = p.device
        c = torch.empty((P, _lib.C_DIM), device=dev, dtype=torch.float32)
        need = any(ctx.needs_input_grad)
        idx = torch.empty((P, pts.k), device=dev, dtype=torch.int32) if need else None
        w = torch.empty((P, pts.k), device=dev, dtype=torch.float32) if need else None
        s, keep = pts.descriptor()
        ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
        _lib.check(lib.pnr_point_gather(ctypes.byref(s), _lib.ptr(p), P, _lib.ptr(c), _lib.ptr(idx), _lib.ptr(w),
                                        _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)), 'point_gather')
        if need:
            ctx.pts = pts
            ctx.save_for_backward(p, idx, w, c)
        return c

    @staticmethod
    def backward(ctx, g_c):
        lib = _lib.load()
        p, idx, w, c = ctx.saved_tensors
        pts = ctx.pts
        dev = p.device
        P = p.shape[0]
        g_feats = torch.zeros_like(pts.feats) if ctx.needs_input_grad[2] else None
        g_p = torch.empty((P, 3), device=dev, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        s, keep = pts.descriptor(g_feats=g_feats)
        ws = torch.empty(lib.pnr_point_gather_bwd_workspace_bytes(ctypes.byref(s), P), dtype=torch.uint8, device=dev)
        _lib.check(lib.pnr_point_gather_bwd(ctypes.byref(s), _lib.ptr(p), P, _lib.ptr(idx), _lib.ptr(w), _lib.ptr(c),
                                            _lib.ptr(g_c.contiguous()), _lib.ptr(g_p), _lib.ptr(ws), ws.numel(),
                                            _lib.stream_of(dev)), 'point_gather_bwd')
        return (None if g_p is None else g_p.double(), None, g_feats)


def find_points(c, decoders):
    """The NeuralPoints of decoder `decoders` in the Renderer's `c` dict (None = reference path)."""
    if not getattr(decoders, 'c_dim', 0):
        return None
    name = getattr(decoders, 'name', '')
    if isinstance(c, NeuralPoints):
        return c
    if isinstance(c, dict):
        for key in ('points_' + name, 'grid_' + name):
            v = c.get(key)
            if isinstance(v, NeuralPoints):
                return v
    raise ValueError(f"pnr: decoder '{name}' has c_dim={decoders.c_dim}: pass its NeuralPoints as "
                     f"c['points_{name}']")
