"""Drop-in decoder: the iMAP* MLP of src/conv_onet/models/decoder.py:91-203, state_dict-compatible.

`MLP` keeps the reference constructor signature and parameter names (`embedder._B`,
`pts_linears.{0..3}.{weight,bias}`, `output_linear.{weight,bias}`) so reference checkpoints
(`decoder_state_dict` written by src/utils/Logger.py:23-32) load unchanged, `copy.deepcopy`
(src/Tracker.py:349) and `.share_memory()` (src/NICE_SLAM.py:153) keep working, and
`forward(p, c_grid=None)` runs the fused HIP kernel.  Native configurations: the one
`get_model(cfg, nice=False)` builds (src/conv_onet/config.py:29-31: c_dim=0, fourier, 4 blocks,
256 hidden, color) and the same decoder with c_dim=32 neural-point features:
`fc_c.{0..3}` (decoder.py:122-125) inject the gathered features, h = relu(W h + b) + fc_c[i](c)
(decoder.py:196-197).  Other configurations are refused.
"""
from __future__ import annotations

import torch
import torch.nn as nn

from . import _lib
from .packing import PackedFC, PackedMLP
from .points import find_points

PARAM_ORDER = ('embedder._B',
               'pts_linears.0.weight', 'pts_linears.0.bias', 'pts_linears.1.weight', 'pts_linears.1.bias',
               'pts_linears.2.weight', 'pts_linears.2.bias', 'pts_linears.3.weight', 'pts_linears.3.bias',
               'output_linear.weight', 'output_linear.bias')


class GaussianFourierFeatureTransform(nn.Module):
    """decoder.py:7-30: sin(x @ B), B ~ N(0,1)*scale, learnable."""

    def __init__(self, num_input_channels, mapping_size=93, scale=25, learnable=True):
        super().__init__()
        B = torch.randn((num_input_channels, mapping_size)) * scale
        if learnable:
            self._B = nn.Parameter(B)
        else:
            self.register_buffer('_B', B)


class DenseLayer(nn.Linear):
    """decoder.py:70-79: xavier_uniform with the activation's gain, zero bias."""

    def __init__(self, in_dim: int, out_dim: int, activation: str = 'relu', *args, **kwargs) -> None:
        self.activation = activation
        super().__init__(in_dim, out_dim, *args, **kwargs)

    def reset_parameters(self) -> None:
        nn.init.xavier_uniform_(self.weight, gain=nn.init.calculate_gain(self.activation))
        if self.bias is not None:
            nn.init.zeros_(self.bias)


class _MLPFn(torch.autograd.Function):
    """raw = MLP(p) on the HIP path with the fused backward (pnr_mlp_fwd_train / pnr_mlp_bwd)."""

    @staticmethod
    def forward(ctx, p, packed_owner, prec, *params):
        lib = _lib.load()
        P = p.shape[0]
        packed = packed_owner.image(params)
        raw = torch.empty((P, 4), device=p.device, dtype=torch.float32)
        st = _lib.stream_of(p.device)
        need = any(ctx.needs_input_grad)  # (inside forward grad mode is off; ask autograd)
        if need:
            ws = torch.empty(lib.pnr_mlp_train_workspace_bytes(P), dtype=torch.uint8, device=p.device)
            _lib.check(lib.pnr_mlp_fwd_train(_lib.ptr(packed), _lib.ptr(p), P, _lib.ptr(raw), _lib.ptr(ws),
                                             ws.numel(), prec, st), 'mlp_fwd_train')
            ctx.save_for_backward(ws, packed)
            ctx.P = P
            ctx.prec = prec
            ctx.p_grad = ctx.needs_input_grad[0]
        else:
            _lib.check(lib.pnr_eval_points_f32(_lib.ptr(packed), _lib.ptr(p), P, None, _lib.ptr(raw), prec, st),
                       'mlp_fwd')
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        lib = _lib.load()
        ws, packed = ctx.saved_tensors
        P = ctx.P
        dev = g_raw.device
        grads = [torch.zeros(s, device=dev, dtype=torch.float32) for s in _MLPFn.shapes]
        gp = torch.empty((P, 3), device=dev, dtype=torch.float32) if ctx.p_grad else None
        bws = torch.empty(lib.pnr_mlp_bwd_workspace_bytes(P), dtype=torch.uint8, device=dev)
        arr = _lib.PtrArray(*[g.data_ptr() for g in grads])
        _lib.check(lib.pnr_mlp_bwd(_lib.ptr(packed), P, _lib.ptr(g_raw.contiguous()), arr, _lib.ptr(gp),
                                   _lib.ptr(ws), ws.numel(), _lib.ptr(bws), bws.numel(), ctx.prec,
                                   _lib.stream_of(dev)), 'mlp_bwd')
        return (gp, None, None, *grads)

    shapes = ((3, 93), (256, 93), (256,), (256, 256), (256,), (256, 256), (256,), (256, 256), (256,), (4, 256), (4,))


FC_ORDER = tuple(f'fc_c.{i}.{k}' for i in range(4) for k in ('weight', 'bias'))
FC_SHAPES = ((256, 32), (256,)) * 4


class _MLPFnC(torch.autograd.Function):
    """raw = MLP(p, c) with per-point features c (P,32) (pnr_mlp_fwd_train_c / pnr_mlp_bwd_c)."""

    @staticmethod
    def forward(ctx, p, c, packed_owner, fc_owner, prec, *tensors):
        lib = _lib.load()
        P = p.shape[0]
        params, fc = tensors[:_lib.N_PARAMS], tensors[_lib.N_PARAMS:]
        packed = packed_owner.image(params)
        fcp = fc_owner.image(fc)
        raw = torch.empty((P, 4), device=p.device, dtype=torch.float32)
        st = _lib.stream_of(p.device)
        if any(ctx.needs_input_grad):
            ws = torch.empty(lib.pnr_mlp_train_workspace_bytes(P), dtype=torch.uint8, device=p.device)
            _lib.check(lib.pnr_mlp_fwd_train_c(_lib.ptr(packed), _lib.ptr(fcp), _lib.ptr(p), _lib.ptr(c), P,
                                               _lib.ptr(raw), _lib.ptr(ws), ws.numel(), prec, st), 'mlp_fwd_train_c')
            ctx.save_for_backward(ws, packed, fcp, c)
            ctx.P = P
            ctx.prec = prec
        else:
            dp = p.double().contiguous()
            _lib.check(lib.pnr_eval_points_c(_lib.ptr(packed), _lib.ptr(fcp), _lib.ptr(dp), _lib.ptr(c), P, None,
                                             _lib.ptr(raw), prec, st), 'eval_points_c')
        return raw

    @staticmethod
    def backward(ctx, g_raw):
        lib = _lib.load()
        ws, packed, fcp, c = ctx.saved_tensors
        P = ctx.P
        dev = g_raw.device
        grads = [torch.zeros(s, device=dev, dtype=torch.float32) for s in _MLPFn.shapes]
        g_fc = [torch.zeros(s, device=dev, dtype=torch.float32) for s in FC_SHAPES]
        gp = torch.empty((P, 3), device=dev, dtype=torch.float32) if ctx.needs_input_grad[0] else None
        gc = torch.empty((P, _lib.C_DIM), device=dev, dtype=torch.float32) if ctx.needs_input_grad[1] else None
        bws = torch.empty(lib.pnr_mlp_bwd_workspace_bytes_c(P), dtype=torch.uint8, device=dev)
        arr = _lib.PtrArray(*[g.data_ptr() for g in grads])
        farr = _lib.FcPtrArray(*[g.data_ptr() for g in g_fc])
        _lib.check(lib.pnr_mlp_bwd_c(_lib.ptr(packed), _lib.ptr(fcp), _lib.ptr(c), P, _lib.ptr(g_raw.contiguous()),
                                     arr, farr, _lib.ptr(gc), _lib.ptr(gp), _lib.ptr(ws), ws.numel(), _lib.ptr(bws),
                                     bws.numel(), ctx.prec, _lib.stream_of(dev)), 'mlp_bwd_c')
        return (gp, gc, None, None, None, *grads, *g_fc)


class MLP(nn.Module):
    """src/conv_onet/models/decoder.py:91-203 (same signature)."""

    def __init__(self, name='', dim=3, c_dim=128, hidden_size=256, n_blocks=5, leaky=False, sample_mode='bilinear',
                 color=False, skips=[2], grid_len=0.16, pos_embedding_method='fourier', concat_feature=False):
        super().__init__()
        if not (dim == 3 and c_dim in (0, _lib.C_DIM) and hidden_size == 256 and n_blocks == 4 and color
                and not skips and not leaky and pos_embedding_method == 'fourier' and not concat_feature):
            raise NotImplementedError('pnr.MLP: only the iMAP* decoder of get_model(cfg, nice=False) '
                                      '(c_dim=0 or 32, fourier, 4x256, color, no skips) has a native path')
        self.name = name
        self.color = color
        self.no_grad_feature = False
        self.c_dim = c_dim
        self.grid_len = grid_len
        self.concat_feature = concat_feature
        self.n_blocks = n_blocks
        self.skips = skips
        self.sample_mode = sample_mode
        if c_dim != 0:  # created first, like decoder.py:122-125 (same RNG consumption order)
            self.fc_c = nn.ModuleList([nn.Linear(c_dim, hidden_size) for _ in range(n_blocks)])
            self._packed_fc = PackedFC()
        self.embedder = GaussianFourierFeatureTransform(dim, mapping_size=93, scale=25)
        self.pts_linears = nn.ModuleList([DenseLayer(93, hidden_size, activation='relu')] +
                                         [DenseLayer(hidden_size, hidden_size, activation='relu')
                                          for _ in range(n_blocks - 1)])
        self.output_linear = DenseLayer(hidden_size, 4, activation='linear')
        self._packed = PackedMLP()
        # decoder matmul arithmetic of forward() (pnr extension, not a parameter): 'fp32' | 'bf16x3' | 'bf16'
        self.precision = _lib.DEFAULT_PRECISION

    def ordered_params(self):
        sd = dict(self.named_parameters())
        return [sd[k] for k in PARAM_ORDER]

    def ordered_fc_params(self):
        sd = dict(self.named_parameters())
        return [sd[k] for k in FC_ORDER]

    def packed_fc_image(self) -> torch.Tensor:
        return self._packed_fc.image(self.ordered_fc_params())

    def packed_image(self) -> torch.Tensor:
        """The MFMA-ordered weight image (re-packed only when a parameter changed)."""
        return self._packed.image(self.ordered_params())

    def forward(self, p, c_grid=None):
        """decoder.py:177-203: p (1,P,3) or (P,3), any float dtype -> raw (P,4) float32."""
        x = p.reshape(-1, 3)
        _lib.require_cuda(x)
        params = self.ordered_params()
        if self.c_dim != 0:  # decoder.py:178-181: features first (here: neural-point gather)
            c = find_points(c_grid, self).gather(x)
            xf = x.float().contiguous()
            return _MLPFnC.apply(xf, c, self._packed, self._packed_fc, _lib.precision_code(self.precision), *params,
                                 *self.ordered_fc_params())
        x = x.float().contiguous()
        return _MLPFn.apply(x, self._packed, _lib.precision_code(self.precision), *params)

    def __getstate__(self):
        st = self.__dict__.copy()
        st['_packed'] = PackedMLP()  # device caches never cross pickling / deepcopy
        if '_packed_fc' in st:
            st['_packed_fc'] = PackedFC()
        return st


def get_model(cfg, nice=False):
    """src/config.py:63-79 -> src/conv_onet/config.py:29-31 (the `nice=False` branch)."""
    if nice:
        raise NotImplementedError('pnr.get_model: the NICE hierarchy is out of scope (dead under run.py)')
    return MLP(dim=cfg['data']['dim'], c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4,
               pos_embedding_method=cfg['model']['pos_embedding_method'])
