"""Drop-in `Renderer` (src/utils/Renderer.py:5-301) running on libpnr.so.

Same constructor and method signatures as the reference; every method dispatches to the C ABI
(include/pnr.h) through autograd Functions:

  eval_points       -> pnr_eval_points            Renderer.py:23-61
  render_batch_ray  -> pnr_render_fwd / _bwd      Renderer.py:63-203
  render_img        -> pnr_get_rays + fwd chunks  Renderer.py:205-260
  regulation        -> pnr_regulation_fwd / _bwd  Renderer.py:263-301

The decoder must be `pnr.decoder.MLP` (or any module exposing `ordered_params()` with the
reference state_dict tensors).  Inputs must be CUDA tensors: there is no CPU path here (the CPU
restatement in oracle/ is test infrastructure only).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .packing import PackedFC, PackedMLP
from .points import find_points

_GRAD_SHAPES = ((3, 93), (256, 93), (256,), (256, 256), (256,), (256, 256), (256,), (256, 256), (256,), (4, 256),
                (4,))


def _linspace_table(n):
    """torch.linspace(0,1,n) float32 exactly as the reference computes it (Renderer.py:157)."""
    out = [0.0] * _lib.MAX_SAMPLES
    if n > 0:
        for i, v in enumerate(torch.linspace(0., 1., steps=n).tolist()):
            out[i] = v
    return out


def _decoder_params(decoders):
    if hasattr(decoders, 'ordered_params'):
        return decoders.ordered_params()
    from .decoder import PARAM_ORDER
    sd = dict(decoders.named_parameters())
    return [sd[k] for k in PARAM_ORDER]


def _packer(decoders, attr='_packed', cls=PackedMLP):
    pk = getattr(decoders, attr, None)
    if pk is None:
        pk = cls()
        try:
            setattr(decoders, attr, pk)
        except AttributeError:
            pass
    return pk


def _feature_inputs(c, decoders):
    """(NeuralPoints or None, fc packer, extra autograd tensors [8 fc_c tensors, feats])."""
    pts = find_points(c, decoders)
    if pts is None:
        return None, None, []
    return pts, _packer(decoders, '_packed_fc', PackedFC), [*decoders.ordered_fc_params(), pts.feats]


class _Feat:
    """Per-call neural-point plumbing shared by the render / regulation Functions."""

    def __init__(self, pts, fc_owner, tensors):
        self.pts = pts
        self.fc_owner = fc_owner
        self.params = tensors[:_lib.N_PARAMS]
        self.fc = tensors[_lib.N_PARAMS:_lib.N_PARAMS + _lib.N_FC_PARAMS] if pts is not None else ()
        self.keep = []
        self.prec = None  # PNR_PREC_* of the call when only that precision's images are needed
        # grad mode of the CALLER (inside Function.forward it is always off, and needs_input_grad
        # only reflects requires_grad): an eval call under no_grad saves no activations
        self.train = torch.is_grad_enabled()

    def attach(self, prm, g_feats=None, g_fc=None):
        if self.pts is None:
            return
        s, keep = self.pts.descriptor(self.fc_owner.image(self.fc, prec=self.prec), g_feats, g_fc)
        self.keep = [s, keep]
        prm.points = ctypes.pointer(s)

    def grads(self, dev, needs):
        """Zeroed fc_c / feature grad buffers matching the extra autograd inputs (7 + 11 decoder
        tensors, then 8 fc_c tensors, then the point features), or None where autograd needs no
        gradient: the C ABI then skips the fc_c weight-gradient GEMMs (g_fc NULL) or the feature
        atomics (g_feats NULL), e.g. in the Tracker's camera-only backward."""
        if self.pts is None:
            return None, None, []
        base = 7 + _lib.N_PARAMS
        g_fc, out_fc = None, [None] * _lib.N_FC_PARAMS
        if any(needs[base:base + _lib.N_FC_PARAMS]):
            g_fc = out_fc = [torch.zeros(t.shape, device=dev, dtype=torch.float32) for t in self.fc]
        g_feats, out_feats = None, None
        if needs[base + _lib.N_FC_PARAMS]:
            g_feats = out_feats = torch.zeros_like(self.pts.feats)
        return g_feats, g_fc, [*out_fc, out_feats]


def _param_grads(ctx, dev):
    """Zeroed decoder weight-gradient buffers and their pointer array, or 11 Nones and NULL when
    no decoder tensor needs a gradient (the Tracker: the C ABI then skips every weight-gradient
    launch).  The decoder tensors are autograd inputs 7..17 of both Functions."""
    if not any(ctx.needs_input_grad[7:7 + _lib.N_PARAMS]):
        return [None] * _lib.N_PARAMS, None
    grads = [torch.zeros(s, device=dev, dtype=torch.float32) for s in _GRAD_SHAPES]
    return grads, _lib.PtrArray(*[g.data_ptr() for g in grads])


def _save_mode(ctx):
    """pnr_render_params.save_for_backward: 1 keeps every activation; 2 (ABI 8) keeps the ReLU masks
    and inputs only, when no decoder or fc_c tensor (autograd inputs 7 .. 7 + 11 + 8) needs a
    gradient -- the Tracker's camera-only backward forms no weight gradient, so the forward skips
    the activation stores."""
    return 1 if any(ctx.needs_input_grad[7:7 + _lib.N_PARAMS + _lib.N_FC_PARAMS]) else 2


class _RenderFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prm_bytes, packer, feat, rays_o, rays_d, gt_depth, far_clamp, *tensors):
        lib = _lib.load()
        prm = _lib.RenderParams.from_buffer_copy(prm_bytes)
        n = rays_o.shape[0]
        dev = rays_o.device
        packed = packer.image(feat.params)
        feat.attach(prm)
        need = feat.train and any(ctx.needs_input_grad)  # (inside forward grad mode is off)
        prm.save_for_backward = _save_mode(ctx) if need else 0
        prm.need_ray_grads = 1 if (ctx.needs_input_grad[3] or ctx.needs_input_grad[4]) else 0
        if isinstance(far_clamp, torch.Tensor):  # device value (sharded batch): no host round trip
            far_clamp = far_clamp.reshape(-1)[:1].float().contiguous()
            prm.far_mode = 2
            prm.far_clamp_dev = far_clamp.data_ptr()
        elif far_clamp is not None:
            prm.far_mode = 1
            prm.far_clamp = float(far_clamp)
        ws = torch.empty(lib.pnr_render_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        depth = torch.empty(n, dtype=torch.float64, device=dev)
        var = torch.empty(n, dtype=torch.float64, device=dev)
        rgb = torch.empty((n, 3), dtype=torch.float32, device=dev)
        _lib.check(lib.pnr_render_fwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                      _lib.ptr(gt_depth), n, _lib.ptr(depth), _lib.ptr(var), _lib.ptr(rgb),
                                      _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)), 'render_fwd')
        if need:
            prm.points = None
            ctx.prm = bytes(prm)
            ctx.feat = feat
            ctx.save_for_backward(ws, packed, rays_o, rays_d)
        return depth, var, rgb

    @staticmethod
    def backward(ctx, g_depth, g_var, g_rgb):
        lib = _lib.load()
        ws, packed, rays_o, rays_d = ctx.saved_tensors
        prm = _lib.RenderParams.from_buffer_copy(ctx.prm)
        n = rays_o.shape[0]
        dev = rays_o.device
        grads, arr = _param_grads(ctx, dev)
        g_feats, g_fc, extra = ctx.feat.grads(dev, ctx.needs_input_grad)
        ctx.feat.attach(prm, g_feats, g_fc)
        g_o = g_d = None
        if prm.need_ray_grads:
            g_o = torch.empty((n, 3), device=dev, dtype=torch.float32)
            g_d = torch.empty((n, 3), device=dev, dtype=torch.float32)
        bws = torch.empty(lib.pnr_render_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        gd = None if g_depth is None else g_depth.contiguous()
        gv = None if g_var is None else g_var.contiguous()
        gc = None if g_rgb is None else g_rgb.contiguous()
        _lib.check(lib.pnr_render_bwd(ctypes_ref(prm), _lib.ptr(packed), None, _lib.ptr(rays_o), _lib.ptr(rays_d),
                                      n, _lib.ptr(gd), _lib.ptr(gv), _lib.ptr(gc), arr, _lib.ptr(g_o),
                                      _lib.ptr(g_d), _lib.ptr(ws), ws.numel(), _lib.ptr(bws), bws.numel(),
                                      _lib.stream_of(dev)), 'render_bwd')
        return (None, None, None, g_o, g_d, None, None, *grads, *extra)


class _RegulationFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, prm_bytes, packer, feat, rays_o, rays_d, gt_depth, t_rand, *tensors):
        lib = _lib.load()
        prm = _lib.RenderParams.from_buffer_copy(prm_bytes)
        n = rays_o.shape[0]
        dev = rays_o.device
        packed = packer.image(feat.params)
        feat.attach(prm)
        need = feat.train and any(ctx.needs_input_grad)  # (inside forward grad mode is off)
        prm.save_for_backward = _save_mode(ctx) if need else 0
        prm.need_ray_grads = 1 if (ctx.needs_input_grad[3] or ctx.needs_input_grad[4]) else 0
        ws = torch.empty(lib.pnr_regulation_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        sigma = torch.empty(n * prm.n_samples, dtype=torch.float32, device=dev)
        _lib.check(lib.pnr_regulation_fwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                          _lib.ptr(gt_depth), _lib.ptr(t_rand), n, _lib.ptr(sigma), _lib.ptr(ws),
                                          ws.numel(), _lib.stream_of(dev)), 'regulation_fwd')
        if need:
            prm.points = None
            ctx.prm = bytes(prm)
            ctx.feat = feat
            ctx.save_for_backward(ws, packed, rays_o, rays_d)
        return sigma

    @staticmethod
    def backward(ctx, g_sigma):
        lib = _lib.load()
        ws, packed, rays_o, rays_d = ctx.saved_tensors
        prm = _lib.RenderParams.from_buffer_copy(ctx.prm)
        n = rays_o.shape[0]
        dev = rays_o.device
        grads, arr = _param_grads(ctx, dev)
        g_feats, g_fc, extra = ctx.feat.grads(dev, ctx.needs_input_grad)
        ctx.feat.attach(prm, g_feats, g_fc)
        g_o = g_d = None
        if prm.need_ray_grads:
            g_o = torch.empty((n, 3), device=dev, dtype=torch.float32)
            g_d = torch.empty((n, 3), device=dev, dtype=torch.float32)
        bws = torch.empty(lib.pnr_regulation_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        _lib.check(lib.pnr_regulation_bwd(ctypes_ref(prm), _lib.ptr(packed), None, _lib.ptr(rays_o),
                                          _lib.ptr(rays_d), n, _lib.ptr(g_sigma.contiguous()), arr, _lib.ptr(g_o),
                                          _lib.ptr(g_d), _lib.ptr(ws), ws.numel(), _lib.ptr(bws), bws.numel(),
                                          _lib.stream_of(dev)), 'regulation_bwd')
        return (None, None, None, g_o, g_d, None, None, *grads, *extra)


def ctypes_ref(prm):
    return ctypes.byref(prm)


class TrainPass:
    """One forward + backward of render_batch_ray or regulation for pnr.mapping.MapStep, without
    autograd: the forward keeps every activation (save_for_backward = 1, no ray gradients), the
    backward takes the upstream gradients from pnr_map_loss and adds the decoder / fc_c / point
    feature gradients into caller-given buffers (the flat gradient views of a MapStep).  Same C ABI
    calls as _RenderFn / _RegulationFn, minus the autograd plumbing (~20 elementwise launches of the
    torch loss and its backward per mapping iteration)."""

    def __init__(self, renderer, c, decoders, kind):
        self.r, self.kind = renderer, kind
        self.params = _decoder_params(decoders)
        self.pts, fc_owner, extra = _feature_inputs(c, decoders)
        self.feat = _Feat(self.pts, fc_owner, [*self.params, *extra])
        self.packer = _packer(decoders)

    def forward(self, rays_o, rays_d, gt_depth, t_rand=None, far_clamp=None):
        lib = _lib.load()
        r = self.r
        dev = rays_o.device
        n = rays_o.shape[0]
        prm = r.params(n_importance=0) if self.kind == 'regulation' else r.params()
        prm.status = r.status_word(dev).data_ptr()
        prm.save_for_backward = 1
        prm.need_ray_grads = 0
        packed = self.packer.image(self.feat.params, prec=prm.precision)
        self.feat.prec = prm.precision
        self.feat.attach(prm)
        if isinstance(far_clamp, torch.Tensor):
            far_clamp = far_clamp.reshape(-1)[:1].float().contiguous()
            prm.far_mode = 2
            prm.far_clamp_dev = far_clamp.data_ptr()
        elif far_clamp is not None:
            prm.far_mode = 1
            prm.far_clamp = float(far_clamp)
        st = _lib.stream_of(dev)
        if self.kind == 'regulation':
            ws = torch.empty(lib.pnr_regulation_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
            sigma = torch.empty(n * prm.n_samples, dtype=torch.float32, device=dev)
            _lib.check(lib.pnr_regulation_fwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                              _lib.ptr(gt_depth), _lib.ptr(t_rand), n, _lib.ptr(sigma), _lib.ptr(ws),
                                              ws.numel(), st), 'regulation_fwd')
            out = (sigma,)
        else:
            ws = torch.empty(lib.pnr_render_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
            depth = torch.empty(n, dtype=torch.float64, device=dev)
            var = torch.empty(n, dtype=torch.float64, device=dev)
            rgb = torch.empty((n, 3), dtype=torch.float32, device=dev)
            _lib.check(lib.pnr_render_fwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                          _lib.ptr(gt_depth), n, _lib.ptr(depth), _lib.ptr(var), _lib.ptr(rgb),
                                          _lib.ptr(ws), ws.numel(), st), 'render_fwd')
            out = (depth, var, rgb)
        prm.points = None
        self.prm, self.ws, self.packed, self.rays = prm, ws, packed, (rays_o, rays_d, far_clamp)
        return out

    def backward(self, grads, g_fc=None, g_feats=None, g_depth=None, g_rgb=None, g_sigma=None):
        """grads: the 11 decoder gradient tensors to add into (contiguous float32); g_fc: the 8 fc_c
        ones, g_feats: the point features' (with neural points)."""
        lib = _lib.load()
        prm, ws, packed = self.prm, self.ws, self.packed
        rays_o, rays_d, _ = self.rays
        dev = rays_o.device
        n = rays_o.shape[0]
        arr = _lib.PtrArray(*[g.data_ptr() for g in grads])
        self.feat.attach(prm, g_feats, g_fc)
        st = _lib.stream_of(dev)
        if self.kind == 'regulation':
            bws = torch.empty(lib.pnr_regulation_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8,
                              device=dev)
            _lib.check(lib.pnr_regulation_bwd(ctypes_ref(prm), _lib.ptr(packed), None, _lib.ptr(rays_o),
                                              _lib.ptr(rays_d), n, _lib.ptr(g_sigma), arr, None, None, _lib.ptr(ws),
                                              ws.numel(), _lib.ptr(bws), bws.numel(), st), 'regulation_bwd')
        else:
            bws = torch.empty(lib.pnr_render_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
            _lib.check(lib.pnr_render_bwd(ctypes_ref(prm), _lib.ptr(packed), None, _lib.ptr(rays_o), _lib.ptr(rays_d),
                                          n, _lib.ptr(g_depth), None, _lib.ptr(g_rgb), arr, None, None, _lib.ptr(ws),
                                          ws.numel(), _lib.ptr(bws), bws.numel(), st), 'render_bwd')
        self.ws = self.packed = None  # release the saved activations


class MapPass:
    """One Mapper iteration's render_batch_ray (with gt depth) AND regulation as ONE decoder pass
    (pnr_map_fwd / pnr_map_bwd, ABI 10): the regulation and coarse samples share one MLP launch, the
    importance samples take a second, and the backward is one delta-chain / weight-gradient pass over
    every sample (src/Mapper.py:623-655).  Same outputs as TrainPass('render') + TrainPass('regulation')
    bit for bit; the gradient sums differ from that pair's only in association."""

    def __init__(self, renderer, c, decoders):
        self.r = renderer
        self.params = _decoder_params(decoders)
        self.pts, fc_owner, extra = _feature_inputs(c, decoders)
        self.feat = _Feat(self.pts, fc_owner, [*self.params, *extra])
        self.packer = _packer(decoders)

    def forward(self, rays_o, rays_d, gt_depth, t_rand, far_clamp=None):
        lib = _lib.load()
        r = self.r
        dev = rays_o.device
        n = rays_o.shape[0]
        prm = r.params()
        prm.status = r.status_word(dev).data_ptr()
        prm.save_for_backward = 1
        prm.need_ray_grads = 0
        packed = self.packer.image(self.feat.params, prec=prm.precision)
        self.feat.prec = prm.precision
        self.feat.attach(prm)
        if isinstance(far_clamp, torch.Tensor):
            far_clamp = far_clamp.reshape(-1)[:1].float().contiguous()
            prm.far_mode = 2
            prm.far_clamp_dev = far_clamp.data_ptr()
        elif far_clamp is not None:
            prm.far_mode = 1
            prm.far_clamp = float(far_clamp)
        ws = torch.empty(lib.pnr_map_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        depth = torch.empty(n, dtype=torch.float64, device=dev)
        var = torch.empty(n, dtype=torch.float64, device=dev)
        rgb = torch.empty((n, 3), dtype=torch.float32, device=dev)
        sigma = torch.empty(n * prm.n_samples, dtype=torch.float32, device=dev)
        _lib.check(lib.pnr_map_fwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                   _lib.ptr(gt_depth), _lib.ptr(t_rand), n, _lib.ptr(depth), _lib.ptr(var),
                                   _lib.ptr(rgb), _lib.ptr(sigma), _lib.ptr(ws), ws.numel(), _lib.stream_of(dev)),
                   'map_fwd')
        prm.points = None
        self.prm, self.ws, self.packed, self.rays = prm, ws, packed, (rays_o, rays_d, far_clamp)
        return depth, var, rgb, sigma

    def backward(self, grads, g_fc=None, g_feats=None, g_depth=None, g_rgb=None, g_sigma=None, overwrite=False):
        """Adds the decoder / fc_c gradients into grads / g_fc, or stores them (overwrite: no zero fill
        needed, pnr_render_params.grads_overwrite); the point-feature gradients always add."""
        lib = _lib.load()
        prm, ws, packed = self.prm, self.ws, self.packed
        prm.grads_overwrite = 1 if overwrite else 0
        rays_o, rays_d, _ = self.rays
        dev = rays_o.device
        n = rays_o.shape[0]
        arr = _lib.PtrArray(*[g.data_ptr() for g in grads])
        self.feat.attach(prm, g_feats, g_fc)
        bws = torch.empty(lib.pnr_map_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        _lib.check(lib.pnr_map_bwd(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_d), n, _lib.ptr(g_depth),
                                   _lib.ptr(g_rgb), _lib.ptr(g_sigma), arr, _lib.ptr(ws), ws.numel(), _lib.ptr(bws),
                                   bws.numel(), _lib.stream_of(dev)), 'map_bwd')
        self.ws = self.packed = None

    def step(self, rays_o, rays_d, gt_depth, gt_color, t_rand, w_color, w_reg, loss_ws, grads, g_fc=None,
             g_feats=None, far_clamp=None, overwrite=False):
        """forward + map_loss + backward in ONE C call (pnr_map_step, ABI 13): at batches up to 32,768 rays
        the compositing, the loss and the compositing backward are one fused launch.  Same gradients as
        the three-call form bit for bit; returns the float64 loss (0-dim, on the device)."""
        lib = _lib.load()
        r = self.r
        dev = rays_o.device
        n = rays_o.shape[0]
        prm = r.params()
        prm.status = r.status_word(dev).data_ptr()
        prm.save_for_backward = 1
        prm.need_ray_grads = 0
        prm.grads_overwrite = 1 if overwrite else 0
        packed = self.packer.image(self.feat.params, prec=prm.precision)
        self.feat.prec = prm.precision
        self.feat.attach(prm, g_feats, g_fc)
        if isinstance(far_clamp, torch.Tensor):
            far_clamp = far_clamp.reshape(-1)[:1].float().contiguous()
            prm.far_mode = 2
            prm.far_clamp_dev = far_clamp.data_ptr()
        elif far_clamp is not None:
            prm.far_mode = 1
            prm.far_clamp = float(far_clamp)
        ws = torch.empty(lib.pnr_map_step_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        bws = torch.empty(lib.pnr_map_bwd_workspace_bytes(ctypes_ref(prm), n), dtype=torch.uint8, device=dev)
        loss = torch.empty((), dtype=torch.float64, device=dev)
        arr = _lib.PtrArray(*[g.data_ptr() for g in grads])
        _lib.check(lib.pnr_map_step(ctypes_ref(prm), _lib.ptr(packed), _lib.ptr(rays_o), _lib.ptr(rays_d),
                                    _lib.ptr(gt_depth), _lib.ptr(gt_color), _lib.ptr(t_rand), n, float(w_color),
                                    float(w_reg), _lib.ptr(loss), arr, _lib.ptr(ws), ws.numel(), _lib.ptr(bws),
                                    bws.numel(), _lib.ptr(loss_ws), _lib.stream_of(dev)), 'map_step')
        prm.points = None
        return loss


def map_loss_workspace(device):
    """A zero-filled pnr_map_loss workspace (each call leaves it zero-filled: reuse it for the calls of
    one stream; two streams need two)."""
    return torch.zeros(_lib.load().pnr_map_loss_workspace_bytes(), dtype=torch.uint8, device=device)


def map_loss(gt_depth, depth, gt_color, color, w_color, sigma=None, w_reg=0.0, ws=None):
    """pnr_map_loss: the Mapper loss terms (src/Mapper.py:628-655) and their gradients in one pass.
    Returns (loss float64 0-dim, g_depth, g_color, g_sigma); either part may be None.  `ws`: a
    map_loss_workspace of the calling stream (default: a fresh zero-filled one)."""
    lib = _lib.load()
    ref = depth if depth is not None else sigma
    dev = ref.device
    n = 0 if depth is None else depth.shape[0]
    ns = 0 if sigma is None else sigma.numel()
    loss = torch.empty((), dtype=torch.float64, device=dev)
    if ws is None:
        ws = map_loss_workspace(dev)
    g_d = torch.empty(n, dtype=torch.float64, device=dev) if n else None
    g_c = torch.empty((n, 3), dtype=torch.float32, device=dev) if n else None
    g_s = torch.empty(ns, dtype=torch.float32, device=dev) if ns else None
    _lib.check(lib.pnr_map_loss(_lib.ptr(gt_depth if n else None), _lib.ptr(depth), _lib.ptr(gt_color if n else None),
                                _lib.ptr(color), n, float(w_color), _lib.ptr(sigma), ns, float(w_reg), _lib.ptr(loss),
                                _lib.ptr(g_d), _lib.ptr(g_c), _lib.ptr(g_s), _lib.ptr(ws), _lib.stream_of(dev)),
               'map_loss')
    return loss, g_d, g_c, g_s


class Renderer(object):
    """src/utils/Renderer.py:5-21 (same signature and cfg keys)."""

    def __init__(self, cfg, args, slam, points_batch_size=500000, ray_batch_size=100000):
        self.ray_batch_size = ray_batch_size
        self.points_batch_size = points_batch_size
        self.lindisp = cfg['rendering']['lindisp']
        self.perturb = cfg['rendering']['perturb']
        self.N_samples = cfg['rendering']['N_samples']
        self.N_surface = cfg['rendering']['N_surface']
        self.N_importance = cfg['rendering']['N_importance']
        self.scale = cfg['scale']
        self.occupancy = cfg['occupancy']
        self.nice = False
        self.bound = slam.bound
        self.H, self.W, self.fx, self.fy, self.cx, self.cy = slam.H, slam.W, slam.fx, slam.fy, slam.cx, slam.cy
        # decoder matmul arithmetic (pnr extension; cfg['pnr']['precision'], default _lib.DEFAULT_PRECISION)
        self.precision = (cfg.get('pnr') or {}).get('precision', _lib.DEFAULT_PRECISION)
        _lib.precision_code(self.precision)
        if self.N_surface > 0 or self.occupancy or self.perturb > 0.:
            raise NotImplementedError('pnr.Renderer: N_surface>0 / occupancy / perturb>0 are not on the '
                                      'configs/pointNeRF_slam.yaml path (SURVEY.md section 8)')
        if self.N_samples + self.N_importance > _lib.MAX_SAMPLES or self.N_samples < 3:
            raise ValueError('pnr.Renderer: need 3 <= N_samples and N_samples + N_importance <= 64')

    def __getstate__(self):  # the status words are per process (device memory)
        st = dict(self.__dict__)
        st.pop('_status', None)
        return st

    # -- f16-range status (include/pnr.h PNR_STATUS_*) ------------------------------------------
    def status_word(self, device):
        """Device int32 the kernels OR PNR_STATUS_* bits into (one per device, lazily created)."""
        sw = self.__dict__.setdefault('_status', {})
        dev = torch.device(device)
        if dev not in sw:
            sw[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
        return sw[dev]

    def status(self, device='cuda:0', clear=False):
        """PNR_STATUS_* bits raised since the last clear (synchronises with the device)."""
        w = self.status_word(device)
        v = int(w.item())
        if clear:
            w.zero_()
        return v

    def check_status(self, device='cuda:0'):
        """Raise FloatingPointError when an f16x3 forward met a value outside the f16 range: its
        results are not fp32-faithful (include/pnr.h PNR_STATUS_F16_RANGE).  Use precision 'fp32'."""
        if self.status(device) & _lib.STATUS_F16_RANGE:
            raise FloatingPointError('pnr: an f16x3 decoder forward met |value| >= 65504 (f16 range); '
                                     "results since the last check are not fp32-faithful: use precision 'fp32'")

    # -- helpers --------------------------------------------------------------------------------
    def _bound6(self):
        # the bound is fixed per renderer (src/NICE_SLAM.py:208-213): read once, so a render issues no
        # device-to-host copy (a graph capture of the mapping step forbids one)
        if getattr(self, '_b6_src', None) is not self.bound:
            self._b6_src = self.bound
            b = self.bound
            b = b.detach().cpu().double().reshape(3, 2) if isinstance(b, torch.Tensor) else torch.tensor(b).double()
            self._b6 = [float(v) for v in b.reshape(-1)]
        return self._b6

    def params(self, n_samples=None, n_importance=None):
        prm = _lib.RenderParams()
        prm.n_samples = self.N_samples if n_samples is None else n_samples
        prm.n_importance = self.N_importance if n_importance is None else n_importance
        prm.lindisp = 1 if self.lindisp else 0
        prm.far_mode = 0
        for i, v in enumerate(self._bound6()):
            prm.bound[i] = v
        for i, v in enumerate(_linspace_table(prm.n_samples)):
            prm.t_vals[i] = v
        for i, v in enumerate(_linspace_table(prm.n_importance)):
            prm.u_vals[i] = v
        prm.precision = _lib.precision_code(self.precision)
        return prm

    # -- reference API ------------------------------------------------------------------------------
    def eval_points(self, p, decoders, c=None, stage='color', device='cuda:0'):
        """Renderer.py:23-61: raw (P,4) float32, density := 100 outside the bound (strict)."""
        _lib.require_cuda(p)
        lib = _lib.load()
        packed = _packer(decoders).image(_decoder_params(decoders))
        P = p.shape[0]
        raw = torch.empty((P, 4), dtype=torch.float32, device=p.device)
        bound = (ctypes.c_double * 6)(*self._bound6())
        pts, fc_owner, _ = _feature_inputs(c, decoders)
        if pts is not None:  # features: gather, then the MLP with fc_c injection (no autograd here)
            with torch.no_grad():
                dp = p.double().contiguous()
                cf = pts.gather(dp)
                fcp = fc_owner.image(decoders.ordered_fc_params())
                _lib.check(lib.pnr_eval_points_c(_lib.ptr(packed), _lib.ptr(fcp), _lib.ptr(dp), _lib.ptr(cf), P, bound,
                                                 _lib.ptr(raw), _lib.precision_code(self.precision),
                                                 _lib.stream_of(p.device)), 'eval_points_c')
            return raw
        if p.dtype == torch.float64:
            fn = lib.pnr_eval_points
        else:
            fn = lib.pnr_eval_points_f32
            p = p.float()
        _lib.check(fn(_lib.ptr(packed), _lib.ptr(p.contiguous()), P, bound, _lib.ptr(raw),
                      _lib.precision_code(self.precision), _lib.stream_of(p.device)), 'eval_points')
        return raw

    def render_batch_ray(self, c, decoders, rays_d, rays_o, device, stage, gt_depth=None, far_clamp=None):
        """Renderer.py:63-203 -> (depth f64 (N,), uncertainty f64 (N,), color f32 (N,3)).

        `far_clamp` (extension, default None = reference behaviour) overrides the batch-global
        max(1.2*gt) of Renderer.py:112 -- used by a ray-sharded caller to keep 1-GPU semantics: a
        float, or a one-element device tensor (read on the device: no host sync, graph-capturable)."""
        _lib.require_cuda(rays_o, rays_d, gt_depth)
        rays_o = rays_o.float().contiguous()
        rays_d = rays_d.float().contiguous()
        gt = None if gt_depth is None else gt_depth.reshape(-1).float().contiguous()
        prm = self.params()
        prm.status = self.status_word(rays_o.device).data_ptr()
        params = _decoder_params(decoders)
        pts, fc_owner, extra = _feature_inputs(c, decoders)
        feat = _Feat(pts, fc_owner, [*params, *extra])
        return _RenderFn.apply(bytes(prm), _packer(decoders), feat, rays_o, rays_d, gt, far_clamp, *params, *extra)

    def render_img(self, c, decoders, c2w, device, stage, gt_depth=None):
        """Renderer.py:205-260: full frame in ray_batch_size chunks, float64 depth/uncertainty."""
        with torch.no_grad():
            H, W = self.H, self.W
            rays_o, rays_d = get_rays(H, W, self.fx, self.fy, self.cx, self.cy, c2w, device)
            rays_o = rays_o.reshape(-1, 3)
            rays_d = rays_d.reshape(-1, 3)
            gt = None if gt_depth is None else gt_depth.reshape(-1)
            ds, vs, cs = [], [], []
            for i in range(0, rays_d.shape[0], self.ray_batch_size):
                g = None if gt is None else gt[i:i + self.ray_batch_size]
                d, v, col = self.render_batch_ray(c, decoders, rays_d[i:i + self.ray_batch_size],
                                                  rays_o[i:i + self.ray_batch_size], device, stage, gt_depth=g)
                ds.append(d.double()); vs.append(v.double()); cs.append(col)
            return (torch.cat(ds).reshape(H, W), torch.cat(vs).reshape(H, W), torch.cat(cs).reshape(H, W, 3))

    def regulation(self, c, decoders, rays_d, rays_o, gt_depth, device, stage='color', t_rand=None):
        """Renderer.py:263-301: density at N_samples jittered depths in [0, 0.85*gt].
        `t_rand` (extension) supplies the jitter; default draws torch.rand on the device."""
        _lib.require_cuda(rays_o, rays_d, gt_depth)
        rays_o = rays_o.float().contiguous()
        rays_d = rays_d.float().contiguous()
        gt = gt_depth.reshape(-1).float().contiguous()
        n = rays_o.shape[0]
        if t_rand is None:
            t_rand = torch.rand((n, self.N_samples), device=rays_o.device)
        t_rand = t_rand.float().contiguous()
        prm = self.params(n_importance=0)
        prm.status = self.status_word(rays_o.device).data_ptr()
        params = _decoder_params(decoders)
        pts, fc_owner, extra = _feature_inputs(c, decoders)
        feat = _Feat(pts, fc_owner, [*params, *extra])
        return _RegulationFn.apply(bytes(prm), _packer(decoders), feat, rays_o, rays_d, gt, t_rand, *params, *extra)


def get_rays(H, W, fx, fy, cx, cy, c2w, device):
    """src/common.py:248-266 on the device: (H,W,3) rays_o, rays_d float32."""
    lib = _lib.load()
    if not isinstance(c2w, torch.Tensor):
        c2w = torch.as_tensor(c2w)
    c2w = c2w.to(device=device, dtype=torch.float32)
    if c2w.shape[0] == 3:
        c2w = torch.cat([c2w, torch.tensor([[0., 0., 0., 1.]], device=c2w.device)], 0)
    c2w = c2w.contiguous()
    _lib.require_cuda(c2w)
    ro = torch.empty((H, W, 3), dtype=torch.float32, device=c2w.device)
    rd = torch.empty((H, W, 3), dtype=torch.float32, device=c2w.device)
    _lib.check(lib.pnr_get_rays(H, W, float(fx), float(fy), float(cx), float(cy), _lib.ptr(c2w), _lib.ptr(ro),
                                _lib.ptr(rd), _lib.stream_of(c2w.device)), 'get_rays')
    return ro, rd


def get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device):
    """src/common.py:74-89 on the device: rays for pixel coordinates (i column, j row)."""
    lib = _lib.load()
    if not isinstance(c2w, torch.Tensor):
        c2w = torch.as_tensor(c2w)
    c2w = c2w.to(device=device, dtype=torch.float32)
    if c2w.shape[0] == 3:
        c2w = torch.cat([c2w, torch.tensor([[0., 0., 0., 1.]], device=c2w.device)], 0)
    c2w = c2w.contiguous()
    i = i.reshape(-1).float().contiguous()
    j = j.reshape(-1).float().contiguous()
    _lib.require_cuda(c2w, i, j)
    n = i.shape[0]
    ro = torch.empty((n, 3), dtype=torch.float32, device=c2w.device)
    rd = torch.empty((n, 3), dtype=torch.float32, device=c2w.device)
    _lib.check(lib.pnr_rays_from_uv(_lib.ptr(i), _lib.ptr(j), n, float(fx), float(fy), float(cx), float(cy),
                                    _lib.ptr(c2w), _lib.ptr(ro), _lib.ptr(rd), _lib.stream_of(c2w.device)),
               'rays_from_uv')
    return ro, rd


def get_samples(H0, H1, W0, W1, n, H, W, fx, fy, cx, cy, c2w, depth, color, device, generator=None):
    """src/common.py:110-134 (get_sample_uv + select_uv + get_rays_from_uv) on the device: n uniform
    torch.randint pixels of the region H0..H1 x W0..W1 (row-major region index), their rays
    (pnr_rays_from_uv), depth and colour.  The reference's linspace pixel grid holds exact
    integers, so pixel (i, j) = (idx % w + W0, idx // w + H0)."""
    from .common import select_uv_indices
    d = depth[H0:H1, W0:W1].reshape(-1)
    col = color[H0:H1, W0:W1].reshape(-1, 3)
    w = W1 - W0
    idx = select_uv_indices(d.numel(), n, d.device, generator)
    i = (idx % w + W0).float()
    j = (torch.div(idx, w, rounding_mode='floor') + H0).float()
    ro, rd = get_rays_from_uv(i, j, c2w, H, W, fx, fy, cx, cy, device)
    return ro, rd, d[idx], col[idx]

