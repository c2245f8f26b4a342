"""One Mapper iteration on the HIP path (src/Mapper.py:335-694).

`MapStep` is the inner loop body of Mapper.optimize_map for the imap* decoder
(src/Mapper.py:507-662): render the sampled rays with gt depth (Renderer.render_batch_ray,
:623-624), L1 depth over gt>0 + w_color * L1 colour (:641-646), 0.0005 * |sigma| of the
regulation query (:650-655), backward, Adam step with lr = imap_decoders_lr (:540, :657-662).

The decoder parameters live in ONE flat float32 buffer (and so do their grads), so a data-
parallel caller reduces a single 891 KB buffer per step and Adam is one kernel
(pnr_adam_step).  With neural points the fc_c tensors and the point features
join the same buffer (features last, with their own learning rate: a second Adam launch over the
tail of the buffer), still one all-reduce per step -- or, with DataParallel(shard_points=True), a
reduce-scatter of the feature tail, Adam on the owned feature range and an all-gather.  `ddp`
(pnr.dist.DataParallel) adds the cross-GPU gradient all-reduce and the
global far clamp; without it the step is single-GPU.  The step is deterministic: every weight-
gradient GEMM stores per-workgroup partial tiles that one reduction adds in a fixed order (no float
atomics), so a replay or a rerun reproduces it bit for bit.  It is not the reference's float32
summation order (no GPU sum is); tests/test_gpu_precision.py holds it to the correctly-rounded
gradient.  The point-feature gradient (neural points) is summed exactly in int64 fixed point
(include/pnr.h, ABI 10), so it does not depend on scheduling either: a neural-point step reruns and
replays bit for bit too.
"""
from __future__ import annotations

import torch

from . import _lib


class FlatParams:
    """Re-seat every parameter of `module` (and its .grad) as a view of one flat buffer."""

    def __init__(self, params):
        self.params = list(params)
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.data = torch.empty(n, device=dev, dtype=torch.float32)
        self.grad = torch.zeros(n, device=dev, dtype=torch.float32)
        off = 0
        for p in self.params:
            k = p.numel()
            self.data[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.data[off:off + k].view_as(p)
            p.grad = self.grad[off:off + k].view_as(p)
            off += k
        self.numel = n

    def zero_grad(self):
        self.grad.zero_()


class Adam:
    """torch.optim.Adam(lr, betas=(0.9, 0.999), eps=1e-8) over a FlatParams buffer, one launch per
    learning-rate segment.  `segments` = [(first word, words, lr)], default the whole buffer.
    `use_device_step()` switches the step number to a device counter (pnr_adam_multi_dev: every
    segment and the step advance in one launch), so a step captured in a graph replays with the right
    bias corrections."""

    def __init__(self, flat: FlatParams, lr: float, betas=(0.9, 0.999), eps=1e-8, on_update=None, segments=None,
                 half=None):
        """`half` (optional): {segment index: float16 device tensor of the segment's length} -- with the
        device step counter, the Adam launch also writes float16 of the updated values there (the
        gather's f16 feature copy, pnr_adam_multi_dev_h) and `wrote_half` is set after the step."""
        self.flat = flat
        self.half = dict(half or {})
        self.wrote_half = False
        self.on_update = on_update
        self.lr = lr
        self.segments = segments if segments is not None else [(0, flat.numel, lr)]
        self.b1, self.b2 = betas
        self.eps = eps
        # moments per segment, sized to it: a sharded feature tail holds only the owned range's m / v
        self.mv = [(torch.zeros(n, device=flat.data.device), torch.zeros(n, device=flat.data.device))
                   for _, n, _ in self.segments]
        self.step_count = 0
        self.step_dev = None  # int32 device counter of completed steps (graph mode)

    def use_device_step(self):
        """step_dev = int32 {completed steps, ticket 0} on the device (pnr_adam_multi_dev): every
        segment and the step advance in ONE launch per step."""
        if self.step_dev is None:
            import ctypes
            self.step_dev = torch.tensor([self.step_count, 0], dtype=torch.int32, device=self.flat.data.device)
            k = len(self.segments)
            self._seg_args = ((ctypes.c_int64 * k)(*[a for a, _, _ in self.segments]),
                              (ctypes.c_int64 * k)(*[n for _, n, _ in self.segments]),
                              (ctypes.c_void_p * k)(*[m.data_ptr() for m, _ in self.mv]),
                              (ctypes.c_void_p * k)(*[v.data_ptr() for _, v in self.mv]),
                              (ctypes.c_float * k)(*[lr for _, _, lr in self.segments]))
            self._half_arr = None
            if self.half:
                self._half_arr = (ctypes.c_void_p * k)(*[self.half[q].data_ptr() if q in self.half else None
                                                         for q in range(k)])

    def step(self):
        self.step_count += 1
        lib = _lib.load()
        f = self.flat
        st = _lib.stream_of(f.data.device)
        self.wrote_half = False
        if self.step_dev is not None:
            off, n, m, v, lr = self._seg_args
            if self._half_arr is not None:
                _lib.check(lib.pnr_adam_multi_dev_h(_lib.ptr(f.data), _lib.ptr(f.grad), len(self.segments), off, n, m,
                                                    v, lr, self.b1, self.b2, self.eps, self._half_arr,
                                                    _lib.ptr(self.step_dev), st), 'adam_multi_dev_h')
                self.wrote_half = True
            else:
                _lib.check(lib.pnr_adam_multi_dev(_lib.ptr(f.data), _lib.ptr(f.grad), len(self.segments), off, n, m,
                                                  v, lr, self.b1, self.b2, self.eps, _lib.ptr(self.step_dev), st),
                           'adam_multi_dev')
        else:
            for (a, n, lr), (m, v) in zip(self.segments, self.mv):
                _lib.check(lib.pnr_adam_step(_lib.ptr(f.data[a:]), _lib.ptr(f.grad[a:]), _lib.ptr(m),
                                             _lib.ptr(v), n, lr, self.b1, self.b2, self.eps, self.step_count,
                                             st), 'adam_step')
        if self.on_update is not None:  # weights changed behind autograd: drop the packed image
            self.on_update()


class MapStep:
    """One Mapper iteration.  Default (`fused=True`): the render and the regulation are ONE decoder
    pass (pnr.renderer.MapPass -> pnr_map_fwd / pnr_map_bwd): the regulation and coarse samples share
    one MLP launch, the importance samples take a second, pnr_map_loss forms both loss terms and their
    gradients in one launch, and one delta-chain / weight-gradient pass covers every sample.  (The MLP
    kernels hold every CU's registers and LDS, so two chains on two streams could only take turns,
    and the small ray kernels of one chain waited behind the other's MLP launches.)
    `fused=False` keeps the two-chain form: the regulation's forward, loss term and backward on a side
    stream with its own gradient buffer (`overlap` True / 'auto' up to OVERLAP_MAX_RAYS rays) or on the
    caller's stream (`overlap=False`), joined before the gradients are summed (render + regulation, a
    fixed order).  No path goes through autograd (MapStep.loss is the autograd drop-in form)."""

    OVERLAP_MAX_RAYS = 32768
    # the fused path as one pnr_map_step call (ABI 13) rather than pnr_map_fwd + pnr_map_loss + pnr_map_bwd
    one_call = True

    def __init__(self, renderer, decoder, lr=2e-4, w_color_loss=0.05, w_reg=0.0005, ddp=None, points=None,
                 feat_lr=None, overlap='auto', fused=True):
        self.renderer = renderer
        self.decoder = decoder
        self.points = points
        params = list(decoder.ordered_params())
        if points is not None:
            params += list(decoder.ordered_fc_params())
        n_dec = sum(p.numel() for p in params)
        if points is not None:
            params.append(points.feats)
        self.flat = FlatParams(params)
        segs = [(0, n_dec, lr)]
        self.n_dec = n_dec
        self.shard = points is not None and ddp is not None and getattr(ddp, 'shard_points', False)
        if points is not None:
            flr = lr if feat_lr is None else feat_lr
            if self.shard:  # Adam on this rank's owned feature range only (pnr.dist reduce_scatter_)
                a, b, _ = ddp.feature_shard(points.feats.numel())
                if b > a:
                    segs.append((n_dec + a, b - a, flr))
            else:
                segs.append((n_dec, points.feats.numel(), flr))
        # float16 features (C5): the captured step's Adam launch refreshes the gather's f16 copy itself
        # (the whole-table conversion was a pass of its own); the sharded update all-gathers after Adam
        half = None
        if points is not None and points.feat_dtype == 'float16' and not self.shard and len(segs) == 2:
            half = {1: points._feats_for_gather()}
        self.opt = Adam(self.flat, lr, on_update=self._invalidate, segments=segs, half=half)
        self.c = {} if points is None else {'points_' + getattr(decoder, 'name', ''): points}
        self.w_color = w_color_loss
        self.w_reg = w_reg
        self.ddp = ddp
        if overlap not in (True, False, 'auto'):
            raise ValueError(f'overlap must be True, False or "auto", not {overlap!r}')
        self.overlap = overlap
        self.fused = bool(fused)
        self.side = None   # the side stream and the regulation chain's gradient buffer (same layout
        self.grad2 = None  # as flat.grad) with its views: made on the first overlapped step
        self._views = {'main': self._split(self.flat.grad)}

    def _loss_ws(self, chain):
        """The pnr_map_loss workspace of a chain's stream (zero-filled once; each call leaves it zero)."""
        ws = self.__dict__.setdefault('_lws', {})
        if chain not in ws:
            from .renderer import map_loss_workspace
            ws[chain] = map_loss_workspace(self.flat.data.device)
        return ws[chain]

    def _overlaps(self, n_rays):
        if self.overlap != 'auto':
            return bool(self.overlap)
        return n_rays <= self.OVERLAP_MAX_RAYS

    def _split(self, buf):
        """(11 decoder, 8 fc_c or None, features or None) views of a flat-gradient-shaped buffer."""
        views, off = [], 0
        for p in self.flat.params:
            views.append(buf[off:off + p.numel()].view_as(p))
            off += p.numel()
        if self.points is None:
            return views, None, None
        return views[:11], views[11:19], views[19]

    def _invalidate(self):
        self.decoder._packed.invalidate()
        if self.points is not None:
            self.decoder._packed_fc.invalidate()
            if self.opt.wrote_half:  # Adam wrote the f16 feature copy with the fp32 master
                self.points.mark_feats_fresh()
            else:
                self.points.invalidate_feats()  # the f16 feature copy, if any

    def _regulation_chain(self, views, rays_o, rays_d, gt_depth, t_rand):
        from .renderer import TrainPass, map_loss
        reg = TrainPass(self.renderer, self.c, self.decoder, 'regulation')
        (sigma,) = reg.forward(rays_o, rays_d, gt_depth, t_rand=t_rand)
        loss, _, _, g_s = map_loss(None, None, None, None, 0.0, sigma=sigma, w_reg=self.w_reg, ws=self._loss_ws('side'))
        reg.backward(views[0], g_fc=views[1], g_feats=views[2], g_sigma=g_s)
        return loss

    def __call__(self, rays_o, rays_d, gt_depth, gt_color, t_rand=None, far_clamp=None):
        """One Mapper iteration.  far_clamp (optional): the batch's max(1.2 gt) as a device scalar
        (e.g. from WindowSampler), else computed by the render pass (or all-reduced, data parallel)."""
        from .renderer import TrainPass, map_loss
        r = self.renderer
        dev = rays_o.device
        rays_o = rays_o.float().contiguous()
        rays_d = rays_d.float().contiguous()
        gt_depth = gt_depth.reshape(-1).float().contiguous()
        gt_color = gt_color.float().contiguous()
        if t_rand is None:
            t_rand = torch.rand((rays_o.shape[0], r.N_samples), device=dev)
        t_rand = t_rand.float().contiguous()
        if self.fused:  # the map pass stores the decoder / fc_c gradients (grads_overwrite): zero the rest
            if self.points is not None:
                self._views['main'][2].zero_()
        else:
            self.flat.zero_grad()
        if self.ddp is not None:
            far_clamp = self.ddp.global_far_clamp(gt_depth, far_clamp)
        ren = TrainPass(r, self.c, self.decoder, 'render')
        # the weight images, the point index and the f16 feature copy: built on this stream before the
        # chains fork (both read them)
        prec = _lib.precision_code(r.precision)
        ren.packer.image(ren.feat.params, prec=prec)
        if self.points is not None:
            ren.feat.fc_owner.image(ren.feat.fc, prec=prec)
            self.points.index()
            self.points._feats_for_gather()
        if self.fused:  # render + regulation as ONE decoder pass (pnr_map_fwd / pnr_map_bwd)
            from .renderer import MapPass
            mp = MapPass(r, self.c, self.decoder)
            views = self._views['main']
            if self.one_call:  # pnr_map_step: forward, loss and backward in one C call, fused tail
                loss = mp.step(rays_o, rays_d, gt_depth, gt_color, t_rand, self.w_color, self.w_reg,
                               self._loss_ws('main'), views[0], g_fc=views[1], g_feats=views[2],
                               far_clamp=far_clamp, overwrite=True)
                return self._finish(loss)
            d, _, c, sigma = mp.forward(rays_o, rays_d, gt_depth, t_rand, far_clamp=far_clamp)
            loss, g_d, g_c, g_s = map_loss(gt_depth, d, gt_color, c, self.w_color, sigma=sigma, w_reg=self.w_reg,
                                           ws=self._loss_ws('main'))
            views = self._views['main']
            mp.backward(views[0], g_fc=views[1], g_feats=views[2], g_depth=g_d, g_rgb=g_c, g_sigma=g_s,
                        overwrite=True)
            return self._finish(loss)
        main = torch.cuda.current_stream(dev)
        overlap = self._overlaps(rays_o.shape[0])
        if overlap and self.side is None:
            self.side = torch.cuda.Stream(dev)
            self.grad2 = torch.zeros_like(self.flat.grad)
            self._views['side'] = self._split(self.grad2)
        if overlap:
            self.side.wait_stream(main)
            with torch.cuda.stream(self.side):
                self.grad2.zero_()
                l_reg = self._regulation_chain(self._views['side'], rays_o, rays_d, gt_depth, t_rand)
        d, _, c = ren.forward(rays_o, rays_d, gt_depth, far_clamp=far_clamp)
        l_ren, g_d, g_c, _ = map_loss(gt_depth, d, gt_color, c, self.w_color, ws=self._loss_ws('main'))
        views = self._views['main']
        ren.backward(views[0], g_fc=views[1], g_feats=views[2], g_depth=g_d, g_rgb=g_c)
        if overlap:
            main.wait_stream(self.side)
            self.flat.grad.add_(self.grad2)  # render + regulation gradients, a fixed order
        else:
            l_reg = self._regulation_chain(views, rays_o, rays_d, gt_depth, t_rand)
        return self._finish(l_ren + l_reg)

    def _finish(self, loss):
        """The gradient exchange (data parallel) and the Adam step."""
        if self.ddp is not None and self.shard:
            self.ddp.allreduce_(self.flat.grad[:self.n_dec])
            self.ddp.reduce_scatter_(self.flat.grad[self.n_dec:])
        elif self.ddp is not None:
            self.ddp.allreduce_(self.flat.grad)
        self.opt.step()
        if self.shard:
            self.ddp.all_gather_(self.flat.data[self.n_dec:])
            self.points.invalidate_feats()
        return loss

    def loss(self, rays_o, rays_d, gt_depth, gt_color, t_rand=None, far_clamp=None):
        """The Mapper loss through the autograd Renderer API (src/Mapper.py:623-655): the drop-in form
        of what __call__ computes on its fused path."""
        r, dec = self.renderer, self.decoder
        dev = rays_o.device
        d, _, c = r.render_batch_ray(self.c, dec, rays_d, rays_o, dev, 'color', gt_depth, far_clamp=far_clamp)
        m = gt_depth > 0
        loss = torch.where(m, torch.abs(gt_depth - d), torch.zeros_like(d)).sum()
        loss = loss + self.w_color * torch.abs(gt_color - c).sum()
        sigma = r.regulation(self.c, dec, rays_d, rays_o, gt_depth, dev, 'color', t_rand=t_rand)
        return loss + self.w_reg * torch.abs(sigma).sum()


class MapGraph:
    """A MapStep captured once in a HIP graph (torch.cuda.CUDAGraph) and replayed per iteration.

    The Mapper runs `mapping.iters` (60) iterations per keyframe on a fixed-size pixel batch
    (1,000 rays under configs/pointNeRF_slam.yaml); at that size a step is ~130 launches whose host
    overhead rivals the GPU time.  Replaying the captured step removes it.  The graph owns static
    input buffers (rays, gt depth / colour and the regulation jitter t_rand): each call copies the
    batch in, replays, and returns the loss tensor (overwritten by the next call).  Capture needs a
    fixed batch shape and Adam's device step counter (`Adam.use_device_step`).  A caller that
    produces its batch in place (into `inputs`: rays_o, rays_d, gt_depth, gt_color, t_rand) skips the
    five copies, ~25 us of launches at the 1,000-ray batch.  A data-parallel
    step (ddp) is captured with its collectives when the process group is RCCL ('nccl'): the far
    clamp is all-reduced and read on the device (far_mode 2), so the step has no host sync; gloo
    collectives cannot be captured.  `warmup` ordinary steps run first on the given batch (torch
    requires work on a side stream before a capture); they are real optimisation steps.
    """

    def __init__(self, mstep: MapStep, rays_o=None, rays_d=None, gt_depth=None, gt_color=None, t_rand=None,
                 warmup=2, batch_fn=None):
        """`batch_fn` (optional): a callable producing (rays_o, rays_d, gt_depth, gt_color, t_rand) on
        the device -- e.g. a Mapper iteration's window sampling (WindowSampler) -- captured INTO the
        graph together with the step, so each replay draws a fresh batch (torch's CUDA RNG is
        capture-safe); then `__call__()` takes no arguments."""
        if mstep.ddp is not None and getattr(mstep.ddp, 'active', mstep.ddp.world > 1):
            import torch.distributed as dist
            if dist.get_backend(mstep.ddp.group) != 'nccl':
                raise NotImplementedError('pnr.MapGraph: only RCCL (nccl) collectives can be captured in a graph')
        self.mstep = mstep
        self.batch_fn = batch_fn
        if batch_fn is None:
            dev = rays_o.device
            self.inputs = [t.detach().clone() for t in (rays_o, rays_d, gt_depth, gt_color, t_rand)]
            body = lambda: mstep(*self.inputs)  # noqa: E731
        else:
            dev = batch_fn()[0].device
            self.inputs = None
            body = lambda: mstep(*batch_fn())  # noqa: E731
        mstep.opt.use_device_step()
        side = torch.cuda.Stream(dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(warmup):
                body()
        torch.cuda.current_stream(dev).wait_stream(side)
        mstep._invalidate()  # the captured step starts with the weight repack
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.loss = body()

    def __call__(self, rays_o=None, rays_d=None, gt_depth=None, gt_color=None, t_rand=None):
        """Copy the batch into the static inputs (a tensor that IS the static buffer -- the caller
        wrote its batch into `self.inputs` directly -- is not copied), replay, return the loss.  With a
        captured `batch_fn`, just replay."""
        if self.batch_fn is None:
            for dst, src in zip(self.inputs, (rays_o, rays_d, gt_depth, gt_color, t_rand)):
                if src.data_ptr() != dst.data_ptr():
                    dst.copy_(src, non_blocking=True)
        self.graph.replay()
        # the replay moved the weights through Adam's raw pointers (no _version bump) and repacked only
        # the f16x3 images: a later eager call must not reuse a cached image of any precision
        self.mstep.decoder._packed.invalidate()
        if self.mstep.points is not None:
            self.mstep.decoder._packed_fc.invalidate()
        return self.loss


def window_batch(frames, pixs_per_image, H, W, fx, fy, cx, cy, device, generator=None):
    """The per-iteration pixel batch of Mapper.optimize_map (src/Mapper.py:560-606): for every
    frame of the optimisation window, in window order, `pixs_per_image` uniform pixels of the whole
    image (the effective path for every frame index: SURVEY.md appendix item 7), concatenated.
    frames: iterable of (c2w (3x4 or 4x4), gt depth (H,W), gt colour (H,W,3)) device tensors.
    Returns rays_o, rays_d (N,3), gt depth (N,), gt colour (N,3) float32."""
    from .renderer import get_samples
    out = [get_samples(0, H, 0, W, pixs_per_image, H, W, fx, fy, cx, cy, c2w, d, c, device, generator)
           for c2w, d, c in frames]
    return tuple(torch.cat([o[k].float() for o in out], 0) for k in range(4))



def window_rays(idx, n_per_frame, c2w, depth, color, fx, fy, cx, cy):
    """pnr_window_rays: the window batch of `window_batch` in ONE launch, for given pixel indices.
    c2w (F,4,4) / (F,3,4), depth (F,H,W), color (F,H,W,3) device tensors; idx (F * n_per_frame,) int64
    pixels of the whole image (row-major), frame f's rays at [f n, (f+1) n).  Returns rays_o, rays_d
    (N,3), gt depth (N,), gt colour (N,3) float32 -- equal to window_batch's get_samples on the same
    pixel indices (tests/test_gpu_mapping.py)."""
    lib = _lib.load()
    dev = depth.device
    F, H, W = depth.shape
    if c2w.shape[-2] == 3:
        c2w = torch.cat([c2w, torch.tensor([0., 0., 0., 1.], device=dev).expand(F, 1, 4)], 1)
    c2w = c2w.to(device=dev, dtype=torch.float32).contiguous()
    depth = depth.float().contiguous()
    color = color.float().contiguous()
    idx = idx.to(device=dev, dtype=torch.int64).contiguous()
    n = idx.numel()
    _lib.require_cuda(depth, color, idx, c2w)
    ro = torch.empty((n, 3), device=dev)
    rd = torch.empty((n, 3), device=dev)
    gd = torch.empty(n, device=dev)
    gc = torch.empty((n, 3), device=dev)
    _lib.check(lib.pnr_window_rays(_lib.ptr(idx), n, int(n_per_frame), H, W, float(fx), float(fy), float(cx),
                                   float(cy), _lib.ptr(c2w), _lib.ptr(depth), _lib.ptr(color), _lib.ptr(ro),
                                   _lib.ptr(rd), _lib.ptr(gd), _lib.ptr(gc), _lib.stream_of(dev)), 'window_rays')
    return ro, rd, gd, gc


class WindowSampler:
    """A Mapper iteration's batch over a fixed keyframe window (src/Mapper.py:397, 553-606):
    `pixs_per_image` = mapping.pixels // len(window) uniform pixels per frame, their rays, gt depth
    and colour, and the regulation jitter t_rand (Renderer.py:293).
    frames: list of (c2w, gt depth (H,W), gt colour (H,W,3)) device tensors.

    device_rng=True (default): ONE pnr_window_sample launch draws the pixels and the jitter on the
    device (counter-based hash of `seed` and a device batch counter) and also returns the batch far
    clamp max(1.2 gt) as a device scalar -- a captured iteration (MapGraph(batch_fn=sampler)) then
    spends one launch on its batch.  device_rng=False: torch.randint / torch.rand (torch's Philox
    stream, `generator`) + one pnr_window_rays launch; far clamp None (computed by the render pass).
    __call__ returns (rays_o, rays_d, gt_depth, gt_color, t_rand, far_clamp)."""

    def __init__(self, frames, pixs_per_image, fx, fy, cx, cy, n_samples=32, generator=None, device_rng=True,
                 seed=0):
        self.c2w = torch.stack([f[0][:3] if f[0].shape[0] == 3 else f[0] for f in frames]).float()
        if self.c2w.shape[1] == 3:
            self.c2w = torch.cat([self.c2w, torch.tensor([0., 0., 0., 1.], device=self.c2w.device)
                                  .expand(len(frames), 1, 4)], 1)
        self.c2w = self.c2w.contiguous()
        self.depth = torch.stack([f[1].float() for f in frames]).contiguous()
        self.color = torch.stack([f[2].float() for f in frames]).contiguous()
        self.n = int(pixs_per_image)
        self.cam = (fx, fy, cx, cy)
        self.n_samples = n_samples
        self.generator = generator
        self.device_rng = device_rng
        self.seed = int(seed) & ((1 << 64) - 1)
        self.idx = None  # the last batch's pixel indices (device_rng)
        if device_rng:
            lib = _lib.load()
            dev = self.depth.device
            self.state = torch.zeros(lib.pnr_window_sample_state_bytes(), dtype=torch.uint8, device=dev)

    def __call__(self):
        F, H, W = self.depth.shape
        dev = self.depth.device
        N = F * self.n
        if not self.device_rng:
            idx = torch.randint(H * W, (N,), device=dev, generator=self.generator)
            ro, rd, gd, gc = window_rays(idx, self.n, self.c2w, self.depth, self.color, *self.cam)
            t_rand = torch.rand((N, self.n_samples), device=dev, generator=self.generator)
            return ro, rd, gd, gc, t_rand, None
        lib = _lib.load()
        _lib.require_cuda(self.depth, self.color, self.c2w)
        ro = torch.empty((N, 3), device=dev)
        rd = torch.empty((N, 3), device=dev)
        gd = torch.empty(N, device=dev)
        gc = torch.empty((N, 3), device=dev)
        t_rand = torch.empty((N, self.n_samples), device=dev)
        self.idx = torch.empty(N, dtype=torch.int64, device=dev)
        far = torch.empty(1, device=dev)
        _lib.check(lib.pnr_window_sample(self.seed, _lib.ptr(self.state), N, self.n, H, W,
                                         *[float(v) for v in self.cam], _lib.ptr(self.c2w), _lib.ptr(self.depth),
                                         _lib.ptr(self.color), self.n_samples, _lib.ptr(ro), _lib.ptr(rd),
                                         _lib.ptr(gd), _lib.ptr(gc), _lib.ptr(t_rand), _lib.ptr(self.idx),
                                         _lib.ptr(far), _lib.stream_of(dev)), 'window_sample')
        return ro, rd, gd, gc, t_rand, far
