"""One Tracker iteration on the HIP path (src/Tracker.py:253-335).

`TrackStep` is Tracker.optimize_cam_in_batch:
- pixel sampling in the edge-cropped frame (`get_samples`, :191-251): every pixel with depth
  > 0.01 under weak depth, in `np.where` (row-major) order, else `torch.randint` pixels;
- rays from the differentiable camera tensor (A3, `get_camera_from_tensor`);
- `render_batch_ray` with gt depth (:300-303);
- the loss: |gt_d - d| / sqrt(var.detach() + 1e-10) over gt > 0, plus w_color * |gt_c - c|
  over gt > 0 (:305-330), with the handle_dynamic median mask as an option;
- backward and the camera optimizer step (:332-335).

`track_frame` is the per-frame loop of Tracker.run (:860-921): Adam on the camera tensor (or
on T and quad separately, lr and 0.2 lr), keeping the minimum-loss candidate.

Data parallel (`TrackStep(ddp=pnr.dist.DataParallel())`): every rank draws the
same pixel set (weak depth: deterministic; random pixels: pass the same-seeded `generator` on every
rank) and renders its contiguous shard of it; the batch-global far clamp is an all_reduce(MAX)
read on the device, the dynamic-object median (handle_dynamic) runs over the all-gathered
residuals, and the camera gradient and the loss are all_reduce(SUM)ed before the camera Adam
step -- the loss is a sum over pixels, so every rank then takes the single-process step.

The rays are built on the device by `pnr_rays_from_uv`.  `_RaysFromUV`
carries the gradient to the 3x4 pose: dL/dR = g_dᵀ·dirs and dL/dt = Σ g_o, the exact adjoint
of rays_d = Σ_c dirs_c R[:, c] and rays_o = t.  The decoder's parameters get no gradient:
the Tracker only optimises the camera.
"""
from __future__ import annotations

import torch

from . import _lib
from .common import get_camera_from_tensor, select_uv_indices
from .dist import shard_bounds


class _RaysFromUV(torch.autograd.Function):
    @staticmethod
    def forward(ctx, c2w34, i, j, fx, fy, cx, cy):
        lib = _lib.load()
        dev = c2w34.device
        c2w = torch.cat([c2w34.detach().float(), torch.tensor([[0., 0., 0., 1.]], device=dev)], 0).contiguous()
        i = i.reshape(-1).float().contiguous()
        j = j.reshape(-1).float().contiguous()
        _lib.require_cuda(c2w, i, j)
        n = i.shape[0]
        ro = torch.empty((n, 3), dtype=torch.float32, device=dev)
        rd = torch.empty((n, 3), dtype=torch.float32, device=dev)
        if n:
            _lib.check(lib.pnr_rays_from_uv(_lib.ptr(i), _lib.ptr(j), n, float(fx), float(fy), float(cx), float(cy),
                                            _lib.ptr(c2w), _lib.ptr(ro), _lib.ptr(rd), _lib.stream_of(dev)),
                       'rays_from_uv')
        ctx.save_for_backward(i, j)
        ctx.k = (fx, fy, cx, cy)
        return ro, rd

    @staticmethod
    def backward(ctx, g_ro, g_rd):
        i, j = ctx.saved_tensors
        fx, fy, cx, cy = ctx.k
        dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
        g = torch.zeros((3, 4), dtype=torch.float32, device=i.device)
        if g_rd is not None:
            g[:, :3] = g_rd.t() @ dirs
        if g_ro is not None:
            g[:, 3] = g_ro.sum(0)
        return g, None, None, None, None, None, None


def rays_from_uv(i, j, c2w34, fx, fy, cx, cy):
    """src/common.py:74-89 with the pose differentiable: (N,3) rays_o, rays_d float32."""
    return _RaysFromUV.apply(c2w34, i, j, fx, fy, cx, cy)


class TrackStep:
    def __init__(self, renderer, decoder, c=None, w_color_loss=0.5, use_color_in_tracking=True,
                 depth_supervision=True, handle_dynamic=False, weak_depth=True, ignore_edge_W=100,
                 ignore_edge_H=100, generator=None, ddp=None):
        self.renderer = renderer
        self.ddp = ddp if (ddp is not None and ddp.world > 1) else None
        self.rays_fn = rays_from_uv  # (i, j, c2w34, fx, fy, cx, cy) -> rays_o, rays_d
        self.decoder = decoder
        self.c = {} if c is None else c
        self.w_color = w_color_loss
        self.use_color = use_color_in_tracking
        self.depth_supervision = depth_supervision
        self.handle_dynamic = handle_dynamic
        self.weak_depth = weak_depth
        self.Wedge = ignore_edge_W
        self.Hedge = ignore_edge_H
        self.generator = generator

    def samples(self, c2w, gt_depth, gt_color, n):
        """get_samples (src/Tracker.py:191-251 under weak depth, src/common.py:92-134 else):
        rays_o, rays_d, depth (N,), colour (N,3) of the sampled pixels."""
        r = self.renderer
        H, W = r.H, r.W
        H0, H1, W0, W1 = self.Hedge, H - self.Hedge, self.Wedge, W - self.Wedge
        depth = gt_depth[H0:H1, W0:W1].reshape(-1)
        color = gt_color[H0:H1, W0:W1].reshape(-1, 3)
        if self.weak_depth:
            idx = torch.nonzero(depth > 0.01).reshape(-1)
        else:
            idx = select_uv_indices(depth.numel(), n, depth.device, self.generator)
        if self.ddp is not None:  # this rank's contiguous shard of the (identical) global pixel set
            import torch.distributed as dist
            a, b = shard_bounds(idx.numel(), dist.get_rank(self.ddp.group), self.ddp.world)
            idx = idx[a:b]
        w = W1 - W0
        i = (idx % w + W0).float()
        j = (torch.div(idx, w, rounding_mode='floor') + H0).float()
        ro, rd = self.rays_fn(i, j, c2w, r.fx, r.fy, r.cx, r.cy)
        return ro, rd, depth[idx], color[idx]

    def _global_median(self, t):
        """torch.median over every rank's values (the lower median, as torch.median)."""
        import torch.distributed as dist
        n = torch.tensor([t.numel()], device=t.device, dtype=torch.int64)
        ns = [torch.zeros_like(n) for _ in range(self.ddp.world)]
        dist.all_gather(ns, n, group=self.ddp.group)
        m = int(max(int(x) for x in ns))
        buf = torch.zeros(m, device=t.device, dtype=t.dtype)
        buf[:t.numel()] = t
        outs = [torch.zeros_like(buf) for _ in range(self.ddp.world)]
        dist.all_gather(outs, buf, group=self.ddp.group)
        return torch.cat([o[:int(k)] for o, k in zip(outs, ns)]).median()

    def loss(self, camera_tensor, gt_color, gt_depth, batch_size):
        dec = self.decoder
        # the Tracker optimises the camera only (src/Tracker.py:870-874): decoder weights and point
        # features take no gradient (no weight-gradient GEMMs, no feature atomics)
        frozen = list(dec.parameters()) + [v.feats for v in self.c.values() if hasattr(v, 'feats')]
        req = [p.requires_grad for p in frozen]
        for p in frozen:
            p.requires_grad_(False)
        try:
            c2w = get_camera_from_tensor(camera_tensor)
            ro, rd, gd, gc = self.samples(c2w, gt_depth, gt_color, batch_size)
            fc = self.ddp.global_far_clamp(gd) if self.ddp is not None else None
            d, v, col = self.renderer.render_batch_ray(self.c, dec, rd, ro, rd.device, 'color', gt_depth=gd,
                                                       far_clamp=fc)
        finally:
            for p, q in zip(frozen, req):
                p.requires_grad_(q)
        v = v.detach()
        if self.handle_dynamic:
            tmp = torch.abs(gd - d) / torch.sqrt(v + 1e-10)
            med = self._global_median(tmp.detach()) if self.ddp is not None else tmp.median()
            mask = (tmp < 10 * med) & (gd > 0)
        else:
            mask = gd > 0
        if not self.depth_supervision:
            return torch.abs(gc - col)[mask].sum()
        loss = (torch.abs(gd - d) / torch.sqrt(v + 1e-10))[mask].sum()
        if self.use_color:
            loss = loss + self.w_color * torch.abs(gc - col)[mask].sum()
        return loss

    def __call__(self, camera_tensor, gt_color, gt_depth, batch_size, optimizer):
        optimizer.zero_grad()
        loss = self.loss(camera_tensor, gt_color, gt_depth, batch_size)
        loss.backward()
        if self.ddp is not None:  # the pixel-sum loss: summed camera gradients = the full-batch step
            for grp in optimizer.param_groups:
                for p in grp['params']:
                    if p.grad is not None:
                        self.ddp.allreduce_(p.grad)
            loss = self.ddp.allreduce_(loss.detach().reshape(1).clone())
        optimizer.step()
        optimizer.zero_grad()
        return float(loss.reshape(-1)[0].item())


def track_frame(step: TrackStep, camera_tensor, gt_color, gt_depth, iters, cam_lr, batch_size,
                separate_lr=False):
    """src/Tracker.py:860-921: optimise the camera tensor for `iters` iterations from its initial
    value; returns (minimum-loss camera tensor, its 4x4 c2w, the per-iteration losses)."""
    dev = gt_depth.device
    camera_tensor = camera_tensor.detach().to(dev).clone()
    if separate_lr:
        T = camera_tensor[-3:].clone().requires_grad_(True)
        quad = camera_tensor[:4].clone().requires_grad_(True)
        opt = torch.optim.Adam([{'params': [T], 'lr': cam_lr}, {'params': [quad], 'lr': cam_lr * 0.2}])
    else:
        camera_tensor.requires_grad_(True)
        opt = torch.optim.Adam([camera_tensor], lr=cam_lr)
    best, best_loss, losses = None, 1e10, []
    for _ in range(iters):
        if separate_lr:
            camera_tensor = torch.cat([quad, T], 0)
        loss = step(camera_tensor, gt_color, gt_depth, batch_size, opt)
        losses.append(loss)
        if loss < best_loss:
            best_loss = loss
            best = camera_tensor.clone().detach()
    c2w = get_camera_from_tensor(best.clone())
    c2w = torch.cat([c2w, torch.tensor([[0., 0., 0., 1.]], device=dev)], 0)
    return best, c2w, losses
