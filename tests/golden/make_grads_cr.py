"""Correctly-rounded Mapper-loss gradients (tests/golden/grads_cr.npz) -- test infrastructure.

Same inputs as grads.npz's map case (made by importing the reference, make_golden.py), evaluated by
the oracle (oracle/ref_render.py, pinned bit-exactly to the reference by test_oracle_golden.py) with
oracle.ref_render.mlp_forward_cr: every hidden / output GEMM summed in float64 and rounded to
float32 per layer, forward and backward.  The reference's own float32 gradient (grads.npz) differs
from this by its summation-order rounding (up to ~4e-6 of max|g| per tensor, recorded in
`golden_vs_cr/<name>`); an fp32-class implementation is judged against both.

    python tests/golden/make_grads_cr.py     (CPU, ~1 min; no reference import)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, 'tests')]
from conftest import load_golden, golden_params  # noqa: E402
from oracle import ref_render as ref  # noqa: E402
from oracle import ref_points as RP  # noqa: E402


def _rel(g, gref):
    return np.array(np.abs(g - gref).max() / max(np.abs(g).max(), 1e-30))


def track_scene(bound):
    """The weak-depth frame of tests/test_gpu_parity.py::_track_scene: a 68x120 oracle render at
    room0 pose 1 (every 7th row / 5th column depth zeroed) and a camera tensor perturbed off it."""
    params = golden_params('trained')
    H, W, fx, fy, cx, cy = 68, 120, 60., 60., 59.5, 33.5
    c2w = torch.from_numpy(load_golden('scene.npz')['poses'][1]).float()
    gd, _, gc = ref.render_img(params, c2w, bound, H, W, fx, fy, cx, cy)
    gd = gd.float().clone()
    gd[::7, ::5] = 0.
    ct0 = ref.tensor_from_camera(c2w) + torch.tensor([0.003, -0.002, 0.001, 0.002, 0.004, -0.003, 0.002])
    return params, (H, W, fx, fy, cx, cy), gd, gc.float(), ct0


def camera_grad(params, cam, gd, gc, ct0, bound, eval_fn=None, e=10):
    """Tracker.optimize_cam_in_batch's loss (src/Tracker.py:253-330, weak depth, edge e) and its
    camera-tensor gradient."""
    H, W, fx, fy, cx, cy = cam
    crop = gd[e:H - e, e:W - e].reshape(-1)
    idx = torch.nonzero(crop > 0.01).reshape(-1)
    i = (idx % (W - 2 * e) + e).float()
    j = (idx // (W - 2 * e) + e).float()
    ct = ct0.clone().requires_grad_(True)
    ro, rd = ref.rays_from_uv(i, j, ref.camera_from_tensor(ct), fx, fy, cx, cy)
    g_d, g_c = crop[idx], gc[e:H - e, e:W - e].reshape(-1, 3)[idx]
    d, v, c = ref.render_batch_ray(params, rd.reshape(-1, 3), ro.reshape(-1, 3), bound, gt_depth=g_d,
                                   eval_fn=eval_fn)
    loss = ref.tracking_loss(d, v, c, g_d, g_c)
    loss.backward()
    return loss.item(), ct.grad.numpy().copy()


def main():
    torch.set_num_threads(8)
    G = load_golden('grads.npz')
    bound = torch.from_numpy(load_golden('scene.npz')['bound'])
    p = {k: v.clone().requires_grad_(True) for k, v in golden_params('trained').items()}
    ro, rd = torch.from_numpy(G['map_rays_o']), torch.from_numpy(G['map_rays_d'])
    gt, gc = torch.from_numpy(G['map_gt_depth']), torch.from_numpy(G['map_gt_color'])
    ev = lambda q: ref.eval_points_cr(p, q, bound)  # noqa: E731
    d, v, c = ref.render_batch_ray(p, rd, ro, bound, gt_depth=gt, eval_fn=ev)
    sig = ref.regulation(p, rd, ro, gt, bound, t_rand=torch.from_numpy(G['map_t_rand']), eval_fn=ev)
    loss = ref.mapping_loss(d, c, gt, gc, sig)
    loss.backward()
    out = {'map_loss': np.array(loss.item())}
    for k, t in p.items():
        g = t.grad.numpy().copy()
        gref = G[f'map_grad/{k}']
        out[f'map_grad/{k}'] = g
        out[f'golden_vs_cr/{k}'] = np.array(np.abs(g - gref).max() / np.abs(g).max())
        print(f'{k:24s} |golden - cr| / max = {out[f"golden_vs_cr/{k}"]:.2e}')

    # Tracker loss w.r.t. the rays (grads.npz trk case: frozen decoder, var detached)
    pf = golden_params('trained')
    ro_l, rd_l = ro.clone().requires_grad_(True), rd.clone().requires_grad_(True)
    d, v, c = ref.render_batch_ray(pf, rd_l, ro_l, bound, gt_depth=gt,
                                   eval_fn=lambda q: ref.eval_points_cr(pf, q, bound))
    m = gt > 0
    loss = (torch.abs(gt - d) / torch.sqrt(v.detach() + 1e-10))[m].sum() + 0.5 * torch.abs(gc - c)[m].sum()
    loss.backward()
    for a, t in (('o', ro_l), ('d', rd_l)):
        out[f'trk_grad_rays_{a}'] = t.grad.numpy().copy()
        out[f'golden_vs_cr/trk_rays_{a}'] = _rel(t.grad.numpy(), G[f'trk_grad_rays_{a}'])
        print(f'trk rays_{a:20s} |golden - cr| / max = {out[f"golden_vs_cr/trk_rays_{a}"]:.2e}')

    # Tracker camera-tensor gradient on the weak-depth frame
    params, cam, gd, gcf, ct0 = track_scene(bound)
    l32, g32 = camera_grad(params, cam, gd, gcf, ct0, bound)
    lcr, gcr = camera_grad(params, cam, gd, gcf, ct0, bound, eval_fn=lambda q: ref.eval_points_cr(params, q, bound))
    out.update({'cam/gt_depth': gd.numpy(), 'cam/gt_color': gcf.numpy(), 'cam/ct0': ct0.numpy(),
                'cam/loss_f32': np.array(l32), 'cam/loss_cr': np.array(lcr), 'cam/grad_f32': g32, 'cam/grad_cr': gcr,
                'golden_vs_cr/cam': _rel(gcr, g32)})
    print(f'camera tensor            |f32 oracle - cr| / max = {out["golden_vs_cr/cam"]:.2e}')

    # neural-point decoder (points_c32.npz: the reference MLP(c_dim=32) + F.grid_sample)
    P = load_golden('points_c32.npz')
    pb = torch.from_numpy(P['bound'])
    grid = torch.from_numpy(P['grid'])
    D, Hh, Ww = grid.shape[2:]
    xyz, sp = RP.grid_vertices(pb, D, Hh, Ww)
    feats = RP.grid_features(grid).clone().requires_grad_(True)
    prm = {k[2:]: torch.from_numpy(P[k]).clone().requires_grad_(True) for k in P if k.startswith('w/')}
    pp = torch.from_numpy(P['p']).requires_grad_(True)
    cfe = RP.point_gather(pp, xyz, feats, 'trilinear', spacing=sp, k=8)
    raw = RP.mlp_forward_c_cr(prm, pp, cfe)
    (raw.double() * torch.from_numpy(P['g_raw']).double()).sum().backward()
    for k, t in prm.items():
        out[f'pts/grad/{k}'] = t.grad.numpy().copy()
        out[f'golden_vs_cr/pts/{k}'] = _rel(t.grad.numpy(), P['grad/' + k])
    out['pts/grad_feats'] = feats.grad.numpy().copy()
    out['golden_vs_cr/pts/grad_feats'] = _rel(feats.grad.numpy(),
                                              RP.grid_features(torch.from_numpy(P['grad_grid'])).numpy())
    out['pts/grad_p'] = pp.grad.numpy().copy()
    out['golden_vs_cr/pts/grad_p'] = _rel(pp.grad.numpy(), P['grad_p'])
    for k in sorted(x for x in out if x.startswith('golden_vs_cr/pts/')):
        print(f'{k[17:]:24s} |golden - cr| / max = {out[k]:.2e}')
    np.savez_compressed(os.path.join(HERE, 'grads_cr.npz'), **out)


if __name__ == '__main__':
    main()
