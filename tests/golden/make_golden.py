"""Generate the golden parity vectors by importing the REFERENCE renderer (run in the build
container only; the reference tree never travels to the GPU box).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [/root/reference]

Writes small compressed .npz files next to this script:
  weights.npz    decoder state_dicts: trained room0 ckpt (`trained/*`) + seeded init (`random/*`)
  scene.npz      room0 camera, scaled bound, 4 room0 gt poses
  render.npz     render_batch_ray cases: 4 poses x {gt None, gt = rendered, gt with 10% zeros},
                 outputs for all rays + intermediates (z, raw, weights, importance samples)
                 for the first 64 rays of each case; one random-init case; one edge-ray case
  points.npz     eval_points on 4096 float64 points (in and out of the bound)
  kernels.npz    standalone raw2outputs_nerf_color / sample_pdf vectors with edge cases
  grads.npz      mapping-loss grads (incl. regulation with captured t_rand) w.r.t. every
                 decoder tensor; tracking-loss grads w.r.t. rays_o / rays_d
  render_img.npz render_img on a 24x32 frame

Reference entry points used: src/utils/Renderer.py (Renderer), src/common.py
(get_rays_from_uv, raw2outputs_nerf_color, sample_pdf), src/config.py (load_config, get_model).
Checkpoint loaded with torch.load(weights_only=True).
"""
import os
import sys
import types

import numpy as np
import torch

REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))
CKPT = 'output_pointNeRF_SLAM/Replica/room0_gt-pose_depth-supervise-replica-yaml/ckpts/01999.tar'
POSE_IDS = [0, 500, 1000, 1500]
N_RAYS = 512
N_DETAIL = 64


def main():
    torch.set_num_threads(1)
    os.chdir(REF)
    sys.path.insert(0, REF)
    from src import config                                   # noqa: E402
    import src.utils.Renderer as RM                          # noqa: E402
    from src.common import get_rays_from_uv, raw2outputs_nerf_color, sample_pdf  # noqa: E402

    cfg = config.load_config('configs/Replica/room0_point.yaml', 'configs/pointNeRF_slam.yaml')
    ck = torch.load(CKPT, weights_only=True, map_location='cpu')
    trained = config.get_model(cfg, nice=False)
    trained.load_state_dict(ck['decoder_state_dict'])
    torch.manual_seed(0)
    rand_dec = config.get_model(cfg, nice=False)

    # ---- scene: bound exactly as src/NICE_SLAM.py:208-213 computes it
    scale = cfg['scale']
    bound = torch.from_numpy(np.array(cfg['mapping']['bound']) * scale)
    bd = cfg['grid_len']['bound_divisible']
    bound[:, 1] = (((bound[:, 1] - bound[:, 0]) / bd).int() + 1) * bd + bound[:, 0]
    cam = cfg['cam']
    H, W, fx, fy, cx, cy = cam['H'], cam['W'], cam['fx'], cam['fy'], cam['cx'], cam['cy']
    poses = ck['gt_c2w_list'][POSE_IDS].float()
    np.savez_compressed(os.path.join(OUT, 'scene.npz'), bound=bound.numpy(), poses=poses.numpy(),
                        pose_ids=np.array(POSE_IDS), cam=np.array([H, W, fx, fy, cx, cy], dtype=np.float64),
                        bound_cfg=np.array(cfg['mapping']['bound']), scale=scale, bound_divisible=bd)

    wd = {}
    for tag, dec in (('trained', trained), ('random', rand_dec)):
        for k, v in dec.state_dict().items():
            wd[f'{tag}/{k}'] = v.numpy()
    np.savez_compressed(os.path.join(OUT, 'weights.npz'), **wd)

    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=fx, fy=fy, cx=cx, cy=cy)
    renderer = RM.Renderer(cfg, None, slam)

    # ---- recording wrappers around the reference functions (behaviour unchanged)
    rec = {}
    orig_eval, orig_r2o, orig_pdf = RM.Renderer.eval_points, RM.raw2outputs_nerf_color, RM.sample_pdf

    def eval_rec(self, p, decoders, c=None, stage='color', device='cuda:0'):
        out = orig_eval(self, p, decoders, c, stage, device)
        rec.setdefault('eval', []).append((p.detach().clone(), out.detach().clone()))
        return out

    def r2o_rec(raw, z_vals, rays_d, occupancy=False, device='cuda:0'):
        out = orig_r2o(raw, z_vals, rays_d, occupancy=occupancy, device=device)
        rec.setdefault('r2o', []).append((z_vals.detach().clone(), out[3].detach().clone()))
        return out

    def pdf_rec(bins, weights, N_samples, det=False, device='cuda:0'):
        out = orig_pdf(bins, weights, N_samples, det=det, device=device)
        rec.setdefault('pdf', []).append(out.detach().clone())
        return out

    RM.Renderer.eval_points, RM.raw2outputs_nerf_color, RM.sample_pdf = eval_rec, r2o_rec, pdf_rec

    def render(dec, rd, ro, gt):
        rec.clear()
        with torch.no_grad():
            d, v, c = renderer.render_batch_ray({}, dec, rd, ro, 'cpu', 'color', gt_depth=gt)
        z_c, w_c = rec['r2o'][0]
        z_f, w_f = rec['r2o'][1]
        raw_c = rec['eval'][0][1].reshape(rd.shape[0], -1, 4)
        raw_f = rec['eval'][1][1].reshape(rd.shape[0], -1, 4)
        return d, v, c, dict(z_coarse=z_c, w_coarse=w_c, raw_coarse=raw_c, z_samples=rec['pdf'][0],
                             z_fine=z_f, w_fine=w_f, raw_fine=raw_f)

    rng = np.random.default_rng(1234)
    R = {}
    for pi, pid in enumerate(POSE_IDS):
        pix = rng.integers(0, H * W, N_RAYS)
        i = torch.from_numpy((pix % W).astype(np.float32))
        j = torch.from_numpy((pix // W).astype(np.float32))
        ro, rd = get_rays_from_uv(i, j, poses[pi], H, W, fx, fy, cx, cy, 'cpu')
        ro = ro.reshape(-1, 3).contiguous()
        rd = rd.reshape(-1, 3).contiguous()
        d0, _, _, _ = render(trained, rd, ro, None)
        gt_full = d0.float()
        gt_zero = gt_full.clone()
        gt_zero[::10] = 0.0
        for case, gt in (('none', None), ('gt', gt_full), ('gtzero', gt_zero)):
            key = f'p{pi}_{case}'
            d, v, c, ex = render(trained, rd, ro, gt)
            R[f'{key}/rays_o'] = ro.numpy(); R[f'{key}/rays_d'] = rd.numpy()
            if gt is not None:
                R[f'{key}/gt_depth'] = gt.numpy()
            R[f'{key}/depth'] = d.numpy(); R[f'{key}/var'] = v.numpy(); R[f'{key}/rgb'] = c.numpy()
            for k, t in ex.items():
                R[f'{key}/{k}'] = t[:N_DETAIL].numpy()
    # random-init decoder (dense, wild densities)
    ro, rd = R['p2_none/rays_o'][:256], R['p2_none/rays_d'][:256]
    ro, rd = torch.from_numpy(ro), torch.from_numpy(rd)
    d, v, c, ex = render(rand_dec, rd, ro, None)
    R['rand_none/rays_o'] = ro.numpy(); R['rand_none/rays_d'] = rd.numpy()
    R['rand_none/depth'] = d.numpy(); R['rand_none/var'] = v.numpy(); R['rand_none/rgb'] = c.numpy()
    for k, t in ex.items():
        R[f'rand_none/{k}'] = t[:N_DETAIL].numpy()
    # edge rays: zero direction components, origins on / outside the bound
    ro_e = torch.tensor([[0.3, 0.1, 0.1]] * 6 + [[0.99, 0.1, 0.1], [-1.0, 0.1, 0.1]], dtype=torch.float32)
    rd_e = torch.tensor([[0., 0., -1.], [1., 0., 0.], [0., 1., 0.], [0.5, 0., -1.], [0.2, -0.3, -1.],
                         [-1e-3, 2e-3, -1.], [1., 0.1, 0.], [1., 0.1, 0.05]], dtype=torch.float32)
    d, v, c, ex = render(trained, rd_e, ro_e, None)
    R['edge_none/rays_o'] = ro_e.numpy(); R['edge_none/rays_d'] = rd_e.numpy()
    R['edge_none/depth'] = d.numpy(); R['edge_none/var'] = v.numpy(); R['edge_none/rgb'] = c.numpy()
    for k, t in ex.items():
        R[f'edge_none/{k}'] = t.numpy()
    np.savez_compressed(os.path.join(OUT, 'render.npz'), **R)

    # ---- eval_points
    g = torch.Generator().manual_seed(7)
    lo, hi = bound[:, 0], bound[:, 1]
    p = lo + (hi - lo) * (torch.rand((4096, 3), generator=g, dtype=torch.float64) * 1.2 - 0.1)
    with torch.no_grad():
        raw = orig_eval(renderer, p, trained, None, 'color', 'cpu')
    np.savez_compressed(os.path.join(OUT, 'points.npz'), p=p.numpy(), raw=raw.numpy())

    # ---- standalone compositing / pdf vectors
    K = {}
    g = torch.Generator().manual_seed(11)
    n, s = 96, 32
    z = torch.sort(torch.rand((n, s), generator=g, dtype=torch.float64) * 0.6 + 0.05, -1)[0]
    raw = torch.randn((n, s, 4), generator=g) * 3.0
    raw[:8, :, 3] = -torch.rand((8, s), generator=g)          # sigma <= 0 everywhere
    raw[8:16, :, 3] = 100.0                                      # saturated (out-of-bound style)
    raw[16:24, ::3, 3] = 0.0
    rd = torch.randn((n, 3), generator=g)
    rd[24:28, 0] = 0.0
    dm, dv, rgb, w = orig_r2o(raw.clone(), z, rd, occupancy=False, device='cpu')
    K.update(r2o_raw=raw.numpy(), r2o_z=z.numpy(), r2o_rd=rd.numpy(), r2o_depth=dm.numpy(),
             r2o_var=dv.numpy(), r2o_rgb=rgb.numpy(), r2o_w=w.numpy())
    bins = .5 * (z[..., 1:] + z[..., :-1])
    samp = orig_pdf(bins, w[..., 1:-1], 12, det=True, device='cpu')
    K.update(pdf_bins=bins.numpy(), pdf_w=w[..., 1:-1].numpy(), pdf_out=samp.numpy())
    wz = torch.zeros_like(w[..., 1:-1])
    K.update(pdf_w_zero=wz.numpy(), pdf_out_zero=orig_pdf(bins, wz, 12, det=True, device='cpu').numpy())
    np.savez_compressed(os.path.join(OUT, 'kernels.npz'), **K)

    # ---- gradients (A13/A14): mapping loss with regulation, tracking loss w.r.t. rays
    G = {}
    ro = torch.from_numpy(R['p2_gtzero/rays_o'][:256].copy())
    rd = torch.from_numpy(R['p2_gtzero/rays_d'][:256].copy())
    gt = torch.from_numpy(R['p2_gtzero/gt_depth'][:256].copy())
    gcol = torch.rand((256, 3), generator=torch.Generator().manual_seed(5))
    trained.zero_grad()
    d, v, c = renderer.render_batch_ray({}, trained, rd, ro, 'cpu', 'color', gt_depth=gt)
    m = gt > 0
    loss = torch.abs(gt[m] - d[m]).sum() + 0.05 * torch.abs(gcol - c).sum()
    torch.manual_seed(123)
    sig = renderer.regulation({}, trained, rd, ro, gt, 'cpu', 'color')
    torch.manual_seed(123)
    t_rand = torch.rand((256, cfg['rendering']['N_samples']))
    loss = loss + 0.0005 * torch.abs(sig).sum()
    loss.backward()
    G.update(map_rays_o=ro.numpy(), map_rays_d=rd.numpy(), map_gt_depth=gt.numpy(), map_gt_color=gcol.numpy(),
             map_t_rand=t_rand.numpy(), map_sigma=sig.detach().numpy(), map_loss=np.array(loss.item()))
    for k, prm in trained.named_parameters():
        G[f'map_grad/{k}'] = prm.grad.numpy().copy()
    trained.zero_grad()
    ro_l = ro.clone().requires_grad_(True)
    rd_l = rd.clone().requires_grad_(True)
    d, v, c = renderer.render_batch_ray({}, trained, rd_l, ro_l, 'cpu', 'color', gt_depth=gt)
    v = v.detach()
    loss = (torch.abs(gt - d) / torch.sqrt(v + 1e-10))[m].sum() + 0.5 * torch.abs(gcol - c)[m].sum()
    loss.backward()
    G.update(trk_loss=np.array(loss.item()), trk_grad_rays_o=ro_l.grad.numpy(), trk_grad_rays_d=rd_l.grad.numpy())
    for k, prm in trained.named_parameters():
        G[f'trk_grad/{k}'] = prm.grad.numpy().copy()
    trained.zero_grad()
    np.savez_compressed(os.path.join(OUT, 'grads.npz'), **G)

    # ---- render_img on a small frame (gt_depth must be given: Renderer.py:235 reshapes first)
    RM.Renderer.eval_points, RM.raw2outputs_nerf_color, RM.sample_pdf = orig_eval, orig_r2o, orig_pdf
    small = types.SimpleNamespace(bound=bound, H=24, W=32, fx=30.0, fy=30.0, cx=15.5, cy=11.5)
    r2 = RM.Renderer(cfg, None, small, ray_batch_size=300)
    gt_img = torch.full((24, 32), 0.4)
    gt_img[:, :4] = 0.0
    dimg, vimg, cimg = r2.render_img({}, trained, poses[2], 'cpu', 'color', gt_depth=gt_img)
    np.savez_compressed(os.path.join(OUT, 'render_img.npz'), H=24, W=32, fx=30.0, fy=30.0, cx=15.5, cy=11.5,
                        c2w=poses[2].numpy(), gt_depth=gt_img.numpy(), depth=dimg.numpy(), var=vimg.numpy(),
                        rgb=cimg.numpy(), ray_batch_size=300)
    print('golden vectors written to', OUT)


if __name__ == '__main__':
    main()
