"""PSNR clause of the metric ("PSNR delta vs ref <= 0.1 dB", BASELINE.json) measured per decoder
precision on a proxy ground truth with a realistic residual.

The reference's PSNR compares a render with the captured frame; a SLAM render sits at 25-35 dB of
it.  Here the ground truth is proxied by the fp32 render plus i.i.d. Gaussian noise scaled for
P_ref = 25 / 30 / 35 dB (fp32 against the proxy), and every precision's render is scored against
the same proxy: delta = PSNR(precision, proxy) - PSNR(fp32, proxy).  The direct PSNR against the
fp32 render is printed too (the render-level distance alone).

Scenes: (a) room0: the trained decoder (tests/golden) at pose 1000 on the 680x1200 camera, every
2nd pixel (340 x 600); (b) C3: the office3 200k-neural-point scene of tests/test_gpu_configs.py
(IDW r = 1 cm, c_dim 32 decoder), same sub-sampling.  No gt depth (the evaluator's render).

  python tools/psnr_delta.py > profiles/<tag>_psnr_delta.json"""
import json
import math
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pointnerf-slam_amd'), REPO, os.path.join(REPO, 'tests')]

PRECISIONS = ('fp32', 'f16x3', 'bf16x3', 'bf16')


def frame_rays(c2w, H, W, fx, fy, cx, cy, step, dev):
    j, i = torch.meshgrid(torch.arange(0, H, step).float(), torch.arange(0, W, step).float(), indexing='ij')
    dirs = torch.stack([(i - cx) / fx, -(j - cy) / fy, -torch.ones_like(i)], -1)
    rd = (dirs[..., None, :] * c2w[:3, :3]).sum(-1).reshape(-1, 3)
    ro = c2w[:3, 3].expand(rd.shape).contiguous()
    return ro.to(dev), rd.contiguous().to(dev)


def render(pnr, slam, dec, c, ro, rd, precision, dev, chunk=100_000):
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr.Renderer(cfg, None, slam)
    out = []
    with torch.no_grad():
        for a in range(0, ro.shape[0], chunk):
            out.append(r.render_batch_ray(c, dec, rd[a:a + chunk], ro[a:a + chunk], dev, 'color')[2])
    assert r.status(dev) == 0
    return torch.cat(out).clamp(0, 1).double()


def psnr(a, b):
    mse = float(((a - b) ** 2).mean())
    return 10 * math.log10(1.0 / mse) if mse > 0 else float('inf')


def score(renders, seed=0):
    ref = renders['fp32']
    out = {'direct_psnr_vs_fp32_db': {p: round(psnr(renders[p], ref), 2) for p in PRECISIONS if p != 'fp32'}}
    g = torch.Generator(device=ref.device).manual_seed(seed)
    noise = torch.randn(ref.shape, generator=g, device=ref.device, dtype=torch.float64)
    for target in (25.0, 30.0, 35.0):
        sigma = math.sqrt(10 ** (-target / 10))
        proxy = ref + sigma * noise
        p_ref = psnr(ref, proxy)
        out[f'P_ref_{int(target)}dB'] = {
            'fp32_vs_proxy_db': round(p_ref, 4),
            'delta_db': {p: round(psnr(renders[p], proxy) - p_ref, 5) for p in PRECISIONS if p != 'fp32'}}
    return out


def main():
    import pnr
    from bench import load_scene
    import test_gpu_configs as TC
    pnr.library()
    dev = torch.device('cuda:0')
    res = {'what': __doc__.split('\n\n')[1].replace('\n', ' ')}
    bound, pose, params = load_scene()
    H, W, f, cx, cy = 680, 1200, 600., 599.5, 339.5
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=f, fy=f, cx=cx, cy=cy)
    ro, rd = frame_rays(pose.float(), H, W, f, f, cx, cy, 2, dev)
    renders = {}
    for p in PRECISIONS:
        dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
        dec.load_state_dict(params)
        dec = dec.to(dev)
        renders[p] = render(pnr, slam, dec, {}, ro, rd, p, dev)
    res['room0'] = dict(rays=int(ro.shape[0]), **score(renders))
    print(json.dumps(res['room0']), file=sys.stderr, flush=True)
    cam3 = (680, 1200, 600., 600., 599.5, 339.5)
    bound, xyz, feats, params, _, _, slam, pts = TC.scene_case(pnr, dev, TC.OFFICE3, *cam3, 200_000, 8, 0.01, seed=31)
    ro, rd = frame_rays(TC.centre_pose(bound), *cam3, 2, dev)
    renders = {p: render(pnr, slam, TC.make_decoder(pnr, params, dev, p), {'points_color': pts}, ro, rd, p, dev)
               for p in PRECISIONS}
    res['C3'] = dict(rays=int(ro.shape[0]), points=int(xyz.shape[0]), **score(renders))
    print(json.dumps(res['C3']), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
