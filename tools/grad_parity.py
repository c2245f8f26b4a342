"""Elementwise gradient parity of the HIP backward vs the reference's golden gradients.

For every decoder tensor: max over elements of |g - g_ref| / (rtol |g_ref| + atol * max|g_ref|)
(<= 1 passes `np.allclose(g, g_ref, rtol, atol * max|g_ref|)`), at rtol 1e-3, atol 1e-6, for each
precision.  usage: python tools/grad_parity.py [precisions...]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pointnerf-slam_amd'), os.path.join(REPO, 'tests')]
from conftest import load_golden, golden_params  # noqa: E402
import pnr  # noqa: E402


def main():
    precs = sys.argv[1:] or ['fp32', 'f16x3', 'bf16x3', 'bf16']
    dev = torch.device('cuda:0')
    G = load_golden('grads.npz')
    S = load_golden('scene.npz')
    import types
    bound = torch.from_numpy(S['bound'])
    for prec in precs:
        dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4,
                      pos_embedding_method='fourier')
        dec.load_state_dict({k: v.clone() for k, v in golden_params('trained').items()})
        dec = dec.to(dev)
        slam = types.SimpleNamespace(bound=bound, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
        cfg = dict(pnr.ROOM0_CFG)
        cfg['pnr'] = {'precision': prec}
        r = pnr.Renderer(cfg, None, slam)
        ro = torch.from_numpy(G['map_rays_o']).to(dev)
        rd = torch.from_numpy(G['map_rays_d']).to(dev)
        gt = torch.from_numpy(G['map_gt_depth']).to(dev)
        gcol = torch.from_numpy(G['map_gt_color']).to(dev)
        d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
        sig = r.regulation({}, dec, rd, ro, gt, dev, 'color', t_rand=torch.from_numpy(G['map_t_rand']).to(dev))
        m = gt > 0
        loss = torch.abs(gt[m] - d[m]).sum() + 0.05 * torch.abs(gcol - c).sum() + 0.0005 * torch.abs(sig).sum()
        loss.backward()
        worst = 0.0
        for k, p in dec.named_parameters():
            gref = G[f'map_grad/{k}']
            g = p.grad.detach().cpu().numpy()
            viol = np.abs(g - gref) / (1e-3 * np.abs(gref) + 1e-6 * np.abs(gref).max())
            rel = np.abs(g - gref).max() / np.abs(gref).max()
            worst = max(worst, viol.max())
            print(f'{prec:7s} {k:24s} viol(rtol1e-3,atol1e-6max)={viol.max():8.3f}  '
                  f'frac>1={np.mean(viol > 1):.2e}  maxabs/max={rel:.2e}')
        print(f'{prec:7s} WORST {worst:.3f}  status={r.status(dev)}', flush=True)


if __name__ == '__main__':
    main()
