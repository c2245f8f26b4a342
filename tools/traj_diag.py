"""Diagnose f16x3-vs-fp32 drift over Mapper iterations (tests/test_gpu_precision.py trajectory).

Runs 50 MapStep iterations 2x in fp32 and 2x in f16x3 on identical batches; prints pairwise weight
drift and, at step 1 (same weights), the gradient elements that are exactly 0 in one mode but not
the other, and the sign agreement of the Adam-normalised first update."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pointnerf-slam_amd'), os.path.join(REPO, 'tests')]
from conftest import load_golden, golden_params  # noqa: E402
import pnr  # noqa: E402
from pnr.mapping import MapStep  # noqa: E402


def main():
    dev = torch.device('cuda:0')
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    import types
    params = golden_params('trained')
    g = torch.Generator().manual_seed(11)
    n, steps = 2048, int(sys.argv[1]) if len(sys.argv) > 1 else 50
    batches = []
    for s in range(steps):
        c2w = torch.from_numpy(scene['poses'][s % 4]).float()
        i = torch.randint(0, 1200, (n,), generator=g).float()
        j = torch.randint(0, 680, (n,), generator=g).float()
        batches.append((c2w, i, j, torch.rand(n, generator=g) * 0.4 + 0.15, torch.rand((n, 3), generator=g),
                        torch.rand((n, 32), generator=g)))
    runs = {}
    grads1 = {}
    for tag in ('fp32_a', 'fp32_b', 'f16x3_a', 'f16x3_b'):
        prec = tag.split('_')[0]
        dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4)
        dec.load_state_dict({k: v.clone() for k, v in params.items()})
        dec = dec.to(dev)
        slam = types.SimpleNamespace(bound=bound, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
        cfg = dict(pnr.ROOM0_CFG)
        cfg['pnr'] = {'precision': prec}
        r = pnr.Renderer(cfg, None, slam)
        ms = MapStep(r, dec, lr=2e-4, w_color_loss=0.05)
        losses = []
        for s, (c2w, i, j, gt, col, tr) in enumerate(batches):
            ro, rd = pnr.get_rays_from_uv(i.to(dev), j.to(dev), c2w.to(dev), 680, 1200, 600., 600., 599.5, 339.5,
                                          dev)
            losses.append(float(ms(ro, rd, gt.to(dev), col.to(dev), tr.to(dev))))
            if s == 0:
                grads1[tag] = ms.flat.grad.detach().cpu().clone()
        runs[tag] = (np.array(losses), ms.flat.data.detach().cpu().clone())
    thr = 1e-3 * 2e-4 * steps
    tags = list(runs)
    for a in range(len(tags)):
        for b in range(a + 1, len(tags)):
            la, wa = runs[tags[a]]
            lb, wb = runs[tags[b]]
            dw = (wa - wb).abs()
            print(f'{tags[a]:8s} vs {tags[b]:8s}: loss rel max {np.max(np.abs(la - lb) / np.abs(la)):.2e}  '
                  f'weights > {thr:.0e}: {(dw > thr).float().mean():.4f}  max {dw.max():.2e}')
    from pnr.decoder import PARAM_ORDER
    shapes = {k: tuple(v.shape) for k, v in params.items()}
    off = 0
    ga, gb = grads1['fp32_a'], grads1['f16x3_a']
    for k in PARAM_ORDER:
        nk = int(np.prod(shapes[k]))
        a, b = ga[off:off + nk].reshape(shapes[k]), gb[off:off + nk].reshape(shapes[k])
        extra = torch.nonzero((b == 0) & (a != 0))
        rel = ((a - b).abs().max() / a.abs().max()).item()
        worst = torch.argmax((a - b).abs()).item()
        print(f'{k:24s} max|diff|/max {rel:.2e} at {np.unravel_index(worst, shapes[k])} '
              f'(fp32 {a.reshape(-1)[worst]:.3e}, f16x3 {b.reshape(-1)[worst]:.3e}); '
              f'zero only in f16x3: {extra.shape[0]} {extra[:6].tolist()}')
        off += nk
    # the correctly-rounded gradient of step 1 (oracle, float64 GEMM sums rounded per layer)
    from oracle import ref_render as ref
    torch.set_num_threads(16)
    c2w, i, j, gt, col, tr = batches[0]
    ro, rd = ref.rays_from_uv(i, j, c2w, 600., 600., 599.5, 339.5)
    ro, rd = ro.reshape(-1, 3).contiguous(), rd.reshape(-1, 3).contiguous()
    pr = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    ev = lambda q: ref.eval_points_cr(pr, q, bound)  # noqa: E731
    d, v, c = ref.render_batch_ray(pr, rd, ro, bound, gt_depth=gt, eval_fn=ev)
    sig = ref.regulation(pr, rd, ro, gt, bound, t_rand=tr, eval_fn=ev)
    ref.mapping_loss(d, c, gt, col, sig).backward()
    off = 0
    for k in PARAM_ORDER:
        nk = int(np.prod(shapes[k]))
        cr = pr[k].grad.reshape(-1)
        for tag in ('fp32_a', 'f16x3_a'):
            gx = grads1[tag][off:off + nk]
            rel = ((gx - cr).abs().max() / cr.abs().max()).item()
            zeros = int(((gx == 0) & (cr != 0)).sum())
            viol = ((gx - cr).abs() / (1e-3 * cr.abs() + 1e-6 * cr.abs().max())).max().item()
            print(f'  vs CR {tag:8s} {k:24s} max|diff|/max {rel:.2e}  viol(1e-3,1e-6) {viol:8.2f}  '
                  f'zero where CR is not: {zeros}')
        off += nk
    if len(sys.argv) > 2:
        return
    for a, b in (('fp32_a', 'fp32_b'), ('fp32_a', 'f16x3_a'), ('f16x3_a', 'f16x3_b')):
        ga, gb = grads1[a], grads1[b]
        z_a, z_b = ga == 0, gb == 0
        sign = (torch.sign(ga) == torch.sign(gb)).float().mean()
        rel = (ga - gb).abs().max() / ga.abs().max()
        print(f'step-1 grads {a} vs {b}: zero in one only: {int((z_a ^ z_b).sum())} '
              f'(zeros {int(z_a.sum())}/{int(z_b.sum())}), sign agreement {sign:.5f}, max|diff|/max {rel:.2e}')
        small = ga.abs() < 1e-6 * ga.abs().max()
        print(f'    elements below 1e-6 max: {int(small.sum())}, their sign agreement '
              f'{(torch.sign(ga[small]) == torch.sign(gb[small])).float().mean():.4f}')


if __name__ == '__main__':
    main()
