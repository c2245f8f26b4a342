"""Bitwise A/B of two libpnr.so builds on the same inputs (GPU box): the decoder forward (eval and
training) and a full room0-batch MapStep's gradients, f16x3 and fp32.  A kernel change that should
not move a bit (an instruction-level rewrite) is checked with

  python tools/lib_ab.py --lib xlibs/libpnr_head.so --out /tmp/a.pt
  python tools/lib_ab.py --lib pointnerf-slam_amd/pnr/libpnr.so --out /tmp/b.pt --ref /tmp/a.pt
"""
import argparse
import os
import sys
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--lib', required=True)
    ap.add_argument('--out', required=True)
    ap.add_argument('--ref', default=None)
    ap.add_argument('--points', type=int, default=300000)
    args = ap.parse_args()
    import pnr
    pnr._lib.load(os.path.abspath(args.lib))
    from pnr.mapping import MapStep
    dev = torch.device('cuda:0')
    w = np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz'))
    params = {k[len('trained/'):]: torch.from_numpy(w[k]) for k in w.files if k.startswith('trained/')}
    s = np.load(os.path.join(REPO, 'tests', 'golden', 'scene.npz'))
    bound = torch.from_numpy(s['bound'])
    slam = types.SimpleNamespace(bound=bound, H=480, W=640, fx=577.59, fy=578.73, cx=318.91, cy=242.68)
    g = torch.Generator().manual_seed(5)
    pts = (torch.rand(args.points, 3, generator=g, dtype=torch.float64) * 1.2 - 0.35).to(dev)
    import bench
    ro, rd, gt, col = bench.synth_batch(20000, 0, torch.from_numpy(s['poses'][2]), dev)
    t_rand = torch.rand((20000, 32), generator=g).to(dev)
    out = {}
    for prec in ('f16x3', 'fp32'):
        pnr._lib.DEFAULT_PRECISION = prec
        r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
        dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
        dec.load_state_dict(params)
        dec = dec.to(dev)
        out[f'{prec}/eval'] = r.eval_points(pts, dec).detach().cpu()
        ms = MapStep(r, dec, lr=0.0)
        out[f'{prec}/loss'] = torch.tensor([float(ms(ro, rd, gt, col, t_rand))])
        out[f'{prec}/grad'] = ms.flat.grad.detach().cpu().clone()
        x = pts[:50000].float().requires_grad_(True)
        y = dec(x)
        (y * torch.linspace(-1, 1, 4, device=dev)).sum().backward()
        out[f'{prec}/mlp_fwd'] = y.detach().cpu()
        out[f'{prec}/mlp_gx'] = x.grad.detach().cpu()
        out[f'{prec}/mlp_gw'] = torch.cat([p.grad.reshape(-1) for p in dec.parameters() if p.grad is not None]).cpu()
    torch.save(out, args.out)
    if args.ref:
        ref = torch.load(args.ref, weights_only=True)
        ok = True
        for k, v in out.items():
            eq = torch.equal(v, ref[k])
            d = (v.double() - ref[k].double()).abs().max().item()
            print(f'{k:16s} bitwise {eq}  max|d| {d:.3e}  max|ref| {ref[k].abs().max().item():.3e}', flush=True)
            ok = ok and eq
        print('LIB_AB_BITWISE' if ok else 'LIB_AB_DIFFERS', flush=True)


if __name__ == '__main__':
    main()
