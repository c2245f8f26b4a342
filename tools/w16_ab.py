"""A/B of the two f16x3 forward kernels in ONE process (PNR_FWD_W16 is read per launch):
k_mlp_fwd16 (32-point waves, one per SIMD) against k_mlp_fwd16w (16-point waves, two per SIMD,
csrc/mlp16w.h).  Eval and training forwards over P points (device time per launch from
pnr_timing_read), interleaved rounds; outputs of both against the fp32-MFMA forward, and the decoder
gradients of a training forward + backward of each against fp32.

  python tools/w16_ab.py [--points P] [--rounds R]"""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pointnerf-slam_amd'), REPO]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=4 * 1024 * 1024)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--lib', default=None, help='load this libpnr.so build instead (experiments)')
    args = ap.parse_args()
    import pnr
    if args.lib:
        pnr._lib.load(os.path.abspath(args.lib))
    from pnr._lib import timing_read
    dev = torch.device('cuda:0')
    lib = pnr.library()
    w = np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz'))
    params = {k[len('trained/'):]: torch.from_numpy(w[k]) for k in w.files if k.startswith('trained/')}
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    import types
    s = np.load(os.path.join(REPO, 'tests', 'golden', 'scene.npz'))
    slam = types.SimpleNamespace(bound=torch.from_numpy(s['bound']), H=480, W=640, fx=577.59, fy=578.73,
                                 cx=318.91, cy=242.68)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    P = args.points
    g = torch.Generator(device=dev).manual_seed(0)
    pts = torch.rand(P, 3, device=dev, dtype=torch.float64, generator=g) * 1.2 - 0.35
    x = pts.float()
    gout = torch.randn((P, 4), device=dev, generator=g)

    def run(prec, w16, train):
        os.environ['PNR_FWD_VARIANT'] = str(w16)
        r.precision = prec
        dec.precision = prec
        if not train:
            return r.eval_points(pts, dec), None
        dec.zero_grad()
        out = dec(x)
        (out * gout).sum().backward()
        return out.detach(), [p.grad.clone() for p in dec.ordered_params()]

    ref, gref = run('fp32', 0, True)
    ref_e, _ = run('fp32', 0, False)
    for w16 in (0, 1):
        o, _ = run('f16x3', w16, False)
        ot, gr = run('f16x3', w16, True)
        torch.cuda.synchronize()
        e = ((o - ref_e).abs().max() / ref_e.abs().max()).item()
        et = ((ot - ref).abs().max() / ref.abs().max()).item()
        eg = max(((a - b).abs().max() / b.abs().max().clamp_min(1e-30)).item() for a, b in zip(gr, gref))
        print(f'variant {w16}: eval max|d|/max vs fp32 {e:.3e}, training {et:.3e}, grads max rel (per tensor max) {eg:.3e}',
              flush=True)
    lib.pnr_timing_enable(1)
    res = {v: {'eval': [], 'train': []} for v in (0, 1)}
    for rd in range(args.rounds):
        for w16 in (0, 1):
            for mode in ('eval', 'train'):
                timing_read(0)
                for _ in range(args.reps):
                    run('f16x3', w16, mode == 'train')
                torch.cuda.synchronize()
                n, ms, u = timing_read(0)
                res[w16][mode].append(ms / n)
    lib.pnr_timing_enable(0)
    for w16 in (0, 1):
        for mode in ('eval', 'train'):
            v = res[w16][mode]
            tf = 443438 * P / (np.median(v) * 1e-3) / 1e12
            print(f'variant {w16} {mode:5s}: ms per launch median {np.median(v):.3f} min {min(v):.3f} ({tf:.0f} TF/s, '
                  f'{tf / 833.3:.3f} of the split peak)', flush=True)


if __name__ == '__main__':
    main()
