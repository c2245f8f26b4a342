"""Tracker iteration throughput on one MI355X.

  python tools/track_bench.py [--iters K] [--warmup W] [--with-weight-grads]

Frame: the room0 camera of configs/Replica/replica.yaml (680x1200, fx=fy=600), pseudo depth =
the trained decoder's own render at room0 pose 1000 (tests/golden), edge crop 100 px, weak depth:
every cropped pixel with depth > 0.01 is a ray (src/Tracker.py:191-251), i.e. ~480k rays per
iteration. One iteration = pnr.tracking.TrackStep: device rays from the camera tensor, render
with gt depth, the Tracker loss, backward to the camera tensor, Adam. Prints one JSON line.
--with-weight-grads also times the same iteration with decoder weight gradients computed (what a
backward that ignored requires_grad would do) for comparison.
"""
import argparse
import json
import os
import sys
import time
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)

from bench import load_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--with-weight-grads', action='store_true')
    args = ap.parse_args()
    import pnr
    dev = torch.device('cuda:0')
    bound, pose, params = load_scene()
    H, W, f, cx, cy = 680, 1200, 600., 599.5, 339.5
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=f, fy=f, cx=cx, cy=cy)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    with torch.no_grad():
        gd, _, gc = r.render_img({}, dec, pose.to(dev), dev, 'color')
    gd, gc = gd.float().contiguous(), gc.float().contiguous()
    step = pnr.TrackStep(r, dec)
    ct = pnr.get_tensor_from_camera(pose).to(dev) + torch.tensor([0.002, -0.001, 0.001, 0.001, 0.003, -0.002, 0.001],
                                                                  device=dev)
    ct.requires_grad_(True)
    opt = torch.optim.Adam([ct], lr=1e-3)
    n_rays = int((gd[100:H - 100, 100:W - 100] > 0.01).sum().item())

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / args.iters

    t = timed(lambda: step(ct, gc, gd, 0, opt))
    out = {'metric': 'tracking rays/sec per Tracker iteration (weak depth, room0 camera)', 'value': round(n_rays / t, 1),
           'unit': 'rays/s', 'ms_per_iter': round(t * 1e3, 3), 'rays_per_iter': n_rays, 'iters': args.iters,
           'warmup': args.warmup, 'precision': dec.precision, 'data': 'pseudo depth = trained room0 decoder render at pose 1000'}
    if args.with_weight_grads:
        def full():
            opt.zero_grad()
            c2w = pnr.get_camera_from_tensor(ct)
            ro, rd, d0, c0 = step.samples(c2w, gd, gc, 0)
            d, v, col = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=d0)
            m = d0 > 0
            loss = (torch.abs(d0 - d) / torch.sqrt(v.detach() + 1e-10))[m].sum() + 0.5 * torch.abs(c0 - col)[m].sum()
            loss.backward()
            opt.step()
            for p in dec.parameters():
                p.grad = None
        out['ms_per_iter_with_weight_grads'] = round(timed(full) * 1e3, 3)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
