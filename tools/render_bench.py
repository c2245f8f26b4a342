"""Full-frame render throughput (Renderer.render_img, the
Visualizer's and the PSNR evaluator's render, src/utils/Renderer.py:205-260) on one MI355X.

  python tools/render_bench.py [--iters K] [--precision P] [--parity-rays R]

Frame: the room0 camera (680x1200, fx=fy=600), trained room0 decoder (tests/golden), pose 1000;
816,000 rays in 100,000-ray chunks as the reference (ray_batch_size), no gt depth.  Parity: R
random pixels of that frame rendered by the oracle (oracle/ref_render.py, CPU) against the same
pixels of the HIP frame (without gt depth every ray is independent of the others).  Prints one
JSON line.
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
    ap.add_argument('--iters', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--precision', default=None)
    ap.add_argument('--parity-rays', type=int, default=2048)
    args = ap.parse_args()
    import pnr
    from oracle import ref_render as ref
    dev = torch.device('cuda:0')
    bound, pose, params = load_scene()
    H, W, f, cx, cy = 680, 1200, 600., 599.5, 339.5
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=f, fy=f, cx=cx, cy=cy)
    cfg = dict(pnr.ROOM0_CFG)
    if args.precision:
        cfg['pnr'] = {'precision': args.precision}
    r = pnr.Renderer(cfg, None, slam)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    c2w = pose.to(dev)
    for _ in range(args.warmup):
        r.render_img({}, dec, c2w, dev, 'color')
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        d, v, c = r.render_img({}, dec, c2w, dev, 'color')
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / args.iters
    n = H * W
    g = torch.Generator().manual_seed(0)
    sel = torch.randperm(n, generator=g)[:args.parity_rays]
    ro, rd = ref.full_frame_rays(H, W, f, f, cx, cy, pose.float())
    ro, rd = ro.reshape(-1, 3)[sel], rd.reshape(-1, 3)[sel]
    dr, _, cr = ref.render_batch_ray(params, rd, ro, bound)
    dg = d.reshape(-1)[sel.to(dev)].cpu()
    cg = c.reshape(-1, 3)[sel.to(dev)].cpu()
    rel = float(((dg - dr).abs() / dr.abs().clamp_min(1e-12)).max())
    print(json.dumps({'metric': 'full-frame render_img rays/sec (room0 camera, 680x1200)', 'value': round(n / t, 1),
                      'unit': 'rays/s', 'ms_per_frame': round(t * 1e3, 3), 'rays': n, 'iters': args.iters,
                      'precision': r.precision,
                      'parity': {'rays': args.parity_rays, 'psnr_db_vs_oracle': round(ref.psnr(cg, cr), 2),
                                 'depth_max_rel': float(f'{rel:.3g}')}}))


if __name__ == '__main__':
    main()
