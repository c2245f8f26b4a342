"""The neural-point Mapper iteration at its faithful batch sizes (BASELINE configs C3: office3, 200k
points, mapping.pixels 1,000; C5: Apartment, 1M float16-feature points, 5,000 pixels), eager and
replayed from a captured HIP graph, for rocprofv3 kernel traces (the scenes of tests/test_gpu_configs.py).

  python tools/np_faithful.py [--case C3|C5] [--iters N] [--mode graph|eager|both] [--precision P]

Prints one JSON line: ms per iteration eager and replayed.  Under `rocprofv3 --kernel-trace` the
iterations split at each k_adam_dev launch (tools/timeline.py)."""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, 'pointnerf-slam_amd'), REPO, os.path.join(REPO, 'tests')]

from oracle import ref_render as RR  # noqa: E402  (scene construction only, never timed)
import test_gpu_configs as TC  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--case', default='C3', choices=['C3', 'C5'])
    ap.add_argument('--iters', type=int, default=50)
    ap.add_argument('--mode', default='both', choices=['graph', 'eager', 'both'])
    ap.add_argument('--precision', default='f16x3')
    ap.add_argument('--rays', type=int, default=None)
    args = ap.parse_args()
    import pnr
    from pnr.mapping import MapGraph, MapStep
    pnr.library()
    dev = torch.device('cuda:0')
    if args.case == 'C3':
        cam = (680, 1200, 600., 600., 599.5, 339.5)
        scene = TC.scene_case(pnr, dev, TC.OFFICE3, *cam, 200_000, 8, 0.01, seed=31)
        n = args.rays or 1000
    else:
        cam = (720, 1280, 607.4694, 607.4535, 636.9967, 369.2690)
        scene = TC.scene_case(pnr, dev, TC.APARTMENT, *cam, 1_000_000, 8, 0.008, seed=41, feat_dtype='float16')
        n = args.rays or 5000
    bound, xyz, feats, params, _, _, slam, pts = scene
    H, W, fx, fy, cx, cy = cam
    dec = TC.make_decoder(pnr, params, dev, args.precision)
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': args.precision}
    r = pnr.Renderer(cfg, None, slam)
    g = torch.Generator().manual_seed(3)
    pix = torch.randint(0, H * W, (n,), generator=g)
    ro, rd = RR.rays_from_uv((pix % W).float(), (pix // W).float(), TC.centre_pose(bound), fx, fy, cx, cy)
    ro, rd = ro.reshape(-1, 3).to(dev), rd.reshape(-1, 3).to(dev)
    with torch.no_grad():
        gt = r.render_batch_ray({'points_color': pts}, dec, rd, ro, dev, 'color')[0].float()
    col = torch.rand((n, 3), generator=g).to(dev)
    tr = torch.rand((n, 32), generator=g).to(dev)
    ms = MapStep(r, dec, points=pts, feat_lr=1e-3)
    out = {'case': args.case, 'rays': n, 'points': int(pts.xyz.shape[0]), 'precision': args.precision}

    def timeit(fn, iters):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / iters * 1e3

    if args.mode in ('eager', 'both'):
        out['eager_ms'] = round(timeit(lambda: ms(ro, rd, gt, col, tr), args.iters), 4)
    if args.mode in ('graph', 'both'):
        mg = MapGraph(ms, ro, rd, gt, col, tr)
        out['graph_ms'] = round(timeit(lambda: mg(*mg.inputs), args.iters), 4)
    assert r.status(dev) == 0
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
