"""Dense-grid decoder query of the Mesher (Mesher.get_grid_uniform
+ Mesher.eval_points, src/utils/Mesher.py:281-347, 427-430) on one MI355X.

  python tools/mesh_eval_bench.py [--resolution R] [--precision P] [--iters K]

Grid: R^3 float32 points over the room0 bound padded by 0.05 (np.linspace per axis, meshgrid,
ravel, as get_grid_uniform), queried through pnr.Renderer.eval_points in 500,000-point chunks
(points_batch_size), as the Mesher does.  Parity: 4,096 random grid points against the oracle's
eval_points (CPU).  Prints one JSON line with the decoder FLOP rate (443,438 FLOP per point).
"""
import argparse
import json
import os
import sys
import time
import types

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)

from bench import load_scene, FLOP_PER_POINT_FWD  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--resolution', type=int, default=256)
    ap.add_argument('--precision', default=None)
    ap.add_argument('--iters', type=int, default=3)
    args = ap.parse_args()
    import pnr
    from oracle import ref_render as ref
    dev = torch.device('cuda:0')
    bound, pose, params = load_scene()
    slam = types.SimpleNamespace(bound=bound, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    cfg = dict(pnr.ROOM0_CFG)
    if args.precision:
        cfg['pnr'] = {'precision': args.precision}
    r = pnr.Renderer(cfg, None, slam)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    b = bound.numpy()
    pad, R = 0.05, args.resolution
    x, y, z = (np.linspace(b[a][0] - pad, b[a][1] + pad, R) for a in range(3))
    xx, yy, zz = np.meshgrid(x, y, z)
    grid = torch.tensor(np.vstack([xx.ravel(), yy.ravel(), zz.ravel()]).T, dtype=torch.float)
    gd = grid.to(dev)
    bs = 500000

    def query():
        return torch.cat([r.eval_points(pi, dec, None, 'color', dev) for pi in torch.split(gd, bs)], 0)

    out = query()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.iters):
        out = query()
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / args.iters
    n = grid.shape[0]
    sel = torch.randperm(n, generator=torch.Generator().manual_seed(0))[:4096]
    rr = ref.eval_points(params, grid[sel], bound)
    og = out[sel.to(dev)].cpu()
    err = float((og - rr).abs().max() / rr.abs().max())
    print(json.dumps({'metric': 'Mesher dense-grid decoder query points/sec', 'value': round(n / t, 1),
                      'unit': 'points/s', 'ms': round(t * 1e3, 3), 'points': n, 'resolution': R,
                      'tflops': round(n * FLOP_PER_POINT_FWD / t / 1e12, 1), 'precision': r.precision,
                      'parity': {'points': 4096, 'max_abs_err_over_max': float(f'{err:.3g}')}}))


if __name__ == '__main__':
    main()
