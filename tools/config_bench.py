"""Throughput records of BASELINE.json configs C3 and C5 on one MI355X (the scenes of
tests/test_gpu_configs.py, which holds their parity against the oracle).

  C3  office3 scaled bound, 200k neural points (IDW r = 1 cm, k = 8), Replica 680x1200 camera, bf16 and
      f16x3 decoders: the Mapper iteration at mapping.pixels = 1,000 (eager MapStep and replayed from a
      captured HIP graph, pnr.mapping.MapGraph) and at a 307,200-ray batch
  C5  Apartment scaled bound, 1M points with float16 features, 720x1280 camera: the Mapper
      iteration at mapping.pixels = 5,000 (eager and graph-replayed) and at 307,200 rays

  python tools/config_bench.py [--iters N] > profiles/<tag>_configs.json"""
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


def map_rate(pnr, slam, dec, pts, bound, cam, n, precision, iters, seed, graph=False):
    from pnr.mapping import MapStep
    H, W, fx, fy, cx, cy = cam
    dev = torch.device('cuda:0')
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr.Renderer(cfg, None, slam)
    g = torch.Generator().manual_seed(seed)
    pix = torch.randint(0, H * W, (n,), generator=g)
    ro, rd = RR.rays_from_uv((pix % W).float(), (pix // W).float(), TC.centre_pose(bound), fx, fy, cx, cy)
    ro, rd = ro.reshape(-1, 3).to(dev), rd.reshape(-1, 3).to(dev)
    with torch.no_grad():
        gt = r.render_batch_ray({'points_color': pts}, dec, rd, ro, dev, 'color')[0].float()
    ms = MapStep(r, dec, points=pts, feat_lr=1e-3)
    col = torch.rand((n, 3), generator=g).to(dev)
    tr = torch.rand((n, 32), generator=g).to(dev)
    for _ in range(2):
        ms(ro, rd, gt, col, tr)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        ms(ro, rd, gt, col, tr)
    torch.cuda.synchronize()
    el = (time.perf_counter() - t0) / iters
    assert r.status(dev) == 0
    out = {'rays': n, 'ms_per_iter': round(el * 1e3, 3), 'rays_per_s': round(n / el, 1), 'precision': precision,
           'iters': iters}
    if graph:  # the same step captured once (gather, fc_c injection, deterministic feature backward, Adam)
        from pnr.mapping import MapGraph
        mg = MapGraph(ms, ro, rd, gt, col, tr)
        gi = max(iters, 20)
        for _ in range(3):
            mg(*mg.inputs)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(gi):
            mg(*mg.inputs)
        torch.cuda.synchronize()
        eg = (time.perf_counter() - t0) / gi
        assert r.status(dev) == 0
        out['graph'] = {'ms_per_iter': round(eg * 1e3, 3), 'rays_per_s': round(n / eg, 1), 'iters': gi}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--iters', type=int, default=5)
    args = ap.parse_args()
    import pnr
    pnr.library()
    dev = torch.device('cuda:0')
    out = {'what': 'MapStep (render + regulation + L1 losses + backward + decoder and point-feature Adam) with '
                   'the neural-point decoder (c_dim 32, fc_c injection), synthetic room scenes of '
                   'tests/test_gpu_configs.py; eager launches, mean of --iters after 2 warm-ups; `graph`: the '
                   'same step replayed from a captured HIP graph (MapGraph), mean of max(--iters, 20)'}
    cam3 = (680, 1200, 600., 600., 599.5, 339.5)
    bound, xyz, feats, params, _, _, slam, pts = TC.scene_case(pnr, dev, TC.OFFICE3, *cam3, 200_000, 8, 0.01, seed=31)
    out['C3'] = {'points': int(pts.xyz.shape[0]), 'bound': bound.tolist(), 'runs': []}
    for prec in ('bf16', 'f16x3'):
        dec = TC.make_decoder(pnr, params, dev, prec)
        for n in (1000, 307200):
            out['C3']['runs'].append(map_rate(pnr, slam, dec, pts, bound, cam3, n, prec, args.iters, 3,
                                              graph=n <= 5000))
            print(json.dumps(out['C3']['runs'][-1]), file=sys.stderr, flush=True)
    del pts
    cam5 = (720, 1280, 607.4694, 607.4535, 636.9967, 369.2690)
    bound, xyz, feats, params, _, _, slam, pts = TC.scene_case(pnr, dev, TC.APARTMENT, *cam5, 1_000_000, 8, 0.008,
                                                               seed=41, feat_dtype='float16')
    out['C5'] = {'points': int(pts.xyz.shape[0]), 'point_features': 'float16', 'bound': bound.tolist(), 'runs': []}
    dec = TC.make_decoder(pnr, params, dev, 'f16x3')
    for n in (5000, 307200):
        out['C5']['runs'].append(map_rate(pnr, slam, dec, pts, bound, cam5, n, 'f16x3', args.iters, 5,
                                          graph=n <= 5000))
        print(json.dumps(out['C5']['runs'][-1]), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
