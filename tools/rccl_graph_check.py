"""The RCCL collectives of a data-parallel MapStep, eager and captured in a HIP graph, on one GPU.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 \
        --master-port 29513 tools/rccl_graph_check.py [--points] [--out out.json]

RCCL refuses two ranks on one GPU, so a 1-GPU box cannot run the 2-rank data path over RCCL (the
driver's 8-GPU scaling run does).  What it can run is every RCCL call of the step at world size 1:
DataParallel(force_collectives=True) issues the far-clamp all_reduce(MAX) and the gradient
all_reduce(SUM) (with --points: the feature reduce_scatter and all_gather of shard_points=True) over
the `nccl` backend, and pnr.MapGraph captures them in the step's HIP graph -- the capture path a node
replays per mapping iteration (pnr/mapping.py MapGraph; graphs cannot hold gloo collectives).
Checked: the replayed steps equal the eager steps with the same collectives bit for bit (losses and
parameters), and equal the plain 1-process step (no collectives) bit for bit.
"""
import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pointnerf-slam_amd')]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', action='store_true')
    ap.add_argument('--out', default=None)
    args = ap.parse_args()
    sys.argv = sys.argv[:1]
    import dp_check  # the case builders (same directory)
    import pnr
    from pnr.dist import DataParallel
    from pnr.mapping import MapGraph, MapStep
    dev = torch.device('cuda', int(os.environ.get('LOCAL_RANK', 0)))
    torch.cuda.set_device(dev)
    dist.init_process_group(backend='nccl')
    assert dist.get_world_size() == 1 and dist.get_backend() == 'nccl'
    case = 'points' if args.points else 'room0'
    mk_r, mk_dec, mk_pts, (ro, rd, gt, col), n = dp_check.build_case(case, dev)
    n = 2048
    ro, rd, gt, col = ro[:n].contiguous(), rd[:n].contiguous(), gt[:n].contiguous(), col[:n].contiguous()
    g = torch.Generator().manual_seed(1)
    batches = [(ro, rd, gt, col, torch.rand((n, 32), generator=g).to(dev)) for _ in range(4)]
    runs = {}
    for mode in ('plain', 'eager', 'graph'):
        ddp = None if mode == 'plain' else DataParallel(shard_points=args.points, force_collectives=True)
        ms = MapStep(mk_r(), mk_dec(), lr=2e-4, w_color_loss=0.05, ddp=ddp, points=mk_pts() if mk_pts else None)
        ms.opt.use_device_step()
        losses = []
        if mode == 'graph':
            mg = MapGraph(ms, *batches[0], warmup=2)
            for b in batches[1:]:
                losses.append(float(mg(*b)))
        else:
            for _ in range(2):
                ms(*batches[0])
            for b in batches[1:]:
                losses.append(float(ms(*b)))
        torch.cuda.synchronize()
        runs[mode] = (losses, ms.flat.data.detach().cpu().clone())
    res = {'case': case, 'backend': dist.get_backend(), 'world': 1, 'collectives': 'forced at world size 1',
           'rays': n, 'losses': {k: v[0] for k, v in runs.items()},
           'graph_equals_eager_bitwise': runs['graph'][0] == runs['eager'][0] and torch.equal(runs['graph'][1],
                                                                                            runs['eager'][1]),
           'eager_equals_plain_bitwise': runs['eager'][0] == runs['plain'][0] and torch.equal(runs['eager'][1],
                                                                                            runs['plain'][1])}
    print(json.dumps(res), flush=True)
    if args.out:
        json.dump(res, open(args.out, 'w'), indent=1)
    assert res['graph_equals_eager_bitwise'] and res['eager_equals_plain_bitwise'], res
    print('RCCL_GRAPH_OK', flush=True)
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
