"""Data-parallel MapStep on the HIP path vs the 1-process step over the same global batch.

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29511 tools/dp_check.py [out.json]

Each rank takes its contiguous share of one global batch (pnr.dist.shard_bounds)
and runs pnr.mapping.MapStep(ddp=DataParallel()): the global far clamp is all-reduced (MAX) and
read on the device (far_mode 2), the flat gradient is all-reduced (SUM), Adam runs identically on
every rank.  Rank 0 then runs the plain 1-process MapStep on the whole batch and compares.  Launched
by torchrun before any GPU call; on a 1-GPU box both ranks share cuda:0 over gloo (RCCL needs one
GPU per rank), on a node the same code runs over RCCL (PNR_DIST_BACKEND=nccl).
"""
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pointnerf-slam_amd')]


def main():
    import bench
    import pnr
    from pnr import dist as pdist
    from pnr.mapping import MapStep
    rank, world, local = pdist.init(backend=os.environ.get('PNR_DIST_BACKEND', 'gloo'))
    dev = torch.device('cuda', local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    bound, pose, params = bench.load_scene()
    import types
    slam = types.SimpleNamespace(bound=bound, H=bench.H, W=bench.W, fx=bench.FX, fy=bench.FY, cx=bench.CX,
                                 cy=bench.CY)
    n, steps = 8192, 3
    ro, rd, gt, col = bench.synth_batch(n, 0, pose, dev)  # the global batch (seed 0), every rank
    g = torch.Generator().manual_seed(1)
    t_rands = [torch.rand((n, 32), generator=g).to(dev) for _ in range(steps)]
    a, b = pdist.shard_bounds(n, rank, world)
    ddp = pdist.DataParallel()
    dec = bench.make_decoder(pnr, pnr.ROOM0_CFG, params, dev)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    ms = MapStep(r, dec, lr=2e-4, w_color_loss=0.05, ddp=ddp)
    local_losses = [float(ms(ro[a:b], rd[a:b], gt[a:b], col[a:b], t[a:b])) for t in t_rands]
    lt = torch.tensor(local_losses, device=dev, dtype=torch.float64)
    torch.distributed.all_reduce(lt)  # the global loss = sum of the shards' losses (sums, A14)
    w_dp = ms.flat.data.detach().cpu().clone()
    # every rank holds the same weights, bit for bit (Adam on identical all-reduced gradients)
    wmax, wmin = ms.flat.data.detach().clone(), ms.flat.data.detach().clone()
    torch.distributed.all_reduce(wmax, op=torch.distributed.ReduceOp.MAX)
    torch.distributed.all_reduce(wmin, op=torch.distributed.ReduceOp.MIN)
    ranks_identical = bool(torch.equal(wmax, wmin))
    if rank == 0:
        dec1 = bench.make_decoder(pnr, pnr.ROOM0_CFG, params, dev)
        ms1 = MapStep(pnr.Renderer(pnr.ROOM0_CFG, None, slam), dec1, lr=2e-4, w_color_loss=0.05)
        full = [float(ms1(ro, rd, gt, col, t)) for t in t_rands]
        w1 = ms1.flat.data.detach().cpu().clone()
        # the 1-process step is deterministic: a second run gives identical bits
        dec2 = bench.make_decoder(pnr, pnr.ROOM0_CFG, params, dev)
        ms2 = MapStep(pnr.Renderer(pnr.ROOM0_CFG, None, slam), dec2, lr=2e-4, w_color_loss=0.05)
        full2 = [float(ms2(ro, rd, gt, col, t)) for t in t_rands]
        rerun_identical = full2 == full and torch.equal(ms2.flat.data.detach().cpu(), w1)
        dw = (w_dp - w1).abs()
        loss_rel = [abs(x - y) / abs(y) for x, y in zip(lt.tolist(), full)]
        res = {'world': world, 'backend': torch.distributed.get_backend(), 'global_batch': n,
               'rays_per_rank': [list(pdist.shard_bounds(n, k, world)) for k in range(world)], 'steps': steps,
               'loss_dp': lt.tolist(), 'loss_1proc': full, 'loss_rel_diff': loss_rel,
               'weights_max_abs_diff': float(dw.max()),
               'weights_frac_beyond_1e-5_rel': float((dw > 1e-7 + 1e-5 * w1.abs()).float().mean()),
               'far_clamp': 'device (far_mode 2), all_reduce MAX', 'precision': pnr._lib.DEFAULT_PRECISION,
               'ranks_bitwise_identical': ranks_identical, 'one_process_rerun_bitwise_identical': rerun_identical}
        print(json.dumps(res), flush=True)
        if len(sys.argv) > 1:
            json.dump(res, open(sys.argv[1], 'w'), indent=1)
        assert ranks_identical and rerun_identical, res
        # step 1 starts from the same weights: the losses agree to summation order (each rank sums
        # its own half of the points, then the all-reduce adds the halves: a different association
        # of the same float32 terms than the 1-process sum); Adam then moves near-zero-gradient
        # elements by up to lr per step
        assert loss_rel[0] < 1e-6, loss_rel
        assert max(loss_rel) < 1e-4, loss_rel
        assert float(dw.max()) <= steps * 2 * 2e-4 and res['weights_frac_beyond_1e-5_rel'] < 0.01, res
        print('DP_CHECK_OK', flush=True)
    ddp.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
