"""Data-parallel Tracker step on the HIP path vs the 1-process step (pixel batches
shard across GPUs, the pose gradient is all-reduced).

    python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 --master-addr 127.0.0.1 \
        --master-port 29512 tools/dp_track_check.py [out.json]

Every rank builds the same weak-depth frame (the trained room0 decoder's render at pose 1000,
340x600 camera) and runs pnr.TrackStep(ddp=DataParallel()) from the same perturbed camera for a few
Adam iterations: each renders its shard of the pixel set with the all-reduced far clamp, the camera
gradient and the loss are all-reduced.  Rank 0 then runs the 1-process TrackStep and compares.  On
a 1-GPU box both ranks share cuda:0 over gloo; on a node the same code runs over RCCL
(PNR_DIST_BACKEND=nccl)."""
import json
import os
import sys
import types

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, 'pointnerf-slam_amd')]


def run(pnr, ddp, dev, iters=3):
    import bench
    bound, pose, params = bench.load_scene()
    H, W, f, cx, cy = 340, 600, 300., 299.5, 169.5
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=f, fy=f, cx=cx, cy=cy)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    dec = bench.make_decoder(pnr, pnr.ROOM0_CFG, params, dev)
    with torch.no_grad():
        gd, _, gc = r.render_img({}, dec, pose.to(dev), dev, 'color')
    gd, gc = gd.float().contiguous(), gc.float().contiguous()
    step = pnr.TrackStep(r, dec, ignore_edge_W=50, ignore_edge_H=50, ddp=ddp)
    ct = pnr.get_tensor_from_camera(pose).to(dev) + torch.tensor([0.002, -0.001, 0.001, 0.001, 0.003, -0.002, 0.001],
                                                                  device=dev)
    ct.requires_grad_(True)
    opt = torch.optim.Adam([ct], lr=1e-3)
    losses = [step(ct, gc, gd, 0, opt) for _ in range(iters)]
    return losses, ct.detach().cpu().clone()


def main():
    import pnr
    from pnr import dist as pdist
    rank, world, local = pdist.init(backend=os.environ.get('PNR_DIST_BACKEND', 'gloo'))
    dev = torch.device('cuda', local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    ddp = pdist.DataParallel()
    l_dp, ct_dp = run(pnr, ddp, dev)
    cmax, cmin = ct_dp.clone().to(dev), ct_dp.clone().to(dev)
    torch.distributed.all_reduce(cmax, op=torch.distributed.ReduceOp.MAX)
    torch.distributed.all_reduce(cmin, op=torch.distributed.ReduceOp.MIN)
    ranks_identical = bool(torch.equal(cmax, cmin))  # the camera Adam runs on the all-reduced gradient
    if rank == 0:
        l1, ct1 = run(pnr, None, dev)
        l2, ct2 = run(pnr, None, dev)
        rerun_identical = l1 == l2 and torch.equal(ct1, ct2)
        rel = [abs(x - y) / abs(y) for x, y in zip(l_dp, l1)]
        res = {'world': world, 'backend': torch.distributed.get_backend(), 'iters': len(l1), 'loss_dp': l_dp,
               'loss_1proc': l1, 'loss_rel_diff': rel, 'camera_max_abs_diff': float((ct_dp - ct1).abs().max()),
               'precision': pnr._lib.DEFAULT_PRECISION, 'ranks_bitwise_identical': ranks_identical,
               'one_process_rerun_bitwise_identical': rerun_identical}
        print(json.dumps(res), flush=True)
        if len(sys.argv) > 1:
            json.dump(res, open(sys.argv[1], 'w'), indent=1)
        assert ranks_identical and rerun_identical, res
        assert rel[0] < 1e-6 and max(rel) < 1e-4, rel
        assert res['camera_max_abs_diff'] < 1e-5, res
        print('DP_TRACK_CHECK_OK', flush=True)
    ddp.barrier()
    torch.distributed.destroy_process_group()


if __name__ == '__main__':
    main()
