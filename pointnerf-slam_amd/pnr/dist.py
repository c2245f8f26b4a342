"""Data parallelism over one node: pixel batches shard across GPUs.

One process per GPU (torch.distributed, backend 'nccl' = RCCL over xGMI on ROCm; 'gloo' on CPU
for tests).  Each rank renders its own rays with a replicated decoder; per mapping iteration
there are exactly two collectives:
  * all_reduce(MAX) of one scalar: the batch-global far clamp max(1.2*gt) of
    src/utils/Renderer.py:112 (a cross-ray coupling), so sharded results equal 1-GPU results;
  * all_reduce(SUM) of the one flat fp32 gradient buffer (222,747 words = 891 KB), latency-bound
    on xGMI, issued once per step; Adam then runs identically on every rank.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def env_rank_world():
    return int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)), int(os.environ.get('LOCAL_RANK', 0))


def init(backend=None):
    """Initialise the process group from torchrun's env (no-op for world size 1)."""
    rank, world, local = env_rank_world()
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = os.environ.get('PNR_DIST_BACKEND') or ('nccl' if torch.cuda.is_available() else 'gloo')
        if torch.cuda.is_available():
            torch.cuda.set_device(local % torch.cuda.device_count())
        dist.init_process_group(backend=backend)
    return rank, world, local


def shard_bounds(n, rank, world):
    """Contiguous slice [a, b) of n items for `rank` (sizes differ by at most one)."""
    base, rem = divmod(n, world)
    a = rank * base + min(rank, rem)
    return a, a + base + (1 if rank < rem else 0)


class DataParallel:
    def __init__(self, group=None):
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1

    def global_far_clamp(self, gt_depth_local):
        m = (gt_depth_local.reshape(-1).float() * 1.2).max() if gt_depth_local.numel() else \
            torch.tensor(float('-inf'), device=gt_depth_local.device)
        m = m.reshape(1).clone()
        if self.world > 1:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        return float(m.item())

    def allreduce_(self, flat_grad):
        if self.world > 1:
            dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)
        return flat_grad

    def barrier(self):
        if self.world > 1:
            dist.barrier(group=self.group)
