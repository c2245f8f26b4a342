"""Data parallelism over one node: pixel batches shard across GPUs.

One process per GPU (torch.distributed, backend 'nccl' = RCCL over xGMI on ROCm; 'gloo' on CPU
for tests).  Each rank renders its own rays with a replicated decoder; per mapping iteration
there are exactly two collectives:
  * all_reduce(MAX) of one scalar: the batch-global far clamp max(1.2*gt) of
    src/utils/Renderer.py:112 (a cross-ray coupling), so sharded results equal 1-GPU results;
  * all_reduce(SUM) of the one flat fp32 gradient buffer (222,747 words = 891 KB), latency-bound
    on xGMI, issued once per step; Adam then runs identically on every rank.
With neural points and `DataParallel(shard_points=True)` the point-feature tail of that buffer
is reduce-scattered instead, Adam updates each rank's owned feature range, and the features are
all-gathered (reduce_scatter_ / all_gather_).
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
    """`force_collectives` issues the collectives even at world size 1 (a 1-GPU box has one rank per
    GPU at most under RCCL: this is how the RCCL calls of a step, and their graph capture, run there)."""

    def __init__(self, group=None, shard_points=False, force_collectives=False):
        self.group = group
        self.shard_points = bool(shard_points)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.active = dist.is_initialized() and (self.world > 1 or force_collectives)
        # gloo has no CUDA reduce-scatter / all-gather: those two stage through host copies (the gloo
        # path is a CPU-test / 1-GPU rehearsal of the RCCL one)
        self.stage = dist.is_initialized() and dist.get_backend(group) == 'gloo'
        self._bufs = {}  # padded send / receive buffers of the sharded feature update, reused per step

    def _buf(self, name, n, like):
        """A cached device buffer of n words (allocated once per shape / dtype / device)."""
        key = (name, n, like.dtype, like.device)
        b = self._bufs.get(key)
        if b is None:
            b = torch.zeros(n, dtype=like.dtype, device=like.device)
            self._bufs[key] = b
        return b

    def global_far_clamp(self, gt_depth_local, local_far=None):
        """max(1.2 * gt) over every rank's rays (Renderer.py:112), as a one-element float32 device
        tensor: the renderer reads it on the device (far_mode 2), so the step has no host sync and
        can be captured in a graph.  local_far: this rank's value if already on the device."""
        if local_far is not None:
            m = local_far.reshape(-1)[:1].float().clone()
        else:
            g = gt_depth_local.reshape(-1).float()
            if g.numel():
                m = (g * 1.2).amax().reshape(1)
            else:
                m = torch.full((1,), float('-inf'), device=g.device)
        if self.active:
            dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        return m

    def allreduce_(self, flat_grad):
        if self.active:
            dist.all_reduce(flat_grad, op=dist.ReduceOp.SUM, group=self.group)
        return flat_grad

    # -- sharded point-feature update (the 1M-point C5 budget) --------------------
    # The point features are the bulk of the gradient (1M x 32 fp32 = 128 MB) and each rank only
    # needs the update of its own slice: reduce-scatter the feature gradient into owned ranges,
    # run Adam on the owned range, all-gather the updated features.  The bytes on the wire equal
    # one all-reduce; the Adam work is divided by the world size.
    def feature_shard(self, n):
        """This rank's owned range [a, b) of an n-word segment (equal padded shards)."""
        per = -(-n // self.world) if n > 0 else 0
        rank = dist.get_rank(self.group) if self.world > 1 else 0
        a = min(n, rank * per)
        return a, min(n, a + per), per

    def reduce_scatter_(self, seg):
        """Sum `seg` (1-D) over ranks into this rank's owned range of `seg` (other words are left
        as they were).  Returns (a, b)."""
        n = seg.numel()
        a, b, per = self.feature_shard(n)
        if not self.active:
            return a, b
        staged = self.stage and seg.is_cuda
        ref = seg.cpu() if staged else seg
        buf = ref
        if per * self.world != n or staged:  # the padded tail stays zero: only [:n] is ever written
            buf = self._buf('rs_in', per * self.world, ref)
            buf[:n].copy_(ref)
        out = self._buf('rs_out', per, ref)
        dist.reduce_scatter_tensor(out, buf, op=dist.ReduceOp.SUM, group=self.group)
        seg[a:b].copy_(out[:b - a])
        return a, b

    def all_gather_(self, seg):
        """Every rank's owned range of `seg` (1-D) to every rank."""
        n = seg.numel()
        a, b, per = self.feature_shard(n)
        if not self.active:
            return seg
        ref = seg.new_empty(0, device='cpu') if (self.stage and seg.is_cuda) else seg
        mine = self._buf('ag_in', per, ref)  # words past b - a stay zero (the last rank's padding)
        mine[:b - a].copy_(seg[a:b])
        out = self._buf('ag_out', per * self.world, ref)
        dist.all_gather_into_tensor(out, mine, group=self.group)
        seg.copy_(out[:n])
        return seg

    def barrier(self):
        if self.active:
            dist.barrier(group=self.group)
