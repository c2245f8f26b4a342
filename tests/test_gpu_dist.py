"""Data parallelism on the HIP path, driver-run, as fresh child processes that
make no GPU call before torchrun starts them.

  * tools/dp_check.py at 2 ranks, three cases: room0 rays; config C4's own workload (the scene0000
    bound and a 5,000-pixel 10-frame window batch of the cropped ScanNet camera); the neural-point
    decoder with DataParallel(shard_points=True) (reduce-scatter of the feature gradient, Adam on the
    owned range, all-gather).  Asserted: the first step's reduced gradient is bitwise the sum of the
    per-shard 1-process gradients and agrees elementwise with the whole-batch gradient (rtol 1e-6 +
    the association bound); after the steps every rank holds bit-identical parameters and a second
    1-process run reproduces the first bit for bit.
  * tools/dp_track_check.py at 2 ranks: the Tracker's sharded pixel set and pose-gradient all-reduce.
On a 1-GPU box both ranks share cuda:0 over gloo (RCCL needs one GPU per rank).
  * tools/rccl_graph_check.py at 1 rank over RCCL (`nccl`): every collective of the step forced at
    world size 1 and captured in the step's HIP graph (pnr.MapGraph) -- replay equals eager bitwise.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _torchrun(tool, args, nproc, backend, timeout=300):
    env = dict(os.environ, PNR_DIST_BACKEND=backend, MASTER_ADDR='127.0.0.1', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes', '1', '--nproc-per-node', str(nproc),
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.join(REPO, 'tools', tool),
           *args]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=timeout)
    print(p.stdout[-4000:])
    print(p.stderr[-4000:])
    assert p.returncode == 0, p.stderr[-2000:]
    return p


@pytest.mark.parametrize('case', ['room0', 'scannet', 'points'])
def test_two_rank_map_step(case, tmp_path):
    out = tmp_path / 'res.json'
    p = _torchrun('dp_check.py', ['--case', case, '--out', str(out)], 2, 'gloo')
    assert 'DP_CHECK_OK' in p.stdout
    res = json.loads(out.read_text())
    assert res['world'] == 2 and res['case'] == case
    assert res['ranks_bitwise_identical'] and res['one_process_rerun_bitwise_identical']
    assert res['first_step_grad']['equals_sum_of_shard_grads_bitwise']
    assert res['first_step_grad']['worst_ratio_to_bound'] <= 1.0


def test_two_rank_track_step(tmp_path):
    out = tmp_path / 'res.json'
    p = _torchrun('dp_track_check.py', [str(out)], 2, 'gloo')
    assert 'DP_TRACK_CHECK_OK' in p.stdout
    res = json.loads(out.read_text())
    assert res['world'] == 2
    assert res['ranks_bitwise_identical'] and res['one_process_rerun_bitwise_identical']


@pytest.mark.parametrize('points', [False, True])
def test_rccl_collectives_captured_in_graph(points, tmp_path):
    out = tmp_path / 'res.json'
    p = _torchrun('rccl_graph_check.py', (['--points'] if points else []) + ['--out', str(out)], 1, 'nccl')
    assert 'RCCL_GRAPH_OK' in p.stdout
    res = json.loads(out.read_text())
    assert res['backend'] == 'nccl'
    assert res['graph_equals_eager_bitwise'] and res['eager_equals_plain_bitwise']
