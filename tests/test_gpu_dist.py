"""Data parallelism on the HIP path, driver-run: tools/dp_check.py (MapStep) and
tools/dp_track_check.py (TrackStep) under torchrun with 2 ranks, launched as fresh child processes
that make no GPU call before torchrun starts them.  On a 1-GPU box both ranks share cuda:0 over gloo
(RCCL needs one GPU per rank); the data-path code is the one RCCL runs on a node.

Asserted by the tools: every rank holds bit-identical weights / camera tensors after the steps,
a second 1-process run reproduces the first bit for bit (the weight-gradient sums have a fixed
order), and the 2-rank losses / weights equal the 1-process ones to float32 association (each rank
sums its half of the points before the all-reduce adds the halves)."""
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


@pytest.mark.parametrize('tool,tag', [('dp_check.py', 'DP_CHECK_OK'), ('dp_track_check.py', 'DP_TRACK_CHECK_OK')])
def test_two_rank_data_parallel(tool, tag, tmp_path):
    out = tmp_path / 'res.json'
    env = dict(os.environ, PNR_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes', '1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_free_port()), os.path.join(REPO, 'tools', tool),
           str(out)]
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=240)
    print(p.stdout[-4000:])
    print(p.stderr[-4000:])
    assert p.returncode == 0, p.stderr[-2000:]
    assert tag in p.stdout
    res = json.loads(out.read_text())
    assert res['world'] == 2
    assert res['ranks_bitwise_identical'] and res['one_process_rerun_bitwise_identical']
