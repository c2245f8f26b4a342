"""bench.py's --gpus N contract on the CPU (no GPU calls): N > 1 outside a launcher starts N ranks
through torch.distributed.run as a child process, a node with fewer GPUs fails loudly, and a rank
whose launcher started a different world size than --gpus refuses to run (it would otherwise print an
`n_gpus` that is not what was asked for)."""
import json
import os
import subprocess
import sys
import types

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), *args], env=env, capture_output=True,
                          text=True, timeout=300)


def test_gpus_more_than_present_fails():
    # more GPUs than any node has: fails before launching ranks, whatever machine runs the test
    r = _run(['--gpus', '4096'])
    assert r.returncode != 0
    assert 'needs 4096 GPUs' in r.stderr
    assert '"n_gpus"' not in r.stdout


def test_world_mismatch_fails():
    r = _run(['--gpus', '4'], {'WORLD_SIZE': '2', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert r.returncode == 2
    assert 'launcher started 2 rank(s)' in r.stderr


def test_launcher_command(monkeypatch):
    import bench
    seen = {}
    monkeypatch.setattr(bench.torch.cuda, 'device_count', lambda: 8)

    def fake_run(cmd, env=None):
        seen['cmd'], seen['env'] = cmd, env
        return types.SimpleNamespace(returncode=7)
    monkeypatch.setattr(subprocess, 'run', fake_run)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '4', '--steps', '3'])
    args = types.SimpleNamespace(gpus=4)
    assert bench.launch_ranks(args) == 7
    cmd = seen['cmd']
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node=4' in cmd and '--nnodes=1' in cmd
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-4:] == ['--gpus', '4', '--steps', '3'] and cmd[-5].endswith('bench.py')
    assert seen['env']['PNR_DIST_BACKEND'] == 'nccl'


def test_main_launches_when_no_world(monkeypatch):
    import bench
    monkeypatch.delenv('WORLD_SIZE', raising=False)
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2'])
    monkeypatch.setattr(bench, 'launch_ranks', lambda a: 0 if a.gpus == 2 else 1)
    with pytest.raises(SystemExit) as e:
        bench.main()
    assert e.value.code == 0


def test_rank0_line_at_n2_carries_the_scaling_keys(monkeypatch, capsys):
    """Rank 0's line of a 2-rank run (every GPU workload stubbed: no GPU, no process group) carries the
    keys the driver's 1/2/4/8 curve reads -- the headline, `smap`, `fixed_global_batch`, the north
    star's S-fwd batch in its weak and fixed-global forms, the gather line and `distributed` -- with the
    same key names as the N = 1 line."""
    import bench
    from pnr import dist as pdist
    import pnr
    calls = []
    monkeypatch.setenv('WORLD_SIZE', '2')
    monkeypatch.setenv('RANK', '0')
    monkeypatch.setenv('LOCAL_RANK', '0')
    monkeypatch.setattr(sys, 'argv', ['bench.py', '--gpus', '2', '--steps', '3', '--warmup', '1'])
    monkeypatch.setattr(bench.torch.cuda, 'device_count', lambda: 2)
    monkeypatch.setattr(bench.torch.cuda, 'set_device', lambda d: None)
    monkeypatch.setattr(pdist, 'init', lambda backend=None: (0, 2, 0))

    class DP:
        world = 2

        def barrier(self):
            calls.append('barrier')
    monkeypatch.setattr(pdist, 'DataParallel', DP)
    import torch.distributed as tdist
    monkeypatch.setattr(tdist, 'get_backend', lambda *a: 'nccl')
    monkeypatch.setattr(tdist, 'get_world_size', lambda *a: 2)
    monkeypatch.setattr(tdist, 'destroy_process_group', lambda *a: calls.append('destroy'))
    monkeypatch.setattr(pnr, 'library', lambda: None)
    monkeypatch.setattr(bench, 'load_scene', lambda: (None, None, {'w': 0}))
    monkeypatch.setattr(bench, 'room0_extra', lambda *a, **k: {
        'rays_per_s': 1.0e6, 'ms_per_iter': 1.0, 'workload': 'room0', 'rays_per_iter': 1000,
        'roofline': {'frac': 0.3}, 'cpu_baseline': None})
    monkeypatch.setattr(bench, 'smap_run', lambda *a, **k: {'value': 5.0e6, 'n_gpus': a[-2] if len(a) > 11 else 2})
    monkeypatch.setattr(bench, 'fixed_global_run', lambda *a, **k: {'value': 4.0e6, 'scaling': 'strong'})

    def sfwd(*a, **k):
        calls.append(('sfwd', k.get('world'), k.get('fixed_global', False)))
        return {'value': 2.0e7, 'n_gpus': k.get('world'), 'scaling': 'strong' if k.get('fixed_global') else 'weak'}
    monkeypatch.setattr(bench, 'sfwd_extra', sfwd)
    monkeypatch.setattr(bench, 'gather_roofline', lambda dev, feat_dtype='float32': {'frac': 0.5})
    bench.main()
    out = json.loads(capsys.readouterr().out.strip().splitlines()[-1])
    assert out['n_gpus'] == 2 and out['value'] == 2.0e6
    assert out['distributed']['world_size'] == 2
    for key in ('smap', 'smap_value', 'fixed_global_batch', 'sfwd', 'sfwd_fixed_global', 'gather_roofline'):
        assert key in out, key
    assert out['sfwd']['scaling'] == 'weak' and out['sfwd_fixed_global']['scaling'] == 'strong'
    assert ('sfwd', 2, False) in calls and ('sfwd', 2, True) in calls
    assert calls[-2:] == ['barrier', 'destroy']
