"""bench.py's --gpus N contract on the CPU (no GPU calls): N > 1 outside a launcher starts N ranks
through torch.distributed.run as a child process, a node with fewer GPUs fails loudly, and a rank
whose launcher started a different world size than --gpus refuses to run (it would otherwise print an
`n_gpus` that is not what was asked for)."""
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
    r = _run(['--gpus', '2'])
    assert r.returncode != 0
    assert 'needs 2 GPUs' in r.stderr
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
