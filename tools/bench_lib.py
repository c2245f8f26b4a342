"""Run bench.py (or another benchmark script) against another libpnr.so build (A/B of builds).

  python tools/bench_lib.py <lib.so> [--script tools/track_bench.py] [script args...]"""
import os
import runpy
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)
lib = os.path.abspath(sys.argv[1])
rest = sys.argv[2:]
script = os.path.join(REPO, 'bench.py')
if rest[:1] == ['--script']:
    script, rest = os.path.abspath(rest[1]), rest[2:]
sys.argv = [script] + rest
import pnr._lib  # noqa: E402
pnr._lib.load(lib)
runpy.run_path(script, run_name='__main__')
