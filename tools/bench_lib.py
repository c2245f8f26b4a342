"""Run bench.py against another libpnr.so build (A/B of experiment builds).

  python tools/bench_lib.py <lib.so> [bench.py args...]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)
lib = os.path.abspath(sys.argv[1])
sys.argv = ['bench.py'] + sys.argv[2:]
import pnr._lib  # noqa: E402
pnr._lib.load(lib)
import bench  # noqa: E402
bench.main()
