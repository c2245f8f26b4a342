"""Kernel microbenchmarks for the MLP kernels (device time via pnr_timing_* hipEvents).

  python tools/kbench.py [--points P] [--reps R]

Prints one line per case: launches, mean ms, achieved TFLOP/s (443,438 FLOP/point fwd,
442,880 FLOP/point delta chain) and the fraction of the 157.3 TF fp32 MFMA peak."""
import argparse
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=4 * 1024 * 1024)
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--precision', default='fp32,bf16x3,bf16')
    ap.add_argument('--lib', default=None, help='load this libpnr.so build instead (experiments)')
    ap.add_argument('--eval-only', action='store_true')
    args = ap.parse_args()
    import pnr
    if args.lib:
        pnr._lib.load(os.path.abspath(args.lib))
    from pnr._lib import timing_read
    dev = torch.device('cuda:0')
    lib = pnr.library()
    w = np.load(os.path.join(REPO, 'tests', 'golden', 'weights.npz'))
    params = {k[len('trained/'):]: torch.from_numpy(w[k]) for k in w.files if k.startswith('trained/')}
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    import types
    s = np.load(os.path.join(REPO, 'tests', 'golden', 'scene.npz'))
    slam = types.SimpleNamespace(bound=torch.from_numpy(s['bound']), H=480, W=640, fx=577.59, fy=578.73, cx=318.91,
                                 cy=242.68)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    P = args.points
    pts = (torch.rand(P, 3, device=dev, dtype=torch.float64) * 1.2 - 0.35)

    def report(name, kind, fl):
        n, ms, u = timing_read(kind)
        tf = fl * u / (ms * 1e-3) / 1e12 if ms > 0 else 0
        print(f'{name:34s} launches={n:3d} mean_ms={ms / max(n, 1):9.3f} TF/s={tf:7.2f} frac={tf / 157.3:.3f}',
              flush=True)

    ref = None
    for prec in args.precision.split(','):
        r.precision = prec
        dec.precision = prec
        # forward, inference (no save)
        out = r.eval_points(pts, dec)
        torch.cuda.synchronize()
        if ref is None:
            ref = out.clone()
        err = ((out - ref).abs() / (ref.abs() + 1e-3)).max().item()
        rel = ((out - ref).abs().max() / ref.abs().max()).item()
        print(f'[{prec}] eval vs first precision: max rel err {err:.3e}, max abs/max {rel:.3e}', flush=True)
        lib.pnr_timing_enable(1)
        timing_read(0)
        for _ in range(args.reps):
            r.eval_points(pts, dec)
        torch.cuda.synchronize()
        report(f'[{prec}] k_mlp_fwd eval (f64 pts)', 0, 443438)
        if hasattr(lib, 'pnr_dbg_read'):  # experiment build: s_memtime timeline of one workgroup
            import ctypes
            buf = (ctypes.c_ulonglong * (4 * 48))()
            lib.pnr_dbg_read(buf)
            for w in range(4):
                t = [buf[w * 48 + i] for i in range(48)]
                d = [t[i + 1] - t[i] for i in range(0, 39)] + [t[40] - t[36]]
                print(f'wave {w}: start->prologue {d[0]}, steps:', ' '.join(str(x) for x in d[1:]), flush=True)
        if args.eval_only:
            lib.pnr_timing_enable(0)
            continue
        # forward with save + backward (MLP autograd path)
        x = pts.float().requires_grad_(False)
        timing_read(0), timing_read(1), timing_read(3), timing_read(6)
        for _ in range(args.reps):
            out = dec(x)
            out.sum().backward()
        torch.cuda.synchronize()
        report(f'[{prec}] k_mlp_fwd train (save)', 0, 443438)
        report(f'[{prec}] k_mlp_bwd delta chain', 1, 442880)
        n, ms, u = timing_read(3)  # dWo / dB (or the fp32 GEMMs) ...
        n6, ms6, _ = timing_read(6)  # ... and the grouped split GEMMs (pnr_timing_read kind 6)
        n, ms = n + n6, ms + ms6
        print(f'[{prec}] k_wgrad* (all shapes)            launches={n:3d} ms/backward={ms / args.reps:9.3f}', flush=True)
        lib.pnr_timing_enable(0)


if __name__ == '__main__':
    main()
