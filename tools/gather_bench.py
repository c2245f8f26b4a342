"""Point-gather microbenchmark on a neural-point scene.

  python tools/gather_bench.py [--points M] [--rays N] [--radius R] [--reps K] [--mode idw|trilinear]

Scene: neural points on the trained room0 decoder's own rendered surface (640x480 frame at room0
pose 1000, ScanNet-style intrinsics), voxel-downsampled like Point-NeRF's point initialisation: at
most one point per voxel of edge `--voxel` (the first pixel landing in it), features N(0, 0.1).
The gather radius defaults to 2 voxels (~12 points inside it on a surface, k = 8 kept).
Samples: for N random pixels, 32 stratified depths in [0.01 d, 1.2 d] + 12 around the surface
(sigma 5 mm), as float64 points -- the sample distribution of one mapping iteration.

Prints per-launch device time of k_gather (hipEvents through pnr_timing_*), the neighbour
statistics and the algorithmic HBM bytes (SURVEY.md 8(d) with the 8 probes made: per sample 24 B point + 8 x 8 B bucket
headers + n_nb x (4 B idx + 12 B xyz + 128 B features) + 128 B c + k x 8 B idx/weight saves).
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0


from bench import gather_bytes, neural_point_scene  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--voxel', type=float, default=0.001)
    ap.add_argument('--rays', type=int, default=640 * 480)
    ap.add_argument('--radius', type=float, default=None, help='default: 2 voxels')
    ap.add_argument('--k', type=int, default=8)
    ap.add_argument('--mode', default='idw')
    ap.add_argument('--reps', type=int, default=5)
    ap.add_argument('--lib', default=None, help='load this libpnr.so build instead (experiments)')
    ap.add_argument('--feat-dtype', default='float32', choices=['float32', 'float16'])
    ap.add_argument('--dump', default=None, help='save the first launch\'s c / idx / w here (A/B bitwise checks)')
    args = ap.parse_args()
    import pnr
    if args.lib:
        pnr._lib.load(os.path.abspath(args.lib))
    from pnr._lib import timing_read
    dev = torch.device('cuda:0')
    lib = pnr.library()
    xyz, feats, p, _ = neural_point_scene(dev, args.voxel, args.rays)
    args.points = xyz.shape[0]
    if args.radius is None:
        args.radius = 2 * args.voxel
    pts = pnr.NeuralPoints(xyz, feats, mode=args.mode, radius=args.radius, k=args.k,
                           spacing=[args.radius] * 3, feat_dtype=args.feat_dtype).to(dev)
    P = p.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, args.k), device=dev, dtype=torch.int32)
    w = torch.empty((P, args.k), device=dev)
    s, _ = pts.descriptor()
    st = pnr._lib.stream_of(dev)
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)

    def run():
        pnr._lib.check(lib.pnr_point_gather(ctypes.byref(s), p.data_ptr(), P, c.data_ptr(), idx.data_ptr(),
                                            w.data_ptr(), ws.data_ptr(), ws.numel(), st), 'gather')

    c.fill_(float('nan'))  # every row must be written (zero-filled or gathered)
    idx.fill_(-7)
    w.fill_(float('nan'))
    run()
    torch.cuda.synchronize()
    if args.dump:
        torch.save({'c': c.cpu(), 'idx': idx.cpu(), 'w': w.cpu()}, args.dump)
    nb = int((idx >= 0).sum().item())
    n_work = int(ws[:64 * 32 * 4].view(torch.int32)[::32].sum().item())
    hist = torch.bincount((idx >= 0).sum(1), minlength=args.k + 1).tolist()
    lib.pnr_timing_enable(1)
    timing_read(4)
    for _ in range(args.reps):
        run()
    torch.cuda.synchronize()
    lib.pnr_timing_enable(0)
    launches, ms, _ = timing_read(4)
    if hasattr(lib, 'pnr_dbg_phase'):  # experiment build: per-phase s_memtime cycles of k_gather_search
        buf = (ctypes.c_ulonglong * 16)()
        lib.pnr_dbg_phase(buf)
        ph = [buf[i] for i in range(8)]
        tot = max(ph[5], 1)
        names = ['setup', 'scan', 'select', 'weights', 'features', 'total', 'rounds', 'trips']
        print('phases (wave-cycles, share of total):', ', '.join(f'{n} {ph[i]:.3e} ({ph[i] / tot:.2f})' for i, n in enumerate(names[:6])),
              f'rounds {ph[6]}, trips {ph[7]}, cycles/round {ph[5] / max(ph[6], 1):.0f}')
    avg = ms / launches
    byt = gather_bytes(P, n_work, nb, args.k)
    gbs = byt / (avg * 1e-3) / 1e9
    # backward (feature grads + position grads)
    gf = torch.zeros_like(feats)
    gc = torch.randn_like(c)
    gp = torch.empty((P, 3), device=dev)
    sb, _ = pts.descriptor(g_feats=gf)
    bws = torch.empty(lib.pnr_point_gather_bwd_workspace_bytes(ctypes.byref(sb), P), dtype=torch.uint8, device=dev)
    lib.pnr_timing_enable(1)
    timing_read(5)
    for _ in range(args.reps):
        pnr._lib.check(lib.pnr_point_gather_bwd(ctypes.byref(sb), p.data_ptr(), P, idx.data_ptr(), w.data_ptr(),
                                                c.data_ptr(), gc.data_ptr(), gp.data_ptr(), bws.data_ptr(), bws.numel(),
                                                st), 'gather_bwd')
    torch.cuda.synchronize()
    lib.pnr_timing_enable(0)
    bl, bms, _ = timing_read(5)
    bavg = bms / bl
    # feature grads only (the Mapper's case: no dL/dp)
    lib.pnr_timing_enable(1)
    timing_read(5)
    for _ in range(args.reps):
        pnr._lib.check(lib.pnr_point_gather_bwd(ctypes.byref(sb), p.data_ptr(), P, idx.data_ptr(), w.data_ptr(),
                                                c.data_ptr(), gc.data_ptr(), None, bws.data_ptr(), bws.numel(),
                                                st), 'gather_bwd')
    torch.cuda.synchronize()
    lib.pnr_timing_enable(0)
    fl, fms, _ = timing_read(5)
    n_at = ctypes.c_int64(0)
    pnr._lib.check(lib.pnr_point_gather_bwd_atomics(ctypes.byref(sb), bws.data_ptr(), P, ctypes.byref(n_at), st),
                   'gather_bwd_atomics')
    print(f'bwd int64 atomic instructions issued (256 B each): {n_at.value}')
    with torch.no_grad():  # neighbours shared with the previous row that has neighbours
        rows = idx[idx[:, 0] >= 0].long()
        prev, cur = rows[:-1], rows[1:]
        shared = ((cur[:, :, None] == prev[:, None, :]) & (cur[:, :, None] >= 0)).any(2).sum().item()
        print(f'bwd rows {rows.shape[0]}, neighbour slots {int((rows >= 0).sum().item())}, shared with the '
              f'previous row {shared}; feature-grad-only bwd {fms / fl:.3f} ms/launch')
    # bwd algorithmic bytes: 24 B point + 128 g_c + 128 c + k*8 idx/w + per neighbour (128 feats + 12 xyz
    # + 128 B feature-grad atomics) + 12 B g_p
    bbyt = P * (24 + 128 + 128 + args.k * 8 + 12) + nb * (128 + 12 + 128)
    # candidate statistics: points scanned per sample = points in its 8 probe cells (torch, untimed)
    with torch.no_grad():
        o = torch.tensor(pts.origin, device=dev, dtype=torch.float32)
        inv = 1.0 / pts.cell
        cq = torch.floor((xyz - o) * inv).long()
        off = 1 << 20
        ck = ((cq[:, 0] + off) << 42) | ((cq[:, 1] + off) << 21) | (cq[:, 2] + off)
        uk, cnt = torch.unique(ck, return_counts=True)
        t = (p.float() - o) * inv
        fl = torch.floor(t)
        b = fl.long() - (t - fl < 0.5).long()
        cand = torch.zeros(P, device=dev, dtype=torch.long)
        for n in range(8):
            k3 = ((b[:, 0] + (n & 1) + off) << 42) | ((b[:, 1] + ((n >> 1) & 1) + off) << 21) | (b[:, 2] + (n >> 2) + off)
            pos = torch.searchsorted(uk, k3).clamp(max=uk.numel() - 1)
            cand += torch.where(uk[pos] == k3, cnt[pos], torch.zeros_like(cnt[pos]))
        cw = cand[cand > 0]
        nw = cw.numel() // 64 * 64
        wmax = cw[:nw].view(-1, 64).max(1).values.float().mean().item() if nw else 0.0
        print(f'cells {uk.numel()} (points/cell {cnt.float().mean().item():.2f}); samples with candidates '
              f'{cw.numel()}: {cw.float().mean().item():.1f} candidates each, mean per-wave max {wmax:.1f}')
        # probe blocks per 64-item chunk of the block-grouped list (k_gather_search's segments)
        bk = ((b[:, 0] + off) << 42) | ((b[:, 1] + off) << 21) | (b[:, 2] + off)
        bk = torch.sort(bk[cand > 0]).values
        nc = bk.numel() // 64 * 64
        if nc:
            ch = bk[:nc].view(-1, 64)
            segs = 1 + (ch[:, 1:] != ch[:, :-1]).sum(1)
            _, bc = torch.unique(bk, return_counts=True)
            print(f'search segments: {segs.float().mean().item():.1f} probe blocks per 64-item chunk '
                  f'(max {int(segs.max().item())}); samples per block {bc.float().mean().item():.1f}')
    print(f'voxel {args.voxel} points {args.points} samples {P} ({args.rays} rays x 44) mode {args.mode} r {args.radius} k {args.k}')
    print(f'neighbours: mean {nb / P:.2f}/sample, histogram {hist}; samples with candidates {n_work} '
          f'({100 * n_work / P:.1f}%)')
    print(f'k_gather     {avg:.3f} ms/launch  {P / avg / 1e6:.1f} Msamples/ms... algorithmic {byt / 1e9:.2f} GB '
          f'-> {gbs:.0f} GB/s = {gbs / HBM_PEAK_GBS:.3f} of HBM peak')
    print(f'k_gather_bwd {bavg:.3f} ms/launch  algorithmic {bbyt / 1e9:.2f} GB -> {bbyt / (bavg * 1e-3) / 1e9:.0f} GB/s')


if __name__ == '__main__':
    main()
