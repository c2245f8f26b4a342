#!/usr/bin/env python3
"""Benchmark: rendered rays/s per mapping iteration (BASELINE.json metric) on MI355X.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload room0|map|fwd|map-points] [--rays R]
                  [--global-batch B] [--precision P] [--graph] [--no-extras] [--no-cpu-baseline]

Workload `room0` (default; the metric's own iteration, configs/Replica/replica.yaml:21-22 +
configs/pointNeRF_slam.yaml): ONE room0 Mapper iteration of src/Mapper.py:507-662 at its real size --
1,000 rays over the 5-frame keyframe window of the 680x1200 room0 camera, window sampling on the
device, render (32 stratified + 12 importance samples, gt-depth near/far) + regulation (32 jittered
samples) + L1 depth + 0.05 L1 colour + 0.0005 |sigma| + backward + Adam lr 2e-4 -- replayed from one
captured HIP graph; `value` = rays/s over all ranks, `ms_per_step` = ms per iteration.
Workload `map` ("S-map"): the same iteration over R rays per GPU (default 307,200 = one
640x480 pixel batch).  Workload `fwd` ("S-fwd"): render_batch_ray forward, 640x480 rays x 64 stratified
samples.  Decoder arithmetic: f16x3 by default -- fp32-class end to end (every forward and backward GEMM
on 22-bit split operands with fp32 accumulation, include/pnr.h); `--precision fp32` runs fp32 MFMA.

Extra keys of the default line (measured after the timed region, never part of `value`):
  smap            S-map at 307,200 rays per GPU with its MLP rooflines and the oracle's CPU rate
                  (`smap_value` repeats its rays/s at the top level)
  sfwd            the north-star S-fwd batch (640x480 x 64 samples, forward) with its own roofline
                  and the oracle's CPU rate at 64 samples
  faithful_n1000  the Mapper iteration on synthetic rays at N = 1,000 and 5,000 (C4/C5), graph replay
  map_points      the neural-point Mapper iteration (A15) at 307,200 rays with its MLP roofline and
                  the oracle's CPU rate
  fp32            the S-map step with fp32-MFMA decoder arithmetic
  gather_roofline the neural-point gather (A15) on its HBM roofline
  room0_iter_fp32 the headline's room0 iteration (graph replay) in strict fp32 MFMA (config C2's precision)
N>1 lines (one rank per GPU, RCCL) carry `smap` (weak: 307,200 rays per GPU), `fixed_global_batch`
(ONE 307,200-ray batch split over the ranks: strong scaling), `sfwd` (weak: 640x480 x 64
samples per GPU) and `sfwd_fixed_global` (one 640x480 batch split over the ranks), rank 0's
`gather_roofline`, and `distributed` (the backend and world size the ranks saw).

Data: synthetic.  Decoder = the trained room0 weights committed as a golden fixture
(tests/golden/weights.npz, from the reference's own checkpoint) -- random init if absent.  room0: renders
of that decoder at four room0 poses + a moved current pose as the window frames (gt = rendered depth /
colour).  S-map: rays from room0 pose gt_c2w_list[1000] through ScanNet-style 640x480 intrinsics; gt
depth U[0.05,0.6] with 10% zeros; gt colour U[0,1]; seed 0 + rank.

Multi-GPU: `python bench.py --gpus N` starts N ranks itself (torch.distributed.run as a child
process, before any GPU call) unless it already runs under a launcher (WORLD_SIZE set, which must equal
N); fewer than N GPUs is an error.  Every rank maps its own batch (weak scaling); per iteration one scalar
all_reduce(MAX) (global far clamp, read on the device) and one 891 KB gradient all_reduce(SUM), captured
in the graph.  Rank 0 prints ONE JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
sys.path.insert(0, REPO)

METRIC = 'rendered rays/sec per mapping iter (Replica room0); PSNR Δ vs ref ≤0.1 dB'
FP32_MFMA_PEAK_TF = 157.3          # MI355X_MICROARCH.md: f32 MFMA dense = f32 vector peak
F16_MFMA_PEAK_TF = 2500.0          # MI355X_MICROARCH.md: f16/bf16 MFMA dense (~2.5 PF, no sparsity)
# Peak of the ALGORITHMIC (fp32-equivalent) FLOP rate per decoder precision: a split form runs
# 3 f16/bf16 MFMA products per fp32 product (include/pnr.h PNR_PREC_*)
ALGO_PEAK_TF = {'fp32': FP32_MFMA_PEAK_TF, 'f16x3': F16_MFMA_PEAK_TF / 3, 'bf16x3': F16_MFMA_PEAK_TF / 3,
                'bf16': F16_MFMA_PEAK_TF}
HBM_PEAK_GBS = 8000.0
FLOP_PER_POINT_FWD = 443438        # 2 x (279 + 23,808 + 3 x 65,536 + 1,024) MAC
FLOP_PER_POINT_BWD = 442880        # delta chain: 2 x (1,024 + 3 x 65,536 + 23,808) MAC
# the grouped weight-gradient launch (k_wgrad16_group, with the skinny dWo / dB jobs): algorithmic fp32
# operand bytes per training point (profiles/r06_traffic.json: W3 h3 1,024 + g_out 16 + h4 mask words 32;
# W2, W1 delta 1,024 + h 1,024 each; W0 delta1 1,024 + x 16; dWo h4 1,024 + g_out 16; dB g_arg 384 + x 16)
# and with the feature branch + the four fc_c GEMMs (dL/dh_l 1,024 + c 128 for l < 3; dWc_3 rebuilds its
# A from g_out: 16 + 128).  Its FLOP per point over those bytes (58.5; 45.5 with fc_c) is below the
# machine balance (833 TF / 8 TB/s = 104 FLOP/B): the launch sits on the HBM side of the roofline
WGRAD_B_PER_POINT = 7580
WGRAD_FC_B_PER_POINT = 3 * (1024 + 128) + (16 + 128)
WGRAD_FLOP_PER_POINT = 443430
WGRAD_FC_FLOP_PER_POINT = 4 * 2 * 256 * 32
W, H = 640, 480
FX, FY, CX, CY = 577.59, 578.73, 318.91, 242.68   # configs/ScanNet/scannet.yaml:30-35


def load_scene():
    s = np.load(os.path.join(REPO, 'tests', 'golden', 'scene.npz'))
    bound = torch.from_numpy(s['bound'])
    pose = torch.from_numpy(s['poses'][2])            # room0 gt_c2w_list[1000]
    wpath = os.path.join(REPO, 'tests', 'golden', 'weights.npz')
    params = None
    if os.path.exists(wpath):
        w = np.load(wpath)
        params = {k[len('trained/'):]: torch.from_numpy(w[k]) for k in w.files if k.startswith('trained/')}
    return bound, pose, params


def synth_batch(n, rank, pose, dev, seed=0):
    g = torch.Generator().manual_seed(seed + 1000 * rank)
    pix = torch.randint(0, W * H, (n,), generator=g)
    i, j = (pix % W).float(), (pix // W).float()
    dirs = torch.stack([(i - CX) / FX, -(j - CY) / FY, -torch.ones_like(i)], -1)
    rd = torch.sum(dirs[:, None, :] * pose[:3, :3], -1)
    ro = pose[:3, 3].expand(rd.shape)
    gt = torch.rand(n, generator=g) * 0.55 + 0.05
    gt[torch.rand(n, generator=g) < 0.1] = 0.0
    col = torch.rand((n, 3), generator=g)
    return (ro.contiguous().to(dev), rd.contiguous().to(dev), gt.to(dev), col.to(dev))


def pmc_traffic(kernel, units_per_launch, workload=None):
    """HBM bytes per launch of `kernel` from the newest committed PMC measurement that holds it
    (profiles/r*_traffic.json, written by tools/traffic_json.py from separate FETCH_SIZE / WRITE_SIZE
    rocprofv3 passes): measured bytes per unit x units per launch, or None.  Files are ordered by
    name (round, then pass letter); a newer file measuring other kernels does not hide an older
    measurement of this one."""
    import glob
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_traffic*.json')), reverse=True)
    # a measurement of this workload first (the room0 batch: its split-K partial tiles are a larger
    # share of the grouped launch's bytes than at S-map), then any
    for key in ([f'{kernel}@{workload}'] if workload else []) + [kernel]:
        for f in files:
            t = json.load(open(f)).get(key)
            if t:
                return round((t['fetch_B'] + t['write_B']) * units_per_launch)
    return None


def neural_point_scene(dev, voxel=0.001, n_rays=W * H, seed=0):
    """Neural points on the trained decoder's own rendered surface at room0 pose 1000 (640x480,
    ScanNet intrinsics), voxel-downsampled like Point-NeRF's point initialisation (at most one
    point per `voxel` cube), features N(0, 0.1); plus the sample positions of one mapping
    iteration over `n_rays` random pixels (32 stratified in [0.01 d, 1.2 d] + 12 around the
    surface, sigma 5 mm) as float64 points.  Returns xyz, feats, p, (rays_o, rays_d, depth) of
    those pixels."""
    import types
    import pnr
    bound, pose, params = load_scene()
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=FX, fy=FY, cx=CX, cy=CY)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    with torch.no_grad():
        depth, _, _ = r.render_img({}, dec, pose, dev, 'color')
    ro, rd = pnr.get_rays(H, W, FX, FY, CX, CY, pose, dev)
    depth = depth.reshape(-1).float()
    surf = ro.reshape(-1, 3) + rd.reshape(-1, 3) * depth[:, None]
    g = torch.Generator(device=dev).manual_seed(seed)
    valid = surf[depth > 0]
    key = torch.floor(valid / voxel).long()
    key = (key[:, 0] + 4096) * (8192 * 8192) + (key[:, 1] + 4096) * 8192 + (key[:, 2] + 4096)
    uniq, inv = torch.unique(key, return_inverse=True)
    first = torch.full((uniq.shape[0],), valid.shape[0], device=dev, dtype=torch.long)
    first.scatter_reduce_(0, inv, torch.arange(valid.shape[0], device=dev), reduce='amin')
    xyz = valid[first].contiguous()
    feats = (0.1 * torch.randn((xyz.shape[0], 32), device=dev, generator=g)).contiguous()
    rays = torch.randint(0, surf.shape[0], (n_rays,), device=dev, generator=g)
    o = ro.reshape(-1, 3)[rays].double()
    d = rd.reshape(-1, 3)[rays].double()
    gt = depth[rays].double()
    t = torch.linspace(0, 1, 32, device=dev, dtype=torch.float64)
    z = (0.01 * gt)[:, None] * (1 - t) + (1.2 * gt)[:, None] * t
    zi = gt[:, None] + 0.005 * torch.randn((n_rays, 12), device=dev, dtype=torch.float64, generator=g)
    z = torch.sort(torch.cat([z, zi], 1), 1).values
    p = (o[:, None, :] + d[:, None, :] * z[:, :, None]).reshape(-1, 3).contiguous()
    return xyz, feats, p, (o.float().contiguous(), d.float().contiguous(), gt.float().contiguous())


def gather_bytes(n_samples, n_probed, n_nb_total, k, save=True, feat_bytes=128):
    """Algorithmic bytes of one pnr_point_gather: per sample 24 B point + 128 B c
    (+ k x 8 B idx/weight saves); 8 x 8 B bucket headers only for the `n_probed` samples whose probe
    block is occupied (the others stop at one L2-resident filter bit); per neighbour 4 B idx + 12 B
    xyz + 128 B features (64 B with float16 features)."""
    return (n_samples * (24 + 128 + (k * 8 if save else 0)) + n_probed * 8 * 8 +
            n_nb_total * (4 + 12 + feat_bytes))


def gather_roofline(dev, voxel=0.001, k=8, reps=5, feat_dtype='float32'):
    """Time the point-gather kernels (k_gather_probe, the group scan / scatter and k_gather_search,
    hipEvents on their stream) on the neural-point scene; roofline against the HBM peak.  Then the
    gather backward (feature gradients) against its HBM + float-atomic floor."""
    import ctypes
    import pnr
    from pnr._lib import timing_read
    lib = pnr.library()
    xyz, feats, p, _ = neural_point_scene(dev, voxel)
    pts = pnr.NeuralPoints(xyz, feats, mode='idw', radius=2 * voxel, k=k, feat_dtype=feat_dtype).to(dev)
    P = p.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, k), device=dev, dtype=torch.int32)
    w = torch.empty((P, k), device=dev)
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    s, _ = pts.descriptor()
    st = pnr._lib.stream_of(dev)

    def run():
        pnr._lib.check(lib.pnr_point_gather(ctypes.byref(s), p.data_ptr(), P, c.data_ptr(), idx.data_ptr(),
                                            w.data_ptr(), ws.data_ptr(), ws.numel(), st), 'point_gather')
    run()
    torch.cuda.synchronize()
    nb = int((idx >= 0).sum().item())
    # samples on the search's work list: the 64 sub-list counters at the head of the workspace
    # (csrc/points.hip WorkList: counter r at int32 offset 32 r)
    probed = int(ws[:64 * 32 * 4].view(torch.int32)[::32].sum().item())
    lib.pnr_timing_enable(1)
    timing_read(4)
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    lib.pnr_timing_enable(0)
    launches, ms, _ = timing_read(4)
    avg = ms / launches
    byt = gather_bytes(P, probed, nb, k, feat_bytes=64 if feat_dtype == 'float16' else 128)
    gbs = byt / (avg * 1e-3) / 1e9
    # backward, the Mapper's form (feature gradients only: dL/df_i += w_k dL/dc), deterministic: exact
    # int64 fixed-point terms added by 64-bit integer atomics, converted once into g_feats (ABI 10)
    gf = torch.zeros_like(feats)
    gc = torch.randn_like(c)
    sb, _ = pts.descriptor(g_feats=gf)
    bws = torch.empty(lib.pnr_point_gather_bwd_workspace_bytes(ctypes.byref(sb), P), dtype=torch.uint8, device=dev)
    rows = int((idx[:, 0] >= 0).sum().item())
    touched = int(torch.unique(idx[idx >= 0]).numel())  # feature rows some sample names
    lib.pnr_timing_enable(1)
    timing_read(5)
    for _ in range(reps):
        pnr._lib.check(lib.pnr_point_gather_bwd(ctypes.byref(sb), p.data_ptr(), P, idx.data_ptr(), w.data_ptr(),
                                                c.data_ptr(), gc.data_ptr(), None, bws.data_ptr(), bws.numel(), st),
                       'point_gather_bwd')
    torch.cuda.synchronize()
    lib.pnr_timing_enable(0)
    bl, bms, _ = timing_read(5)
    bavg = bms / bl
    n_instr = ctypes.c_int64(0)
    pnr._lib.check(lib.pnr_point_gather_bwd_atomics(ctypes.byref(sb), bws.data_ptr(), P, ctypes.byref(n_instr), st),
                   'gather_bwd_atomics')
    M = int(xyz.shape[0])
    # HBM: per sample 4 B (its first neighbour index, the probe); per row with neighbours 128 B g_c
    # read twice (max |g_c| pass, then the sums) + k x 8 B idx/w (read twice: the max pass marks the
    # rows it names); per touched feature row its int64 accumulators zeroed, read once, and the
    # features' gradient read + written by the conversion (256 + 256 + 256 B); the M-bit touched map
    # zeroed and read (sparse calls; dense ones -- this bench scene -- zero and convert all M rows).  Atomics: the 64-bit add instructions the kernel counted as it issued them (256 B
    # each: 32 lanes x 8 B; shared neighbours are carried between a ray's rows, so far fewer go out than
    # rows x neighbours)
    sparse = P * k < 4 * M  # points.hip launch_gather_bwd: touched rows only, else every row
    b_hbm = P * 4 + rows * (2 * 128 + (2 if sparse else 1) * k * 8) + \
        ((touched * (256 + 256 + 256) + 2 * (M // 8)) if sparse else M * (256 + 256 + 256))
    b_atomic = int(n_instr.value) * 256
    t_floor = (b_hbm / (HBM_PEAK_GBS * 1e9) + b_atomic / 1.3e12) * 1e3
    bwd = {'kernel': 'k_gather_bwd_probe + k_gather_bwd_gmax + k_gather_bwd + k_gather_bwd_fin (feature gradients, '
                     'the Mapper case; deterministic int64 fixed point)',
           'avg_launch_ms': round(bavg, 4), 'bytes_hbm': b_hbm, 'bytes_atomic_issued': b_atomic,
           'atomic_instructions': int(n_instr.value), 'neighbour_terms': nb, 'rows': rows,
           'touched_feature_rows': touched,
           'achieved_gbs': round((b_hbm + b_atomic) / (bavg * 1e-3) / 1e9, 1),
           'floor_ms': round(t_floor, 4), 'frac_of_floor': round(t_floor / bavg, 4),
           'floor_basis': 'HBM bytes at 8 TB/s + the issued 64-bit atomic bytes (counted in the kernel) at the '
                          '1.3 TB/s chip-wide atomic byte rate MI355X_MICROARCH.md measured for 32-bit float '
                          'atomics (64-B memory-side requests; assumed the same byte rate for 64-bit integer adds)'}
    return {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
            'frac': round(gbs / HBM_PEAK_GBS, 4),
            # PMC bytes per sample were measured on the float32-feature gather only
            'traffic': pmc_traffic('k_gather', P) if feat_dtype == 'float32' else None,
            'kernel': 'k_gather_probe+k_group_scatter+k_gather_search',
            'avg_launch_ms': round(avg, 3), 'launches': launches, 'samples': P, 'points': int(xyz.shape[0]),
            'neighbours_per_sample': round(nb / P, 3), 'probed_samples': probed, 'radius': 2 * voxel, 'k': k,
            'point_features': feat_dtype, 'bytes_per_launch': byt,
            'byte_basis': 'per sample 24 B point + 128 B c + k x 8 B idx/weight; 8 x 8 B bucket headers per '
                          'probed sample (occupied probe block); per neighbour 4 + 12 + 128 B',
            'backward': bwd}


def cpu_threads():
    """Threads of the CPU baseline: torch's intra-op pool (OMP_NUM_THREADS = this host's CPU share,
    16 on the GPU box), capped at the physical cores psutil reports."""
    n = torch.get_num_threads()
    try:
        import psutil
        n = min(n, psutil.cpu_count(logical=False) or n)
    except ImportError:
        pass
    return max(1, n)


def host_cpus():
    """What the CPU baseline's `cores` is drawn from: torch's pool, the CPUs this process may run on
    (sched_getaffinity), and the machine's physical / logical counts (psutil, when importable).
    On the GPU box the affinity set is the whole machine while the job's share is 16 CPUs
    (OMP_NUM_THREADS), so `cores` is the pool size, not the affinity count."""
    h = {'torch_threads': torch.get_num_threads(), 'omp_num_threads': os.environ.get('OMP_NUM_THREADS')}
    try:
        h['affinity_cpus'] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        pass
    try:
        import psutil
        h['physical_cores'] = psutil.cpu_count(logical=False)
        h['logical_cpus'] = psutil.cpu_count(logical=True)
    except ImportError:
        pass
    return h


def cpu_baseline(bound, pose, params, workload, gpu_render=None, reps=5):
    """The oracle (oracle/ref_render.py, a bit-exact restatement of the reference CPU path pinned
    by tests/test_oracle_golden.py) timed on this host on a bounded sample, median of `reps` after
    one warm-up, at the physical-core thread count and at 1 thread.  `gpu_render(ro,
    rd, gt) -> (depth, colour)` renders the same rays on the measured HIP path with the initial
    weights; the leg then reports the metric's PSNR condition on them."""
    from oracle import ref_render as ref
    cores = cpu_threads()
    prev = torch.get_num_threads()
    # rays per sample: ~1-3 s per timed step at each thread count
    sizes = {'map': (2048, 256), 'fwd': (8192, 1024)}[workload]

    def rate(n_rays, threads):
        torch.set_num_threads(threads)
        ro, rd, gt, col = [t.cpu() for t in synth_batch(n_rays, 0, pose, 'cpu', seed=7)]
        p = {k: v.clone().requires_grad_(workload == 'map') for k, v in params.items()}
        opt = torch.optim.Adam(list(p.values()), lr=2e-4) if workload == 'map' else None

        def step():
            if workload == 'map':
                opt.zero_grad()
                d, v, c = ref.render_batch_ray(p, rd, ro, bound, gt_depth=gt)
                sig = ref.regulation(p, rd, ro, gt, bound)
                ref.mapping_loss(d, c, gt, col, sig).backward()
                opt.step()
            else:
                with torch.no_grad():
                    ref.render_batch_ray(p, rd, ro, bound, n_samples=64, n_importance=0)

        step()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            step()
            ts.append(time.perf_counter() - t0)
        return n_rays / float(np.median(ts))

    v_all = rate(sizes[0], cores)
    v_one = rate(sizes[1], 1)
    torch.set_num_threads(prev)
    what = {'map': 'map step (render + regulation + L1 losses + backward + Adam)',
            'fwd': 'render_batch_ray forward, 64 samples'}[workload]
    out = {'value': round(v_all, 1), 'unit': 'rays/s', 'cores': cores, 'kind': 'port',
           'sample': f'{what} on {sizes[0]} rays ({cores} threads) and {sizes[1]} rays (1 thread), oracle (torch '
                     f'CPU restatement of src/utils/Renderer.py), median of {reps} after 1 warm-up',
           'value_1thread': round(v_one, 1), 'host': host_cpus()}
    if gpu_render is not None:
        ro, rd, gt, col = [t.cpu() for t in synth_batch(2048, 0, pose, 'cpu', seed=7)]
        with torch.no_grad():
            if workload == 'map':
                d_r, _, c_r = ref.render_batch_ray(params, rd, ro, bound, gt_depth=gt)
            else:
                d_r, _, c_r = ref.render_batch_ray(params, rd, ro, bound, n_samples=64, n_importance=0)
        d_g, c_g = gpu_render(ro, rd, gt if workload == 'map' else None)
        rel = ((d_g.double() - d_r.double()).abs() / d_r.double().abs().clamp_min(1e-12)).max().item()
        out['parity'] = {'psnr_db': round(ref.psnr(c_g, c_r), 2), 'depth_max_rel': float(f'{rel:.3g}'),
                         'rays': 2048,
                         'what': 'PSNR of the HIP render vs the oracle render of the same rays (initial weights); '
                                 'the metric\'s PSNR delta vs GT <= 0.1 dB holds when this exceeds PSNR(ref, GT) '
                                 '+ 39 dB (SURVEY.md 8(d))'}
    return out


def timed(step, steps, warmup, ddp, lib):
    """W untimed steps, then exactly K steps between barrier + device syncs; wall seconds (max over
    ranks) and the libpnr kernel timings (hipEvents on each launch's stream) of the K steps."""
    from pnr._lib import timing_read
    for _ in range(warmup):
        step()
    ddp.barrier()
    torch.cuda.synchronize()
    lib.pnr_timing_enable(1)
    for kind in range(7):
        timing_read(kind)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    ddp.barrier()
    el = time.perf_counter() - t0
    lib.pnr_timing_enable(0)
    kt = {'mlp_fwd': timing_read(0), 'mlp_bwd': timing_read(1), 'wgrad': timing_read(3), 'gather': timing_read(4),
          'gather_bwd': timing_read(5), 'wgrad_group': timing_read(6)}
    kt = {k: v for k, v in kt.items() if v[0] > 0}
    if ddp.world > 1:
        t = torch.tensor([el], device='cuda', dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        el = float(t.item())
    return el, kt


def kernel_roofline(kt, prec, el_s, traffic_units=True, fc=False, workload=None):
    """Roofline of the dominant hand-written kernel of the step -- the one with the most device time
    among the fused forward, the delta chain and the grouped weight-gradient launch -- per launch.
    The MLP kernels (arithmetic intensity above the machine balance) on the MFMA roof: algorithmic
    fp32-equivalent FLOP per point x points / mean launch time.  The grouped weight-gradient launch
    (58.5 FLOP per byte of fp32 operands, 45.5 with fc_c: below the 104 of 833 TF / 8 TB/s) on the HBM
    roof: algorithmic operand bytes per point x the delta chain's points / mean launch time, with its
    fraction of the split MFMA peak beside it (its MACs from pnr_timing_read kind 6: units of 65,536
    MACs = 131,072 FLOP)."""
    best = None
    for name, (launches, ms, units) in kt.items():
        if name not in ('mlp_fwd', 'mlp_bwd', 'wgrad_group'):
            continue
        if name == 'wgrad_group':  # f16x3 GEMMs in every split precision
            fl, kprec, kname = 131072, 'f16x3', 'k_wgrad16_group'
        else:
            fl = FLOP_PER_POINT_FWD if name == 'mlp_fwd' else FLOP_PER_POINT_BWD
            # the delta chain is fp32 in the fp32 mode and the f16x3 split in every other mode
            kprec = prec if name == 'mlp_fwd' else ('fp32' if prec == 'fp32' else 'f16x3')
            # (the f16x3 forward without features runs the 16-point-wave kernel, csrc/mlp16w.h)
            kname = ({'fp32': 'k_mlp_fwd', 'f16x3': 'k_mlp_fwd16w'}.get(prec, 'k_mlp_fwd16') if name == 'mlp_fwd' else
                     ('k_mlp_bwd16' if prec != 'fp32' else 'k_mlp_bwd'))
        # PMC traffic is kept per training point: the grouped launch's points are the delta chain's
        pts = (kt['mlp_bwd'][2] / launches if 'mlp_bwd' in kt else None) if name == 'wgrad_group' else units / launches
        cand = {'kernel': kname, 'launches': launches, 'prec': kprec, 'peak': ALGO_PEAK_TF[kprec],
                'avg_ms': ms / launches, 'share_of_step': ms / (el_s * 1e3), 'units': units / launches,
                'points': pts, 'achieved': fl * units / launches / (ms / launches * 1e-3) / 1e12, '_ms': ms}
        if best is None or ms > best['_ms']:
            best = cand
    if best is None:
        return None
    tkey = {'k_mlp_fwd': 'k_mlp_fwd_train', 'k_mlp_fwd16': 'k_mlp_fwd16_train', 'k_mlp_fwd16w': 'k_mlp_fwd16_train',
            'k_mlp_bwd': 'k_mlp_bwd',
            'k_mlp_bwd16': 'k_mlp_bwd16', 'k_wgrad16_group': 'k_wgrad16_group'}
    traffic = (pmc_traffic(tkey[best['kernel']], best['points'], workload) if traffic_units and best['points']
               else None)
    if best['kernel'] == 'k_wgrad16_group' and best['points']:
        bpp = WGRAD_B_PER_POINT + (WGRAD_FC_B_PER_POINT if fc else 0)
        fpp = WGRAD_FLOP_PER_POINT + (WGRAD_FC_FLOP_PER_POINT if fc else 0)
        gbs = bpp * best['points'] / (best['avg_ms'] * 1e-3) / 1e9
        return {'bound': 'hbm', 'achieved': round(gbs, 1), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(gbs / HBM_PEAK_GBS, 4), 'traffic': traffic,
                'kernel': best['kernel'], 'avg_launch_ms': round(best['avg_ms'], 3), 'launches': best['launches'],
                'kernel_share_of_step': round(best['share_of_step'], 3),
                'byte_basis': f'algorithmic fp32 operand bytes, {bpp:,} per training point x {best["points"]:,.0f} '
                              'points per launch (bench.py WGRAD_B_PER_POINT); traffic = PMC bytes per launch',
                'arithmetic_intensity': round(fpp / bpp, 1), 'ridge_flop_per_byte': round(best['peak'] * 1e3 /
                                                                                         HBM_PEAK_GBS, 1),
                'achieved_tflops': round(best['achieved'], 2),
                'frac_of_split_peak': round(best['achieved'] / best['peak'], 4)}
    return {'bound': 'mfma', 'achieved': round(best['achieved'], 2), 'peak': round(best['peak'], 1),
            'unit': 'TFLOP/s', 'frac': round(best['achieved'] / best['peak'], 4), 'traffic': traffic,
            'kernel': best['kernel'], 'avg_launch_ms': round(best['avg_ms'], 3), 'launches': best['launches'],
            'kernel_share_of_step': round(best['share_of_step'], 3),
            'flop_basis': ('algorithmic fp32-equivalent FLOP (2 x the multiply-adds of the launch\'s weight-gradient '
                           'GEMMs); peak = ' if best['kernel'] == 'k_wgrad16_group' else
                           'algorithmic fp32-equivalent FLOP (443,438 fwd / 442,880 bwd per point); peak = ')
                          + ('fp32 MFMA 157.3 TF' if best['prec'] == 'fp32' else
                             'f16/bf16 MFMA 2.5 PF dense / 3 products per fp32 product'
                             if best['prec'] != 'bf16' else 'bf16 MFMA 2.5 PF dense')}


def kernel_table(kt, prec, el_s, steps, fc=False):
    """Every timed MLP kernel family of the step on its MFMA roofline (algorithmic fp32-equivalent
    FLOP / measured time; the split modes against 833 TF, fp32 against 157.3 TF), with the MFMA-busy
    fraction of the newest committed rocprofv3 PMC pass (profiles/r*_mfma_busy_map.json)."""
    import glob
    busy = {}
    files = sorted(glob.glob(os.path.join(REPO, 'profiles', 'r*_mfma_busy_map.json')))
    if files:
        for k, v in json.load(open(files[-1])).get('kernels', {}).items():
            busy[k] = v.get('mfma_busy_frac')
    peak = ALGO_PEAK_TF['fp32' if prec == 'fp32' else 'f16x3']
    out = {}
    kt = dict(kt)
    if 'wgrad_group' in kt or 'wgrad' in kt:  # every weight-gradient launch: the group + dWo / dB (or fp32 GEMMs)
        g = kt.get('wgrad_group', (0, 0.0, 0))
        w = kt.get('wgrad', (0, 0.0, 0))
        kt['wgrad_all'] = (g[0] + w[0], g[1] + w[1], 0)
    fwd_label = 'k_mlp_fwd16w (training, saves)' if prec == 'f16x3' else 'k_mlp_fwd16 (training, saves)'
    for name, fl, kname in (('mlp_fwd', FLOP_PER_POINT_FWD, fwd_label),
                            ('mlp_bwd', FLOP_PER_POINT_BWD, 'k_mlp_bwd16 (delta chain)'),
                            ('wgrad_all', 443430 + (65536 if fc else 0),
                             'k_wgrad16_group + k_wgrad_skinny (all weight gradients)')):
        if name not in kt:
            continue
        launches, ms, units = kt[name]
        # the weight gradients over the delta chain's points (fc: + the four 256 x 32 fc_c GEMMs)
        pts = kt['mlp_bwd'][2] if name == 'wgrad_all' and 'mlp_bwd' in kt else units
        tf = fl * pts / (ms * 1e-3) / 1e12
        out[kname] = {'achieved_tf': round(tf, 1), 'peak_tf': round(peak, 1), 'frac': round(tf / peak, 4),
                      'ms_per_step': round(ms / steps, 3),
                      'share_of_step': round(ms / (el_s * 1e3), 3)}
    pm = {'k_mlp_fwd16 (training, saves)': ('void pnr::k_mlp_fwd16<3, false, 1>', 'void pnr::k_mlp_fwd16<3, false, true>'),
          'k_mlp_fwd16w (training, saves)': ('void pnr::k_mlp_fwd16w<1, 8>', 'void pnr::k_mlp_fwd16w<1>'),
          'k_mlp_bwd16 (delta chain)': ('void pnr::k_mlp_bwd16<false>',)}
    for k, names in pm.items():
        for b in names:
            if k in out and b in busy:
                out[k]['mfma_busy_pmc'] = busy[b]
    return out


DTYPE = {'fp32': 'fp32 (fp32 MFMA forward, delta chain and weight gradients)',
         'f16x3': 'fp32-class f16x3 throughout: forward, delta chain (per-point power-of-two scaled) and weight-'
                  'gradient GEMMs (on fp32-stored operands) all split every operand into 2 f16 parts (22 '
                  'significant bits), 3 MFMA products, fp32 accumulation; dWo/dB fp32 FMA',
         'bf16x3': 'bf16x3 split forward (16 significant bits); f16x3 backward as the default',
         'bf16': 'bf16 MFMA forward (fp32 accumulate); f16x3 backward as the default'}


def make_decoder(pnr, cfg, params, dev):
    dec = pnr.get_model(cfg, nice=False)
    if params is not None:
        dec.load_state_dict(params)
    return dec.to(dev)


def map_step_fn(pnr, renderer, dec, cfg, ro, rd, gt, col, dev, ddp=None, points=None, graph=False):
    from pnr.mapping import MapStep, MapGraph
    n = ro.shape[0]
    ns = cfg['rendering']['N_samples']
    mstep = MapStep(renderer, dec, lr=cfg['mapping']['imap_decoders_lr'], w_color_loss=cfg['mapping']['w_color_loss'],
                    ddp=ddp, points=points)
    if graph:
        mgraph = MapGraph(mstep, ro, rd, gt, col, torch.rand((n, ns), device=dev))

        def step():  # the same iteration, replayed; a fresh regulation jitter drawn per step, in place
            # into the graph's static input (the rays already sit in its other inputs: no copies)
            torch.rand((n, ns), device=dev, out=mgraph.inputs[4])
            mgraph(*mgraph.inputs)
        return step

    def step():
        mstep(ro, rd, gt, col, torch.rand((n, ns), device=dev))
    return step


def sfwd_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib, steps=10, cpu=True, rank=0, world=1,
               fixed_global=False):
    """S-fwd: render_batch_ray forward over the 640x480 batch at 64 stratified
    samples, no importance, gt_depth None; roofline of k_mlp_fwd16 (eval) and the oracle CPU rate.
    Data parallel: every rank renders its own 640x480 batch (weak, seed = rank), or -- fixed_global --
    its contiguous share of ONE 640x480 batch (strong).  gt_depth None leaves no batch-global coupling
    (the far clamp of src/utils/Renderer.py:112 needs gt), so the ranks exchange nothing."""
    import copy
    cfg = copy.deepcopy(pnr.ROOM0_CFG)
    cfg['rendering']['N_samples'], cfg['rendering']['N_importance'] = 64, 0
    r = pnr.Renderer(cfg, None, slam)
    dec = make_decoder(pnr, cfg, params, dev)
    if fixed_global:
        from pnr import dist as pdist
        a, b = pdist.shard_bounds(W * H, rank, world)
        ro, rd = [t[a:b].contiguous() for t in synth_batch(W * H, 0, pose, dev)[:2]]
    else:
        ro, rd, _, _ = synth_batch(W * H, rank, pose, dev)
    total = W * H if fixed_global else W * H * world

    def step():
        with torch.no_grad():
            r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=None)
    el, kt = timed(step, steps, 2, ddp, lib)
    prec = plib.DEFAULT_PRECISION
    out = {'workload': 'S-fwd: render_batch_ray forward, 640x480 rays x 64 stratified samples, gt_depth None'
                       + (' (ONE batch split over the ranks)' if fixed_global else ' per GPU'),
           'value': round(total * steps / el, 1), 'unit': 'rays/s', 'ms_per_step': round(el / steps * 1e3, 3),
           'steps': steps, 'n_gpus': world, 'scaling': 'strong' if fixed_global else 'weak',
           'rays_per_gpu': int(ro.shape[0]), 'global_batch': total,
           'roofline': kernel_roofline(kt, prec, el, traffic_units=False)}
    if out['roofline'] is not None:
        out['roofline']['kernel'] += ' (eval, no activation saves)'
    if cpu and params is not None and world == 1:
        def gpu_render(ro_c, rd_c, gt_c):
            with torch.no_grad():
                d, _, c = r.render_batch_ray({}, dec, rd_c.to(dev), ro_c.to(dev), dev, 'color', gt_depth=None)
            return d.cpu(), c.cpu()
        out['cpu_baseline'] = cpu_baseline(bound, pose, params, 'fwd', gpu_render=gpu_render)
        out['speedup_vs_cpu'] = round(out['value'] / out['cpu_baseline']['value'], 1)
    return out


MAP_FLOP_PER_RAY = 115.29e6        # (32 + 3 x 44 + 3 x 32) x 443,438 per mapping iteration


def oracle_map_rate(bound, pose, params, n, reps=3, threads=None, rays=None):
    """The oracle's Mapper iteration (render + regulation + L1 losses + backward + Adam) on n rays on
    this host's cores, rays/s (median of `reps` after one warm-up).  `rays` = (ro, rd, gt, col) to
    use instead of the synthetic S-map batch."""
    from oracle import ref_render as ref
    prev = torch.get_num_threads()
    torch.set_num_threads(threads or cpu_threads())
    if rays is not None:
        ro, rd, gt, col = [t.detach().cpu().float() for t in rays]
        n = ro.shape[0]
    else:
        ro, rd, gt, col = [t.cpu() for t in synth_batch(n, 0, pose, 'cpu', seed=7)]
    p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    opt = torch.optim.Adam(list(p.values()), lr=2e-4)

    def step():
        opt.zero_grad()
        d, v, c = ref.render_batch_ray(p, rd, ro, bound, gt_depth=gt)
        sig = ref.regulation(p, rd, ro, gt, bound)
        ref.mapping_loss(d, c, gt, col, sig).backward()
        opt.step()
    step()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        step()
        ts.append(time.perf_counter() - t0)
    torch.set_num_threads(prev)
    return n / float(np.median(ts))


def faithful_extra(pnr, slam, params, bound, pose, dev, ddp, lib, sizes=(1000, 5000), steps=50, cpu=True):
    """The Mapper iteration at its real batch sizes (room0: mapping.pixels = 1,000; ScanNet /
    Apartment: 5,000), replayed from a captured HIP graph; the algorithmic fraction of the split
    peak (115.29 MFLOP per ray) and the oracle's CPU rate at the same batch."""
    out = {}
    for n in sizes:
        cfg = pnr.ROOM0_CFG
        r = pnr.Renderer(cfg, None, slam)
        dec = make_decoder(pnr, cfg, params, dev)
        ro, rd, gt, col = synth_batch(n, 0, pose, dev)
        step = map_step_fn(pnr, r, dec, cfg, ro, rd, gt, col, dev, graph=True)
        el, _ = timed(step, steps, 3, ddp, lib)
        rate = n * steps / el
        tf = MAP_FLOP_PER_RAY * rate / 1e12
        peak = ALGO_PEAK_TF['f16x3']
        e = {'ms_per_iter': round(el / steps * 1e3, 4), 'rays_per_s': round(rate, 1), 'graph': True, 'iters': steps,
             'achieved_tflops': round(tf, 2), 'frac_of_split_peak': round(tf / peak, 4),
             'flop_basis': '115.29 MFLOP per ray per mapping iteration (SURVEY.md 8(d)); peak 833 TF (f16 MFMA / 3)'}
        if cpu:
            cr = oracle_map_rate(bound, pose, params, n)
            e['cpu_baseline'] = {'value': round(cr, 1), 'unit': 'rays/s', 'cores': cpu_threads(), 'kind': 'port',
                                 'sample': f'the oracle Mapper iteration on the same {n} rays, median of 3 after 1 '
                                           f'warm-up'}
            e['speedup_vs_cpu'] = round(rate / cr, 1)
        out[f'n{n}'] = e
    return out


# the room0 camera (configs/Replica/replica.yaml:22-28, inherited by configs/Replica/room0_point.yaml)
ROOM0_CAM = {'H': 680, 'W': 1200, 'fx': 600.0, 'fy': 600.0, 'cx': 599.5, 'cy': 339.5}
ROOM0_PIXELS, ROOM0_WINDOW = 1000, 5   # mapping.pixels (replica.yaml:21), mapping_window_size (pointNeRF_slam.yaml)


def room0_window(pnr, params, bound, dev):
    """The room0 Mapper's keyframe window (mapping_window_size 5: three random keyframes, the last
    keyframe and the current frame, src/Mapper.py:362-380) as synthetic frames on the room0 camera:
    renders of the trained decoder at the four fixture poses (tests/golden/scene.npz: gt_c2w_list
    entries of room0) and at the current pose (pose 1000 moved 2 cm), each frame's gt depth = its
    rendered depth (S-ref) and gt colour = its rendered colour.  The dataset frames
    are not in the image (no network)."""
    import types
    s = np.load(os.path.join(REPO, 'tests', 'golden', 'scene.npz'))
    poses = [torch.from_numpy(s['poses'][k]).float() for k in (0, 1, 3, 2)]
    cur = poses[3].clone()
    cur[:3, 3] += torch.tensor([0.02, -0.01, 0.01])
    poses.append(cur)
    slam = types.SimpleNamespace(bound=bound, **ROOM0_CAM)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    dec = make_decoder(pnr, pnr.ROOM0_CFG, params, dev)
    frames = []
    with torch.no_grad():
        for c2w in poses:
            d, _, c = r.render_img({}, dec, c2w.to(dev), dev, 'color')
            frames.append((c2w.to(dev), d.float().contiguous(), c.float().clamp(0, 1).contiguous()))
    return slam, frames


def room0_extra(pnr, params, bound, pose, dev, ddp, lib, steps=100, warmup=5, cpu=True, graph=True, rank=0,
                prec='f16x3'):
    """The metric's own workload: ONE room0 Mapper iteration (src/Mapper.py:507-662) at its real size,
    1,000 rays over the 5-frame window (200 per frame) of the room0 camera, gt = the decoder's own
    rendered depth / colour.  Timed per iteration: the window batch (pnr_window_sample: pixels, jitter
    and far clamp drawn on the device in one launch, src/Mapper.py:553-606), render (32 + 12 samples) + regulation (32) + fused L1 losses + backward +
    Adam, all replayed from one captured HIP graph (pnr.MapGraph(batch_fn=pnr.mapping.WindowSampler))."""
    from pnr.mapping import MapGraph, MapStep, WindowSampler
    slam, frames = room0_window(pnr, params, bound, dev)
    cfg = pnr.ROOM0_CFG
    r = pnr.Renderer(cfg, None, slam)
    dec = make_decoder(pnr, cfg, params, dev)
    per = ROOM0_PIXELS // ROOM0_WINDOW
    # data parallel: every rank draws its own 1,000-ray window batch (seed = rank), the
    # batch far clamp is all-reduced (MAX) on the device and the 891 KB gradient all-reduced (SUM) once
    # per iteration, both captured in the graph with the step (RCCL)
    sampler = WindowSampler(frames, per, ROOM0_CAM['fx'], ROOM0_CAM['fy'], ROOM0_CAM['cx'], ROOM0_CAM['cy'],
                            n_samples=cfg['rendering']['N_samples'], seed=rank)
    mstep = MapStep(r, dec, lr=cfg['mapping']['imap_decoders_lr'], w_color_loss=cfg['mapping']['w_color_loss'],
                    ddp=ddp if ddp.world > 1 else None)
    if graph:
        mg = MapGraph(mstep, batch_fn=sampler)
        step = mg
    else:
        def step():
            mstep(*sampler())
    el, _ = timed(step, steps, warmup, ddp, lib)
    n = per * ROOM0_WINDOW
    rate = n * steps / el
    # the same iteration launched eagerly, for the live per-kernel times (hipEvents around each launch;
    # a graph replay has no per-launch host hook): the MLP kernels' rooflines at this batch size
    el_e, kt = timed(lambda: mstep(*sampler()), 20, 3, ddp, lib)
    tf = MAP_FLOP_PER_RAY * rate / 1e12
    peak = ALGO_PEAK_TF['fp32' if prec == 'fp32' else 'f16x3']
    out = {'workload': 'room0 Mapper iteration: 1,000 rays = 5-frame window x 200 uniform pixels on the 680x1200 '
                       'fx=fy=600 camera, gt = rendered depth / colour (S-ref); window sampling + render (32+12) + '
                       'regulation (32) + L1 losses + backward + Adam in one replayed HIP graph',
           'rays_per_iter': n, 'ms_per_iter': round(el / steps * 1e3, 4), 'rays_per_s': round(rate, 1),
           'graph': graph, 'iters': steps, 'achieved_tflops': round(tf, 2), 'frac_of_split_peak': round(tf / peak, 4),
           'flop_basis': '115.29 MFLOP per ray per mapping iteration (SURVEY.md 8(d)); peak '
                         + ('157.3 TF (fp32 MFMA)' if prec == 'fp32' else '833 TF (f16 MFMA / 3)'),
           'decoder_precision': prec, 'dtype': DTYPE[prec],
           'eager_ms_per_iter': round(el_e / 20 * 1e3, 4),
           'roofline': kernel_roofline(kt, prec, el_e, traffic_units=prec != 'fp32', workload='room0'),
           'kernel_rooflines': kernel_table(kt, prec, el_e, 20) if prec != 'fp32' else None,
           'kernel_profile': 'profiles/r06_room0_timeline.txt, profiles/r06_room0_kernel_stats.csv (rocprofv3 of '
                             'the graph replay)'}
    if cpu and prec != 'fp32':
        rays = sampler()[:4]
        cr = oracle_map_rate(bound, pose, params, n, rays=rays)
        out['cpu_baseline'] = {'value': round(cr, 1), 'unit': 'rays/s', 'cores': cpu_threads(), 'kind': 'port',
                               'sample': f'the oracle Mapper iteration on one drawn window batch ({n} rays), median '
                                         f'of 3 after 1 warm-up'}
        out['speedup_vs_cpu'] = round(rate / cr, 1)
    return out


def map_points_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib, n=W * H, steps=3, cpu=True):
    """The neural-point Mapper iteration (--workload map-points) at 307,200 rays:
    rays/s, the roofline of its dominant MLP kernel, the gather and gather-backward HBM rates, and the
    oracle's CPU rate (brute-force neighbour search over the points near 32 of the rays)."""
    dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    sd = dec.state_dict()
    sd.update(params)
    dec.load_state_dict(sd)
    dec = dec.to(dev)
    xyz, feats, _, (ro, rd, gt) = neural_point_scene(dev, n_rays=n, seed=0)
    points = pnr.NeuralPoints(xyz, feats, mode='idw', radius=0.002, k=8).to(dev)
    col = torch.rand((n, 3), device=dev, generator=torch.Generator(device=dev).manual_seed(0))
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    step = map_step_fn(pnr, r, dec, pnr.ROOM0_CFG, ro, rd, gt, col, dev, points=points)
    el, kt = timed(step, steps, 1, ddp, lib)
    prec = plib.DEFAULT_PRECISION
    out = {'workload': 'S-map with neural points: c_dim=32 decoder, IDW k=8 r=2 mm gather, fc_c injection, '
                       'feature + decoder Adam', 'rays': n, 'points': int(xyz.shape[0]),
           'value': round(n * steps / el, 1), 'unit': 'rays/s', 'ms_per_step': round(el / steps * 1e3, 3),
           'steps': steps, 'roofline': kernel_roofline(kt, prec, el, traffic_units=False, fc=True),
           'kernel_rooflines': kernel_table(kt, prec, el, steps, fc=True),
           'kernels': {k: {'launches': v[0], 'ms': round(v[1], 3), 'units': v[2]} for k, v in kt.items()}}
    if 'gather_bwd' in kt:
        launches, ms, units = kt['gather_bwd']
        out['gather_bwd_ms_per_step'] = round(ms / steps, 3)
    if cpu:
        from oracle import ref_points as RP
        from oracle import ref_render as ref
        m = 32
        ro_c, rd_c, gt_c = ro[:m].cpu().double().float(), rd[:m].cpu(), gt[:m].cpu()
        xyz_c, f_c = xyz.cpu(), feats.cpu()
        # the points near these rays (a superset of every sample's neighbourhood)
        far = float(gt_c.max()) * 1.2 + 0.01
        t = torch.linspace(0, 1, 256)
        segs = (ro_c[:, None, :] + rd_c[:, None, :] * (t[None, :, None] * far)).reshape(-1, 3)
        keep = torch.zeros(xyz_c.shape[0], dtype=torch.bool)
        for a in range(0, segs.shape[0], 512):
            keep |= (torch.cdist(segs[a:a + 512], xyz_c) <= 0.004 + far / 255).any(0)
        sub = torch.nonzero(keep).reshape(-1)
        prm = {k: v.detach().cpu().clone().requires_grad_(True) for k, v in dec.state_dict().items()}
        fr = f_c[sub].clone().requires_grad_(True)
        pdict = dict(xyz=xyz_c[sub], feats=fr, mode='idw', radius=0.002, k=8, eps=1e-6)
        ev = lambda q: RP.eval_points_c(prm, q, bound, pdict)  # noqa: E731
        colc = col[:m].cpu()
        torch.set_num_threads(cpu_threads())

        def cstep():
            d, v, c = ref.render_batch_ray(prm, rd_c, ro_c, bound, gt_depth=gt_c, eval_fn=ev)
            sig = ref.regulation(prm, rd_c, ro_c, gt_c, bound, eval_fn=ev)
            ref.mapping_loss(d, c, gt_c, colc, sig).backward()
        cstep()
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            cstep()
            ts.append(time.perf_counter() - t0)
        cr = m / float(np.median(ts))
        out['cpu_baseline'] = {'value': round(cr, 1), 'unit': 'rays/s', 'cores': cpu_threads(), 'kind': 'port',
                               'sample': f'oracle Mapper loss + backward with the brute-force IDW gather on {m} of the '
                                         f'rays over the {int(sub.numel())} points near them (no Adam), median of 3'}
        out['speedup_vs_cpu'] = round(out['value'] / cr, 1)
    return out


def launch_ranks(args):
    """`--gpus N` (N > 1) outside torchrun: start N ranks, one per GPU, as ONE child process
    (python -m torch.distributed.run --nproc-per-node N, rendezvous on 127.0.0.1) and return its exit
    code.  Nothing here touches the GPU (torch.cuda.device_count does not initialise it on this image),
    so the launcher never replaces a process that holds a GPU context."""
    import socket
    import subprocess
    n_dev = torch.cuda.device_count()
    if n_dev < args.gpus:
        print(f'bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this node has {n_dev}', file=sys.stderr,
              flush=True)
        return 2
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(('127.0.0.1', 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.gpus}',
           '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault('PNR_DIST_BACKEND', 'nccl')   # RCCL over xGMI
    return subprocess.run(cmd, env=env).returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=None, help='timed steps (default: 100 room0 / 5 other workloads)')
    ap.add_argument('--warmup', type=int, default=None, help='untimed steps (default: 5 room0 / 2 others)')
    ap.add_argument('--workload', choices=['room0', 'map', 'fwd', 'map-points'], default='room0',
                    help='room0 (default, the metric\'s own iteration) | map (S-map, 307,200 rays) | fwd (S-fwd) | '
                         'map-points (neural-point S-map)')
    ap.add_argument('--rays', type=int, default=W * H, help='rays per GPU per step of the S-map workloads (weak scaling)')
    ap.add_argument('--global-batch', type=int, default=None,
                    help='fixed global batch split over the ranks (strong scaling; SURVEY.md 8(e))')
    ap.add_argument('--graph', action='store_true',
                    help='replay the S-map iteration from a captured HIP graph (pnr.mapping.MapGraph)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-gather', action='store_true', help='skip the point-gather roofline line')
    ap.add_argument('--no-extras', action='store_true', help='skip the extra workloads (smap, sfwd, faithful, ...)')
    ap.add_argument('--precision', default=None, help="decoder matmuls: f16x3 (default) | fp32 | bf16x3 | bf16")
    ap.add_argument('--feat-dtype', default='float32', choices=['float32', 'float16'],
                    help='neural-point feature storage (map-points workload and the gather line; C5: float16)')
    args = ap.parse_args()
    if args.steps is None:
        args.steps = 100 if args.workload == 'room0' else 5
    if args.warmup is None:
        args.warmup = 5 if args.workload == 'room0' else 2
    if args.gpus < 1:
        ap.error('--gpus must be >= 1')
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        sys.exit(launch_ranks(args))

    import pnr
    from pnr import _lib as plib
    from pnr import dist as pdist
    if args.precision is not None:
        plib.precision_code(args.precision)
        plib.DEFAULT_PRECISION = args.precision
    prec = plib.DEFAULT_PRECISION

    env_world = pdist.env_rank_world()[1]
    if env_world != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but the launcher started {env_world} rank(s)', file=sys.stderr, flush=True)
        sys.exit(2)
    if torch.cuda.device_count() < env_world:
        print(f'bench.py: {env_world} ranks need {env_world} GPUs, this node has {torch.cuda.device_count()}',
              file=sys.stderr, flush=True)
        sys.exit(2)
    rank, world, local = pdist.init()
    dev = torch.device('cuda', local % torch.cuda.device_count())
    torch.cuda.set_device(dev)
    dist_info = None
    if world > 1:
        import torch.distributed as tdist
        dist_info = {'backend': tdist.get_backend(), 'world_size': tdist.get_world_size(),
                     'collective': 'RCCL over xGMI' if tdist.get_backend() == 'nccl' else tdist.get_backend()}
        if rank == 0:
            print(f'bench.py: {dist_info["backend"]} process group, world size {dist_info["world_size"]}',
                  file=sys.stderr, flush=True)
    lib = pnr.library()
    bound, pose, params = load_scene()
    import types
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=FX, fy=FY, cx=CX, cy=CY)
    ddp = pdist.DataParallel()
    cpu_ok = not args.no_cpu_baseline and world == 1 and params is not None

    if args.workload == 'room0':  # the metric's own iteration (1,000 rays per GPU and iteration)
        e = room0_extra(pnr, params, bound, pose, dev, ddp, lib, steps=args.steps, warmup=args.warmup, cpu=cpu_ok,
                        rank=rank)
        extras = {}
        if not args.no_extras:
            extras['smap'] = smap_run(pnr, plib, slam, params, bound, pose, dev, ddp, lib, rank, world, prec,
                                      steps=5, warmup=2, cpu=cpu_ok)
            if world > 1:
                extras['fixed_global_batch'] = fixed_global_run(pnr, slam, params, pose, dev, ddp, lib, rank, world,
                                                                steps=5, warmup=2)
                # the north star's S-fwd curve (640x480 x 64 samples) at every N: weak and fixed-global forms
                extras['sfwd'] = sfwd_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib, cpu=False, rank=rank,
                                            world=world)
                extras['sfwd_fixed_global'] = sfwd_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib,
                                                         cpu=False, rank=rank, world=world, fixed_global=True)
            elif params is not None:
                extras.update(n1_extras(pnr, plib, slam, params, bound, pose, dev, ddp, lib, prec, args, cpu_ok))
        if rank == 0:
            out = {'metric': METRIC, 'value': round(e['rays_per_s'] * world, 1), 'unit': 'rays/s', 'n_gpus': world,
                   'steps': args.steps, 'warmup': args.warmup, 'ms_per_step': e['ms_per_iter'],
                   'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': DTYPE[prec],
                   'data': 'synthetic (renders of the trained room0 decoder fixture on the room0 camera)',
                   'config': {'workload': e['workload'], 'rays_per_gpu': e['rays_per_iter'],
                              'global_batch': e['rays_per_iter'] * world,
                              'parallelism': f'dp{world}' if world > 1 else 'dp1',
                              'decoder_precision': prec, 'graph': True},
                   'roofline': e.get('roofline'), 'cpu_baseline': e.get('cpu_baseline'),
                   'room0_iter': e}
            if dist_info:
                out['distributed'] = dist_info
            if 'smap' in extras:  # the S-map rays/s next to the headline (SURVEY.md 8(d) throughput batch)
                out['smap_value'] = extras['smap']['value']
            out.update(extras)
            if not args.no_gather and not args.no_extras and params is not None:
                # single-GPU kernel line (rank 0's GPU at N > 1, after every rank's timed regions)
                out['gather_roofline'] = gather_roofline(dev, feat_dtype=args.feat_dtype)
            print(json.dumps(out), flush=True)
        if world > 1:
            ddp.barrier()
            torch.distributed.destroy_process_group()
        return

    cfg = pnr.ROOM0_CFG
    if args.workload == 'fwd':
        import copy
        cfg = copy.deepcopy(cfg)
        cfg['rendering']['N_samples'], cfg['rendering']['N_importance'] = 64, 0
    renderer = pnr.Renderer(cfg, None, slam)
    strong = args.global_batch is not None
    if strong:  # this rank's contiguous share of one global batch
        a, b = pdist.shard_bounds(args.global_batch, rank, world)
        n = b - a
    else:
        n = args.rays
    points = None
    if args.workload == 'map-points':
        # the neural-point decoder: trained base weights + fresh fc_c, points on
        # the rendered surface, the same pixels' rendered depth as gt
        dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
        sd = dec.state_dict()
        sd.update(params)
        dec.load_state_dict(sd)
        dec = dec.to(dev)
        xyz, feats, _, (ro, rd, gt) = neural_point_scene(dev, n_rays=n, seed=rank)
        points = pnr.NeuralPoints(xyz, feats, mode='idw', radius=0.002, k=8, feat_dtype=args.feat_dtype).to(dev)
        col = torch.rand((n, 3), device=dev, generator=torch.Generator(device=dev).manual_seed(rank))
    else:
        dec = make_decoder(pnr, cfg, params, dev)
        if strong:  # the global batch drawn once (seed 0), this rank's slice
            ro, rd, gt, col = [t[a:b].contiguous() for t in synth_batch(args.global_batch, 0, pose, dev)]
        else:
            ro, rd, gt, col = synth_batch(n, rank, pose, dev)

    if args.workload in ('map', 'map-points'):
        step = map_step_fn(pnr, renderer, dec, cfg, ro, rd, gt, col, dev, ddp=ddp if world > 1 else None,
                           points=points, graph=args.graph)
    else:
        def step():
            with torch.no_grad():
                renderer.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=None)

    el, kt = timed(step, args.steps, args.warmup, ddp, lib)
    ms_per_step = el / args.steps * 1e3
    total = args.global_batch if strong else n * world
    value = total / (el / args.steps)
    roofline = kernel_roofline(kt, prec, el, traffic_units=args.workload == 'map')
    if renderer.status(dev):
        raise FloatingPointError('bench: the f16x3 forward met a value outside the f16 range (PNR_STATUS_F16_RANGE)')

    extras = {}
    if not args.no_extras and args.workload == 'map' and not strong and world > 1:
        extras['fixed_global_batch'] = fixed_global_run(pnr, slam, params, pose, dev, ddp, lib, rank, world,
                                                        steps=args.steps, warmup=args.warmup)

    if rank == 0:
        cpu = None
        if cpu_ok and args.workload != 'map-points':
            cpu = cpu_baseline(bound, pose, params, args.workload, gpu_render=gpu_render_fn(pnr, renderer, cfg, params,
                                                                                            dev))
        samples = '64' if args.workload == 'fwd' else '32+12 (+32 regulation)'
        out = {
            'metric': METRIC, 'value': round(value, 1), 'unit': 'rays/s', 'n_gpus': world, 'steps': args.steps,
            'warmup': args.warmup, 'ms_per_step': round(ms_per_step, 3), 'higher_is_better': True,
            'scaling': 'strong' if strong else 'weak', 'vs_baseline': None,
            'dtype': DTYPE[prec],
            'data': 'synthetic (640x480 ScanNet-intrinsics rays at room0 pose 1000, U[0.05,0.6] gt depth, trained '
                    'room0 decoder fixture)',
            'config': {'workload': WL_NAME[args.workload],
                       'rays_per_gpu': n, 'global_batch': total, 'samples_per_ray': samples,
                       'parallelism': f'dp{world}', 'decoder_precision': prec,
                       'graph': bool(args.graph and args.workload == 'map'),
                       **({'point_features': args.feat_dtype} if args.workload == 'map-points' else {})},
            'roofline': roofline, 'cpu_baseline': cpu,
            'kernel_rooflines': kernel_table(kt, prec, el, args.steps, fc=args.workload == 'map-points')
            if args.workload != 'fwd' else None,
            'kernels': {k: {'launches': v[0], 'ms': round(v[1], 3), 'units': v[2]} for k, v in kt.items()},
        }
        if dist_info:
            out['distributed'] = dist_info
        if cpu is not None:
            out['speedup_vs_cpu'] = round(value / cpu['value'], 1)
        out.update(extras)
        if world == 1 and not args.no_gather and params is not None and args.workload != 'fwd':
            # the neural-point gather on its own roofline, after the timed region
            out['gather_roofline'] = gather_roofline(dev, feat_dtype=args.feat_dtype)
        print(json.dumps(out), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


WL_NAME = {'map': 'S-map: full mapping iteration (render+regulation+L1 losses+backward+Adam)',
           'fwd': 'S-fwd: render_batch_ray forward',
           'map-points': 'S-map with neural points (A15): c_dim=32 decoder, IDW k=8 r=2 mm gather, fc_c injection, '
                         'feature + decoder Adam'}


def gpu_render_fn(pnr, renderer, cfg, params, dev):
    """The HIP render of the CPU baseline's rays with the initial weights (the parity line)."""
    def gpu_render(ro_c, rd_c, gt_c):
        d0 = make_decoder(pnr, cfg, params, dev)
        with torch.no_grad():
            d, _, c = renderer.render_batch_ray({}, d0, rd_c.to(dev), ro_c.to(dev), dev, 'color',
                                                gt_depth=None if gt_c is None else gt_c.to(dev))
        return d.cpu(), c.cpu()
    return gpu_render


def smap_run(pnr, plib, slam, params, bound, pose, dev, ddp, lib, rank, world, prec, steps=5, warmup=2, cpu=True):
    """S-map: one full Mapper iteration over 307,200 rays per GPU (weak scaling), with
    the roofline of its dominant MLP kernel, every MLP kernel family's roofline and the oracle's CPU rate."""
    cfg = pnr.ROOM0_CFG
    renderer = pnr.Renderer(cfg, None, slam)
    dec = make_decoder(pnr, cfg, params, dev)
    n = W * H
    ro, rd, gt, col = synth_batch(n, rank, pose, dev)
    step = map_step_fn(pnr, renderer, dec, cfg, ro, rd, gt, col, dev, ddp=ddp if world > 1 else None)
    el, kt = timed(step, steps, warmup, ddp, lib)
    if renderer.status(dev):
        raise FloatingPointError('bench: the f16x3 forward met a value outside the f16 range (PNR_STATUS_F16_RANGE)')
    value = n * world * steps / el
    out = {'workload': WL_NAME['map'] + ', 307,200 rays per GPU (640x480 ScanNet-intrinsics rays at room0 pose '
                                        '1000, U[0.05,0.6] gt depth)',
           'value': round(value, 1), 'unit': 'rays/s', 'n_gpus': world, 'scaling': 'weak', 'steps': steps,
           'ms_per_step': round(el / steps * 1e3, 3),
           'roofline': kernel_roofline(kt, prec, el, traffic_units=True),
           'kernel_rooflines': kernel_table(kt, prec, el, steps),
           'kernels': {k: {'launches': v[0], 'ms': round(v[1], 3), 'units': v[2]} for k, v in kt.items()}}
    if cpu and rank == 0:
        out['cpu_baseline'] = cpu_baseline(bound, pose, params, 'map',
                                           gpu_render=gpu_render_fn(pnr, renderer, cfg, params, dev))
        out['speedup_vs_cpu'] = round(value / out['cpu_baseline']['value'], 1)
    return out


def fixed_global_run(pnr, slam, params, pose, dev, ddp, lib, rank, world, steps=5, warmup=2):
    """The fixed-global-batch (strong-scaling) form of S-map: ONE 307,200-ray batch split over the
    ranks, the global far clamp all-reduced, one gradient all-reduce per step."""
    cfg = pnr.ROOM0_CFG
    from pnr import dist as pdist
    ga, gb = pdist.shard_bounds(W * H, rank, world)
    sro, srd, sgt, scol = [t[ga:gb].contiguous() for t in synth_batch(W * H, 0, pose, dev)]
    sdec = make_decoder(pnr, cfg, params, dev)
    sstep = map_step_fn(pnr, pnr.Renderer(cfg, None, slam), sdec, cfg, sro, srd, sgt, scol, dev,
                        ddp=ddp if world > 1 else None)
    sel, _ = timed(sstep, steps, warmup, ddp, lib)
    return {'global_batch': W * H, 'rays_per_gpu': gb - ga, 'scaling': 'strong', 'n_gpus': world,
            'ms_per_step': round(sel / steps * 1e3, 3), 'value': round(W * H * steps / sel, 1), 'unit': 'rays/s'}


def n1_extras(pnr, plib, slam, params, bound, pose, dev, ddp, lib, prec, args, cpu_ok):
    """The 1-GPU extras of the default line, measured after the headline's timed region."""
    extras = {'sfwd': sfwd_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib, cpu=cpu_ok),
              'faithful_n1000': faithful_extra(pnr, slam, params, bound, pose, dev, ddp, lib, cpu=cpu_ok),
              'map_points': map_points_extra(pnr, plib, slam, params, bound, pose, dev, ddp, lib, cpu=cpu_ok)}
    if prec != 'fp32':
        cfg = pnr.ROOM0_CFG
        n = W * H
        ro, rd, gt, col = synth_batch(n, 0, pose, dev)
        saved = plib.DEFAULT_PRECISION
        plib.DEFAULT_PRECISION = 'fp32'
        fdec = make_decoder(pnr, cfg, params, dev)
        fstep = map_step_fn(pnr, pnr.Renderer(cfg, None, slam), fdec, cfg, ro, rd, gt, col, dev)
        fel, fkt = timed(fstep, 3, 1, ddp, lib)
        plib.DEFAULT_PRECISION = saved
        extras['fp32'] = {'value': round(n * 3 / fel, 1), 'unit': 'rays/s',
                          'ms_per_step': round(fel / 3 * 1e3, 3), 'steps': 3, 'dtype': DTYPE['fp32'],
                          'roofline': kernel_roofline(fkt, 'fp32', fel, traffic_units=False)}
        # the headline's own iteration (room0, 1,000 rays, graph replay) in strict fp32 (config C2's precision)
        plib.DEFAULT_PRECISION = 'fp32'
        try:
            extras['room0_iter_fp32'] = room0_extra(pnr, params, bound, pose, dev, ddp, lib, steps=100, warmup=5,
                                                    cpu=False, prec='fp32')
        finally:
            plib.DEFAULT_PRECISION = saved
    return extras


if __name__ == '__main__':
    main()
