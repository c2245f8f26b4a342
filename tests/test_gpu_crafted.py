"""Crafted-input parity of the HIP path against the oracle: the compositing and sample_pdf edge
cases of src/common.py:19-63,204-245 reached through the real kernels, and the gather's rare
search paths (points.hip).

Decoders are crafted by their output layer (src/conv_onet/models/decoder.py:200):
  * sigma <= 0 on every sample (bias -1e3): every alpha is 0, every weight is 0, the pdf is the
    +1e-5 floor alone (uniform), depth/colour collapse to 0;
  * saturated sigma (bias +1e3): alpha = 1 at the first sample, the pdf is one bin plus the 1e-5
    floor, so importance samples land in bins whose cdf step is < 1e-5 -- the `denom < 1e-5 -> 1`
    branch of sample_pdf (common.py:55-56);
  * sigma = 0 inside the bound (zero output weights and bias): only the sigma = 100 of points
    outside the bound (Renderer.py:57) carries density -- a step from 0 to 100 along each ray.
Each case: depth / colour / variance of render_batch_ray (with and without gt depth) and the decoder
gradients of a Mapper-style loss vs the oracle, in fp32 and f16x3 (the tolerances of
tests/test_gpu_parity.py; a gradient that is exactly zero in the reference must be zero here).
Gather: forced hash collisions (table_bits = 10 for ~7.8k occupied cells), one bucket of > 65,535
points (the unordered-bucket fallback), and a row sample of the bench's own scene (neural points on
the trained decoder's rendered room0 surface, r = 2 mm).
"""
import ctypes

import numpy as np
import pytest
import torch

from conftest import load_golden, golden_params
from oracle import ref_points as RP
from oracle import ref_render as RR

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


@pytest.fixture(scope='module')
def pnr_mod():
    import pnr
    pnr.library()
    return pnr


def close(a, b, rtol, atol, what):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


def crafted(kind):
    p = {k: v.clone() for k, v in golden_params('trained').items()}
    if kind == 'sigma_neg':
        p['output_linear.bias'][3] = -1e3
    elif kind == 'sigma_sat':
        p['output_linear.bias'][3] = 1e3
    elif kind == 'sigma_zero':
        p['output_linear.weight'][3] = 0.
        p['output_linear.bias'][3] = 0.
    return p


def rays(scene, n=384, seed=0):
    g = torch.Generator().manual_seed(seed)
    pix = torch.randint(0, 680 * 1200, (n,), generator=g)
    ro, rd = RR.rays_from_uv((pix % 1200).float(), (pix // 1200).float(), torch.from_numpy(scene['poses'][1]),
                             600., 600., 599.5, 339.5)
    gt = torch.rand(n, generator=g) * 0.5 + 0.1
    gt[::7] = 0.
    return ro.reshape(-1, 3).contiguous(), rd.reshape(-1, 3).contiguous(), gt, torch.rand((n, 3), generator=g)


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
@pytest.mark.parametrize('kind', ['sigma_neg', 'sigma_sat', 'sigma_zero'])
@pytest.mark.parametrize('with_gt', [False, True])
def test_crafted_decoder_render_and_grads(kind, with_gt, precision, pnr_mod, dev, scene):
    import types
    params = crafted(kind)
    ro, rd, gt, col = rays(scene)
    slam = types.SimpleNamespace(bound=scene['bound_t'], H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    cfg = dict(pnr_mod.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr_mod.Renderer(cfg, None, slam)
    dec = pnr_mod.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4,
                      pos_embedding_method='fourier')
    dec.load_state_dict(params)
    dec = dec.to(dev)
    g = gt.to(dev) if with_gt else None
    d, v, c = r.render_batch_ray({}, dec, rd.to(dev), ro.to(dev), dev, 'color', gt_depth=g)
    loss = (d - 0.3).abs().sum() + 0.05 * (c - col.to(dev)).abs().sum() + 1e-3 * v.sum()
    loss.backward()
    pr = {k: t.clone().requires_grad_(True) for k, t in params.items()}
    dr, vr, cr, ex = RR.render_batch_ray(pr, rd, ro, scene['bound_t'], gt_depth=gt if with_gt else None,
                                         return_extras=True)
    lr = (dr - 0.3).abs().sum() + 0.05 * (cr - col).abs().sum() + 1e-3 * vr.sum()
    lr.backward()
    wc = ex['w_coarse']
    if kind == 'sigma_neg':  # zero weight wherever the sample is inside the bound (sigma := 100 outside)
        assert (wc == 0).float().mean() > 0.5
    if kind == 'sigma_sat':  # one dominant bin: importance samples fall in cdf steps below 1e-5
        zs = ex['z_samples']
        assert (wc[:, 0] > 0.99).float().mean() > 0.5 and torch.isfinite(zs).all()
    assert r.status(dev) == 0
    close(d, dr, 1e-4, 1e-9, f'{kind} depth')
    close(c, cr, 1e-4, 2e-5, f'{kind} rgb')
    close(v, vr, 2e-3, 1e-8, f'{kind} var')
    for k, t in dec.named_parameters():
        gref = pr[k].grad
        if float(gref.abs().max()) == 0.0:
            assert t.grad is None or float(t.grad.abs().max()) == 0.0, f'{kind} grad {k} must be 0'
            continue
        close(t.grad, gref, 0, 2e-3 * float(gref.abs().max()), f'{kind} grad {k}')


def oracle_gather(q, xyz, feats, radius, k=8, batch=256):
    """RP.point_gather in batches of queries (rows are independent, so this is exact) over the
    points within 2 radius of some query (ascending original index: the (d2, index) tie order is
    kept); indices mapped back to the full cloud."""
    qf = q.float()
    keep = torch.zeros(xyz.shape[0], dtype=torch.bool)
    for a in range(0, qf.shape[0], 512):
        keep |= (torch.cdist(qf[a:a + 512], xyz) <= 2 * radius).any(0)
    sub = torch.nonzero(keep).reshape(-1)
    cs, idxs, ws = [], [], []
    for a in range(0, q.shape[0], batch):
        c, idx, w = RP.point_gather(q[a:a + batch], xyz[sub], feats[sub], 'idw', radius=radius, k=k,
                                    return_idx=True)
        cs.append(c)
        idxs.append(torch.where(idx >= 0, sub[idx.clamp(min=0)], idx))
        ws.append(w)
    return torch.cat(cs), torch.cat(idxs), torch.cat(ws)


def _gather_vs_oracle(pnr_mod, dev, xyz, feats, q, radius, k=8, **kw):
    lib = pnr_mod.library()
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=radius, k=k, **kw).to(dev)
    P = q.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, k), device=dev, dtype=torch.int32)
    w = torch.empty((P, k), device=dev)
    s, _ = pts.descriptor()
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    qd = q.to(dev).contiguous()
    assert lib.pnr_point_gather(ctypes.byref(s), qd.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    c_ref, idx_ref, w_ref = oracle_gather(q, xyz, feats, radius, k)
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32)), 'neighbour indices'
    close(w, w_ref, 0, 1e-6, 'weights')
    close(c, c_ref, 0, 1e-5 * float(c_ref.abs().max()), 'c')
    return idx_ref


def test_gather_forced_hash_collisions(pnr_mod, dev):
    """100k points over ~7.8k occupied cells hashed into 2^10 buckets: every bucket holds several
    cells, so each probe meets foreign cells (skipped by key) and colliding buckets (per-point cell
    test) -- the neighbour lists must still be the oracle's."""
    gen = torch.Generator().manual_seed(21)
    n = 100_000
    xyz = torch.rand((n, 3), generator=gen) * torch.tensor([1.2, 0.9, 0.9]) - 0.3
    feats = torch.randn((n, 32), generator=gen) * 0.5
    q = (xyz[torch.randint(0, n, (3000,), generator=gen)] + 0.02 * torch.randn((3000, 3), generator=gen)).double()
    idx = _gather_vs_oracle(pnr_mod, dev, xyz, feats, q, radius=0.025, table_bits=10)
    assert (idx >= 0).sum(1).float().mean() > 2


def test_gather_bucket_beyond_65535_points(pnr_mod, dev):
    """70,000 points inside ONE hash cell: the bucket is too large for the u16 sub-cell table and
    is scanned whole (points.hip unordered-bucket fallback)."""
    gen = torch.Generator().manual_seed(22)
    n = 70_000
    radius = 0.01
    cell = 2 * radius * 1.003
    xyz = 0.1 + torch.rand((n, 3), generator=gen) * (cell * 0.98)
    xyz = xyz + 0.001 * cell  # strictly inside one cell of the grid anchored at `origin`
    feats = torch.randn((n, 32), generator=gen) * 0.5
    q = (xyz[torch.randint(0, n, (512,), generator=gen)] + 0.004 * torch.randn((512, 3), generator=gen)).double()
    idx = _gather_vs_oracle(pnr_mod, dev, xyz, feats, q, radius=radius, k=8, cell=cell, origin=[0.1, 0.1, 0.1])
    assert (idx >= 0).all(1).float().mean() > 0.9  # dense: full neighbour lists


def test_gather_bench_scene_rows(pnr_mod, dev):
    """The bench's gather scene itself (bench.py neural_point_scene: points on the trained decoder's
    rendered room0 surface at 1-mm voxels, radius 2 mm, k = 8, 32+12 samples per ray over 307,200
    rays): 4,096 sampled rows of the full 13.5M-sample gather vs the oracle."""
    import bench
    xyz, feats, p, _ = bench.neural_point_scene(dev)
    lib = pnr_mod.library()
    pts = pnr_mod.NeuralPoints(xyz, feats, mode='idw', radius=0.002, k=8).to(dev)
    P = p.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, 8), device=dev, dtype=torch.int32)
    w = torch.empty((P, 8), device=dev)
    s, _ = pts.descriptor()
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    assert lib.pnr_point_gather(ctypes.byref(s), p.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    gen = torch.Generator(device=dev).manual_seed(5)
    has = torch.nonzero(idx[:, 0] >= 0).reshape(-1)
    sel = torch.cat([has[torch.randint(0, has.numel(), (3072,), device=dev, generator=gen)],
                     torch.randint(0, P, (1024,), device=dev, generator=gen)])
    c_ref, idx_ref, w_ref = oracle_gather(p[sel].cpu(), xyz.cpu(), feats.detach().cpu(), 0.002)
    assert np.array_equal(idx[sel].cpu().numpy(), idx_ref.numpy().astype(np.int32)), 'neighbour indices'
    close(w[sel], w_ref, 0, 1e-6, 'weights')
    close(c[sel], c_ref, 0, 1e-5 * float(c_ref.abs().max()), 'c')
    assert xyz.shape[0] > 100_000 and (idx_ref[:3072] >= 0).sum(1).float().mean() > 2
