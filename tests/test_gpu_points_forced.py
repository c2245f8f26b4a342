"""Teacher-forced neural-point gradients (decoder.py:168-175, 196-197).

The end-to-end render tests (tests/test_gpu_points.py) let each side form its own sample positions:
the HIP renderer's importance samples follow its own coarse MLP outputs, so a few samples land on
the other side of a decision edge (a neighbour radius, a ReLU threshold) and those tests carry an
allowance for them.  Here the HIP gather + decoder are fed the ORACLE's own sample positions (the
coarse, importance and regulation points its render_batch_ray / regulation evaluated for the golden
rays), so the inputs are identical; the samples that still sit on a decision edge are identified in
float64 and left out of BOTH sides:
  * a ReLU pre-activation within 1e-5 of its layer's largest |pre-activation| (a float32 order can
    take either branch there), and
  * a candidate point within 1e-5 relative of the neighbourhood radius (IDW) or of the box (trilinear).
On the remaining samples the neighbour sets are asserted identical, and every gradient -- the 11
decoder tensors, the 8 fc_c tensors, the point features and dL/dp -- is held ELEMENTWISE at rtol 1e-3
against the correctly-rounded gradient (float64 GEMMs, rounded per layer: oracle.ref_points
.mlp_forward_c_cr) and the float32 oracle, with the float32 summation floor 64 u M and NO flip
allowance (test_gpu_points.grad_elementwise with flips=False).

The f16x3 weight-gradient GEMM of fc_c is batch-invariant as well: the gradient of a batch equals the
sum of the gradients of its halves to float32 association (|dg| <= 1e-6 |g| + 1e-5 max|g|), the
data-parallel contract of tools/dp_check.py.
"""
import numpy as np
import pytest
import torch

from conftest import golden_params, load_golden
from oracle import ref_points as RP
from oracle import ref_render as RR
from test_gpu_points import grad_elementwise, mag_arrays, surface_cloud

pytestmark = pytest.mark.gpu

EDGE_TAU = 1e-5


@pytest.fixture(autouse=True, params=['fp32', 'f16x3'])
def precision(request, monkeypatch):
    from pnr import _lib
    monkeypatch.setattr(_lib, 'DEFAULT_PRECISION', request.param)
    return request.param


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


def oracle_samples(params, ro, rd, gt, bound, pdict):
    """Every point the oracle's Mapper forward evaluates for these rays (src/Mapper.py:623-655): the
    32 coarse and 44 sorted fine samples of render_batch_ray and the 32 regulation samples, float64."""
    seen = []

    def ev(q):
        seen.append(q.detach().reshape(-1, 3).clone())
        return RP.eval_points_c(params, q, bound, pdict)
    with torch.no_grad():
        RR.render_batch_ray(params, rd, ro, bound, gt_depth=gt, eval_fn=ev)
        RR.regulation(params, rd, ro, gt, bound, eval_fn=ev, t_rand=torch.rand(
            (ro.shape[0], 32), generator=torch.Generator().manual_seed(17)))
    return torch.cat(seen).double()


def edge_free(params, q, xyz, pdict):
    """Samples with no ReLU pre-activation and no candidate distance on a decision edge (float64)."""
    keep = torch.ones(q.shape[0], dtype=torch.bool)
    # neighbourhood edge: a point at the radius (IDW) or on the box faces (trilinear)
    for a in range(0, q.shape[0], 4096):
        qa = q[a:a + 4096].float().double()
        dl = qa[:, None, :] - xyz.double()[None]
        if pdict['mode'] == 'idw':
            d2 = (dl * dl).sum(-1)
            r2 = pdict['radius'] ** 2
            bad = ((d2 - r2).abs() <= EDGE_TAU * r2).any(1)
        else:
            h = torch.tensor(pdict['spacing'], dtype=torch.float64)
            bad = (((dl.abs() - h).abs() <= EDGE_TAU * h).any(-1)).any(1)
        keep[a:a + 4096] &= ~bad
    # ReLU edges: pre-activations of every hidden layer in float64 on the float32 inputs
    c = RP.point_gather(q, xyz, pdict['feats'].detach(), pdict['mode'], pdict.get('radius', 0.0),
                        pdict.get('spacing'), pdict['k'], pdict['eps']).double()
    x = q.float().double()
    h = torch.sin(x @ params['embedder._B'].double())
    for li in range(4):
        z = h @ params[f'pts_linears.{li}.weight'].double().t() + params[f'pts_linears.{li}.bias'].double()
        keep &= ~((z.abs() <= EDGE_TAU * z.abs().max()).any(1))
        h = torch.relu(z) + c @ params[f'fc_c.{li}.weight'].double().t() + params[f'fc_c.{li}.bias'].double()
    return keep


@pytest.mark.parametrize('mode', ['idw', 'trilinear'])
def test_decoder_with_points_teacher_forced(pnr_mod, dev, mode, precision):
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev, seed=8)
    n = 48
    ro, rd, gt = ro[:n], rd[:n], gt[:n]
    params = RP.init_fc_c(golden_params('trained'), seed=3)
    kw = dict(mode=mode, k=8, radius=0.04, eps=1e-6, spacing=[0.03, 0.03, 0.03])
    pdict = dict(xyz=xyz, feats=feats, **kw)
    q_all = oracle_samples(params, ro, rd, gt, bound, pdict)
    keep = edge_free(params, q_all, xyz, pdict)
    q = q_all[keep].contiguous()
    print(f'{mode}: {q_all.shape[0]} oracle samples, {q.shape[0]} off every decision edge')
    assert q.shape[0] > 0.7 * q_all.shape[0]
    G = torch.randn((q.shape[0], 4), generator=torch.Generator().manual_seed(23), dtype=torch.float64).float()

    # HIP: gather + decoder with fc_c injection on the oracle's points (float64 in, as the renderer)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), **kw).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    qd = q.to(dev).requires_grad_(True)
    raw = dec(qd, c_grid={'points_color': pts})
    (raw * G.to(dev)).sum().backward()
    torch.cuda.synchronize()

    # identical neighbour sets on every kept sample
    from test_gpu_points import _gather_c_abi
    _, idx, _ = _gather_c_abi(pnr_mod, dev, pts, q, 8)
    _, idx_ref, _ = RP.point_gather(q, xyz, feats, mode, 0.04, [0.03] * 3, 8, 1e-6, return_idx=True)
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))

    refs = {}
    for cr_ in (False, True):
        ref_p = {k: t.clone().requires_grad_(True) for k, t in params.items()}
        fr = feats.clone().requires_grad_(True)
        qr = q.clone().requires_grad_(True)
        with RP.magnitudes() as mag:
            c = RP.point_gather(qr, xyz, fr, mode, 0.04, [0.03] * 3, 8, 1e-6)
            out = (RP.mlp_forward_c_cr if cr_ else RP.mlp_forward_c)(ref_p, qr, c)
            (out * G).sum().backward()
        refs[cr_] = ({k: t.grad for k, t in ref_p.items()}, fr.grad, qr.grad)
        if not cr_:
            mags = mag_arrays(mag, params)
            np.testing.assert_allclose(raw.detach().cpu().numpy(), out.detach().numpy(), rtol=0,
                                       atol=2e-5 * out.abs().max().item())
    for k, t in dec.named_parameters():
        grad_elementwise(t.grad, refs[True][0][k], refs[False][0][k], k, mag=mags[k])
    grad_elementwise(pts.feats.grad, refs[True][1], refs[False][1], 'dL/dfeats', mag=mags['feats'])
    # dL/dp: the Fourier backward and the gather weights' derivative (no magnitude record: rtol + atol)
    grad_elementwise(qd.grad.float(), refs[True][2].float(), refs[False][2].float(), 'dL/dp', atol=1e-5)


def test_fc_c_gradient_batch_invariant(pnr_mod, dev, precision):
    """The neural-point MapStep gradient of a batch equals the sum of the gradients of its two halves
    (the global far clamp fixed): every part -- decoder, fc_c and point features -- to float32
    association, |dg| <= 1e-6 |g| + 1e-5 max|g| (tools/dp_check.py's contract for sharded DP)."""
    from pnr.mapping import MapStep
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev, seed=9)
    n = 8192
    reps = -(-n // ro.shape[0])
    jit = torch.randn((n, 3), generator=torch.Generator().manual_seed(30)) * 2e-3
    ro, rd, gt = [t.repeat(reps, *([1] * (t.dim() - 1)))[:n] for t in (ro, rd, gt)]
    rd = rd + jit  # distinct rays over the golden surface
    ro, rd, gt = [t.contiguous().to(dev) for t in (ro, rd, gt)]
    gen = torch.Generator().manual_seed(31)
    col = torch.rand((n, 3), generator=gen).to(dev)
    tr = torch.rand((n, 32), generator=gen).to(dev)
    params = RP.init_fc_c(golden_params('trained'), seed=5)
    far = (gt.float() * 1.2).amax().reshape(1).contiguous()

    import types
    from test_gpu_points import make_renderer

    def grad(a, b):
        pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.04, k=8).to(dev)
        dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
        dec.load_state_dict({k: v.clone() for k, v in params.items()})
        ms = MapStep(make_renderer(pnr_mod, bound), dec.to(dev), points=pts, lr=0.0, feat_lr=0.0)
        ms(ro[a:b], rd[a:b], gt[a:b], col[a:b], tr[a:b], far_clamp=far)
        torch.cuda.synchronize()
        return ms.flat.grad.clone(), ms.n_dec
    cut = 3 * n // 8  # unequal shares: the weight-gradient GEMMs split K differently on each side
    g_all, n_dec = grad(0, n)
    g_a, _ = grad(0, cut)
    g_b, _ = grad(cut, n)
    g_sum = g_a + g_b
    for name, sl in (('decoder', slice(0, 222747)), ('fc_c', slice(222747, n_dec)), ('features', slice(n_dec, None))):
        d = (g_all[sl] - g_sum[sl]).abs()
        scale = g_all[sl].abs().max()
        worst = float((d / (1e-6 * g_all[sl].abs() + 1e-5 * scale)).max())
        print(f'{name}: max|g| {float(scale):.3e}, nonzero {int((g_all[sl] != 0).sum())} of {g_all[sl].numel()}, '
              f'bitwise equal {bool(torch.equal(g_all[sl], g_sum[sl]))}, max |g - (g_a + g_b)| / max|g| = '
              f'{float(d.max() / scale):.2e}, worst/bound {worst:.3f}')
        assert float(scale) > 0, name
        assert worst <= 1.0, name
