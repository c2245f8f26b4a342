"""Teacher-forced neural-point gradients (decoder.py:168-175, 196-197).

The end-to-end render tests (tests/test_gpu_points.py) let each side form its own sample positions:
the HIP renderer's importance samples follow its own coarse MLP outputs, so a few samples land on
the other side of a decision edge (a neighbour radius, a ReLU threshold) and those tests carry an
allowance for them.  Here the HIP gather + decoder are fed the ORACLE's own sample positions (the
coarse, importance and regulation points its render_batch_ray / regulation evaluated for the golden
rays), so the inputs are identical; the samples that still sit on a decision edge are identified in
float64 and left out of BOTH sides.  The edges are tied to rounding bounds, per element:
  * a ReLU pre-activation z_j = sum_i W_ji h_i + b_j with |z_j| <= RELU_ULPS u M_j, M_j = sum_i |W_ji h_i|
    + |b_j| its own summation magnitude (u = 2^-24): no float32 order of the sum (the torch CPU order,
    the MFMA's blocked fp32 order), nor the f16x3 split (3 x 2^-22 per product), moves z_j by more
    (measured: the oracle's float32 forward stays within 44 u M_j of the float64 one, inputs' own
    rounding included), and
  * a candidate point within NB_ULPS u of the neighbourhood radius (|d^2 - r^2| <= NB_ULPS u r^2, IDW)
    or of the box (||dx| - h| <= NB_ULPS u h, trilinear): float32 point coordinates and a three-term
    float32 distance.
The filter is checked against the kernel itself: the HIP training forward's saved ReLU masks are read
back, and every HIP decision that differs from the float64 one must lie inside the filter; on the
kept samples the HIP and float64 decisions are identical.  The dropped share is printed; the keep
floor is 0.9.
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

RELU_ULPS = 64.0
NB_ULPS = 16.0
U32 = 2.0 ** -24


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


def edge_free(params, q, xyz, pdict, return_z=False):
    """Samples with no ReLU pre-activation and no candidate distance on a decision edge (float64, the
    rounding bounds of the module docstring).  return_z: also the float64 pre-activations z (4, P, 256),
    their edge flags and the samples off every neighbourhood edge."""
    keep = torch.ones(q.shape[0], dtype=torch.bool)
    # neighbourhood edge: a point at the radius (IDW) or on the box faces (trilinear)
    for a in range(0, q.shape[0], 4096):
        qa = q[a:a + 4096].float().double()
        dl = qa[:, None, :] - xyz.double()[None]
        if pdict['mode'] == 'idw':
            d2 = (dl * dl).sum(-1)
            r2 = pdict['radius'] ** 2
            bad = ((d2 - r2).abs() <= NB_ULPS * U32 * r2).any(1)
        else:
            h = torch.tensor(pdict['spacing'], dtype=torch.float64)
            bad = (((dl.abs() - h).abs() <= NB_ULPS * U32 * h).any(-1)).any(1)
        keep[a:a + 4096] &= ~bad
    nb_ok = keep.clone()
    nb_keep = int(keep.sum())
    # ReLU edges: pre-activations of every hidden layer in float64 on the float32 inputs, each against
    # its own summation magnitude
    c = RP.point_gather(q, xyz, pdict['feats'].detach(), pdict['mode'], pdict.get('radius', 0.0),
                        pdict.get('spacing'), pdict['k'], pdict['eps']).double()
    x = q.float().double()
    h = torch.sin(x @ params['embedder._B'].double())
    zs, es = [], []
    for li in range(4):
        W, b = params[f'pts_linears.{li}.weight'].double(), params[f'pts_linears.{li}.bias'].double()
        z = h @ W.t() + b
        M = h.abs() @ W.abs().t() + b.abs()
        e = z.abs() <= RELU_ULPS * U32 * M
        keep &= ~e.any(1)
        zs.append(z)
        es.append(e)
        h = (torch.relu(z) + c @ params[f'fc_c.{li}.weight'].double().t() + params[f'fc_c.{li}.bias'].double()).float()
        h = h.double()
    print(f'decision edges: {q.shape[0] - nb_keep} samples at a neighbourhood edge, '
          f'{nb_keep - int(keep.sum())} more at a ReLU edge; {q.shape[0] - int(keep.sum())} of {q.shape[0]} dropped')
    if return_z:
        return keep, torch.stack(zs), torch.stack(es), nb_ok
    return keep


def hip_relu_decisions(pnr_mod, dec, x, c, prec):
    """The ReLU decisions [z > 0] of the HIP training forward (pnr_mlp_fwd_train_c) for points x (P,3)
    float32 and features c (P,32): its saved mask words (capi.cpp carve_save: e [ld][96], h [4][ld][256]
    fp32, x [ld] float4, then the masks [4][ld/32][64 lanes] uint4; unit u of lane half (u >> 2) & 1,
    word u >> 6, bit 16 ((u >> 5) & 1) + 4 ((u >> 3) & 3) + (u & 3): k_mlp_fwd16 conv1 / mlp.hip
    save_mask), decoded to a bool (4, P, 256)."""
    from pnr import _lib
    lib = pnr_mod.library()
    P = x.shape[0]
    ld = -(-P // 128) * 128
    dev = x.device
    ws = torch.empty(lib.pnr_mlp_train_workspace_bytes(P), dtype=torch.uint8, device=dev)
    raw = torch.empty((P, 4), device=dev)
    packed = dec._packed.image(dec.ordered_params())
    fcp = dec._packed_fc.image(dec.ordered_fc_params())
    _lib.check(lib.pnr_mlp_fwd_train_c(_lib.ptr(packed), _lib.ptr(fcp), _lib.ptr(x), _lib.ptr(c), P, _lib.ptr(raw),
                                       _lib.ptr(ws), ws.numel(), _lib.precision_code(prec), _lib.stream_of(dev)),
               'mlp_fwd_train_c')
    torch.cuda.synchronize()
    off = (96 + 4 * 256) * 4 * ld + 16 * ld
    words = ws[off:off + 128 * ld].view(torch.int32).view(4, ld // 32, 2, 32, 4).cpu().long() & 0xFFFFFFFF
    u = torch.arange(256)
    hh, wi, bit = (u >> 2) & 1, u >> 6, 16 * ((u >> 5) & 1) + 4 * ((u >> 3) & 3) + (u & 3)
    p = torch.arange(P)
    w = words[:, (p >> 5)[:, None], hh[None, :], (p & 31)[:, None], wi[None, :]]  # (4, P, 256)
    return ((w >> bit[None, None, :]) & 1).bool()


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
    keep, z64, edge, nb_ok = edge_free(params, q_all, xyz, pdict, return_z=True)
    q = q_all[keep].contiguous()
    print(f'{mode}: {q_all.shape[0]} oracle samples, {q.shape[0]} off every decision edge, '
          f'{q_all.shape[0] - q.shape[0]} dropped ({1 - q.shape[0] / q_all.shape[0]:.2%})')
    assert q.shape[0] >= 0.9 * q_all.shape[0]
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

    # the filter against the kernel's own ReLU decisions on ALL oracle samples off a neighbourhood edge
    # (where the neighbour sets, hence the features, agree): a HIP decision that differs from the
    # float64 one lies on a filtered ReLU edge, and none survives on a kept sample
    xa = q_all.float().to(dev).contiguous()
    with torch.no_grad():
        ca = pts.gather(q_all.to(dev)).contiguous()
    dec_hip = hip_relu_decisions(pnr_mod, dec, xa, ca, precision)
    dec64 = z64 > 0
    diff = (dec_hip != dec64) & nb_ok[None, :, None]
    clear = ~edge & (z64.abs() > 1e-3 * z64.abs().amax(-1, keepdim=True))
    assert not diff[clear].any(), 'HIP ReLU decisions away from every edge equal the float64 ones (mask decode)'
    print(f'HIP ReLU decisions differing from float64: {int(diff.sum())} of {diff.numel()}, on '
          f'{int(diff.any(-1).any(0).sum())} samples; outside the filter: {int((diff & ~edge).sum())}')
    assert not (diff & ~edge).any(), 'every HIP decision flip lies inside the rounding-bound filter'
    assert not diff[:, keep].any()

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
