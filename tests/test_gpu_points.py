"""Parity of the neural-point stage on the GPU: spatial-hash gather,
decoder with fc_c feature injection, and render_batch_ray / regulation with features, against
the CPU oracle (oracle/ref_points.py) and the reference's grid_sample decoder fixtures
(tests/golden/points_c32.npz).

Tolerances: gather idx exact; c / weights 1e-5 * max; raw 2e-5 * max; depth / colour 1e-4 rel
(north_star).  Gradients ELEMENTWISE (grad_elementwise): rtol 1e-3 with atol (1e-6 + d32) * max|g|
against the correctly-rounded gradient (every decoder / fc_c GEMM and the Fourier backward summed in
float64 and rounded, oracle.ref_points.mlp_forward_c_cr), d32 = the float32 gradient's own distance
from it (max |g_f32 - g_cr| / max |g_cr|), and rtol 1e-3 with atol (1e-6 + d32) * max|g| against
the float32 gradient.  For the reference's grid decoder (points_c32.npz) the correctly-rounded
gradient is the fixture tests/golden/grads_cr.npz `pts/*` and the float32 one the reference's own;
for the IDW / trilinear render / regulation / tracking cases both are the oracle's, formed in the
test, and elements may exceed the bound by up to FLIP_CAP max|g| (decision-edge samples, below).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, golden_params, maybe_dump_grads
from oracle import ref_points as RP
from oracle import ref_render as RR

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=['fp32', 'f16x3'])
def precision(request, monkeypatch):
    """Every GPU test runs under both decoder precisions (include/pnr.h PNR_PREC_*): the exact
    fp32 MFMA path and the f16x3 split path (the default), against the same tolerances."""
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


# Render / regulation / tracking with IDW or trilinear features over a random cloud: a few samples sit
# on a decision edge (a ReLU pre-activation, a neighbour's distance or a pdf bin boundary within
# rounding of the threshold), where two float32 orders take different branches (the end-to-end tests
# let each side place its own importance samples: tests/test_gpu_points_forced.py feeds the oracle's
# samples to the kernels and holds every kept sample to the strict bound with no allowance at all).
# A flipped sample changes ONE rank-1 term of every weight gradient -- dW = sum_p delta_p h_p^T, and with
# the bias as one more column [dW | db] = sum_p delta_p [h_p; 1]^T -- and of dL/dfeats and dL/drays
# (its own rows), so what a flip may move is a rank-1 matrix, not a share of the elements.  The
# allowance (round 6, replacing round 5's FLIP_FRAC share of elements and its 2% fp32-trilinear
# exception): the deviation from each reference may exceed the strict elementwise bound only by at most
# FLIP_RANK rank-1 terms -- after removing its best rank-k approximation (SVD, k <= FLIP_RANK) EVERY
# element is inside the strict bound -- and the removed part stays within FLIP_CAP max|g| elementwise.
# Measured (tools/flip_dump.sh + tools/flip_analysis.py, profiles/r06_flip_rank.txt): every tensor of
# every end-to-end case that leaves the strict bound is brought inside it by ONE rank-1 term.
FLIP_CAP = 5e-4
FLIP_RANK = 2
# summation-magnitude floor, in ulps (u = 2^-24) of M = sum_p |t_p|: a gradient element is a sum over
# samples of terms that each carry a few ulps from the forward / delta chain, and the sum itself
# rounds in a blocked order; 64 u M bounds both (an element without cancellation has M ~ |g|, where
# rtol 1e-3 = ~16,000 u dominates)
MAG_ULPS = 64.0


def strict_bound(ref, cr, d32, mfloor, rtol, atol):
    """rtol |ref| + (atol + d32) max|g_cr| + the summation floor: the elementwise bound of grad_elementwise."""
    return rtol * np.abs(ref) + (atol + d32) * max(np.abs(cr).max(), 1e-30) + mfloor


def flip_rank(D, B, cap, kmax=FLIP_RANK):
    """Smallest k <= kmax such that D minus its best rank-k approximation lies inside B everywhere and
    the removed rank-k part inside cap (2-D D), else None (see FLIP_RANK)."""
    if (np.abs(D) <= B).all():
        return 0
    if D.ndim != 2:  # (a 1-D gradient has no rank structure to name a flip by: no relief)
        return None
    D2, B2 = D, np.broadcast_to(B, D.shape)
    u, s, vt = np.linalg.svd(D2, full_matrices=False)
    for k in range(1, min(kmax, len(s)) + 1):
        Rk = (u[:, :k] * s[:k]) @ vt[:k]
        if (np.abs(D2 - Rk) <= B2).all() and (np.abs(Rk) <= cap).all():
            return k
    return None


def _np(t):
    return t.detach().cpu().numpy().astype(np.float64) if isinstance(t, torch.Tensor) else np.asarray(t, np.float64)


def grad_elementwise(g, cr, f32, what, rel_f32=None, rtol=1e-3, atol=1e-6, flips=False, mag=None):
    """|g - g_cr| <= rtol |g_cr| + (atol + d32) max|g_cr| + MAG_ULPS u M and |g - g_f32| <= the same
    with g_f32 elementwise, d32 = rel_f32 or max |g_f32 - g_cr| / max |g_cr|, M = the element's
    summation magnitude sum_p |t_p| (oracle.ref_points.magnitudes; 0 when not given): the float32
    rounding floor of a sum that cancels.  flips: beyond that bound only by at most FLIP_RANK rank-1
    terms of at most FLIP_CAP max|g| (decision-edge samples, see above)."""
    g, cr, f32 = _np(g), _np(cr), _np(f32)
    mfloor = 0.0 if mag is None else MAG_ULPS * 2.0 ** -24 * np.asarray(mag)
    scale = max(np.abs(cr).max(), 1e-30)
    d32 = float(rel_f32) if rel_f32 is not None else float(np.abs(f32 - cr).max() / scale)
    maybe_dump_grads(what, g, cr, f32, mag, d32, rtol, atol, (atol + d32) * scale + mfloor)
    for ref, tag in ((cr, 'correctly rounded'), (f32, 'float32')):
        B = strict_bound(ref, cr, d32, mfloor, rtol, atol)
        viol = np.abs(g - ref) / B
        print(f'{what} vs {tag} (d32 {d32:.2e}): worst |g - g_ref| / bound = {viol.max():.3f}, '
              f'beyond: {float(np.mean(viol > 1)):.1e}')
        if flips:
            k = flip_rank(g - ref, B, FLIP_CAP * max(np.abs(ref).max(), 1e-30))
            print(f'    flipped-sample terms needed: {k}')
            assert k is not None, f'{what} vs {tag}: the deviation beyond the strict bound is not {FLIP_RANK} rank-1 terms'
        else:
            np.testing.assert_array_less(np.abs(g - ref), B + 1e-45, err_msg=f'{what} vs {tag}')


def grad_layers(named, cr, f32, mags, flips=True):
    """grad_elementwise over a decoder's parameter gradients (named: name -> tensor), each weight held
    together with its bias as one more column ([dW | db]: one flipped sample is one rank-1 term of it)."""
    done = set()
    for k, t in named.items():
        if k in done:
            continue
        if k.endswith('.weight') and k[:-7] + '.bias' in named:
            kb = k[:-7] + '.bias'
            cat = lambda a, b: np.concatenate([_np(a), _np(b)[:, None]], 1)  # noqa: E731
            m = None if mags is None else np.concatenate([np.asarray(mags[k]), np.asarray(mags[kb])[:, None]], 1)
            grad_elementwise(cat(t, named[kb]), cat(cr[k], cr[kb]), cat(f32[k], f32[kb]), k + ' | bias',
                             flips=flips, mag=m)
            done.update((k, kb))
        elif not k.endswith('.bias') or k[:-5] + '.weight' not in named:
            grad_elementwise(t, cr[k], f32[k], k, flips=flips, mag=None if mags is None else mags[k])
            done.add(k)


def mag_arrays(mag, params):
    """Summation magnitudes recorded by RP.magnitudes(), per parameter and for the features."""
    out = {k: RP.magnitude_of(mag, k).numpy() for k in params}
    out['feats'] = mag['feats'].numpy()
    return out


def close(a, b, atol, what, rtol=0.0):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


def grid_setup(pnr, dev):
    g = load_golden('points_c32.npz')
    bound = torch.from_numpy(g['bound'])
    pts = pnr.NeuralPoints.from_grid(torch.from_numpy(g['grid']).to(dev), bound).to(dev)
    dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k[2:]: torch.from_numpy(g[k]) for k in g if k.startswith('w/')})
    return g, pts, dec.to(dev)


def random_cloud(n=3000, seed=3):
    gen = torch.Generator().manual_seed(seed)
    lo = torch.tensor([-0.29, -0.32, -0.35])
    hi = torch.tensor([0.99, 0.64, 0.61])
    xyz = lo + (hi - lo) * torch.rand((n, 3), generator=gen)
    feats = torch.randn((n, 32), generator=gen) * 0.5
    q = xyz[torch.randint(0, n, (4096,), generator=gen)] + 0.03 * torch.randn((4096, 3), generator=gen)
    return xyz, feats, q.double()


def test_gather_trilinear_equals_grid_sample(pnr_mod, dev):
    g, pts, _ = grid_setup(pnr_mod, dev)
    c = pts.gather(torch.from_numpy(g['p']).to(dev))
    close(c, g['c'], 1e-5 * np.abs(g['c']).max(), 'c vs F.grid_sample')


@pytest.mark.parametrize('k', [8, 3])
def test_gather_idw_matches_oracle(pnr_mod, dev, k):
    import ctypes
    lib = pnr_mod.library()
    xyz, feats, q = random_cloud()
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.06, k=k).to(dev)
    P = q.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, k), device=dev, dtype=torch.int32)
    w = torch.empty((P, k), device=dev)
    qd = q.to(dev)
    s, _ = pts.descriptor()
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    assert lib.pnr_point_gather(ctypes.byref(s), qd.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    c_ref, idx_ref, w_ref = RP.point_gather(q, xyz, feats, 'idw', radius=0.06, k=k, return_idx=True)
    assert (idx_ref >= 0).sum() > P, 'test cloud must give neighbours'
    assert (idx_ref < 0).any(), 'and some samples without a full neighbourhood'
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))
    close(w, w_ref, 1e-6, 'weights')
    close(c, c_ref, 1e-5 * c_ref.abs().max().item(), 'c')


def test_gather_many_tasks_per_block(pnr_mod, dev):
    """2M samples: every persistent search block walks many work-list chunks of several
    sub-lists. A random subset of rows is checked against the oracle (rows are independent)."""
    import ctypes
    lib = pnr_mod.library()
    xyz, feats, _ = random_cloud(seed=11)
    gen = torch.Generator().manual_seed(12)
    P = 2_000_000
    q = (xyz[torch.randint(0, xyz.shape[0], (P,), generator=gen)] + 0.08 * torch.randn((P, 3), generator=gen)).double()
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.03, k=8).to(dev)
    s, _ = pts.descriptor()
    qd = q.to(dev)
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    c = torch.full((P, 32), float('nan'), device=dev)
    idx = torch.full((P, 8), -7, device=dev, dtype=torch.int32)
    w = torch.full((P, 8), float('nan'), device=dev)
    assert lib.pnr_point_gather(ctypes.byref(s), qd.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    assert not torch.isnan(c).any() and not torch.isnan(w).any() and not (idx == -7).any(), 'every row written'
    frac = (idx[:, 0] >= 0).float().mean().item()
    assert 0.05 < frac < 0.95, f'a mix of samples with and without neighbours ({frac:.2f})'
    sel = torch.randint(0, P, (4096,), generator=gen)
    c_ref, idx_ref, w_ref = RP.point_gather(q[sel], xyz, feats, 'idw', radius=0.03, k=8, return_idx=True)
    assert np.array_equal(idx[sel.to(dev)].cpu().numpy(), idx_ref.numpy().astype(np.int32))
    close(w[sel.to(dev)], w_ref, 1e-6, 'weights')
    close(c[sel.to(dev)], c_ref, 1e-5 * c_ref.abs().max().item(), 'c')


def test_gather_large_batch_paths(pnr_mod, dev, precision):
    """P = 2,700,000 >= 2,621,440 samples along 45,000 short rays: the paths the S-map and map-points
    batches take -- the forward search in 64-item chunks (csrc/points.hip launch: a.chunk = 64, the
    scalar bucket-header loads) and the backward in 32-row half-wave runs that carry a neighbour shared
    with the previous row of the ray forward (a.run = 32).  Forward: a random row subset against the
    oracle.  Backward: dL/dfeats against a float64 scatter of the gather's own (index, weight) rows (the
    forward check pins those), dL/dp elementwise on a row subset against the float64 gradient."""
    if precision == 'fp32':
        pytest.skip('the gather has no decoder precision: run once')
    import ctypes
    lib = pnr_mod.library()
    xyz, feats, _ = random_cloud(seed=31)
    gen = torch.Generator().manual_seed(32)
    n_rays, S = 45_000, 60
    P = n_rays * S
    assert P >= 64 * 5 * 1024 * 8 and P // 32 >= 2 * 5 * 1024 * 8, 'the large-batch thresholds of points.hip'
    o = xyz[torch.randint(0, xyz.shape[0], (n_rays,), generator=gen)] + 0.02 * torch.randn((n_rays, 3), generator=gen)
    d = torch.nn.functional.normalize(torch.randn((n_rays, 3), generator=gen), dim=1)
    t = torch.linspace(-0.03, 0.03, S)
    q = (o[:, None, :] + t[None, :, None] * d[:, None, :]).reshape(-1, 3).double()
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.03, k=8).to(dev)
    c, idx, w = _gather_c_abi(pnr_mod, dev, pts, q, 8)
    assert not torch.isnan(c).any() and not (idx == -7).any(), 'every row written'
    frac = (idx[:, 0] >= 0).float().mean().item()
    assert 0.05 < frac < 0.95, f'a mix of samples with and without neighbours ({frac:.2f})'
    sel = torch.randint(0, P, (4096,), generator=gen)
    c_ref, idx_ref, w_ref = RP.point_gather(q[sel], xyz, feats, 'idw', radius=0.03, k=8, return_idx=True)
    assert np.array_equal(idx[sel.to(dev)].cpu().numpy(), idx_ref.numpy().astype(np.int32))
    close(w[sel.to(dev)], w_ref, 1e-6, 'weights')
    close(c[sel.to(dev)], c_ref, 1e-5 * c_ref.abs().max().item(), 'c')
    del c
    # backward through the autograd op (pnr_point_gather_backward)
    dgen = torch.Generator(device=dev).manual_seed(33)
    gc = torch.randn((P, 32), generator=dgen, device=dev)
    qd = q.to(dev).requires_grad_(True)
    pts.feats.grad = None
    (pts.gather(qd) * gc).sum().backward()
    torch.cuda.synchronize()
    valid = idx >= 0
    rows = torch.arange(P, device=dev)[:, None].expand(-1, 8)[valid]
    ref = torch.zeros((xyz.shape[0], 32), dtype=torch.float64, device=dev)
    ref.index_add_(0, idx[valid].long(), w[valid].double()[:, None] * gc[rows].double())
    mag = torch.zeros_like(ref).index_add_(0, idx[valid].long(), w[valid].double()[:, None] * gc[rows].double().abs())
    err = (pts.feats.grad.double() - ref).abs()
    bound = 1e-5 * ref.abs() + 2.0 ** -20 * mag + 1e-7 * ref.abs().max()
    print(f'dL/dfeats: worst |g - g64| / bound = {(err / bound).max().item():.3f}')
    assert bool((err <= bound).all()), 'dL/dfeats vs the float64 scatter of the gather rows'
    sub = sel[:1024]
    gsub = gc[sub.to(dev)].cpu()
    qr = q[sub].clone().requires_grad_(True)
    (RP.point_gather(qr, xyz, feats, 'idw', radius=0.03, k=8) * gsub).sum().backward()
    gcr, mag_p = idw_grad_p_cr(q[sub].float().double(), xyz.double(), feats.double(), idx_ref[:1024], gsub.double())
    grad_elementwise(qd.grad[sub.to(dev)], gcr, qr.grad, 'dL/dp (large batch)', mag=mag_p)


def _gather_c_abi(pnr_mod, dev, pts, q, k):
    import ctypes
    lib = pnr_mod.library()
    P = q.shape[0]
    c = torch.full((P, 32), float('nan'), device=dev)
    idx = torch.full((P, k), -7, device=dev, dtype=torch.int32)
    w = torch.full((P, k), float('nan'), device=dev)
    qd = q.to(dev)
    s, _ = pts.descriptor()
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    assert lib.pnr_point_gather(ctypes.byref(s), qd.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    return c, idx, w


def test_gather_dense_cluster_many_candidate_batches(pnr_mod, dev):
    """4,000 points in a 3 cm cube with a 1 cm radius: a probe block holds far more than the
    search's 128-candidate LDS batch, so every segment runs several batches and an odd remainder
    (the paired scan's padding entry)."""
    gen = torch.Generator().manual_seed(21)
    xyz = 0.5 + 0.03 * torch.rand((4000, 3), generator=gen)
    feats = torch.randn((4000, 32), generator=gen) * 0.5
    q = (0.5 + 0.03 * torch.rand((2048, 3), generator=gen) + 0.004 * torch.randn((2048, 3), generator=gen)).double()
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.01, k=8).to(dev)
    c, idx, w = _gather_c_abi(pnr_mod, dev, pts, q, 8)
    c_ref, idx_ref, w_ref = RP.point_gather(q, xyz, feats, 'idw', radius=0.01, k=8, return_idx=True)
    assert (idx_ref[:, 7] >= 0).float().mean() > 0.5, 'most samples keep a full neighbourhood'
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))
    close(w, w_ref, 1e-6, 'weights')
    close(c, c_ref, 1e-5 * c_ref.abs().max().item(), 'c')


def test_gather_lattice_ties_break_by_index(pnr_mod, dev):
    """Exact distance ties: dyadic lattice points (spacing 1/64) under a random index permutation,
    queries at cube centres (8 equidistant corners) and on edge midpoints (2 equidistant), k = 3:
    the kept neighbours are the lowest point indices among the tied ones, as the oracle's stable
    sort on (d2, index) keeps them, whatever order the hash buckets list them in."""
    gen = torch.Generator().manual_seed(22)
    n = 16
    ii = torch.stack(torch.meshgrid(torch.arange(n), torch.arange(n), torch.arange(n), indexing='ij'), -1).reshape(-1, 3)
    perm = torch.randperm(ii.shape[0], generator=gen)
    xyz = (ii[perm].float() / 64.0)
    feats = torch.randn((xyz.shape[0], 32), generator=gen)
    cc = torch.randint(1, n - 2, (1024, 3), generator=gen).double()
    centres = (cc + 0.5) / 64.0
    edges = (cc + torch.tensor([0.5, 0.0, 0.0], dtype=torch.float64)) / 64.0
    q = torch.cat([centres, edges])
    r = 0.0141  # > sqrt(3)/128 (the 8 corners of a centre), < the next shell
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=r, k=3).to(dev)
    c, idx, w = _gather_c_abi(pnr_mod, dev, pts, q, 3)
    c_ref, idx_ref, w_ref = RP.point_gather(q, xyz, feats, 'idw', radius=r, k=3, return_idx=True)
    assert (idx_ref[:1024] >= 0).all(), 'every centre keeps 3 of its 8 tied corners'
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))
    close(w, w_ref, 1e-6, 'weights')
    close(c, c_ref, 1e-5 * c_ref.abs().max().item(), 'c')


def test_gather_backward_matches_oracle(pnr_mod, dev):
    xyz, feats, q = random_cloud(seed=5)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.06, k=8).to(dev)
    gen = torch.Generator().manual_seed(9)
    gc = torch.randn((q.shape[0], 32), generator=gen)
    qd = q.to(dev).requires_grad_(True)
    c = pts.gather(qd)
    (c * gc.to(dev)).sum().backward()
    fr = feats.clone().requires_grad_(True)
    qr = q.clone().requires_grad_(True)
    (RP.point_gather(qr, xyz, fr, 'idw', radius=0.06, k=8) * gc).sum().backward()
    close(pts.feats.grad, fr.grad, 2e-5 * fr.grad.abs().max().item(), 'dL/dfeats')
    # dL/dp elementwise at rtol 1e-3 against the correctly-rounded gradient (float64 weights, sums and
    # backward over the same neighbour sets, the inputs rounded to float32 as the kernels read them),
    # with the float32 summation floor 64 u M, M = sum_j |dw_j/dp| (|g_j| + sum_k wn_k |g_k|) / W
    _, idx, _ = _gather_c_abi(pnr_mod, dev, pts, q, 8)
    _, idx_ref, _ = RP.point_gather(q, xyz, feats, 'idw', radius=0.06, k=8, return_idx=True)
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))
    gcr, mag = idw_grad_p_cr(q.float().double(), xyz.double(), feats.double(), idx_ref, gc.double())
    grad_elementwise(qd.grad, gcr, qr.grad, 'dL/dp', mag=mag)


def idw_grad_p_cr(p, xyz, feats, idx, gc, eps=1e-6):
    """d(sum c(p) . gc)/dp of the IDW gather (oracle.ref_points.neighbour_weights / point_gather) in
    float64 on a fixed neighbour set, and each element's summation magnitude M."""
    p = p.clone().requires_grad_(True)
    valid = idx >= 0
    ic = idx.clamp(min=0)
    dl = p[:, None, :] - xyz[ic]
    d2 = (dl * dl).sum(-1)
    d = torch.sqrt(torch.clamp(d2, min=eps * eps * 0.25))
    w = torch.where(valid, 1.0 / torch.clamp(d, min=eps), torch.zeros_like(d))
    W = w.sum(1)
    W = torch.where(W > 0, W, torch.ones_like(W))
    wn = w / W[:, None]
    fk = feats[ic]
    c = (wn[:, :, None] * fk).sum(1)
    (c * gc).sum().backward()
    with torch.no_grad():
        gabs = torch.where(valid, (fk.abs() * gc.abs()[:, None, :]).sum(-1), torch.zeros_like(d))  # |g_j|
        dw = torch.where(valid, 1.0 / torch.clamp(d, min=eps) ** 2, torch.zeros_like(d))[..., None] * \
            (dl.abs() / torch.clamp(d, min=eps)[..., None])                                      # |dw_j/dp|
        a = (gabs + (wn * gabs).sum(1, keepdim=True)) / W[:, None]
        mag = (dw * a[..., None]).sum(1)
    return p.grad.detach(), mag.numpy()


def test_decoder_c32_matches_reference(pnr_mod, dev):
    """pnr.MLP(c_dim=32) on lattice points == the reference MLP(c_dim=32) with F.grid_sample."""
    g, pts, dec = grid_setup(pnr_mod, dev)
    p = torch.from_numpy(g['p']).to(dev).requires_grad_(True)
    raw = dec(p, c_grid={'points_color': pts})
    close(raw, g['raw'], 2e-5 * np.abs(g['raw']).max(), 'raw')
    (raw * torch.from_numpy(g['g_raw']).to(dev)).sum().backward()
    CR = load_golden('grads_cr.npz')
    for k, t in dec.named_parameters():
        grad_elementwise(t.grad, CR[f'pts/grad/{k}'], g['grad/' + k], k, CR[f'golden_vs_cr/pts/{k}'])
    ref = RP.grid_features(torch.from_numpy(g['grad_grid'])).numpy()
    grad_elementwise(pts.feats.grad, CR['pts/grad_feats'], ref, 'dL/dgrid', CR['golden_vs_cr/pts/grad_feats'])
    grad_elementwise(p.grad, CR['pts/grad_p'], g['grad_p'], 'dL/dp', CR['golden_vs_cr/pts/grad_p'])


def test_fc_weight_scale_covers_every_weight(pnr_mod, dev):
    """The f16 scale of each fc_c weight (k_wscale) must come from ALL its entries: the largest one
    sits alone at the last flat index, 1000x the rest. A scale from a partial scan overflows f16
    there, so the split path must still match the fp32 path."""
    g, pts, dec = grid_setup(pnr_mod, dev)
    with torch.no_grad():
        for i in range(4):
            wt = getattr(dec.fc_c[i], 'weight')
            wt.mul_(1e-3)
            wt.view(-1)[-1] = 0.5
    p = torch.from_numpy(g['p']).to(dev)
    with torch.no_grad():
        raw = dec(p, c_grid={'points_color': pts}).clone()
        dec.precision = 'fp32'
        ref = dec(p, c_grid={'points_color': pts})
    assert torch.isfinite(raw).all()
    close(raw, ref, 2e-5 * ref.abs().max().item(), 'raw vs the fp32 path')


def surface_cloud(dev, seed=4):
    """Neural points scattered around the golden pose-1000 surface (gt = rendered depth)."""
    r = load_golden('render.npz')
    ro = torch.from_numpy(r['p2_gt/rays_o'])
    rd = torch.from_numpy(r['p2_gt/rays_d'])
    gt = torch.from_numpy(r['p2_gt/gt_depth'])
    gen = torch.Generator().manual_seed(seed)
    surf = ro + rd * gt[:, None]
    xyz = (surf.repeat(4, 1) + 0.01 * torch.randn((4 * surf.shape[0], 3), generator=gen)).float()
    feats = torch.randn((xyz.shape[0], 32), generator=gen) * 0.5
    return ro, rd, gt, xyz, feats


def make_renderer(pnr, scene_bound):
    import types
    slam = types.SimpleNamespace(bound=scene_bound, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    return pnr.Renderer(pnr.ROOM0_CFG, None, slam)


@pytest.mark.parametrize('mode', ['idw', 'trilinear'])
def test_render_with_points_matches_oracle(pnr_mod, dev, mode, precision):
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev)
    n = 256
    ro, rd, gt = ro[:n], rd[:n], gt[:n]
    base = golden_params('trained')
    params = RP.init_fc_c(base, seed=1)
    kw = dict(mode=mode, k=8, radius=0.04, eps=1e-6, spacing=[0.03, 0.03, 0.03])
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), **kw).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    r = make_renderer(pnr_mod, bound)
    c = {'points_color': pts}
    d, v, col = r.render_batch_ray(c, dec, rd.to(dev), ro.to(dev), dev, 'color', gt_depth=gt.to(dev))
    gc_ = torch.randn(col.shape, generator=torch.Generator().manual_seed(2), dtype=col.dtype).to(dev)  # seeded: the flip count is a function of it
    loss = (d - gt.to(dev).double()).abs().sum() + 0.05 * (col * gc_).sum() + 1e-3 * v.sum()
    loss.backward()

    refs = {}
    for cr_ in (False, True):
        ref_p = {k: t.clone().requires_grad_(True) for k, t in params.items()}
        fr = feats.clone().requires_grad_(True)
        pdict = dict(xyz=xyz, feats=fr, mode=mode, radius=0.04, spacing=[0.03] * 3, k=8, eps=1e-6)
        ev = lambda q: RP.eval_points_c(ref_p, q, bound, pdict, cr=cr_)  # noqa: E731
        with RP.magnitudes() as mag:
            dr, vr, cr = RR.render_batch_ray(ref_p, rd, ro, bound, gt_depth=gt, eval_fn=ev)
            lr = (dr - gt.double()).abs().sum() + 0.05 * (cr * gc_.cpu()).sum() + 1e-3 * vr.sum()
            lr.backward()
        refs[cr_] = ({k: t.grad for k, t in ref_p.items()}, fr.grad)
        if not cr_:
            mags = mag_arrays(mag, params)
            close(d, dr, 0, 'depth', rtol=1e-4)
            close(col, cr, 2e-5, 'rgb', rtol=1e-4)
            close(v, vr, 1e-8, 'var', rtol=2e-3)
    # (round 5 allowed 2% of the fc_c weight elements here (fp32, trilinear): one flipped sample's rank-1
    # term, which FLIP_RANK now names as such)
    grad_layers({k: t.grad for k, t in dec.named_parameters()}, refs[True][0], refs[False][0], mags)
    grad_elementwise(pts.feats.grad, refs[True][1], refs[False][1], 'dL/dfeats', flips=True, mag=mags['feats'])


def test_render_with_small_features_matches_oracle(pnr_mod, dev):
    """Features of the reference's fine-grid magnitude (std 1e-4, decoder.py's grid init): the f16x3
    path splits them under a power-of-two scale of their own (forward: per wave; dWc: per-wave
    running scale), so dWc and dL/dfeats keep the elementwise fp32-class bound. Unscaled, the lo
    parts of 1e-4 values fall into the f16 subnormals and keep ~11 bits."""
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev, seed=7)
    feats = feats * 2e-4
    n = 256
    # (gt 2% beyond the render: with features this small the render is the golden depth to ~1e-7, and
    # the depth loss's sign(depth - gt) would hinge on rounding)
    ro, rd, gt = ro[:n], rd[:n], gt[:n] * 1.02
    params = RP.init_fc_c(golden_params('trained'), seed=4)
    kw = dict(mode='idw', k=8, radius=0.04, eps=1e-6)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), **kw).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    r = make_renderer(pnr_mod, bound)
    d, v, col = r.render_batch_ray({'points_color': pts}, dec, rd.to(dev), ro.to(dev), dev, 'color',
                                   gt_depth=gt.to(dev))
    gc_ = torch.randn(col.shape, generator=torch.Generator().manual_seed(2))
    ((d - gt.to(dev).double()).abs().sum() + 0.05 * (col * gc_.to(dev)).sum()).backward()
    refs = {}
    for cr_ in (False, True):
        ref_p = {k: t.clone().requires_grad_(True) for k, t in params.items()}
        fr = feats.clone().requires_grad_(True)
        pdict = dict(xyz=xyz, feats=fr, **kw)
        ev = lambda q: RP.eval_points_c(ref_p, q, bound, pdict, cr=cr_)  # noqa: E731
        with RP.magnitudes() as mag:
            dr, vr, cr = RR.render_batch_ray(ref_p, rd, ro, bound, gt_depth=gt, eval_fn=ev)
            ((dr - gt.double()).abs().sum() + 0.05 * (cr * gc_).sum()).backward()
        refs[cr_] = ({k: t.grad for k, t in ref_p.items()}, fr.grad)
        if not cr_:
            mags = mag_arrays(mag, params)
            close(d, dr, 0, 'depth', rtol=1e-4)
            close(col, cr, 2e-5, 'rgb', rtol=1e-4)
    grad_layers({k: t.grad for k, t in dec.named_parameters()}, refs[True][0], refs[False][0], mags)
    grad_elementwise(pts.feats.grad, refs[True][1], refs[False][1], 'dL/dfeats', flips=True, mag=mags['feats'])


def test_tracking_ray_grads_with_points(pnr_mod, dev):
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev, seed=6)
    n = 128
    ro, rd, gt = ro[:n], rd[:n], gt[:n]
    params = RP.init_fc_c(golden_params('trained'), seed=2)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.04, k=8).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev).requires_grad_(False)
    pts.feats.requires_grad_(False)
    r = make_renderer(pnr_mod, bound)
    rod = ro.to(dev).requires_grad_(True)
    rdd = rd.to(dev).requires_grad_(True)
    d, v, col = r.render_batch_ray({'points_color': pts}, dec, rdd, rod, dev, 'color', gt_depth=gt.to(dev))
    ((d - gt.to(dev).double()).abs() / torch.sqrt(v.detach() + 1e-10)).sum().backward()
    refs = {}
    for cr_ in (False, True):
        ror = ro.clone().requires_grad_(True)
        rdr = rd.clone().requires_grad_(True)
        pdict = dict(xyz=xyz, feats=feats, mode='idw', radius=0.04, k=8, eps=1e-6)
        ev = lambda q: RP.eval_points_c(params, q, bound, pdict, cr=cr_)  # noqa: E731
        dr, vr, _ = RR.render_batch_ray(params, rdr, ror, bound, gt_depth=gt, eval_fn=ev)
        ((dr - gt.double()).abs() / torch.sqrt(vr.detach() + 1e-10)).sum().backward()
        refs[cr_] = (ror.grad, rdr.grad)
    grad_elementwise(rod.grad, refs[True][0], refs[False][0], 'dL/drays_o', flips=True)
    grad_elementwise(rdd.grad, refs[True][1], refs[False][1], 'dL/drays_d', flips=True)


def test_regulation_with_points(pnr_mod, dev):
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev, seed=8)
    n = 128
    ro, rd, gt = ro[:n], rd[:n], gt[:n]
    params = RP.init_fc_c(golden_params('trained'), seed=3)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.05, k=8).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    t_rand = torch.rand((n, 32), generator=torch.Generator().manual_seed(1))
    r = make_renderer(pnr_mod, bound)
    s = r.regulation({'points_color': pts}, dec, rd.to(dev), ro.to(dev), gt.to(dev), dev, t_rand=t_rand.to(dev))
    s.abs().sum().backward()
    refs = {}
    for cr_ in (False, True):
        ref_p = {k: t.clone().requires_grad_(True) for k, t in params.items()}
        fr = feats.clone().requires_grad_(True)
        pdict = dict(xyz=xyz, feats=fr, mode='idw', radius=0.05, k=8, eps=1e-6)
        with RP.magnitudes() as mag:
            sr = RR.regulation(ref_p, rd, ro, gt, bound, t_rand=t_rand,
                               eval_fn=lambda q: RP.eval_points_c(ref_p, q, bound, pdict, cr=cr_))
            sr.abs().sum().backward()
        refs[cr_] = ({k: t.grad for k, t in ref_p.items()}, fr.grad)
        if not cr_:
            mags = mag_arrays(mag, params)
            close(s, sr, 2e-5 * sr.abs().max().item(), 'sigma')
    grad_elementwise(pts.feats.grad, refs[True][1], refs[False][1], 'dL/dfeats', flips=True, mag=mags['feats'])
    grad_layers({k: t.grad for k, t in dec.named_parameters()}, refs[True][0], refs[False][0], mags)


def test_gather_f16_features_equal_rounded_fp32(pnr_mod, dev):
    """feat_dtype='float16' (pnr_points.feat_half, the C5 budget): the gather reads an f16 copy
    of the fp32 features and sums in fp32, so it equals the fp32 gather over the f16-rounded
    features -- c bit for bit, dL/dfeats (independent of the features) and dL/dp to fp32 atomic
    ordering (1e-6 of max)."""
    xyz, feats, q = random_cloud(seed=6)
    kw = dict(mode='idw', radius=0.06, k=8)
    p16 = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), feat_dtype='float16', **kw).to(dev)
    p32 = pnr_mod.NeuralPoints(xyz.to(dev), feats.half().float().to(dev), **kw).to(dev)
    gc = torch.randn((q.shape[0], 32), generator=torch.Generator().manual_seed(2)).to(dev)
    outs = []
    for pts in (p16, p32):
        qd = q.to(dev).requires_grad_(True)
        c = pts.gather(qd)
        (c * gc).sum().backward()
        outs.append((c.detach(), pts.feats.grad.clone(), qd.grad.clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert (outs[0][0] != 0).any()
    close(outs[0][1], outs[1][1], 1e-6 * outs[1][1].abs().max().item(), 'dL/dfeats')
    close(outs[0][2], outs[1][2], 1e-6 * outs[1][2].abs().max().item(), 'dL/dp')
    # the f16 copy follows in-place updates of the fp32 master
    with torch.no_grad():
        p16.feats.mul_(0.5)
        p32.feats.copy_((feats * 0.5).half().float().to(dev))
    assert torch.equal(p16.gather(q.to(dev)), p32.gather(q.to(dev)))


def test_map_step_with_f16_features(pnr_mod, dev):
    """A mapping step with f16 features: loss equal to the fp32-feature step on the rounded
    features; Adam updates the fp32 master and the next gather sees the new f16 copy."""
    from pnr.mapping import MapStep
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev)
    n = 512
    ro, rd, gt = ro[:n].to(dev), rd[:n].to(dev), gt[:n].to(dev)
    col = torch.rand((n, 3), generator=torch.Generator().manual_seed(1)).to(dev)
    t_rand = torch.rand((n, 32), generator=torch.Generator().manual_seed(2)).to(dev)
    params = RP.init_fc_c(golden_params('trained'), seed=1)
    losses = []
    for fd, f0 in (('float16', feats), ('float32', feats.half().float())):
        pts = pnr_mod.NeuralPoints(xyz.to(dev), f0.to(dev), mode='idw', radius=0.04, k=8, feat_dtype=fd).to(dev)
        dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
        dec.load_state_dict({k: v.clone() for k, v in params.items()})
        ms = MapStep(make_renderer(pnr_mod, bound), dec.to(dev), points=pts, feat_lr=1e-2)
        l1 = float(ms(ro, rd, gt, col, t_rand))
        l2 = float(ms(ro, rd, gt, col, t_rand))
        losses.append((l1, l2))
        if fd == 'float16':
            assert torch.equal(pts._feats_for_gather(), pts.feats.detach().half())
    assert abs(losses[0][0] - losses[1][0]) <= 1e-5 * abs(losses[1][0])
    assert losses[0][1] != losses[0][0]


def test_map_step_sharded_features_single_rank(pnr_mod, dev):
    """MapStep(ddp=DataParallel(shard_points=True)) at world size 1 takes the sharded code path
    (owned-range Adam segment, reduce-scatter / all-gather no-ops) and must equal the plain step bit
    for bit (the feature backward is an exact int64 sum since ABI 10: no run-to-run spread)."""
    from pnr.mapping import MapStep
    from pnr.dist import DataParallel
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    ro, rd, gt, xyz, feats = surface_cloud(dev)
    n = 256
    ro, rd, gt = ro[:n].to(dev), rd[:n].to(dev), gt[:n].to(dev)
    col = torch.rand((n, 3), generator=torch.Generator().manual_seed(1)).to(dev)
    t_rand = torch.rand((n, 32), generator=torch.Generator().manual_seed(2)).to(dev)
    params = RP.init_fc_c(golden_params('trained'), seed=1)
    out = []
    for ddp in (None, DataParallel(shard_points=True)):
        pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.04, k=8).to(dev)
        dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
        dec.load_state_dict({k: v.clone() for k, v in params.items()})
        ms = MapStep(make_renderer(pnr_mod, bound), dec.to(dev), points=pts, feat_lr=1e-2, ddp=ddp)
        assert ms.shard == (ddp is not None)
        losses = [float(ms(ro, rd, gt, col, t_rand)) for _ in range(2)]
        out.append((losses, ms.flat.data.clone(), ms.opt.segments))
    assert out[0][2] == out[1][2]
    assert out[0][0] == out[1][0]
    assert torch.equal(out[1][1], out[0][1])


def test_track_step_with_points_leaves_features_alone(pnr_mod, dev):
    """The Tracker optimises the camera only (src/Tracker.py:870-874): a TrackStep over a
    neural-point decoder produces the camera gradient and leaves the point features' and the
    decoder's .grad untouched (no feature atomics, no fc_c weight-gradient GEMMs)."""
    scene = load_golden('scene.npz')
    bound = torch.from_numpy(scene['bound'])
    _, _, _, xyz, feats = surface_cloud(dev, seed=9)
    params = RP.init_fc_c(golden_params('trained'), seed=4)
    pts = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.04, k=8).to(dev)
    dec = pnr_mod.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    import types
    H, W = 68, 120
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=60., fy=60., cx=59.5, cy=33.5)
    r = pnr_mod.Renderer(pnr_mod.ROOM0_CFG, None, slam)
    c2w = torch.from_numpy(scene['poses'][2]).float()
    gd = torch.full((H, W), 0.3, device=dev)
    gc = torch.rand((H, W, 3), generator=torch.Generator().manual_seed(3)).to(dev)
    step = pnr_mod.TrackStep(r, dec, c={'points_color': pts}, ignore_edge_W=10, ignore_edge_H=10)
    ct = pnr_mod.get_tensor_from_camera(c2w).to(dev).requires_grad_(True)
    loss = step.loss(ct, gc, gd, 0)
    loss.backward()
    assert ct.grad is not None and torch.isfinite(ct.grad).all() and ct.grad.abs().sum() > 0
    assert pts.feats.grad is None
    assert all(p.grad is None for p in dec.parameters())
    assert pts.feats.requires_grad and all(p.requires_grad for p in dec.parameters())
