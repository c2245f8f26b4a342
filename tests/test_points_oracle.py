"""The neural-point oracle (oracle/ref_points.py) against the reference's MLP(c_dim=32) with a
feature grid (tests/golden/points_c32.npz, made by tests/golden/make_golden_points.py).

Neural points on the grid vertices + trilinear weights must reproduce MLP.sample_grid_feature
(src/conv_onet/models/decoder.py:168-175, F.grid_sample align_corners=True) on interior samples,
and the whole decoder forward/backward with the fc_c injection (decoder.py:196-197).
Tolerances: c, raw: 1e-5 * max; grads 1e-4 * max (float32, different summation order).
"""
import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import ref_points as RP


@pytest.fixture(scope='module')
def g():
    return load_golden('points_c32.npz')


def _setup(g):
    bound = torch.from_numpy(g['bound'])
    grid = torch.from_numpy(g['grid'])
    D, H, W = grid.shape[2:]
    xyz, sp = RP.grid_vertices(bound, D, H, W)
    feats = RP.grid_features(grid).clone().requires_grad_(True)
    params = {k[2:]: torch.from_numpy(g[k]).clone().requires_grad_(True) for k in g if k.startswith('w/')}
    return xyz, sp, feats, params


def test_trilinear_gather_equals_grid_sample(g):
    xyz, sp, feats, _ = _setup(g)
    c, idx, wn = RP.point_gather(torch.from_numpy(g['p']), xyz, feats.detach(), 'trilinear', spacing=sp, k=8,
                                 return_idx=True)
    assert (idx >= 0).all(), 'every interior sample has its 8 cell corners'
    np.testing.assert_allclose(c.numpy(), g['c'], atol=1e-5 * np.abs(g['c']).max(), rtol=0)
    np.testing.assert_allclose(wn.sum(1).numpy(), 1.0, atol=1e-6)


def test_decoder_c32_forward_backward(g):
    xyz, sp, feats, params = _setup(g)
    p = torch.from_numpy(g['p']).requires_grad_(True)
    c = RP.point_gather(p, xyz, feats, 'trilinear', spacing=sp, k=8)
    raw = RP.mlp_forward_c(params, p, c)
    np.testing.assert_allclose(raw.detach().numpy(), g['raw'], atol=1e-5 * np.abs(g['raw']).max(), rtol=0)
    (raw * torch.from_numpy(g['g_raw'])).sum().backward()
    for k, t in params.items():
        ref = g['grad/' + k]
        np.testing.assert_allclose(t.grad.numpy(), ref, atol=1e-4 * max(np.abs(ref).max(), 1e-12), rtol=0, err_msg=k)
    ref = RP.grid_features(torch.from_numpy(g['grad_grid'])).numpy()
    np.testing.assert_allclose(feats.grad.numpy(), ref, atol=1e-4 * np.abs(ref).max(), rtol=0)
    np.testing.assert_allclose(p.grad.numpy(), g['grad_p'], atol=1e-4 * np.abs(g['grad_p']).max(), rtol=0)


def test_reference_init_order(g):
    """pnr.MLP(c_dim=32) consumes the RNG like the reference (fc_c first, decoder.py:122-125):
    the same seed gives bit-identical initial weights."""
    import pnr
    torch.manual_seed(7)
    dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256,
                  pos_embedding_method='fourier')
    for k, v in dec.state_dict().items():
        assert np.array_equal(v.numpy(), g['w/' + k]), k


def test_idw_selection_and_weights():
    """Hand-checkable IDW case: k nearest inside the radius, ties broken by index, 1/max(d, eps)."""
    xyz = torch.tensor([[0., 0., 0.], [0.1, 0., 0.], [-0.1, 0., 0.], [0., 0.3, 0.], [0., 0., 0.05]])
    feats = torch.eye(5, 32)
    p = torch.tensor([[0., 0., 0.], [0.05, 0., 0.], [1., 1., 1.]], dtype=torch.float64)
    c, idx, wn = RP.point_gather(p, xyz, feats, 'idw', radius=0.2, k=3, eps=1e-6, return_idx=True)
    # sample 0: d = 0 (w = 1e6), 0.05, then a tie at 0.1 between points 1 and 2 -> index 1 first
    assert idx[0].tolist() == [0, 4, 1]
    # sample 1: d(1) = 0.05, d(0) = 0.05 -> tie, index 0 first; then point 4 at 0.0707
    assert idx[1].tolist() == [0, 1, 4]
    assert idx[2].tolist() == [-1, -1, -1] and float(c[2].abs().sum()) == 0.0
    w = torch.tensor([1e6, 1 / 0.05, 1 / 0.1])
    np.testing.assert_allclose(wn[0].numpy(), (w / w.sum()).numpy(), rtol=1e-6)
