"""Host-side logic of the pnr mirror that needs no GPU: config loading, pose helpers, bound,
linspace tables, decoder construction / state_dict compatibility, CPU-tensor refusal."""
import os
import sys
import types

import numpy as np
import pytest
import torch

from conftest import REPO, load_golden, golden_params

sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
import pnr  # noqa: E402
from pnr import renderer as R  # noqa: E402
from oracle import ref_render as ref  # noqa: E402


def test_linspace_tables_match_torch():
    for n in (1, 2, 12, 32, 44, 64):
        t = R._linspace_table(n)
        assert np.array_equal(np.array(t[:n], dtype=np.float32), torch.linspace(0., 1., n).numpy())


def test_scaled_bound_matches_golden():
    s = load_golden('scene.npz')
    b = pnr.scaled_bound(s['bound_cfg'], float(s['scale']), float(s['bound_divisible']))
    assert torch.equal(b, torch.from_numpy(s['bound']))


def test_pose_helpers_roundtrip():
    s = load_golden('scene.npz')
    for c2w in s['poses']:
        t = pnr.get_tensor_from_camera(torch.from_numpy(c2w))
        RT = pnr.get_camera_from_tensor(t)
        np.testing.assert_allclose(RT.numpy(), c2w[:3, :4], atol=2e-6)
        np.testing.assert_allclose(RT.numpy(), ref.camera_from_tensor(t).numpy(), atol=0)


def test_decoder_state_dict_compat():
    params = golden_params('trained')
    dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4, pos_embedding_method='fourier')
    assert set(dec.state_dict().keys()) == set(params.keys())
    dec.load_state_dict(params)
    assert sum(p.numel() for p in dec.parameters()) == 222747
    import copy
    dec2 = copy.deepcopy(dec)
    assert all(torch.equal(a, b) for a, b in zip(dec.parameters(), dec2.parameters()))
    dec.share_memory()
    with pytest.raises(NotImplementedError):
        pnr.MLP(c_dim=64, color=True, skips=[], n_blocks=4, hidden_size=256)
    with pytest.raises(NotImplementedError):
        pnr.MLP(c_dim=32, color=True, skips=[2], n_blocks=4, hidden_size=256)
    # the neural-point decoder: 8 extra fc_c tensors, deepcopy drops the device caches
    d32 = pnr.MLP(c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    assert sum(p.numel() for p in d32.parameters()) == 222747 + 4 * (32 * 256 + 256)
    assert [k for k in d32.state_dict() if k.startswith('fc_c')] == list(pnr.FC_ORDER)
    copy.deepcopy(d32)


def test_neural_points_host_config():
    xyz = torch.rand(100, 3)
    p = pnr.NeuralPoints(xyz, mode='idw', radius=0.05, k=4)
    assert p.feats.shape == (100, 32) and p.cell >= 0.05 and p.table_bits == 10
    assert all(o < float(xyz[:, i].min()) for i, o in enumerate(p.origin))
    with pytest.raises(ValueError):
        pnr.NeuralPoints(xyz, k=9)
    with pytest.raises(ValueError):
        pnr.NeuralPoints(xyz, radius=0.05, cell=0.01)
    grid = torch.randn(1, 32, 3, 4, 5)
    q = pnr.NeuralPoints.from_grid(grid, torch.tensor([[0., 1.], [0., 1.5], [0., 1.]]))
    assert q.mode == 'trilinear' and q.xyz.shape == (60, 3)
    np.testing.assert_allclose(q.spacing, [0.25, 0.5, 0.5], rtol=1e-6)
    # row (d,h,w) = (2,3,4) is the far corner and carries grid[0,:,2,3,4]
    assert torch.equal(q.feats[59], grid[0, :, 2, 3, 4]) and torch.allclose(q.xyz[59], torch.tensor([1., 1.5, 1.]))
    dec = pnr.MLP(name='color', c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    from pnr.points import find_points
    assert find_points({'points_color': q}, dec) is q and find_points({}, pnr.get_model(pnr.ROOM0_CFG, nice=False)) is None
    with pytest.raises(ValueError):
        find_points({}, dec)


def test_get_model_from_cfg():
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    assert isinstance(dec, pnr.MLP)
    with pytest.raises(NotImplementedError):
        pnr.get_model(pnr.ROOM0_CFG, nice=True)


def test_load_config_inherit(tmp_path):
    (tmp_path / 'base.yaml').write_text('rendering:\n  N_samples: 32\n  N_importance: 12\nscale: 1\n')
    (tmp_path / 'mid.yaml').write_text(f'inherit_from: {tmp_path}/base.yaml\nscale: 0.1\n')
    (tmp_path / 'leaf.yaml').write_text(f'inherit_from: {tmp_path}/mid.yaml\nrendering:\n  N_samples: 16\n')
    cfg = pnr.load_config(str(tmp_path / 'leaf.yaml'))
    assert cfg['scale'] == 0.1 and cfg['rendering'] == {'N_samples': 16, 'N_importance': 12}


def test_renderer_refuses_cpu_tensors():
    s = load_golden('scene.npz')
    slam = types.SimpleNamespace(bound=torch.from_numpy(s['bound']), H=680, W=1200, fx=600., fy=600., cx=599.5,
                                 cy=339.5)
    r = pnr.Renderer(pnr.ROOM0_CFG, None, slam)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    with pytest.raises(RuntimeError, match='HIP path only'):
        r.render_batch_ray({}, dec, torch.zeros(4, 3), torch.zeros(4, 3), 'cpu', 'color')
    with pytest.raises(RuntimeError, match='HIP path only'):
        dec(torch.zeros(1, 5, 3))
    prm = r.params()
    assert prm.n_samples == 32 and prm.n_importance == 12 and list(prm.bound)[:2] == [float(s['bound'][0, 0]),
                                                                                       float(s['bound'][0, 1])]


def test_renderer_rejects_out_of_scope_cfg():
    s = load_golden('scene.npz')
    slam = types.SimpleNamespace(bound=torch.from_numpy(s['bound']), H=1, W=1, fx=1., fy=1., cx=0., cy=0.)
    import copy
    cfg = copy.deepcopy(pnr.ROOM0_CFG)
    cfg['rendering']['N_surface'] = 4
    with pytest.raises(NotImplementedError):
        pnr.Renderer(cfg, None, slam)


def test_fourier_sincos_reduction_matches_libm():
    """The sin / cos of the split-precision kernels (csrc/dev_common.h fourier_sc): k = rint(2x/pi),
    r = x - k pi/2 by three fma steps with pi/2 = C1 + C2 + C3 (fp32 parts), minimax polynomials on
    [-pi/4, pi/4].  Emulated here in exact rational arithmetic per fp32 operation; the max abs error
    over the Fourier argument range must stay at the fp32 libm level (~1 ulp of 1)."""
    from fractions import Fraction
    f32 = np.float32

    def fma(a, b, c):
        return f32(float(Fraction(float(a)) * Fraction(float(b)) + Fraction(float(c))))

    C1, C2, C3 = f32(1.5707963705062866), f32(-4.3711388286737929e-08), f32(-1.7151245100058819e-15)
    # C1 + C2 + C3 is pi/2 to ~1e-22
    assert abs(float(C1) + float(C2) + float(C3) - np.pi / 2) < 1e-15

    def sc(x, cos):
        x = f32(x)
        k = f32(np.rint(f32(x * f32(0.636619772367581343))))
        r = fma(-k, C1, x)
        r = fma(-k, C2, r)
        r = fma(-k, C3, r)
        z = f32(r * r)
        sn = fma(fma(fma(f32(-1.9515295891e-4), z, f32(8.3321608736e-3)), z, f32(-1.6666654611e-1)), f32(z * r), r)
        cs = fma(fma(fma(fma(f32(2.443315711809948e-5), z, f32(-1.388731625493765e-3)), z,
                         f32(4.166664568298827e-2)), z, f32(-0.5)), z, f32(1.0))
        q = (int(k) + (1 if cos else 0)) & 3
        v = cs if q & 1 else sn
        return -v if q & 2 else v

    rng = np.random.default_rng(0)
    xs = np.concatenate([rng.uniform(-300, 300, 3000), rng.uniform(-3000, 3000, 500),
                         rng.uniform(-1, 1, 300)]).astype(np.float32)
    es = max(abs(float(sc(x, False)) - np.sin(np.float64(x))) for x in xs)
    ec = max(abs(float(sc(x, True)) - np.cos(np.float64(x))) for x in xs)
    assert es < 1e-7 and ec < 1e-7, (es, ec)


def test_random_select_keyframe_window():
    """src/common.py:66-71: k distinct indices of 0..l-1 (min(l, k) of them), numpy's RNG stream."""
    import numpy as np
    from pnr.common import random_select
    np.random.seed(3)
    a = random_select(10, 4)
    np.random.seed(3)
    assert a == list(np.random.permutation(np.array(range(10)))[:4])
    assert len(set(a)) == 4 and all(0 <= x < 10 for x in a)
    assert sorted(random_select(3, 8)) == [0, 1, 2]
