"""Edge cases of the HIP path against the oracle: sample counts at the ABI maximum
(N_samples + N_importance = 64) and with no importance pass, a single ray, empty ray batches,
empty point queries, and an empty neural-point cloud.  Tolerances as tests/test_gpu_parity.py."""
import copy
import types

import numpy as np
import pytest
import torch

from conftest import load_golden, golden_params
from test_gpu_parity import make_decoder, close, precision  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


def _renderer(pnr, scene, n_samples=32, n_importance=12):
    cfg = copy.deepcopy(pnr.ROOM0_CFG)
    cfg['rendering']['N_samples'] = n_samples
    cfg['rendering']['N_importance'] = n_importance
    slam = types.SimpleNamespace(bound=scene['bound_t'], H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    return pnr.Renderer(cfg, None, slam)


@pytest.mark.parametrize('ns,ni', [(48, 16), (52, 12), (32, 0), (3, 1)])
def test_sample_counts_vs_oracle(dev, scene, ns, ni):
    """Renderer.py:157-201 at other (N_samples, N_importance), up to the 64-sample maximum."""
    import pnr
    from oracle import ref_render as ref
    g = load_golden('render.npz')
    params = golden_params('trained')
    dec = make_decoder(pnr, params, dev)
    r = _renderer(pnr, scene, ns, ni)
    ro = torch.from_numpy(g['p1_gt/rays_o'][:256].copy())
    rd = torch.from_numpy(g['p1_gt/rays_d'][:256].copy())
    gt = torch.from_numpy(g['p1_gt/gt_depth'][:256].copy())
    for gd in (None, gt):
        with torch.no_grad():
            d, v, c = r.render_batch_ray({}, dec, rd.to(dev), ro.to(dev), dev, 'color',
                                         gt_depth=None if gd is None else gd.to(dev))
        dr, vr, cr = ref.render_batch_ray(params, rd, ro, scene['bound_t'], n_samples=ns, n_importance=ni,
                                          gt_depth=gd)
        close(d, dr, 1e-4, 1e-9, f'depth {ns}+{ni}')
        close(c, cr, 1e-4, 2e-5, f'rgb {ns}+{ni}')
        close(v, vr, 2e-3, 1e-8, f'var {ns}+{ni}')


def test_more_than_64_samples_refused(scene):
    import pnr
    with pytest.raises(ValueError):
        _renderer(pnr, scene, 56, 12)


def test_single_ray_and_grads(dev, scene):
    import pnr
    from oracle import ref_render as ref
    g = load_golden('render.npz')
    params = golden_params('trained')
    dec = make_decoder(pnr, params, dev)
    r = _renderer(pnr, scene)
    ro = torch.from_numpy(g['p0_gt/rays_o'][5:6].copy())
    rd = torch.from_numpy(g['p0_gt/rays_d'][5:6].copy())
    gt = torch.from_numpy(g['p0_gt/gt_depth'][5:6].copy())
    d, v, c = r.render_batch_ray({}, dec, rd.to(dev), ro.to(dev), dev, 'color', gt_depth=gt.to(dev))
    (d.sum() + c.sum()).backward()
    rp = {k: t.clone().requires_grad_(True) for k, t in params.items()}
    dr, vr, cr = ref.render_batch_ray(rp, rd, ro, scene['bound_t'], gt_depth=gt)
    (dr.sum() + cr.sum()).backward()
    close(d, dr, 1e-4, 1e-9, 'depth')
    close(c, cr, 1e-4, 2e-5, 'rgb')
    for k, t in dec.named_parameters():
        ref_g = rp[k].grad
        close(t.grad, ref_g, 0, 2e-3 * max(ref_g.abs().max().item(), 1e-12), k)


def test_empty_ray_batch(dev, scene):
    """N = 0 without gt depth: empty outputs of the reference dtypes (with gt depth the reference
    itself fails on the empty max of Renderer.py:112)."""
    import pnr
    dec = make_decoder(pnr, golden_params('trained'), dev)
    r = _renderer(pnr, scene)
    e = torch.empty((0, 3), device=dev)
    with torch.no_grad():
        d, v, c = r.render_batch_ray({}, dec, e, e, dev, 'color')
    assert d.shape == (0,) and v.shape == (0,) and c.shape == (0, 3)
    assert d.dtype == torch.float64 and c.dtype == torch.float32
    raw = r.eval_points(torch.empty((0, 3), device=dev, dtype=torch.float64), dec)
    assert raw.shape == (0, 4)


def test_empty_point_cloud(dev, scene):
    """A neural-point cloud with no points gives c = 0 everywhere: the render equals the one of the
    same decoder with a far-away cloud, and the gather of any query is zero."""
    import pnr
    from oracle import ref_points as RP
    params = RP.init_fc_c(golden_params('trained'), seed=1)
    dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    empty = pnr.NeuralPoints(torch.empty((0, 3), device=dev), torch.empty((0, 32), device=dev), radius=0.04)
    far = pnr.NeuralPoints(torch.full((4, 3), 50.0, device=dev), torch.randn((4, 32), device=dev), radius=0.04)
    q = torch.rand((1000, 3), device=dev, dtype=torch.float64)
    assert torch.equal(empty.gather(q), torch.zeros((1000, 32), device=dev))
    g = load_golden('render.npz')
    ro = torch.from_numpy(g['p2_gt/rays_o'][:128].copy()).to(dev)
    rd = torch.from_numpy(g['p2_gt/rays_d'][:128].copy()).to(dev)
    gt = torch.from_numpy(g['p2_gt/gt_depth'][:128].copy()).to(dev)
    r = _renderer(pnr, scene)
    with torch.no_grad():
        a = r.render_batch_ray({'points_color': empty}, dec, rd, ro, dev, 'color', gt_depth=gt)
        b = r.render_batch_ray({'points_color': far}, dec, rd, ro, dev, 'color', gt_depth=gt)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    assert np.isfinite(a[0].cpu().numpy()).all()
