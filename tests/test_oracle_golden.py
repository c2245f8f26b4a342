"""Pin the CPU oracle (oracle/ref_render.py) to the golden vectors made by importing the
reference renderer (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import load_golden, golden_params
from oracle import ref_render as ref

torch.set_num_threads(1)
CASES = [f'p{i}_{c}' for i in range(4) for c in ('none', 'gt', 'gtzero')]


def _close(a, b, rtol, atol, what):
    a = a.detach().numpy() if isinstance(a, torch.Tensor) else a
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


def test_bound(scene):
    b = ref.scaled_bound(scene['bound_cfg'], float(scene['scale']), float(scene['bound_divisible']))
    assert torch.equal(b, scene['bound_t'])
    np.testing.assert_allclose(scene['bound'], [[-0.29, 0.99], [-0.32, 0.64], [-0.35, 0.61]], atol=1e-9)


def test_eval_points(scene, trained_params):
    z = load_golden('points.npz')
    raw = ref.eval_points(trained_params, torch.from_numpy(z['p']), scene['bound_t'])
    assert torch.equal(raw, torch.from_numpy(z['raw']))


@pytest.mark.parametrize('case', CASES + ['rand_none', 'edge_none'])
def test_render_batch_ray_bitexact(case, scene):
    g = load_golden('render.npz')
    params = golden_params('random' if case.startswith('rand') else 'trained')
    ro = torch.from_numpy(g[f'{case}/rays_o']); rd = torch.from_numpy(g[f'{case}/rays_d'])
    gt = torch.from_numpy(g[f'{case}/gt_depth']) if f'{case}/gt_depth' in g else None
    d, v, c, ex = ref.render_batch_ray(params, rd, ro, scene['bound_t'], gt_depth=gt, return_extras=True)
    n = g[f'{case}/z_fine'].shape[0]
    for k in ('z_coarse', 'w_coarse', 'raw_coarse', 'z_samples', 'z_fine', 'w_fine', 'raw_fine'):
        assert np.array_equal(ex[k][:n].numpy(), g[f'{case}/{k}']), k
    assert np.array_equal(d.numpy(), g[f'{case}/depth'])
    assert np.array_equal(v.numpy(), g[f'{case}/var'])
    assert np.array_equal(c.numpy(), g[f'{case}/rgb'])
    assert d.dtype == torch.float64 and v.dtype == torch.float64 and c.dtype == torch.float32


def test_composite_and_pdf_vectors():
    k = load_golden('kernels.npz')
    d, v, c, w = ref.composite(torch.from_numpy(k['r2o_raw']), torch.from_numpy(k['r2o_z']),
                               torch.from_numpy(k['r2o_rd']))
    assert np.array_equal(d.numpy(), k['r2o_depth']) and np.array_equal(v.numpy(), k['r2o_var'])
    assert np.array_equal(c.numpy(), k['r2o_rgb']) and np.array_equal(w.numpy(), k['r2o_w'])
    s = ref.sample_pdf(torch.from_numpy(k['pdf_bins']), torch.from_numpy(k['pdf_w']), 12)
    assert np.array_equal(s.numpy(), k['pdf_out'])
    s0 = ref.sample_pdf(torch.from_numpy(k['pdf_bins']), torch.from_numpy(k['pdf_w_zero']), 12)
    assert np.array_equal(s0.numpy(), k['pdf_out_zero'])


def test_mapping_grads(scene):
    G = load_golden('grads.npz')
    params = {k: v.clone().requires_grad_(True) for k, v in golden_params('trained').items()}
    ro, rd = torch.from_numpy(G['map_rays_o']), torch.from_numpy(G['map_rays_d'])
    gt, gcol = torch.from_numpy(G['map_gt_depth']), torch.from_numpy(G['map_gt_color'])
    d, v, c = ref.render_batch_ray(params, rd, ro, scene['bound_t'], gt_depth=gt)
    sig = ref.regulation(params, rd, ro, gt, scene['bound_t'], t_rand=torch.from_numpy(G['map_t_rand']))
    assert np.array_equal(sig.detach().numpy(), G['map_sigma'])
    loss = ref.mapping_loss(d, c, gt, gcol, sig)
    loss.backward()
    assert loss.item() == float(G['map_loss'])
    for k, p in params.items():
        _close(p.grad, G[f'map_grad/{k}'], 1e-5, 1e-7, k)


def test_tracking_grads(scene):
    G = load_golden('grads.npz')
    params = golden_params('trained')
    ro = torch.from_numpy(G['map_rays_o']).clone().requires_grad_(True)
    rd = torch.from_numpy(G['map_rays_d']).clone().requires_grad_(True)
    gt, gcol = torch.from_numpy(G['map_gt_depth']), torch.from_numpy(G['map_gt_color'])
    d, v, c = ref.render_batch_ray(params, rd, ro, scene['bound_t'], gt_depth=gt)
    loss = ref.tracking_loss(d, v, c, gt, gcol)
    loss.backward()
    _close(loss.detach(), float(G['trk_loss']), 1e-6, 0, 'loss')
    _close(ro.grad, G['trk_grad_rays_o'], 1e-5, 1e-6, 'rays_o')
    _close(rd.grad, G['trk_grad_rays_d'], 1e-5, 1e-6, 'rays_d')


def test_render_img(scene, trained_params):
    z = load_golden('render_img.npz')
    d, v, c = ref.render_img(trained_params, torch.from_numpy(z['c2w']), scene['bound_t'], int(z['H']), int(z['W']),
                             float(z['fx']), float(z['fy']), float(z['cx']), float(z['cy']),
                             gt_depth=torch.from_numpy(z['gt_depth']), ray_batch_size=int(z['ray_batch_size']))
    assert np.array_equal(d.numpy(), z['depth']) and np.array_equal(v.numpy(), z['var'])
    assert np.array_equal(c.numpy(), z['rgb'])


def test_pose_roundtrip(scene):
    for c2w in scene['poses']:
        t = ref.tensor_from_camera(c2w)
        RT = ref.camera_from_tensor(t)
        np.testing.assert_allclose(RT.numpy(), c2w[:3, :4], atol=2e-6)
