"""The wave-per-ray compositing kernels (k_pdf_w / k_fine_w / k_fine_bwd_w, batches up to 32,768 rays)
against the thread-per-ray ones (larger batches): compositing is independent per ray, so the first
rays of a 40,000-ray batch (thread-per-ray kernels) and the same rays as a batch of their own
(wave-per-ray kernels) must give the same depth / variance / colour, importance samples, map-pass
densities and ray gradients bit for bit -- both follow the reference's accumulation order
(Renderer.py:157-201, common.py:204-245) with the same roundings.  The far clamp is fixed so both
batches share Renderer.py:112's bound.  Rays include gt depth 0 (bound-limited sampling), rays
that start beyond the gt surface (far < near: the unsorted-merge branch of sort_ray) and rays
that leave the scene bound."""
import pytest
import torch

from conftest import golden_params
from test_gpu_parity import make_decoder, make_renderer

pytestmark = pytest.mark.gpu

N_BIG, N_SMALL = 40000, 1000


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


def _rays(scene, dev, n, seed=0):
    g = torch.Generator().manual_seed(seed)
    c2w = torch.from_numpy(scene['poses'][2]).float()
    i = torch.rand(n, generator=g) * 1200
    j = torch.rand(n, generator=g) * 680
    dirs = torch.stack([(i - 599.5) / 600., -(j - 339.5) / 600., -torch.ones(n)], -1)
    rd = (dirs[:, None, :] * c2w[:3, :3]).sum(-1)
    ro = c2w[:3, 3].expand(n, 3).clone()
    ro += 0.05 * torch.randn((n, 3), generator=g)
    gt = 0.3 + 2.0 * torch.rand(n, generator=g)
    gt[torch.rand(n, generator=g) < 0.1] = 0.
    gt[torch.rand(n, generator=g) < 0.05] = 0.01  # near > far on bound-limited rays
    return ro.to(dev), rd.to(dev), gt.to(dev)


def test_render_wave_equals_thread(dev, scene):
    import pnr
    dec = make_decoder(pnr, golden_params('trained'), dev)
    for p_ in dec.parameters():
        p_.requires_grad_(False)
    r = make_renderer(pnr, scene)
    ro, rd, gt = _rays(scene, dev, N_BIG)
    far = float((gt * 1.2).max())
    out = {}
    for n in (N_BIG, N_SMALL):
        o = ro[:n].clone().requires_grad_(True)
        d_ = rd[:n].clone().requires_grad_(True)
        d, v, c = r.render_batch_ray({}, dec, d_, o, dev, 'color', gt_depth=gt[:n], far_clamp=far)
        (d.sum() + 0.5 * c.sum() + 1e-3 * v.sum()).backward()
        out[n] = [t.detach()[:N_SMALL].clone() for t in (d, v, c, o.grad, d_.grad)]
    for a, b, what in zip(out[N_BIG], out[N_SMALL], ('depth', 'var', 'rgb', 'grad rays_o', 'grad rays_d')):
        eq = (a == b) | (torch.isnan(a) & torch.isnan(b))
        assert bool(eq.all()), f'{what}: {int((~eq).sum())} differ'


def test_map_pass_wave_equals_thread(dev, scene):
    """pnr_map_fwd's compositing outputs (depth, var, rgb and the regulation densities, with the
    importance rows k_pdf forms for the second MLP launch) per ray, both kernel forms."""
    import pnr
    from pnr.renderer import MapPass
    dec = make_decoder(pnr, golden_params('trained'), dev)
    r = make_renderer(pnr, scene)
    ro, rd, gt = _rays(scene, dev, N_BIG, seed=1)
    t_rand = torch.rand((N_BIG, r.N_samples), device=dev, generator=torch.Generator(device=dev).manual_seed(2))
    far = torch.tensor([float((gt * 1.2).max())], device=dev)
    out = {}
    for n in (N_BIG, N_SMALL):
        mp = MapPass(r, {}, dec)
        with torch.no_grad():
            res = mp.forward(ro[:n].contiguous(), rd[:n].contiguous(), gt[:n].contiguous(), t_rand[:n].contiguous(),
                             far_clamp=far)
        out[n] = [t[:N_SMALL].clone() for t in res]
    for a, b, what in zip(out[N_BIG], out[N_SMALL], ('depth', 'var', 'rgb', 'sigma')):
        eq = (a == b) | (torch.isnan(a) & torch.isnan(b))
        assert bool(eq.all()), f'{what}: {int((~eq).sum())} differ'
