"""The Mesher's decoder consumers on the HIP path against the
oracle: the dense grid query (Mesher.py:427-430) and the render_ray_along_normal vertex colouring
(Mesher.py:526-556) of a sphere mesh inside the room0 bound.
Tolerances as tests/test_gpu_parity.py: raw atol 2e-5*max|raw|; colour rtol 1e-4, atol 2e-5;
uint8 vertex colours within 1 step (truncation of values within 2e-5 of a step boundary)."""
import numpy as np
import pytest
import torch

from conftest import golden_params
from mesh_util import uv_sphere
from test_gpu_parity import make_decoder, make_renderer, close, precision  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


def _setup(dev, scene):
    import pnr
    params = golden_params('trained')
    return pnr, params, make_decoder(pnr, params, dev), make_renderer(pnr, scene, ray_batch_size=1000,
                                                                       points_batch_size=5000)


def test_eval_grid_vs_oracle(dev, scene):
    from oracle import ref_render as ref
    pnr, params, dec, r = _setup(dev, scene)
    g = pnr.mesher.get_grid_uniform(scene['bound_t'], 20)['grid_points']
    raw = pnr.mesher.eval_grid(r, dec, {}, g.to(dev), dev)
    rr = ref.eval_points(params, g, scene['bound_t'])
    close(raw, rr, 0, 2e-5 * float(rr.abs().max()), 'grid raw')
    assert np.array_equal(raw[:, 3].cpu().numpy() == 100., rr[:, 3].numpy() == 100.)


def test_color_along_normal_vs_oracle(dev, scene):
    from oracle import ref_mesh
    pnr, params, dec, r = _setup(dev, scene)
    b = scene['bound']
    v, f = uv_sphere(b.mean(1), 0.2, 24, 48)  # 1,106 vertices: two ray_batch_size chunks
    n = pnr.mesher.vertex_normals(torch.from_numpy(v).to(dev), torch.from_numpy(f).to(dev))
    np.testing.assert_allclose(n.cpu().numpy(), ref_mesh.vertex_normals(v, f), rtol=0, atol=1e-12)
    col = pnr.mesher.color_along_normal(r, dec, {}, torch.from_numpy(v), n, dev)
    cr = ref_mesh.color_along_normal(params, v, n.cpu().numpy(), scene['bound_t'])
    close(col, cr, 1e-4, 2e-5, 'vertex colour')
    u8 = pnr.mesher.mesh_colors(r, dec, {}, v, f, dev)
    ur = (np.clip(cr.numpy(), 0, 1) * 255).astype(np.uint8)
    assert u8.dtype == np.uint8 and np.abs(u8.astype(int) - ur.astype(int)).max() <= 1


def test_direct_point_query_vs_oracle(dev, scene):
    from oracle import ref_render as ref
    pnr, params, dec, r = _setup(dev, scene)
    v, _ = uv_sphere(scene['bound'].mean(1), 0.2, 8, 16)
    col = pnr.mesher.direct_point_query(r, dec, {}, torch.from_numpy(v), dev)
    rr = ref.eval_points(params, torch.from_numpy(v).float(), scene['bound_t'])[..., :3]
    close(col, rr, 0, 2e-5 * float(rr.abs().max()), 'vertex raw colour')
