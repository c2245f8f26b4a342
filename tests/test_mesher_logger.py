"""Host logic of the Mesher colour branch and the Logger checkpoint interop (SURVEY.md section 8
(f) row F4): grid, vertex normals (vs the oracle's per-triangle loop restatement of open3d's
compute_vertex_normals; parity unpinned beyond it, open3d is absent), colour quantisation, and
checkpoint round trips in the reference's format (src/utils/Logger.py:23-32)."""
import types
import zipfile

import numpy as np
import torch

from conftest import golden_params
from mesh_util import uv_sphere


def test_grid_uniform_matches_oracle(scene):
    from pnr import mesher
    from oracle import ref_mesh
    g = mesher.get_grid_uniform(scene['bound_t'], 17)
    assert g['grid_points'].dtype == torch.float32 and g['grid_points'].shape == (17 ** 3, 3)
    assert torch.equal(g['grid_points'], ref_mesh.grid_uniform(scene['bound'], 17))


def test_vertex_normals_match_restatement():
    from pnr import mesher
    from oracle import ref_mesh
    v, f = uv_sphere([0.3, 0.1, 0.05], 0.2, 8, 12)
    rng = np.random.default_rng(0)
    v = v + rng.normal(scale=1e-3, size=v.shape)
    # an isolated vertex (no face) and a degenerate triangle: both take (0,0,1) / a zero contribution
    v = np.vstack([v, [[0.0, 0.0, 0.0]] * 3])
    V = v.shape[0]
    f = np.vstack([f, [[V - 2, V - 1, V - 1]]])
    n = mesher.vertex_normals(torch.from_numpy(v), torch.from_numpy(f)).numpy()
    r = ref_mesh.vertex_normals(v, f)
    np.testing.assert_allclose(n, r, rtol=0, atol=1e-12)
    assert np.allclose(n[V - 3], [0, 0, 1]) and np.allclose(n[V - 1], [0, 0, 1])
    # outward on the sphere
    c = v[:V - 3] - np.array([0.3, 0.1, 0.05])
    assert (np.sum(n[:V - 3] * c, 1) > 0).all()


def test_vertex_colors_u8():
    from pnr import mesher
    c = torch.tensor([[-0.5, 0.0, 0.5], [1.0, 1.2, 0.99999]])
    assert mesher.vertex_colors_u8(c).tolist() == [[0, 0, 127], [255, 255, 254]]


def _slam(tmp_path, dec, c):
    return types.SimpleNamespace(verbose=False, ckptsdir=str(tmp_path), shared_c=c, shared_decoders=dec,
                                 gt_c2w_list=torch.eye(4).repeat(5, 1, 1),
                                 estimate_c2w_list=torch.eye(4).repeat(5, 1, 1) * 2)


def test_logger_roundtrip_reference_format(tmp_path):
    import pnr
    from pnr import logger
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    dec.load_state_dict(golden_params('trained'))
    lg = logger.Logger(None, None, _slam(tmp_path, dec, {}))
    path = lg.log(7, {}, [0, 3], selected_keyframes={7: [0, 3]})
    assert path.endswith('00007.tar')
    assert not zipfile.is_zipfile(path)  # legacy serialisation (_use_new_zipfile_serialization=False)
    raw = torch.load(path, map_location='cpu', weights_only=True)
    assert tuple(sorted(raw)) == tuple(sorted(logger.CKPT_KEYS))
    assert raw['c'] == {} and raw['idx'] == 7 and raw['keyframe_list'] == [0, 3]
    ref_keys = sorted(golden_params('trained'))
    assert sorted(raw['decoder_state_dict']) == ref_keys
    dec2 = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    ck = logger.load_ckpt(path, dec2)
    for k, v in dec.state_dict().items():
        assert torch.equal(v, dec2.state_dict()[k])
    assert torch.equal(ck['estimate_c2w_list'], torch.eye(4).repeat(5, 1, 1) * 2)


def test_logger_neural_points_roundtrip(tmp_path):
    import pnr
    from pnr import logger
    g = torch.Generator().manual_seed(0)
    pts = pnr.NeuralPoints(torch.rand(50, 3, generator=g), torch.randn(50, 32, generator=g), radius=0.05, k=4)
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
    path = logger.Logger(None, None, _slam(tmp_path, dec, {'points_color': pts})).log(1, {}, [])
    ck = logger.load_ckpt(path)
    p2 = ck['c']['points_color']
    assert isinstance(p2, pnr.NeuralPoints)
    assert torch.equal(p2.xyz, pts.xyz) and torch.equal(p2.feats.data, pts.feats.data)
    for f in ('mode', 'k', 'radius', 'eps', 'spacing', 'cell', 'origin', 'table_bits'):
        assert getattr(p2, f) == getattr(pts, f), f
