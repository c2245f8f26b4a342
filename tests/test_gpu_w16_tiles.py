"""The 16-point-wave forward (csrc/mlp16w.h) runs 128-point tiles of 8 waves, or -- for a batch whose
128-point tiles would fill at most half the CUs once -- 64-point tiles of 4 waves (k_mlp_fwd16w<SV, 4>,
the Mapper's importance launch).  Each point's arithmetic is the same in both (its own 16-point wave,
the same MFMA shapes and order), so the two forms must agree bit for bit on the same points: a small
batch (4-wave tiles) against the same points inside a large one (8-wave tiles), for the eval forward
(Renderer.eval_points, src/utils/Renderer.py:23-61) and the training forward with saves
(MLP.forward, src/conv_onet/models/decoder.py:177-203).  Ragged sizes included."""
import types

import pytest
import torch

pytestmark = pytest.mark.gpu

P_BIG = 65536   # 512 tiles of 128 points: the 8-wave form on any CU count up to 1,024
SMALL = (8192, 8192 + 37, 1, 63)  # <= 16,384 points: the 4-wave form on a 256-CU MI355X


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


@pytest.fixture(scope='module')
def setup(dev, scene, trained_params):
    import pnr
    pnr.library()
    slam = types.SimpleNamespace(bound=scene['bound_t'], H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': 'f16x3'}
    r = pnr.Renderer(cfg, None, slam)
    dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4, pos_embedding_method='fourier')
    dec.load_state_dict({k: v.clone() for k, v in trained_params.items()})
    dec = dec.to(dev)
    dec.precision = 'f16x3'
    g = torch.Generator(device=dev).manual_seed(7)
    lo, hi = scene['bound_t'][:, 0].to(dev), scene['bound_t'][:, 1].to(dev)
    pts = lo + (hi - lo) * torch.rand(P_BIG, 3, device=dev, dtype=torch.float64, generator=g)
    pts = pts * 1.1 - 0.05 * (hi - lo)  # some points outside the bound (sigma = 100 there)
    return r, dec, pts


def test_w16_tile_forms_agree_eval(setup):
    r, dec, pts = setup
    with torch.no_grad():
        big = r.eval_points(pts, dec)
        for n in SMALL:
            small = r.eval_points(pts[:n].contiguous(), dec)
            torch.cuda.synchronize()
            assert torch.equal(small, big[:n]), n


def test_w16_tile_forms_agree_training(setup):
    r, dec, pts = setup
    x = pts.float()
    big = dec(x).detach()
    for n in SMALL:
        small = dec(x[:n].contiguous()).detach()
        torch.cuda.synchronize()
        assert torch.equal(small, big[:n]), n
