"""BASELINE.json config C4 (ScanNet scene0000_00) on one MI355X, against the oracle.

The effective config is configs/ScanNet/scene0000.yaml <- configs/ScanNet/scannet.yaml under
configs/pointNeRF_slam.yaml:
  * bound [[-2,11],[-2,11.5],[-2,5.5]] (scene0000.yaml:3) x scale 0.1, upper ends rounded to
    bound_divisible 0.32 (src/NICE_SLAM.py:208-213);
  * the 640x480 camera fx 577.590698, fy 578.729797, cx 318.905426, cy 242.683609 with crop_edge 10
    (scannet.yaml:23-30): 620x460, cx - 10, cy - 10 (src/NICE_SLAM.py:194-198);
  * mapping: 5,000 pixels over a window of 10 frames (mapping.pixels / mapping_window_size,
    scannet.yaml:19-20): 500 uniform pixels per frame (src/Mapper.py:560-606, pnr.window_batch);
  * tracking: 1,000 pixels (tracking.pixels), lr 5e-4, ignore_edge 20 (scannet.yaml:4-11).

The dataset is absent (no network): the frames are renders of the trained room0 decoder at ten
poses around the scene's centre, the gt depth those renders perturbed by 2% (every 9th pixel 0).
Checked, in fp32 and the default f16x3:
  * Mapper iteration (render + regulation + L1 losses, src/Mapper.py:623-655) on the 5,000-pixel
    window batch: loss vs the oracle and all 11 decoder gradients ELEMENTWISE vs the
    correctly-rounded gradient (oracle.ref_render.eval_points_cr), rtol 1e-3 with atol
    (1e-6 + d32) max|g|, d32 = the float32 oracle's own distance from it on the same batch;
  * Tracker iteration (src/Tracker.py:253-335) on 1,000 random pixels: loss and camera-tensor
    gradient elementwise likewise; then 20 camera Adam iterations at lr 5e-4 lower the loss.
"""
import math
import types

import numpy as np
import pytest
import torch

from conftest import golden_params
from oracle import ref_render as RR

pytestmark = pytest.mark.gpu

SCENE0000 = [[-2.0, 11.0], [-2.0, 11.5], [-2.0, 5.5]]
EDGE = 10
H, W = 480 - 2 * EDGE, 640 - 2 * EDGE
FX, FY, CX, CY = 577.590698, 578.729797, 318.905426 - EDGE, 242.683609 - EDGE
MAP_PIXELS, WINDOW, TRACK_PIXELS, TRACK_LR, TRACK_EDGE = 5000, 10, 1000, 5e-4, 20


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


@pytest.fixture(autouse=True, params=['fp32', 'f16x3'])
def precision(request, monkeypatch):
    from pnr import _lib
    monkeypatch.setattr(_lib, 'DEFAULT_PRECISION', request.param)
    return request.param


def pose(bound, k):
    """Camera k of 10: at the bound's centre, yaw 36 k degrees, pitch -10 degrees."""
    c = bound.float().mean(1)
    yaw, pitch = math.radians(36.0 * k), math.radians(-10.0)
    Ry = torch.tensor([[math.cos(yaw), 0., math.sin(yaw)], [0., 1., 0.], [-math.sin(yaw), 0., math.cos(yaw)]])
    Rx = torch.tensor([[1., 0., 0.], [0., math.cos(pitch), -math.sin(pitch)], [0., math.sin(pitch), math.cos(pitch)]])
    c2w = torch.eye(4)
    c2w[:3, :3] = Ry @ Rx
    c2w[:3, 3] = c + 0.02 * torch.tensor([math.cos(yaw), 0.3, math.sin(yaw)])
    return c2w


@pytest.fixture(scope='module')
def scannet(pnr_mod, dev):
    """Bound, slam stand-in and the 10 frames (c2w, gt depth, gt colour) on the device."""
    bound = RR.scaled_bound(SCENE0000, 0.1, 0.32)
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=FX, fy=FY, cx=CX, cy=CY)
    params = golden_params('trained')
    cfg = dict(pnr_mod.ROOM0_CFG)
    cfg['pnr'] = {'precision': 'fp32'}
    r = pnr_mod.Renderer(cfg, None, slam)
    dec = pnr_mod.get_model(pnr_mod.ROOM0_CFG, nice=False)
    dec.load_state_dict(params)
    dec = dec.to(dev)
    g = torch.Generator().manual_seed(40)
    frames = []
    with torch.no_grad():
        for k in range(WINDOW):
            c2w = pose(bound, k)
            d, _, col = r.render_img({}, dec, c2w.to(dev), dev, 'color')
            gd = (d.float() * (1 + 0.02 * torch.randn(d.shape, generator=g).to(dev))).contiguous()
            gd.view(-1)[::9] = 0.
            frames.append((c2w.to(dev), gd, col.float().clamp(0, 1).contiguous()))
    return bound, slam, params, frames


def _elementwise(g, cr, f32, what):
    """|g - g_cr| <= 1e-3 |g_cr| + (1e-6 + d32) max|g_cr|, d32 = max|g_f32 - g_cr| / max|g_cr|."""
    g = g.detach().cpu().numpy() if isinstance(g, torch.Tensor) else g
    scale = max(np.abs(cr).max(), 1e-30)
    d32 = np.abs(f32 - cr).max() / scale
    atol = (1e-6 + d32) * scale
    viol = np.abs(g - cr) / (1e-3 * np.abs(cr) + atol)
    print(f'{what}: float32 oracle vs cr {d32:.2e} max; worst |g - g_cr| / (rtol |g_cr| + atol) = {viol.max():.3f}')
    return viol.max()


def test_c4_scannet_map_step(pnr_mod, dev, scannet, precision):
    from pnr.mapping import MapStep, window_batch
    bound, slam, params, frames = scannet
    r = pnr_mod.Renderer(pnr_mod.ROOM0_CFG, None, slam)
    dec = pnr_mod.get_model(pnr_mod.ROOM0_CFG, nice=False)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    gen = torch.Generator(device=dev).manual_seed(3)
    ro, rd, gd, gc = window_batch(frames, MAP_PIXELS // WINDOW, H, W, FX, FY, CX, CY, dev, generator=gen)
    assert ro.shape == (MAP_PIXELS, 3)
    t_rand = torch.rand((MAP_PIXELS, 32), generator=torch.Generator().manual_seed(4))
    ms = MapStep(r, dec, lr=2e-4, w_color_loss=0.05)
    loss = float(ms(ro, rd, gd, gc, t_rand.to(dev)))
    torch.cuda.synchronize()
    assert r.status(dev) == 0
    ro_c, rd_c, gd_c, gc_c = (t.cpu() for t in (ro, rd, gd, gc))
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    refs = {}
    for tag, ev in (('f32', None), ('cr', 'cr')):
        p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
        fn = (lambda q, p=p: RR.eval_points_cr(p, q, bound)) if ev else None
        d, v, c = RR.render_batch_ray(p, rd_c, ro_c, bound, gt_depth=gd_c, eval_fn=fn)
        sig = RR.regulation(p, rd_c, ro_c, gd_c, bound, t_rand=t_rand, eval_fn=fn)
        lr_ = RR.mapping_loss(d, c, gd_c, gc_c, sig)
        lr_.backward()
        refs[tag] = (lr_.item(), {k: t.grad.numpy().copy() for k, t in p.items()})
    print(f'C4 map loss: HIP {loss:.6f}, oracle {refs["f32"][0]:.6f}')
    assert abs(loss - refs['f32'][0]) <= 1e-5 * abs(refs['f32'][0])
    from pnr.decoder import PARAM_ORDER
    off = 0
    worst = {}
    for k, t in zip(PARAM_ORDER, ms.flat.params):
        gk = ms.flat.grad[off:off + t.numel()].view_as(t)
        off += t.numel()
        worst[k] = _elementwise(gk, refs['cr'][1][k], refs['f32'][1][k], f'{precision} C4 map grad {k}')
    assert max(worst.values()) <= 1.0, worst


def test_c4_scannet_track_step(pnr_mod, dev, scannet, precision):
    bound, slam, params, frames = scannet
    r = pnr_mod.Renderer(pnr_mod.ROOM0_CFG, None, slam)
    dec = pnr_mod.get_model(pnr_mod.ROOM0_CFG, nice=False)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec = dec.to(dev)
    c2w, gd, gc = frames[3]
    ct_true = pnr_mod.get_tensor_from_camera(c2w.cpu())
    ct0 = ct_true + torch.tensor([0.002, -0.001, 0.0015, 0.001, 0.003, -0.002, 0.0025])

    def step_for(seed):
        return pnr_mod.TrackStep(r, dec, weak_depth=False, ignore_edge_W=TRACK_EDGE, ignore_edge_H=TRACK_EDGE,
                                 generator=torch.Generator(device=dev).manual_seed(seed))
    ct = ct0.clone().to(dev).requires_grad_(True)
    loss = step_for(11).loss(ct, gc, gd, TRACK_PIXELS)
    loss.backward()
    # the same pixels on the CPU (select_uv_indices with the same seeded device generator)
    from pnr.common import select_uv_indices
    w = W - 2 * TRACK_EDGE
    npix = (H - 2 * TRACK_EDGE) * w
    idx = select_uv_indices(npix, TRACK_PIXELS, dev, torch.Generator(device=dev).manual_seed(11)).cpu()
    i = (idx % w + TRACK_EDGE).float()
    j = (idx // w + TRACK_EDGE).float()
    gdc = gd[TRACK_EDGE:H - TRACK_EDGE, TRACK_EDGE:W - TRACK_EDGE].reshape(-1).cpu()[idx]
    gcc = gc[TRACK_EDGE:H - TRACK_EDGE, TRACK_EDGE:W - TRACK_EDGE].reshape(-1, 3).cpu()[idx]
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    refs = {}
    for tag in ('f32', 'cr'):
        ctr = ct0.clone().requires_grad_(True)
        ro, rd = RR.rays_from_uv(i, j, RR.camera_from_tensor(ctr), FX, FY, CX, CY)
        fn = (lambda q: RR.eval_points_cr(params, q, bound)) if tag == 'cr' else None
        d, v, c = RR.render_batch_ray(params, rd.reshape(-1, 3), ro.reshape(-1, 3), bound, gt_depth=gdc, eval_fn=fn)
        lr_ = RR.tracking_loss(d, v, c, gdc, gcc)
        lr_.backward()
        refs[tag] = (lr_.item(), ctr.grad.numpy().copy())
    print(f'C4 track loss: HIP {float(loss):.6f}, oracle {refs["f32"][0]:.6f}')
    assert abs(float(loss) - refs['f32'][0]) <= 1e-4 * abs(refs['f32'][0])
    assert _elementwise(ct.grad, refs['cr'][1], refs['f32'][1], f'{precision} C4 camera tensor grad') <= 1.0
    # the per-frame loop at the config's lr: 20 iterations from the perturbed pose
    best, _, losses = pnr_mod.track_frame(step_for(12), ct0.to(dev), gc, gd, 20, TRACK_LR, TRACK_PIXELS)
    print(f'C4 tracking losses {losses[0]:.4f} -> {min(losses):.4f}')
    assert min(losses) < losses[0]
    assert all(math.isfinite(x) for x in losses)
