"""C1 plumbing (BASELINE.json configs[0]: "Replica room0, first 20 frames"): the Mapper / Tracker
loop over a 20-frame sequence, the way src/Mapper.py:700-933 and src/Tracker.py:651-944 drive the
renderer, on the HIP path -- in fp32 and in the default f16x3.

The dataset is absent: the frames are rendered by the ORACLE (oracle/ref_render.py, the reference
CPU arithmetic) with the trained room0 decoder along a synthetic camera path near room0 pose 1
(0.15 deg of yaw and ~0.9 mm per frame), at 48x64.  The loop:
  * frame 0: gt pose;
  * every frame > 0: track from the constant-speed prediction of the last two estimates
    (tracking.const_speed_assumption, src/Tracker.py:857-868; pnr.track_frame: TrackStep x 10,
    camera Adam lr 1e-3, weak depth, best-loss candidate; src/Tracker.py:860-921);
  * every 5th frame (mapping.every_frame): a window of the last 4 keyframes + the frame
    (mapping_window_size 5), 10 Mapper iterations (window_batch -> MapStep, src/Mapper.py:507-662),
    then the frame becomes a keyframe.
The decoder starts slightly perturbed (so mapping has work to do).

Checked, in both modes: the free-running loop keeps the tracked path within a few frames' motion
of the true one (camera Adam at lr 1e-3 resolves ~1e-3 per frame, the size of one frame's motion).
Two free-running loops diverge chaotically (the best-loss candidate of each frame is an argmin),
so the modes are compared on the same loop teacher-forced -- mapping on the true poses, every frame
tracked from its true pose plus a fixed offset: per-iteration tracking losses and the final decoder
of f16x3 must equal fp32's to 1e-4.
"""
import math

import numpy as np
import pytest
import torch

from conftest import golden_params
from oracle import ref_render as RR

pytestmark = pytest.mark.gpu

H, W, FX, FY, CX, CY = 48, 64, 40., 40., 31.5, 23.5
N_FRAMES, EVERY, WINDOW, MAP_ITERS, TRACK_ITERS = 20, 5, 5, 10, 10


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    return torch.device('cuda:0')


def path(scene):
    base = torch.from_numpy(scene['poses'][1]).double()
    out = []
    for f in range(N_FRAMES):
        a = math.radians(0.15 * f)
        R = torch.tensor([[math.cos(a), -math.sin(a), 0.], [math.sin(a), math.cos(a), 0.], [0., 0., 1.]],
                         dtype=torch.float64)
        c2w = base.clone()
        c2w[:3, :3] = R @ base[:3, :3]
        c2w[:3, 3] = base[:3, 3] + torch.tensor([0.0008, 0.0004, 0.], dtype=torch.float64) * f
        out.append(c2w.float())
    return out


@pytest.fixture(scope='module')
def sequence(scene):
    params = golden_params('trained')
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    frames = []
    for c2w in path(scene):
        d, _, c = RR.render_img(params, c2w, scene['bound_t'], H, W, FX, FY, CX, CY)
        frames.append((c2w, d.float(), c.float()))
    return params, frames


def run_loop(pnr, scene, params, frames, precision, dev, teacher=False):
    import types
    from pnr.mapping import MapStep, window_batch
    slam = types.SimpleNamespace(bound=scene['bound_t'], H=H, W=W, fx=FX, fy=FY, cx=CX, cy=CY)
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr.Renderer(cfg, None, slam)
    start = {k: v.clone() for k, v in params.items()}
    g = torch.Generator().manual_seed(7)
    start['pts_linears.3.weight'] += 0.01 * start['pts_linears.3.weight'].std() * torch.randn(
        start['pts_linears.3.weight'].shape, generator=g)
    dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4)
    dec.load_state_dict(start)
    dec = dec.to(dev)
    ms = MapStep(r, dec, lr=2e-4, w_color_loss=0.05)
    gen = torch.Generator(device=dev).manual_seed(3)
    trand = torch.Generator().manual_seed(4)
    est, keyframes, map_losses, track_losses = [], [], [], []
    offset = torch.tensor([0.0005, -0.0004, 0.0003, 0.0002, 0.0008, -0.0006, 0.0004])
    for idx, (c2w_gt, depth, colour) in enumerate(frames):
        gd, gc = depth.to(dev), colour.to(dev)
        if idx == 0:
            est.append(c2w_gt.to(dev))
        else:
            step = pnr.TrackStep(r, dec, ignore_edge_W=4, ignore_edge_H=4)
            if teacher:
                ct0 = pnr.get_tensor_from_camera(c2w_gt) + offset
            else:
                pred = est[-1] if idx < 2 else est[-1] @ torch.linalg.inv(est[-2]) @ est[-1]  # constant speed
                ct0 = pnr.get_tensor_from_camera(pred.cpu())
            _, c2w, tl = pnr.track_frame(step, ct0.to(dev), gc, gd, TRACK_ITERS, 1e-3, 0)
            track_losses.append(tl)
            est.append(c2w.detach().float())
        if idx % EVERY == 0:
            window = keyframes[-(WINDOW - 1):] + [idx]
            poses = [frames[k][0].to(dev) for k in window] if teacher else [est[k] for k in window]
            fr = [(poses[n], frames[k][1].to(dev), frames[k][2].to(dev)) for n, k in enumerate(window)]
            for _ in range(MAP_ITERS):
                ro, rd, bd, bc = window_batch(fr, 200, H, W, FX, FY, CX, CY, dev, generator=gen)
                t_rand = torch.rand((ro.shape[0], 32), generator=trand).to(dev)
                map_losses.append(float(ms(ro, rd, bd, bc, t_rand)))
            keyframes.append(idx)
    assert r.status(dev) == 0
    poses = torch.stack([p[:3, :4].cpu() for p in est])
    return poses, ms.flat.data.detach().cpu().clone(), map_losses, np.array(track_losses)


def test_twenty_frame_loop(sequence, scene, dev):
    """The free-running loop: bounded tracking drift and finite losses in both modes."""
    import pnr
    params, frames = sequence
    gt = torch.stack([f[0][:3, :4] for f in frames])
    for p in ('fp32', 'f16x3'):
        poses, w, ml, tl = run_loop(pnr, scene, params, frames, p, dev)
        terr = (poses[:, :, 3] - gt[:, :, 3]).norm(dim=1)
        print(f'{p}: translation error mean {terr.mean():.2e} max {terr.max():.2e}; '
              f'map loss {ml[0]:.3f} -> {ml[-1]:.3f}; tracking loss per frame {tl[:, 0].mean():.3f} -> '
              f'{tl.min(1).mean():.3f}')
        assert all(math.isfinite(x) for x in ml) and np.isfinite(tl).all()
        # ~0.9e-3 of motion per frame and ~1e-3 of camera-Adam resolution: no runaway drift
        assert terr.mean().item() < 1.5e-3 and terr.max().item() < 4e-3, (p, terr)
        assert (tl.min(1) <= tl[:, 0]).all()


def test_twenty_frame_loop_teacher_forced_modes_agree(sequence, scene, dev):
    """The same loop with mapping on the true poses and each frame tracked from its true pose +
    a fixed offset: f16x3 follows fp32 iteration by iteration."""
    import pnr
    params, frames = sequence
    out = {p: run_loop(pnr, scene, params, frames, p, dev, teacher=True) for p in ('fp32', 'f16x3')}
    (p32, w32, m32, t32), (p16, w16, m16, t16) = out['fp32'], out['f16x3']
    rel_w = ((w16 - w32).norm() / w32.norm()).item()
    rel_t = np.max(np.abs(t16 - t32) / np.abs(t32))
    rel_m = np.max(np.abs(np.array(m16) - np.array(m32)) / np.array(m32))
    gt = torch.stack([f[0][:3, :4] for f in frames])
    terr = (p32[:, :, 3] - gt[:, :, 3]).norm(dim=1)
    print(f'teacher-forced f16x3 vs fp32: decoder rel L2 {rel_w:.2e}, tracking losses rel max {rel_t:.2e}, '
          f'map losses rel max {rel_m:.2e}, max pose diff {(p16 - p32).abs().max():.2e}; fp32 translation error '
          f'after tracking: mean {terr.mean():.2e}')
    # the first mapping round (10 iterations on frame 0, before any tracking) and the first tracking
    # iteration of frame 1 (after it) follow fp32 closely; later rounds amplify rounding through Adam's
    # per-element normalisation and the Tracker's 1/sqrt(var) weights (var is a cancellation-heavy
    # float64 second moment), so the loop as a whole is held to what the loop does to an fp32-class
    # perturbation of fp32 itself (the control below), not to a fixed bound
    m0 = np.max(np.abs(np.array(m16[:MAP_ITERS]) - np.array(m32[:MAP_ITERS])) / np.array(m32[:MAP_ITERS]))
    t0 = abs(t16[0, 0] - t32[0, 0]) / abs(t32[0, 0])
    print(f'first mapping round: map losses rel max {m0:.2e}; frame 1 first tracking loss rel {t0:.2e}')
    assert m0 < 1e-3 and t0 < 1e-3
    assert rel_w < 1e-3
    # control: fp32 against itself with every decoder weight moved by 2^-22 relative (the size of one
    # f16x3 product's rounding).  If the loop amplifies rounding, that run drifts from fp32 as well;
    # f16x3 must not drift more than twice as far as this fp32-class perturbation (+ a small floor)
    g = torch.Generator().manual_seed(11)
    pert = {k: v * (1.0 + 2.0 ** -22 * (2.0 * torch.randint(0, 2, v.shape, generator=g).float() - 1.0))
            for k, v in params.items()}
    pc, wc, mc, tc = run_loop(pnr, scene, pert, frames, 'fp32', dev, teacher=True)
    cw = ((wc - w32).norm() / w32.norm()).item()
    ct = np.max(np.abs(tc - t32) / np.abs(t32))
    cm = np.max(np.abs(np.array(mc) - np.array(m32)) / np.array(m32))
    print(f'control (fp32, weights x (1 +- 2^-22)) vs fp32: decoder rel L2 {cw:.2e}, tracking losses rel max '
          f'{ct:.2e}, map losses rel max {cm:.2e}')
    assert rel_w <= 2 * cw + 1e-5 and rel_t <= 2 * ct + 1e-3 and rel_m <= 2 * cm + 1e-3, (rel_w, cw, rel_t, ct, rel_m, cm)
