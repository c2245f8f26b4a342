"""BASELINE.json configs C3 and C5 on one MI355X, against the oracle.

  C3  Replica office3 (larger scene: configs/Replica/office3.yaml:3 bound x scale 0.1, rounded to
      bound_divisible 0.32, src/NICE_SLAM.py:208-213), bf16 MLP on MFMA, 200k neural points.
  C5  Apartment multi-room (configs/Apartment/apartment.yaml:11-36: 720x1280 camera, 5,000 mapping
      pixels per iteration), float16 point features and a 1M-point budget.

The datasets are absent (no network): the scenes are synthetic -- neural points on the walls of a
room filling the scaled bound plus boxes inside it, features N(0, 0.1), the trained room0 decoder
with fresh fc_c layers (src/conv_onet/models/decoder.py:122-125), a camera at the room's centre.
Parity: rays through the HIP path vs the oracle (oracle/ref_points.py gather + oracle/ref_render.py)
over the points near those rays (a superset of every sample's neighbourhood: exact) -- the render,
and the gradient of one MapStep (Mapper loss with regulation, src/Mapper.py:623-655) w.r.t. every
decoder / fc_c tensor and the point features, elementwise for f16x3: rtol 1e-3 with atol
(1e-6 + d32) max|g| against the correctly-rounded gradient (oracle.ref_points.mlp_forward_c_cr),
d32 = the float32 oracle's own distance from it; bf16 to 5% in norm.  f16x3 is
held to the fp32 tolerances of tests/test_gpu_parity.py.  bf16 (8 significant bits per operand)
is held to PSNR(bf16 HIP render, fp32 oracle render) > 45 dB and depth within 3e-2 relative: it
does NOT meet the metric's 0.1 dB PSNR clause (that needs ~70 dB); f16x3 does.
"""
import math
import types

import numpy as np
import pytest
import torch

from conftest import golden_params, maybe_dump_grads
from oracle import ref_points as RP
from oracle import ref_render as RR

pytestmark = pytest.mark.gpu

OFFICE3 = [[-6.7, 5.1], [-7.5, 4.9], [-2.8, 3.5]]       # configs/Replica/office3.yaml:3
# summation-magnitude floor in ulps of M = sum_p |t_p| (tests/test_gpu_points.py MAG_ULPS) and the
# decision-edge allowance (tests/test_gpu_points.py FLIP_CAP)
MAG_ULPS = 64.0
FLIP_CAP = 5e-4
# the share of a tensor's elements that may use it, >= 1.  Round 6: 3e-3 (was 1e-2).  Measured at the
# round-6 code (tools/flip_dump.sh, profiles/r06_flip_rank.txt): C3 f16x3 fc_c.0 / fc_c.1.weight 2.4-2.8e-3
# beyond the strict bound -- NOT a flipped sample's rank-1 term (flat singular spectrum, |dg| <= 1.8e-5
# max|g|): the f16x3 split of dL/dh under the per-wave running scale of the dWc GEMM (wgrad16.hip BSC)
# keeps 22 bits relative to the wave's largest |dL/dh|, not to each element's own terms; one element
# of 256 in fc_c.2.bias / pts_linears.2.bias; pts_linears.2 / .3.weight one flipped sample's term.
FLIP_FRAC = 3e-3
APARTMENT = [[-5.8, 11.3], [-4.0, 4.5], [-7.9, 4.9]]    # configs/Apartment/apartment.yaml:27


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


def room_points(bound, n, seed):
    """n points on the 6 walls of the room inset 5% in `bound` plus 8 boxes inside it (1 mm jitter)."""
    g = torch.Generator().manual_seed(seed)
    lo, hi = bound[:, 0].float(), bound[:, 1].float()
    span = hi - lo
    rlo, rhi = lo + 0.05 * span, hi - 0.05 * span
    boxes = [(rlo, rhi)]
    for _ in range(8):
        c = rlo + (rhi - rlo) * torch.rand(3, generator=g)
        h = 0.05 + 0.1 * torch.rand(3, generator=g) * span
        boxes.append((torch.maximum(c - h, rlo), torch.minimum(c + h, rhi)))
    pts = []
    per = n // len(boxes)
    for bl, bh in boxes:
        face = torch.randint(0, 6, (per,), generator=g)
        u = bl + (bh - bl) * torch.rand((per, 3), generator=g)
        ax = face // 2
        u[torch.arange(per), ax] = torch.where(face % 2 == 0, bl[ax], bh[ax])
        pts.append(u)
    xyz = torch.cat(pts)
    xyz = xyz + 0.001 * torch.randn(xyz.shape, generator=g)
    feats = 0.1 * torch.randn((xyz.shape[0], 32), generator=g)
    return xyz.contiguous(), feats.contiguous()


def centre_pose(bound, yaw=0.6):
    c = bound.float().mean(1)
    cy, sy = math.cos(yaw), math.sin(yaw)
    c2w = torch.eye(4)
    c2w[:3, :3] = torch.tensor([[cy, 0., sy], [0., 1., 0.], [-sy, 0., cy]])
    c2w[:3, 3] = c
    return c2w


def near_ray_points(xyz, ro, rd, far, reach):
    """Indices of the points within `reach` of any ray segment o + t d, t in [0, far] (ascending)."""
    keep = torch.zeros(xyz.shape[0], dtype=torch.bool)
    for a in range(0, ro.shape[0], 64):
        o, d = ro[a:a + 64], rd[a:a + 64]
        v = xyz[None] - o[:, None]                                    # (r, M, 3)
        t = ((v * d[:, None]).sum(-1) / (d * d).sum(-1)[:, None]).clamp(0, far)
        dist = (v - t[..., None] * d[:, None]).norm(dim=-1)
        keep |= (dist <= reach).any(0)
    return torch.nonzero(keep).reshape(-1)


def scene_case(pnr, dev, bound_cfg, H, W, fx, fy, cx, cy, n_points, n_rays, radius, seed, feat_dtype='float32'):
    bound = RR.scaled_bound(bound_cfg, 0.1, 0.32)
    xyz, feats = room_points(bound, n_points, seed)
    params = RP.init_fc_c(golden_params('trained'), seed=seed)
    c2w = centre_pose(bound)
    g = torch.Generator().manual_seed(seed + 1)
    pix = torch.randint(0, H * W, (n_rays,), generator=g)
    ro, rd = RR.rays_from_uv((pix % W).float(), (pix // W).float(), c2w, fx, fy, cx, cy)
    ro, rd = ro.reshape(-1, 3).contiguous(), rd.reshape(-1, 3).contiguous()
    slam = types.SimpleNamespace(bound=bound, H=H, W=W, fx=fx, fy=fy, cx=cx, cy=cy)
    pts = pnr.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=radius, k=8,
                           feat_dtype=feat_dtype).to(dev)
    return bound, xyz, feats, params, ro, rd, slam, pts


def make_decoder(pnr, params, dev, precision):
    dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    dec.precision = precision
    return dec.to(dev)


def render(pnr, slam, dec, pts, ro, rd, gt, dev, precision):
    cfg = dict(pnr.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr.Renderer(cfg, None, slam)
    with torch.no_grad():
        d, v, c = r.render_batch_ray({'points_color': pts}, dec, rd.to(dev), ro.to(dev), dev, 'color',
                                     gt_depth=None if gt is None else gt.to(dev))
    assert r.status(dev) == 0
    return d.cpu(), v.cpu(), c.cpu(), r


def map_grad_parity(pnr, ms, params, bound, xyz, feats, ro, rd, gt, radius, precision, seed):
    """One MapStep on (ro, rd, gt) leaves the step's gradient in ms.flat.grad; the oracle forms the
    same Mapper loss (render + regulation with the same t_rand, src/Mapper.py:623-655) over the points
    near the rays and its autograd gradient is compared tensor by tensor (points: feature rows)."""
    dev = ms.flat.data.device
    g = torch.Generator().manual_seed(seed)
    n = ro.shape[0]
    col = torch.rand((n, 3), generator=g)
    t_rand = torch.rand((n, 32), generator=g)
    ms(ro.to(dev), rd.to(dev), gt.to(dev), col.to(dev), t_rand.to(dev))
    torch.cuda.synchronize()
    far = float(((bound[:, 1] - bound[:, 0]) ** 2).sum().sqrt()) * 2
    sub = near_ray_points(xyz, ro, rd, far, 2 * radius)
    refs = {}
    for cr in (False, True):
        ref_p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
        fr = feats[sub].clone().requires_grad_(True)
        pdict = dict(xyz=xyz[sub], feats=fr, mode='idw', radius=radius, k=8, eps=1e-6)
        ev = lambda q, ref_p=ref_p, pdict=pdict, cr=cr: RP.eval_points_c(ref_p, q, bound, pdict, cr=cr)  # noqa: E731
        with RP.magnitudes() as mag:  # (recorded by the float32 pass; the CR pass has no hooks)
            d, v, c = RR.render_batch_ray(ref_p, rd, ro, bound, gt_depth=gt, eval_fn=ev)
            sig = RR.regulation(ref_p, rd, ro, gt, bound, t_rand=t_rand, eval_fn=ev)
            RR.mapping_loss(d, c, gt, col, sig).backward()
        refs[cr] = {k: t.grad for k, t in ref_p.items()}
        refs[cr]['feats'] = fr.grad
        if not cr:
            mags = {k: RP.magnitude_of(mag, k).numpy() for k in params}
            mags['feats'] = mag['feats'].numpy()
    got = {}
    off = 0
    from pnr.decoder import PARAM_ORDER, FC_ORDER
    for name, t in zip(PARAM_ORDER + FC_ORDER, ms.flat.params[:-1]):
        got[name] = ms.flat.grad[off:off + t.numel()].view_as(t).cpu()
        off += t.numel()
    got['feats'] = ms.flat.grad[off:].view(-1, 32).cpu()[sub]
    assert float(refs[False]['feats'].abs().max()) > 0, 'the rays must reach neural points'
    for k in got:
        a, b, bcr = got[k].numpy(), refs[False][k].numpy(), refs[True][k].numpy()
        if precision == 'bf16':  # 8-bit operands: a norm bound only
            rel = np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30)
            print(f'{precision} {k}: |g - g_oracle| / |g_oracle| = {rel:.2e}')
            assert rel < 5e-2, (k, rel)
            continue
        # elementwise: rtol 1e-3, atol (1e-6 + d32) max|g_cr| + MAG_ULPS u M vs the correctly-rounded
        # gradient, M = sum_p |t_p| of the element's sum (RP.magnitudes: the float32 rounding floor
        # of a cancelling sum, which no relative bound on g covers), plus the decision-edge allowance
        # of tests/test_gpu_points.py (FLIP_CAP max|g|: ~20k samples x 1,024 ReLU decisions each, a few
        # of which sit within rounding of zero and flip between two float32 orders; measured: one
        # element of 65,536 in dW2 at 1.5e-6 absolute)
        scale = max(np.abs(bcr).max(), 1e-30)
        d32 = np.abs(b - bcr).max() / scale
        atol = (1e-6 + d32) * scale + MAG_ULPS * 2.0 ** -24 * mags[k]
        viol = np.abs(a - bcr) / (1e-3 * np.abs(bcr) + atol)
        maybe_dump_grads(k, a, bcr, b, mags[k], d32, 1e-3, 1e-6, atol)
        print(f'{precision} {k}: d32 {d32:.2e}, worst |g - g_cr| / (rtol |g_cr| + atol) = {viol.max():.3f}, '
              f'beyond: {float(np.mean(viol > 1)):.1e}')
        np.testing.assert_array_less(np.abs(a - bcr), 1e-3 * np.abs(bcr) + atol + FLIP_CAP * scale + 1e-45, err_msg=k)
        assert int(np.sum(viol > 1)) <= max(1, FLIP_FRAC * a.size), (k, float(np.mean(viol > 1)))


def oracle_render(params, bound, xyz, feats, ro, rd, gt, radius):
    far = float(((bound[:, 1] - bound[:, 0]) ** 2).sum().sqrt()) * 2
    sub = near_ray_points(xyz, ro, rd, far, 2 * radius)
    pdict = dict(xyz=xyz[sub], feats=feats[sub], mode='idw', radius=radius, k=8, eps=1e-6)
    ev = lambda q: RP.eval_points_c(params, q, bound, pdict)  # noqa: E731
    with torch.no_grad():
        return RR.render_batch_ray(params, rd, ro, bound, gt_depth=gt, eval_fn=ev)


@pytest.mark.parametrize('precision', ['bf16', 'f16x3'])
def test_c3_office3_200k_points(precision, pnr_mod, dev):
    """C3: office3 scaled bound, 200k neural points (IDW, r = 1 cm, k = 8), the 680x1200 Replica
    camera; 192 rays with gt depth vs the oracle; then Mapper iterations at 1,000 rays."""
    from pnr.mapping import MapStep
    bound, xyz, feats, params, ro, rd, slam, pts = scene_case(
        pnr_mod, dev, OFFICE3, 680, 1200, 600., 600., 599.5, 339.5, 200_000, 192, 0.01, seed=31)
    assert float(bound[0, 1]) > 0.6 and pts.xyz.shape[0] >= 199_000
    dec = make_decoder(pnr_mod, params, dev, precision)
    d0, _, _, _ = render(pnr_mod, slam, dec, pts, ro, rd, None, dev, 'fp32')
    gt = d0.float()
    d, v, c, _ = render(pnr_mod, slam, dec, pts, ro, rd, gt, dev, precision)
    dr, vr, cr = oracle_render(params, bound, xyz, feats, ro, rd, gt, 0.01)
    p = RR.psnr(c.clamp(0, 1), cr.clamp(0, 1))
    print(f'C3 {precision}: PSNR(HIP, fp32 oracle) = {p:.2f} dB')
    if precision == 'bf16':  # 8-bit operands: sigma ~0.4%, depth ~1% (measured 53 dB, depth 1.0e-2)
        assert p > 45.0
        np.testing.assert_allclose(d.numpy(), dr.numpy(), rtol=3e-2, atol=1e-6)
    else:
        np.testing.assert_allclose(d.numpy(), dr.numpy(), rtol=1e-4, atol=1e-9)
        np.testing.assert_allclose(c.numpy(), cr.numpy(), rtol=1e-4, atol=2e-5)
        assert p > 80.0
    # gradient of one Mapper iteration on the 192 rays vs the oracle
    cfg = dict(pnr_mod.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    pts_g = pnr_mod.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.01, k=8).to(dev)
    ms = MapStep(pnr_mod.Renderer(cfg, None, slam), make_decoder(pnr_mod, params, dev, precision), points=pts_g,
                 feat_lr=1e-3)
    # (gt 2% beyond the render: the depth loss's sign(gt - depth) must not hinge on rounding)
    map_grad_parity(pnr_mod, ms, params, bound, xyz, feats, ro, rd, gt * 1.02, 0.01, precision, seed=7)
    # Mapper iterations at the config's batch (mapping.pixels = 1,000), the decoder in `precision`
    cfg = dict(pnr_mod.ROOM0_CFG)
    cfg['pnr'] = {'precision': precision}
    r = pnr_mod.Renderer(cfg, None, slam)
    g = torch.Generator().manual_seed(3)
    pix = torch.randint(0, 680 * 1200, (1000,), generator=g)
    mro, mrd = RR.rays_from_uv((pix % 1200).float(), (pix // 1200).float(), centre_pose(bound), 600., 600.,
                               599.5, 339.5)
    mro, mrd = mro.reshape(-1, 3).to(dev), mrd.reshape(-1, 3).to(dev)
    with torch.no_grad():
        mgt = r.render_batch_ray({'points_color': pts}, dec, mrd, mro, dev, 'color')[0].float()
    ms = MapStep(r, dec, points=pts, feat_lr=1e-3)
    col = torch.rand((1000, 3), generator=g).to(dev)
    losses = [float(ms(mro, mrd, mgt, col, torch.rand((1000, 32), generator=g).to(dev))) for _ in range(3)]
    assert all(math.isfinite(x) for x in losses) and losses[-1] < losses[0]
    assert r.status(dev) == 0


def test_c5_apartment_1m_points_f16(pnr_mod, dev):
    """C5: Apartment scaled bound, 1M neural points with float16 features (64 B each: the budget
    of BASELINE C5), the 720x1280 camera; gather rows and 96 rendered rays vs the oracle; then
    Mapper iterations at mapping.pixels = 5,000."""
    import ctypes
    from pnr.mapping import MapStep
    bound, xyz, feats, params, ro, rd, slam, pts = scene_case(
        pnr_mod, dev, APARTMENT, 720, 1280, 607.4694, 607.4535, 636.9967, 369.2690, 1_000_000, 96, 0.008,
        seed=41, feat_dtype='float16')
    assert pts.xyz.shape[0] >= 999_000
    feats16 = feats.half().float()  # the f16 features are the fp32 master rounded (gather sums in fp32)
    # gather rows: samples along the rays, checked against the oracle over the nearby points
    lib = pnr_mod.library()
    g4 = torch.Generator().manual_seed(4)
    t = torch.rand((ro.shape[0], 64), generator=g4) * 2.0
    q = (ro[:, None] + rd[:, None] * t[..., None]).reshape(-1, 3)
    # plus samples on the surfaces (the rays' own samples are mostly free space)
    q = torch.cat([q, xyz[torch.randint(0, xyz.shape[0], (2048,), generator=g4)] +
                   0.004 * torch.randn((2048, 3), generator=g4)]).double()
    P = q.shape[0]
    c = torch.empty((P, 32), device=dev)
    idx = torch.empty((P, 8), device=dev, dtype=torch.int32)
    w = torch.empty((P, 8), device=dev)
    s, _ = pts.descriptor()
    ws = torch.empty(lib.pnr_point_gather_workspace_bytes(P), dtype=torch.uint8, device=dev)
    qd = q.to(dev).contiguous()
    assert lib.pnr_point_gather(ctypes.byref(s), qd.data_ptr(), P, c.data_ptr(), idx.data_ptr(), w.data_ptr(),
                                ws.data_ptr(), ws.numel(), None) == 0
    torch.cuda.synchronize()
    keep = torch.zeros(xyz.shape[0], dtype=torch.bool)
    keep[near_ray_points(xyz, ro, rd, 2.0, 2 * 0.008)] = True
    qf = q[-2048:].float()
    for a in range(0, 2048, 256):
        keep |= (torch.cdist(qf[a:a + 256], xyz) <= 2 * 0.008).any(0)
    sub = torch.nonzero(keep).reshape(-1)
    c_ref, idx_ref, w_ref = RP.point_gather(q, xyz[sub], feats16[sub], 'idw', radius=0.008, k=8, return_idx=True)
    idx_ref = torch.where(idx_ref >= 0, sub[idx_ref.clamp(min=0)], idx_ref)
    assert (idx_ref >= 0).any(1).sum() > 1500
    assert np.array_equal(idx.cpu().numpy(), idx_ref.numpy().astype(np.int32))
    np.testing.assert_allclose(w.cpu().numpy(), w_ref.numpy(), rtol=0, atol=1e-6)
    np.testing.assert_allclose(c.cpu().numpy(), c_ref.numpy(), rtol=0, atol=1e-5 * float(c_ref.abs().max()))
    # render parity (default precision) on 96 rays
    dec = make_decoder(pnr_mod, params, dev, 'f16x3')
    d, v, col, _ = render(pnr_mod, slam, dec, pts, ro, rd, None, dev, 'f16x3')
    dr, vr, cr = oracle_render(params, bound, xyz, feats16, ro, rd, None, 0.008)
    np.testing.assert_allclose(d.numpy(), dr.numpy(), rtol=1e-4, atol=1e-9)
    np.testing.assert_allclose(col.numpy(), cr.numpy(), rtol=1e-4, atol=2e-5)
    # gradient of one Mapper iteration on the 96 rays (gt = the fp32 render) vs the oracle on the
    # f16-rounded features
    r = pnr_mod.Renderer(pnr_mod.ROOM0_CFG, None, slam)
    # The rays stop at the decoder's own surfaces, in front of the synthetic walls: samples near the
    # walls sit behind the surface (transmittance ~1e-30), so their gradients are ~1e-32 and the check
    # would compare float32 denormal noise.  The last 96 x 8 points of the cloud move onto the rendered
    # surface of the 96 rays (1 cm jitter, fresh features), as Point-NeRF seeds points from depth.
    gs = torch.Generator().manual_seed(9)
    surf = (ro + rd * d.float()[:, None]).repeat(8, 1)
    xyz_g = xyz.clone()
    feats_g = feats.clone()
    xyz_g[-surf.shape[0]:] = surf + 0.01 * torch.randn(surf.shape, generator=gs)
    feats_g[-surf.shape[0]:] = 0.1 * torch.randn((surf.shape[0], 32), generator=gs)
    pts_g = pnr_mod.NeuralPoints(xyz_g.to(dev), feats_g.to(dev), mode='idw', radius=0.03, k=8,
                                 feat_dtype='float16').to(dev)
    ms = MapStep(r, make_decoder(pnr_mod, params, dev, 'f16x3'), points=pts_g, feat_lr=1e-3)
    map_grad_parity(pnr_mod, ms, params, bound, xyz_g, feats_g.half().float(), ro, rd, d.float() * 1.02, 0.03,
                    'f16x3', seed=8)
    # Mapper iterations at 5,000 pixels with the 1M f16-feature cloud
    g = torch.Generator().manual_seed(5)
    pix = torch.randint(0, 720 * 1280, (5000,), generator=g)
    mro, mrd = RR.rays_from_uv((pix % 1280).float(), (pix // 1280).float(), centre_pose(bound), 607.4694,
                               607.4535, 636.9967, 369.2690)
    mro, mrd = mro.reshape(-1, 3).to(dev), mrd.reshape(-1, 3).to(dev)
    with torch.no_grad():
        mgt = r.render_batch_ray({'points_color': pts}, dec, mrd, mro, dev, 'color')[0].float()
    ms = MapStep(r, dec, points=pts, feat_lr=1e-3)
    colr = torch.rand((5000, 3), generator=g).to(dev)
    losses = [float(ms(mro, mrd, mgt, colr, torch.rand((5000, 32), generator=g).to(dev))) for _ in range(3)]
    assert all(math.isfinite(x) for x in losses) and losses[-1] < losses[0]
    # the update reached the float16 copy the gather reads
    assert torch.equal(pts._feats_for_gather(), pts.feats.detach().half())
