"""Parity of the HIP renderer (libpnr.so through the pnr host mirror) against the reference's
golden vectors (tests/golden, made by importing the reference) and the CPU oracle.

Tolerances (north_star: depth/colour within 1e-4 relative):
  depth      rtol 1e-4 (atol 1e-6 in the render_img frame, whose zero-gt columns have depths
             ~1e-3 where 1e-7 absolute is already 1e-4 relative)
  colour     rtol 1e-4, atol 2e-5   (absolute floor for near-zero channels)
  variance   rtol 2e-3, atol 1e-8   (a cancellation-heavy second moment: fp32 reordering of the
             MLP sums alone moves it ~6e-5 relative on CPU, measured)
  raw MLP    atol 2e-5 * max|raw|
  gradients  decoder (Mapper) atol 2e-3 * max|g| per tensor here, and ELEMENTWISE in
             test_gpu_precision.py; Tracker ray / camera-tensor gradients ELEMENTWISE (grad_elementwise):
             rtol 1e-3 with atol 1e-6 * max|g| against the correctly-rounded gradient
             (tests/golden/grads_cr.npz), and atol (1e-6 + golden_vs_cr) * max|g| against the
             reference's float32 gradient (its own summation-order rounding, recorded in grads_cr.npz)
"""
import numpy as np
import pytest
import torch

from conftest import load_golden, golden_params

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=['fp32', 'f16x3'])
def precision(request, monkeypatch):
    """Every GPU test runs under both decoder precisions (include/pnr.h PNR_PREC_*): the exact
    fp32 MFMA path and the f16x3 split path (the default), against the same tolerances."""
    from pnr import _lib
    monkeypatch.setattr(_lib, 'DEFAULT_PRECISION', request.param)
    return request.param

CASES = [f'p{i}_{c}' for i in range(4) for c in ('none', 'gt', 'gtzero')] + ['rand_none', 'edge_none']


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


def make_decoder(pnr, params, dev):
    dec = pnr.MLP(dim=3, c_dim=0, color=True, hidden_size=256, skips=[], n_blocks=4, pos_embedding_method='fourier')
    dec.load_state_dict({k: v.clone() for k, v in params.items()})
    return dec.to(dev)


def make_renderer(pnr, scene, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5, **kw):
    import types
    slam = types.SimpleNamespace(bound=scene['bound_t'], H=H, W=W, fx=fx, fy=fy, cx=cx, cy=cy)
    return pnr.Renderer(pnr.ROOM0_CFG, None, slam, **kw)


def close(a, b, rtol, atol, what):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = b.detach().cpu().numpy() if isinstance(b, torch.Tensor) else np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=atol, err_msg=what)


GRAD_RTOL, GRAD_ATOL = 1e-3, 1e-6


def grad_elementwise(g, cr, f32, rel_f32, what):
    """|g - g_cr| <= 1e-3 |g_cr| + 1e-6 max|g_cr| elementwise (the correctly-rounded gradient), and
    |g - g_f32| <= 1e-3 |g_f32| + (1e-6 + rel_f32) max|g_f32| (the reference's float32 gradient,
    which sits rel_f32 * max from the correctly-rounded one)."""
    g = g.detach().cpu().numpy() if isinstance(g, torch.Tensor) else np.asarray(g)
    for ref, atol_rel, tag in ((cr, GRAD_ATOL, 'correctly rounded'), (f32, GRAD_ATOL + float(rel_f32), 'float32')):
        ref = np.asarray(ref)
        atol = atol_rel * np.abs(ref).max()
        viol = np.abs(g - ref) / (GRAD_RTOL * np.abs(ref) + atol)
        print(f'{what} vs {tag}: worst |g - g_ref| / (rtol |g_ref| + atol) = {viol.max():.3f}')
        np.testing.assert_allclose(g, ref, rtol=GRAD_RTOL, atol=atol, err_msg=f'{what} vs {tag}')


def test_library_info(pnr_mod):
    lib = pnr_mod.library()
    assert lib.pnr_abi_version() == 14
    assert lib.pnr_mlp_packed_floats() > 0


def test_eval_points_golden(pnr_mod, dev, scene, trained_params):
    z = load_golden('points.npz')
    dec = make_decoder(pnr_mod, trained_params, dev)
    r = make_renderer(pnr_mod, scene)
    raw = r.eval_points(torch.from_numpy(z['p']).to(dev), dec)
    ref = z['raw']
    close(raw, ref, 0, 2e-5 * np.abs(ref).max(), 'raw')
    # the bound mask (strict, float64) must agree exactly
    assert np.array_equal(raw[:, 3].cpu().numpy() == 100., ref[:, 3] == 100.)


@pytest.mark.parametrize('case', CASES)
def test_render_batch_ray_golden(case, pnr_mod, dev, scene):
    g = load_golden('render.npz')
    params = golden_params('random' if case.startswith('rand') else 'trained')
    dec = make_decoder(pnr_mod, params, dev)
    r = make_renderer(pnr_mod, scene)
    ro = torch.from_numpy(g[f'{case}/rays_o']).to(dev)
    rd = torch.from_numpy(g[f'{case}/rays_d']).to(dev)
    gt = torch.from_numpy(g[f'{case}/gt_depth']).to(dev) if f'{case}/gt_depth' in g else None
    with torch.no_grad():
        d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
    assert d.dtype == torch.float64 and v.dtype == torch.float64 and c.dtype == torch.float32
    close(d, g[f'{case}/depth'], 1e-4, 1e-9, 'depth')
    close(c, g[f'{case}/rgb'], 1e-4, 2e-5, 'rgb')
    close(v, g[f'{case}/var'], 2e-3, 1e-8, 'var')


def test_mlp_forward_backward_vs_oracle(pnr_mod, dev, trained_params):
    from oracle import ref_render as ref
    torch.manual_seed(0)
    P = 3000  # not a multiple of 128: exercises the padded tail
    pts = torch.rand(P, 3) * 0.8 - 0.3
    g_raw = torch.randn(P, 4)
    cpu_p = {k: v.clone().requires_grad_(True) for k, v in trained_params.items()}
    x = pts.clone().requires_grad_(True)
    out = ref.mlp_forward(cpu_p, x)
    (out * g_raw).sum().backward()
    dec = make_decoder(pnr_mod, trained_params, dev)
    xg = pts.to(dev).requires_grad_(True)
    outg = dec(xg)
    close(outg, out.detach(), 0, 2e-5 * out.abs().max().item(), 'mlp out')
    (outg * g_raw.to(dev)).sum().backward()
    for k, prm in dec.named_parameters():
        gref = cpu_p[k].grad
        close(prm.grad, gref, 0, 2e-3 * gref.abs().max().item(), f'grad {k}')
    close(xg.grad, x.grad, 0, 2e-3 * x.grad.abs().max().item(), 'grad x')


def test_mapping_grads_golden(pnr_mod, dev, scene):
    """Mapper.optimize_map loss (src/Mapper.py:628-655) incl. regulation, vs reference autograd."""
    G = load_golden('grads.npz')
    dec = make_decoder(pnr_mod, golden_params('trained'), dev)
    r = make_renderer(pnr_mod, scene)
    ro = torch.from_numpy(G['map_rays_o']).to(dev)
    rd = torch.from_numpy(G['map_rays_d']).to(dev)
    gt = torch.from_numpy(G['map_gt_depth']).to(dev)
    gcol = torch.from_numpy(G['map_gt_color']).to(dev)
    d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
    sig = r.regulation({}, dec, rd, ro, gt, dev, 'color', t_rand=torch.from_numpy(G['map_t_rand']).to(dev))
    close(sig, G['map_sigma'], 0, 2e-5 * np.abs(G['map_sigma']).max(), 'sigma_reg')
    m = gt > 0
    loss = torch.abs(gt[m] - d[m]).sum() + 0.05 * torch.abs(gcol - c).sum() + 0.0005 * torch.abs(sig).sum()
    close(loss.detach(), float(G['map_loss']), 1e-5, 0, 'loss')
    loss.backward()
    for k, prm in dec.named_parameters():
        gref = G[f'map_grad/{k}']
        close(prm.grad, gref, 0, 2e-3 * np.abs(gref).max(), f'grad {k}')


def test_tracking_ray_grads_golden(pnr_mod, dev, scene):
    """Tracker.optimize_cam_in_batch loss (src/Tracker.py:306-330): grads reach rays_o / rays_d,
    elementwise against the correctly-rounded and the reference's float32 gradients."""
    G = load_golden('grads.npz')
    CR = load_golden('grads_cr.npz')
    dec = make_decoder(pnr_mod, golden_params('trained'), dev)
    for p_ in dec.parameters():
        p_.requires_grad_(False)
    r = make_renderer(pnr_mod, scene)
    ro = torch.from_numpy(G['map_rays_o']).to(dev).requires_grad_(True)
    rd = torch.from_numpy(G['map_rays_d']).to(dev).requires_grad_(True)
    gt = torch.from_numpy(G['map_gt_depth']).to(dev)
    gcol = torch.from_numpy(G['map_gt_color']).to(dev)
    d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
    m = gt > 0
    loss = (torch.abs(gt - d) / torch.sqrt(v.detach() + 1e-10))[m].sum() + 0.5 * torch.abs(gcol - c)[m].sum()
    close(loss.detach(), float(G['trk_loss']), 1e-4, 0, 'loss')
    loss.backward()
    for a, t in (('o', ro), ('d', rd)):
        grad_elementwise(t.grad, CR[f'trk_grad_rays_{a}'], G[f'trk_grad_rays_{a}'], CR[f'golden_vs_cr/trk_rays_{a}'],
                         f'rays_{a}')


def test_masks_only_save_equals_full_save_ray_grads(pnr_mod, dev, scene):
    """ABI 8 save_for_backward = 2 (decoder frozen: the Tracker's step): the forward keeps only the
    ReLU masks and inputs, and the ray gradients equal those of a full-save forward whose decoder
    gradients are requested too (same kernels on the same values: bit-identical)."""
    G = load_golden('grads.npz')
    r = make_renderer(pnr_mod, scene)
    gt = torch.from_numpy(G['map_gt_depth']).to(dev)
    out = {}
    for frozen in (True, False):
        dec = make_decoder(pnr_mod, golden_params('trained'), dev)
        for p_ in dec.parameters():
            p_.requires_grad_(not frozen)
        ro = torch.from_numpy(G['map_rays_o']).to(dev).requires_grad_(True)
        rd = torch.from_numpy(G['map_rays_d']).to(dev).requires_grad_(True)
        d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
        (d.sum() + 0.5 * c.sum() + v.sum()).backward()
        out[frozen] = (ro.grad.clone(), rd.grad.clone(), d.detach().clone())
        assert all((p_.grad is None) == frozen for p_ in dec.parameters())
    for a, b in zip(out[True], out[False]):
        assert torch.equal(a, b)


def test_render_img_golden(pnr_mod, dev, scene):
    z = load_golden('render_img.npz')
    dec = make_decoder(pnr_mod, golden_params('trained'), dev)
    r = make_renderer(pnr_mod, scene, H=int(z['H']), W=int(z['W']), fx=float(z['fx']), fy=float(z['fy']),
                      cx=float(z['cx']), cy=float(z['cy']), ray_batch_size=int(z['ray_batch_size']))
    d, v, c = r.render_img({}, dec, torch.from_numpy(z['c2w']).to(dev), dev, 'color',
                           gt_depth=torch.from_numpy(z['gt_depth']).to(dev))
    close(d, z['depth'], 1e-4, 1e-6, 'depth')
    close(c, z['rgb'], 1e-4, 2e-5, 'rgb')
    close(v, z['var'], 2e-3, 1e-8, 'var')


def test_rays_vs_oracle(pnr_mod, dev, scene):
    from oracle import ref_render as ref
    c2w = torch.from_numpy(scene['poses'][1])
    ro, rd = pnr_mod.get_rays(48, 64, 50., 51., 31.5, 23.5, c2w.to(dev), dev)
    ro_r, rd_r = ref.full_frame_rays(48, 64, 50., 51., 31.5, 23.5, c2w)
    close(ro, ro_r, 0, 0, 'rays_o')
    close(rd, rd_r, 1e-6, 1e-7, 'rays_d')
    i = torch.tensor([0., 5., 1199., 17.]); j = torch.tensor([0., 9., 679., 300.])
    ro2, rd2 = pnr_mod.get_rays_from_uv(i.to(dev), j.to(dev), c2w.to(dev), 680, 1200, 600., 600., 599.5, 339.5, dev)
    ro2r, rd2r = ref.rays_from_uv(i, j, c2w, 600., 600., 599.5, 339.5)
    close(rd2, rd2r.reshape(-1, 3), 1e-6, 1e-7, 'uv rays_d')
    close(ro2, ro2r.reshape(-1, 3), 0, 0, 'uv rays_o')


def test_window_batch_vs_oracle(pnr_mod, dev, scene):
    """Mapper.optimize_map's per-iteration batch (src/Mapper.py:560-606): pixs_per_image uniform
    pixels per window frame through get_samples (src/common.py:110-134), concatenated."""
    from oracle import ref_render as ref
    from pnr.mapping import window_batch
    H, W, fx, fy, cx, cy = 48, 64, 50., 51., 31.5, 23.5
    g = torch.Generator().manual_seed(5)
    frames = []
    for k in (1, 2):
        c2w = torch.from_numpy(scene['poses'][k]).float()
        frames.append((c2w, torch.rand((H, W), generator=g), torch.rand((H, W, 3), generator=g)))
    n = 100
    gen = torch.Generator(device=dev).manual_seed(7)
    ro, rd, gd, gc = window_batch([(c.to(dev), d.to(dev), col.to(dev)) for c, d, col in frames], n, H, W,
                                  fx, fy, cx, cy, dev, generator=gen)
    assert ro.shape == (2 * n, 3) and gd.shape == (2 * n,) and gc.shape == (2 * n, 3)
    gen = torch.Generator(device=dev).manual_seed(7)
    for f, (c2w, d, col) in enumerate(frames):
        idx = torch.randint(H * W, (n,), device=dev, generator=gen).cpu()
        i, j = (idx % W).float(), (idx // W).float()
        ro_r, rd_r = ref.rays_from_uv(i, j, c2w, fx, fy, cx, cy)
        sl = slice(f * n, (f + 1) * n)
        close(rd[sl], rd_r.reshape(-1, 3), 1e-6, 1e-7, 'rays_d')
        close(ro[sl], ro_r.reshape(-1, 3), 0, 0, 'rays_o')
        assert torch.equal(gd[sl].cpu(), d.reshape(-1)[idx]) and torch.equal(gc[sl].cpu(), col.reshape(-1, 3)[idx])


def test_window_rays_equal_window_batch(pnr_mod, dev, scene):
    """pnr_window_rays (the whole window batch in one launch, pnr.mapping.WindowSampler) gives the
    values of window_batch's per-frame get_samples on the same pixel indices, bit for bit; the
    WindowSampler draws one uniform index per ray over the whole image, 5 frames x 200 pixels."""
    from pnr.mapping import WindowSampler, window_batch, window_rays
    H, W, fx, fy, cx, cy = 68, 120, 60., 61., 59.5, 33.5
    g = torch.Generator().manual_seed(6)
    frames = []
    for k in (0, 1, 2, 3, 2):
        c2w = torch.from_numpy(scene['poses'][k]).float()
        frames.append((c2w.to(dev), torch.rand((H, W), generator=g).to(dev), torch.rand((H, W, 3), generator=g).to(dev)))
    n = 200
    ref = window_batch(frames, n, H, W, fx, fy, cx, cy, dev, generator=torch.Generator(device=dev).manual_seed(9))
    gen = torch.Generator(device=dev).manual_seed(9)
    idx = torch.cat([torch.randint(H * W, (n,), device=dev, generator=gen) for _ in frames])
    c2w = torch.stack([f[0] for f in frames])
    out = window_rays(idx, n, c2w, torch.stack([f[1] for f in frames]), torch.stack([f[2] for f in frames]),
                      fx, fy, cx, cy)
    for a, b, what in zip(out, ref, ('rays_o', 'rays_d', 'gt depth', 'gt colour')):
        assert torch.equal(a, b), what
    ws = WindowSampler(frames, n, fx, fy, cx, cy, generator=torch.Generator(device=dev).manual_seed(3),
                       device_rng=False)
    ro, rd, gd, gc, tr, far = ws()
    assert ro.shape == (5 * n, 3) and tr.shape == (5 * n, 32) and gd.shape == (5 * n,) and far is None
    assert bool((tr >= 0).all() and (tr < 1).all())


def test_window_sample_device_draws(pnr_mod, dev, scene):
    """pnr_window_sample (the batch drawn on the device in one launch): its rays and gt are
    pnr_window_rays' on the pixels it drew, bit for bit; far clamp = max(1.2 gt) exactly (the value
    Renderer.py:112 computes); every call draws a new batch (device counter), a fresh state with
    the same seed repeats the sequence, another seed does not; draws are uniform: pixel rows /
    columns and jitter means within 5 sigma of uniform over 100 batches (parity of the distribution,
    not of torch's Philox sequence -- documented in include/pnr.h)."""
    from pnr.mapping import WindowSampler, window_rays
    H, W, fx, fy, cx, cy = 68, 120, 60., 61., 59.5, 33.5
    g = torch.Generator().manual_seed(7)
    frames = []
    for k in (0, 1, 2, 3, 2):
        c2w = torch.from_numpy(scene['poses'][k]).float()
        frames.append((c2w.to(dev), torch.rand((H, W), generator=g).to(dev), torch.rand((H, W, 3), generator=g).to(dev)))
    n = 200
    ws = WindowSampler(frames, n, fx, fy, cx, cy, seed=11)
    c2w = torch.stack([f[0] for f in frames])
    dep, col = torch.stack([f[1] for f in frames]), torch.stack([f[2] for f in frames])
    idxs, trs = [], []
    for it in range(100):
        ro, rd, gd, gc, tr, far = ws()
        idx = ws.idx.clone()
        if it < 3:
            ref = window_rays(idx, n, c2w, dep, col, fx, fy, cx, cy)
            for a, b, what in zip((ro, rd, gd, gc), ref, ('rays_o', 'rays_d', 'gt depth', 'gt colour')):
                assert torch.equal(a, b), what
            assert torch.equal(far, (gd * 1.2).max().reshape(1)), 'far clamp'
        idxs.append(idx)
        trs.append(tr.clone())
    idx = torch.stack(idxs)
    assert bool(((idx >= 0) & (idx < H * W)).all())
    assert not torch.equal(idxs[0], idxs[1])
    ws2 = WindowSampler(frames, n, fx, fy, cx, cy, seed=11)
    ws2()
    assert torch.equal(ws2.idx, idxs[0])
    ws3 = WindowSampler(frames, n, fx, fy, cx, cy, seed=12)
    ws3()
    assert not torch.equal(ws3.idx, idxs[0])
    tr = torch.stack(trs).double()
    assert bool((tr >= 0).all() and (tr < 1).all())
    N = tr.numel()
    assert abs(tr.mean().item() - 0.5) < 5 * (1 / 12) ** 0.5 / N ** 0.5
    for cnt, k in ((torch.bincount((idx // W).reshape(-1), minlength=H), H),
                   (torch.bincount((idx % W).reshape(-1), minlength=W), W)):
        e = idx.numel() / k
        chi2 = (((cnt.double() - e) ** 2) / e).sum().item()
        assert abs(chi2 - (k - 1)) < 5 * (2 * (k - 1)) ** 0.5, chi2


def test_adam_matches_torch(pnr_mod, dev):
    import ctypes
    lib = pnr_mod.library()
    torch.manual_seed(1)
    p = torch.randn(10007, device=dev)
    p_ref = p.clone().requires_grad_(True)
    opt = torch.optim.Adam([p_ref], lr=2e-4)
    m = torch.zeros_like(p); v = torch.zeros_like(p)
    for step in range(1, 4):
        g = torch.randn_like(p)
        p_ref.grad = g.clone()
        opt.step()
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        rc = lib.pnr_adam_step(ctypes.c_void_p(p.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                               ctypes.c_void_p(m.data_ptr()), ctypes.c_void_p(v.data_ptr()), p.numel(), 2e-4, 0.9,
                               0.999, 1e-8, step, st)
        assert rc == 0
    close(p, p_ref.detach(), 1e-6, 1e-7, 'adam')


def test_batch_invariance_with_global_far(pnr_mod, dev, scene):
    """Size-independent property at a large batch: with the far clamp fixed (the sharded mode of
    Renderer.py:112), rendering a batch whole or in 7 uneven slices gives identical bits."""
    dec = make_decoder(pnr_mod, golden_params('trained'), dev)
    r = make_renderer(pnr_mod, scene)
    from oracle import ref_render as ref
    N = 40000
    g = torch.Generator().manual_seed(3)
    pix = torch.randint(0, 680 * 1200, (N,), generator=g)
    ro, rd = ref.rays_from_uv((pix % 1200).float(), (pix // 1200).float(), torch.from_numpy(scene['poses'][2]),
                              600., 600., 599.5, 339.5)
    ro, rd = ro.reshape(-1, 3).contiguous().to(dev), rd.reshape(-1, 3).contiguous().to(dev)
    gt = (torch.rand(N, generator=g) * 0.5 + 0.1).to(dev)
    fc = float((gt * 1.2).max())
    with torch.no_grad():
        d, v, c = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt)
        d2, v2, c2 = r.render_batch_ray({}, dec, rd, ro, dev, 'color', gt_depth=gt, far_clamp=fc)
        cuts = [0, 1, 129, 5000, 5001, 17000, 33333, N]
        parts = [r.render_batch_ray({}, dec, rd[a:b], ro[a:b], dev, 'color', gt_depth=gt[a:b], far_clamp=fc)
                 for a, b in zip(cuts[:-1], cuts[1:])]
    for t_full, t_alt in ((d, d2), (v, v2), (c, c2)):
        assert torch.equal(t_full, t_alt)
    assert torch.equal(torch.cat([p[0] for p in parts]), d)
    assert torch.equal(torch.cat([p[2] for p in parts]), c)
    assert torch.isfinite(d).all() and torch.isfinite(c).all()


@pytest.fixture(scope='module')
def oracle_frame(scene):
    """Oracle render of a strided 170x300 sub-frame of room0 pose 1000 (trained decoder)."""
    from oracle import ref_render as ref
    params = golden_params('trained')
    c2w = torch.from_numpy(scene['poses'][2])
    ro, rd = ref.full_frame_rays(680, 1200, 600., 600., 599.5, 339.5, c2w)
    ro, rd = ro[::4, ::4].reshape(-1, 3).contiguous(), rd[::4, ::4].reshape(-1, 3).contiguous()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    dr, vr, cr = ref.render_batch_ray(params, rd, ro, scene['bound_t'])
    return params, ro, rd, dr, vr, cr


def test_psnr_bf16_frame(pnr_mod, dev, scene, oracle_frame):
    """BASELINE config C3 (bf16 MLP on MFMA): PSNR(HIP bf16 render, oracle fp32 render) on the
    same sub-frame.  bf16 operands are not fp32-faithful; the bar is the 0.1 dB PSNR budget, shown
    here as a PSNR against the fp32 render far above the frame's own PSNR scale (> 50 dB)."""
    from oracle import ref_render as ref
    params, ro, rd, dr, vr, cr = oracle_frame
    dec = make_decoder(pnr_mod, params, dev)
    dec.precision = 'bf16'
    r = make_renderer(pnr_mod, scene)
    r.precision = 'bf16'
    with torch.no_grad():
        d, v, c = r.render_batch_ray({}, dec, rd.to(dev), ro.to(dev), dev, 'color')
    p = ref.psnr(c.cpu().clamp(0, 1), cr.clamp(0, 1))
    print(f'PSNR(bf16 HIP, fp32 oracle) = {p:.2f} dB')
    assert p > 50.0, p


def test_psnr_vs_oracle_frame(pnr_mod, dev, scene, oracle_frame):
    """PSNR(HIP render, oracle render) on a strided 170x300 sub-frame of room0 pose 1000: far
    above the 39 dB margin that bounds the PSNR delta vs ground truth by 0.1 dB."""
    from oracle import ref_render as ref
    params, ro, rd, dr, vr, cr = oracle_frame
    dec = make_decoder(pnr_mod, params, dev)
    r = make_renderer(pnr_mod, scene)
    with torch.no_grad():
        d, v, c = r.render_batch_ray({}, dec, rd.to(dev), ro.to(dev), dev, 'color')
    p = ref.psnr(c.cpu().clamp(0, 1), cr.clamp(0, 1))
    assert p > 80.0, p
    close(d, dr, 1e-4, 1e-9, 'depth')


def _track_scene(scene):
    """A 68x120 frame (edge 10 px) rendered by the oracle at room0 pose 1, every 7th row / 5th
    column depth zeroed, and a camera tensor perturbed off that pose."""
    from oracle import ref_render as ref
    import pnr
    params = golden_params('trained')
    H, W, fx, fy, cx, cy = 68, 120, 60., 60., 59.5, 33.5
    c2w = torch.from_numpy(scene['poses'][1]).float()
    gd, _, gc = ref.render_img(params, c2w, scene['bound_t'], H, W, fx, fy, cx, cy)
    gd = gd.float().clone()
    gd[::7, ::5] = 0.
    ct_true = pnr.get_tensor_from_camera(c2w)
    ct0 = ct_true + torch.tensor([0.003, -0.002, 0.001, 0.002, 0.004, -0.003, 0.002])
    return params, (H, W, fx, fy, cx, cy), gd, gc.float(), ct_true, ct0


def test_track_step_vs_oracle(pnr_mod, dev, scene):
    """Tracker.optimize_cam_in_batch (src/Tracker.py:253-335, weak depth): loss and camera-tensor
    gradient of one step vs the oracle (rays, render and loss restated on the CPU), elementwise
    against the correctly-rounded and the float32-oracle gradients of tests/golden/grads_cr.npz
    (the frame and the start camera are the fixture's, made by tests/golden/make_grads_cr.py)."""
    CR = load_golden('grads_cr.npz')
    params = golden_params('trained')
    H, W, fx, fy, cx, cy = 68, 120, 60., 60., 59.5, 33.5
    e = 10
    gd, gc, ct0 = (torch.from_numpy(CR[f'cam/{k}']) for k in ('gt_depth', 'gt_color', 'ct0'))
    dec = make_decoder(pnr_mod, params, dev)
    r = make_renderer(pnr_mod, scene, H=H, W=W, fx=fx, fy=fy, cx=cx, cy=cy)
    step = pnr_mod.TrackStep(r, dec, ignore_edge_W=e, ignore_edge_H=e)
    ct = ct0.clone().to(dev).requires_grad_(True)
    loss = step.loss(ct, gc.to(dev), gd.to(dev), 0)
    loss.backward()
    assert all(p.grad is None for p in dec.parameters())  # the Tracker optimises the camera only
    close(loss.detach(), float(CR['cam/loss_f32']), 1e-4, 0, 'tracking loss')
    grad_elementwise(ct.grad, CR['cam/grad_cr'], CR['cam/grad_f32'], CR['golden_vs_cr/cam'], 'camera tensor grad')


def test_track_frame_converges(pnr_mod, dev, scene):
    """src/Tracker.py:860-921: 12 Adam iterations from the perturbed pose lower the loss, and the
    minimum-loss candidate is closer to the rendering pose than the start."""
    params, (H, W, fx, fy, cx, cy), gd, gc, ct_true, ct0 = _track_scene(scene)
    dec = make_decoder(pnr_mod, params, dev)
    r = make_renderer(pnr_mod, scene, H=H, W=W, fx=fx, fy=fy, cx=cx, cy=cy)
    step = pnr_mod.TrackStep(r, dec, ignore_edge_W=10, ignore_edge_H=10)
    best, c2w, losses = pnr_mod.track_frame(step, ct0.to(dev), gc.to(dev), gd.to(dev), 12, 1e-3, 0)
    assert len(losses) == 12 and min(losses) < 0.7 * losses[0]
    err0 = (ct0 - ct_true).abs().mean().item()
    err = (best.cpu() - ct_true).abs().mean().item()
    assert err < err0
    assert c2w.shape == (4, 4)


def test_map_graph_matches_eager(pnr_mod, dev, scene):
    """pnr.mapping.MapGraph: the mapping iteration captured in a HIP graph and replayed gives the
    same weights and losses as the same iterations run eagerly (device-step Adam in both), bit for
    bit: the backward's gradient sums have a fixed order."""
    from pnr.mapping import MapStep, MapGraph
    params = golden_params('trained')
    g = torch.Generator().manual_seed(5)
    n = 1024
    c2w = torch.from_numpy(scene['poses'][1]).float()
    i = torch.randint(0, 1200, (n,), generator=g).float()
    j = torch.randint(0, 680, (n,), generator=g).float()
    ro, rd = pnr_mod.get_rays_from_uv(i.to(dev), j.to(dev), c2w.to(dev), 680, 1200, 600., 600., 599.5, 339.5, dev)
    batches = []
    for s in range(4):
        gt = (torch.rand(n, generator=g) * 0.4 + 0.15).to(dev)
        col = torch.rand((n, 3), generator=g).to(dev)
        t_rand = torch.rand((n, 32), generator=g).to(dev)
        batches.append((ro, rd, gt, col, t_rand))
    runs = []
    for graph in (False, True):
        dec = make_decoder(pnr_mod, params, dev)
        r = make_renderer(pnr_mod, scene)
        ms = MapStep(r, dec, lr=2e-4, w_color_loss=0.05)
        ms.opt.use_device_step()
        losses = []
        if graph:
            mg = MapGraph(ms, *batches[0], warmup=2)  # two eager steps on batch 0, then the capture
            for b in batches[1:]:
                losses.append(float(mg(*b)))
        else:
            for _ in range(2):
                ms(*batches[0])
            for b in batches[1:]:
                losses.append(float(ms(*b)))
        torch.cuda.synchronize()
        runs.append((losses, ms.flat.data.detach().cpu().clone(), int(ms.opt.step_dev[0].item())))
    (l_e, w_e, s_e), (l_g, w_g, s_g) = runs
    assert s_e == s_g == 5
    # every weight-gradient GEMM flushes per-workgroup partials that k_part_reduce sums in a fixed
    # order (no float atomics): the replayed iterations equal the eager ones bit for bit
    assert l_g == l_e, (l_g, l_e)
    assert torch.equal(w_g, w_e), int((w_g != w_e).sum())
