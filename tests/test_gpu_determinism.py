"""Determinism of the mapping step on the HIP path, with and without neural points.

Every sum of the backward has a fixed result whatever the scheduling: the weight-gradient GEMMs
store per-workgroup partial tiles that one launch adds in a fixed order, and the point-feature
gradient (pnr_point_gather_bwd ABI 10) is an exact int64 fixed-point sum.  So:
  * two runs of a neural-point MapStep are bitwise equal (src/Mapper.py:657-662 on the features);
  * a neural-point MapStep captured in a HIP graph (pnr.MapGraph) replays bitwise like the eager step;
  * the map pass (render + regulation as one decoder pass, pnr_map_fwd / _bwd) gives the two-chain
    outputs bit for bit and its gradients to float32 association;
  * the two-chain MapStep with the regulation chain on a side stream (overlap) equals the serial one bitwise;
  * the fused Mapper loss (pnr_map_loss, src/Mapper.py:628-655) and its gradients equal the
    autograd drop-in path (render_batch_ray + regulation + the torch loss, MapStep.loss).
Run under both decoder precisions (fp32 MFMA and the default f16x3).
"""
import pytest
import torch

from conftest import golden_params, load_golden
from oracle import ref_points as RP

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=['fp32', 'f16x3'])
def precision(request, monkeypatch):
    from pnr import _lib
    monkeypatch.setattr(_lib, 'DEFAULT_PRECISION', request.param)
    return request.param


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


def _renderer(pnr, bound):
    import types
    slam = types.SimpleNamespace(bound=bound, H=680, W=1200, fx=600., fy=600., cx=599.5, cy=339.5)
    return pnr.Renderer(pnr.ROOM0_CFG, None, slam)


def _setup(pnr, dev, n=512, points=True, seed=4):
    """Rays at the golden pose-1000 surface (gt = rendered depth), neural points scattered around
    it, the trained decoder (+ seeded fc_c), and 4 batches (gt colour, jitter) for 4 steps."""
    r = load_golden('render.npz')
    ro = torch.from_numpy(r['p2_gt/rays_o'])[:n]
    rd = torch.from_numpy(r['p2_gt/rays_d'])[:n]
    gt = torch.from_numpy(r['p2_gt/gt_depth'])[:n]
    gen = torch.Generator().manual_seed(seed)
    surf = ro + rd * gt[:, None]
    xyz = (surf.repeat(4, 1) + 0.01 * torch.randn((4 * n, 3), generator=gen)).float()
    feats = torch.randn((xyz.shape[0], 32), generator=gen) * 0.5
    batches = [(ro.to(dev), rd.to(dev), gt.to(dev), torch.rand((n, 3), generator=gen).to(dev),
                torch.rand((n, 32), generator=gen).to(dev)) for _ in range(4)]
    base = golden_params('trained')
    params = RP.init_fc_c(base, seed=1) if points else base
    bound = torch.from_numpy(load_golden('scene.npz')['bound'])

    def make():
        if points:
            dec = pnr.MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256)
            pts = pnr.NeuralPoints(xyz.to(dev), feats.to(dev), mode='idw', radius=0.04, k=8).to(dev)
        else:
            dec = pnr.get_model(pnr.ROOM0_CFG, nice=False)
            pts = None
        dec.load_state_dict({k: v.clone() for k, v in params.items()})
        return _renderer(pnr, bound), dec.to(dev), pts
    return make, batches


@pytest.mark.parametrize('points', [True, False])
def test_map_step_reruns_bitwise(pnr_mod, dev, points):
    """Two runs of the same 3 mapping steps give identical losses, gradients and parameters."""
    from pnr.mapping import MapStep
    make, batches = _setup(pnr_mod, dev, points=points)
    runs = []
    for _ in range(2):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2)
        losses = [float(ms(*b)) for b in batches[:3]]
        torch.cuda.synchronize()
        runs.append((losses, ms.flat.grad.clone(), ms.flat.data.clone()))
    assert runs[0][0] == runs[1][0]
    assert torch.equal(runs[0][1], runs[1][1])
    assert torch.equal(runs[0][2], runs[1][2])


def test_points_map_graph_matches_eager(pnr_mod, dev):
    """pnr.MapGraph over a neural-point MapStep (gather, fc_c injection, deterministic feature
    backward, two Adam segments): the replayed iterations equal the eager ones bit for bit."""
    from pnr.mapping import MapGraph, MapStep
    make, batches = _setup(pnr_mod, dev, points=True)
    runs = []
    for graph in (False, True):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2)
        ms.opt.use_device_step()
        losses = []
        if graph:
            mg = MapGraph(ms, *batches[0], warmup=2)
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
    assert l_g == l_e, (l_g, l_e)
    assert torch.equal(w_g, w_e)


@pytest.mark.parametrize('points', [True, False])
def test_map_step_overlap_equals_serial(pnr_mod, dev, points):
    """The two-chain MapStep (fused=False): overlap=True runs the regulation chain on a side stream with its own gradient
    buffer and adds it after the join; overlap=False accumulates both chains into one buffer on
    the caller's stream.  Both add the same two per-chain sums once: the gradients are bitwise equal."""
    from pnr.mapping import MapStep
    make, batches = _setup(pnr_mod, dev, points=points)
    out = []
    for ov in (True, False):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2, overlap=ov, fused=False)
        assert ms._overlaps(batches[0][0].shape[0]) == ov
        loss = float(ms(*batches[0]))
        torch.cuda.synchronize()
        out.append((loss, ms.flat.grad.clone(), ms.flat.data.clone()))
    assert out[0][0] == out[1][0]
    assert torch.equal(out[0][1], out[1][1])
    assert torch.equal(out[0][2], out[1][2])


@pytest.mark.parametrize('points', [True, False])
def test_fused_map_loss_matches_autograd(pnr_mod, dev, points, precision):
    """The fused path (TrainPass + pnr_map_loss) against the drop-in autograd path
    (Renderer.render_batch_ray / regulation + the reference's loss in torch, MapStep.loss): the loss
    and every gradient (decoder, fc_c, point features).  The two reach the same kernels with the same
    upstream gradients (sign terms), so the gradients agree to float32 association (the fused step sums
    the render and regulation samples in one GEMM, the autograd path in two)."""
    from pnr.mapping import MapStep
    make, batches = _setup(pnr_mod, dev, points=points)
    ro, rd, gt, col, t_rand = batches[0]
    r, dec, pts = make()
    ms = MapStep(r, dec, points=pts, feat_lr=1e-2, lr=0.0)  # lr 0: Adam leaves the parameters alone
    l_fused = float(ms(ro, rd, gt, col, t_rand))
    g_fused = ms.flat.grad.clone()
    r2, dec2, pts2 = make()
    ms2 = MapStep(r2, dec2, points=pts2, feat_lr=1e-2, lr=0.0)
    ms2.flat.grad.zero_()
    loss = ms2.loss(ro, rd, gt, col, t_rand=t_rand)
    loss.backward()
    torch.cuda.synchronize()
    # the colour term: torch sums |gt - c| in float32, pnr_map_loss in float64
    assert abs(float(loss) - l_fused) <= 1e-6 * abs(l_fused)
    g_auto = ms2.flat.grad.clone()  # autograd accumulated into the flat views (FlatParams)
    scale = g_fused.abs().max()
    diff = (g_fused - g_auto).abs()
    print(f'fused vs autograd: max |dg| {float(diff.max()):.3e} of max |g| {float(scale):.3e}; '
          f'bitwise equal {bool(torch.equal(g_fused, g_auto))}')
    # the fused step is the map pass (one GEMM over render + regulation samples) and the autograd path
    # two passes summed: equal up to float32 association -- and, in f16x3, up to the split scales the
    # weight-gradient GEMMs pick per wave from the points they see (2^-22 of a wave's largest term)
    floor = 1e-6 if precision == 'fp32' else 1e-5
    assert bool((diff <= 1e-6 * g_auto.abs() + floor * scale).all())


@pytest.mark.parametrize('points', [True, False])
def test_map_pass_equals_two_chains(pnr_mod, dev, points, precision):
    """pnr_map_fwd (regulation + coarse samples in one MLP launch, importance in a second, points and
    bound tests formed by the ray kernels) against pnr_render_fwd + pnr_regulation_fwd on the same rays
    and jitter: depth, variance, colour and the regulation densities bit for bit; the step's gradients
    (one delta-chain / weight-gradient pass over all samples against two summed) to float32 association:
    |dg| <= 1e-6 |g| + 1e-6 max|g|."""
    from pnr.mapping import MapStep
    from pnr.renderer import MapPass, TrainPass
    make, batches = _setup(pnr_mod, dev, points=points)
    ro, rd, gt, col, t_rand = batches[0]
    r, dec, pts = make()
    c = {} if pts is None else {'points_color': pts}
    with torch.no_grad():
        d1, v1, c1, s1 = MapPass(r, c, dec).forward(ro, rd, gt, t_rand)
        d2, v2, c2 = TrainPass(r, c, dec, 'render').forward(ro, rd, gt)
        (s2,) = TrainPass(r, c, dec, 'regulation').forward(ro, rd, gt, t_rand=t_rand)
    torch.cuda.synchronize()
    for a, b, what in ((d1, d2, 'depth'), (v1, v2, 'var'), (c1, c2, 'rgb'), (s1, s2, 'sigma')):
        assert torch.equal(a, b), what
    out = []
    for fused in (True, False):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2, fused=fused, overlap=False)
        loss = float(ms(ro, rd, gt, col, t_rand))
        torch.cuda.synchronize()
        out.append((loss, ms.flat.grad.clone()))
    assert abs(out[0][0] - out[1][0]) <= 1e-12 * abs(out[1][0])
    g1, g2 = out[0][1], out[1][1]
    diff = (g1 - g2).abs()
    print(f'map pass vs two chains: max |dg| {float(diff.max()):.3e} of max |g| {float(g2.abs().max()):.3e}')
    floor = 1e-6 if precision == 'fp32' else 1e-5  # f16x3: per-wave split scales (see above)
    assert bool((diff <= 1e-6 * g2.abs() + floor * g2.abs().max()).all())


@pytest.mark.parametrize('points', [True, False])
def test_map_step_stores_over_dirty_grads(pnr_mod, dev, points, precision):
    """The fused MapStep stores the decoder / fc_c gradients (grads_overwrite) instead of zeroing the
    buffer first: a buffer full of garbage from an earlier step must give exactly the gradients of a
    clean one (a regression to accumulation would add the garbage in)."""
    from pnr.mapping import MapStep
    make, batches = _setup(pnr_mod, dev, points=points)
    ro, rd, gt, col, t_rand = batches[0]
    out = []
    for dirty in (False, True):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2, lr=0.0)
        if dirty:
            ms.flat.grad.copy_(torch.randn_like(ms.flat.grad) * 1e3)
        ms(ro, rd, gt, col, t_rand)
        torch.cuda.synchronize()
        out.append(ms.flat.grad.clone())
    assert torch.equal(out[0], out[1])


@pytest.mark.parametrize('points', [True, False])
def test_map_bwd_empty_batch_zeroes_stored_grads(pnr_mod, dev, points, precision):
    """pnr_map_bwd with n = 0 and grads_overwrite: the stored decoder / fc_c gradients of an empty
    batch are zero (autograd's), not the previous step's values left in the buffer."""
    from pnr.mapping import MapStep
    from pnr.renderer import MapPass
    make, _ = _setup(pnr_mod, dev, points=points)
    r, dec, pts = make()
    c = {} if pts is None else {'points_color': pts}
    ms = MapStep(r, dec, points=pts, lr=0.0)
    views, g_fc, g_feats = ms._views['main']
    ms.flat.grad.fill_(7.0)
    e3 = torch.empty((0, 3), device=dev)
    e1 = torch.empty(0, device=dev)
    mp = MapPass(r, c, dec)
    mp.forward(e3, e3, e1, torch.empty((0, 32), device=dev))
    mp.backward(views, g_fc=g_fc, g_feats=g_feats, g_depth=torch.empty(0, dtype=torch.float64, device=dev),
                g_rgb=e3, g_sigma=e1, overwrite=True)
    torch.cuda.synchronize()
    n_dec = ms.n_dec
    assert bool((ms.flat.grad[:n_dec] == 0).all())
    if points:  # point-feature gradients always accumulate: left as they were
        assert bool((ms.flat.grad[n_dec:] == 7.0).all())


def test_map_step_multi_chunk_store(pnr_mod, dev, precision):
    """More rows than one backward chunk (kBwdChunk = 4M rows: 56,000 rays x 76 rows): the first chunk
    stores, later chunks add.  Over a dirty buffer the fused step must equal the two-chain step (zero
    fill + accumulate) to float32 association, like test_map_pass_equals_two_chains."""
    from pnr.mapping import MapStep
    make, _ = _setup(pnr_mod, dev, points=False)
    r0 = load_golden('render.npz')
    n = 56000
    ro = torch.from_numpy(r0['p2_gt/rays_o'])
    rd = torch.from_numpy(r0['p2_gt/rays_d'])
    gt = torch.from_numpy(r0['p2_gt/gt_depth'])
    reps = -(-n // ro.shape[0])
    gen = torch.Generator().manual_seed(11)
    ro, rd, gt = [t.repeat(reps, *([1] * (t.dim() - 1)))[:n].to(dev) for t in (ro, rd, gt)]
    col = torch.rand((n, 3), generator=gen).to(dev)
    t_rand = torch.rand((n, 32), generator=gen).to(dev)
    out = []
    for fused in (True, False):
        r, dec, _ = make()
        ms = MapStep(r, dec, lr=0.0, fused=fused, overlap=False)
        ms.flat.grad.copy_(torch.randn_like(ms.flat.grad) * 1e3)
        ms(ro, rd, gt, col, t_rand)
        torch.cuda.synchronize()
        out.append(ms.flat.grad.clone())
    g1, g2 = out
    diff = (g1 - g2).abs()
    floor = 1e-6 if precision == 'fp32' else 1e-5
    assert bool((diff <= 1e-6 * g2.abs() + floor * g2.abs().max()).all()), float(diff.max())


@pytest.mark.parametrize('points,n', [(True, 512), (False, 512), (False, 33000)])
def test_map_step_one_call_matches_three_calls(pnr_mod, dev, points, n, precision):
    """pnr_map_step (ABI 13: forward, loss and backward in one C call; up to 32,768 rays the final
    compositing, the loss and the compositing backward are ONE fused launch, k_fine_loss_w) against
    pnr_map_fwd + pnr_map_loss + pnr_map_bwd: every gradient bit for bit (the fused kernel forms each
    value with the same expressions), the loss to its summation order.  33,000 rays: the unfused tail."""
    from pnr.mapping import MapStep
    make, batches = _setup(pnr_mod, dev, points=points)
    ro, rd, gt, col, t_rand = batches[0]
    if n > ro.shape[0]:
        reps = -(-n // ro.shape[0])
        gen = torch.Generator().manual_seed(12)
        ro, rd, gt = [t.repeat(reps, *([1] * (t.dim() - 1)))[:n].contiguous() for t in (ro, rd, gt)]
        col = torch.rand((n, 3), generator=gen).to(dev)
        t_rand = torch.rand((n, 32), generator=gen).to(dev)
    out = []
    for one in (True, False):
        r, dec, pts = make()
        ms = MapStep(r, dec, points=pts, feat_lr=1e-2, lr=0.0)
        ms.one_call = one
        ms.flat.grad.copy_(torch.randn_like(ms.flat.grad))
        if points:
            ms.flat.grad[ms.n_dec:].zero_()
        loss = float(ms(ro, rd, gt, col, t_rand))
        torch.cuda.synchronize()
        out.append((loss, ms.flat.grad.clone()))
    assert abs(out[0][0] - out[1][0]) <= 1e-12 * abs(out[1][0]), (out[0][0], out[1][0])
    assert torch.equal(out[0][1], out[1][1])


def test_map_step_empty_batch(pnr_mod, dev, precision):
    """pnr_map_step with n = 0: loss 0 and (grads_overwrite) zero decoder gradients."""
    from pnr.mapping import MapStep
    make, _ = _setup(pnr_mod, dev, points=False)
    r, dec, _ = make()
    ms = MapStep(r, dec, lr=0.0)
    ms.flat.grad.fill_(7.0)
    e3 = torch.empty((0, 3), device=dev)
    loss = ms(e3, e3, torch.empty(0, device=dev), e3, torch.empty((0, 32), device=dev))
    torch.cuda.synchronize()
    assert float(loss) == 0.0
    assert bool((ms.flat.grad == 0).all())


@pytest.mark.parametrize('points', [True, False])
def test_f16x3_only_pack_matches_full(pnr_mod, dev, points):
    """ABI 14: the Mapper's repack asks for the f16x3 images only (pnr_mlp_pack2 / pnr_fc_pack2
    PNR_PACK_F16X3_ONLY: no fp32 / bf16 images).  After a few MapSteps, its images of the final weights
    equal a fresh full pack's bit for bit on everything the f16x3 kernels read: the f16x3 forward and
    delta-chain images and the raw table (biases, Fourier B, scales, Wo)."""
    from pnr import _lib
    from pnr.mapping import MapStep
    from pnr.packing import PackedFC, PackedMLP
    make, batches = _setup(pnr_mod, dev, points=points)
    r, dec, pts = make()
    ms = MapStep(r, dec, points=pts, feat_lr=1e-2)
    for b in batches[:2]:
        ms(*b)
    torch.cuda.synchronize()
    lib = _lib.load()
    f16 = _lib.PRECISIONS['f16x3']
    # (compared as int32 words: two f16 parts in a float32 word can spell a NaN)
    img = dec._packed.image(list(dec.ordered_params()), prec=f16).clone().view(torch.int32)
    ref = PackedMLP().image([p.detach().clone() for p in dec.ordered_params()]).view(torch.int32)
    w16 = 225280                                # the 16-point-wave forward image (mlp16w.h), after the raw table
    raw0 = lib.pnr_mlp_packed_floats() - w16 - 3072   # kOffRaw: the raw table's 12 KiB, then that image
    lo = raw0 - (917504 + 901120) // 4          # kOffH2: f16x3 main image, then the delta-chain image
    # raw words: biases / bo / Fourier B [0, 1344), inverse scales [1344, 1349), scales [1352, 1357), Wo [2048, 3072)
    for a, b in ((lo, raw0 + 1349), (raw0 + 1352, raw0 + 1357), (raw0 + 2048, raw0 + 3072 + w16)):
        assert torch.equal(img[a:b], ref[a:b]), (a, b)
    if points:
        fimg = dec._packed_fc.image(list(dec.ordered_fc_params()), prec=f16).clone().view(torch.int32)
        fref = PackedFC().image([p.detach().clone() for p in dec.ordered_fc_params()]).view(torch.int32)
        fraw0 = lib.pnr_fc_packed_floats() - 2048  # kOffFcRaw
        flo = fraw0 - 2 * 32768                    # kOffFcH2: f16x3 fc image, then the fc backward image
        assert torch.equal(fimg[flo:fraw0 + 1032], fref[flo:fraw0 + 1032])  # (bc, inverse [4], forward [4])
