"""Correctly-rounded Mapper-loss gradients (tests/golden/grads_cr.npz) -- test infrastructure.

Same inputs as grads.npz's map case (made by importing the reference, make_golden.py), evaluated by
the oracle (oracle/ref_render.py, pinned bit-exactly to the reference by test_oracle_golden.py) with
oracle.ref_render.mlp_forward_cr: every hidden / output GEMM summed in float64 and rounded to
float32 per layer, forward and backward.  The reference's own float32 gradient (grads.npz) differs
from this by its summation-order rounding (up to ~4e-6 of max|g| per tensor, recorded in
`golden_vs_cr/<name>`); an fp32-class implementation is judged against both.

    python tests/golden/make_grads_cr.py     (CPU, ~1 min; no reference import)
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [REPO, os.path.join(REPO, 'tests')]
from conftest import load_golden, golden_params  # noqa: E402
from oracle import ref_render as ref  # noqa: E402


def main():
    torch.set_num_threads(8)
    G = load_golden('grads.npz')
    bound = torch.from_numpy(load_golden('scene.npz')['bound'])
    p = {k: v.clone().requires_grad_(True) for k, v in golden_params('trained').items()}
    ro, rd = torch.from_numpy(G['map_rays_o']), torch.from_numpy(G['map_rays_d'])
    gt, gc = torch.from_numpy(G['map_gt_depth']), torch.from_numpy(G['map_gt_color'])
    ev = lambda q: ref.eval_points_cr(p, q, bound)  # noqa: E731
    d, v, c = ref.render_batch_ray(p, rd, ro, bound, gt_depth=gt, eval_fn=ev)
    sig = ref.regulation(p, rd, ro, gt, bound, t_rand=torch.from_numpy(G['map_t_rand']), eval_fn=ev)
    loss = ref.mapping_loss(d, c, gt, gc, sig)
    loss.backward()
    out = {'map_loss': np.array(loss.item())}
    for k, t in p.items():
        g = t.grad.numpy().copy()
        gref = G[f'map_grad/{k}']
        out[f'map_grad/{k}'] = g
        out[f'golden_vs_cr/{k}'] = np.array(np.abs(g - gref).max() / np.abs(g).max())
        print(f'{k:24s} |golden - cr| / max = {out[f"golden_vs_cr/{k}"]:.2e}')
    np.savez_compressed(os.path.join(HERE, 'grads_cr.npz'), **out)


if __name__ == '__main__':
    main()
