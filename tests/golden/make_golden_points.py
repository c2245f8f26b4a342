"""Golden vectors for the neural-point feature stage, made by importing the
REFERENCE decoder with a feature grid (run in the build container only).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_points.py [/root/reference]

The reference has no neural-point gather.  Its nearest analogue is `MLP(c_dim=32)` with a dense
feature grid: `MLP.sample_grid_feature` (src/conv_onet/models/decoder.py:168-175, trilinear
`F.grid_sample`, align_corners=True) followed by the `fc_c` injection
`h = relu(W h + b) + fc_c[i](c)` (decoder.py:196-197).  A neural-point cloud placed on the grid
vertices, gathered with trilinear weights, must reproduce that on interior samples -- this file
holds the reference side of that pin:

  points_c32.npz
    bound (3,2) f64             room0 scaled bound (src/NICE_SLAM.py:208-213)
    grid  (1,32,D,H,W) f32      feature grid (x <-> W, y <-> H, z <-> D)
    p     (P,3) f64             interior sample points
    c     (P,32) f32            MLP.sample_grid_feature(p, grid)
    raw   (P,4) f32             MLP.forward(p, {'grid_color': grid})
    g_raw (P,4) f32             upstream gradient of the fixed loss sum(raw * g_raw)
    grad/<param>                d loss / d decoder tensor (incl. fc_c.{i}.{weight,bias})
    grad_grid (1,32,D,H,W) f32  d loss / d grid
    grad_p (P,3) f64            d loss / d p
    w/<param>                   the decoder state_dict
"""
import os
import sys

import numpy as np
import torch

REF = sys.argv[1] if len(sys.argv) > 1 else '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))
GRID_DHW = (13, 13, 17)   # z, y, x vertices: 0.08 spacing on every axis of the room0 bound
N_PTS = 2048


def main():
    torch.set_num_threads(1)
    os.chdir(REF)
    sys.path.insert(0, REF)
    from src import config                                   # noqa: E402
    from src.conv_onet.models.decoder import MLP             # noqa: E402

    cfg = config.load_config('configs/Replica/room0_point.yaml', 'configs/pointNeRF_slam.yaml')
    scale = cfg['scale']
    bound = torch.from_numpy(np.array(cfg['mapping']['bound']) * scale)
    bd = cfg['grid_len']['bound_divisible']
    bound[:, 1] = (((bound[:, 1] - bound[:, 0]) / bd).int() + 1) * bd + bound[:, 0]

    torch.manual_seed(7)
    dec = MLP(name='color', dim=3, c_dim=32, color=True, skips=[], n_blocks=4, hidden_size=256,
              pos_embedding_method='fourier', sample_mode='bilinear')
    dec.bound = bound
    g = torch.Generator().manual_seed(11)
    D, H, W = GRID_DHW
    grid = (torch.randn((1, 32, D, H, W), generator=g) * 0.5).requires_grad_(True)
    lo, hi = bound[:, 0], bound[:, 1]
    margin = 1e-3
    p = lo + margin + (hi - lo - 2 * margin) * torch.rand((N_PTS, 3), generator=g, dtype=torch.float64)
    p.requires_grad_(True)

    c = dec.sample_grid_feature(p, grid).transpose(1, 2).squeeze(0)
    raw = dec(p, c_grid={'grid_color': grid})
    g_raw = torch.randn(raw.shape, generator=g)
    (raw * g_raw).sum().backward()

    out = {'bound': bound.numpy(), 'grid': grid.detach().numpy(), 'p': p.detach().numpy(),
           'c': c.detach().numpy(), 'raw': raw.detach().numpy(), 'g_raw': g_raw.numpy(),
           'grad_grid': grid.grad.numpy(), 'grad_p': p.grad.numpy()}
    for k, v in dec.state_dict().items():
        out['w/' + k] = v.numpy()
    for k, v in dec.named_parameters():
        out['grad/' + k] = v.grad.numpy()
    np.savez_compressed(os.path.join(OUT, 'points_c32.npz'), **out)
    print('wrote points_c32.npz', {k: v.shape for k, v in out.items() if not k.startswith(('w/', 'grad/'))})


if __name__ == '__main__':
    main()
