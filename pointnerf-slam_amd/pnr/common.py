"""Device-agnostic pose / bound helpers of src/common.py and src/NICE_SLAM.py (host logic).

These are small tensor expressions (no hot-path arithmetic), written for any torch device so
the Tracker's differentiable pose (src/common.py:137-176) works on the GPU tensors the renderer
consumes.  `quad2rotation` in the reference fails on CPU tensors (`.to(get_device())`, :150).
"""
from __future__ import annotations

import math

import numpy as np
import torch


def scaled_bound(bound_cfg, scale, bound_divisible):
    """src/NICE_SLAM.py:208-213: (3,2) float64 bound scaled and rounded up to bound_divisible."""
    b = torch.from_numpy(np.array(bound_cfg) * scale)
    b[:, 1] = (((b[:, 1] - b[:, 0]) / bound_divisible).int() + 1) * bound_divisible + b[:, 0]
    return b


def quad2rotation(quad):
    """src/common.py:137-160 (batched (B,4) quaternion (r,i,j,k) -> (B,3,3))."""
    qr, qi, qj, qk = quad[:, 0], quad[:, 1], quad[:, 2], quad[:, 3]
    two_s = 2.0 / (quad * quad).sum(-1)
    m = [1 - two_s * (qj ** 2 + qk ** 2), two_s * (qi * qj - qk * qr), two_s * (qi * qk + qj * qr),
         two_s * (qi * qj + qk * qr), 1 - two_s * (qi ** 2 + qk ** 2), two_s * (qj * qk - qi * qr),
         two_s * (qi * qk - qj * qr), two_s * (qj * qk + qi * qr), 1 - two_s * (qi ** 2 + qj ** 2)]
    return torch.stack(m, -1).reshape(-1, 3, 3)


def get_camera_from_tensor(inputs):
    """src/common.py:163-176: (qw,qx,qy,qz,tx,ty,tz) -> [R|t] (3,4), differentiable."""
    single = inputs.dim() == 1
    if single:
        inputs = inputs.unsqueeze(0)
    R = quad2rotation(inputs[:, :4])
    RT = torch.cat([R, inputs[:, 4:, None]], 2)
    return RT[0] if single else RT


def get_tensor_from_camera(RT, Tquad=False):
    """src/common.py:179-201 without `mathutils`: rotation matrix -> (w,x,y,z) quaternion + t."""
    dev = RT.device if isinstance(RT, torch.Tensor) else None
    A = np.asarray(RT.detach().cpu() if isinstance(RT, torch.Tensor) else RT, dtype=np.float64)
    R, T = A[:3, :3], A[:3, 3]
    tr = R[0, 0] + R[1, 1] + R[2, 2]
    if tr > 0:
        s = math.sqrt(tr + 1.0) * 2
        q = [0.25 * s, (R[2, 1] - R[1, 2]) / s, (R[0, 2] - R[2, 0]) / s, (R[1, 0] - R[0, 1]) / s]
    elif R[0, 0] > R[1, 1] and R[0, 0] > R[2, 2]:
        s = math.sqrt(1.0 + R[0, 0] - R[1, 1] - R[2, 2]) * 2
        q = [(R[2, 1] - R[1, 2]) / s, 0.25 * s, (R[0, 1] + R[1, 0]) / s, (R[0, 2] + R[2, 0]) / s]
    elif R[1, 1] > R[2, 2]:
        s = math.sqrt(1.0 + R[1, 1] - R[0, 0] - R[2, 2]) * 2
        q = [(R[0, 2] - R[2, 0]) / s, (R[0, 1] + R[1, 0]) / s, 0.25 * s, (R[1, 2] + R[2, 1]) / s]
    else:
        s = math.sqrt(1.0 + R[2, 2] - R[0, 0] - R[1, 1]) * 2
        q = [(R[1, 0] - R[0, 1]) / s, (R[0, 2] + R[2, 0]) / s, (R[1, 2] + R[2, 1]) / s, 0.25 * s]
    t = np.concatenate([T, q]) if Tquad else np.concatenate([q, T])
    out = torch.from_numpy(t).float()
    return out if dev is None else out.to(dev)


def select_uv_indices(n_pixels, n, device, generator=None):
    """src/common.py:99-100: uniform torch.randint pixel indices (clamped like the reference)."""
    idx = torch.randint(n_pixels, (n,), device=device, generator=generator)
    return idx.clamp(0, n_pixels)


def random_select(l, k):
    """src/common.py:66-71: k distinct values of 0..l-1 in random order (keyframe window)."""
    return list(np.random.permutation(np.array(range(l)))[:min(l, k)])

