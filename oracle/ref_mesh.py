"""CPU restatement of the Mesher's decoder consumers -- TEST INFRASTRUCTURE ONLY.

Only `tests/` may import this module, as the checker of `pnr.mesher` (SURVEY.md section 8 (f)
row F4).  Sources (paths relative to thua919/pointNeRF-SLAM):
  * get_grid_uniform: src/utils/Mesher.py:321-347;
  * render_ray_along_normal colouring: src/utils/Mesher.py:526-556, over
    oracle.ref_render.render_batch_ray (pinned by tests/test_oracle_golden.py);
  * vertex normals: the reference calls open3d's TriangleMesh.compute_vertex_normals
    (Mesher.py:530-534; open3d is a third-party dependency absent from this image, pinned at
    open3d==0.13.0 in the reference's environment.yaml:158).  Its published algorithm
    (TriangleMesh::ComputeVertexNormals / MeshBase::NormalizeNormals) is restated here as a plain
    per-triangle loop: unnormalised triangle normals cross(v1-v0, v2-v0) summed per vertex, then
    normalised, a NaN result replaced by (0,0,1).  No open3d output is available: the normals are
    "parity unpinned" beyond this restatement.
"""
from __future__ import annotations

import numpy as np
import torch

from . import ref_render


def grid_uniform(bound, resolution, padding=0.05):
    """src/utils/Mesher.py:331-345."""
    b = np.asarray(bound, dtype=np.float64).reshape(3, 2)
    x = np.linspace(b[0][0] - padding, b[0][1] + padding, resolution)
    y = np.linspace(b[1][0] - padding, b[1][1] + padding, resolution)
    z = np.linspace(b[2][0] - padding, b[2][1] + padding, resolution)
    xx, yy, zz = np.meshgrid(x, y, z)
    return torch.tensor(np.vstack([xx.ravel(), yy.ravel(), zz.ravel()]).T, dtype=torch.float)


def vertex_normals(vertices, faces):
    """open3d ComputeVertexNormals(normalized=True), one triangle at a time (float64)."""
    v = np.asarray(vertices, dtype=np.float64)
    n = np.zeros_like(v)
    for a, b, c in np.asarray(faces):
        e1 = v[b] - v[a]
        e2 = v[c] - v[a]
        tn = np.array([e1[1] * e2[2] - e1[2] * e2[1], e1[2] * e2[0] - e1[0] * e2[2], e1[0] * e2[1] - e1[1] * e2[0]])
        n[a] += tn
        n[b] += tn
        n[c] += tn
    out = np.empty_like(n)
    for i in range(n.shape[0]):
        norm = np.sqrt(n[i] @ n[i])
        out[i] = n[i] / norm if norm > 0 else np.array([0.0, 0.0, 1.0])
    return out


def color_along_normal(params, vertices, normals, bound, length=0.1):
    """src/utils/Mesher.py:535-553 on the CPU oracle: rays_o = v - length n (float64, as the
    reference's numpy arrays), rays_d = n, gt_depth = length (float32)."""
    rays_d = torch.from_numpy(np.asarray(normals, dtype=np.float64))
    rays_o = torch.from_numpy(np.asarray(vertices, dtype=np.float64) + (-1.0) * length * np.asarray(normals))
    gt = torch.full((rays_d.shape[0],), length, dtype=torch.float32)
    _, _, col = ref_render.render_batch_ray(params, rays_d, rays_o, bound, gt_depth=gt)
    return col
