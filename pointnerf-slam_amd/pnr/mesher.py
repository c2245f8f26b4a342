"""The Mesher's decoder consumers on the HIP path.

Under configs/pointNeRF_slam.yaml (`meshing.color_mesh_extraction_method: render_ray_along_normal`,
:37) Mesher.get_mesh (src/utils/Mesher.py:349-570) calls the decoder twice:
  * the dense grid query: get_grid_uniform (:321-347) + Mesher.eval_points (:281-319) over
    resolution^3 points in points_batch_size chunks, occupancy = raw[:, -1] (:427-430);
  * the vertex colouring (:526-553): one ray per mesh vertex, started `length`=0.1 behind the
    vertex along its normal (rays_o = v - 0.1 n, rays_d = n), rendered by
    Renderer.render_batch_ray with gt_depth = 0.1 in ray_batch_size chunks; the colour is clipped
    to [0,1] and stored as uint8 (:555-556).  `direct_point_query` (:513-524, the nice-slam
    setting) is eval_points(vertices)[..., :3].
Marching cubes (skimage), mesh cleaning / culling (trimesh) and the forecast masks stay with the
caller: they are host-side geometry, not this path.  The vertex normals the reference takes from
open3d (`compute_vertex_normals`, open3d is not in this image) are restated by `vertex_normals` on
the device: area-weighted sums of the unnormalised triangle normals, normalised, with (0,0,1) for a
vertex whose sum vanishes (open3d TriangleMesh::ComputeVertexNormals + MeshBase::NormalizeNormals).
That restatement is "parity unpinned" (no open3d output is available to pin it); the colouring
itself is pinned through render_batch_ray against the oracle (tests/test_gpu_parity.py).
"""
from __future__ import annotations

import numpy as np
import torch

from . import _lib


def get_grid_uniform(bound, resolution, padding=0.05):
    """src/utils/Mesher.py:321-347: float32 (R^3, 3) grid points over `bound` (3,2) padded by
    `padding` (np.linspace per axis, np.meshgrid 'xy' order, ravel) and the per-axis coordinates."""
    b = np.asarray(bound.cpu() if isinstance(bound, torch.Tensor) else bound, dtype=np.float64).reshape(3, 2)
    x, y, z = (np.linspace(b[a][0] - padding, b[a][1] + padding, resolution) for a in range(3))
    xx, yy, zz = np.meshgrid(x, y, z)
    grid_points = torch.tensor(np.vstack([xx.ravel(), yy.ravel(), zz.ravel()]).T, dtype=torch.float)
    return {'grid_points': grid_points, 'xyz': [x, y, z]}


def eval_grid(renderer, decoders, c, points, device, stage='color'):
    """The Mesher's grid query (src/utils/Mesher.py:427-430): raw (P,4) float32 of `points` in
    renderer.points_batch_size chunks through the HIP eval_points (the occupancy is raw[:, -1])."""
    _lib.require_cuda(points)
    with torch.no_grad():
        out = [renderer.eval_points(p, decoders, c, stage, device)
               for p in torch.split(points, renderer.points_batch_size)]
    return torch.cat(out, 0) if out else torch.empty((0, 4), device=points.device)


def vertex_normals(vertices: torch.Tensor, faces: torch.Tensor) -> torch.Tensor:
    """open3d compute_vertex_normals restated on the device (float64): per triangle the
    unnormalised cross((v1 - v0), (v2 - v0)), summed into its three vertices, then normalised;
    a zero sum gives (0, 0, 1).  vertices (V,3), faces (F,3) int -> (V,3) float64."""
    v = vertices.double()
    f = faces.long()
    tn = torch.cross(v[f[:, 1]] - v[f[:, 0]], v[f[:, 2]] - v[f[:, 0]], dim=1)
    n = torch.zeros_like(v)
    for a in range(3):
        n.index_add_(0, f[:, a], tn)
    norm = n.norm(dim=1, keepdim=True)
    z = torch.zeros_like(n)
    z[:, 2] = 1.0
    return torch.where(norm > 0, n / torch.where(norm > 0, norm, torch.ones_like(norm)), z)


def color_along_normal(renderer, decoders, c, vertices, normals, device, length=0.1, stage='color'):
    """src/utils/Mesher.py:526-553: vertex colour (V,3) float32 from one ray per vertex,
    rays_o = v - length * n, rays_d = n, gt_depth = length, rendered in ray_batch_size chunks."""
    v = vertices.to(device).double()
    n = normals.to(device).double()
    _lib.require_cuda(v)
    rays_d = n
    rays_o = v + (-1.0) * length * n
    gt_depth = torch.full((v.shape[0],), length, device=v.device)
    out = []
    with torch.no_grad():
        bs = renderer.ray_batch_size
        for i in range(0, rays_d.shape[0], bs):
            _, _, col = renderer.render_batch_ray(c, decoders, rays_d[i:i + bs], rays_o[i:i + bs], device,
                                                  stage=stage, gt_depth=gt_depth[i:i + bs])
            out.append(col)
    return torch.cat(out, 0) if out else torch.empty((0, 3), device=v.device)


def direct_point_query(renderer, decoders, c, vertices, device, stage='color'):
    """src/utils/Mesher.py:513-524 (`direct_point_query`): eval_points(vertices)[..., :3]."""
    return eval_grid(renderer, decoders, c, vertices.to(device).float(), device, stage)[..., :3]


def vertex_colors_u8(colors: torch.Tensor) -> np.ndarray:
    """src/utils/Mesher.py:555-556: clip to [0,1], x255, uint8 (truncation, as numpy astype)."""
    return (np.clip(colors.detach().cpu().numpy(), 0, 1) * 255).astype(np.uint8)


def mesh_colors(renderer, decoders, c, vertices, faces, device, method='render_ray_along_normal'):
    """The colour branch of Mesher.get_mesh (:512-556) for a mesh from the caller's marching cubes:
    uint8 (V,3) vertex colours by the configured `color_mesh_extraction_method`."""
    v = torch.as_tensor(vertices)
    if method == 'render_ray_along_normal':
        n = vertex_normals(v.to(device), torch.as_tensor(faces).to(device))
        col = color_along_normal(renderer, decoders, c, v, n, device)
    elif method == 'direct_point_query':
        col = direct_point_query(renderer, decoders, c, v, device)
    else:
        raise ValueError(f'pnr.mesher: unknown color_mesh_extraction_method {method!r}')
    return vertex_colors_u8(col)
