"""A small closed test mesh (lat-long sphere) for the Mesher colouring tests."""
import numpy as np


def uv_sphere(center, radius, n_lat=24, n_lon=48):
    """Vertices (V,3) float64 and faces (F,3) int64, outward winding, poles shared."""
    c = np.asarray(center, dtype=np.float64)
    verts = [c + [0, 0, radius]]
    for i in range(1, n_lat):
        th = np.pi * i / n_lat
        for j in range(n_lon):
            ph = 2 * np.pi * j / n_lon
            verts.append(c + radius * np.array([np.sin(th) * np.cos(ph), np.sin(th) * np.sin(ph), np.cos(th)]))
    verts.append(c + [0, 0, -radius])
    V = len(verts)
    ring = lambda i, j: 1 + (i - 1) * n_lon + (j % n_lon)  # noqa: E731
    faces = []
    for j in range(n_lon):
        faces.append([0, ring(1, j), ring(1, j + 1)])
        faces.append([V - 1, ring(n_lat - 1, j + 1), ring(n_lat - 1, j)])
    for i in range(1, n_lat - 1):
        for j in range(n_lon):
            a, b, c2, d = ring(i, j), ring(i, j + 1), ring(i + 1, j), ring(i + 1, j + 1)
            faces.append([a, c2, b])
            faces.append([b, c2, d])
    return np.asarray(verts), np.asarray(faces, dtype=np.int64)
