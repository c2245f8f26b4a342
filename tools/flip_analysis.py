"""Offline analysis of the decision-edge flips behind the end-to-end neural-point gradient tests
(the .npz dumps of tools/flip_dump.sh: HIP gradient g, correctly-rounded cr and float32 f32 references,
summation magnitudes M).

A sample whose ReLU decision (or neighbour set) flips between two float32 orders changes ONE rank-1
term of every weight gradient dW = sum_p delta_p h_p^T -- its delta times its activations -- so the
deviation D = g - g_ref of a weight tensor beyond the strict elementwise bound is (nearly) a matrix of
rank <= the number of flipped samples.  For each dumped tensor this prints the share of elements
beyond the strict bound and the smallest K such that D minus its best rank-K approximation (SVD) lies
inside the strict bound on EVERY element: the number of flipped samples the tensor's deviation needs.

  python tools/flip_analysis.py gpurun_out/flips_r06
"""
import glob
import os
import sys

import numpy as np

U = 2.0 ** -24
MAG_ULPS = 64.0


def strict_bound(ref, cr, mag, d32, rtol, atol):
    scale = max(np.abs(cr).max(), 1e-30)
    return rtol * np.abs(ref) + (atol + d32) * scale + MAG_ULPS * U * np.asarray(mag)


def flip_rank(D, B, kmax=8):
    """Smallest k <= kmax with |D - D_k| <= B everywhere (D_k: best rank-k approximation), or None."""
    if (np.abs(D) <= B).all():
        return 0, D
    if D.ndim != 2:
        return None, D
    u, s, vt = np.linalg.svd(D, full_matrices=False)
    for k in range(1, min(kmax, len(s)) + 1):
        R = D - (u[:, :k] * s[:k]) @ vt[:k]
        if (np.abs(R) <= B).all():
            return k, R
    return None, D


def main(d):
    for f in sorted(glob.glob(os.path.join(d, '*.npz'))):
        z = np.load(f)
        g, cr, f32, mag = z['g'].astype(np.float64), z['cr'], z['f32'].astype(np.float64), z['mag']
        d32, rtol, atol = float(z['d32']), float(z['rtol']), float(z['atol'])
        name = os.path.basename(f)[:-4]
        for ref, tag in ((cr, 'cr'), (f32, 'f32')):
            B = strict_bound(ref, cr, mag, d32, rtol, atol)
            D = g - ref
            beyond = float(np.mean(np.abs(D) > B))
            k, R = flip_rank(D, B)
            worst = float((np.abs(D) / B).max())
            m = max(np.abs(cr).max(), 1e-30)
            print(f'{name:90s} vs {tag:3s}: beyond {beyond:.2e}, worst {worst:7.2f}, '
                  f'max|D|/max|g| {np.abs(D).max() / m:.2e}, flip rank {k}')


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/flips_r06')
