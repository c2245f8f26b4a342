"""Shared pytest setup: markers, repo paths, golden-vector loaders."""
import os
import sys

import numpy as np
import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, 'pointnerf-slam_amd')
GOLDEN = os.path.join(REPO, 'tests', 'golden')
for p in (REPO, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (runs through the HIP C-ABI library)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def load_golden(name):
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def golden_params(tag='trained'):
    w = load_golden('weights.npz')
    pre = tag + '/'
    return {k[len(pre):]: torch.from_numpy(v) for k, v in w.items() if k.startswith(pre)}


@pytest.fixture(scope='session')
def scene():
    s = load_golden('scene.npz')
    s['bound_t'] = torch.from_numpy(s['bound'])
    return s


@pytest.fixture(scope='session')
def trained_params():
    return golden_params('trained')


@pytest.fixture(scope='session')
def random_params():
    return golden_params('random')


def maybe_dump_grads(what, g, cr, f32, mag, d32, rtol, atol, a):
    """Diagnostics (tools/flip_dump.sh, env PNR_DUMP_GRADS=<dir>): save the HIP gradient, the
    correctly-rounded and float32 references and the summation magnitudes of any tensor with an
    element beyond the strict elementwise bound (a = its absolute term), one .npz per test and tensor."""
    import os
    dump = os.environ.get('PNR_DUMP_GRADS')
    if not dump:
        return
    g, cr, f32 = (np.asarray(x, dtype=np.float64) for x in (g, cr, f32))
    if (np.abs(g - cr) > rtol * np.abs(cr) + a).any() or (np.abs(g - f32) > rtol * np.abs(f32) + a).any():
        os.makedirs(dump, exist_ok=True)
        tag = (os.environ.get('PYTEST_CURRENT_TEST', 'x').split(' ')[0] + '__' + what)
        for ch in '/:[]':
            tag = tag.replace(ch, '_')
        np.savez_compressed(os.path.join(dump, tag + '.npz'), g=g.astype(np.float32), cr=cr, f32=f32.astype(np.float32),
                            mag=np.asarray(0.0 if mag is None else mag), d32=d32, rtol=rtol, atol=atol)
