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
