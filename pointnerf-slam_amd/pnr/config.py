"""Config loading mirror of src/config.py:10-79 (yaml `inherit_from` chain + recursive merge)."""
from __future__ import annotations

import yaml


def load_config(path, default_path=None):
    """src/config.py:10-42."""
    with open(path, 'r') as f:
        cfg_special = yaml.safe_load(f)
    inherit_from = cfg_special.get('inherit_from')
    if inherit_from is not None:
        cfg = load_config(inherit_from, default_path)
    elif default_path is not None:
        with open(default_path, 'r') as f:
            cfg = yaml.safe_load(f)
    else:
        cfg = dict()
    update_recursive(cfg, cfg_special)
    return cfg


def update_recursive(dict1, dict2):
    """src/config.py:45-59."""
    for k, v in dict2.items():
        if k not in dict1:
            dict1[k] = dict()
        if isinstance(v, dict):
            update_recursive(dict1[k], v)
        else:
            dict1[k] = v


def get_model(cfg, nice=True):
    """src/config.py:63-79 (only the `nice=False` decoder has a native path)."""
    from .decoder import get_model as _gm
    return _gm(cfg, nice=nice)


# Effective rendering config of configs/pointNeRF_slam.yaml + configs/Replica/room0_point.yaml
# (SURVEY.md section 8), used by the bench and tests when no yaml tree is at hand.
ROOM0_CFG = {
    'rendering': {'N_samples': 32, 'N_surface': 0, 'N_importance': 12, 'lindisp': False, 'perturb': 0.0},
    'scale': 0.1, 'occupancy': False, 'data': {'dim': 3}, 'model': {'c_dim': 32, 'pos_embedding_method': 'fourier'},
    'mapping': {'pixels': 1000, 'iters': 60, 'imap_decoders_lr': 2e-4, 'w_color_loss': 0.05,
                'bound': [[-2.9, 8.9], [-3.2, 5.5], [-3.5, 3.3]]},
    'tracking': {'pixels': 200, 'iters': 10, 'lr': 1e-3, 'w_color_loss': 0.5},
    'grid_len': {'bound_divisible': 0.32},
    'cam': {'H': 680, 'W': 1200, 'fx': 600.0, 'fy': 600.0, 'cx': 599.5, 'cy': 339.5},
}
