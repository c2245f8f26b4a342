"""Checkpoint interop with the reference's Logger (SURVEY.md section 8 (f) row F4;
src/utils/Logger.py:6-32).

`Logger.log` writes `<ckptsdir>/<idx:05d>.tar` with the reference's keys and legacy
(non-zip) serialisation, so the reference's eval tools and `run.py` resume read it, and
`load_ckpt` reads a reference checkpoint (a `.tar` from the reference's output tree) with
`torch.load(weights_only=True)` -- nothing in the file is executed.

The decoder state_dict has the reference's key names (pnr.MLP is state_dict-compatible).  Neural
points ride in `c` as plain tensors -- {'points_<name>': {'xyz', 'feats', 'mode',
'k', 'radius', 'eps', 'spacing', 'cell', 'origin', 'table_bits'}} -- so a checkpoint never
pickles a module; an empty `c` is the reference's own `{}`.
"""
from __future__ import annotations

import os

import torch

from .points import NeuralPoints

CKPT_KEYS = ('c', 'decoder_state_dict', 'gt_c2w_list', 'estimate_c2w_list', 'keyframe_list',
             'selected_keyframes', 'idx')  # src/utils/Logger.py:23-31
_PT_FIELDS = ('mode', 'k', 'radius', 'eps', 'spacing', 'cell', 'origin', 'table_bits', 'feat_dtype')


def c_state(c):
    """`c` with NeuralPoints replaced by plain tensors / scalars (weights_only-loadable)."""
    out = {}
    for key, v in (c or {}).items():
        if isinstance(v, NeuralPoints):
            d = {'xyz': v.xyz.detach().cpu(), 'feats': v.feats.detach().cpu()}
            d.update({f: getattr(v, f) for f in _PT_FIELDS})
            out[key] = d
        elif isinstance(v, torch.Tensor):
            out[key] = v.detach().cpu()
        else:
            out[key] = v
    return out


def c_from_state(cs, device='cpu'):
    """Inverse of c_state: rebuild NeuralPoints on `device`."""
    out = {}
    for key, v in (cs or {}).items():
        if isinstance(v, dict) and 'xyz' in v and 'feats' in v:
            kw = {f: v[f] for f in _PT_FIELDS if f in v}
            out[key] = NeuralPoints(v['xyz'].to(device), v['feats'].to(device), c_dim=v['feats'].shape[1], **kw)
        else:
            out[key] = v
    return out


class Logger(object):
    """src/utils/Logger.py:6-17: reads ckptsdir, shared_c, gt_c2w_list, shared_decoders and
    estimate_c2w_list from `slam`."""

    def __init__(self, cfg, args, slam):
        self.verbose = getattr(slam, 'verbose', False)
        self.ckptsdir = slam.ckptsdir
        self.shared_c = slam.shared_c
        self.gt_c2w_list = slam.gt_c2w_list
        self.shared_decoders = slam.shared_decoders
        self.estimate_c2w_list = slam.estimate_c2w_list

    def log(self, idx, keyframe_dict, keyframe_list, selected_keyframes=None):
        """src/utils/Logger.py:19-35 (keyframe_dict is not saved, as in the reference)."""
        path = os.path.join(self.ckptsdir, '{:05d}.tar'.format(idx))
        save_ckpt(path, self.shared_c, self.shared_decoders, self.gt_c2w_list, self.estimate_c2w_list,
                  keyframe_list, selected_keyframes, idx)
        if self.verbose:
            print('Saved checkpoints at', path)
        return path


def save_ckpt(path, c, decoders, gt_c2w_list, estimate_c2w_list, keyframe_list, selected_keyframes, idx):
    sd = {k: v.detach().cpu() for k, v in decoders.state_dict().items()}
    torch.save({
        'c': c_state(c),
        'decoder_state_dict': sd,
        'gt_c2w_list': gt_c2w_list.detach().cpu() if isinstance(gt_c2w_list, torch.Tensor) else gt_c2w_list,
        'estimate_c2w_list': (estimate_c2w_list.detach().cpu() if isinstance(estimate_c2w_list, torch.Tensor)
                              else estimate_c2w_list),
        'keyframe_list': keyframe_list,
        'selected_keyframes': selected_keyframes,
        'idx': idx,
    }, path, _use_new_zipfile_serialization=False)


def load_ckpt(path, decoders=None, device='cpu'):
    """Read a checkpoint (ours or the reference's) with torch.load(weights_only=True).  Loads the
    decoder weights into `decoders` when given; returns the dict with `c` rebuilt on `device`."""
    ck = torch.load(path, map_location='cpu', weights_only=True)
    missing = [k for k in ('decoder_state_dict', 'gt_c2w_list', 'estimate_c2w_list', 'idx') if k not in ck]
    if missing:
        raise KeyError(f'pnr.load_ckpt: {path} lacks {missing}')
    if decoders is not None:
        decoders.load_state_dict(ck['decoder_state_dict'])
    ck['c'] = c_from_state(ck.get('c', {}), device)
    return ck
