"""Device cache of the MFMA-ordered weight image (pnr_mlp_pack, csrc/mlp.hip:k_pack).

The image is a pure function of the 11 decoder tensors; it is rebuilt only when one of them
changed (data pointer or in-place version counter, e.g. after optimizer.step()).  One pack is a
~2 MB device-to-device permutation, negligible next to a render call.
"""
from __future__ import annotations

import torch

from . import _lib


class PackedMLP:
    """Image of the 11 reference tensors (pnr_mlp_pack)."""
    _floats = 'pnr_mlp_packed_floats'
    _pack = 'pnr_mlp_pack'
    _arr = 'PtrArray'

    def __init__(self):
        self._key = None
        self._img = None

    def invalidate(self):
        """Force a re-pack (weights were written in place outside autograd, e.g. pnr_adam_step)."""
        self._key = None

    def image(self, params) -> torch.Tensor:
        key = tuple((t.data_ptr(), t._version, t.device.index) for t in params)
        if self._img is not None and key == self._key:
            return self._img
        _lib.require_cuda(*params)
        lib = _lib.load()
        dev = params[0].device
        if self._img is None or self._img.device != dev:
            self._img = torch.empty(getattr(lib, self._floats)(), device=dev, dtype=torch.float32)
        srcs = [t.detach().float().contiguous() for t in params]
        arr = getattr(_lib, self._arr)(*[t.data_ptr() for t in srcs])
        _lib.check(getattr(lib, self._pack)(arr, _lib.ptr(self._img), _lib.stream_of(dev)), self._pack)
        self._srcs = srcs  # keep converted copies alive until the pack kernel ran
        self._key = key
        return self._img


class PackedFC(PackedMLP):
    """Image of the 8 fc_c tensors of MLP(c_dim=32) (pnr_fc_pack)."""
    _floats = 'pnr_fc_packed_floats'
    _pack = 'pnr_fc_pack'
    _arr = 'FcPtrArray'
