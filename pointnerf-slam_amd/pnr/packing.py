"""Device cache of the MFMA-ordered weight image (pnr_mlp_pack, csrc/mlp.hip:k_pack).

The image is a pure function of the 11 decoder tensors; it is rebuilt only when one of them
changed (data pointer or in-place version counter, e.g. after optimizer.step()).  One pack is a
~2 MB device-to-device permutation, negligible next to a render call.

A Mapper iteration repacks after every Adam step, on its critical path: a caller that runs only the
f16x3 kernels asks for their images alone (`image(params, prec=PNR_PREC_F16X3)`, pnr_mlp_pack2 ABI 14:
no fp32 / bf16 images, bit for bit the f16x3 parts of a full pack); a later call that needs every
precision repacks.
"""
from __future__ import annotations

import torch

from . import _lib


class PackedMLP:
    """Image of the 11 reference tensors (pnr_mlp_pack)."""
    _floats = 'pnr_mlp_packed_floats'
    _pack = 'pnr_mlp_pack2'
    _arr = 'PtrArray'

    def __init__(self):
        self._key = None
        self._img = None
        self._cover_all = False  # the image holds every precision's parts (else the f16x3 ones only)

    def invalidate(self):
        """Force a re-pack (weights were written in place outside autograd, e.g. pnr_adam_step)."""
        self._key = None
        self._cover_all = False

    def image(self, params, prec=None) -> torch.Tensor:
        """The packed image of `params`; prec = PNR_PREC_F16X3 (int): only the f16x3 kernels will read it."""
        key = tuple((t.data_ptr(), t._version, t.device.index) for t in params)
        only = prec == _lib.PRECISIONS['f16x3']
        if self._img is not None and key == self._key and (self._cover_all or only):
            return self._img
        _lib.require_cuda(*params)
        lib = _lib.load()
        dev = params[0].device
        if self._img is None or self._img.device != dev:
            self._img = torch.empty(getattr(lib, self._floats)(), device=dev, dtype=torch.float32)
        srcs = [t.detach().float().contiguous() for t in params]
        arr = getattr(_lib, self._arr)(*[t.data_ptr() for t in srcs])
        flags = _lib.PACK_F16X3_ONLY if only else 0
        _lib.check(getattr(lib, self._pack)(arr, _lib.ptr(self._img), flags, _lib.stream_of(dev)), self._pack)
        self._srcs = srcs  # keep converted copies alive until the pack kernel ran
        self._key = key
        self._cover_all = not only
        return self._img


class PackedFC(PackedMLP):
    """Image of the 8 fc_c tensors of MLP(c_dim=32) (pnr_fc_pack)."""
    _floats = 'pnr_fc_packed_floats'
    _pack = 'pnr_fc_pack2'
    _arr = 'FcPtrArray'
