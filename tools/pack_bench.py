"""Weight-image repack timing (pnr_mlp_pack2 / pnr_fc_pack2, ABI 14): the full pack (flags 0) against
the f16x3-only pack (PNR_PACK_F16X3_ONLY), device time per call from hipEvents around 200 calls."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'pointnerf-slam_amd'))


def main():
    import pnr
    from pnr import _lib
    dev = torch.device('cuda:0')
    dec = pnr.get_model(pnr.ROOM0_CFG, nice=False).to(dev)
    params = [p.detach().float().contiguous() for p in dec.ordered_params()]
    lib = _lib.load()
    img = torch.empty(lib.pnr_mlp_packed_floats(), device=dev)
    arr = _lib.PtrArray(*[t.data_ptr() for t in params])
    st = _lib.stream_of(dev)
    out = {}
    for name, flags in (('full', 0), ('f16x3_only', _lib.PACK_F16X3_ONLY)):
        for _ in range(10):
            lib.pnr_mlp_pack2(arr, _lib.ptr(img), flags, st)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            lib.pnr_mlp_pack2(arr, _lib.ptr(img), flags, st)
        b.record()
        torch.cuda.synchronize()
        out[name + '_us'] = round(a.elapsed_time(b) / 200 * 1e3, 2)
    print(json.dumps(out))


if __name__ == '__main__':
    main()
