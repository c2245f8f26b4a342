"""ctypes binding of libpnr.so (the C ABI declared in include/pnr.h).

The library is built in-tree (`pointnerf-slam_amd/pnr/libpnr.so`, see the Makefile) and loaded
lazily on first use, after torch, so that it shares torch's HIP runtime (same SONAME).  There is
no fallback: if the library is missing or cannot be loaded every GPU entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

# PNR_LIB_PATH: an experiment build (tools/xbuild.sh) to run the tests against instead
LIB_PATH = os.environ.get('PNR_LIB_PATH') or os.path.join(os.path.dirname(os.path.abspath(__file__)), 'libpnr.so')
MAX_SAMPLES = 64
N_PARAMS = 11
N_FC_PARAMS = 8
C_DIM = 32
MAX_K = 8
GATHER_IDW, GATHER_TRILINEAR = 0, 1
# decoder matmul arithmetic (include/pnr.h PNR_PREC_*)
PRECISIONS = {'fp32': 0, 'bf16x3': 1, 'bf16': 2, 'f16x3': 3}
# f16x3: fp32-class forward AND backward (every GEMM on 22-bit split operands with fp32
# accumulation; tests/test_gpu_parity.py runs every case under fp32 and f16x3 at the same tolerances)
DEFAULT_PRECISION = os.environ.get('PNR_PRECISION', 'f16x3')
ABI_VERSION = 14
STATUS_F16_RANGE = 1  # include/pnr.h PNR_STATUS_F16_RANGE


def precision_code(name) -> int:
    """PNR_PREC_* code of a precision name ('fp32' | 'bf16x3' | 'bf16')."""
    if name not in PRECISIONS:
        raise ValueError(f'pnr: unknown decoder precision {name!r} (one of {sorted(PRECISIONS)})')
    return PRECISIONS[name]

c_void_p = ctypes.c_void_p
c_int64 = ctypes.c_int64
c_int32 = ctypes.c_int32
c_size_t = ctypes.c_size_t
c_float = ctypes.c_float


class Points(ctypes.Structure):
    """Mirror of `pnr_points` (include/pnr.h)."""
    _fields_ = [
        ('xyz', c_void_p), ('feats', c_void_p), ('n_points', c_int64), ('mode', c_int32), ('k', c_int32),
        ('radius', c_float), ('eps', c_float), ('spacing', c_float * 3), ('cell', c_float),
        ('origin', c_float * 3), ('table_bits', c_int32), ('index', c_void_p), ('fc_packed', c_void_p),
        ('g_feats', c_void_p), ('g_fc', c_void_p), ('feat_half', c_int32),
    ]


class RenderParams(ctypes.Structure):
    """Mirror of `pnr_render_params` (include/pnr.h)."""
    _fields_ = [
        ('n_samples', c_int32), ('n_importance', c_int32), ('lindisp', c_int32), ('far_mode', c_int32),
        ('bound', ctypes.c_double * 6), ('far_clamp', ctypes.c_double),
        ('t_vals', c_float * MAX_SAMPLES), ('u_vals', c_float * MAX_SAMPLES),
        ('save_for_backward', c_int32), ('need_ray_grads', c_int32),
        ('points', ctypes.POINTER(Points)), ('precision', c_int32), ('grads_overwrite', c_int32),
        ('status', c_void_p), ('far_clamp_dev', c_void_p),
    ]


PtrArray = c_void_p * N_PARAMS
FcPtrArray = c_void_p * N_FC_PARAMS
PPoints = ctypes.POINTER(Points)
PACK_F16X3_ONLY = 2  # include/pnr.h PNR_PACK_F16X3_ONLY

# name -> (restype, argtypes)
_SIGS = {
    'pnr_abi_version': (ctypes.c_int, []),
    'pnr_build_info': (ctypes.c_char_p, []),
    'pnr_mlp_packed_floats': (c_size_t, []),
    'pnr_mlp_pack': (ctypes.c_int, [PtrArray, c_void_p, c_void_p]),
    'pnr_mlp_pack2': (ctypes.c_int, [PtrArray, c_void_p, c_int32, c_void_p]),
    'pnr_eval_points': (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p]),
    'pnr_eval_points_f32': (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_void_p]),
    'pnr_mlp_train_workspace_bytes': (c_size_t, [c_int64]),
    'pnr_mlp_fwd_train': (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_size_t, c_int32,
                                         c_void_p]),
    'pnr_mlp_bwd_workspace_bytes': (c_size_t, [c_int64]),
    'pnr_mlp_bwd': (ctypes.c_int, [c_void_p, c_int64, c_void_p, PtrArray, c_void_p, c_void_p, c_size_t,
                                   c_void_p, c_size_t, c_int32, c_void_p]),
    'pnr_render_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_render_fwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    'pnr_render_bwd_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_render_bwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p, c_int64,
                                      c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                      c_void_p, c_size_t, c_void_p, c_size_t, c_void_p]),  # grads: PtrArray or None
    'pnr_regulation_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_regulation_fwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_void_p, c_int64, c_void_p, c_void_p, c_size_t, c_void_p]),
    'pnr_regulation_bwd_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_regulation_bwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                          c_void_p, c_size_t, c_void_p]),
    'pnr_map_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_map_fwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t, c_void_p]),
    'pnr_map_bwd_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_map_bwd': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_void_p]),
    'pnr_map_step_workspace_bytes': (c_size_t, [ctypes.POINTER(RenderParams), c_int64]),
    'pnr_map_step': (ctypes.c_int, [ctypes.POINTER(RenderParams), c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_void_p, c_int64, c_float, c_float, c_void_p, c_void_p, c_void_p, c_size_t,
                                    c_void_p, c_size_t, c_void_p, c_void_p]),
    'pnr_get_rays': (ctypes.c_int, [c_int32, c_int32, c_float, c_float, c_float, c_float, c_void_p, c_void_p,
                                    c_void_p, c_void_p]),
    'pnr_rays_from_uv': (ctypes.c_int, [c_void_p, c_void_p, c_int64, c_float, c_float, c_float, c_float, c_void_p,
                                        c_void_p, c_void_p, c_void_p]),
    'pnr_window_rays': (ctypes.c_int, [c_void_p, c_int64, c_int64, c_int32, c_int32, c_float, c_float, c_float,
                                       c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                       c_void_p]),
    'pnr_window_sample_state_bytes': (c_size_t, []),
    'pnr_window_sample': (ctypes.c_int, [ctypes.c_uint64, c_void_p, c_int64, c_int64, c_int32, c_int32, c_float,
                                         c_float, c_float, c_float, c_void_p, c_void_p, c_void_p, c_int32, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'pnr_adam_step': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float, c_float,
                                     c_float, c_int64, c_void_p]),
    'pnr_adam_step_dev': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_float,
                                         c_float, c_float, c_void_p, c_void_p]),
    'pnr_step_advance': (ctypes.c_int, [c_void_p, c_void_p]),
    'pnr_adam_multi_dev': (ctypes.c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                          c_float, c_float, c_float, c_void_p, c_void_p]),
    'pnr_adam_multi_dev_h': (ctypes.c_int, [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_float, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    'pnr_map_loss_workspace_bytes': (c_size_t, []),
    'pnr_map_loss': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_float, c_void_p, c_int64,
                                    c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    'pnr_points_index_bytes': (c_size_t, [c_int64, c_int32]),
    'pnr_points_build': (ctypes.c_int, [PPoints, c_void_p]),
    'pnr_point_gather_workspace_bytes': (c_size_t, [c_int64]),
    'pnr_point_gather': (ctypes.c_int, [PPoints, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_size_t,
                                        c_void_p]),
    'pnr_point_gather_bwd_workspace_bytes': (c_size_t, [PPoints, c_int64]),
    'pnr_point_gather_bwd': (ctypes.c_int, [PPoints, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p,
                                            c_void_p, c_void_p, c_size_t, c_void_p]),
    'pnr_point_gather_bwd_atomics': (ctypes.c_int, [PPoints, c_void_p, c_int64, ctypes.POINTER(c_int64), c_void_p]),
    'pnr_fc_packed_floats': (c_size_t, []),
    'pnr_fc_pack': (ctypes.c_int, [FcPtrArray, c_void_p, c_void_p]),
    'pnr_fc_pack2': (ctypes.c_int, [FcPtrArray, c_void_p, c_int32, c_void_p]),
    'pnr_eval_points_c': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                         c_int32, c_void_p]),
    'pnr_mlp_fwd_train_c': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p,
                                           c_size_t, c_int32, c_void_p]),
    'pnr_mlp_bwd_workspace_bytes_c': (c_size_t, [c_int64]),
    'pnr_mlp_bwd_c': (ctypes.c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, PtrArray, FcPtrArray,
                                     c_void_p, c_void_p, c_void_p, c_size_t, c_void_p, c_size_t, c_int32, c_void_p]),
    'pnr_timing_enable': (ctypes.c_int, [ctypes.c_int]),
    'pnr_timing_read': (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_int64), ctypes.POINTER(ctypes.c_double),
                                       ctypes.POINTER(c_int64)]),
}
SYMBOLS = tuple(_SIGS)


def timing_read(kernel: int):
    """(launches, device ms, units) recorded for `kernel` since the last read (pnr_timing_read)."""
    n, ms, u = c_int64(0), ctypes.c_double(0.0), c_int64(0)
    check(load().pnr_timing_read(kernel, ctypes.byref(n), ctypes.byref(ms), ctypes.byref(u)), 'timing_read')
    return n.value, ms.value, u.value

_lib = None
_lock = threading.Lock()


def load(path: str = LIB_PATH):
    """Load (once) and return the ctypes library; raises RuntimeError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(path):
                raise RuntimeError(f'pnr: HIP library {path} not built (run `make -C pointnerf-slam_amd`)')
            lib = ctypes.CDLL(path)
            for name, (res, args) in _SIGS.items():
                fn = getattr(lib, name)
                fn.restype = res
                fn.argtypes = args
            _lib = lib
    return _lib


def check(rc: int, what: str):
    if rc != 0:
        kind = {-1: 'bad argument', -2: 'workspace too small'}.get(rc, f'hipError {rc}')
        raise RuntimeError(f'pnr: {what} failed ({kind})')


def ptr(t) -> c_void_p:
    return c_void_p(0 if t is None else t.data_ptr())


def stream_of(device=None) -> c_void_p:
    return c_void_p(torch.cuda.current_stream(device).cuda_stream)


def require_cuda(*tensors):
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError('pnr: the renderer runs on the MI355X HIP path only; got a CPU tensor '
                               '(the CPU restatement lives in oracle/, test infrastructure only)')
