"""The C-ABI library loads and exports every symbol include/pnr.h declares (no GPU needed)."""
import ctypes
import os
import re

import pytest

from conftest import REPO

HDR = os.path.join(REPO, 'include', 'pnr.h')
LIB = os.path.join(REPO, 'pointnerf-slam_amd', 'pnr', 'libpnr.so')


def declared_symbols():
    txt = open(HDR).read()
    txt = re.sub(r'/\*.*?\*/', '', txt, flags=re.S)
    return sorted(set(re.findall(r'\b(pnr_[a-z0-9_]+)\s*\(', txt)))


@pytest.fixture(scope='module')
def lib():
    if not os.path.exists(LIB):
        pytest.fail(f'{LIB} missing: run `make -C pointnerf-slam_amd` (or __graft_entry__.build())')
    return ctypes.CDLL(LIB)


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert 'pnr_render_fwd' in syms and 'pnr_render_bwd' in syms and len(syms) >= 20


def test_every_declared_symbol_exported(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_python_binding_covers_header():
    import sys
    sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
    from pnr import _lib
    assert set(_lib.SYMBOLS) == set(declared_symbols())


def test_host_only_calls(lib):
    lib.pnr_abi_version.restype = ctypes.c_int
    assert lib.pnr_abi_version() == 14
    lib.pnr_mlp_packed_floats.restype = ctypes.c_size_t
    # fp32 images 486,688 + bf16x3 / bf16 / f16x3 forward streams 229,376 / 118,784 / 229,376
    # + f16x3 delta-chain stream 225,280 + raw table 2,048 + fp32 Wo 1,024
    assert lib.pnr_mlp_packed_floats() == 486688 + 229376 + 118784 + 229376 + 225280 + 3072 + 225280
    lib.pnr_build_info.restype = ctypes.c_char_p
    assert b'gfx950' in lib.pnr_build_info()


def test_params_struct_layout():
    import sys
    sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
    from pnr import _lib
    # int32 x4, double[6], double, float[64] x2, int32 x2, pointer, int32, 2 pointers (ABI 7)
    assert ctypes.sizeof(_lib.RenderParams) == 624
    assert _lib.RenderParams.precision.offset == 600
    assert _lib.RenderParams.status.offset == 608 and _lib.RenderParams.far_clamp_dev.offset == 616
    assert _lib.RenderParams.bound.offset == 16 and _lib.RenderParams.t_vals.offset == 72
    assert _lib.RenderParams.points.offset == 592
    # pnr_points: 2 ptr, int64, 2 int32, 2 float, float[3], float, float[3], int32, 4 ptr, int32 (ABI 6)
    assert _lib.Points.n_points.offset == 16 and _lib.Points.spacing.offset == 40
    assert _lib.Points.table_bits.offset == 68 and _lib.Points.index.offset == 72
    assert _lib.Points.feat_half.offset == 104 and ctypes.sizeof(_lib.Points) == 112


def test_workspace_queries_and_arg_errors(lib):
    import sys
    sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
    from pnr import _lib
    L = _lib.load()
    prm = _lib.RenderParams()
    prm.n_samples, prm.n_importance = 32, 12
    assert L.pnr_render_workspace_bytes(ctypes.byref(prm), 1000) > 1000 * 44 * (8 + 16)
    prm.save_for_backward = 1
    big = L.pnr_render_workspace_bytes(ctypes.byref(prm), 1000)
    assert big > 1000 * 44 * 4 * 1024
    assert L.pnr_render_bwd_workspace_bytes(ctypes.byref(prm), 1000) > 0
    bad = _lib.RenderParams()
    bad.n_samples, bad.n_importance = 40, 30          # > 64 samples per ray
    assert L.pnr_render_workspace_bytes(ctypes.byref(bad), 10) == 0
    bad2 = _lib.RenderParams()
    bad2.n_samples, bad2.n_importance, bad2.far_mode = 32, 12, 2   # device far clamp without a pointer
    assert L.pnr_render_workspace_bytes(ctypes.byref(bad2), 10) == 0
    # argument errors are reported without touching the device
    assert L.pnr_render_fwd(ctypes.byref(bad), None, None, None, None, 10, None, None, None, None, 0, None) == -1
    assert L.pnr_eval_points(None, None, 5, None, None, 0, None) == -1
    assert L.pnr_adam_step(None, None, None, None, 5, 1e-3, 0.9, 0.999, 1e-8, 0, None) == -1
    assert L.pnr_adam_step_dev(None, None, None, None, 5, 1e-3, 0.9, 0.999, 1e-8, None, None) == -1
    assert L.pnr_step_advance(None, None) == -1
    # ABI 13 / 14: the one-call map step (workspace = the map workspace + its per-ray scratch; a missing
    # loss or loss workspace is an argument error) and the flagged repacks (unknown flag bits refused)
    mp = _lib.RenderParams()
    mp.n_samples, mp.n_importance, mp.precision = 32, 12, 3
    assert L.pnr_map_step_workspace_bytes(ctypes.byref(mp), 1000) > L.pnr_map_workspace_bytes(ctypes.byref(mp), 1000)
    assert L.pnr_map_step_workspace_bytes(ctypes.byref(bad), 1000) == 0
    assert L.pnr_map_step(ctypes.byref(mp), ctypes.c_void_p(1), None, None, None, None, None, 10, 0.2, 5e-4, None,
                          None, None, 0, None, 0, None, None) == -1
    arr = _lib.PtrArray(*([1] * _lib.N_PARAMS))
    assert L.pnr_mlp_pack2(arr, ctypes.c_void_p(1), 4, None) == -1
    assert L.pnr_mlp_pack2(arr, None, _lib.PACK_F16X3_ONLY, None) == -1
    farr = _lib.FcPtrArray(*([1] * _lib.N_FC_PARAMS))
    assert L.pnr_fc_pack2(farr, ctypes.c_void_p(1), 1, None) == -1
    # zero-sized calls are no-ops
    assert L.pnr_eval_points(ctypes.c_void_p(1), None, 0, None, None, 0, None) == 0


def test_point_queries_and_arg_errors(lib):
    import sys
    sys.path.insert(0, os.path.join(REPO, 'pointnerf-slam_amd'))
    from pnr import _lib
    L = _lib.load()
    assert L.pnr_fc_packed_floats() == 12 * 8192 + 4 * 32768 + 2048  # fp32 + four 16-bit images + raw
    b20 = L.pnr_points_index_bytes(100000, 20)
    assert b20 >= (2 * (1 << 20) + 2 * 100000) * 4 + 100000 * 16
    assert L.pnr_points_index_bytes(100000, 9) == 0 and L.pnr_points_index_bytes(-1, 12) == 0
    pts = _lib.Points()
    pts.k, pts.table_bits, pts.cell = 9, 12, 0.1           # k > PNR_MAX_K
    assert L.pnr_point_gather(ctypes.byref(pts), None, 0, None, None, None, None, 0, None) == -1
    assert L.pnr_point_gather_workspace_bytes(1000) >= 16000
    # the cell-size bound at its limit (points.hip kCellMargin): cell = 2 radius is refused, a cell
    # just above 2 radius (1 + 2^-9) is accepted (P = 0: no compute, no device access)
    edge = _lib.Points()
    edge.mode, edge.k, edge.table_bits, edge.radius, edge.n_points = 0, 8, 12, 0.05, 0
    edge.index = ctypes.c_void_p(16)
    edge.cell = 0.1
    assert L.pnr_point_gather(ctypes.byref(edge), None, 0, None, None, None, None, 0, None) == -1
    edge.cell = 0.1 * (1 + 2.0 ** -8)
    assert L.pnr_point_gather(ctypes.byref(edge), None, 0, None, None, None, None, 0, None) == 0
    assert L.pnr_points_build(None, None) == -1
    assert L.pnr_eval_points_c(None, None, None, None, 3, None, None, 0, None) == -1
