"""The bench line's roofline bookkeeping on the CPU (no GPU calls): the grouped weight-gradient launch
sits on the HBM side of the roofline (its FLOP per algorithmic operand byte is below the machine
balance), its traffic comes from the committed PMC measurement of the same workload when there is one,
and the traffic tool maps the 16-point-wave forward's template arguments <save mode, waves> to the right
kernel family."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, 'tools'))


def test_weight_gradients_are_below_the_ridge():
    import bench
    ridge = bench.ALGO_PEAK_TF['f16x3'] * 1e3 / bench.HBM_PEAK_GBS  # FLOP per byte at the roof's corner
    assert bench.WGRAD_FLOP_PER_POINT / bench.WGRAD_B_PER_POINT < ridge
    assert ((bench.WGRAD_FLOP_PER_POINT + bench.WGRAD_FC_FLOP_PER_POINT)
            / (bench.WGRAD_B_PER_POINT + bench.WGRAD_FC_B_PER_POINT)) < ridge
    # and the MLP kernels above it (their roofline stays the MFMA one)
    assert bench.FLOP_PER_POINT_FWD / 4096 > ridge


def test_kernel_roofline_hbm_basis_for_the_grouped_launch():
    import bench
    pts, launches, ms = 76032, 10, 1.55  # ten launches of 155 us over 76,032 points each
    macs = 443430 // 2 * pts // 65536   # pnr_timing_read kind 6 units per launch
    kt = {'wgrad_group': (launches, ms, macs * launches), 'mlp_bwd': (launches, 1.4, pts * launches)}
    r = bench.kernel_roofline(kt, 'f16x3', 5e-3, traffic_units=True, workload='room0')
    assert r['bound'] == 'hbm' and r['unit'] == 'GB/s' and r['kernel'] == 'k_wgrad16_group'
    gbs = bench.WGRAD_B_PER_POINT * pts / 155e-6 / 1e9
    assert abs(r['achieved'] - gbs) < 1.0 and abs(r['frac'] - gbs / bench.HBM_PEAK_GBS) < 1e-3
    assert 0 < r['frac_of_split_peak'] < r['frac']
    # the room0 PMC pass (profiles/r06_traffic_room0.json) holds the launch's own bytes
    t = json.load(open(os.path.join(REPO, 'profiles', 'r06_traffic_room0.json')))['k_wgrad16_group@room0']
    assert r['traffic'] == round((t['fetch_B'] + t['write_B']) * pts)


def test_pmc_traffic_prefers_the_workload_measurement():
    import bench
    room0 = bench.pmc_traffic('k_wgrad16_group', 1000, 'room0')
    smap = bench.pmc_traffic('k_wgrad16_group', 1000)
    assert room0 is not None and smap is not None and room0 > smap  # the partial tiles' writes at room0


def test_traffic_family_of_the_16_point_wave_forward():
    import traffic_json
    assert traffic_json.family('void pnr::k_mlp_fwd16w<1, 8>(pnr::BfFwdArgs, int, pnr::MapRowsArgs)') == \
        'k_mlp_fwd16_train'
    assert traffic_json.family('void pnr::k_mlp_fwd16w<1, 4>(pnr::BfFwdArgs, int, pnr::MapRowsArgs)') == \
        'k_mlp_fwd16_train'
    assert traffic_json.family('void pnr::k_mlp_fwd16w<0, 4>(pnr::BfFwdArgs, int, pnr::MapRowsArgs)') == \
        'k_mlp_fwd16_eval'
    assert traffic_json.family('void pnr::k_mlp_fwd16w<2, 8>(pnr::BfFwdArgs, int, pnr::MapRowsArgs)') == \
        'k_mlp_fwd16_masks'
