"""Per-unit HBM traffic (profiles/r*_traffic.json, read by bench.py pmc_traffic) from a
tools/prof_bench.sh traffic directory.

  python tools/traffic_json.py <gpurun_out/prof_<tag>_traffic> <out.json> [source note] [--mlp-points=N]

Per kernel family, the mean over its launches of (2 x FETCH_SIZE + WRITE_SIZE) bytes divided by the
units of that launch (tools/traffic.py documents the counter units and the gfx950 FETCH correction):
  k_mlp_fwd16_train  split-precision forward with activation saves, per point (128 points / 256-thread block)
  k_mlp_fwd16_eval   the same without saves
  k_mlp_bwd16        split-precision delta chain, per point (128 points / block)
  k_mlp_fwd_train    fp32 forward with saves, per point (grid = points)
  k_gather           probe + search of one gather, per sample (probe grid = sample rows)
  k_wgrad16_group    the grouped split weight-gradient GEMMs, per point (--mlp-points)
  k_wgrad_skinny     dWo + dB (fp32 FMA skinny GEMMs), per point (--mlp-points)
"""
import collections
import csv
import json
import os
import sys


def per_launch(d):
    """[(kernel, grid, bytes)] in launch order, FETCH x2 + WRITE, from the two pass directories."""
    out = {}
    for c, scale in (('FETCH_SIZE', 2.0), ('WRITE_SIZE', 1.0)):
        p = os.path.join(d, f'{c}_counter_collection.csv')
        rows = list(csv.DictReader(open(p)))
        per = collections.defaultdict(list)
        for r in rows:
            per[(r['Kernel_Name'], int(r['Grid_Size']))].append(float(r['Counter_Value']) * 1024.0 * scale)
        out[c] = per
    return out


def family(name):
    if 'k_mlp_fwd16w<' in name:  # the 16-point-wave forward (csrc/mlp16w.h): <save mode, waves>
        sv = name.split('<')[1].split('>')[0].split(',')[0].strip()
        return {'1': 'k_mlp_fwd16_train', '2': 'k_mlp_fwd16_masks'}.get(sv, 'k_mlp_fwd16_eval')
    if 'k_mlp_fwd16<' in name:  # last template argument: save mode (true / 1 training, 2 masks only)
        sv = name.split('>')[0].split(',')[-1].strip()
        return {'true': 'k_mlp_fwd16_train', '1': 'k_mlp_fwd16_train', '2': 'k_mlp_fwd16_masks'}.get(sv, 'k_mlp_fwd16_eval')
    if 'k_mlp_bwd16<' in name:
        return 'k_mlp_bwd16'
    if 'k_mlp_fwd<' in name and 'true' in name.split('>')[0]:
        return 'k_mlp_fwd_train'
    if 'k_gather_probe' in name:
        return 'k_gather_probe'
    if 'k_wgrad16_group' in name:
        return 'k_wgrad16_group'
    if 'k_wgrad_skinny' in name:
        return 'k_wgrad_skinny'
    if 'k_gather_search' in name or 'k_group_scatter' in name:
        return 'k_gather_search'  # (round 3: the grouped list's scatter belongs to the gather too)
    return None


def main():
    args = [a for a in sys.argv[1:] if not a.startswith('--mlp-points=')]
    mlp_pts = [int(a.split('=')[1]) for a in sys.argv[1:] if a.startswith('--mlp-points=')]
    d, dst = args[0], args[1]
    note = args[2] if len(args) > 2 else ''
    pl = per_launch(d)
    acc = collections.defaultdict(lambda: [0.0, 0.0, 0])  # fetch, write, units
    for c, per in pl.items():
        for (name, grid), vals in per.items():
            fam = family(name)
            if fam is None or fam == 'k_gather_search':
                continue
            units = grid / 2 if fam.startswith('k_mlp_') and '16' in fam else grid
            a = acc['k_gather' if fam == 'k_gather_probe' else fam]
            a[0 if c == 'FETCH_SIZE' else 1] += sum(vals)
            if c == 'FETCH_SIZE':
                a[2] += units * len(vals)
    # the search launches belong to the gather whose probe they follow: add their bytes
    for c, per in pl.items():
        for (name, grid), vals in per.items():
            if family(name) == 'k_gather_search':
                acc['k_gather'][0 if c == 'FETCH_SIZE' else 1] += sum(vals)
    # persistent MLP kernels run one workgroup per CU: their grid says nothing about the points, so
    # --mlp-points=N (the run's training points, the same for the forward and the delta chain)
    # replaces the grid-derived unit count of both families
    if mlp_pts:
        for fam in ('k_mlp_fwd16_train', 'k_mlp_bwd16', 'k_wgrad16_group', 'k_wgrad_skinny'):
            if fam in acc:
                acc[fam][2] = mlp_pts[0]
    res = {'source': note}
    for fam, (f, w, u) in sorted(acc.items()):
        if u <= 0:
            continue
        res[fam] = {'unit': 'sample' if fam == 'k_gather' else 'point',
                    'fetch_B': round(f / u, 1), 'write_B': round(w / u, 1)}
    json.dump(res, open(dst, 'w'), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
