"""MFMA-busy per kernel from a rocprofv3 --pmc pass of SQ_VALU_MFMA_BUSY_CYCLES + GRBM_GUI_ACTIVE.

  python tools/mfma_busy.py <dir> [out.json]

SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over every SIMD (32 per
v_mfma_*_32x32x16 instruction, MI355X_MICROARCH.md); GRBM_GUI_ACTIVE counts the dispatch's cycles
summed over the 8 XCDs.  busy = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8): the fraction of the
chip's MFMA issue slots the kernel filled.  The f16x3 kernels issue 3 MFMAs per fp32-equivalent
product, so busy x 833 TF is their fp32-equivalent rate at full clock."""
import collections
import csv
import glob
import json
import os
import sys

N_SIMD = 256 * 4


def main():
    d = sys.argv[1]
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for f in sorted(glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0]
            agg[k][r['Counter_Name']] += float(r['Counter_Value'])
            if r['Counter_Name'] == 'GRBM_GUI_ACTIVE':
                n[k] += 1
    out = {}
    for k, c in sorted(agg.items(), key=lambda kv: -kv[1].get('SQ_VALU_MFMA_BUSY_CYCLES', 0)):
        g = c.get('GRBM_GUI_ACTIVE', 0)
        if g <= 0 or c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) <= 0:
            continue
        busy = c['SQ_VALU_MFMA_BUSY_CYCLES'] / (N_SIMD * g / 8)
        out[k] = {'launches': n[k], 'mfma_busy_frac': round(busy, 4),
                  'SQ_VALU_MFMA_BUSY_CYCLES': c['SQ_VALU_MFMA_BUSY_CYCLES'], 'GRBM_GUI_ACTIVE': g,
                  'SQ_BUSY_CYCLES': c.get('SQ_BUSY_CYCLES')}
        print(f'{k[:60]:60s} launches {n[k]:4d}  MFMA busy {busy:6.3f}')
    if len(sys.argv) > 2:
        json.dump({'source': d, 'formula': 'SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8)',
                   'kernels': out}, open(sys.argv[2], 'w'), indent=1)


if __name__ == '__main__':
    main()
