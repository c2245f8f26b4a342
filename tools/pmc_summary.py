"""Average PMC counter values per kernel from rocprofv3 --pmc csv passes in a directory.

  python tools/pmc_summary.py <dir> [kernel-filter]
"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    res = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(os.path.join(d, '*_counter_collection.csv'))):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            if filt and filt not in k:
                continue
            res[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, dd in res.items():
        print(k[:90])
        for c, v in sorted(dd.items()):
            print(f'    {c:34s} {sum(v) / len(v):14.4g}   (n={len(v)})')


if __name__ == '__main__':
    main()
