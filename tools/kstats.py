"""Per-kernel duration summary from a rocprofv3 results database (.db) or kernel_trace.csv.

  python tools/kstats.py <file> [name-filter]
"""
import collections
import csv
import sqlite3
import sys


def rows(path):
    if path.endswith('.csv'):
        for r in csv.DictReader(open(path)):
            yield r['Kernel_Name'], int(r['End_Timestamp']) - int(r['Start_Timestamp'])
        return
    db = sqlite3.connect(path)
    q = ("select s.kernel_name, d.end - d.start from rocpd_kernel_dispatch d "
         "join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
    for name, dur in db.execute(q):
        yield name, dur


def main():
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ''
    agg = collections.defaultdict(list)
    for name, dur in rows(path):
        if filt in name:
            agg[name].append(dur)
    tot = sum(sum(v) for v in agg.values())
    print(f'{"kernel":70s} {"calls":>6s} {"total ms":>10s} {"avg ms":>9s} {"%":>6s}')
    for name, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f'{name[:70]:70s} {len(v):6d} {sum(v) / 1e6:10.3f} {sum(v) / len(v) / 1e6:9.4f} {100 * sum(v) / tot:6.1f}')


if __name__ == '__main__':
    main()
