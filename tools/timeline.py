"""Timeline of one replayed iteration from a rocprofv3 kernel trace (--kernel-trace, csv).

    python tools/timeline.py <dir with *kernel_trace.csv> [--iter K] [--period-kernel NAME]

Splits the dispatches into iterations at each launch of the period kernel (default: the Adam
kernel, the last of a mapping step), prints iteration K's dispatches in start order with their start
offset, duration and queue, and the sum of the gaps where no kernel runs (launch / dependency
latency) against the iteration's span."""
import argparse
import csv
import glob
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--iter', type=int, default=-3)
    ap.add_argument('--period-kernel', default='k_adam_dev')
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.dir, '**', '*kernel_trace.csv'), recursive=True)
    rows = []
    for f in files:
        rows += list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    cuts = [i for i, r in enumerate(rows) if a.period_kernel in r['Kernel_Name']]
    if len(cuts) < 3:
        print('too few iterations', len(cuts))
        return
    k = a.iter
    lo, hi = cuts[k - 1] + 1, cuts[k] + 1
    it = rows[lo:hi]
    t0 = int(it[0]['Start_Timestamp'])
    busy_end, gaps = t0, 0
    print(f'{len(cuts)} iterations; iteration {k}: {len(it)} dispatches')
    for r in it:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        if s > busy_end:
            gaps += s - busy_end
        busy_end = max(busy_end, e)
        q = r.get('Queue_Id', r.get('Stream_Id', ''))
        print(f'{(s - t0) / 1e3:8.1f} us  {(e - s) / 1e3:7.1f} us  q{q:>3}  {r["Kernel_Name"][:100]}')
    span = busy_end - t0
    per = [(int(rows[cuts[i]]['End_Timestamp']) - int(rows[cuts[i - 1]]['End_Timestamp'])) / 1e3
           for i in range(1, len(cuts))]
    per.sort()
    print(f'span {span / 1e3:.1f} us, idle gaps {gaps / 1e3:.1f} us; median iteration period '
          f'{per[len(per) // 2]:.1f} us')


if __name__ == '__main__':
    main()
