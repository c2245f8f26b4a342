"""Boundaries of tools/micro/launch_gap.hip's replayed graph: per position of the 16-launch body, the mean
duration and the mean gap from the previous launch's end (rocprofv3 kernel trace, csv).

    python tools/micro/launch_gap.py gpurun_out/lgap"""
import csv
import glob
import os
import sys

import numpy as np

rows = []
for f in glob.glob(os.path.join(sys.argv[1], '**', '*kernel_trace.csv'), recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
B = 16
rows = rows[B:]  # the eager warm-up body
n = len(rows) // B
rows = rows[B * 2:B * n]  # skip the first two replays
n = len(rows) // B
st = np.array([int(r['Start_Timestamp']) for r in rows], dtype=np.float64).reshape(n, B)
en = np.array([int(r['End_Timestamp']) for r in rows], dtype=np.float64).reshape(n, B)
names = [rows[i]['Kernel_Name'].split('(')[0].replace('void ', '') for i in range(B)]
lds = [rows[i].get('LDS_Block_Size', rows[i].get('Lds_Size', '?')) for i in range(B)]
prev_end = np.concatenate([np.full((n, 1), np.nan), en[:, :-1]], axis=1)
gap = (st - prev_end) / 1e3
dur = (en - st) / 1e3
print(f'{n} replays; per position: mean duration / mean gap from the previous end (us)')
for i in range(B):
    g = np.nanmean(gap[:, i]) if i > 0 else float('nan')
    print(f'{i:2d} {names[i]:14s} lds {lds[i]:>7s}  dur {np.mean(dur[:, i]):7.2f}  gap {g:6.2f}')
