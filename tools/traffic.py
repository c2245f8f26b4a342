"""HBM traffic per launch from rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/prof_bench.sh).

  python tools/traffic.py <dir with FETCH_SIZE_/WRITE_SIZE_counter_collection.csv> [filter]

Per (kernel, grid size): launches, mean FETCH and WRITE bytes per launch.  Units and the gfx950
correction follow MI355X_MICROARCH.md "HBM": the counters are in KiB; FETCH_SIZE reports half the
bytes of wide coalesced streaming reads, so fetched bytes are reported x2 (WRITE_SIZE is exact for
16-B-per-lane stores and float atomics).  Both are memory-side (fabric) counts: bytes served by L2
never appear, Infinity-Cache hits may.
"""
import collections
import csv
import json
import os
import sys


def load(path):
    out = collections.defaultdict(list)
    if not os.path.exists(path):
        return out
    for r in csv.DictReader(open(path)):
        out[(r['Kernel_Name'], int(r['Grid_Size']))].append(float(r['Counter_Value']) * 1024.0)
    return out


def summarize(d, filt=''):
    f = load(os.path.join(d, 'FETCH_SIZE_counter_collection.csv'))
    w = load(os.path.join(d, 'WRITE_SIZE_counter_collection.csv'))
    rows = []
    for key in sorted(set(f) | set(w), key=lambda k: -(sum(f.get(k, [0])) + sum(w.get(k, [0])))):
        name, grid = key
        if filt not in name:
            continue
        fv, wv = f.get(key, []), w.get(key, [])
        rows.append({'kernel': name, 'grid': grid, 'launches': max(len(fv), len(wv)),
                     'fetch_bytes': 2.0 * sum(fv) / len(fv) if fv else None,
                     'write_bytes': sum(wv) / len(wv) if wv else None})
    return rows


def main():
    rows = summarize(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else '')
    for r in rows[:40]:
        fb = f"{r['fetch_bytes'] / 1e6:10.1f}" if r['fetch_bytes'] is not None else '         -'
        wb = f"{r['write_bytes'] / 1e6:10.1f}" if r['write_bytes'] is not None else '         -'
        print(f"{r['kernel'][:60]:60s} grid {r['grid']:10d} x{r['launches']:3d}  fetch MB {fb}  write MB {wb}")
    if len(sys.argv) > 3:
        json.dump(rows, open(sys.argv[3], 'w'), indent=1)


if __name__ == '__main__':
    main()
