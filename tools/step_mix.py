"""Per-barrier-segment instruction mix of one kernel in a hipcc -S assembly file (the step program of
the MLP kernels: one s_barrier per step).  usage: python tools/step_mix.py file.s <mangled-name-prefix> [n]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
m = re.search(r'\n(' + re.escape(sys.argv[2]) + r'\w*):[^\n]*\n(.*?)\.Lfunc_end', s, re.S)
segs, cur = [], collections.Counter()
for line in m.group(2).splitlines():
    t = line.strip()
    if not t or t.startswith(('.', ';')) or t.endswith(':'):
        continue
    op = t.split()[0]
    if op == 's_barrier':
        segs.append(cur)
        cur = collections.Counter()
    key = ('mfma' if op.startswith('v_mfma') else 'accr' if op.startswith('v_accvgpr_read') else
           'accw' if op.startswith('v_accvgpr_write') else 'cvt' if op.startswith(('v_cvt', 'v_fma_mix')) else
           'valu' if op.startswith('v_') else 'lds' if op.startswith('ds_') else
           'glds' if 'global_load_lds' in op else 'vmem' if op.startswith(('global', 'buffer')) else
           'wait' if op.startswith('s_waitcnt') else 'nop' if op.startswith('s_nop') else
           'salu' if op.startswith('s_') else op)
    cur[key] += 1
segs.append(cur)
n = int(sys.argv[3]) if len(sys.argv) > 3 else 12
for i, c in enumerate(segs[:n]):
    print(i, dict(sorted(c.items())))
