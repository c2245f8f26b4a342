"""Instruction mix per kernel of a hipcc --cuda-device-only -S assembly file.

  python tools/isa_mix.py file.s [name-filter]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
filt = sys.argv[2] if len(sys.argv) > 2 else ''
for m in re.finditer(r'\n(_Z\w+):[^\n]*\n(.*?)\.Lfunc_end', s, re.S):
    name, body = m.group(1), m.group(2)
    if filt not in name:
        continue
    c = collections.Counter()
    for line in body.splitlines():
        t = line.strip()
        if not t or t.startswith(('.', ';')) or t.endswith(':'):
            continue
        op = t.split()[0]
        key = ('mfma' if op.startswith('v_mfma') else 'accvgpr' if op.startswith('v_accvgpr') else
               'valu' if op.startswith('v_') else 'lds' if op.startswith('ds_') else
               'vmem_ld' if op.startswith(('global_load', 'buffer_load')) else
               'vmem_st' if op.startswith(('global_store', 'buffer_store')) else
               'waitcnt' if op.startswith('s_waitcnt') else 'barrier' if op.startswith('s_barrier') else
               'nop' if op.startswith('s_nop') else 'salu' if op.startswith('s_') else op)
        c[key] += 1
    print(name[:60], dict(sorted(c.items())))
