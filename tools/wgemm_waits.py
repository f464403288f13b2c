#!/usr/bin/env python3
"""Print the VMEM issue / wait / barrier sequence of one wgemm_kernel instantiation from the
--save-temps .s (checks that no vmcnt wait in the main loop waits for the weight stream)."""
import re
import sys

s_file, key = sys.argv[1], sys.argv[2]  # e.g. ILi1ELi2ELi4E
txt = open(s_file).read()
for f in re.split(r'\n(?=_ZN2gq12_GLOBAL__N_112wgemm_kernel\S+:)', txt):
    if not f.startswith('_ZN2gq12_GLOBAL__N_112wgemm_kernel' + key):
        continue
    body = f.split('.Lfunc_end')[0].split('\n')
    out = []
    for l in body:
        t = l.strip()
        if 'buffer_load' in t:
            kind = 'X' if 's[4:7]' in t or 'dwordx4' in t and 'x4' in t else 'W'
            m = re.search(r'(buffer_load_\w+)\s+(\S+)', t)
            out.append(('L', m.group(1).replace('buffer_load_', ''), m.group(2)))
        elif 's_waitcnt' in t and 'vmcnt' in t:
            out.append(('WAIT', t.split('s_waitcnt')[1].strip()))
        elif t == 's_barrier':
            out.append(('BAR',))
        elif 'ds_write' in t:
            out.append(('DSW',))
        elif 'Loop Header' in t:
            out.append(('LOOP',))
        elif t.startswith('v_mfma'):
            if out and out[-1][0] == 'MFMA':
                out[-1] = ('MFMA', out[-1][1] + 1)
            else:
                out.append(('MFMA', 1))
    line = []
    for o in out:
        if o[0] == 'L':
            line.append(o[1])
        else:
            line.append(' '.join(str(x) for x in o))
    print(' | '.join(line))
