"""Instruction mix of every innermost loop (label marked 'Inner Loop Header' .. its back-branch) of
the kernels matching a substring in a hipcc -S listing: isa_loops.py file.s kernel-substring"""
import re, sys
from collections import Counter
s = open(sys.argv[1]).read()
for m in re.finditer(r'^(\S*' + re.escape(sys.argv[2]) + r'\S*):', s, re.M):
    i = m.end(); j = s.index('s_endpgm', i)
    body = s[i:j].split('\n')
    for n, l in enumerate(body):
        if 'Inner Loop Header' in l:
            lab = l.split(':')[0].strip() if l.strip().startswith('.LBB') else body[n - 1].split(':')[0].strip()
            end = next((k for k in range(n + 1, len(body)) if ('s_cbranch' in body[k] or 's_branch' in body[k]) and body[k].strip().endswith(lab)), None)
            if end is None:
                continue
            c = Counter()
            for x in body[n + 1:end + 1]:
                x = x.strip()
                if not x or x.startswith(('.', ';')) or x.endswith(':'):
                    continue
                op = x.split()[0]
                k = ('mfma' if 'mfma' in op else 'trans' if op.startswith(('v_exp', 'v_rcp', 'v_log')) else
                     'pk' if op.startswith('v_pk') else 'valu' if op.startswith('v_') else 'ds_read' if op.startswith('ds_read')
                     else 'ds_write' if op.startswith('ds_write') else 'salu' if op.startswith('s_') else 'vmem' if op.startswith(('buffer', 'global')) else op)
                c[k] += 1
            print(m.group(1)[:60], lab, end - n, dict(c))
