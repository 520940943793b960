"""Instruction-class counts per kernel of a hipcc -S assembly file: isa_mix.py file.s name-substring..."""
import sys
from collections import Counter

s = open(sys.argv[1]).read()
for name in sys.argv[2:]:
    i = s.index(name)
    i = s.index('\n', s.index(':', i))
    j = s.index('s_endpgm', i)
    c = Counter()
    for l in s[i:j].split('\n'):
        l = l.strip()
        if not l or l.startswith(('.', ';', '//')) or l.endswith(':'):
            continue
        x = l.split()[0]
        k = ('mfma' if 'mfma' in x else 'ds_read' if x.startswith('ds_read') else 'ds_write' if x.startswith('ds_write')
             else 'trans' if x.startswith(('v_exp', 'v_rcp', 'v_log', 'v_sqrt', 'v_rsq')) else 'valu' if x.startswith('v_')
             else 'salu' if x.startswith('s_') else 'vmem' if x.startswith(('buffer', 'global')) else x)
        c[k] += 1
    print(name, dict(c))
