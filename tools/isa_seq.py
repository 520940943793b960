"""Compact op sequence of a kernel in a hipcc -S listing between two s_barriers:
isa_seq.py file.s kernel-substring first_barrier_index [n_barriers]
M mfma, R ds_read, W ds_write, D LDS-DMA, G other vmem, a accvgpr move, v valu, s salu, |waitcnt"""
import sys
s = open(sys.argv[1]).read()
i = s.index(sys.argv[2])
i = s.index('\n', s.index(':', i))
j = s.index('s_endpgm', i)
body = [l.strip() for l in s[i:j].split('\n')]
bars = [n for n, l in enumerate(body) if l.startswith('s_barrier')]
k = int(sys.argv[3]); nb = int(sys.argv[4]) if len(sys.argv) > 4 else 1
print(len(bars), 'barriers')
out = []
for l in body[bars[k] - 3: bars[min(k + nb, len(bars) - 1)] + 2]:
    if not l or l.startswith(('.', ';')):
        continue
    if l.endswith(':'):
        out.append('\n' + l + '\n'); continue
    op = l.split()[0]
    t = ('M' if 'mfma' in op else 'R' if op.startswith('ds_read') else 'W' if op.startswith('ds_write') else 'w' if op == 's_waitcnt'
         else 'B' if op == 's_barrier' else 'D' if 'lds' in l and op.startswith('buffer') else 'a' if op.startswith('v_accvgpr')
         else 'v' if op.startswith('v_') else 's' if op.startswith('s_') else 'G' if op.startswith(('global', 'buffer')) else '?')
    out.append(t if t != 'w' else '|' + l.split()[1][:11])
print(' '.join(out))
