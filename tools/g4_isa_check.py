"""Static check of gemm4 instantiations in a hipcc -S listing: the epilogue issues exactly the
vector-memory ops the kernel's vmcnt accounting assumes (L loads, ST stores per tile)."""
import re, sys
s = open(sys.argv[1]).read()
ks = re.findall(r'^(_ZN3csu12_GLOBAL__N_112gemm4_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E(\w+?)EEv\S*):\s*;', s, re.M)
bad = 0
wre = re.compile(r's_waitcnt vmcnt\((\d+)\)')
for name, bm, bn, S, occ, epi, t in ks:
    body = s[s.index(name + ':'):]
    body = body[:body.index('s_endpgm')]
    bm, bn, epi = int(bm), int(bn), int(epi)
    TMW = bm // 64; WC = bn // 2; CPR = WC // 8; RPS = 64 // CPR; Q = 32 // RPS; OS = 4 if t.startswith('f') else 2
    L = 2 + (2 if epi == 3 else 1 if epi == 2 else 0) * TMW * Q
    ST = TMW * Q * ((2 if OS == 4 else 1) + (1 if epi == 1 else 0))
    nl = len([x for x in re.findall(r'\bbuffer_load_dword[^\n]*', body) if not x.rstrip().endswith('lds')]); ns = len(re.findall(r'\bbuffer_store_dword', body))
    vg = re.search(r'\.vgpr_count:\s+(\d+)', s[s.index(name + ':'):]).group(1)
    waits = sorted(set(int(x) for x in wre.findall(body)))
    ok = nl == L and ns == ST
    bad += not ok
    print(f"{bm}x{bn} S{S} occ{occ} epi{epi} {t[:6]}: loads {nl}/{L} stores {ns}/{ST} vgpr {vg} waits {waits} {'OK' if ok else 'MISMATCH'}")
sys.exit(1 if bad else 0)
