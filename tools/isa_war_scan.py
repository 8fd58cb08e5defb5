"""ISA scan for the gjr solve: every buffer load / store whose
SGPR soffset is rewritten before a vmcnt(0) wait, with the distance in
instructions.  Usage: hipcc --save-temps ... ba.hip; python tools/isa_war_scan.py
ba-hip-amdgcn-amd-amdhsa-gfx950.s.  Round 5 finding: the
soffset-store build rewrites the stores' soffset by v_readfirstlane 1-5
instructions after the record's last dwordx4 store; the shipped build has no
store with an SGPR soffset."""
import re, sys
path = sys.argv[1]
lines = open(path).read().split('\n')
starts = [i for i,l in enumerate(lines) if re.match(r'^_ZN3sfm3gjr11k_gjr_solve.*:', l)]
def dst_regs(tok):
    m = re.match(r's\[(\d+):(\d+)\]', tok)
    if m: return set(f"s{k}" for k in range(int(m.group(1)), int(m.group(2))+1))
    return {tok}
for s in starts:
    name = lines[s].split(':')[0]
    i = s; res = []
    while not lines[i].startswith('.Lfunc_end'):
        l = lines[i].split(';')[0].strip()
        toks = re.split(r'[\s,]+', l)
        if toks[0].startswith('buffer_') and len(toks) > 4 and re.match(r's\d+$', toks[4]):
            sreg = toks[4]; n = 0
            for j in range(i+1, min(i+200, len(lines))):
                lj = lines[j].split(';')[0].strip()
                if not lj or lj.startswith('.') or lj.endswith(':'): continue
                tj = re.split(r'[\s,]+', lj)
                n += 1
                if tj[0].startswith('s_waitcnt') and 'vmcnt(0)' in lj: break
                if tj[0].startswith('s_cbranch') or tj[0].startswith('s_branch'): break
                if len(tj) > 1 and not tj[0].startswith('buffer_') and not tj[0].startswith('s_waitcnt') and sreg in dst_regs(tj[1]) and not tj[0].startswith('s_cmp'):
                    res.append((n, i, l, lj)); break
        i += 1
    from collections import Counter
    c = Counter(min(r[0], 20) for r in res)
    print(name, "vmem with sgpr soffset rewritten before vmcnt(0):", len(res), sorted(c.items()))
    for r in sorted(res)[:4]: print("   ", r)
