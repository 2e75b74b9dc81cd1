"""Developer probe: static instruction mix of the substep loop per phase, from the
disassembly of a GM_ISA_MARKERS build (an s_nop 15 / s_nop k pair marks every PH(k)).
usage: python tools/isa_phase_mix.py <substep_loop disassembly .s>"""
import re, sys
L=open(sys.argv[1]).read().split('\n')
names={0:'kin',1:'crb',2:'mass',5:'coll',6:'newton',8:'integ',9:'update',10:'monitor',15:'k:A',16:'k:B',17:'crb:ch',3:'n:QF',4:'n:scans',7:'n:H',11:'n:setup',12:'n:warm',13:'n:jar/ls',14:'n:factor',24:'n:solve',22:'body'}
cur='start'; cnt={}; segs=[]
def cat(op,l):
    if re.match(r'v_(fma|fmac|mul|add)_f64',op) or op in('v_rcp_f64_e32','v_rsq_f64_e32','v_sqrt_f64_e32'): return 'f64'
    if '_dpp' in l: return 'dpp'
    if op.startswith('v_readlane') or op.startswith('v_writelane'): return 'lane'
    if op.startswith('v_mov'): return 'mov'
    if op.startswith('v_cndmask'): return 'cnd'
    if op.startswith('v_'): return 'v'
    if op.startswith('ds_'): return 'ds'
    if op=='s_waitcnt': return 'wait'
    if op.startswith('s_cbranch'): return 'br'
    if op.startswith('s_load'): return 'smem'
    if op.startswith('global_') or op.startswith('scratch_'): return 'vmem'
    return 's'
i=0
while i < len(L):
    l=L[i]; m=re.match(r'\s+([a-z_0-9]+)(.*)',l)
    if m and m.group(1)=='s_nop' and m.group(2).strip().startswith('15'):
        m2=re.match(r'\s+s_nop (\d+)',L[i+1]); k=int(m2.group(1))
        segs.append((cur,dict(cnt))); cnt={}; cur='after PH(%d) %s'%(k,names.get(k,'?')); i+=2; continue
    if m:
        c=cat(m.group(1),l); cnt[c]=cnt.get(c,0)+1
    i+=1
segs.append((cur,cnt))
for n,c in segs:
    t=sum(c.values())
    print(f"{n:24s} {t:6d} "+" ".join(f"{k}:{v}" for k,v in sorted(c.items())))
