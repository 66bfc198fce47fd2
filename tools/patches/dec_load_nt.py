# the decoder's 64-B refill loads (asm) non-temporal
import sys, re
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
n0 = s.count('asm volatile("global_load_dwordx4 %0, %1, off')
s = s.replace('asm volatile("global_load_dwordx4 %0, %1, off" :', 'asm volatile("global_load_dwordx4 %0, %1, off nt" :')
s = s.replace('asm volatile("global_load_dwordx4 %0, %1, off offset:%2" :', 'asm volatile("global_load_dwordx4 %0, %1, off offset:%2 nt" :')
for o in (16, 32, 48):
    s = s.replace('asm volatile("global_load_dwordx4 %%0, %%1, off offset:%d" :' % o, 'asm volatile("global_load_dwordx4 %%0, %%1, off offset:%d nt" :' % o)
assert s.count(' nt"') == n0, (n0, s.count(' nt"'))
open(p, "w").write(s)
