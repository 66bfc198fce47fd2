# the compaction's scratch loads non-temporal (the scratch is dead once read)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "v[k] = *reinterpret_cast<const v4u *>((nv[k] && !(ABL & 4)) ? src : sbase + (lane % CS) * 16);"
assert a in s
s = s.replace(a, "v[k] = __builtin_nontemporal_load(reinterpret_cast<const v4u *>((nv[k] && !(ABL & 4)) ? src : sbase + (lane % CS) * 16));")
open(p, "w").write(s)
