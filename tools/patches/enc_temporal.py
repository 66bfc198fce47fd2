# k_enc_xn's input pieces with the default cache policy
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "pend = __builtin_nontemporal_load((gcv4u *)(rowb + loff));"
assert a in s
s = s.replace(a, "pend = *(gcv4u *)(rowb + loff);")
open(p, "w").write(s)
