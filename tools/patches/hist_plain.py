# the histogram's 16-B loads with the default cache policy (not non-temporal)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "cur[k] = __builtin_nontemporal_load(q + u + k * T);"
b = "nxt[k] = __builtin_nontemporal_load(q + u + k * T);"
assert a in s and b in s
s = s.replace(a, "cur[k] = q[u + k * T];").replace(b, "nxt[k] = q[u + k * T];")
open(p, "w").write(s)
