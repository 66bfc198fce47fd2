# the compaction's output stores with the default cache policy
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "__builtin_nontemporal_store(*reinterpret_cast<const v4u *>(img + 16 * u), reinterpret_cast<v4u *>(dst));"
assert a in s
s = s.replace(a, "*reinterpret_cast<v4u *>(dst) = *reinterpret_cast<const v4u *>(img + 16 * u);")
open(p, "w").write(s)
