# the wide decoder's output as byte stores (no 4-lane transpose)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "#define ZR_DEC_PK 1  // full waves"
assert a in s
s = s.replace(a, "#define ZR_DEC_PK 0  // full waves")
open(p, "w").write(s)
