# the prefetching tile (symbols first, each group's entries one group ahead)
# in the 256-lane encoder too
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "if constexpr (ZR_ENC_PF != 0 && EW == 1024 && !(ABL & 2)) {"
assert a in s
s = s.replace(a, "if constexpr (ZR_ENC_PF != 0 && EW >= 256 && !(ABL & 2)) {")
open(p, "w").write(s)
