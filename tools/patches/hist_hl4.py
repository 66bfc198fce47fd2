# 4 loads per thread per round in the histogram
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "    constexpr uint32_t HL = 8;\n"
assert a in s
s = s.replace(a, "    constexpr uint32_t HL = 4;\n")
open(p, "w").write(s)
