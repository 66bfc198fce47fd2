# 16 loads per thread per round in the histogram (32 in flight while counting)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "    constexpr uint32_t HL = 8;\n"
assert a in s
s = s.replace(a, "    constexpr uint32_t HL = 16;\n")
open(p, "w").write(s)
