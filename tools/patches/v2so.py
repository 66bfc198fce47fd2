# A/B variant: the V2 step with the round-3 accumulator output (V2O = false)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "    constexpr bool V2O = V2;"
assert s.count(a) == 1
s = s.replace(a, "    constexpr bool V2O = false;")
open(p, "w").write(s)
