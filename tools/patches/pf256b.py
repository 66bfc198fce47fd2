# A/B variant: the group-ahead table prefetch (tile_fast_pf) at 256 lanes too
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "if constexpr (ZR_ENC_PF != 0 && EW == 1024 && !(ABL & 2))"
assert s.count(a) == 1
s = s.replace(a, "if constexpr (ZR_ENC_PF != 0 && EW >= 256 && !(ABL & 2))")
open(p, "w").write(s)
