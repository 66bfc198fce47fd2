# A/B variant: the software-pipelined tile in the 256-lane encoder too
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("if constexpr (ZR_ENC_PF != 0 && EW == 1024 && !(ABL & 2)) {", "if constexpr (ZR_ENC_PF != 0 && !(ABL & 2)) {")
open(p, "w").write(s)
