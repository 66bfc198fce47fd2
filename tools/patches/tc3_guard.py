# 3 table copies and the encoder ring's guard row (ZR_ENC_GUARD)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_TC256 3\n#define ZR_ENC_GUARD 1\n" + s
open(p, "w").write(s)
