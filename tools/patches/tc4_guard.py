# 4 table copies and the encoder ring's guard row (41 KiB: 3 workgroups per CU)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_GUARD 1\n" + s
open(p, "w").write(s)
