# A/B variant: the round-3 encoder step and output (ZR_ENC_V2 = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_ENC_V2 1", "#define ZR_ENC_V2 0")
open(p, "w").write(s)
