# A/B variant: record decoder with its round-3 16-step tiles (ZR_X1_T32 = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_X1_T32 1", "#define ZR_X1_T32 0")
open(p, "w").write(s)
