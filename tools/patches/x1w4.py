# A/B variant: record decoder with 4-byte mirrored slot entries (ZR_X1_W8 = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_X1_W8 1", "#define ZR_X1_W8 0")
open(p, "w").write(s)
