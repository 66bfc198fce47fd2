# A/B variant: the 256-lane encoder everywhere (ZR_ENC_1024 = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_ENC_1024 1", "#define ZR_ENC_1024 0")
open(p, "w").write(s)
