# A/B variant: V2 step with start' added after the mad (ZR_ENC_YS = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_ENC_YS 1", "#define ZR_ENC_YS 0")
open(p, "w").write(s)
