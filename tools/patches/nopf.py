# A/B variant: no software-pipelined encoder tile (ZR_ENC_PF = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_ENC_PF 1", "#define ZR_ENC_PF 0")
open(p, "w").write(s)
