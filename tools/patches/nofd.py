# A/B variant: the scratch stores of a flush right after its ring reads (ZR_ENC_FD = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_ENC_FD 1", "#define ZR_ENC_FD 0")
open(p, "w").write(s)
