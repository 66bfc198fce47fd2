# A/B variant: record encoder loads both 64-B halves of each input line together (ZR_X1PAIR = 1)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("#define ZR_X1PAIR 0", "#define ZR_X1PAIR 1")
open(p, "w").write(s)
