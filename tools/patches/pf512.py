# the prefetching tile in the 512-lane encoder
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_PF512 1\n" + s
open(p, "w").write(s)
