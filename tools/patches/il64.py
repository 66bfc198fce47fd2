# the 64-stream scratch interleave (rounds 2-5) instead of 16
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_IL_SPAN 64\n" + s
open(p, "w").write(s)
