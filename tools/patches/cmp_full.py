# the 16-stream, 256-lane compaction (rounds 2-5) instead of 8-stream, 128-lane
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_CMP_HALF 0\n" + s
open(p, "w").write(s)
