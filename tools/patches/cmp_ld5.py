# five 16-B loads per lane per round in the interleaved compaction
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_CMP_LD 5\n" + s
open(p, "w").write(s)
