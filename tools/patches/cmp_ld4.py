# four 16-B loads per lane per round in the interleaved compaction (rounds 2-5)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_CMP_LD 4\n" + s
open(p, "w").write(s)
