# the 256-lane encoder with N copies of the encode table (lane l reads copy l % N)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_TC256 4\n" + s
open(p, "w").write(s)
