# the 256-lane encoder with 3 copies of the encode table (lane l reads copy l % 3)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_TC256 3\n" + s
open(p, "w").write(s)
