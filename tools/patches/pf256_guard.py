# pf256 plus 3 table copies and the guard row
import sys
exec(open(sys.argv[0].replace("pf256_guard.py", "pf256.py")).read())
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = "#define ZR_ENC_TC256 3\n#define ZR_ENC_GUARD 1\n" + s
open(p, "w").write(s)
