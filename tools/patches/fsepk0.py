# A/B variant: FSE decoder packing symbols with a mask and shift-or each (ZR_FSE_PK = 0)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_fse.hip"
s = open(p).read()
s = s.replace("#define ZR_FSE_PK 1", "#define ZR_FSE_PK 0")
open(p, "w").write(s)
