# the decoder's packed output stores non-temporal (aux = 2: nt on gfx950)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "__builtin_amdgcn_raw_buffer_store_b32(q, orsrc, voff_pk, (ABL & 256) ? 0 : row - 2 * N, 0);"
assert s.count(a) == 1
s = s.replace(a, a[:-3] + "2);")
open(p, "w").write(s)
