# the histogram's 16-B loads as buffer loads with cache-policy bits AUX (env
# HIST_AUX: 2 nt, 18 nt sc1, 3 sc0 nt, 19 sc0 sc1 nt)
import os, sys
aux = int(os.environ.get("HIST_AUX", "2"))
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = "cur[k] = __builtin_nontemporal_load(q + u + k * T);"
b = "nxt[k] = __builtin_nontemporal_load(q + u + k * T);"
assert a in s and b in s
ld = "__builtin_amdgcn_raw_buffer_load_b128(hr, (uint32_t)((u + k * T) * 16), 0, %d)" % aux
s = s.replace(a, "cur[k] = " + ld + ";").replace(b, "nxt[k] = " + ld + ";")
c = "    if (u + (HL - 1) * T < units) {\n        v4u cur[HL];\n"
assert c in s
s = s.replace(c, "    if (u + (HL - 1) * T < units) {\n        const __amdgpu_buffer_rsrc_t hr = byte_rsrc((void *)q);\n        v4u cur[HL];\n")
open(p, "w").write(s)
