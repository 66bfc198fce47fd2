# A/B variant: the 1024-lane encoder by default
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
s = s.replace("static std::atomic<uint32_t> g_enc_width{256};", "static std::atomic<uint32_t> g_enc_width{1024};")
open(p, "w").write(s)
