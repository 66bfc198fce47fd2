# A/B variant: the host pipeline with two device slots (ZR_PIPE_SLOTS = 2)
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_pipe.cpp"
s = open(p).read()
s = s.replace("#define ZR_PIPE_SLOTS 3", "#define ZR_PIPE_SLOTS 2")
open(p, "w").write(s)
