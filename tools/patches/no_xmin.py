# timing only: the 256-lane encoder's tile loop without the not-in-table check
# (the two v_min3 per four steps); not a correct encoder for foreign tables
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
old = """            const uint4 e3 = ent(s3), e2 = ent(s2), e1 = ent(s1), e0 = ent(s0);
            xmin = min(min(xmin, e3.x), e2.x);  // two v_min3 per group
            xmin = min(min(xmin, e1.x), e0.x);
"""
assert old in s
s = s.replace(old, """            const uint4 e3 = ent(s3), e2 = ent(s2), e1 = ent(s1), e0 = ent(s0);
""", 1)
open(p, "w").write(s)
