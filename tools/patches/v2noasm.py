# A/B variant: the V2 update in plain C (compiler-scheduled) instead of the mad + SDWA add asm
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = '''            uint32_t xn;
            asm("v_mad_u32_u24 %0, %1, %2, %3\\n\\t"
                "v_add_u32_sdwa %0, %0, %4 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0"
                : "=&v"(xn)
                : "v"(q), "v"(e.w), "v"(y), "v"(e.y));'''
assert s.count(a) == 1, s.count(a)
s = s.replace(a, "            const uint32_t xn = __umul24(q, e.w) + y + (e.y & 0xFFFFu);")
open(p, "w").write(s)
