# Store cache-policy variants for same-box A/B (argv[2]: which, argv[3]: the policy text, e.g. "sc1" or "nt sc1")
#   cmp: k_enc_compact_lds's 16-B output stores; enc: k_enc_xn's scratch bursts; dec: k_dec_xn_fast's packed stores
import sys
root, which, pol = sys.argv[1], sys.argv[2], sys.argv[3]
p = root + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
if which == "cmp":
    a = "__builtin_nontemporal_store(*reinterpret_cast<const v4u *>(img + 16 * u), reinterpret_cast<v4u *>(dst));"
    assert s.count(a) == 1
    s = s.replace(a, '{ const v4u x_ = *reinterpret_cast<const v4u *>(img + 16 * u); '
                     'asm volatile("global_store_dwordx4 %0, %1, off ' + pol + '\\n\\ts_nop 1" :: "v"(dst), "v"(x_) : "memory"); }')
elif which == "enc":
    a = """                    *reinterpret_cast<v4u *>(reinterpret_cast<uint8_t *>(q0) + k * qstride) =
                        v4u{fd[4 * k], fd[4 * k + 1], fd[4 * k + 2], fd[4 * k + 3]};"""
    assert s.count(a) == 1
    s = s.replace(a, """                    { const v4u x_ = v4u{fd[4 * k], fd[4 * k + 1], fd[4 * k + 2], fd[4 * k + 3]};
                      uint8_t *d_ = reinterpret_cast<uint8_t *>(q0) + k * qstride;
                      asm volatile("global_store_dwordx4 %0, %1, off """ + pol + """\\n\\ts_nop 1" :: "v"(d_), "v"(x_) : "memory"); }""")
elif which == "dec":
    a = "__builtin_amdgcn_raw_buffer_store_b32(q, orsrc, voff_pk, (ABL & 256) ? 0 : row - 2 * N, 0);"
    assert s.count(a) == 1
    aux = {"sc1": 16, "nt sc1": 18, "nt": 2, "sc0": 1}[pol]
    s = s.replace(a, a[:-3] + "%d);" % aux)
open(p, "w").write(s)
