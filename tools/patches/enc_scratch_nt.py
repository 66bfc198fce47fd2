# the encoder's 16-B scratch bursts non-temporal
import sys
p = sys.argv[1] + "/zipora_amd/csrc/zr_rans.hip"
s = open(p).read()
a = """                    *reinterpret_cast<v4u *>(reinterpret_cast<uint8_t *>(q0) + k * qstride) =
                        v4u{fd[4 * k], fd[4 * k + 1], fd[4 * k + 2], fd[4 * k + 3]};"""
assert a in s
s = s.replace(a, """                    __builtin_nontemporal_store(v4u{fd[4 * k], fd[4 * k + 1], fd[4 * k + 2], fd[4 * k + 3]},
                        reinterpret_cast<v4u *>(reinterpret_cast<uint8_t *>(q0) + k * qstride));""")
open(p, "w").write(s)
