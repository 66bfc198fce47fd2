"""PA-Zip FSE stage and the DictZipBlobStore entropy stage:
dict_zip/compression_types.rs:2272-2340, dict_zip/blob_store.rs:1075-1224."""
import pytest


def _streams(zr):
    z = zr.synth("z", 100000, seed=21)
    return [b"", b"x", b"short record", z[:31], z[:32], z[:5000], zr.synth("u", 4000, seed=2), z]


def test_oracle_pazip_framing(zr, oracle):
    cfg = oracle.pazip_fse_config()
    z = zr.synth("z", 5000, seed=1)
    assert oracle.pazip_apply(b"", cfg) == b""
    assert oracle.pazip_apply(z[:31], cfg) == b"UN" + z[:31]
    fs = oracle.pazip_apply(z, cfg)
    assert fs[:2] == b"\xfeS" and len(fs) < len(z) + 2
    u = zr.synth("u", 4000, seed=2)
    assert oracle.pazip_apply(u, cfg) == b"UN" + u  # incompressible: kept raw
    for s in (fs, b"UN" + u, b"q"):
        assert oracle.pazip_remove(s, cfg) == (z if s is fs else (u if s[:2] == b"UN" else s))


@pytest.mark.gpu
def test_pazip_fse_parity(zr, oracle):
    for table_log, level in ((12, 3), (11, 6), (9, 1)):
        cfg = zr.PaZipFseConfig(table_log=table_log, compression_level=level)
        ocfg = oracle.pazip_fse_config(table_log, level)
        for d in _streams(zr):
            got = zr.apply_fse_compression(d, cfg)
            assert got == oracle.pazip_apply(d, ocfg), (len(d), table_log)
            assert zr.remove_fse_compression(got, cfg) == d
        # old format (no magic) and pass-through
        raw_fse = oracle.fse_compress(_streams(zr)[5], oracle.pazip_fse_config(table_log, level))
        assert zr.remove_fse_compression(raw_fse, cfg) == _streams(zr)[5]
        assert zr.remove_fse_compression(b"q", cfg) == b"q"
    with pytest.raises(zr.ZiporaError):
        zr.apply_fse_compression(_streams(zr)[5], zr.PaZipFseConfig(table_log=4))
    assert zr.apply_fse_compression(b"tiny", zr.PaZipFseConfig(table_log=4)) == b"UNtiny"  # < 32: no validation


@pytest.mark.gpu
def test_dictzip_entropy_stage(zr, oracle):
    dictionary = zr.synth("t", 50000, seed=4)
    records = [dictionary[1000:3000], zr.synth("z", 20000, seed=5), b"", b"ab", zr.synth("u", 3000, seed=6)]
    octx = oracle.Ctx(dictionary, 1)
    for algo in (0, 1, 2):
        for inter in (0, 1, 2, 4, 8):
            for ratio in (0.8, 1.0, 2.0):
                st = zr.DictZipEntropyStage(algo, inter, dictionary, ratio)
                for r in records:
                    enc, used = st.encode(r)
                    oenc, oused = oracle.dictzip_encode(algo, inter, octx, ratio, r)
                    assert (enc, int(used)) == (oenc, oused), (algo, inter, ratio, len(r))
                    try:
                        want = oracle.dictzip_decode(oused, octx, oenc, len(r))
                    except oracle.OracleError:
                        want = None
                    try:
                        got = st.decode(enc, used, len(r))
                    except zr.ZiporaError:
                        got = None
                    assert got == want, (algo, inter, ratio, len(r))
    with pytest.raises(zr.ZiporaError):
        zr.DictZipEntropyStage(1, 3, dictionary).encode(b"abc")
