"""Host logic around the kernels (CPU): filter design parity with the oracle,
LO table semantics, framing, frame parsing, decompression, decoder dispatch."""
import binascii
import contextlib
import io
import os

import numpy as np
import pytest


def test_design_matches_oracle_plan():
    import _amr
    from oracle import oracle
    for kind, baud in (("qpsk", 9600), ("qpsk", 19200), ("bpsk", 1200), ("qpsk", 1000)):
        sps, first, bp, lp, lo4 = _amr.design_psk(kind, 5000, baud)
        op = oracle.PskPlan(kind, 5000, baud)
        assert (sps, first) == (op.sps, op.first)
        for got, want in zip(bp + lp, op.bp + op.lp):
            assert np.array_equal(got, want)
        assert np.array_equal(lo4[:, :2].ravel(), op.lo)


def test_lo_table_addends_are_numpys():
    """(f + 0j) * lo == fma(f, lo_re, c2), fma(f, lo_im, c3) incl. signed zeros."""
    import _amr
    lo4 = _amr.lo_table(257, 3000.0, 96000)
    lo = lo4[:, 0] + 1j * lo4[:, 1]
    f = np.random.default_rng(1).normal(size=257)
    f[::5] = 0.0
    f[1::7] = -0.0
    prod = f * lo
    from fractions import Fraction as F

    def fma(x, y, z):
        r = F(x) * F(y) + F(z)
        if r == 0:
            return -0.0 if (np.signbit(x * y) and np.signbit(z)) else 0.0
        return float(r)
    for i in range(257):
        assert np.float64(fma(f[i], lo4[i, 0], lo4[i, 2])).view(np.uint64) == prod.real[i].view(np.uint64)
        assert np.float64(fma(f[i], lo4[i, 1], lo4[i, 3])).view(np.uint64) == prod.imag[i].view(np.uint64)


def test_frame_and_parse_roundtrip():
    import decoder
    import synth
    payload = b"RAW" + b"\x00hello" * 20
    fr = synth.frame_data("a.txt", payload, 0, 1, 100, 7)
    raw = b"\x13\x37" + fr + b"junk" + fr
    with contextlib.redirect_stdout(io.StringIO()):
        got = decoder.parse_fbp_stream_enhanced(raw)
    assert [g["name"] for g in got] == ["a.txt", "a.txt"]
    assert got[0]["data"] == payload and got[0]["final_crc"] == 7
    bad = bytearray(fr)
    bad[-1] ^= 1
    with contextlib.redirect_stdout(io.StringIO()):
        assert decoder.parse_fbp_stream_enhanced(bytes(bad)) == []


def test_decompress_tags_and_raw_off_by_one():
    import lzma
    import zlib
    import compression
    data = bytes(range(256)) * 3
    assert compression.intelligent_decompress(b"ZLIB" + zlib.compress(data)) == data
    assert compression.intelligent_decompress(b"LZMA" + lzma.compress(data)) == data
    d = compression.delta_compress(data)
    assert compression.delta_decompress(d) == data
    assert compression.intelligent_decompress(b"DLZM" + lzma.compress(d)) == data
    assert compression.intelligent_decompress(b"RAW" + data) == data[1:]   # reference off-by-one
    assert compression.intelligent_decompress(b"zz") == b"zz"


def test_delta_matches_reference_loop():
    import compression
    rng = np.random.default_rng(0)
    data = rng.integers(0, 256, 999, dtype=np.uint8).tobytes()
    out = bytearray([data[0]])
    cur = data[0]
    for dlt in data[1:]:
        cur = (cur + dlt) & 0xFF
        out.append(cur)
    assert compression.delta_decompress(data) == bytes(out)


def test_decoder_swallows_errors_like_reference(tmp_path, monkeypatch):
    """Config 1 plumbing: FSK1200 at the reference's default tones raises in
    scipy.butter; decode_from_buffer prints and returns []."""
    import decoder
    monkeypatch.chdir(tmp_path)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        assert decoder.decode_from_buffer(np.zeros(10000), "FSK1200", 1200) == []
    assert "Erro crítico na demodulação: filter critical frequencies must be greater than 0" in buf.getvalue()


@pytest.mark.gpu
def test_decode_wav_file_config1_plumbing(golden, tmp_path, monkeypatch):
    """BASELINE config 1: 10 s 44.1 kHz FSK1200 WAV -> GPU resample -> [] (reference's own result)."""
    import decoder
    manifest, inputs = golden
    case = [d for d in manifest["decoder"] if d["id"] == "dec_FSK1200_44k"][0]
    p = tmp_path / "in.wav"
    p.write_bytes(inputs["dec_FSK1200_44k"].tobytes())
    monkeypatch.chdir(tmp_path)
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf), contextlib.redirect_stderr(io.StringIO()):
        assert decoder.decode_wav_file(str(p), "FSK1200", 1200) == case["saved"] == []
    assert ("Erro crítico" in buf.getvalue()) == case["log_has_error"]


def test_synth_qpsk_matches_reference_modulator_shape():
    import synth
    fr = synth.frame_data("x", b"abc")
    w = synth.qpsk_waveform(fr, 1000)
    assert w.dtype == np.float32 and w.size == (40 + 4 * len(fr)) * 96


def test_fec_encode_matches_golden(golden):
    import fec
    manifest, _ = golden
    rs = fec.ReedSolomonFEC()
    enc = rs.encode(b"hello world!")
    assert enc.hex() in [f["in"] for f in manifest["fec"]]
