"""The oracle (oracle/amr_oracle.c) against the reference's own outputs.

The golden fixtures were produced by running the reference itself
(tests/golden/make_golden.py); this pins the oracle before it is trusted as
the checker of the GPU path.  CPU only."""
import numpy as np
import pytest

from oracle import oracle
from _util import call_case, call_sweep_case, expected, outcome


class _OracleModem:
    qpsk_demodulate = staticmethod(oracle.qpsk_demodulate)
    bpsk_demodulate = staticmethod(oracle.bpsk_demodulate)
    fsk_demodulate = staticmethod(oracle.fsk_demodulate)

    @staticmethod
    def psk8_demodulate(s, b=1200, c=3000.0, s_r=96000):
        return oracle.qpsk_demodulate(s, b, c, s_r)

    @staticmethod
    def ofdm_demodulate_simple(s, baud, carrier, nsc, samp_rate=96000):
        return oracle.qpsk_demodulate(s, baud, carrier, samp_rate)

    @staticmethod
    def fsk_high_speed_demodulate(s, baud=19200, s_r=96000):
        return oracle.fsk_demodulate(s, baud, 8000, 16000, s_r)


def test_oracle_matches_every_golden_demod_case(golden):
    manifest, inputs = golden
    bad = []
    for case in manifest["cases"]:
        got = outcome(lambda: call_case(_OracleModem, case, inputs[case["id"]]))
        if got != expected(case):
            bad.append(case["id"])
    assert not bad, f"oracle differs from the reference on {bad}"


def test_oracle_fec_matches_reference(golden):
    manifest, _ = golden
    for f in manifest["fec"]:
        data = bytes.fromhex(f["in"])
        out, ok = oracle.fec_decode(data)
        assert out.hex() == f["out"]
        if len(data) >= 4:
            assert ok == (not f["crc_warn"])


def test_oracle_intermediates_bitwise():
    """filtfilt restatement == scipy bit for bit, symbols == the reference pipeline."""
    import os
    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "intermediates.npz"))
    bp = oracle.filtfilt(d["bp_b"], d["bp_a"], d["x"])
    assert np.array_equal(bp.view(np.uint64), d["bp"].view(np.uint64))
    out = oracle.qpsk_demodulate(d["x"], baud=9600)
    assert out == d["out"].tobytes()


def test_oracle_batch_equals_single():
    rng = np.random.default_rng(3)
    x = rng.normal(0, 0.3, (5, 3000)).astype(np.float32)
    batch, sync = oracle.psk_demod_batch("qpsk", x, 2400, n_threads=2)
    for i in range(5):
        assert batch[i] == oracle.qpsk_demodulate(x[i], baud=2400)


def test_crc32_matches_zlib():
    import zlib
    rng = np.random.default_rng(0)
    for n in (0, 1, 7, 100, 4097):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert oracle.crc32(d) == (zlib.crc32(d) & 0xFFFFFFFF)


@pytest.mark.parametrize("n", [28, 29, 101, 1000])
def test_oracle_filtfilt_vs_scipy_random(n):
    from scipy import signal
    rng = np.random.default_rng(n)
    b, a = signal.butter(4, [0.05, 0.4], btype="band")
    for dt in (np.float32, np.float64):
        x = rng.normal(0, 1, n).astype(dt)
        ref = signal.filtfilt(b, a, x)
        got = oracle.filtfilt(b, a, x)
        assert np.array_equal(ref.view(np.uint64), got.view(np.uint64))


def test_oracle_matches_reference_sweep(sweep_golden):
    """The oracle against the reference's own outputs on a seeded draw of 72
    configurations (PSK and FSK; baud 300-19200, carriers / tones, 96 / 48 /
    44.1 kHz, 28-24 000 samples, f32 / f64 / int16, levels down to 1 %,
    leading silence, noise) and 12 FSK streams between stretches of exact
    digital silence, where only pocketfft's own rounding decides
    (tests/golden/make_sweep_golden.py): bytes or exception text equal,
    every case."""
    manifest, inputs = sweep_golden
    bad = [c["id"] for c in manifest["cases"]
           if outcome(lambda: call_sweep_case(oracle, c, inputs[c["id"]])) != expected(c)]
    assert not bad, f"oracle differs from the reference on {bad}"


def test_oracle_matches_reference_rawint(rawint_golden):
    """Raw integer (int8 / uint8 / int16 / uint16 / int32 / int64), bool and
    float16 captures: the reference hands the caller's array to filtfilt as
    it is (modem.py:77, 198, 308), so its odd extension wraps / rounds in the
    array's dtype -- the oracle's AMR_DT_RAW_* restate that arithmetic in C
    (amr_oracle.c odd_pair).  Bytes equal the reference's on all 24 fixtures
    (tests/golden/make_rawint_golden.py), 13 of them cases where the wrap
    decides the bytes (the reference's float64 bytes differ)."""
    manifest, inputs = rawint_golden
    assert sum(c["differs_from_float64"] for c in manifest["cases"]) >= 10
    bad = []
    for c in manifest["cases"]:
        x, p = inputs[c["id"]], c["params"]
        if c["fn"] == "fsk":
            got = outcome(lambda: oracle.fsk_demodulate(x, p["baud"], p["f0"], p["f1"], p["samp_rate"], raw_int16=True))
        else:
            f = oracle.qpsk_demodulate if c["fn"] == "qpsk" else oracle.bpsk_demodulate
            got = outcome(lambda: f(x, p["baud"], p["f0"], p["samp_rate"], raw_int16=True))
        if got != expected(c):
            bad.append((c["id"], c["fn"], c["dtype"]))
    assert not bad, f"oracle differs from the reference on {bad}"


def test_oracle_raw_filtfilt_is_scipys():
    """oracle.filtfilt on raw arrays of every integer width, bool and
    float16 == scipy.signal.filtfilt on the same array, bit for bit
    (full-scale values: the odd extension wraps / overflows)."""
    from scipy import signal
    rng = np.random.default_rng(5)
    b, a = signal.butter(4, [0.05, 0.2], btype="band")
    bad = []
    for dt in (np.int8, np.uint8, np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64, np.bool_, np.float16):
        for t in range(40):
            n = int(rng.integers(28, 300))
            if dt == np.bool_:
                x = rng.integers(0, 2, n).astype(bool)
            elif dt == np.float16:
                x = (rng.standard_normal(n) * float(rng.choice([1e-6, 1.0, 3e4, 6e4]))).astype(np.float16)
            else:
                info = np.iinfo(dt)
                x = rng.integers(int(info.min), int(info.max), n, dtype=dt, endpoint=True)
            with np.errstate(all="ignore"):
                want = signal.filtfilt(b, a, x)
            got = oracle.filtfilt(b, a, x, raw_int16=True)
            if not np.array_equal(np.nan_to_num(got).view(np.uint64), np.nan_to_num(want).view(np.uint64)):
                bad.append((np.dtype(dt).name, t))
    assert not bad, bad


def test_drop_in_raw_edges_are_the_oracles(rawint_golden):
    """The product's host half of a raw capture (_amr.raw_input: numpy's own
    odd extension in the caller's dtype, the samples' exact float copy) ==
    the oracle's C restatement of the extension (oracle_odd_edges) and of the
    samples' float64 cast, on every fixture and a random draw of each dtype."""
    import _amr
    manifest, inputs = rawint_golden
    rng = np.random.default_rng(6)
    arrays = [inputs[c["id"]] for c in manifest["cases"]]
    for dt in (np.int8, np.uint8, np.int16, np.uint16, np.int32, np.uint32, np.int64, np.uint64):
        info = np.iinfo(dt)
        arrays.append(rng.integers(int(info.min), int(info.max), 500, dtype=dt, endpoint=True))
    with np.errstate(over="ignore"):
        arrays.append((rng.standard_normal(500) * 5e4).astype(np.float16))
    arrays.append(rng.integers(0, 2, 500).astype(bool))
    arrays.append(rng.integers(-30000, 30000, 500).astype(">i2"))      # non-native byte order
    for pad in (21, 27):
        for x in arrays:
            xk, edges = _amr.raw_input(x[None, :], pad)
            assert xk.dtype in (np.float32, np.float64) and xk.shape == (1, x.size)
            assert np.array_equal(xk[0].astype(np.float64), x.astype(np.float64)), x.dtype
            want = oracle.odd_edges(x, pad)
            assert np.array_equal(np.nan_to_num(edges[0]), np.nan_to_num(want)), (x.dtype, pad)


def _host_numpy_is_modelled():
    """The restatement models numpy's complex multiply (FMA) and complex abs
    (AVX-512 hypot form) as the fixtures' host runs them; on a host whose
    numpy dispatches differently the live-scipy comparisons are skipped
    (the reference fixtures still pin the oracle)."""
    if not oracle.numpy_complex_is_modelled():
        pytest.skip("this host's numpy complex multiply / abs differ from the modelled AVX-512 kernels")


def test_oracle_pocketfft_every_length():
    """amr_pocketfft.c's scipy.fft.rfft / irfft / fft / ifft and
    |scipy.signal.hilbert| equal scipy + numpy bit for bit on EVERY length
    1..2000: FFTPACK-style plans of every radix (2, 3, 4, 5, 7, 8, 11 and the
    generic pass) and the Bluestein plans pocketfft picks (488 real / 748
    complex lengths in that range)."""
    import scipy.fft as sf
    from scipy import signal
    _host_numpy_is_modelled()
    rng = np.random.default_rng(11)
    bad = []
    for n in range(1, 2001):
        x = rng.standard_normal(n)
        if not np.array_equal(oracle.rfft(x).view(np.float64), sf.rfft(x).view(np.float64)):
            bad.append(("rfft", n))
        X = sf.rfft(rng.standard_normal(n))
        if not np.array_equal(oracle.irfft(X, n), sf.irfft(X, n)):
            bad.append(("irfft", n))
        c = rng.standard_normal(n) + 1j * rng.standard_normal(n)
        if not np.array_equal(oracle.cfft(c).view(np.float64), sf.fft(c).view(np.float64)):
            bad.append(("fft", n))
        if not np.array_equal(oracle.cfft(c, True).view(np.float64), sf.ifft(c).view(np.float64)):
            bad.append(("ifft", n))
        if not np.array_equal(oracle.hilbert_env(x), np.abs(signal.hilbert(x))):
            bad.append(("hilbert", n))
    assert not bad, bad[:20]
    assert sum(oracle.pf_uses_bluestein(n, True) for n in range(1, 2001)) == 488
    assert sum(oracle.pf_uses_bluestein(n, False) for n in range(1, 2001)) == 748


def test_oracle_hilbert_is_scipys():
    """The oracle's |scipy.signal.hilbert(x)| equals scipy + numpy bit for bit
    on the FSK lengths -- 5-smooth four-step ones, Bluestein ones (24001,
    30011, 96001, 400001) and a generic-radix one (77880 = 59 * 1320) -- for
    noise, for signal between exact-zero stretches, next to a stretch 1e-17
    below the signal and next to a constant (DC) stretch (where the envelopes
    are rounding noise -- DESIGN.md §2 item 6)."""
    from scipy import signal
    _host_numpy_is_modelled()
    rng = np.random.default_rng(7)
    sizes = [960, 1920, 9600, 19200, 24001, 30011, 48000, 77880, 96000, 96001, 153600, 400001]
    bad = []
    for n in sizes:
        for kind in ("noise", "silence", "tiny", "dc"):
            x = rng.normal(size=n)
            if kind == "silence":
                x[: n // 3] = 0.0
                x[2 * n // 3:] = 0.0
            elif kind == "tiny":
                x[n // 4: n // 2] *= 1e-17
            elif kind == "dc":
                x[n // 2:] = -0.25
            if not np.array_equal(oracle.hilbert_env(x), np.abs(signal.hilbert(x))):
                bad.append((n, kind))
    assert not bad, bad


def test_oracle_resample_is_scipys():
    """oracle.resample == scipy.signal.resample bit for bit on the lengths
    decode_wav_file produces (decoder.py:385-387: 44.1 / 48 / 22.05 / 8 kHz
    captures to 96 kHz; 441000 = 2^3 3^2 5^3 7^2 runs the generic radix-7
    pass) and on down-sampling, odd and Bluestein lengths."""
    from scipy import signal
    _host_numpy_is_modelled()
    rng = np.random.default_rng(5)
    cases = [(441000, 960000), (480000, 960000), (44100, 96000), (48000, 96000), (22050, 96000),
             (8000, 96000), (100000, 96000), (77, 1000), (1000, 77), (24001, 52247), (1009, 2003)]
    bad = [(nx, num) for nx, num in cases
           if not np.array_equal(oracle.resample(x := rng.standard_normal(nx), num), signal.resample(x, num))]
    assert not bad, bad


def test_oracle_wav_pipeline_matches_reference(wav_golden):
    """The reference's decode_wav_file (decoder.py:380-389) on 44.1 / 48 /
    22.05 kHz WAVs, restated with the oracle: the WAV's int16 / 32768 (as
    libsndfile reads it), oracle.resample (pocketfft's rfft / irfft), the
    oracle demod, the host frame parse and decompression -- the saved files
    equal the reference's (tests/golden/make_wav_golden.py), or none where
    the reference saved none."""
    import contextlib
    import io
    import wave

    import compression
    import decoder
    manifest, wavs = wav_golden
    for case in manifest["cases"]:
        with wave.open(io.BytesIO(wavs[case["id"]].tobytes()), "rb") as w:
            sr = w.getframerate()
            data = np.frombuffer(w.readframes(w.getnframes()), np.int16).astype(np.float64) / 32768.0
        y = oracle.resample(data, int(round(len(data) * 96000.0 / sr)))
        if case["mode"] == "BPSK":
            raw = oracle.bpsk_demodulate(y, baud=case["symbol_rate"])
        else:
            raw = oracle.qpsk_demodulate(y, baud=case["symbol_rate"])
        with contextlib.redirect_stdout(io.StringIO()):
            frames = decoder.parse_fbp_stream_enhanced(raw)
        got = [{"name": f["name"], "data": compression.intelligent_decompress(f["data"]).hex()} for f in frames]
        assert got == case["files"], case["id"]
