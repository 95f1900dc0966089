"""GPU parity of the FSK path (modem.py:298-341) and its FFT/Hilbert core.

Bars (stated here):
  * decoded bytes and sync index: bit-exact against the reference's golden
    outputs and against the oracle (its C restatement of filtfilt and of
    pocketfft, pinned against scipy) at every length, digital silence
    included (the exact path);
  * FFT / Hilbert intermediates: the GPU's fp64 FFT is not pocketfft, so its
    rounding differs -- max |err| <= 1e-12 * max |X| (1e-11 for Bluestein
    lengths) against numpy.fft, and envelopes within 1e-9 relative of the
    reference's |hilbert(filtfilt(.))| (the tolerance north_star names for
    intermediate magnitudes).
"""
import os

import numpy as np
import pytest

from _util import call_case, expected, outcome

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


@pytest.mark.parametrize("n,batch", [(96000, 3), (51840, 2), (24001, 2), (1000, 5), (7, 4), (390625, 1), (150001, 1),
                                     (97, 3),
                                     (960000, 2),      # past the two-pass limit: six-step
                                     (400001, 1)])     # Bluestein with a six-step convolution length
def test_fft_matches_numpy(n, batch):
    import _amr
    rng = np.random.default_rng(n)
    x = rng.normal(size=(batch, n)) + 1j * rng.normal(size=(batch, n))
    for inverse, ref in ((False, np.fft.fft), (True, np.fft.ifft)):
        got = _amr.fft(x, inverse=inverse)
        want = ref(x, axis=1)
        err = np.abs(got - want).max() / np.abs(want).max()
        tol = 1e-12 if n in (96000, 51840, 1000, 390625) else 1e-11
        assert err <= tol, (n, inverse, err)


@pytest.mark.parametrize("n", [96000, 24001, 51840, 22, 500000, 400001])
def test_hilbert_matches_scipy(n):
    import _amr
    from scipy import signal
    rng = np.random.default_rng(n + 1)
    x = rng.normal(size=(3, n))
    got = _amr.hilbert(x)
    want = signal.hilbert(x, axis=1)
    assert np.abs(got - want).max() <= 1e-11 * np.abs(want).max()


def test_every_golden_fsk_case(golden):
    """Bytes (or the ValueError) of every FSK case the reference produced."""
    import modem
    manifest, inputs = golden
    cases = [c for c in manifest["cases"] if c["fn"].startswith("fsk")]
    assert len(cases) >= 6
    bad = []
    for case in cases:
        got = outcome(lambda: call_case(modem, case, inputs[case["id"]]))
        if got != expected(case):
            bad.append((case["id"], got[:2]))
    assert not bad, f"GPU differs from the reference on {bad}"


def test_fsk_bluestein_length_uses_bluestein(golden):
    import _fsk
    _, inputs = golden
    x = inputs["fsk9600_f32_1"]
    pl = _fsk.FskPlan(x.size, 9600, 12000.0, 24000.0, max_streams=1)
    assert pl.fft_length != x.size and pl.fft_length >= 2 * x.size - 1


@pytest.mark.parametrize("case_id", ["fsk9600_f32_0", "fsk9600_f32_1", "fsk1200_f32"])
def test_fsk_envelopes_within_tolerance(golden, case_id):
    import _fsk
    from oracle import oracle
    from scipy import signal
    manifest, inputs = golden
    case = [c for c in manifest["cases"] if c["id"] == case_id][0]
    p = case["params"]
    x = inputs[case_id]
    pl = _fsk.FskPlan(x.size, p["baud"], p["mark_freq"], p["space_freq"], max_streams=1)
    m, s = pl.envelopes(x[None, :])
    nyq = 48000.0
    for got, f in ((m[0], p["mark_freq"]), (s[0], p["space_freq"])):
        b, a = signal.butter(3, [(f - p["baud"]) / nyq, (f + p["baud"]) / nyq], btype="band")
        want = np.abs(signal.hilbert(oracle.filtfilt(b, a, x)))
        assert np.abs(got - want).max() <= 1e-9 * np.abs(want).max()


@pytest.mark.parametrize("B,N,baud,mark,space,dtype", [
    (64, 96000, 9600, 12000.0, 24000.0, np.float32),
    (33, 48000, 1200, 2400.0, 4800.0, np.float64),
    (20, 30011, 4800, 8000.0, 16000.0, np.float32),     # Bluestein length
    (17, 9600, 19200, 21000.0, 27000.0, np.float32),    # sps 5: windows of 2
    (70, 96000, 9600, 12000.0, 24000.0, np.float64),    # live columns, float64 staged in chunks
    (40, 96000, 4800, 8000.0, 16000.0, np.float32),     # sps 20: 150 live columns (a partial tile)
    (24, 96000, 19200, 21000.0, 27000.0, np.int16),     # sps 5, PCM input
])
def test_fsk_batch_vs_oracle(B, N, baud, mark, space, dtype):
    import _fsk
    import synth
    from oracle import oracle
    x = synth.fsk_batch(B, N, baud, mark, space, seed=B, distinct=4, noise=0.3).astype(dtype)
    pl = _fsk.FskPlan(N, baud, mark, space, max_streams=B)
    got, _ = pl.demod_host(x)
    want = [oracle.fsk_demodulate(x[i], baud, mark, space) for i in range(B)]
    mism = [i for i in range(B) if got[i] != want[i]]
    assert not mism, f"{len(mism)} streams differ, first {mism[:5]}"


def test_fsk_int16_pcm_equals_float64():
    import _fsk
    import synth
    x = synth.fsk_batch(8, 24000, 9600, seed=3, distinct=2, noise=0.1)
    q = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16)
    pl = _fsk.FskPlan(24000, 9600, 12000.0, 24000.0, max_streams=8)
    a, _ = pl.demod_host(q)
    b, _ = pl.demod_host(q.astype(np.float64) / 32768.0)
    assert a == b


def test_fsk_full_batch_round_trip():
    """BASELINE config 3 size (B=16384, N=96000 float32), through size-independent
    properties: (1) the batch is 2048 noisy streams repeated 8 times, and every
    copy must decode identically (streams are independent of their batch
    position); (2) every one of the 2048 distinct streams matches the oracle
    bit for bit -- with (1), all 16384 are oracle-checked;
    (3) clean frames decode to their framed payload (FSK with tones above the
    baud round-trips exactly)."""
    import _fsk
    import synth
    from oracle import oracle
    B, N, U = 16384, 96000, 2048
    base = synth.fsk_batch(U, N, 9600, 12000.0, 24000.0, seed=9, distinct=16, noise=0.05)
    x = np.tile(base, (B // U, 1))
    pl = _fsk.get_fsk_plan(N, 9600, 12000.0, 24000.0, 96000, B)
    assert pl.live_columns
    assert pl.scratch_bytes() <= 56e9, pl.scratch_bytes()     # 2 x n complex per stream (z, C, the dead tiles) + split F1 buffers
    got, sync = pl.demod_host(x)
    bad = [i for i in range(U, B) if got[i] != got[i % U]]
    assert not bad, f"{len(bad)} repeated streams decode differently, first {bad[:5]}"
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        want = list(ex.map(lambda r: oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0), base))
    bad = [i for i in range(U) if got[i] != want[i]]
    assert not bad, f"{len(bad)} of {U} streams differ from the oracle, first {bad[:5]}"
    rng = np.random.default_rng(9)
    spb = 10
    payload = max(1, (N // spb) // 8 - 4 - 40)
    frames = [synth.random_frame(rng, payload) for _ in range(16)]
    clean = synth.fsk_batch(16, N, 9600, 12000.0, 24000.0, seed=9, distinct=16, noise=0.0)
    cg, _ = pl.demod_host(clean)
    for j in range(16):
        m = min(len(frames[j]), 1100)           # the last bytes may fall off the 1-s window
        assert cg[j][:m] == frames[j][:m]


def test_fsk_batch_past_2g_samples():
    """22 400 one-second FSK9600 streams in one plan: 2.15e9 samples, past
    2^31, through the live-column path (F1's z offsets, the FFT passes' per
    stream bases, the compare bits and words must all be 64-bit).  The batch
    cycles through 61 distinct noisy captures (prime: a stream that read
    another stream's rows would decode a different frame); every stream ==
    the oracle's bytes for its capture."""
    import _fsk
    import synth
    from oracle import oracle
    B, N, U = 22400, 96000, 61
    assert B * N > 2 ** 31
    base = synth.fsk_batch(U, N, 9600, 12000.0, 24000.0, seed=61, distinct=U, noise=0.3)
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        want = list(ex.map(lambda r: oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0), base))
    x = base[np.arange(B) % U]
    pl = _fsk.FskPlan(N, 9600, 12000.0, 24000.0, max_streams=B)
    assert pl.live_columns
    got, _ = pl.demod_host(x)
    del pl
    bad = [i for i in range(B) if got[i] != want[i % U]]
    assert not bad, f"{len(bad)} streams differ, first {bad[:5]}"


@pytest.mark.parametrize("n,baud,mark,space", [(77880, 2400, 11229.28, 29833.37), (96000, 9600, 12000.0, 24000.0),
                                                (24001, 1200, 2400.0, 4800.0), (30000, 300, 1200.0, 2200.0),
                                                (96001, 9600, 12000.0, 24000.0),     # Bluestein over a six-step M
                                                (960000, 9600, 12000.0, 24000.0),    # six-step: a 10-s WAV
                                                (1920000, 1200, 2400.0, 4800.0),     # six-step, 20 s
                                                (400001, 4800, 8000.0, 16000.0),     # Bluestein over six-step
                                                (441000, 2400, 7000.0, 19000.0)])    # 44.1 kHz x 10 s: 2^3 3^2 5^3 7^2
def test_envelope_error_is_far_below_the_margin(n, baud, mark, space):
    """F2 flags a stream for the exact path when some compare has
    |env_mark - env_space| <= 2 tau peak|x| (the plan's tau: max(2^-36 =
    kAmbTau, a standard FFT rounding bound, fsk_api.cpp fsk_fft_bound)); unflagged compares are then bit-exact only if the fast path's
    envelopes are within tau peak|x| of the reference's.  F1 computes scipy's
    filtfilt bit for bit, so the difference is the FFTs' rounding alone --
    two-pass (96000, 30000), Bluestein over a two-pass M (24001, 77880),
    six-step (960000, 1920000: more rounding stages) and
    Bluestein over a six-step M (96001, 400001, 441000).  Measure it (GPU
    natural-layout envelopes vs the reference's |hilbert(filtfilt(.))|, the
    oracle's restatement) on noise, signal, digital silence and quiet
    stretches: it must stay below tau / 100.  The ratio per length is printed."""
    import _fsk
    import synth
    from oracle import oracle
    from scipy import signal
    rng = np.random.default_rng(n + baud)
    rows = []
    for i in range(4):
        w = synth.fsk_waveform(synth.random_frame(rng, 40), baud, mark, space, 96000.0)
        row = np.zeros(n)
        off = (0, 5000, n // 3, 100)[i]
        seg = w[:max(0, n - off)]
        row[off:off + seg.size] = seg
        if i == 3:
            row += rng.normal(0, 0.3, n)
            row[n // 2:n // 2 + 3000] *= 1e-9
        rows.append(row)
    x = np.stack(rows)
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=len(rows))
    gm, gs = pl.envelopes(x)
    nyq = 48000.0
    worst = 0.0
    for i, xi in enumerate(x):
        def env(f):
            b, a = signal.butter(3, [(f - baud) / nyq, (f + baud) / nyq], btype="band")
            return oracle.hilbert_env(oracle.filtfilt(b, a, xi))
        peak = np.abs(xi).max()
        worst = max(worst, np.abs(gm[i] - env(mark)).max() / peak, np.abs(gs[i] - env(space)).max() / peak)
    tau = 2.0 ** -36
    # the plan's own scale: max(2^-36, the standard FFT bound, fsk_api.cpp
    # fsk_fft_bound; tests/test_fsk_fft_bound.py)
    tp = pl.margin()["tau"]
    assert tp >= tau and abs(tp - _fsk.fft_margin(n, baud, mark, space)["tau"]) <= 1e-15 * tp
    print(f"n={n}: max |env_gpu - env_ref| / peak|x| = {worst:.3e} (2^-36 = {tau:.3e}, ratio {tau / worst:.0f}; "
          f"the plan's tau {tp:.3e}, ratio {tp / worst:.0f}; exact streams {pl.exact_streams()} of {len(rows)})")
    assert worst < tau / 100


def _silence_batch(rng, B, n, baud, mark, space, dtype):
    import synth
    rows = []
    for i in range(B):
        w = synth.fsk_waveform(synth.random_frame(rng, int(rng.integers(4, 30))), baud, mark, space, 96000.0)
        off = (0, 150, int(rng.integers(0, n // 3)), int(rng.integers(80, 300)))[i % 4]   # short silences too
        row = np.zeros(n)
        seg = w[:max(0, n - off)]
        row[off:off + seg.size] = seg
        if i % 5 == 4:
            row[off + seg.size // 2:off + seg.size // 2 + 700] = 0.0     # a gap inside the frame
        rows.append(row)
    x = np.stack(rows)
    return np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dtype == np.int16 else x.astype(dtype)


@pytest.mark.parametrize("n,baud,mark,space,dtype", [
    (30000, 2400, 11229.28, 29833.37, np.float64),
    (24000, 4800, 7000.0, 19000.0, np.float32),
    (19200, 9600, 12000.0, 24000.0, np.int16),
    (96000, 9600, 12000.0, 24000.0, np.float32),     # live columns
    (96000, 1200, 2400.0, 4800.0, np.float64),
    (77880, 2400, 11229.28, 29833.37, np.float64),   # 59 * 1320: generic radix
    (24001, 4800, 7000.0, 19000.0, np.float32),      # Bluestein
    (30011, 1200, 2400.0, 4800.0, np.int16),         # Bluestein
    (96001, 9600, 12000.0, 24000.0, np.float64),     # Bluestein, six-step fast path
    (960000, 9600, 12000.0, 24000.0, np.int16),      # a 10-s WAV's length: six-step
    (960000, 1200, 2400.0, 4800.0, np.float32),
    (400001, 4800, 7000.0, 19000.0, np.float32),     # Bluestein over a six-step M
    (441000, 2400, 7000.0, 19000.0, np.float64),
])
def test_fsk_digital_silence_exact(n, baud, mark, space, dtype):
    """Digital silence next to signal, at 5-smooth, generic-radix and
    Bluestein lengths: F2 flags the stream (its envelopes there are rounding
    noise) and the exact path (fsk_exact_kernels.hip) recomputes its compare
    bits in scipy's and pocketfft's own operation order -- bytes and sync
    equal to the oracle's (whose pocketfft restatement is pinned against
    scipy, tests/test_oracle_golden.py) on every stream, silent or not."""
    import _fsk
    from oracle import oracle
    rng = np.random.default_rng(n + baud)
    B = 12 if n < 200000 else 6
    x = _silence_batch(rng, B, n, baud, mark, space, dtype)
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    got, _ = pl.demod_host(x)
    flagged = pl.exact_streams()
    want = [oracle.fsk_demodulate(x[i], baud, mark, space) for i in range(B)]
    mism = [i for i in range(B) if got[i] != want[i]]
    assert not mism, f"{len(mism)} of {B} streams differ, first {mism[:5]}"
    print(f"n={n}: {flagged} of {B} streams flagged for the exact path")


@pytest.mark.parametrize("kind", ["dc", "tiny", "zero"])
@pytest.mark.parametrize("n", [30000, 77880, 24001, 960000, 400001])
def test_fsk_quiet_stretches_exact(kind, n):
    """Stretches where both envelopes sink to rounding level without being
    exact zeros: a constant (DC) offset -- butter(3, band)'s
    b = k [1, 0, -3, 0, 3, 0, -1] cancels constants, ramps and parabolas --
    a stretch 1e-17 below the signal, and all-zero streams (never flagged:
    both paths' envelopes are exact zeros).  Bytes == the oracle's.  (Whether
    a quiet stretch puts a compare inside the margin depends on the Hilbert
    transform's 1/t tails of the neighbouring signal, so only the all-zero
    case's flag count is asserted.)"""
    import _fsk
    import synth
    from oracle import oracle
    rng = np.random.default_rng(n + len(kind))
    baud, mark, space = 2400, 7000.0, 19000.0
    B = 6 if n < 200000 else 3
    rows = []
    q = n // 3                      # a quiet lead-in long enough for the band-pass tails to die out
    for i in range(B):
        w = synth.fsk_waveform(synth.random_frame(rng, 30), baud, mark, space, 96000.0)
        row = np.zeros(n)
        seg = w[: n - q]
        row[q:q + seg.size] = seg
        if kind == "dc":
            row[:q] = (-2.0 if i % 2 else 0.37) / 32768
            row[q + seg.size // 2:q + seg.size // 2 + 2000] = 0.125
        elif kind == "tiny":
            row[:q] = rng.normal(0, 1e-17, q)
        else:
            row[:] = 0.0
        rows.append(row)
    x = np.stack(rows)
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    got, _ = pl.demod_host(x)
    want = [oracle.fsk_demodulate(r, baud, mark, space) for r in x]
    assert got == want
    if kind == "zero":
        assert pl.exact_streams() == 0
    print(f"n={n} {kind}: {pl.exact_streams()} of {B} flagged")


def test_fsk_device_entry_lean_plan():
    """A live-layout plan that only ran the device entry holds z and C, not
    the buffer that keeps z through F2 (dd: 9.6 B per sample at FSK9600) --
    its flagged streams re-run F1 from the caller's x (E1) instead.  The
    first host entry allocates dd (it is also that entry's staging) and every
    later call keeps z.  Bytes == the oracle's in both modes, on a batch with
    digital silence (flagged streams)."""
    import _fsk
    from oracle import oracle
    from _util import fsk_device_demod
    n, baud, mark, space, B = 96000, 9600, 12000.0, 24000.0, 8
    x = _silence_batch(np.random.default_rng(7), B, n, baud, mark, space, np.float32)
    want = [oracle.fsk_demodulate(r, baud, mark, space) for r in x]
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    pl.set_layout("serial")                          # the serial F1 (a split call never keeps z)
    assert pl.live_columns
    total = pl.scratch_bytes()
    lean = pl.resident_bytes()
    # counted, allocated by the first split call: the forward outputs, peaks,
    # FS0's start states (chunks >= 128) and tables (w <= n / 4), and the
    # strict margin's per-tone scratch, maxima and tables
    m1 = n + 42
    strict_row = 5 * (-(-m1 // 16)) + 2 * (m1 // 128 + 2)
    split_reserved = (min(B, 1024) * (2 * m1 * 8 + 8 + 96 * (m1 // 128 + 2) + 2 * (strict_row * 8 + 64)) +
                      2 * (2 * (n // 4) + 1) * 48 + 2 * (2 * (n // 4) + 1 + 4 * (2 * (n // 4) // 16 + 64) + 64) * 8)
    dd = B * n * 6 // 10 * 16            # the dead columns' transform: nd / n1 = 6 / 10 at sps 10
    assert total - lean >= dd, (total, lean, dd)
    got, _ = fsk_device_demod(pl, x)
    assert pl.exact_streams() > 0
    assert got == want
    assert pl.resident_bytes() == lean               # the device entry allocated nothing
    got_h, _ = pl.demod_host(x)
    assert got_h == want and pl.exact_streams() > 0
    assert pl.resident_bytes() + split_reserved == total == pl.scratch_bytes()
    got2, _ = fsk_device_demod(pl, x)               # now keeping z
    assert got2 == want
    print(f"plan bytes: device entry only {lean / 1e6:.1f} MB, after a host entry {total / 1e6:.1f} MB")


def test_fsk_every_stream_exact_on_golden(golden):
    """The exact path alone (exact mode 2: every stream recomputed) on every
    golden FSK case through a plan: bytes == the reference's -- the exact
    path is the reference's arithmetic, not just a fix-up of silence."""
    import _fsk
    manifest, inputs = golden
    cases = [c for c in manifest["cases"] if c["fn"] == "fsk_demodulate" and c["status"] == "ok"]
    assert cases
    for c in cases:
        x = np.asarray(inputs[c["id"]])
        a = c["params"]
        baud, mark, space, fs = a.get("baud", 1200), a.get("mark_freq", 1200.0), a.get("space_freq", 2200.0), a.get("samp_rate", 96000)
        pl = _fsk.FskPlan(x.size, baud, mark, space, fs, max_streams=1)
        pl.set_exact_mode(2)
        got, _ = pl.demod_host(x[None])
        assert pl.exact_streams() == 1
        assert got[0] == bytes.fromhex(c["out"]), c["id"]


@pytest.mark.parametrize("n", [20000, 96000])   # 96000 at sps 10: the live-column layout
def test_fsk_timing_hooks(n):
    import _fsk
    import synth
    x = synth.fsk_batch(32, n, 9600, seed=1, distinct=2)
    pl = _fsk.FskPlan(n, 9600, 12000.0, 24000.0, max_streams=32)
    assert pl.live_columns == (n == 96000)
    pl.enable_timing(True)
    pl.demod_host(x)
    t = pl.timings()
    assert set(t) == {"bandpass", "hilbert", "decide", "launch", "exact"} and all(v > 0 for v in t.values())
    assert t["launch"] >= t["hilbert"] + t["exact"]


@pytest.mark.parametrize("nx,num,batch", [(1000, 2177, 2), (2177, 1000, 2), (999, 1500, 1), (1500, 999, 1),
                                          (1001, 1001, 1), (4410, 9600, 3), (48000, 96000, 1),
                                          (441000, 960000, 1)])   # decode_wav_file: 10 s at 44.1 kHz
def test_resample_matches_scipy(nx, num, batch):
    """_amr.resample == scipy.signal.resample (decoder.py:385-387), bit for bit:
    up / down, even / odd lengths (the Nyquist-bin rule), Bluestein lengths."""
    import _amr
    from scipy import signal
    rng = np.random.default_rng(nx + num)
    x = rng.normal(size=(batch, nx))
    got = _amr.resample(x, num)
    want = signal.resample(x, num, axis=1)
    assert np.array_equal(got, want), np.abs(got - want).max()
    assert np.array_equal(_amr.resample(x[0], num), got[0])


def test_fsk_long_stream_vs_oracle():
    """A 10-s stream (960 000 samples: six-step FFT) and a 4.2-s stream of a
    non-5-smooth length (Bluestein over a six-step length): decisions == oracle."""
    import _fsk
    import synth
    from oracle import oracle
    for N in (960000, 400001):
        x = synth.fsk_batch(2, N, 9600, 12000.0, 24000.0, seed=N, distinct=2, noise=0.3)
        pl = _fsk.FskPlan(N, 9600, 12000.0, 24000.0, max_streams=2)
        got, _ = pl.demod_host(x)
        want = [oracle.fsk_demodulate(x[i], 9600, 12000.0, 24000.0) for i in range(2)]
        assert got == want, N


def test_fsk_20s_stream_vs_oracle():
    """A 20-s FSK1200 capture (1 920 000 samples; tones 2400/4800 Hz round-trip,
    SURVEY §4): its compare bits (~240 KB) exceed the decide kernel's LDS
    staging, so the decisions are read from global memory -- still == oracle."""
    import _fsk
    import synth
    from oracle import oracle
    N = 1_920_000
    x = synth.fsk_batch(1, N, 1200, 2400.0, 4800.0, seed=20, distinct=1, noise=0.3)
    pl = _fsk.FskPlan(N, 1200, 2400.0, 4800.0, max_streams=1)
    got, _ = pl.demod_host(x)
    assert got[0] == oracle.fsk_demodulate(x[0], 1200, 2400.0, 4800.0)
    assert len(got[0]) > 1000


@pytest.mark.parametrize("N,baud,live", [(96000, 9600, True), (96000, 19200, True), (96000, 4800, True),
                                         (96000, 1200, False), (30011, 4800, False), (48000, 1200, False)])
def test_fsk_live_column_layout_chosen(N, baud, live):
    """The live-column layout runs when the four-step grid's
    row length n1 is a multiple of sps (96000 = 300 x 320: sps 5, 10, 20),
    else the natural layout (sps 80 at 96000 / 48000, Bluestein lengths)."""
    import _fsk
    mark, space = {9600: (12000.0, 24000.0), 19200: (21000.0, 27000.0), 4800: (8000.0, 16000.0)}.get(baud, (2400.0, 4800.0))
    pl = _fsk.FskPlan(N, baud, mark, space, max_streams=4)
    assert pl.live_columns == live


def test_fsk_natural_layout_forced(tmp_path):
    """AMR_FSK_LIVE=0 (the natural layout: every sample through all three
    Hilbert passes) on the live-column cases: == oracle, and == the live path."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    script = tmp_path / "nat.py"
    script.write_text(f'''
import sys
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import numpy as np
import _fsk, synth
from oracle import oracle
bad = []
for (B, N, baud, m, s) in ((40, 96000, 9600, 12000.0, 24000.0), (9, 96000, 19200, 21000.0, 27000.0)):
    x = synth.fsk_batch(B, N, baud, m, s, seed=B, distinct=4, noise=0.3)
    pl = _fsk.FskPlan(N, baud, m, s, max_streams=B)
    assert not pl.live_columns
    got, _ = pl.demod_host(x)
    bad += [(N, baud, i) for i in range(B) if got[i] != oracle.fsk_demodulate(x[i], baud, m, s)]
print("BAD", bad)
sys.exit(1 if bad else 0)
''')
    env = dict(os.environ, AMR_FSK_LIVE="0")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_fsk_live_async_host_entry():
    """amr_fsk_demod_host_async on a live-column plan: the input is staged on
    the plan's stream (into dd, the buffer that keeps z through F2, allocated
    by this first host entry) while nothing waits on the host; == the
    synchronous entry == oracle."""
    import _amr
    import _fsk
    import synth
    from oracle import oracle
    B, N = 64, 96000
    x = synth.fsk_batch(B, N, 9600, 12000.0, 24000.0, seed=5, distinct=6, noise=0.3).astype(np.float64)
    pl = _fsk.FskPlan(N, 9600, 12000.0, 24000.0, max_streams=B)
    assert pl.live_columns
    o = np.zeros((B, pl.out_cap), np.uint8)
    ln = np.zeros(B, np.int64)
    sy = np.zeros(B, np.int64)
    L = _amr.lib()
    _amr.check(L.amr_fsk_demod_host_async(pl.handle, _amr.ptr(x), _amr.DTYPE_F64, B, N, _amr.ptr(o), pl.out_cap,
                                          _amr.ptr(ln), _amr.ptr(sy)))
    _amr.check(L.amr_fsk_plan_synchronize(pl.handle))
    got = [o[i, :ln[i]].tobytes() for i in range(B)]
    assert got == pl.demod_host(x)[0]
    assert got == [oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0) for r in x]


@pytest.mark.parametrize("env", [{"AMR_FFT_MID_TWG": "0"}, {"AMR_FFT_PRUNE": "0"}, {"AMR_FSK_W1S": "0"},
                                 {"AMR_FSK_BP1": "1"}, {"AMR_FFT_MID_NT": "256"}, {"AMR_FSK_DECIDE_BITS": "0"},
                                 {"AMR_FSK_SPLIT": "1"}, {"AMR_FSK_TILE": "40"}, {"AMR_FSK_TILE": "64"},
                                 {"AMR_FSK_KEEPZ": "0"}, {"AMR_FSK_SPLIT": "1", "AMR_FSK_SPLIT_CONV": "0"}],
                         ids=lambda e: ",".join(f"{k}={v}" for k, v in e.items()))
def test_fsk_live_kernel_variants(tmp_path, env):
    """Every kernel variant of the live-column path, forced through its switch
    (DESIGN.md §3b): middle pass with the W_L table in LDS / with every output
    of the last stage computed, F1 storing z from wave 0 / the one-wave F1:
    float32, float64 and int16 batches == the oracle, bit for bit."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    script = tmp_path / "var.py"
    script.write_text(f'''
import sys
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import numpy as np
import _fsk, synth
from oracle import oracle
bad = []
for (B, N, baud, m, s, dt) in ((40, 96000, 9600, 12000.0, 24000.0, np.float32), (9, 96000, 19200, 21000.0, 27000.0, np.float64),
                               (33, 96000, 4800, 8000.0, 16000.0, np.int16)):
    x = synth.fsk_batch(B, N, baud, m, s, seed=B + 1, distinct=5, noise=0.3)
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dt == np.int16 else x.astype(dt)
    pl = _fsk.FskPlan(N, baud, m, s, max_streams=B)
    assert pl.live_columns
    got, _ = pl.demod_host(x)
    bad += [(N, baud, i) for i in range(B) if got[i] != oracle.fsk_demodulate(x[i], baud, m, s)]
print("BAD", bad)
sys.exit(1 if bad else 0)
''')
    # these batches are small enough for the time-split F1;
    # the serial F1's variants are what this test is for, so it is forced
    # (AMR_FSK_SPLIT=0) unless the variant is about the split itself
    run_env = dict(os.environ, AMR_FSK_SPLIT="0")
    run_env.update(env)
    r = subprocess.run([sys.executable, str(script)], env=run_env, capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
