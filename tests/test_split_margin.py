"""The time-split PSK layout's error premise, on the CPU.

psk_split_kernels.hip cuts each filtfilt pass of qpsk_demodulate /
bpsk_demodulate (modem.py:189-266 / 68-135) into chunks started w samples
early from a zero state, so its symbol samples differ from the reference's
(serial) ones by the zero start's decayed transient and by a different
rounding trajectory.  Its decisions are kept only where a margin of
E = kappa * peak|x| cannot move them (the rest go to the serial kernels), so
bytes are exact provided every symbol error stays below E.  kappa and the
warm-ups come from libamr.so's own design (amr_psk_split_design, host
arithmetic); the chunked passes are the oracle's restatement
(oracle.psk_split_symbols -- tests/test_gpu_split.py checks the device
computes exactly it), the reference symbols the oracle's scipy restatement
(pinned to the reference by tests/test_oracle_golden.py).

Bar: max |split - serial| / peak|x| <= kappa / 16 over tones (carrier,
band edges), square waves, noise, DC offsets, modulated signals and silence
gaps, at 9 filter sets (QPSK / BPSK, 300-19200 Bd, 44.1 / 48 / 96 kHz) and
three chunk lengths.  The measured ratio kappa / error is printed per set
(kappa is 64x the L1 noise gain; the worst measured is ~1.4x that gain)."""
import numpy as np
import pytest

CONFIGS = [("qpsk", 9600, 3000.0, 96000.0), ("qpsk", 19200, 3000.0, 96000.0), ("qpsk", 1200, 3000.0, 96000.0),
           ("qpsk", 300, 3000.0, 96000.0), ("qpsk", 1000, 3000.0, 48000.0), ("qpsk", 4800, 12000.0, 96000.0),
           ("qpsk", 2400, 1800.0, 44100.0), ("bpsk", 1200, 3000.0, 96000.0), ("bpsk", 9600, 6000.0, 96000.0)]


def _inputs(kind, baud, fc, fs, n, rng):
    import synth
    t = np.arange(n) / fs
    nyq = fs / 2
    lo, hi = max(0.01 * nyq, fc - 1.5 * baud), min(0.99 * nyq, fc + 1.5 * baud)
    sq = np.sign(np.sin(2 * np.pi * fc * t))
    gap = np.sin(2 * np.pi * fc * t + np.cumsum(rng.normal(0, 0.05, n)))
    gap[n // 3:n // 2] = 0.0
    ins = {"noise": rng.normal(0, 0.3, n), "tone_c": np.sin(2 * np.pi * fc * t), "tone_lo": np.sin(2 * np.pi * lo * t),
           "tone_hi": np.sin(2 * np.pi * hi * t), "square": sq, "noise_dc": rng.normal(0.5, 0.1, n), "gap": gap}
    if fs / baud >= 10:
        fr = synth.random_frame(rng, 200)
        w = synth.qpsk_waveform(fr, baud, fc, fs) if kind == "qpsk" else synth.bpsk_waveform(fr, baud, fc, fs)
        x = np.zeros(n)
        x[:min(n, w.size)] = w[:n]
        ins["signal"] = x + rng.normal(0, 0.05, n)
    return ins


@pytest.mark.parametrize("kind,baud,fc,fs", CONFIGS, ids=lambda v: str(v))
def test_split_error_far_below_kappa(kind, baud, fc, fs, built_lib):
    import _amr
    from oracle import oracle
    n = 48000 if baud >= 1200 else 96000
    d = _amr.split_design(kind, n, baud, fc, fs)
    assert d is not None and d["kappa"] > 0 and 0 < d["warmup_bp"] <= n // 4
    rng = np.random.default_rng(baud + int(fc))
    worst, where = 0.0, None
    for name, x in _inputs(kind, baud, fc, fs, n, rng).items():
        ref = oracle.psk_symbols(kind, x, baud, fc, fs)
        peak = np.abs(x).max()
        for L in (64, 97, 5000):
            sp = oracle.psk_split_symbols(kind, x, baud, fc, fs, L, d["warmup_bp"], d["warmup_lp"])
            err = np.abs(sp - ref).max() / peak
            if err > worst:
                worst, where = err, (name, L)
    print(f"{kind}@{baud} fc {fc:g} fs {fs:g}: kappa {d['kappa']:.3e}, worst |split - serial| / peak {worst:.3e} "
          f"({where}), kappa / worst = {d['kappa'] / worst:.1f}")
    assert worst <= d["kappa"] / 16


def test_split_design_refuses_what_it_cannot_bound(built_lib):
    """Streams too short for the warm-ups (w > n / 4) get no split layout."""
    import _amr
    assert _amr.split_design("qpsk", 1000, 9600) is None
    assert _amr.split_design("qpsk", 96000, 9600) is not None


def test_split_restatement_with_unbounded_warmup_is_the_reference(built_lib):
    """A chunk whose warm-up reaches back to the pass's start runs the serial
    recursion itself: with w >= the stream the split restatement IS the
    reference's symbol sequence, bit for bit (the chunking bookkeeping adds
    nothing of its own)."""
    import synth
    from oracle import oracle
    x = synth.qpsk_batch(1, 20000, 9600, seed=4, distinct=1, noise=0.1)[0]
    ref = oracle.psk_symbols("qpsk", x, 9600)
    sp = oracle.psk_split_symbols("qpsk", x, 9600, 3000.0, 96000.0, 97, 10 ** 6, 10 ** 6)
    assert np.array_equal(sp, ref)


F32F_CONFIGS = [("qpsk", 9600, 3000.0, 96000.0), ("qpsk", 19200, 3000.0, 96000.0), ("qpsk", 1200, 3000.0, 96000.0),
                ("qpsk", 300, 3000.0, 96000.0), ("bpsk", 1200, 3000.0, 96000.0), ("qpsk", 2400, 1800.0, 44100.0)]


@pytest.mark.parametrize("kind,baud,fc,fs", F32F_CONFIGS, ids=lambda v: str(v))
def test_f32_handoff_error_below_its_bound(kind, baud, fc, fs, built_lib):
    """The lane layout's float32 hand-off: the exact
    band-pass output rounded to float32 before the low-pass moves the symbols
    by at most f32_margin * max|f| (libamr.so's amr_psk_f32_margin: the
    rounding through the low-pass's L1 gain -- a bound, not a fit).  Measured
    on the same inputs as the time-split test; the ratio is printed."""
    import _amr
    from oracle import oracle
    n = 48000
    c = _amr.f32_margin(kind, n, baud, fc, fs)
    assert c > 0
    rng = np.random.default_rng(baud + 7)
    worst = 0.0
    for name, x in _inputs(kind, baud, fc, fs, n, rng).items():
        ref = oracle.psk_symbols(kind, x, baud, fc, fs)
        got, fpeak = oracle.psk_symbols_f32f(kind, x, baud, fc, fs)
        worst = max(worst, np.abs(got - ref).max() / (c * fpeak + 2.0 ** -120))
    print(f"{kind}@{baud} fc {fc:g}: f32 margin {c:.3e} x max|f|; worst error / bound {worst:.3f}")
    assert worst <= 0.5
