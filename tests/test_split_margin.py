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
(kappa is 64x the L1 noise gain; the worst measured is ~1.2x that gain)."""
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
    T = _amr.split_state_tables(kind, n, baud, fc, fs)
    rng = np.random.default_rng(baud + int(fc))
    worst, where = 0.0, None
    for name, x in _inputs(kind, baud, fc, fs, n, rng).items():
        ref = oracle.psk_symbols(kind, x, baud, fc, fs)
        peak = np.abs(x).max()
        for L in (64, 97, 5000):
            for tables in (None, T):     # the w1-step warm-ups, KS0's convolution start states
                sp = oracle.psk_split_symbols(kind, x, baud, fc, fs, L, d["warmup_bp"], d["warmup_lp"], tables=tables)
                err = np.abs(sp - ref).max() / peak
                if err > worst:
                    worst, where = err, (name, L, "warm" if tables is None else "conv")
    print(f"{kind}@{baud} fc {fc:g} fs {fs:g}: kappa {d['kappa']:.3e}, worst |split - serial| / peak {worst:.3e} "
          f"({where}), kappa / worst = {d['kappa'] / worst:.1f}")
    assert worst <= d["kappa"] / 16


def test_split_design_refuses_what_it_cannot_bound(built_lib):
    """Streams too short for the warm-ups (w > n / 4) get no split layout."""
    import _amr
    assert _amr.split_design("qpsk", 1000, 9600) is None
    assert _amr.split_design("qpsk", 96000, 9600) is not None


def test_split_restatement_with_one_chunk_is_the_reference(built_lib):
    """One chunk per pass (L past the stream) starts at the pass's first sample
    with scipy's state and has no warm-up, so it runs the serial recursion
    itself: the split restatement IS the reference's symbol sequence, bit for
    bit (the chunking bookkeeping adds nothing of its own; the warm-up steps'
    FMA form, psk_common.h bp_warm, never runs)."""
    import synth
    from oracle import oracle
    x = synth.qpsk_batch(1, 20000, 9600, seed=4, distinct=1, noise=0.1)[0]
    ref = oracle.psk_symbols("qpsk", x, 9600)
    sp = oracle.psk_split_symbols("qpsk", x, 9600, 3000.0, 96000.0, 10 ** 6, 3565, 136)
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


# ---- the FSK time-split F1 (fsk_kernels.hip FS1-FS3) ----------
FSK_CONFIGS = [(9600, 12000.0, 24000.0, 96000), (4800, 7000.0, 19000.0, 96000), (2400, 11229.28, 29833.37, 96000),
               (1200, 2400.0, 4800.0, 96000), (19200, 21000.0, 27000.0, 96000), (1200, 2400.0, 4800.0, 48000)]


def _fsk_inputs(baud, mark, space, fs, n, rng):
    import synth
    t = np.arange(n) / fs
    ins = {"noise": rng.normal(0, 0.3, n), "mark": np.sin(2 * np.pi * mark * t), "space": np.sin(2 * np.pi * space * t),
           "edge": np.sin(2 * np.pi * (mark + baud) * t), "square": np.sign(np.sin(2 * np.pi * mark * t)),
           "noise_dc": rng.normal(0.5, 0.1, n)}
    w = synth.fsk_waveform(synth.random_frame(rng, 40), baud, mark, space, float(fs))
    x = np.zeros(n)
    x[n // 5:n // 5 + min(w.size, n - n // 5)] = w[:n - n // 5]
    x[n // 2:n // 2 + 3000] = 0.0
    ins["signal_gap"] = x + np.where(x != 0, rng.normal(0, 0.02, n), 0.0)
    return ins


@pytest.mark.parametrize("baud,mark,space,fs", FSK_CONFIGS, ids=lambda v: str(v))
def test_fsk_split_error_far_below_kappa(baud, mark, space, fs, built_lib):
    """The split F1's band-pass output against scipy's filtfilt (the oracle's
    restatements of both): max |split - serial| / peak|x| <= kappa / 16 over
    tones at mark / space / a band edge, a square wave, noise, DC and an FSK
    frame with a silence gap, three chunk lengths.  The envelope error that
    implies is kappa * ||hilbert kernel||_1 (the margin F2 adds); measured
    here too, through the oracle's exact |hilbert|.  Both chunk starts: the
    warm-ups and FS0's convolution states."""
    import _amr
    import _fsk
    from oracle import oracle
    n = 48000
    d = _fsk.split_design(n, baud, mark, space, fs)
    assert d is not None and 0 < d["warmup"] <= n // 4 and d["kappa"] > 0
    _, ((mb, ma, mzi), (sb, sa, szi)) = _fsk.design_fsk(n, baud, mark, space, fs)
    rng = np.random.default_rng(baud + int(mark))
    worst, where, worst_env = 0.0, None, 0.0
    for name, x in _fsk_inputs(baud, mark, space, fs, n, rng).items():
        peak = np.abs(x).max()
        for b, a, zi in ((mb, ma, mzi), (sb, sa, szi)):
            ref = oracle.filtfilt(b, a, x)
            T = _amr.state_tables(b, a, zi, d["warmup"])
            for L in (64, 97, 5000):
                for tables in (None, T):     # w-step warm-ups, FS0's convolution start states
                    sp = oracle.split_filtfilt(b, a, x, L, d["warmup"], tables=tables)
                    err = np.abs(sp - ref).max() / peak
                    if err > worst:
                        worst, where = err, (name, L, "warm" if tables is None else "conv")
                if L == 97 and name in ("signal_gap", "noise"):
                    de = np.abs(oracle.hilbert_env(sp) - oracle.hilbert_env(ref)).max() / peak
                    worst_env = max(worst_env, de)
    env_bound = d["kappa"] * d["hilbert_l1"]
    print(f"fsk@{baud} {mark:g}/{space:g} fs {fs}: warm-up {d['warmup']}, kappa {d['kappa']:.3e}, worst |split - "
          f"serial| / peak {worst:.3e} ({where}), kappa / worst = {d['kappa'] / worst:.1f}; envelope bound "
          f"{env_bound:.3e}, worst {worst_env:.3e}")
    assert worst <= d["kappa"] / 16
    assert worst_env <= env_bound / 16


def test_fsk_split_refused_for_narrow_bands(built_lib):
    """300 Bd at 96 kHz (a 600 Hz band): the rounding noise gain makes the
    margin wider than 2^-16 of the peak, so those plans keep the serial F1."""
    import _fsk
    assert _fsk.split_design(96000, 300, 1200.0, 2200.0, 96000) is None
    assert _fsk.split_design(96000, 9600, 12000.0, 24000.0, 96000) is not None


@pytest.mark.parametrize("n", [2400, 2401, 24001, 96000, 96001])
def test_fsk_split_hilbert_gain(n, built_lib):
    """The design's ||ifft(h)||_1 (scipy.signal.hilbert's kernel, iir_design.h
    hilbert_l1) equals sum |hilbert(unit impulse)| and is not below it, at
    even and odd lengths."""
    import _fsk
    from scipy.signal import hilbert
    d = _fsk.split_design(n, 9600, 12000.0, 24000.0, 96000)
    assert d is not None
    e = np.zeros(n)
    e[0] = 1.0
    want = np.abs(hilbert(e)).sum()
    assert want <= d["hilbert_l1"] <= want * (1 + 1e-5)


# ---- the strict mode's bound (split_strict.h, psk_split_kernels.hip KB) -----
def _adversarial(kind, baud, fc, fs, n, rng):
    """Inputs aimed at the split's weak spots: square waves
    resonant at each band-pass pole's frequency, the sign pattern of the
    slowest state response (the input that maximises a state's accumulated
    error), clipped full-scale PCM, chirps across the band edges, and a
    full-scale capture that opens with a wrapped (+/- full scale) click."""
    import _amr
    import synth
    _, _, bp, lp, _ = _amr.design_psk(kind, n, baud, fc, fs)
    b, a, _ = bp
    t = np.arange(n) / fs
    ins = {}
    poles = np.roots(a)
    for i, p in enumerate(sorted({round(abs(float(np.angle(q))), 9) for q in poles if np.angle(q) > 0})):
        ins[f"pole_sq{i}"] = np.sign(np.sin(p * np.arange(n) + 0.3))
    # sign pattern of the zero-input response from state 0 (the slowest decay), repeated
    z = np.zeros(len(a) - 1)
    z[0] = 1.0
    g = []
    for _ in range(4096):
        y = z[0]
        g.append(y)
        z = np.append(z[1:], 0.0) - a[1:] * y
    pat = np.sign(np.array(g[::-1]))
    pat[pat == 0] = 1.0
    ins["g_sign"] = np.resize(pat, n)
    if fs / baud >= 10:
        w = synth.qpsk_waveform(synth.random_frame(rng, 300), baud, fc, fs) if kind == "qpsk" else \
            synth.bpsk_waveform(synth.random_frame(rng, 300), baud, fc, fs)
        x = np.zeros(n)
        x[:min(n, w.size)] = w[:n]
        ins["clipped"] = np.clip(4.0 * x + rng.normal(0, 0.05, n), -1, 1)
        xc = x.copy()
        xc[0], xc[-1] = 1.0, -1.0
        ins["edge_clicks"] = xc
    nyq = fs / 2
    lo, hi = max(0.01 * nyq, fc - 1.5 * baud), min(0.99 * nyq, fc + 1.5 * baud)
    ins["chirp"] = np.sin(2 * np.pi * (0.7 * lo * t + (1.3 * hi - 0.7 * lo) * t * t / (2 * t[-1])))
    return ins


@pytest.mark.parametrize("kind,baud,fc,fs", CONFIGS, ids=lambda v: str(v))
def test_strict_bound_holds(kind, baud, fc, fs, built_lib):
    """The strict mode's bound (KB restated: tests/_util.py strict_symbol_bounds,
    from the oracle's restatement of KS0-KS2's statistics and libamr.so's
    strict design) is at least the measured |split - serial| on every symbol
    component, over the signal classes above and the adversarial inputs, at
    every filter set; the bound's size against kappa * peak is printed (the
    flag rate scales with it).  The adversarial inputs' measured error is
    also held against the default kappa: kappa / worst >= 16."""
    import _amr
    from oracle import oracle
    from _util import pass1_peak, strict_symbol_bounds
    n = 48000 if baud >= 1200 else 96000
    d = _amr.split_strict_design(kind, n, baud, fc, fs)
    assert d is not None and d["ok"] == 1.0
    sd = _amr.split_design(kind, n, baud, fc, fs)
    T = _amr.split_state_tables(kind, n, baud, fc, fs)
    pl = oracle.PskPlan(kind, n, baud, fc, fs)
    rng = np.random.default_rng(baud + 3 * int(fc))
    ins = _inputs(kind, baud, fc, fs, n, rng)
    ins.update(_adversarial(kind, baud, fc, fs, n, rng))
    worst_ratio, bound_ratio, adv_worst, bad = np.inf, [], 0.0, []
    for name, x in ins.items():
        ref = oracle.psk_symbols(kind, x, baud, fc, fs)
        peak = np.abs(x).max()
        for L in (128, 1024):
            st = oracle.psk_split_stats(kind, x, baud, fc, fs, L, sd["warmup_bp"], T, d)
            e, sc = strict_symbol_bounds(st, d, pass1_peak(x), n, pl.first, pl.sps, L)
            sp = oracle.psk_split_symbols(kind, x, baud, fc, fs, L, sd["warmup_bp"], sd["warmup_lp"], tables=T)
            act = np.abs(sp - ref)                  # the symbol's complex error (e(k) bounds |.|_2)
            if sc[4] and (act > e).any():
                bad.append((name, L, int((act > e).sum())))
            if sc[4]:
                worst_ratio = min(worst_ratio, float((e / np.maximum(act, 1e-300)).min()))
            bound_ratio.append(float(np.median(e)) / (sd["kappa"] * peak))   # both bound |symbol error|_2
            if name in ("g_sign", "clipped", "edge_clicks", "chirp") or name.startswith("pole_sq"):
                adv_worst = max(adv_worst, float(np.abs(sp - ref).max() / peak))
    print(f"{kind}@{baud} fc {fc:g} fs {fs:g}: strict bound / measured >= {worst_ratio:.1f}; median bound "
          f"{np.median(bound_ratio):.2f}x kappa peak; adversarial worst |split - serial| / peak {adv_worst:.3e} "
          f"(kappa / worst = {sd['kappa'] / max(adv_worst, 1e-300):.1f})")
    assert not bad, bad
    assert adv_worst <= sd["kappa"] / 16


# ---- the FSK split F1's strict bound (fsk_kernels.hip KF1-KF2, round 6) -----
def _fsk_adversarial(baud, mark, space, fs, n, rng):
    """The PSK adversarial set (above) aimed at the FSK tones' band-passes:
    square waves at every pole frequency of both filters, the sign pattern of
    each filter's slowest state response, a clipped full-scale FSK frame, a
    frame with full-scale edge clicks, a chirp across both bands."""
    import _fsk
    import synth
    _, tones = _fsk.design_fsk(n, baud, mark, space, fs)
    ins = {}
    for tn, (b, a, _) in zip("ms", tones):
        poles = np.roots(a)
        for i, p in enumerate(sorted({round(abs(float(np.angle(q))), 9) for q in poles if np.angle(q) > 0})):
            ins[f"pole_sq_{tn}{i}"] = np.sign(np.sin(p * np.arange(n) + 0.3))
        z = np.zeros(len(a) - 1)
        z[0] = 1.0
        g = []
        for _ in range(4096):
            y = z[0]
            g.append(y)
            z = np.append(z[1:], 0.0) - a[1:] * y
        pat = np.sign(np.array(g[::-1]))
        pat[pat == 0] = 1.0
        ins[f"g_sign_{tn}"] = np.resize(pat, n)
    w = synth.fsk_waveform(synth.random_frame(rng, 200), baud, mark, space, float(fs))
    x = np.zeros(n)
    x[:min(n, w.size)] = w[:n]
    ins["clipped"] = np.clip(4.0 * x + rng.normal(0, 0.05, n), -1, 1)
    xc = x.copy()
    xc[0], xc[-1] = 1.0, -1.0
    ins["edge_clicks"] = xc
    t = np.arange(n) / fs
    lo, hi = max(10.0, 0.7 * (mark - baud)), min(0.49 * fs, 1.3 * (space + baud))
    ins["chirp"] = np.sin(2 * np.pi * (lo * t + (hi - lo) * t * t / (2 * t[-1])))
    return ins


@pytest.mark.parametrize("baud,mark,space,fs", FSK_CONFIGS, ids=lambda v: str(v))
def test_fsk_strict_bound_holds(baud, mark, space, fs, built_lib):
    """The FSK split F1's strict bound per tone (KF1-KF2 restated:
    tests/_util.py strict_pass_bounds over the oracle's FS0-FS2 statistics and
    libamr.so's per-tone design) is at least the measured max |split - serial|
    of the tone's band-pass output, over the signal classes and the
    adversarial set, at two chunk lengths; its size against kappa peak is
    printed.  The adversarial set's measured error is also held against the
    default kappa: kappa / worst >= 16."""
    import _amr
    import _fsk
    from oracle import oracle
    from _util import pass1_peak, strict_pass_bounds
    n = 48000
    sd = _fsk.split_design(n, baud, mark, space, fs)
    D = _fsk.split_strict_design(n, baud, mark, space, fs)
    assert sd is not None and D is not None and all(d["ok"] == 1.0 for d in D)
    _, tones = _fsk.design_fsk(n, baud, mark, space, fs)
    T = [_amr.state_tables(b, a, zi, sd["warmup"]) for b, a, zi in tones]
    rng = np.random.default_rng(7 * baud + int(space))
    ins = _fsk_inputs(baud, mark, space, fs, n, rng)
    adv = _fsk_adversarial(baud, mark, space, fs, n, rng)
    ins.update(adv)
    worst_ratio, size, adv_worst, bad = np.inf, [], 0.0, []
    for name, x in ins.items():
        p1 = pass1_peak(x, 21)
        peak = np.abs(x).max()
        for t, (b, a, zi) in enumerate(tones):
            ref = oracle.filtfilt(b, a, x)
            for L in (128, 1024):
                st = oracle.fsk_split_stats(x, b, a, L, sd["warmup"], T[t], D[t])
                pb = strict_pass_bounds(st, D[t], p1, n, L, 21)
                sp = oracle.split_filtfilt(b, a, x, L, sd["warmup"], tables=T[t])
                act = float(np.abs(sp - ref).max())
                if pb["ok"]:
                    if act > pb["Fmax"]:
                        bad.append((name, t, L, act, pb["Fmax"]))
                    worst_ratio = min(worst_ratio, pb["Fmax"] / max(act, 1e-300))
                    size.append(pb["Fmax"] / (sd["kappa"] * peak))
                if name in adv:
                    adv_worst = max(adv_worst, act / peak)
    print(f"fsk@{baud} {mark:g}/{space:g} fs {fs}: strict F / measured >= {worst_ratio:.1f}; median F "
          f"{np.median(size):.2f}x kappa peak; adversarial worst |split - serial| / peak {adv_worst:.3e} "
          f"(kappa / worst = {sd['kappa'] / max(adv_worst, 1e-300):.1f})")
    assert not bad, bad
    assert adv_worst <= sd["kappa"] / 16
