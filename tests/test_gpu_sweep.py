"""Randomised parameter sweep of the demod core against the oracle: a seeded
draw of configurations across the space the reference's signatures accept
(modem.py:68, :189, :298 -- baud, carrier / tones, sample rate, stream
length, input dtype, batch size) rather than the benchmark's few, each
through the GPU in the layout drawn (PSK: row = one batch alone, every other
one of them by batch size -- the time-split layout up to 64 streams -- lane =
the plan told many batches are in flight), every stream's bytes and sync index
bit-exact with the oracle -- or the same ValueError text, where the
reference's scipy design raises.  Input: a framed, modulated signal at the
drawn rate (after a drawn stretch of silence) plus noise of a drawn level
(none to heavy -- FSK too: its digital-silence stretches, where only
pocketfft's own rounding decides, go through the exact path at every
length), or plain noise."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# AMR_SWEEP_PSK / AMR_SWEEP_FSK / AMR_SWEEP_SEED: a longer stress draw (a
# progress line every 50 configurations keeps a long run visibly alive)
N_PSK = int(os.environ.get("AMR_SWEEP_PSK", "140"))
N_FSK = int(os.environ.get("AMR_SWEEP_FSK", "36"))
SEED = int(os.environ.get("AMR_SWEEP_SEED", "0"))
FSK_BMAX = int(os.environ.get("AMR_SWEEP_FSK_BMAX", "6"))


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def _signal(rng, kind, B, n, baud, f0, f1, fs):
    import synth
    noise = float(rng.choice([0.0, 0.02, 0.1, 0.4]))
    if rng.random() < 0.15:
        x = rng.normal(0, 0.5, (B, n))
    else:
        rows = []
        for _ in range(B):
            fr = synth.random_frame(rng, int(rng.integers(4, 64)))
            try:
                if kind == "qpsk":
                    w = synth.qpsk_waveform(fr, baud, f0, fs)
                elif kind == "bpsk":
                    w = synth.bpsk_waveform(fr, baud, f0, fs)
                else:
                    w = synth.fsk_waveform(fr, baud, f0, f1, fs)
            except ValueError:        # the reference's PSK modulators raise below 10 samples per symbol
                w = rng.normal(0, 0.5, n)
            off = int(rng.integers(0, max(1, n // 4)))
            row = np.zeros(n)
            seg = w[:max(0, n - off)]
            row[off:off + seg.size] = seg
            rows.append(row)
        x = np.stack(rows) + rng.normal(0, noise, (B, n))
    dt = rng.choice(["f32", "f64", "i16"])
    if dt == "i16":
        return np.round(np.clip(x, -1, 1) * 32767).astype(np.int16)
    return x.astype(np.float32 if dt == "f32" else np.float64)


def _outcome(fn):
    try:
        return "ok", fn()
    except ValueError as e:
        return "ValueError", str(e)


def test_psk_sweep():
    import _amr
    from oracle import oracle
    rng = np.random.default_rng(2024 + SEED)
    bad = []
    for c in range(N_PSK):
        if c and c % 50 == 0:
            print(f"psk sweep: {c} of {N_PSK} configurations, {len(bad)} differ", flush=True)
        kind = "qpsk" if rng.random() < 0.7 else "bpsk"
        fs = float(rng.choice([96000, 96000, 48000, 44100]))
        baud = int(rng.choice([300, 600, 1000, 1200, 1500, 2400, 3000, 4800, 9600, 19200]))
        carrier = float(rng.choice([3000.0, 3000.0, 1800.0, 6000.0, 12000.0]))
        n = int(rng.choice([int(rng.integers(28, 400)), int(rng.integers(400, 20000)), int(rng.integers(20000, 120000))]))
        B = int(rng.integers(1, 40))
        layout = "lane" if rng.random() < 0.5 else "row"
        x = _signal(rng, kind, B, n, baud, carrier, 0.0, fs)
        # int16 batches: the plans' PCM path (int16 / 32768), or every third
        # configuration the reference's raw semantics (the odd extension in
        # int16, wrapping -- the drop-in's public path, _amr.raw_input)
        raw = x.dtype == np.int16 and c % 3 == 0

        def gpu_run():
            plan = _amr.PskPlan(kind, n, baud, carrier, fs, max_streams=B)
            if layout == "lane":
                plan.set_inflight(max(1, 16384 // B + 1))
            elif c % 2 == 0:
                plan.set_layout("row")       # else by batch size: the time-split layout up to 64 streams
            out = plan.demod_host_raw(x) if raw else plan.demod_host(x)
            assert plan.last_layout() in (layout, "row", "split"), plan.last_layout()
            return out[0], [int(s) for s in out[1]]

        def cpu_run():
            o, s = oracle.psk_demod_batch(kind, x, baud, carrier, fs, n_threads=min(16, os.cpu_count() or 1),
                                          raw_int16=raw)
            return o, [int(v) for v in s]
        g, w = _outcome(gpu_run), _outcome(cpu_run)
        if g != w:
            bad.append((c, kind, baud, carrier, fs, n, B, str(x.dtype), layout, g[0], w[0]))
    assert not bad, f"{len(bad)} of {N_PSK} configurations differ: {bad[:5]}"


def test_fsk_sweep():
    import modem
    from oracle import oracle
    rng = np.random.default_rng(4048 + SEED)
    bad = []
    for c in range(N_FSK):
        if c and c % 50 == 0:
            print(f"fsk sweep: {c} of {N_FSK} configurations, {len(bad)} differ", flush=True)
        fs = float(rng.choice([96000, 96000, 48000]))
        baud = int(rng.choice([300, 1200, 2400, 4800, 9600, 19200]))
        nyq = fs / 2
        # tones: mostly valid bands, sometimes the reference's defaults (which raise above ~1200 Bd)
        if rng.random() < 0.2:
            mark, space = 1200.0, 2200.0
        else:
            lo, hi = baud * 1.1, nyq - baud * 1.1
            if hi <= lo:
                mark, space = 1200.0, 2200.0
            else:
                mark, space = sorted(float(v) for v in rng.uniform(lo, hi, 2))
        n = int(rng.choice([int(rng.integers(22, 3000)), int(rng.integers(3000, 100000))]))
        B = int(rng.integers(1, FSK_BMAX))
        x = _signal(rng, "fsk", B, n, baud, mark, space, fs)
        g = _outcome(lambda: modem.fsk_demodulate_batch(x, baud=baud, mark_freq=mark, space_freq=space, samp_rate=fs))
        # the public drop-in takes an int16 capture as the reference does: raw
        # values, the odd extension formed (and wrapping) in int16 -- the
        # oracle's raw int16 (amr_oracle.c AMR_DT_RAW_I16), not its PCM path
        w = _outcome(lambda: [oracle.fsk_demodulate(r, baud, mark, space, fs, raw_int16=True) for r in x])
        if g != w:
            bad.append((c, baud, mark, space, fs, n, B, str(x.dtype), g[0], w[0], str(g[1])[:80], str(w[1])[:80]))
    assert not bad, f"{len(bad)} of {N_FSK} configurations differ: {bad[:5]}"


def test_reference_sweep_through_the_drop_in(sweep_golden):
    """The drop-in modules (modem.qpsk_demodulate / bpsk_demodulate /
    fsk_demodulate on the GPU) against the REFERENCE's own outputs on the 72
    seeded configurations of tests/golden/make_sweep_golden.py: bytes or
    exception text equal, every case -- the FSK cases inside exact digital
    silence, DC and near-silent stretches too, at 5-smooth, generic-radix and
    Bluestein lengths, through the exact path.
    The reference saw int16 fixtures as int16 / 32768 (as libsndfile reads a
    WAV); the public drop-in functions treat integer input as raw values, as
    the reference itself would -- identical decisions up to 2^15 scaling,
    except where the envelopes are rounding noise (c85: a DC lead-in) -- so
    int16 cases go in as int16 / 32768, and the FSK ones also through the
    plans' own PCM16 path (int16 on the device, converted exactly)."""
    import _fsk
    import modem
    from _util import call_sweep_case, expected, outcome
    manifest, inputs = sweep_golden
    bad = []
    for c in manifest["cases"]:
        x = inputs[c["id"]]
        if x.dtype == np.int16:
            xs = x.astype(np.float64) / 32768.0
            got = outcome(lambda: call_sweep_case(modem, c, xs))
            if c["fn"] == "fsk" and got == expected(c) and got[0] == "ok":
                p = c["params"]
                pcm = outcome(lambda: _fsk.fsk_demodulate_batch(x[None], p["baud"], p["f0"], p["f1"], p["samp_rate"])[0])
                if pcm != got:
                    bad.append((c["id"], "pcm16", c["params"], c["n"]))
        else:
            got = outcome(lambda: call_sweep_case(modem, c, x))
        if got != expected(c):
            bad.append((c["id"], c["fn"], c["params"], c["dtype"], c["n"], got[0]))
    assert not bad, f"{len(bad)} of {len(manifest['cases'])} differ from the reference: {bad[:5]}"
