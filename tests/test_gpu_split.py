"""GPU tests of the PSK time-split layout (psk_split_kernels.hip, DESIGN.md
§3.3): the latency path of one capture at a time, the reference's own call
pattern (filebeep_advanced_v2.py:324, 1112 -> modem.qpsk_demodulate,
modem.py:189-266).

Bars:
  * the device's chunked passes compute exactly the oracle's restatement of
    them (oracle.psk_split_symbols; equal values, the sign of a zero aside);
    tests/test_split_margin.py (CPU) shows that restatement's error stays
    >= 55x below the plan's kappa;
  * decoded bytes and sync index bit-exact with the reference / the oracle on
    every golden and sweep case and on seeded batches -- unflagged streams
    from the split passes, flagged ones (silence, specials, near-ties) from the
    gated serial kernels behind them;
  * the flagged fraction of the benchmark's noisy QPSK@9600 captures is
    printed and stays small (every flagged capture costs a serial re-run).
"""
import os
import time

import numpy as np
import pytest

from _util import call_case, call_sweep_case, expected, outcome

pytestmark = pytest.mark.gpu


def _batch(kind, B, n, baud, fc, fs, seed, noise):
    """B noisy framed streams: DQPSK (8-ary DPSK below 10 samples per symbol,
    where the reference's own modulator raises) or DBPSK."""
    import synth
    if kind == "qpsk":
        f = synth.qpsk_batch if fs / baud >= 10 else synth.dpsk8_batch
        return f(B, n, baud, carrier=fc, samp_rate=fs, seed=seed, distinct=B, noise=noise)
    rng = np.random.default_rng(seed)
    rows = [synth.fit(synth.bpsk_waveform(synth.random_frame(rng, 60), baud, fc, fs), n) for _ in range(B)]
    return (np.stack(rows) + rng.normal(0, noise, (B, n))).astype(np.float32)


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


@pytest.mark.parametrize("kind,baud,fc,fs,n,dtype,chunk", [
    ("qpsk", 9600, 3000.0, 96000, 96000, np.float32, 0),
    ("qpsk", 9600, 3000.0, 96000, 96000, np.float64, 193),
    ("qpsk", 19200, 3000.0, 96000, 50001, np.int16, 0),
    ("bpsk", 1200, 3000.0, 96000, 48000, np.float32, 333),
    ("qpsk", 1000, 3000.0, 48000, 40000, np.float64, 0),
    ("qpsk", 9600, 3000.0, 96000, 960000, np.float32, 0),    # a 10-s capture
])
def test_split_symbols_are_the_restatement(kind, baud, fc, fs, n, dtype, chunk):
    import _amr
    import synth
    from oracle import oracle
    B = 3
    x = _batch(kind, B, n, baud, fc, fs, n, 0.2)
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dtype == np.int16 else x.astype(dtype)
    pl = _amr.PskPlan(kind, n, baud, fc, fs, max_streams=B)
    got = pl.split_symbols(x, chunk)
    info = pl.split_info()
    assert info["warmup_bp"] > 0 and info["chunk"] == (chunk or info["chunk"])
    # the default start states: KS0's convolution (AMR_PSK_SPLIT_CONV=0: warm-ups,
    # test_split_warmup_variant)
    tables = _amr.split_state_tables(kind, n, baud, fc, fs) if pl.split_conv() else None
    assert tables is not None or os.environ.get("AMR_PSK_SPLIT_CONV") == "0"
    for i in range(B):
        want = oracle.psk_split_symbols(kind, x[i], baud, fc, fs, info["chunk"], info["warmup_bp"], info["warmup_lp"],
                                        tables=tables)
        assert np.array_equal(got[i], want), (i, np.abs(got[i] - want).max())


def test_split_warmup_variant(tmp_path):
    """AMR_PSK_SPLIT_CONV=0 (a subprocess: the switch is read once): the band-pass
    chunks start from w1-step warm-ups instead of KS0's convolution states --
    the restatement without tables, and bytes == the oracle on a seeded batch."""
    import subprocess
    import sys
    script = tmp_path / "warm.py"
    script.write_text(f'''
import sys
sys.path[:0] = {[os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."),
                 os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "audio-modem-radio_amd"),
                 os.path.dirname(os.path.abspath(__file__))]!r}
import numpy as np
import _amr, synth
from oracle import oracle
bad = []
for kind, baud, n, B in (("qpsk", 9600, 96000, 3), ("bpsk", 1200, 48000, 2)):
    x = synth.qpsk_batch(B, n, baud, seed=B, distinct=B, noise=0.1)
    pl = _amr.PskPlan(kind, n, baud, 3000.0, 96000, max_streams=B)
    assert not pl.split_conv()
    got = pl.split_symbols(x, 0)
    info = pl.split_info()
    for i in range(B):
        want = oracle.psk_split_symbols(kind, x[i], baud, 3000.0, 96000, info["chunk"], info["warmup_bp"], info["warmup_lp"])
        if not np.array_equal(got[i], want):
            bad.append((kind, "sym", i))
    pl.set_layout("split")
    o, s = pl.demod_host(x)
    wo, ws = oracle.psk_demod_batch(kind, x, baud, 3000.0, 96000)
    if list(o) != list(wo) or [int(v) for v in s] != [int(v) for v in ws]:
        bad.append((kind, "bytes"))
print("BAD", bad)
sys.exit(1 if bad else 0)
''')
    env = dict(os.environ, AMR_PSK_SPLIT_CONV="0")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def _split_plan(kind, n, baud, fc=3000.0, fs=96000, B=1):
    import _amr
    pl = _amr.PskPlan(kind, n, baud, fc, fs, max_streams=B)
    pl.set_layout("split")
    return pl


def test_every_golden_psk_case_split_and_row(golden):
    """Every golden PSK case of the reference through a plan forced to the
    time-split layout, and through one forced to the serial row layout: bytes
    (or the ValueError) == the reference's in both."""
    import _amr
    manifest, inputs = golden
    cases = [c for c in manifest["cases"] if c["fn"] in ("qpsk_demodulate", "bpsk_demodulate", "psk8_demodulate",
                                                          "ofdm_demodulate_simple")]
    assert len(cases) >= 20
    bad = []
    for layout in ("split", "row"):
        for case in cases:
            class M:   # the drop-in signature, on a forced-layout plan
                pass

            def run(x, kind, baud, carrier=3000.0, samp_rate=96000):
                x = np.asarray(x)
                if x.dtype not in _amr.DTYPES:
                    x = x.astype(np.float64)
                pl = _amr.PskPlan(kind, x.size, baud, carrier, samp_rate, max_streams=1)
                pl.set_layout(layout)
                out = pl.demod_host(x[None])[0][0]
                if pl.n > 0 and pl.last_layout() not in (layout, "row"):
                    raise AssertionError(pl.last_layout())
                return out
            M.qpsk_demodulate = staticmethod(lambda s, baud=1200, carrier=3000.0, samp_rate=96000:
                                             run(s, "qpsk", baud, carrier, samp_rate))
            M.bpsk_demodulate = staticmethod(lambda s, baud=1200, carrier=3000.0, samp_rate=96000:
                                             run(s, "bpsk", baud, carrier, samp_rate))
            M.psk8_demodulate = staticmethod(lambda s, b=1200, c=3000.0, s_r=96000: run(s, "qpsk", b, c, s_r))
            M.ofdm_demodulate_simple = staticmethod(lambda s, baud, carrier, num_subcarriers, samp_rate=96000:
                                                    run(s, "qpsk", baud, carrier, samp_rate))
            got = outcome(lambda: call_case(M, case, inputs[case["id"]]))
            if got != expected(case):
                bad.append((layout, case["id"], got[:2]))
    assert not bad, f"differs from the reference on {bad[:6]}"


def test_reference_sweep_split(sweep_golden):
    """The 100+ reference-generated sweep cases' PSK ones (tests/golden/
    make_sweep_golden.py) through the drop-in modules -- whose one-capture
    calls now run the time-split layout -- bytes or exception == reference."""
    import modem
    manifest, inputs = sweep_golden
    bad, n_psk = [], 0
    for c in manifest["cases"]:
        if c["fn"] == "fsk":
            continue
        n_psk += 1
        x = inputs[c["id"]]
        xs = x.astype(np.float64) / 32768.0 if x.dtype == np.int16 else x
        got = outcome(lambda: call_sweep_case(modem, c, xs))
        if got != expected(c):
            bad.append((c["id"], c["fn"], c["params"], got[0]))
    assert n_psk >= 40
    assert not bad, f"{len(bad)} differ: {bad[:4]}"


@pytest.mark.parametrize("kind,baud,fc,fs,n,B,dtype", [
    ("qpsk", 9600, 3000.0, 96000, 96000, 16, np.float32),
    ("qpsk", 19200, 3000.0, 96000, 96000, 5, np.float64),
    ("bpsk", 1200, 3000.0, 96000, 48000, 9, np.int16),
    ("qpsk", 300, 3000.0, 96000, 96000, 4, np.float32),
    ("qpsk", 1000, 1800.0, 44100, 44100, 7, np.float64),
    ("qpsk", 9600, 3000.0, 96000, 960000, 2, np.float32),
])
def test_split_batch_vs_oracle(kind, baud, fc, fs, n, B, dtype):
    import synth
    from oracle import oracle
    x = _batch(kind, B, n, baud, fc, fs, B + n, 0.1)
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dtype == np.int16 else x.astype(dtype)
    pl = _split_plan(kind, n, baud, fc, fs, B)
    got, gs = pl.demod_host(x)
    assert pl.last_layout() == "split"
    want, ws = oracle.psk_demod_batch(kind, x, baud, fc, fs, n_threads=min(16, os.cpu_count() or 1))
    assert got == want and np.array_equal(gs, ws)
    print(f"{kind}@{baud} n={n} B={B}: {pl.split_info()['flagged']} flagged")


def test_split_flags_silence_and_special_values():
    """Streams the margin cannot clear -- exact digital silence (leading,
    inside the frame, the whole stream), a NaN, an inf, denormal-level input
    -- are flagged, and the gated serial kernels give the reference's bytes;
    clean noisy streams in the same batch are not flagged."""
    import synth
    from oracle import oracle
    B, n = 8, 48000
    x = synth.qpsk_batch(B, n, 9600, seed=8, distinct=B, noise=0.05).astype(np.float64)
    x[0, :12000] = 0.0
    x[1, 20000:26000] = 0.0
    x[2] = 0.0
    x[3, 30000] = np.nan
    x[4, 100] = np.inf
    x[5] *= 1e-310
    pl = _split_plan("qpsk", n, 9600, B=B)
    got, gs = pl.demod_host(x)
    want, ws = oracle.psk_demod_batch("qpsk", x, 9600)
    assert got == want and np.array_equal(gs, ws)
    assert pl.split_info()["flagged"] >= 5
    assert pl.exact_streams() >= 0
    clean = synth.qpsk_batch(B, n, 9600, seed=9, distinct=B, noise=0.05)
    pl.demod_host(clean)
    assert pl.split_info()["flagged"] == 0
    # nothing flagged: the gated row fallback (and its exact low-pass) did not run
    assert pl.exact_streams() == 0


def test_split_diagnostics_refuse_tiny_chunks():
    """With the convolution chunk starts on, a diagnostic chunk of 1..127
    outputs is refused (its start states would take B m1 / L x 64 B); 0 and
    >= 128 run."""
    import _amr
    import _fsk
    import synth
    n = 48000
    x = synth.qpsk_batch(2, n, 9600, seed=4, distinct=2)
    pl = _amr.PskPlan("qpsk", n, 9600, max_streams=2)
    if pl.split_conv():
        with pytest.raises(_amr.AmrError):
            pl.split_symbols(x, 1)
    assert pl.split_symbols(x, 128).shape[0] == 2
    xf = synth.fsk_batch(2, n, 9600, 12000.0, 24000.0, seed=4, distinct=2)
    fp = _fsk.FskPlan(n, 9600, 12000.0, 24000.0, max_streams=2)
    if fp.split_conv():
        with pytest.raises(_amr.AmrError):
            fp.split_bandpass(xf, 64)
    assert fp.split_bandpass(xf, 128).shape[0] == 2


def test_split_flag_rate_on_benchmark_captures():
    """The benchmark's inputs (clean frames + N(0, 0.05^2) noise, QPSK@9600):
    what fraction of single captures the margin sends to the serial path."""
    import synth
    from oracle import oracle
    n, B = 96000, 256
    x = synth.qpsk_batch(B, n, 9600, seed=1000, distinct=64, noise=0.05)
    pl = _split_plan("qpsk", n, 9600, B=16)
    flagged, got = 0, []
    for s0 in range(0, B, 16):
        g, _ = pl.demod_host(x[s0:s0 + 16])
        got += g
        flagged += pl.split_info()["flagged"]
    want, _ = oracle.psk_demod_batch("qpsk", x, 9600, n_threads=min(16, os.cpu_count() or 1))
    assert got == want
    print(f"QPSK@9600 noisy captures: {flagged} of {B} flagged ({100.0 * flagged / B:.2f} %), kappa "
          f"{pl.split_info()['kappa']:.3e}")
    assert flagged <= B // 10


def test_one_capture_drop_in_latency():
    """modem.qpsk_demodulate on one 1-s capture (the GUI's call) runs the
    time-split layout; its wall time is printed beside the serial row layout's."""
    import _amr
    import modem
    import synth
    x = synth.qpsk_batch(8, 96000, 9600, seed=3, distinct=8, noise=0.05)
    outs = [modem.qpsk_demodulate(x[i], baud=9600) for i in range(8)]   # warm: plan, scratch
    plan = _amr.get_psk_plan("qpsk", 96000, 9600, 3000.0, 96000, 1)
    assert plan.last_layout() == "split"
    ts = []
    for i in range(8):
        t = time.perf_counter()
        assert modem.qpsk_demodulate(x[i], baud=9600) == outs[i]
        ts.append(time.perf_counter() - t)
    row = _amr.PskPlan("qpsk", 96000, 9600, max_streams=1)
    row.set_layout("row")
    row.demod_host(x[:1])
    tr = []
    for i in range(4):
        t = time.perf_counter()
        assert row.demod_host(x[i:i + 1])[0][0] == outs[i]
        tr.append(time.perf_counter() - t)
    print(f"one capture: split {np.median(ts) * 1e3:.3f} ms (min {min(ts) * 1e3:.3f}), "
          f"row {np.median(tr) * 1e3:.3f} ms")
