"""GPU tests of the FSK time-split F1 (fsk_kernels.hip FS1-FS3):
the latency path of one capture at a time, the reference's own call pattern
(filebeep_advanced_v2.py:324 -> modem.fsk_demodulate, modem.py:298-341).

Bars:
  * the device's chunked band-pass computes exactly the oracle's restatement
    of it (oracle.split_filtfilt; equal values), whose error
    tests/test_split_margin.py (CPU) shows >= 90x below the plan's kappa;
  * decoded bytes and sync bit-exact with the reference / the oracle on every
    golden FSK case and on seeded batches, in both layouts: unflagged streams
    from the split F1, flagged ones (silence, DC, near-ties) from the exact
    path, which re-runs the serial F1 for them;
  * the flagged fraction of the benchmark's noisy captures is printed and
    stays small (each flagged capture pays the serial F1).
"""
import os
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def _cast(x, dtype):
    return np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dtype == np.int16 else x.astype(dtype)


@pytest.mark.parametrize("n,baud,mark,space,dtype,chunk", [
    (96000, 9600, 12000.0, 24000.0, np.float32, 0),
    (96000, 9600, 12000.0, 24000.0, np.float64, 193),
    (50001, 4800, 7000.0, 19000.0, np.float64, 0),     # Bluestein length
    (30000, 2400, 11229.28, 29833.37, np.int16, 333),
    (96000, 1200, 2400.0, 4800.0, np.float64, 0),
    (960000, 9600, 12000.0, 24000.0, np.float32, 0),   # a 10-s capture
])
def test_split_bandpass_is_the_restatement(n, baud, mark, space, dtype, chunk):
    import _amr
    import _fsk
    import synth
    from oracle import oracle
    B = 3
    x = _cast(synth.fsk_batch(B, n, baud, mark, space, seed=n % 1000, distinct=B, noise=0.2), dtype)
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    got = pl.split_bandpass(x, chunk)
    info = pl.split_info()
    assert info["warmup"] > 0 and info["chunk"] == (chunk or info["chunk"])
    _, ((mb, ma, mzi), (sb, sa, szi)) = _fsk.design_fsk(n, baud, mark, space, 96000)
    conv = pl.split_conv()      # FS0's convolution start states (AMR_FSK_SPLIT_CONV=0: warm-ups)
    assert conv or os.environ.get("AMR_FSK_SPLIT_CONV") == "0"
    for i in range(B):
        for t, (b, a, zi) in enumerate(((mb, ma, mzi), (sb, sa, szi))):
            tables = _amr.state_tables(b, a, zi, info["warmup"]) if conv else None
            want = oracle.split_filtfilt(b, a, x[i], info["chunk"], info["warmup"], tables=tables)
            assert np.array_equal(got[i, :, t], want), (i, t, np.abs(got[i, :, t] - want).max())


def _plan(n, baud, mark, space, B, layout):
    import _fsk
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    pl.set_layout(layout)
    return pl


def test_every_golden_fsk_case_split_and_serial(golden):
    """Every golden FSK case of the reference through a plan forced to the
    split F1 and through one forced to the serial F1: bytes == the reference's."""
    import _fsk
    manifest, inputs = golden
    cases = [c for c in manifest["cases"] if c["fn"] == "fsk_demodulate" and c["status"] == "ok"]
    assert cases
    split_runs = 0
    for layout in ("split", "serial"):
        for c in cases:
            x = np.asarray(inputs[c["id"]])
            a = c["params"]
            baud, mark, space, fs = (a.get("baud", 1200), a.get("mark_freq", 1200.0), a.get("space_freq", 2200.0),
                                     a.get("samp_rate", 96000))
            pl = _fsk.FskPlan(x.size, baud, mark, space, fs, max_streams=1)
            pl.set_layout(layout)
            got, _ = pl.demod_host(x[None])
            assert got[0] == bytes.fromhex(c["out"]), (layout, c["id"])
            split_runs += pl.split_info()["last_split"]
    print(f"{len(cases)} golden FSK cases x 2 layouts; {split_runs} ran the split F1")


@pytest.mark.parametrize("n,baud,mark,space,B,dtype", [
    (96000, 9600, 12000.0, 24000.0, 16, np.float32),
    (96000, 4800, 7000.0, 19000.0, 5, np.float64),
    (30000, 2400, 11229.28, 29833.37, 9, np.int16),
    (96000, 1200, 2400.0, 4800.0, 4, np.float64),
    (24001, 9600, 12000.0, 24000.0, 6, np.float32),   # Bluestein
    (960000, 9600, 12000.0, 24000.0, 2, np.float32),
])
def test_split_batch_vs_oracle(n, baud, mark, space, B, dtype):
    import synth
    from oracle import oracle
    x = _cast(synth.fsk_batch(B, n, baud, mark, space, seed=B + n, distinct=B, noise=0.1), dtype)
    pl = _plan(n, baud, mark, space, B, "split")
    got, _ = pl.demod_host(x)
    assert pl.split_info()["last_split"]
    want = [oracle.fsk_demodulate(r, baud, mark, space) for r in x]
    assert got == want
    print(f"fsk@{baud} n={n} B={B}: {pl.exact_streams()} flagged")


@pytest.mark.parametrize("layout", ["split", "serial"])
def test_split_silence_and_special_values(layout):
    """Digital silence (leading, inside the frame, the whole stream), a DC
    lead-in, a NaN, an inf, denormal-level input: bytes == the oracle's in
    both layouts.  The split flags the NaN / inf / denormal streams (every
    compare goes exact); silence is flagged only where a compare lands inside
    the margin (the Hilbert transform's 1/t tails of the signal usually keep
    the two envelopes apart there), and clean streams are not flagged."""
    import synth
    from oracle import oracle
    n, baud, mark, space, B = 96000, 9600, 12000.0, 24000.0, 8
    x = synth.fsk_batch(B, n, baud, mark, space, seed=8, distinct=B, noise=0.05).astype(np.float64)
    x[0, :12000] = 0.0
    x[1, 20000:26000] = 0.0
    x[2] = 0.0
    x[3, :9000] = 0.37 / 32768
    x[4, 30000] = np.nan
    x[5, 100] = np.inf
    x[6] *= 1e-310
    pl = _plan(n, baud, mark, space, B, layout)
    got, _ = pl.demod_host(x)
    want = [oracle.fsk_demodulate(r, baud, mark, space) for r in x]
    assert got == want
    if layout == "split":
        assert pl.exact_streams() >= 3
        clean = synth.fsk_batch(B, n, baud, mark, space, seed=9, distinct=B, noise=0.05)
        got, _ = pl.demod_host(clean)
        assert pl.exact_streams() == 0
        assert got == [oracle.fsk_demodulate(r, baud, mark, space) for r in clean]


def test_split_device_entry():
    """amr_fsk_demod_device with <= 1024 streams runs the split F1 too; its
    flagged streams' serial F1 re-run reads the caller's device x.  Bytes ==
    the oracle's on a batch with silence, NaN and clean streams."""
    import _fsk
    import synth
    from oracle import oracle
    from _util import fsk_device_demod
    n, baud, mark, space, B = 96000, 9600, 12000.0, 24000.0, 6
    x = synth.fsk_batch(B, n, baud, mark, space, seed=21, distinct=B, noise=0.05).astype(np.float64)
    x[0, :30000] = 0.0
    x[1, 5000] = np.nan
    x[2] *= 1e-310
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    got, _ = fsk_device_demod(pl, x)
    assert pl.split_info()["last_split"] and pl.exact_streams() >= 2
    assert got == [oracle.fsk_demodulate(r, baud, mark, space) for r in x]


def test_split_flag_rate_on_benchmark_captures():
    """The benchmark's inputs (clean FSK9600 frames + N(0, 0.05^2) noise): what
    fraction of single captures the split's wider margin sends to the exact
    path."""
    import synth
    from oracle import oracle
    n, B = 96000, 128
    x = synth.fsk_batch(B, n, 9600, 12000.0, 24000.0, seed=1000, distinct=64, noise=0.05)
    pl = _plan(n, 9600, 12000.0, 24000.0, 16, "auto")
    flagged, got = 0, []
    for s0 in range(0, B, 16):
        g, _ = pl.demod_host(x[s0:s0 + 16])
        assert pl.split_info()["last_split"]
        got += g
        flagged += pl.exact_streams()
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        want = list(ex.map(lambda r: oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0), x))
    assert got == want
    print(f"FSK9600 noisy captures: {flagged} of {B} flagged ({100.0 * flagged / B:.2f} %), tau "
          f"{pl.split_info()['tau']:.3e}")
    assert flagged <= B // 10


def test_one_capture_drop_in_latency():
    """modem.fsk_demodulate on one 1-s capture (the GUI's call) runs the split
    F1; its wall time is printed beside the serial F1's."""
    import _fsk
    import modem
    import synth
    x = synth.fsk_batch(8, 96000, 9600, 12000.0, 24000.0, seed=3, distinct=8, noise=0.05)
    args = dict(baud=9600, mark_freq=12000.0, space_freq=24000.0)
    outs = [modem.fsk_demodulate(x[i], **args) for i in range(8)]   # warm: plan, scratch
    ts = []
    for i in range(8):
        t = time.perf_counter()
        assert modem.fsk_demodulate(x[i], **args) == outs[i]
        ts.append(time.perf_counter() - t)
    ser = _plan(96000, 9600, 12000.0, 24000.0, 1, "serial")
    ser.demod_host(x[:1])
    tr = []
    for i in range(4):
        t = time.perf_counter()
        assert ser.demod_host(x[i:i + 1])[0][0] == outs[i]
        tr.append(time.perf_counter() - t)
    print(f"one FSK9600 capture: split {np.median(ts) * 1e3:.3f} ms (min {min(ts) * 1e3:.3f}), "
          f"serial {np.median(tr) * 1e3:.3f} ms")


def test_flagged_burst_after_clean_batches_device_entry():
    """The exact path's serial F1 re-run (E1, list mode) takes its grid from
    the plan's recent flagged counts and strides over the flagged streams
    (fsk_kernels.hip k_fsk_bandpass2): after 8 clean device-entry batches the
    grid is one workgroup, and a batch with 100 flagged streams (a NaN each:
    every compare goes exact) must still have all 100 recomputed.  Bytes ==
    the oracle's."""
    import _fsk
    import synth
    from oracle import oracle
    from _util import fsk_device_demod
    n, baud, mark, space, B = 24000, 9600, 12000.0, 24000.0, 128
    clean = synth.fsk_batch(B, n, baud, mark, space, seed=31, distinct=8, noise=0.05).astype(np.float64)
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=B)
    for _ in range(8):
        fsk_device_demod(pl, clean)
        assert pl.exact_streams() == 0
    x = clean.copy()
    x[:100, 777] = np.nan
    got, _ = fsk_device_demod(pl, x)
    assert pl.exact_streams() == 100
    want = [oracle.fsk_demodulate(r, baud, mark, space) for r in x]
    assert got == want
