"""Raw-integer captures through the drop-in on the MI355X.

The reference hands the caller's array straight to scipy.signal.filtfilt
(modem.py:77, 198, 308), which forms its odd extension 2*x[0] - x[k] in the
array's own dtype: a full-scale int16 capture wraps, uint8 wraps below zero,
float16 rounds (and overflows).  The drop-in sends such an array as its exact
float32 / float64 values plus the extension numpy forms in the caller's dtype
(_amr.raw_input -> amr_*_demod_host_edges), and every kernel layout reads that
table instead of forming the extension (odd_ext.h).  Checked here against the
REFERENCE's own bytes (tests/golden/make_rawint_golden.py: 24 captures, 13 of
which the wrap decides) in every PSK layout (time-split, row, lane) and FSK F1
layout (split, serial) with the exact path at its default and on every
stream, and against the oracle's raw dtypes on batches."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _call(modem, c, x):
    p = c["params"]
    if c["fn"] == "fsk":
        return modem.fsk_demodulate(x, baud=p["baud"], mark_freq=p["f0"], space_freq=p["f1"], samp_rate=p["samp_rate"])
    f = modem.qpsk_demodulate if c["fn"] == "qpsk" else modem.bpsk_demodulate
    return f(x, baud=p["baud"], carrier=p["f0"], samp_rate=p["samp_rate"])


def test_rawint_fixtures_default_layouts(rawint_golden):
    """modem.* on each raw capture (one capture per call: the PSK time-split
    and FSK split-F1 layouts, the reference's own call pattern) == the
    reference's bytes."""
    import modem
    from _util import expected, outcome
    manifest, inputs = rawint_golden
    bad = [(c["id"], c["fn"], c["dtype"]) for c in manifest["cases"]
           if outcome(lambda: _call(modem, c, inputs[c["id"]])) != expected(c)]
    assert not bad, f"{len(bad)} of {len(manifest['cases'])} differ from the reference: {bad}"


@pytest.mark.parametrize("layout", ["row", "lane", "split"])
def test_rawint_fixtures_every_psk_layout(rawint_golden, layout):
    """The PSK fixtures with the layout forced on the drop-in's cached plan:
    the row kernels (K1r / K1g), the lane kernels (k_bp_lane2) and the
    time-split passes (KS0 / KS1) each read the edge table."""
    import _amr
    import modem
    from _util import expected, outcome
    manifest, inputs = rawint_golden
    bad = []
    for c in manifest["cases"]:
        if c["fn"] == "fsk":
            continue
        x, p = inputs[c["id"]], c["params"]
        pl = _amr.get_psk_plan(c["fn"], x.size, p["baud"], p["f0"], p["samp_rate"], 1)
        pl.set_layout(layout)
        try:
            got = outcome(lambda: _call(modem, c, x))
            assert pl.last_layout() == layout or (layout == "split" and pl.last_layout() == "row")
        finally:
            pl.set_layout(None)
        if got != expected(c):
            bad.append((c["id"], c["fn"], c["dtype"]))
    assert not bad, f"{layout}: {bad}"


@pytest.mark.parametrize("layout,exact", [("serial", 1), ("split", 1), ("serial", 2), ("split", 2)])
def test_rawint_fixtures_every_fsk_layout(rawint_golden, layout, exact):
    """The FSK fixtures with F1 forced serial / split, the exact path on the
    flagged streams (1) or on every stream (2: E1 re-runs F1 in list mode,
    reading the edge table through the stream list)."""
    import _fsk
    import modem
    from _util import expected, outcome
    manifest, inputs = rawint_golden
    bad = []
    for c in manifest["cases"]:
        if c["fn"] != "fsk":
            continue
        x, p = inputs[c["id"]], c["params"]
        pl = _fsk.get_fsk_plan(x.size, p["baud"], p["f0"], p["f1"], p["samp_rate"], 1)
        pl.set_layout(layout)
        pl.set_exact_mode(exact)
        try:
            got = outcome(lambda: _call(modem, c, x))
            assert pl.split_info()["last_split"] == (layout == "split")
            if exact == 2:
                assert pl.exact_streams() == 1
        finally:
            pl.set_layout("auto")
            pl.set_exact_mode(1)
        if got != expected(c):
            bad.append((c["id"], c["dtype"]))
    assert not bad, f"{layout}/{exact}: {bad}"


def _raw_batch(rng, kind, dt, B, n, baud, f0, f1):
    import synth
    rows = []
    for i in range(B):
        fr = synth.random_frame(rng, int(rng.integers(8, 120)))
        if kind == "qpsk":
            w = synth.qpsk_waveform(fr, baud, f0, 96000.0)
        else:
            w = synth.fsk_waveform(fr, baud, f0, f1, 96000.0)
        x = np.zeros(n)
        x[:min(n, w.size)] = w[:n]
        x = np.clip(0.97 * x + rng.normal(0, 0.03, n), -1, 1)
        if i % 3 == 0:
            x[0] = rng.choice([0.98, -0.98])          # a wrapping left edge
        if i % 4 == 1:
            x[-1] = rng.choice([0.98, -0.98])         # a wrapping right edge
        rows.append(x)
    x = np.stack(rows)
    if dt == np.uint8:
        return np.clip(np.round(128 + 120 * x), 0, 255).astype(np.uint8)
    info = np.iinfo(dt)
    return np.round(x * (info.max if info.max < 2 ** 40 else 2.0 ** 40)).astype(dt)


@pytest.mark.parametrize("dt", [np.int16, np.uint8, np.int32])
def test_raw_psk_batches_every_layout(dt):
    """Batches of 1 / 40 / 97 raw captures (a third with a wrapping left edge,
    a quarter a wrapping right one) in the row, lane and split layouts ==
    the oracle's raw dtype, bytes and sync index, stream by stream."""
    import _amr
    from oracle import oracle
    rng = np.random.default_rng(31 + np.dtype(dt).itemsize)
    nt = min(16, os.cpu_count() or 1)
    bad = []
    for B, layout in ((1, "split"), (40, "row"), (40, "split"), (97, "lane")):
        x = _raw_batch(rng, "qpsk", dt, B, 24000, 9600, 3000.0, 0.0)
        pl = _amr.PskPlan("qpsk", x.shape[1], 9600, max_streams=B)
        pl.set_layout(layout)
        got, gs = pl.demod_host_raw(x)
        assert pl.last_layout() in (layout, "row")
        want, ws = oracle.psk_demod_batch("qpsk", x, 9600, n_threads=nt, raw_int16=True)
        bad += [(B, layout, i) for i in range(B) if got[i] != want[i] or gs[i] != ws[i]]
    assert not bad, bad


@pytest.mark.parametrize("dt", [np.int16, np.uint8])
def test_raw_fsk_batches(dt):
    """FSK batches of raw captures (split F1 at 8 streams, serial at 40) ==
    the oracle's raw dtype."""
    import _fsk
    from oracle import oracle
    rng = np.random.default_rng(41 + np.dtype(dt).itemsize)
    bad = []
    for B, layout in ((8, "split"), (40, "serial")):
        x = _raw_batch(rng, "fsk", dt, B, 24000, 9600, 12000.0, 24000.0)
        pl = _fsk.FskPlan(x.shape[1], 9600, 12000.0, 24000.0, max_streams=B)
        pl.set_layout(layout)
        got, _ = pl.demod_host_raw(x)
        want = [oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0, raw_int16=True) for r in x]
        bad += [(B, layout, i) for i in range(B) if got[i] != want[i]]
    assert not bad, bad
