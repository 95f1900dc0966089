"""Shared test helpers: run a golden case through a demod callable."""
from __future__ import annotations


def call_case(mod, case, x):
    """Dispatch one manifest case to `mod` (the product modem module or the oracle)."""
    fn, p = case["fn"], case["params"]
    if fn == "qpsk_demodulate":
        return mod.qpsk_demodulate(x, **p)
    if fn == "bpsk_demodulate":
        return mod.bpsk_demodulate(x, **p)
    if fn == "psk8_demodulate":
        return mod.psk8_demodulate(x, p["b"])
    if fn == "ofdm_demodulate_simple":
        return mod.ofdm_demodulate_simple(x, p["baud"], p["carrier"], p["num_subcarriers"])
    if fn == "fsk_demodulate":
        return mod.fsk_demodulate(x, **p)
    if fn == "fsk_high_speed_demodulate":
        return mod.fsk_high_speed_demodulate(x, p["baud"])
    raise KeyError(fn)


def outcome(fn):
    try:
        return ("ok", fn().hex())
    except ValueError as e:   # the reference's error contract is scipy's ValueError
        return ("err", "ValueError", str(e))


def expected(case):
    if case["status"] == "ok":
        return ("ok", case["out"])
    return ("err", case["etype"], case["emsg"])


def call_sweep_case(mod, case, x):
    """Dispatch one sweep case (tests/golden/sweep_manifest.json) to `mod`."""
    fn, p = case["fn"], case["params"]
    if fn == "fsk":
        return mod.fsk_demodulate(x, baud=p["baud"], mark_freq=p["f0"], space_freq=p["f1"], samp_rate=p["samp_rate"])
    f = mod.qpsk_demodulate if fn == "qpsk" else mod.bpsk_demodulate
    return f(x, baud=p["baud"], carrier=p["f0"], samp_rate=p["samp_rate"])
