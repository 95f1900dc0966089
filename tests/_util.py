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


def fsk_device_demod(pl, x):
    """amr_fsk_demod_device on x copied to device memory: (bytes list, sync)."""
    import ctypes

    import numpy as np
    import _amr
    L = _amr.lib()
    B, n = x.shape
    cap = max(pl.out_cap, 1)
    ptrs = {}
    for name, nbytes in (("x", x.nbytes), ("out", B * cap), ("len", B * 8), ("sync", B * 8)):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), nbytes))
        ptrs[name] = p
    try:
        _amr.check(L.amr_memcpy_h2d(ptrs["x"], _amr.ptr(x), x.nbytes))
        _amr.check(L.amr_fsk_demod_device(pl.handle, ptrs["x"], _amr.DTYPES[x.dtype], B, n, ptrs["out"], cap,
                                          ptrs["len"], ptrs["sync"]))
        _amr.check(L.amr_fsk_plan_synchronize(pl.handle))
        out, ln, sy = np.empty((B, cap), np.uint8), np.empty(B, np.int64), np.empty(B, np.int64)
        for name, h in (("out", out), ("len", ln), ("sync", sy)):
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(h), ptrs[name], h.nbytes))
    finally:
        for p in ptrs.values():
            L.amr_free(p)
    return [out[i, :ln[i]].tobytes() for i in range(B)], sy
