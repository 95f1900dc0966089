#!/usr/bin/env python3
"""Reference outputs on RAW integer (and bool / float16) captures (this
container only).  The reference's public demodulators hand the caller's array
straight to scipy.signal.filtfilt (modem.py:77, 198, 308), whose odd extension
2*x[0] - x[k] (scipy _arraytools.odd_ext) is formed in the ARRAY's dtype: an
int16 capture with |x[0]| or |x[-1]| above 16383 wraps, uint8 wraps below zero
and above 255, float16 rounds to half (and overflows to inf).  These fixtures
are the REFERENCE's own modem.qpsk_demodulate / bpsk_demodulate /
fsk_demodulate on such arrays.  Committed data only:

  tests/golden/rawint.npz            the inputs, in their own dtype, key r<i>
  tests/golden/rawint_manifest.json  per case: function, parameters, the
                                     reference's bytes (hex) or exception, and
                                     whether they differ from the reference's
                                     bytes on the same values as float64
                                     (i.e. whether the wrap decides the output)

tests/test_oracle_golden.py pins the oracle's raw dtypes to these on the CPU;
tests/test_gpu_rawint.py runs them through the drop-in in every layout.

Run:  python tests/golden/make_rawint_golden.py   (needs /root/reference)
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (the reference import helpers; its main() is not run)
import synth  # noqa: E402

# (function, baud, f0, f1, n, dtype, edge): edge names how the capture's end
# samples sit -- "left" x[0] near full scale, "right" x[-1], "both", "dc" a
# full-scale DC offset (uint8's mid-scale 128, int16's +20000), "none" as drawn
CASES = [
    ("qpsk", 9600, 3000.0, 0.0, 96000, "int16", "left"),
    ("qpsk", 9600, 3000.0, 0.0, 48000, "int16", "right"),
    ("qpsk", 1200, 3000.0, 0.0, 48000, "int16", "both"),
    ("qpsk", 2400, 6000.0, 0.0, 30011, "int16", "dc"),
    ("bpsk", 1200, 3000.0, 0.0, 48000, "int16", "left"),
    ("bpsk", 2400, 3000.0, 0.0, 24000, "int16", "both"),
    ("fsk", 9600, 12000.0, 24000.0, 96000, "int16", "left"),
    ("fsk", 9600, 12000.0, 24000.0, 48000, "int16", "right"),
    ("fsk", 1200, 2400.0, 4800.0, 48000, "int16", "both"),
    ("fsk", 2400, 6000.0, 9000.0, 30011, "int16", "dc"),
    ("qpsk", 9600, 3000.0, 0.0, 48000, "uint8", "dc"),
    ("bpsk", 1200, 3000.0, 0.0, 24000, "uint8", "dc"),
    ("fsk", 9600, 12000.0, 24000.0, 48000, "uint8", "dc"),
    ("fsk", 1200, 2400.0, 4800.0, 24000, "uint8", "left"),
    ("qpsk", 4800, 12000.0, 0.0, 24000, "int8", "both"),
    ("fsk", 4800, 12000.0, 18000.0, 24000, "int8", "left"),
    ("qpsk", 9600, 3000.0, 0.0, 48000, "int32", "left"),
    ("fsk", 9600, 12000.0, 24000.0, 24000, "int32", "both"),
    ("bpsk", 2400, 3000.0, 0.0, 24000, "uint16", "dc"),
    ("qpsk", 2400, 3000.0, 0.0, 24000, "int64", "left"),
    ("fsk", 2400, 6000.0, 12000.0, 24000, "int64", "right"),
    ("bpsk", 1200, 3000.0, 0.0, 24000, "bool", "none"),
    ("qpsk", 9600, 3000.0, 0.0, 24000, "float16", "left"),
    ("fsk", 9600, 12000.0, 24000.0, 24000, "float16", "both"),
]

SCALE = {"int8": 127, "uint8": 127, "int16": 32767, "uint16": 32767, "int32": 2 ** 31 - 1,
         "int64": 2 ** 62, "bool": 1, "float16": 60000.0}


def make(rng, fn, baud, f0, f1, n, dt, edge):
    fr = synth.random_frame(rng, int(rng.integers(8, 200)))
    fs = 96000.0
    if fn == "qpsk":
        w = synth.qpsk_waveform(fr, baud, f0, fs)
    elif fn == "bpsk":
        w = synth.bpsk_waveform(fr, baud, f0, fs)
    else:
        w = synth.fsk_waveform(fr, baud, f0, f1, fs)
    off = int(rng.integers(0, n // 8))
    x = np.zeros(n)
    seg = w[:max(0, n - off)]
    x[off:off + seg.size] = seg
    x = np.clip(0.97 * x + rng.normal(0, 0.02, n), -1, 1)
    if edge in ("left", "both"):
        x[0] = float(rng.choice([0.9765, -0.9765, 0.7]))           # a click: |x[0]| > half scale
    if edge in ("right", "both"):
        x[-1] = float(rng.choice([0.9765, -0.9765, -0.6]))
    if dt == "bool":
        return x > 0
    if dt == "float16":
        return (x * SCALE[dt]).astype(np.float16)
    info = np.iinfo(dt)
    if edge == "dc":                                               # a capture that sits off zero
        mid = 128 if dt == "uint8" else 32768 if dt == "uint16" else 20000
        v = np.round(mid + x * (SCALE[dt] if info.min < 0 else min(SCALE[dt], mid - 1) * 0.9))
    elif info.min == 0:                                            # unsigned without an offset: |x|
        v = np.round(np.abs(x) * SCALE[dt])
    else:
        v = np.round(x * float(SCALE[dt]))
    return np.clip(v, info.min, info.max).astype(dt)


def main():
    rng = np.random.default_rng(20261020)
    draws = [(c, make(rng, *c)) for c in CASES]
    scratch = tempfile.mkdtemp(prefix="amr_rawint_golden_")
    cwd = os.getcwd()
    try:
        modem, _, _ = mg._import_reference(scratch)
        cases, arrays = [], {}
        for i, ((fn, baud, f0, f1, n, dt, edge), x) in enumerate(draws):
            def run(arr):
                if fn == "qpsk":
                    return mg._run(modem.qpsk_demodulate, arr, baud=baud, carrier=f0)
                if fn == "bpsk":
                    return mg._run(modem.bpsk_demodulate, arr, baud=baud, carrier=f0)
                return mg._run(modem.fsk_demodulate, arr, baud=baud, mark_freq=f0, space_freq=f1)
            with np.errstate(all="ignore"):
                res = run(x)                                       # the raw array, as the reference's callers pass it
                as_f64 = run(x.astype(np.float64))                 # the same values as float64: no wrap
            arrays[f"r{i}"] = x
            cases.append(dict(id=f"r{i}", fn=fn, params=dict(baud=baud, f0=f0, f1=f1, samp_rate=96000.0, edge=edge),
                              dtype=str(x.dtype), n=int(x.size), differs_from_float64=res != as_f64, **res))
    finally:
        os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "rawint.npz"), **arrays)
    with open(os.path.join(HERE, "rawint_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_rawint_golden.py", "numpy": np.__version__,
                   "numpy_cpu_features": mg.numpy_cpu_features(), "cases": cases}, f, indent=1)
    ok = sum(c["status"] == "ok" for c in cases)
    dif = sum(c["differs_from_float64"] for c in cases)
    print(f"{len(cases)} cases ({ok} ok, {len(cases) - ok} raise), {dif} whose bytes the dtype's wrap decides")


if __name__ == "__main__":
    main()
