#!/usr/bin/env python3
"""Reference outputs over a seeded draw of demod configurations (this
container only): the REFERENCE's own modem.qpsk_demodulate / bpsk_demodulate
/ fsk_demodulate (modem.py:189-266, 68-135, 298-341) on inputs drawn across
the parameter space their signatures accept -- baud, carrier / tones, sample
rate, length, input dtype, signal level, leading silence (PSK), noise.
Committed data only:

  tests/golden/sweep.npz            the inputs (their own dtype), key c<i>
  tests/golden/sweep_manifest.json  per case: function, parameters, and the
                                    reference's bytes (hex) or exception

tests/test_oracle_golden.py pins the oracle to these on the CPU;
tests/test_gpu_sweep.py checks the GPU against them.  FSK inputs keep a
noise floor, and 12 extra FSK cases sit between stretches of exact digital
silence at 5-smooth lengths (params.silence): there only pocketfft's own
rounding decides.  Round 4 appends 16 more (their own
seed, so the first 84 cases are unchanged) at lengths with a prime factor
above 5 -- Bluestein and generic-radix plans in pocketfft -- with digital
silence, a DC (constant) stretch or a stretch 1e-17 below the signal
(params.quiet).  Round 5 appends 7 long captures (params.long, their own
seed): 10-s (960 000 samples, what decode_wav_file makes of a 10-s WAV) and
20-s streams and the non-5-smooth long lengths 441 000 and 400 001, signal
between digital silence, DC or 1e-17 stretches.  The oracle and the GPU
(through its exact path) must match all of them.

Run:  python tests/golden/make_sweep_golden.py   (needs /root/reference)
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

N_CASES = 72


def draw(rng, c):
    kind = ["qpsk", "bpsk", "fsk"][c % 3]
    fs = float(rng.choice([96000, 96000, 48000, 44100]))
    n = int(rng.choice([int(rng.integers(28, 600)), int(rng.integers(600, 8000)), int(rng.integers(8000, 24000))]))
    if kind == "fsk":
        baud = int(rng.choice([300, 600, 1200, 2400, 4800, 9600]))
        nyq = fs / 2
        lo, hi = baud * 1.1, nyq - baud * 1.1
        if rng.random() < 0.15 or hi <= lo:
            f0, f1 = 1200.0, 2200.0                      # the reference's defaults (raise above ~1000 Bd)
        else:
            f0, f1 = sorted(round(float(v), 3) for v in rng.uniform(lo, hi, 2))
    else:
        baud = int(rng.choice([300, 600, 1000, 1200, 1500, 2400, 3000, 4800, 9600, 19200]))
        f0, f1 = float(rng.choice([3000.0, 3000.0, 1800.0, 6000.0, 12000.0])), 0.0
    noise = float(rng.choice([0.0, 0.02, 0.1, 0.4])) if kind != "fsk" else float(rng.choice([0.02, 0.1, 0.4]))
    if rng.random() < 0.1:
        x = rng.normal(0, 0.5, n)
    else:
        fr = synth.random_frame(rng, int(rng.integers(4, 48)))
        try:
            if kind == "qpsk":
                w = synth.qpsk_waveform(fr, baud, f0, fs)
            elif kind == "bpsk":
                w = synth.bpsk_waveform(fr, baud, f0, fs)
            else:
                w = synth.fsk_waveform(fr, baud, f0, f1, fs)
        except ValueError:                               # the PSK modulators raise below 10 samples per symbol
            w = rng.normal(0, 0.5, n)
        off = int(rng.integers(0, max(1, n // 4))) if kind != "fsk" else 0
        x = np.zeros(n)
        seg = w[:max(0, n - off)]
        x[off:off + seg.size] = seg * float(rng.choice([1.0, 0.3, 0.01]))
        x = x + rng.normal(0, noise, n) * (float(np.abs(x).max()) if np.abs(x).max() > 0 else 1.0)
    dt = str(rng.choice(["float32", "float64", "int16"]))
    if dt == "int16":
        x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16)
    else:
        x = x.astype(dt)
    return kind, dict(baud=baud, f0=f0, f1=f1, samp_rate=fs), x


N_SILENCE = 12


def draw_silence(rng):
    """FSK between stretches of exact digital silence, no noise: the inputs on
    which only pocketfft's own rounding decides."""
    fs = 96000.0
    baud = int(rng.choice([1200, 2400, 4800, 9600]))
    f0, f1 = sorted(round(float(v), 3) for v in rng.uniform(baud * 1.1, fs / 2 - baud * 1.1, 2))
    n = int(rng.choice([9600, 19200, 24000, 30000]))
    fr = synth.random_frame(rng, int(rng.integers(4, 24)))
    w = synth.fsk_waveform(fr, baud, f0, f1, fs)
    off = int(rng.integers(n // 8, n // 3))
    x = np.zeros(n)
    seg = w[:max(0, n - off)]
    x[off:off + seg.size] = seg
    dt = str(rng.choice(["float32", "float64", "int16"]))
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dt == "int16" else x.astype(dt)
    return "fsk", dict(baud=baud, f0=f0, f1=f1, samp_rate=fs, silence=True), x


N_QUIET = 16
QUIET_LENGTHS = [24001, 30011, 77880, 9601, 19207, 12347, 96001, 29999, 14007, 50021, 21001, 7919, 33033, 47999,
                 96017, 11011]


def draw_quiet(rng, i):
    """FSK at a length with a prime factor above 5, next to a stretch whose
    envelopes sink to rounding level: exact digital silence, a DC offset
    (butter(3, band) cancels constants) or a stretch 1e-17 below the signal."""
    fs = 96000.0
    baud = int(rng.choice([1200, 2400, 4800, 9600]))
    f0, f1 = sorted(round(float(v), 3) for v in rng.uniform(baud * 1.1, fs / 2 - baud * 1.1, 2))
    n = QUIET_LENGTHS[i]
    quiet = ["silence", "dc", "tiny", "silence"][i % 4]
    fr = synth.random_frame(rng, int(rng.integers(4, 24)))
    w = synth.fsk_waveform(fr, baud, f0, f1, fs)
    off = int(rng.integers(n // 8, n // 3))
    x = np.zeros(n)
    seg = w[:max(0, n - off)]
    x[off:off + seg.size] = seg
    if quiet == "dc":
        x[:off] = float(rng.choice([0.25, -3.0 / 32768, 1e-3]))
    elif quiet == "tiny":
        x[:off] = rng.normal(0, 1e-17, off)
    dt = str(rng.choice(["float32", "float64", "int16"])) if quiet != "tiny" else "float64"
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dt == "int16" else x.astype(dt)
    return "fsk", dict(baud=baud, f0=f0, f1=f1, samp_rate=fs, silence=True, quiet=quiet), x


# Round 5: long captures -- decode_wav_file makes a 10-s
# recording 960 000 samples (decoder.py:385-387), past the fast path's
# two-pass limit (six-step FFTs), and a non-5-smooth long length runs
# Bluestein over a six-step convolution.  Signal between quiet stretches
# (digital silence, a DC lead-in, a 1e-17 stretch) at valid tones: these
# pin the margin premise (F2's tau) where the fast FFT has the most rounding
# stages.  (n, baud, quiet, dtype); tones drawn like draw_quiet's.
LONG_CASES = [(960000, 9600, "silence", "int16"), (960000, 1200, "dc", "float32"),
              (960000, 4800, "tiny", "float32"), (960000, 2400, "silence", "float64"),
              (441000, 2400, "silence", "int16"), (400001, 9600, "dc", "float32"),
              (1920000, 1200, "silence", "int16")]


def draw_long(rng, i):
    fs = 96000.0
    n, baud, quiet, dt = LONG_CASES[i]
    f0, f1 = sorted(round(float(v), 3) for v in rng.uniform(baud * 1.1, fs / 2 - baud * 1.1, 2))
    if i == 0:
        f0, f1 = 12000.0, 24000.0                        # the benchmark's tones
    fr = synth.random_frame(rng, int(rng.integers(200, 1200)))
    w = synth.fsk_waveform(fr, baud, f0, f1, fs)
    off = int(rng.integers(n // 5, n // 2))              # seconds of quiet before the frame
    x = np.zeros(n)
    seg = w[:max(0, n - off)]
    x[off:off + seg.size] = seg
    if quiet == "dc":
        x[:off] = float(rng.choice([0.25, -3.0 / 32768, 1e-3]))
    elif quiet == "tiny":
        x[:off] = rng.normal(0, 1e-17, off)
    if i == 3:
        g = off + seg.size // 2                          # and a gap of digital silence inside the frame
        x[g:g + 5000] = 0.0
    x = np.round(np.clip(x, -1, 1) * 32767).astype(np.int16) if dt == "int16" else x.astype(dt)
    return "fsk", dict(baud=baud, f0=f0, f1=f1, samp_rate=fs, silence=True, quiet=quiet, long=True), x


def main():
    rng = np.random.default_rng(20261017)
    draws = [draw(rng, c) for c in range(N_CASES)]
    draws += [draw_silence(rng) for _ in range(N_SILENCE)]
    rng_q = np.random.default_rng(20261018)
    draws += [draw_quiet(rng_q, i) for i in range(N_QUIET)]
    rng_l = np.random.default_rng(20261019)
    draws += [draw_long(rng_l, i) for i in range(len(LONG_CASES))]
    scratch = tempfile.mkdtemp(prefix="amr_sweep_golden_")
    cwd = os.getcwd()
    try:
        modem, _, _ = mg._import_reference(scratch)
        cases, arrays = [], {}
        for c, (kind, p, x) in enumerate(draws):
            # the reference reads int16 WAV samples as int16 / 32768 (soundfile, decoder.py:383)
            xr = x.astype(np.float64) / 32768.0 if x.dtype == np.int16 else x
            if kind == "qpsk":
                res = mg._run(modem.qpsk_demodulate, xr, baud=p["baud"], carrier=p["f0"], samp_rate=p["samp_rate"])
            elif kind == "bpsk":
                res = mg._run(modem.bpsk_demodulate, xr, baud=p["baud"], carrier=p["f0"], samp_rate=p["samp_rate"])
            else:
                res = mg._run(modem.fsk_demodulate, xr, baud=p["baud"], mark_freq=p["f0"], space_freq=p["f1"],
                              samp_rate=p["samp_rate"])
            arrays[f"c{c}"] = x
            cases.append(dict(id=f"c{c}", fn=kind, params=p, dtype=str(x.dtype), n=int(x.size), **res))
    finally:
        os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "sweep.npz"), **arrays)
    with open(os.path.join(HERE, "sweep_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_sweep_golden.py", "numpy": np.__version__,
                   "numpy_cpu_features": mg.numpy_cpu_features(), "cases": cases}, f, indent=1)
    ok = sum(c["status"] == "ok" for c in cases)
    print(f"{len(cases)} cases ({ok} ok, {len(cases) - ok} raise)")


if __name__ == "__main__":
    main()
