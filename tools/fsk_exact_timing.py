#!/usr/bin/env python3
"""How long the FSK exact fallback takes when every stream is flagged
(zero-padded captures), against the same batch with a
noise floor (nothing flagged).  GPU box:  python tools/fsk_exact_timing.py"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "audio-modem-radio_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
import _fsk  # noqa: E402
import synth  # noqa: E402


def batch(B, n, noise, seed=5):
    rng = np.random.default_rng(seed)
    rows = []
    for i in range(B):
        w = synth.fsk_waveform(synth.random_frame(rng, 40), 9600, 12000.0, 24000.0, 96000.0)
        off = 2000 + 37 * i
        row = np.zeros(n)
        seg = w[:n - off]
        row[off:off + seg.size] = seg
        rows.append(row)
    x = np.stack(rows)
    if noise:
        x = x + rng.normal(0, noise, x.shape)
    return x.astype(np.float32)


def main():
    n = 96000
    for B in (16, 128, 512, 2048):
        pl = _fsk.FskPlan(n, 9600, 12000.0, 24000.0, max_streams=B)
        for label, noise in (("silent-padded", 0.0), ("noise floor", 0.01)):
            x = batch(B, n, noise)
            pl.demod_host(x)                       # warm
            t = time.perf_counter()
            for _ in range(3):
                pl.demod_host(x)
            ms = (time.perf_counter() - t) / 3 * 1e3
            print(f"B={B:4d} {label:14s} {ms:9.2f} ms per batch (host entry, incl. copies)", flush=True)


if __name__ == "__main__":
    main()
