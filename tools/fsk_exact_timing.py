#!/usr/bin/env python3
"""How long the FSK exact path takes: zero-padded captures (F2 flags the
streams whose compares fall inside the margin), every
stream forced through it (exact mode 2), against the same batch with a noise
floor (nothing flagged).  GPU box:  python tools/fsk_exact_timing.py [B ...]
(`burst`: the first all-flagged batch after 0 / 1 / 8 / 20 clean ones)"""
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
    sizes = [int(v) for v in sys.argv[1:]] or [1, 16, 128, 512, 2048]
    for B in sizes:
        pl = _fsk.FskPlan(n, 9600, 12000.0, 24000.0, max_streams=B)
        pl.enable_timing(True)
        for label, noise, mode in (("silent-padded", 0.0, 1), ("all exact", 0.0, 2), ("noise floor", 0.01, 1)):
            x = batch(B, n, noise)
            pl.set_exact_mode(mode)
            pl.demod_host(x)                       # warm
            t = time.perf_counter()
            for _ in range(3):
                pl.demod_host(x)
            ms = (time.perf_counter() - t) / 3 * 1e3
            tm = pl.timings()
            print(f"B={B:4d} {label:14s} {ms:9.2f} ms per batch (host entry, incl. copies); flagged "
                  f"{pl.exact_streams():4d}; exact stage {tm.get('exact', -1):8.2f} ms, launch {tm.get('launch', -1):8.2f} ms",
                  flush=True)


def burst(B=2048, clean_runs=(0, 1, 8, 20)):
    """E2's grid follows the counts of the plan's last 8 launches.
    A fresh plan per row: `c` clean (noise-floor) batches, then one
    silent-padded batch whose every stream is flagged, with no warm-up of that
    input -- the first flagged batch after a run of clean ones."""
    n = 96000
    noisy, silent = batch(B, n, 0.01), batch(B, n, 0.0)
    for c in clean_runs:
        pl = _fsk.FskPlan(n, 9600, 12000.0, 24000.0, max_streams=B)
        pl.enable_timing(True)
        for _ in range(c):
            pl.demod_host(noisy)
        t = time.perf_counter()
        pl.demod_host(silent)
        ms = (time.perf_counter() - t) * 1e3
        tm = pl.timings()
        print(f"B={B} after {c:2d} clean batches: all-flagged batch {ms:9.2f} ms (host entry); flagged "
              f"{pl.exact_streams():4d}; exact stage {tm.get('exact', -1):8.2f} ms", flush=True)
        del pl


if __name__ == "__main__":
    if sys.argv[1:2] == ["burst"]:
        burst()
    else:
        main()
