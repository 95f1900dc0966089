#!/usr/bin/env python3
"""Transmit-side benchmark: batched modulators on one GPU.

    python tools/bench_tx.py [--kind qpsk|bpsk|fsk] [--batch 4096] [--steps 10] [--warmup 2]

A step = amr_modulate_device over B payloads already resident in HBM, writing
B x 96 000 float32 samples + the WAV's int16 samples (the reference's
modulate + wav_from_array, modem.py:28-65/138-186/270-295/360-368).  The
payload size makes each natural waveform exactly 1 s at 96 kHz (QPSK@9600:
40 + 4n symbols of 10 samples).  Prints one JSON line like bench.py, with
the CPU baseline = the host numpy synthesiser (synth.py, pinned to the
reference's tx fixtures) on a sample of the streams.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem-radio_amd"))
import _amr  # noqa: E402
import synth  # noqa: E402

HBM_PEAK_GBS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kind", choices=["qpsk", "bpsk", "fsk"], default="qpsk")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--cpu-streams", type=int, default=64)
    ap.add_argument("--no-pcm", action="store_true")
    args = ap.parse_args()
    B, N, baud = args.batch, 96000, 9600.0
    mode = _amr.TX_MODES[args.kind]
    f0, f1 = (12000.0, 24000.0) if args.kind == "fsk" else (3000.0, 0.0)
    # payload bytes for a 1-s waveform: QPSK (40+4n)*10, BPSK (80+8n)*10, FSK 8*(4+n)*10
    nb = {"qpsk": (N // 10 - 40) // 4, "bpsk": (N // 10 - 80) // 8, "fsk": N // 80 - 4}[args.kind]
    rng = np.random.default_rng(7)
    data = rng.integers(0, 256, (B, nb), dtype=np.uint8)
    lens = np.full(B, nb, np.int64)
    assert _amr.tx_samples(mode, nb, baud, 96000) == N
    L = _amr.lib()
    _amr.check(L.amr_set_device(0))

    def dmalloc(n):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), int(n)))
        return p

    wb = L.amr_tx_work_bytes(mode, baud, 96000.0, B, N)
    d_data, d_len, d_out, d_work = dmalloc(data.nbytes), dmalloc(B * 8), dmalloc(B * N * 4), dmalloc(wb)
    d_pcm = None if args.no_pcm else dmalloc(B * N * 2)
    _amr.check(L.amr_memcpy_h2d(d_data, _amr.ptr(data), data.nbytes))
    _amr.check(L.amr_memcpy_h2d(d_len, _amr.ptr(lens), B * 8))

    def step():
        _amr.check(L.amr_modulate_device(None, mode, baud, f0, f1, 96000.0, d_data, nb, d_len, B, d_out, N, N,
                                         d_pcm, N, d_work, wb))

    for _ in range(args.warmup):
        step()
    _amr.check(L.amr_device_synchronize())
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    _amr.check(L.amr_device_synchronize())
    dt = (time.perf_counter() - t0) / args.steps
    value = B * N / dt / 1e6

    # spot parity (untimed) against the host synthesiser, and the CPU baseline
    out = np.empty((B, N), np.float32)
    _amr.check(L.amr_memcpy_d2h(_amr.ptr(out), d_out, out.nbytes))
    wave = {"qpsk": lambda x: synth.qpsk_waveform(x, baud, f0), "bpsk": lambda x: synth.bpsk_waveform(x, baud, f0),
            "fsk": lambda x: synth.fsk_waveform(x, baud, f0, f1)}[args.kind]
    idx = np.linspace(0, B - 1, num=min(args.cpu_streams, B)).astype(int)
    t1 = time.perf_counter()
    ref = [wave(data[i].tobytes()) for i in idx]
    cdt = time.perf_counter() - t1
    diff = sum(int(np.count_nonzero(out[i] != r)) for i, r in zip(idx, ref))
    bytes_per_sample = 4 + (0 if args.no_pcm else 2)
    sym = N // 10
    alg = B * (N * bytes_per_sample + sym * 8 + nb)     # output + the phase table read + the payload
    print(json.dumps({
        "metric": f"{args.kind.upper()}@9600 modulate Msamples/s (batch, float32 + int16 WAV samples)",
        "value": round(value, 1), "unit": "Msamples/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(dt * 1e3, 4), "higher_is_better": True, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"{args.kind} modulate, {B} payloads of {nb} B -> {B} x {N} samples"},
        "roofline": {"bound": "hbm", "achieved_step": round(alg / dt / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac_step": round(alg / dt / 1e9 / HBM_PEAK_GBS, 4)},
        "cpu_baseline": {"value": round(len(idx) * N / cdt / 1e6, 2), "unit": "Msamples/s", "cores": 1,
                         "kind": "port", "sample": f"{len(idx)} streams through synth.py (numpy), {cdt:.2f} s"},
        "parity": f"{diff} float32 samples differ from the host synthesiser over {len(idx)} streams",
    }))


if __name__ == "__main__":
    main()
