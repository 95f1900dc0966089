#!/usr/bin/env python3
"""Throughput with 1 vs 2 batches in flight (two PSK plans = two HIP streams):
does batch k+1's band-pass overlap batch k's low-pass passes?
    python tools/overlap_probe.py [--workload qpsk|fsk]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "audio-modem-radio_amd"))
import _amr  # noqa: E402
import synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="qpsk")
ap.add_argument("--steps", type=int, default=8)
a = ap.parse_args()
L = _amr.lib()
_amr.check(L.amr_set_device(0))
N = 96000
if a.workload == "qpsk":
    B = 4096
    x = synth.qpsk_batch(B, N, 9600, seed=1, distinct=16)
    mk = lambda: _amr.PskPlan("qpsk", N, 9600, 3000.0, 96000, max_streams=B, device=0)  # noqa: E731
    demod, sync = L.amr_psk_demod_device, L.amr_psk_plan_synchronize
else:
    import _fsk
    B = 16384
    x = synth.fsk_batch(B, N, 9600, 12000.0, 24000.0, seed=1, distinct=16)
    mk = lambda: _fsk.FskPlan(N, 9600, 12000.0, 24000.0, 96000, max_streams=B, device=0)  # noqa: E731
    demod, sync = L.amr_fsk_demod_device, L.amr_fsk_plan_synchronize


def dmalloc(n):
    p = ctypes.c_void_p()
    _amr.check(L.amr_malloc(ctypes.byref(p), int(n)))
    return p


d_x = dmalloc(x.nbytes)
_amr.check(L.amr_memcpy_h2d(d_x, _amr.ptr(x), x.nbytes))
plans = [mk(), mk()]
cap = plans[0].out_cap
outs = [(dmalloc(B * cap), dmalloc(B * 8), dmalloc(B * 8)) for _ in plans]
for inflight in (1, 2, 1, 2):
    for k in range(2):
        for i in range(inflight):
            _amr.check(demod(plans[i].handle, d_x, _amr.DTYPE_F32, B, N, *outs[i][:1], cap, *outs[i][1:]))
    _amr.check(L.amr_device_synchronize())
    t0 = time.perf_counter()
    for k in range(a.steps):
        i = k % inflight
        _amr.check(demod(plans[i].handle, d_x, _amr.DTYPE_F32, B, N, *outs[i][:1], cap, *outs[i][1:]))
        if inflight == 1:
            _amr.check(sync(plans[i].handle))
    _amr.check(L.amr_device_synchronize())
    dt = (time.perf_counter() - t0) / a.steps
    print(f"{a.workload} inflight={inflight}: {dt * 1e3:.2f} ms/step", flush=True)
o = np.empty((2, B, cap), np.uint8)
for i in range(2):
    _amr.check(L.amr_memcpy_d2h(_amr.ptr(o[i]), outs[i][0], B * cap))
print("outputs of the two plans equal:", bool(np.array_equal(o[0], o[1])))
