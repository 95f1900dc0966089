"""Where one capture's time goes: modem.qpsk_demodulate on one 96000-sample
stream, per-kernel HIP-event times of its plan (row layout) and the wall time."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-modem-radio_amd"), ROOT]
import _amr  # noqa: E402
import synth  # noqa: E402

x = synth.qpsk_batch(1, 96000, 9600, seed=3)
for B in (1, 64, 4096):
    xb = np.repeat(x, B, axis=0) if B > 1 else x
    pl = _amr.PskPlan("qpsk", 96000, 9600, max_streams=B, device=0)
    pl.enable_timing(True)
    pl.demod_host(xb)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        pl.demod_host(xb)
        ts.append(time.perf_counter() - t0)
    print(f"B={B} wall {np.median(ts) * 1e3:.3f} ms layout {pl.last_layout()} kernels "
          f"{ {k: round(v, 3) for k, v in pl.timings().items() if v > 0} }", flush=True)
