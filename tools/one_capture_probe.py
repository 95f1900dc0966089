"""Where one capture's time goes: modem.qpsk_demodulate / modem.fsk_demodulate
on one 96000-sample stream (the time-split layouts),
wall time per call and, under rocprofv3 --kernel-trace, the kernels' own
durations (their sum against the wall time is the host side's share).
    rocprofv3 --kernel-trace --stats -d gpurun_out/oc -o run --output-format csv -- python3 tools/one_capture_probe.py
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-modem-radio_amd"), ROOT]
import modem  # noqa: E402
import synth  # noqa: E402

K = int(os.environ.get("K", "20"))
xq = synth.qpsk_batch(8, 96000, 9600, seed=3, distinct=8, noise=0.05)
xf = synth.fsk_batch(8, 96000, 9600, 12000.0, 24000.0, seed=3, distinct=8, noise=0.05)
for name, fn, x in (("qpsk", lambda v: modem.qpsk_demodulate(v, baud=9600), xq),
                    ("fsk", lambda v: modem.fsk_demodulate(v, baud=9600, mark_freq=12000.0, space_freq=24000.0), xf)):
    fn(x[0])
    ts = []
    for i in range(K):
        t0 = time.perf_counter()
        fn(x[i % 8])
        ts.append(time.perf_counter() - t0)
    print(f"{name}: {K} calls, wall median {np.median(ts) * 1e3:.3f} ms, min {min(ts) * 1e3:.3f} ms", flush=True)

# FSK batches: the split F1 (AUTO) against the serial F1, host entry, cached plans
if os.environ.get("FSK_BATCHES"):
    import _fsk
    for B in [int(v) for v in os.environ["FSK_BATCHES"].split(",")]:
        xb = synth.fsk_batch(B, 96000, 9600, 12000.0, 24000.0, seed=B, distinct=min(B, 64), noise=0.05)
        row = {}
        for layout in ("auto", "serial"):
            pl = _fsk.FskPlan(96000, 9600, 12000.0, 24000.0, max_streams=B)
            pl.set_layout(layout)
            ref = pl.demod_host(xb)[0]
            ts = []
            for _ in range(3):
                t0 = time.perf_counter()
                got = pl.demod_host(xb)[0]
                ts.append(time.perf_counter() - t0)
            assert got == ref
            row[layout] = (round(min(ts) * 1e3, 3), pl.split_info()["last_split"], pl.exact_streams())
            del pl
        print(f"fsk batch B={B}: auto {row['auto']} serial {row['serial']}", flush=True)
