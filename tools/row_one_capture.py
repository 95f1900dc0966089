"""One 96000-sample QPSK@9600 capture through a chosen layout, 20 calls (for
rocprofv3 --kernel-trace --stats: the per-kernel split).  argv: layout (row |
split | lane) [strict]: the serial row layout is a flagged capture's fallback;
"split strict" runs the time-split layout with the strict margin."""
import os
import sys
import time

import numpy as np
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "audio-modem-radio_amd"), root]
import _amr  # noqa: E402
import synth  # noqa: E402

x = synth.qpsk_batch(1, 96000, 9600, seed=3, distinct=1)
pl = _amr.PskPlan("qpsk", 96000, 9600, max_streams=1)
pl.set_layout(sys.argv[1] if len(sys.argv) > 1 else "row")
if len(sys.argv) > 2 and sys.argv[2] == "strict":
    pl.set_split_strict(True)
pl.demod_host(x)
ts = []
for _ in range(20):
    t = time.perf_counter()
    pl.demod_host(x)
    ts.append(time.perf_counter() - t)
print(pl.last_layout(), "strict" if pl.last_strict() else "", "median ms", round(float(np.median(ts)) * 1e3, 3))
