"""PSK time-split layout: demod_host wall time per call at batches of 1-64
96000-sample QPSK@9600 captures (plan forced to the split layout).  A/B knobs:
AMR_PSK_SPLIT_CONV, AMR_PSK_SPLIT_MINL (api.cpp split_params)."""
import os, sys, time, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-modem-radio_amd"), ROOT]
import _amr, synth
x = synth.qpsk_batch(64, 96000, 9600, seed=5, distinct=64, noise=0.05)
out = []
for B in (1, 4, 8, 16, 32, 64):
    pl = _amr.PskPlan("qpsk", 96000, 9600, 3000.0, 96000, max_streams=64)
    pl.set_layout("split")
    pl.demod_host(x[:B])
    pl.enable_timing(True)
    pl.demod_host(x[:B])
    bp = pl.timings().get("bandpass", float("nan"))
    pl.enable_timing(False)
    ts = []
    for i in range(10):
        t0 = time.perf_counter(); pl.demod_host(x[:B]); ts.append(time.perf_counter() - t0)
    out.append(f"B={B}: {np.median(ts)*1e3:.3f} ms (band-pass passes {bp:.3f} ms, L {pl.split_info()['chunk']}, flagged {pl.split_info()['flagged']})")
print("\n".join(out), flush=True)
