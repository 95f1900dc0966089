"""Timing-only ablations of the low-pass forward kernel (AMR_K2_VARIANT); results are wrong by design."""
import os, sys, ctypes
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-modem-radio_amd"), ROOT]
import numpy as np, _amr, synth
B, N = 4096, 96000
x = synth.qpsk_batch(B, N, 9600, seed=1, distinct=16)
L = _amr.lib()
plan = _amr.PskPlan("qpsk", N, 9600, max_streams=B)
plan.enable_timing(True)
cap = plan.out_cap
def dm(nb):
    p = ctypes.c_void_p(); _amr.check(L.amr_malloc(ctypes.byref(p), nb)); return p
dx, do, dl, ds = dm(x.nbytes), dm(B * cap), dm(B * 8), dm(B * 8)
_amr.check(L.amr_memcpy_h2d(dx, _amr.ptr(x), x.nbytes))
for var in ["0", "12", "14", "18", "1", "0"]:
    os.environ["AMR_K2_VARIANT"] = var
    ts = []
    for it in range(4):
        _amr.check(L.amr_psk_demod_device(plan.handle, dx, 0, B, N, do, cap, dl, ds))
        t = plan.timings()
        if it: ts.append(t["lowpass_fwd"])
    print(f"variant {var}: lowpass_fwd {np.mean(ts):.3f} ms  (bandpass {t['bandpass']:.3f}, lowpass_bwd {t['lowpass_bwd']:.3f})", flush=True)
