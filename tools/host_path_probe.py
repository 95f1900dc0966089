"""Where the FSK host-API time goes (run on the GPU box): amr_fsk_demod_host
vs amr_memcpy_h2d + amr_fsk_demod_device on the same batch."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", "audio-modem-radio_amd"))
import _amr  # noqa: E402
import _fsk  # noqa: E402
import synth  # noqa: E402

B, N = int(sys.argv[1]) if len(sys.argv) > 1 else 16384, 96000
L = _amr.lib()
x = synth.fsk_batch(B, N, 9600, 12000.0, 24000.0, seed=3, distinct=64)
print("x", x.dtype, x.flags["C_CONTIGUOUS"], x.nbytes / 1e9, flush=True)
pl = _fsk.FskPlan(N, 9600, 12000.0, 24000.0, 96000, max_streams=B, device=0)
cap = pl.out_cap
out = np.empty((B, cap), np.uint8)
ln = np.empty(B, np.int64)
sy = np.empty(B, np.int64)
for i in range(3):
    t0 = time.perf_counter()
    _amr.check(L.amr_fsk_demod_host(pl.handle, _amr.ptr(x), _amr.DTYPE_F32, B, N, _amr.ptr(out), cap, _amr.ptr(ln),
                                    _amr.ptr(sy)))
    print(f"host call {i}: {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)


def dmalloc(n):
    p = ctypes.c_void_p()
    _amr.check(L.amr_malloc(ctypes.byref(p), int(n)))
    return p


dx, do, dl, ds = dmalloc(x.nbytes), dmalloc(B * cap), dmalloc(B * 8), dmalloc(B * 8)
for i in range(3):
    t0 = time.perf_counter()
    _amr.check(L.amr_memcpy_h2d(dx, _amr.ptr(x), x.nbytes))
    t1 = time.perf_counter()
    _amr.check(L.amr_fsk_demod_device(pl.handle, dx, _amr.DTYPE_F32, B, N, do, cap, dl, ds))
    _amr.check(L.amr_fsk_plan_synchronize(pl.handle))
    t2 = time.perf_counter()
    print(f"split {i}: h2d {(t1 - t0) * 1e3:.1f} ms, device demod {(t2 - t1) * 1e3:.1f} ms", flush=True)
