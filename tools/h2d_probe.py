"""H2D bandwidth from pageable numpy memory through libamr's amr_memcpy_h2d,
by transfer size and by chunking (host-path tuning probe; run on the GPU box)."""
import ctypes
import sys
import time

import numpy as np

sys.path.insert(0, __import__("os").path.join(__import__("os").path.dirname(__import__("os").path.abspath(__file__)), "..", "audio-modem-radio_amd"))
import _amr  # noqa: E402

L = _amr.lib()
_amr.check(L.amr_set_device(0))
p = ctypes.c_void_p()
_amr.check(L.amr_malloc(ctypes.byref(p), 6_400_000_000))
for gb in (0.4, 1.6, 3.2, 6.3):
    x = np.ones(int(gb * 1e9) // 4, np.float32)
    for chunk in (0, 256 << 20, 1 << 30):
        ts = []
        for _ in range(3):
            t0 = time.perf_counter()
            if chunk == 0:
                _amr.check(L.amr_memcpy_h2d(p, _amr.ptr(x), x.nbytes))
            else:
                base = x.ctypes.data
                for o in range(0, x.nbytes, chunk):
                    n = min(chunk, x.nbytes - o)
                    _amr.check(L.amr_memcpy_h2d(ctypes.c_void_p(p.value + o), ctypes.c_void_p(base + o), n))
            ts.append(time.perf_counter() - t0)
        print(f"{gb:.1f} GB chunk={chunk >> 20} MiB: {x.nbytes / min(ts) / 1e9:.1f} GB/s (first {x.nbytes / ts[0] / 1e9:.1f})",
              flush=True)
    del x
L.amr_free(p)
