"""Diagnostic: the device pocketfft's real transforms alone vs the oracle (AMR_PF_STAGE=1: rfft, 2: irfft)."""
import sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "audio-modem-radio_amd"), os.path.join(os.path.dirname(__file__), "..")]
import _amr
from oracle import oracle
stage = int(os.environ["AMR_PF_STAGE"])
rng = np.random.default_rng(12)
bad = []
for n in [62, 63, 93, 186, 189, 227, 271, 124, 31, 7, 21, 550, 377]:
    x = rng.standard_normal((1, n))
    got = _amr.hilbert_env_exact(x)[0]
    if stage == 1:
        X = oracle.rfft(x[0])
        hc = np.empty(n); hc[0] = X[0].real
        for i in range(1, (n + 1) // 2): hc[2 * i - 1] = X[i].real; hc[2 * i] = X[i].imag
        if n % 2 == 0: hc[n - 1] = X[n // 2].real
        want = hc
    else:
        hc = x[0]
        X = np.zeros(n // 2 + 1, complex); X[0] = hc[0]
        for i in range(1, (n + 1) // 2): X[i] = hc[2 * i - 1] + 1j * hc[2 * i]
        if n % 2 == 0: X[n // 2] = hc[n - 1]
        want = oracle.irfft(X, n) * n
    d = np.nonzero(got != want)[0]
    print(n, "stage", stage, "ndiff", d.size, "first", d[:8], flush=True)
