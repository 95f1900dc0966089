"""Diagnostic: which lengths does the device pocketfft restatement get wrong,
and by how much (GPU exact |hilbert| vs the oracle)."""
import sys, os
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "audio-modem-radio_amd"), os.path.join(os.path.dirname(__file__), "..")]
import _amr
from oracle import oracle
lo, hi = int(sys.argv[1]), int(sys.argv[2])
rng = np.random.default_rng(12)
bad = []
for n in range(lo, hi):
    x = rng.standard_normal((1, n))
    got = _amr.hilbert_env_exact(x)[0]
    want = oracle.hilbert_env(x[0])
    if not np.array_equal(got, want):
        d = np.nonzero(got != want)[0]
        bad.append(n)
        print(n, "ndiff", d.size, "first", d[:5], "maxrel", float(np.max(np.abs(got - want) / np.abs(want).max())), flush=True)
print("bad lengths:", bad)
