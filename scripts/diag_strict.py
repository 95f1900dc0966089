"""Diagnostic: device strict bound vs the numpy restatement, per stream."""
import os, sys
import numpy as np
root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(root, "audio-modem-radio_amd"), root, os.path.join(root, "tests")]
import _amr
from oracle import oracle
from _util import strict_symbol_bounds
from test_gpu_split_strict import _signals, CASES
for kind, baud, fc, fs, n in CASES[:2]:
    x = _signals(kind, baud, fc, fs, n, baud)
    d = _amr.split_strict_design(kind, n, baud, fc, fs)
    sd = _amr.split_design(kind, n, baud, fc, fs)
    T = _amr.split_state_tables(kind, n, baud, fc, fs)
    pl = _amr.PskPlan(kind, n, baud, fc, fs, max_streams=x.shape[0])
    sym, eb, sc = pl.split_bounds(x)
    L = pl.split_info()["chunk"]
    op = oracle.PskPlan(kind, n, baud, fc, fs)
    for i in range(x.shape[0]):
        st = oracle.psk_split_stats(kind, x[i], baud, fc, fs, L, sd["warmup_bp"], T, d)
        e, scal = strict_symbol_bounds(st, d, float(np.abs(x[i]).max()), n, op.first, op.sps, L)
        r = eb[i] / e - 1
        print(kind, baud, i, "dev", sc[i], "np", scal[:4], "ok", scal[4], "rel", np.abs(r).max(),
              "argmax", int(np.abs(r).argmax()), "of", r.size, "neg", (r < -1e-9).sum(), "pos", (r > 1e-9).sum(),
              "stats", st["D1max"], st["y1max"], st["D2max"], st["fmax"], flush=True)
