"""Diagnostic: F2's ambiguity flags on one sweep fixture (bytes vs the
reference, flagged count, the fast envelopes' closest compare)."""
import sys, os, json
import numpy as np
sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", "audio-modem-radio_amd"), os.path.join(os.path.dirname(__file__), "..")]
import _fsk
from oracle import oracle
g = os.path.join(os.path.dirname(__file__), "..", "tests", "golden")
m = json.load(open(os.path.join(g, "sweep_manifest.json")))["cases"]
d = np.load(os.path.join(g, "sweep.npz"))
for cid in sys.argv[1:]:
    c = [c for c in m if c["id"] == cid][0]
    p = c["params"]
    x = d[cid]
    want = bytes.fromhex(c["out"])
    for label, xx in (("native", x), ("f64", x.astype(np.float64) / 32768 if x.dtype == np.int16 else x.astype(np.float64)),
                      ("f32", (x.astype(np.float64) / 32768 if x.dtype == np.int16 else x).astype(np.float32))):
        for B in (1, 4):
            pl = _fsk.FskPlan(x.size, p["baud"], p["f0"], p["f1"], p["samp_rate"], max_streams=B)
            got, _ = pl.demod_host(np.stack([xx] * B))
            print(cid, label, "B", B, "fft_len", pl.fft_length, "live", pl.live_columns, "flagged", pl.exact_streams(),
                  "bytes ok", all(gg == want for gg in got), flush=True)
    pl = _fsk.FskPlan(x.size, p["baud"], p["f0"], p["f1"], p["samp_rate"], max_streams=1)
    xf = x.astype(np.float64) / 32768 if x.dtype == np.int16 else x.astype(np.float64)
    gm, gs = pl.envelopes(xf[None])
    r = np.abs(gm[0] - gs[0]) / np.abs(xf).max()
    print(cid, "fast envelopes: min |gm - gs| / peak", r.min(), "count < 2 tau", int((r < 2 * 2.0 ** -36).sum()), flush=True)

import modem
for cid in sys.argv[1:]:
    c = [c for c in m if c["id"] == cid][0]
    p = c["params"]
    x = d[cid]
    want = bytes.fromhex(c["out"])
    for ms in (1, 2, 16, 33):
        pl = _fsk.FskPlan(x.size, p["baud"], p["f0"], p["f1"], p["samp_rate"], max_streams=ms)
        got, _ = pl.demod_host(x[None])
        print(cid, "max_streams", ms, "B 1 flagged", pl.exact_streams(), "ok", got[0] == want, flush=True)
    got = modem.fsk_demodulate(x, baud=p["baud"], mark_freq=p["f0"], space_freq=p["f1"], samp_rate=p["samp_rate"])
    print(cid, "drop-in ok", got == want, flush=True)
