"""Scan a large QPSK batch against the oracle and list the streams that differ
(debug aid; run on the GPU box):  python tools/parity_scan.py [B] [runs]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "audio-modem-radio_amd"), ROOT]
import numpy as np, _amr, synth, modem
from oracle import oracle
B = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
runs = int(sys.argv[2]) if len(sys.argv) > 2 else 2
x = synth.qpsk_batch(B, 96000, 9600, seed=1000, distinct=64)
want, _ = oracle.psk_demod_batch("qpsk", x, 9600, n_threads=16)
for r in range(runs):
    got = modem.qpsk_demodulate_batch(x, baud=9600)
    bad = [i for i in range(B) if got[i] != want[i]]
    print(f"run {r}: {len(bad)} bad; first {bad[:40]}", flush=True)
    if bad:
        i = bad[0]
        g, w_ = np.frombuffer(got[i], np.uint8), np.frombuffer(want[i], np.uint8)
        d = np.nonzero(g[:min(len(g), len(w_))] != w_[:min(len(g), len(w_))])[0]
        print(f"  stream {i}: len {len(g)} vs {len(w_)}, first diff byte {d[:5]}, ndiff {len(d)}", flush=True)
