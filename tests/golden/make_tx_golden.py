#!/usr/bin/env python3
"""Generate the transmit-side golden fixtures by running the REFERENCE's modulators
(this container only).

Committed output is data only:
  tests/golden/tx.npz        per case: the input bytes ("<id>.in", uint8), the
                             reference waveform ("<id>.out", float32) and the
                             WAV file the reference writes for it ("<id>.wav",
                             uint8 -- modem.wav_from_array's bytes)
  tests/golden/tx_manifest.json  per case: the reference call and its parameters,
                             or the exception type + message it raised

Reference calls (file:line in /root/reference):
  modem.bpsk_modulate   modem.py:28-65
  modem.qpsk_modulate   modem.py:138-186
  modem.fsk_modulate    modem.py:270-295
  modem.wav_from_array  modem.py:360-368

Run:  python tests/golden/make_tx_golden.py        (needs /root/reference)
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (reference import helper + our synth for frames)
import synth  # noqa: E402


def main():
    scratch = tempfile.mkdtemp(prefix="amr_tx_golden_")
    cwd = os.getcwd()
    modem, _, _ = make_golden._import_reference(scratch)
    rng = np.random.default_rng(20261016)
    arrays = {}
    cases = []

    def add(case_id, fn_name, data: bytes, **params):
        fn = getattr(modem, fn_name)
        arrays[f"{case_id}.in"] = np.frombuffer(data, dtype=np.uint8)
        try:
            out = fn(data, **params)
        except Exception as e:          # the reference's error contract is part of parity
            cases.append({"id": case_id, "fn": fn_name, "params": params, "n_bytes": len(data),
                          "status": "err", "etype": type(e).__name__, "emsg": str(e)})
            return
        arrays[f"{case_id}.out"] = np.asarray(out)
        arrays[f"{case_id}.wav"] = np.frombuffer(modem.wav_from_array(out), dtype=np.uint8)
        cases.append({"id": case_id, "fn": fn_name, "params": params, "n_bytes": len(data),
                      "status": "ok", "dtype": str(np.asarray(out).dtype), "n": int(np.asarray(out).size)})

    frame = lambda n: synth.random_frame(rng, n)            # noqa: E731
    rnd = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()   # noqa: E731

    # DQPSK: the headline baud, the reference's round-trip bauds, odd sps, other carrier
    add("qpsk9600", "qpsk_modulate", frame(200), baud=9600)
    add("qpsk1200", "qpsk_modulate", frame(40))
    add("qpsk1000", "qpsk_modulate", frame(60), baud=1000)
    add("qpsk4800_fc12k", "qpsk_modulate", frame(80), baud=4800, carrier=12000.0)
    add("qpsk1234_5", "qpsk_modulate", rnd(30), baud=1234.5)
    add("qpsk9600_44k", "qpsk_modulate", rnd(50), baud=4410, samp_rate=44100)
    add("qpsk_empty", "qpsk_modulate", b"", baud=9600)
    add("qpsk_ff", "qpsk_modulate", b"\xff" * 300, baud=9600)   # +pi every symbol: the phase grows
    add("qpsk19200_err", "qpsk_modulate", rnd(8), baud=19200)   # ramp = 0 -> broadcast error
    add("qpsk_sps0", "qpsk_modulate", rnd(8), baud=200000)      # sps = 0 -> empty waveform
    # DBPSK
    add("bpsk1200", "bpsk_modulate", frame(30))
    add("bpsk9600", "bpsk_modulate", frame(100), baud=9600)
    add("bpsk2400_fc5k", "bpsk_modulate", rnd(40), baud=2400, carrier=5000.0)
    add("bpsk_empty", "bpsk_modulate", b"")
    add("bpsk48000_err", "bpsk_modulate", rnd(4), baud=48000)
    # CPFSK
    add("fsk1200", "fsk_modulate", frame(20))
    add("fsk9600", "fsk_modulate", frame(100), baud=9600, mark_freq=12000.0, space_freq=24000.0)
    add("fsk19200_hs", "fsk_modulate", rnd(60), baud=19200, mark_freq=8000.0, space_freq=16000.0)
    add("fsk300", "fsk_modulate", rnd(6), baud=300, mark_freq=1070.0, space_freq=1270.0)
    add("fsk_odd", "fsk_modulate", rnd(25), baud=1234.5, mark_freq=3333.3, space_freq=5555.5, samp_rate=48000)
    add("fsk_empty", "fsk_modulate", b"")

    os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "tx.npz"), **arrays)
    manifest = {"generator": "tests/golden/make_tx_golden.py",
                "reference": "szumanski/Audio-Modem-Radio @ /root/reference",
                "numpy": np.__version__, "cases": cases}
    with open(os.path.join(HERE, "tx_manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    for c in cases:
        print(c["id"], c["status"], c["n"] if c["status"] == "ok" else c["emsg"][:80])


if __name__ == "__main__":
    main()
