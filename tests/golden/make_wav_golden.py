#!/usr/bin/env python3
"""decode_wav_file fixtures at capture rates other than 96 kHz, from the
REFERENCE itself (this container only): decoder.decode_wav_file
(decoder.py:380-389) reads the WAV, resamples it to 96 kHz with
scipy.signal.resample (pocketfft's rfft / irfft: 441000 = 2^3 3^2 5^3 7^2
runs its generic radix-7 pass) and decodes -- the saved files are the
reference's bytes.  Inputs: framed QPSK / 8PSK / OFDM8 @ 1000 Bd, QPSK @ 9600
and BPSK @ 1200, modulated by the reference at 96 kHz, brought to 44.1 or
48 kHz (the builder's own resample; the WAV is the fixture), padded with
exact digital silence, written as 16-bit WAV.  Committed data only:

  tests/golden/wav.npz             the WAV files' bytes, key = case id
  tests/golden/wav_manifest.json   per case: mode, symbol rate, rate, and the
                                   reference's saved files (name, hex bytes)

tests/test_gpu_wav.py checks the drop-in decoder (GPU resample and demod)
against them.

Run:  python tests/golden/make_wav_golden.py   (needs /root/reference)
"""
from __future__ import annotations

import binascii
import contextlib
import io
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402  (the reference import helpers; its main() is not run)
import synth  # noqa: E402

CASES = [  # mode, symbol rate, capture rate, seconds of WAV, leading silence (s)
    ("QPSK", 1000, 44100, 10.0, 1.5),
    ("8PSK", 1000, 44100, 10.0, 0.25),
    ("OFDM8", 1000, 48000, 10.0, 2.0),
    ("QPSK", 1000, 48000, 3.0, 0.5),
    ("QPSK", 9600, 48000, 2.0, 0.3),
    ("BPSK", 1200, 44100, 3.0, 0.7),
    ("QPSK", 1000, 22050, 4.0, 1.0),
]


def main():
    from scipy import signal
    scratch = tempfile.mkdtemp(prefix="amr_wav_golden_")
    cwd = os.getcwd()
    rng = np.random.default_rng(20261019)
    arrays, cases = {}, []
    try:
        modem, _, decoder = mg._import_reference(scratch)
        for mode, sym, rate, secs, lead in CASES:
            payload = bytes(rng.integers(0, 256, int(rng.integers(60, 200)), dtype=np.uint8))
            fr = synth.frame_data(f"w{rate}_{mode}.bin", b"RAW" + payload, 0, 1, len(payload),
                                  binascii.crc32(payload) & 0xFFFFFFFF)
            arr96 = modem.bpsk_modulate(fr, baud=sym) if mode == "BPSK" else modem.qpsk_modulate(fr, baud=sym)
            arr = signal.resample(arr96, int(round(arr96.size * rate / 96000)))
            n = int(round(secs * rate))
            x = np.zeros(n)
            off = int(round(lead * rate))
            seg = arr[: n - off]
            x[off:off + seg.size] = seg * 0.9
            wav = synth.wav_bytes(x, rate)
            cid = f"wav_{mode}_{sym}_{rate // 1000}k"
            path = os.path.join(scratch, cid + ".wav")
            with open(path, "wb") as f:
                f.write(wav)
            arrays[cid] = np.frombuffer(wav, dtype=np.uint8)
            with contextlib.redirect_stdout(io.StringIO()):
                saved = decoder.decode_wav_file(path, mode, sym)
            files = []
            for p in saved:
                with open(p, "rb") as f:
                    files.append({"name": os.path.basename(p).split("_", 1)[1], "data": f.read().hex()})
            cases.append({"id": cid, "mode": mode, "symbol_rate": sym, "rate": rate, "n": n,
                          "payload": payload.hex(), "files": files})
            print(cid, n, [f["name"] for f in files])
    finally:
        os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "wav.npz"), **arrays)
    with open(os.path.join(HERE, "wav_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_wav_golden.py", "numpy": np.__version__, "cases": cases}, f,
                  indent=1)


if __name__ == "__main__":
    main()
