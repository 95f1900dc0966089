#!/usr/bin/env python3
"""Generate the golden fixtures by running the REFERENCE itself (this container only).

The reference (szumanski/Audio-Modem-Radio, read-only at /root/reference) is
imported from a scratch cwd; nothing of it is copied.  What is committed is
data only:

  tests/golden/inputs.npz      modulated input streams (float32 / float64 / int16)
  tests/golden/manifest.json   per case: the reference call, its parameters and
                               the reference's output bytes (hex) or the exact
                               exception type + message it raised
  tests/golden/intermediates.npz  reference-pipeline intermediates for one
                               stream (BP filtfilt output, baseband at the
                               symbol centres, diff products, angles)

Reference calls exercised (file:line in /root/reference):
  modem.qpsk_demodulate     modem.py:189-266
  modem.bpsk_demodulate     modem.py:68-135
  modem.fsk_demodulate      modem.py:298-341
  modem.psk8_demodulate / ofdm_demodulate_simple / fsk_high_speed_demodulate
                            modem.py:348, 375-376, 355-356
  fec.ReedSolomonFEC.decode fec.py:34-69
  decoder.decode_from_buffer / decode_wav_file  decoder.py:417-464, 380-389

Run:  python tests/golden/make_golden.py        (needs /root/reference)
"""
from __future__ import annotations

import binascii
import contextlib
import io
import json
import os
import sys
import tempfile
import types
import wave

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, os.path.join(REPO, "audio-modem-radio_amd"))
import synth  # noqa: E402  (our own transmit-side helpers)


def _stub_audio_modules():
    """decoder.py imports sounddevice/soundfile (decoder.py:6,8); neither is installed.

    soundfile.read is stubbed with libsndfile's default PCM16 -> float64
    normalisation (int16 / 32768.0)."""
    sd = types.ModuleType("sounddevice")
    sf = types.ModuleType("soundfile")

    def read(path):
        with wave.open(path, "rb") as w:
            sr = w.getframerate()
            nch = w.getnchannels()
            raw = np.frombuffer(w.readframes(w.getnframes()), dtype=np.int16)
        data = raw.astype(np.float64) / 32768.0
        if nch > 1:
            data = data.reshape(-1, nch)
        return data, sr

    sf.read = read
    sys.modules.setdefault("sounddevice", sd)
    sys.modules.setdefault("soundfile", sf)


def _import_reference(scratch):
    os.chdir(scratch)                       # decoder.py creates ./recv at import (decoder.py:17-18)
    sys.dont_write_bytecode = True          # never write into the read-only reference tree
    sys.path.insert(0, REF)
    _stub_audio_modules()
    import modem  # noqa
    import fec  # noqa
    with contextlib.redirect_stdout(io.StringIO()):
        import decoder  # noqa
    return modem, fec, decoder


def _run(fn, *args, **kw):
    """Call a reference function; return ("ok", bytes) or ("err", type, message)."""
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            out = fn(*args, **kw)
        return {"status": "ok", "out": bytes(out).hex()}
    except Exception as e:  # the reference's error contract is part of parity
        return {"status": "err", "etype": type(e).__name__, "emsg": str(e)}


def main():
    scratch = tempfile.mkdtemp(prefix="amr_golden_")
    cwd = os.getcwd()
    modem, fec, decoder = _import_reference(scratch)
    rng = np.random.default_rng(20251128)
    inputs = {}
    cases = []

    def add(case_id, fn_name, x, params, result_fn, **call_kw):
        inputs[case_id] = x
        res = result_fn(x, **call_kw)
        cases.append({"id": case_id, "fn": fn_name, "params": params, "dtype": str(x.dtype),
                      "n": int(x.size), **res})

    noise = lambda n, s: rng.normal(0.0, s, n).astype(np.float32)  # noqa: E731

    # --- QPSK @ 9600 (BASELINE config 2; OFDM8 config 4 is the same call) -------------
    for i in range(4):
        frame = synth.random_frame(rng, 2390 - 40 - 40)
        x = synth.fit(modem.qpsk_modulate(frame, baud=9600), 96000) + noise(96000, 0.05)
        add(f"qpsk9600_f32_{i}", "qpsk_demodulate", x.astype(np.float32), {"baud": 9600},
            lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    # float64 input (the decode_wav_file path hands float64 to the demod), odd length
    x = synth.fit(modem.qpsk_modulate(synth.random_frame(rng, 600), baud=9600), 48003).astype(np.float64)
    x = x + rng.normal(0, 0.05, x.size)
    add("qpsk9600_f64_odd", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    # int16-quantised WAV-like float64 (int16/32768)
    q = (synth.fit(modem.qpsk_modulate(synth.random_frame(rng, 300), baud=9600), 30000) * 32767).astype(np.int16)
    x = q.astype(np.float64) / 32768.0
    add("qpsk9600_wav", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))

    # --- QPSK loopback-exact rates (3000/baud integer) and other rates -----------------
    for baud, n_payload in [(1000, 120), (600, 40), (1500, 200), (3000, 150), (1200, 100), (2400, 100)]:
        frame = synth.random_frame(rng, n_payload)
        x = modem.qpsk_modulate(frame, baud=baud)
        x = (x + noise(x.size, 0.02)).astype(np.float32)
        add(f"qpsk{baud}_f32", "qpsk_demodulate", x, {"baud": baud},
            lambda x, b=baud: _run(modem.qpsk_demodulate, x, baud=b))

    # --- "8PSK" @ 19200 (BASELINE config 5: live alias -> QPSK demod) ------------------
    for i in range(2):
        x = synth.fit(synth.dpsk8_waveform(rng.integers(0, 8, 19200), 19200), 96000) + noise(96000, 0.05)
        add(f"psk8_19200_f32_{i}", "psk8_demodulate", x.astype(np.float32), {"b": 19200},
            lambda x: _run(modem.psk8_demodulate, x, 19200))
    # OFDM alias (modem.py:375-376) with its positional signature
    x = synth.fit(modem.qpsk_modulate(synth.random_frame(rng, 200), baud=9600), 20000) + noise(20000, 0.05)
    add("ofdm8_9600_f32", "ofdm_demodulate_simple", x.astype(np.float32),
        {"baud": 9600, "carrier": 3000.0, "num_subcarriers": 8},
        lambda x: _run(modem.ofdm_demodulate_simple, x, 9600, 3000.0, 8))
    # QPSK at a non-default carrier (12 kHz) through the plain signature
    x = synth.fit(modem.qpsk_modulate(synth.random_frame(rng, 200), baud=4800, carrier=12000.0), 30000)
    x = (x + noise(x.size, 0.05)).astype(np.float32)
    add("qpsk4800_fc12k_f32", "qpsk_demodulate", x, {"baud": 4800, "carrier": 12000.0},
        lambda x: _run(modem.qpsk_demodulate, x, baud=4800, carrier=12000.0))

    # --- BPSK ---------------------------------------------------------------------------
    for baud, n_payload in [(1200, 150), (9600, 900), (2400, 300)]:
        x = modem.bpsk_modulate(synth.random_frame(rng, n_payload), baud=baud)
        x = (x + noise(x.size, 0.03)).astype(np.float32)
        add(f"bpsk{baud}_f32", "bpsk_demodulate", x, {"baud": baud},
            lambda x, b=baud: _run(modem.bpsk_demodulate, x, baud=b))
    x = modem.bpsk_modulate(synth.random_frame(rng, 100), baud=31.25 * 32)
    add("bpsk1000_f64", "bpsk_demodulate", x.astype(np.float64) * 0.5, {"baud": 1000},
        lambda x: _run(modem.bpsk_demodulate, x, baud=1000))

    # --- edge cases & error contracts ---------------------------------------
    add("qpsk_n28", "qpsk_demodulate", rng.normal(0, 1, 28).astype(np.float32), {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    add("qpsk_n27_err", "qpsk_demodulate", rng.normal(0, 1, 27).astype(np.float32), {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    add("qpsk_lt2sym", "qpsk_demodulate", rng.normal(0, 1, 60).astype(np.float32), {"baud": 1200},
        lambda x: _run(modem.qpsk_demodulate, x, baud=1200))
    add("qpsk_zeros", "qpsk_demodulate", np.zeros(5000, np.float32), {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    add("qpsk_const", "qpsk_demodulate", np.full(5000, 0.25, np.float32), {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    add("qpsk_wn_err", "qpsk_demodulate", rng.normal(0, 1, 4000).astype(np.float32), {"baud": 48000},
        lambda x: _run(modem.qpsk_demodulate, x, baud=48000))
    add("bpsk_n27_err", "bpsk_demodulate", rng.normal(0, 1, 27).astype(np.float32), {"baud": 1200},
        lambda x: _run(modem.bpsk_demodulate, x, baud=1200))
    add("bpsk_lt2sym", "bpsk_demodulate", rng.normal(0, 1, 200).astype(np.float32), {"baud": 1200},
        lambda x: _run(modem.bpsk_demodulate, x, baud=1200))

    # --- FSK (BASELINE config 3 numeric path uses valid tones 12k/24k) -------------------
    for i, n in enumerate([96000, 24001]):
        fr = synth.random_frame(rng, 60)
        x = synth.fit(modem.fsk_modulate(fr, baud=9600, mark_freq=12000.0, space_freq=24000.0), n)
        x = (x + noise(n, 0.05)).astype(np.float32)
        add(f"fsk9600_f32_{i}", "fsk_demodulate", x,
            {"baud": 9600, "mark_freq": 12000.0, "space_freq": 24000.0},
            lambda x: _run(modem.fsk_demodulate, x, 9600, 12000.0, 24000.0))
    x = modem.fsk_modulate(synth.random_frame(rng, 40), baud=1200, mark_freq=2400.0, space_freq=4800.0)
    add("fsk1200_f32", "fsk_demodulate", (x + noise(x.size, 0.05)).astype(np.float32),
        {"baud": 1200, "mark_freq": 2400.0, "space_freq": 4800.0},
        lambda x: _run(modem.fsk_demodulate, x, 1200, 2400.0, 4800.0))
    add("fsk_default_err", "fsk_demodulate", rng.normal(0, 1, 9600).astype(np.float32), {"baud": 1200},
        lambda x: _run(modem.fsk_demodulate, x, baud=1200))
    add("fsk_hs_err", "fsk_high_speed_demodulate", rng.normal(0, 1, 9600).astype(np.float32), {"baud": 19200},
        lambda x: _run(modem.fsk_high_speed_demodulate, x, 19200))
    add("fsk_n21_err", "fsk_demodulate", rng.normal(0, 1, 21).astype(np.float32),
        {"baud": 1200, "mark_freq": 2400.0, "space_freq": 4800.0},
        lambda x: _run(modem.fsk_demodulate, x, 1200, 2400.0, 4800.0))

    # --- signed zeros, silence, denormals, non-finite (exact-zero semantics) ----------
    sig = synth.fit(modem.qpsk_modulate(synth.random_frame(rng, 400), baud=9600), 20000)
    add("qpsk_negzero", "qpsk_demodulate", np.full(5000, -0.0, np.float32), {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = np.concatenate([sig + noise(20000, 0.05), np.zeros(60000, np.float32)]).astype(np.float32)
    add("qpsk_tail_silence", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = np.concatenate([np.zeros(40000, np.float32), sig + noise(20000, 0.05)]).astype(np.float32)
    add("qpsk_head_silence", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = (sig[:8000].astype(np.float64) + rng.normal(0, 0.05, 8000)) * 1e-310
    add("qpsk_denorm_f64", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = ((sig[:8000] + noise(8000, 0.05)) * np.float32(1e-41)).astype(np.float32)
    add("qpsk_denorm_f32", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = (sig[:6000] + noise(6000, 0.05)).astype(np.float32)
    x[3000] = np.nan
    add("qpsk_nan", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = (sig[:6000] + noise(6000, 0.05)).astype(np.float32)
    x[100] = np.inf
    add("qpsk_inf", "qpsk_demodulate", x, {"baud": 9600},
        lambda x: _run(modem.qpsk_demodulate, x, baud=9600))
    x = np.zeros(3000, np.float32)
    x[::7] = -0.0
    x[1::11] = 0.5
    add("qpsk_sparse", "qpsk_demodulate", x, {"baud": 2400},
        lambda x: _run(modem.qpsk_demodulate, x, baud=2400))
    x = modem.bpsk_modulate(synth.random_frame(rng, 60), baud=2400)
    x = np.concatenate([x, np.zeros(50000, np.float32)]).astype(np.float32)
    add("bpsk_tail_silence", "bpsk_demodulate", x, {"baud": 2400},
        lambda x: _run(modem.bpsk_demodulate, x, baud=2400))
    add("bpsk_zeros", "bpsk_demodulate", np.zeros(4000, np.float64), {"baud": 1200},
        lambda x: _run(modem.bpsk_demodulate, x, baud=1200))

    # --- FEC parity-XOR + CRC32 decode (fec.py:34-69) ------------------------------------
    rs = fec.ReedSolomonFEC()
    fec_cases = []
    for ln in [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 31, 100, 1001]:
        d = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        fec_cases.append(d)
    fec_cases.append(rs.encode(b"hello world!"))
    fec_cases.append(rs.encode(b"odd"))
    corrupted = bytearray(rs.encode(bytes(range(50))))
    corrupted[7] ^= 0x10
    fec_cases.append(bytes(corrupted))
    fec_golden = []
    for d in fec_cases:
        with contextlib.redirect_stdout(io.StringIO()) as so:
            out = rs.decode(d)
        fec_golden.append({"in": d.hex(), "out": out.hex(), "crc_warn": "CRC" in so.getvalue()})

    # --- decoder end to end (decoder.py:380-464) ----------------------------------------
    dec_cases = []
    payload = bytes(rng.integers(0, 256, 150, dtype=np.uint8))
    fr = synth.frame_data("hello.bin", b"RAW" + payload, 0, 1, len(payload), binascii.crc32(payload) & 0xFFFFFFFF)
    for mode, sr_sym in [("QPSK", 1000), ("8PSK", 1000), ("OFDM8", 1000), ("QPSK", 9600), ("BPSK", 1200)]:
        if mode == "BPSK":
            arr = modem.bpsk_modulate(fr, baud=sr_sym)
        else:
            arr = modem.qpsk_modulate(fr, baud=sr_sym)
        wav = modem.wav_from_array(arr, 96000)
        case_id = f"dec_{mode}_{sr_sym}"
        path = os.path.join(scratch, case_id + ".wav")
        with open(path, "wb") as f:
            f.write(wav)
        inputs[case_id] = np.frombuffer(wav, dtype=np.uint8)
        with contextlib.redirect_stdout(io.StringIO()):
            saved = decoder.decode_wav_file(path, mode, sr_sym)
        files = []
        for p in saved:
            with open(p, "rb") as f:
                files.append({"name": os.path.basename(p).split("_", 1)[1], "data": f.read().hex()})
        dec_cases.append({"id": case_id, "mode": mode, "symbol_rate": sr_sym, "files": files})
    # config 1 plumbing: FSK1200, 10 s at 44.1 kHz -> resample -> FSK raises -> []
    x = synth.fit(synth.fsk_waveform(fr, 1200, 1200.0, 2200.0, 44100), 441000)
    wav = synth.wav_bytes(x, 44100)
    path = os.path.join(scratch, "dec_fsk1200_44k.wav")
    with open(path, "wb") as f:
        f.write(wav)
    inputs["dec_FSK1200_44k"] = np.frombuffer(wav, dtype=np.uint8)
    with contextlib.redirect_stdout(io.StringIO()) as so:
        saved = decoder.decode_wav_file(path, "FSK1200", 1200)
    dec_cases.append({"id": "dec_FSK1200_44k", "mode": "FSK1200", "symbol_rate": 1200,
                      "files": [], "saved": saved, "log_has_error": "Erro crítico" in so.getvalue()})

    # --- intermediates for one QPSK@9600 stream (float tolerances) ----------
    from scipy import signal
    x = inputs["qpsk9600_f32_0"][:24000]
    sps, nyq, baud, fc = 10, 48000.0, 9600, 3000.0
    b, a = signal.butter(4, [max(0.01, (fc - baud * 1.5) / nyq), min(0.99, (fc + baud * 1.5) / nyq)], btype="band")
    filt = signal.filtfilt(b, a, x)
    t = np.arange(len(filt)) / 96000
    bb = filt * np.exp(-1j * 2 * np.pi * fc * t)
    bl, al = signal.butter(4, baud / nyq, btype="low")
    bb = signal.filtfilt(bl, al, bb)
    sym = bb[sps // 2::sps]
    diff = sym[1:] * np.conj(sym[:-1])
    inter = {"x": x, "bp": filt, "sym": sym, "diff": diff, "angle": np.angle(diff),
             "bp_b": b, "bp_a": a, "lp_b": bl, "lp_a": al,
             "out": np.frombuffer(modem.qpsk_demodulate(x, baud=9600), dtype=np.uint8)}

    os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "inputs.npz"), **inputs)
    np.savez_compressed(os.path.join(HERE, "intermediates.npz"), **inter)
    import scipy
    manifest = {"generator": "tests/golden/make_golden.py",
                "reference": "szumanski/Audio-Modem-Radio @ /root/reference",
                "numpy": np.__version__, "scipy": scipy.__version__,
                # numpy's arctan2 (np.angle) dispatch on the generating host: the
                # QPSK slicer's near-tie decisions depend on it
                "numpy_cpu_features": numpy_cpu_features(),
                "cases": cases, "fec": fec_golden, "decoder": dec_cases}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(f"{len(cases)} demod cases, {len(fec_golden)} fec cases, {len(dec_cases)} decoder cases")
    for c in cases:
        print(c["id"], c["status"], (len(c["out"]) // 2) if c["status"] == "ok" else c["emsg"][:70])
    for d in dec_cases:
        print(d["id"], [f["name"] for f in d["files"]])


def numpy_cpu_features() -> dict:
    from numpy._core._multiarray_umath import __cpu_features__ as f
    return {k: bool(f.get(k, False)) for k in ("AVX512F", "AVX512_SKX", "AVX2", "FMA3")}


if __name__ == "__main__":
    main()
