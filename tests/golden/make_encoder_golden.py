#!/usr/bin/env python3
"""Generate the encoder / compression golden fixtures by running the REFERENCE's
encoder.py and utils/compression.py (this container only).

Committed output is data only:
  tests/golden/encoder.npz           "<id>.in" input bytes, "<id>.out" output bytes
                                     (compressed payloads, frames, WAV files)
  tests/golden/encoder_manifest.json per case: the reference call, its parameters and
                                     either the scalar/dict result or the exception

Reference calls (file:line in /root/reference):
  utils/compression.py  IntelligentCompressor :11-69, intelligent_compress :72-100,
                        intelligent_decompress :103-123, compress_data :152-156,
                        super_compress :201-226, adaptive_compress :276-285
  encoder.py            adaptive_compress :50-60, calculate_transmission_stats :63-91,
                        _frame_data :94-114, split_file_for_transmission :117-151,
                        encode_file_parts :154-252, encode_file :260-306,
                        get_encoding_stats :309-315, verify_audio_output :318-348

encoder.py imports pygame and PyQt5.QtCore (encoder.py:12-14) for the GUI only;
both are absent here and are replaced by empty stub modules.

Run:  python tests/golden/make_encoder_golden.py        (needs /root/reference)
"""
from __future__ import annotations

import contextlib
import io
import json
import logging
import os
import sys
import tempfile
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402  (reference import helper)


def _import_encoder(scratch):
    make_golden._import_reference(scratch)          # modem / fec / decoder, cwd = scratch
    pg = types.ModuleType("pygame")
    qt = types.ModuleType("PyQt5")
    qtc = types.ModuleType("PyQt5.QtCore")
    qtc.QTimer = object
    qt.QtCore = qtc
    for name, mod in (("pygame", pg), ("PyQt5", qt), ("PyQt5.QtCore", qtc)):
        sys.modules.setdefault(name, mod)
    with contextlib.redirect_stdout(io.StringIO()):
        import encoder  # noqa
        from utils import compression  # noqa
    return encoder, compression


def payloads(rng):
    """Named inputs covering each branch of the compressor's analysis."""
    text = (b"The quick brown fox jumps over the lazy dog. " * 3
            + rng.choice(list(b"abcdefghijklmnopqrstuvwxyz ,.\n"), 1800).astype(np.uint8).tobytes())
    return {
        "empty": b"",
        "tiny": b"hello",
        "short150": rng.integers(0, 256, 150, dtype=np.uint8).tobytes(),
        "b199": rng.integers(0, 256, 199, dtype=np.uint8).tobytes(),
        "b200": rng.integers(0, 256, 200, dtype=np.uint8).tobytes(),
        "random2k": rng.integers(0, 256, 2000, dtype=np.uint8).tobytes(),
        "random600": rng.integers(0, 256, 600, dtype=np.uint8).tobytes(),
        "lowent": rng.integers(0, 3, 3000, dtype=np.uint8).tobytes(),
        "repeat": (b"ABCDEFGH" * 40) + rng.integers(0, 256, 1500, dtype=np.uint8).tobytes(),
        "text": text,
        "ramp": (np.arange(5000) * 7 % 256).astype(np.uint8).tobytes(),
        "sine": (128 + 100 * np.sin(np.arange(4000) / 9.0)).astype(np.uint8).tobytes(),
        "zeros": bytes(1200),
        "binary_hi": rng.integers(0, 256, 1100, dtype=np.uint8).tobytes(),
        "randtext": rng.choice(list(b"abcdefghijklmnopqrstuvwxyz ,.\n"), 1500).astype(np.uint8).tobytes(),
        "mostlytext": rng.choice(list(b"abcdefghijklmnopqrstuvwxyz"), 850).astype(np.uint8).tobytes() + bytes(range(150)),
    }


def main():
    scratch = tempfile.mkdtemp(prefix="amr_enc_golden_")
    cwd = os.getcwd()
    encoder, comp = _import_encoder(scratch)
    logging.getLogger("filebeep").disabled = True
    rng = np.random.default_rng(20261016)
    arrays, cases = {}, []

    def b2a(b):
        return np.frombuffer(bytes(b), np.uint8)

    def call(case_id, fn_name, fn, data=None, *args, **kw):
        if data is not None:
            arrays[f"{case_id}.in"] = b2a(data)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                out = fn(*((data,) if data is not None else ()), *args, **kw)
        except Exception as e:
            cases.append({"id": case_id, "fn": fn_name, "args": list(args), "kw": kw,
                          "status": "err", "etype": type(e).__name__, "emsg": str(e)})
            return None
        rec = {"id": case_id, "fn": fn_name, "args": list(args), "kw": kw, "status": "ok"}
        if isinstance(out, (bytes, bytearray)):
            arrays[f"{case_id}.out"] = b2a(out)
            rec["kind"] = "bytes"
        else:
            rec["kind"] = "value"
            rec["value"] = out if not isinstance(out, np.bool_) else bool(out)
        cases.append(rec)
        return out

    ins = payloads(rng)
    ic = comp.IntelligentCompressor()
    for name, d in ins.items():
        call(f"analyze.{name}", "IntelligentCompressor.analyze_data_pattern",
             lambda x: {k: v for k, v in ic.analyze_data_pattern(x).items()}, d)
        out = call(f"icomp.{name}", "intelligent_compress", comp.intelligent_compress, d)
        for m in ("lzma", "delta+lzma", "zlib", "none"):
            call(f"icomp_{m}.{name}", "intelligent_compress", comp.intelligent_compress, d, mode=m)
        if out is not None:
            call(f"idecomp.{name}", "intelligent_decompress", comp.intelligent_decompress, out)
        call(f"super.{name}", "super_compress", comp.super_compress, d)
        call(f"cdata.{name}", "compress_data", comp.compress_data, d)
        for mode in ("QPSK", "8PSK", "APSK16", "FSK1200"):
            call(f"uadapt_{mode}.{name}", "compression.adaptive_compress", comp.adaptive_compress, d, mode)
            call(f"eadapt_{mode}.{name}", "encoder.adaptive_compress", encoder.adaptive_compress, d, mode)

    # framing
    for i, (fname, n, part, total) in enumerate([("a.txt", 0, 0, 1), ("photo.jpg", 333, 2, 5),
                                                 ("n" * 300, 17, 0, 1), ("ção ünï.bin", 64, 1, 2)]):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        call(f"frame.{i}", "_frame_data", lambda x, fn=fname, p=part, t=total:
             encoder._frame_data(fn, x, p, t, 123456 + i, 0xDEADBEEF - i), d)
    for mode in ("FSK1200", "FSK9600", "BPSK", "QPSK", "8PSK", "OFDM8", "SSTV", "HELLSCHREIBER", "XYZ"):
        for sr, fs, c in ((9600, 100000, True), (1200, 5000, False), (300, 1, True)):
            call(f"stats.{mode}.{sr}.{fs}.{int(c)}", "calculate_transmission_stats",
                 encoder.calculate_transmission_stats, None, fs, mode, sr, c)

    # files on disk (split / encode)
    files = {}
    for name, n in (("small.bin", 40), ("mid.txt", 700), ("big.bin", 7000)):
        p = os.path.join(scratch, name)
        d = ins["text"][:n] if name.endswith(".txt") else rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        with open(p, "wb") as f:
            f.write(d)
        files[name] = d
        arrays[f"file.{name}"] = b2a(d)

    for name in files:
        for mode, sr, dur in (("QPSK", 1200, 1), ("FSK1200", 1200, 60), ("BPSK", 300, 2)):
            cid = f"split.{name}.{mode}.{sr}.{dur}"
            parts = call(cid, "split_file_for_transmission",
                         lambda _, nm=name, m=mode, s=sr, t=dur: [
                             [p[0], p[1].hex(), p[2], p[3], p[4], p[5]]
                             for p in encoder.split_file_for_transmission(os.path.join(scratch, nm), m, s, t)],
                         b"")
            del parts
        cases.append({"id": f"encstats.{name}", "fn": "get_encoding_stats", "status": "ok", "kind": "value",
                      "value": encoder.get_encoding_stats(os.path.join(scratch, name), "QPSK", True, 9600),
                      "args": [name, "QPSK", True, 9600], "kw": {}})

    # encode_file: the WAV the reference writes (encoder.py:297-304)
    for name in ("small.bin", "mid.txt"):
        for mode, sr, c in (("QPSK", 9600, True), ("BPSK", 4800, True), ("FSK9600", 9600, False),
                            ("8PSK", 9600, True), ("QPSK", 1200, False)) + ((("FSK1200", 1200, True),)
                                                                           if name == "small.bin" else ()):
            with contextlib.redirect_stdout(io.StringIO()):
                out = encoder.encode_file(os.path.join(scratch, name), mode, c, sr)
            cid = f"encode.{name}.{mode}.{sr}.{int(c)}"
            rec = {"id": cid, "fn": "encode_file", "args": [name, mode, c, sr], "kw": {}, "status": "ok",
                   "kind": "wav", "path": os.path.relpath(out, scratch) if out else ""}
            if out:
                with open(out, "rb") as f:
                    arrays[f"{cid}.out"] = b2a(f.read())
            cases.append(rec)

    # encode_file_parts: modes that run and the ones whose alias calls raise
    parts = [("p.bin", rng.integers(0, 256, 30, dtype=np.uint8).tobytes(), 0, 1, 30, 7)]
    for mode, sr in (("QPSK", 9600), ("OFDM4", 4800), ("FSK19200", 19200), ("8PSK", 9600),
                     ("APSK16", 9600), ("MSK", 1200), ("NOPE", 1200)):
        cid = f"parts.{mode}.{sr}"
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                outs = encoder.encode_file_parts(parts, mode, True, sr)
            rec = {"id": cid, "fn": "encode_file_parts", "args": [mode, True, sr], "kw": {}, "status": "ok",
                   "kind": "wav", "path": os.path.relpath(outs[0], scratch)}
            with open(outs[0], "rb") as f:
                arrays[f"{cid}.out"] = b2a(f.read())
        except Exception as e:
            rec = {"id": cid, "fn": "encode_file_parts", "args": [mode, True, sr], "kw": {}, "status": "err",
                   "etype": type(e).__name__, "emsg": str(e)}
        cases.append(rec)
    arrays["parts.in"] = b2a(parts[0][1])

    # verify_audio_output
    sig = {"ok": 0.5 * np.sin(np.arange(20000) / 7.0).astype(np.float32), "zeros": np.zeros(20000, np.float32),
           "short": 0.5 * np.sin(np.arange(500) / 7.0), "clip": 1.5 * np.sin(np.arange(20000) / 7.0),
           "nan": np.where(np.arange(20000) == 5, np.nan, np.sin(np.arange(20000.0))),
           "quiet": 0.001 * np.sin(np.arange(20000) / 7.0)}
    for name, a in sig.items():
        arrays[f"verify.{name}.in"] = np.asarray(a, np.float64)
        cases.append({"id": f"verify.{name}", "fn": "verify_audio_output", "status": "ok", "kind": "value",
                      "value": bool(encoder.verify_audio_output(a)), "args": [], "kw": {}})

    os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "encoder.npz"), **arrays)
    with open(os.path.join(HERE, "encoder_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_encoder_golden.py", "cases": cases}, f, indent=0)
    print(f"{len(cases)} cases, {sum(a.nbytes for a in arrays.values())} bytes of arrays")


if __name__ == "__main__":
    main()
