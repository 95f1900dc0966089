#!/usr/bin/env python3
"""Golden fixtures for the receive-side file handling the reference's decoder.py
keeps next to the demodulator (this container only):

  FileAssembly / AdvancedFileAssembly  decoder.py:20-122
  save_decoded_files                   decoder.py:247-310
  decode_with_retry                    decoder.py:313-377

Committed output is data only:
  tests/golden/assembly.npz            "<id>.<k>" byte strings (inputs, saved files,
                                       demodulated_attempt_<k>.bin dumps) and the
                                       decode_with_retry input waveform
  tests/golden/assembly_manifest.json  per case: calls, return values, stats

Run:  python tests/golden/make_assembly_golden.py      (needs /root/reference)
"""
from __future__ import annotations

import contextlib
import glob
import io
import json
import os
import sys
import tempfile
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402
import synth  # noqa: E402


def main():
    scratch = tempfile.mkdtemp(prefix="amr_asm_golden_")
    cwd = os.getcwd()
    modem, _, decoder = make_golden._import_reference(scratch)
    rng = np.random.default_rng(20261017)
    arrays, cases = {}, []

    def b(x):
        return np.frombuffer(bytes(x), np.uint8)

    # --- signal quality -------------------------------------------------------------
    payloads = {"empty": b"", "zeros": bytes(50), "rand": rng.integers(0, 256, 300, dtype=np.uint8).tobytes(),
                "rep5": b"abcde" * 20, "rep5tail": b"abcde" * 20 + b"xy", "short": b"abcdeabcde",
                "half0": bytes(100) + rng.integers(1, 256, 100, dtype=np.uint8).tobytes(),
                "text": b"hello world, this is a part of a file " * 3}
    fa = decoder.FileAssembly("q.bin", 1, 0, 0)
    for name, p in payloads.items():
        arrays[f"quality.{name}"] = b(p)
        cases.append({"id": f"quality.{name}", "value": fa.calculate_signal_quality(p)})

    # --- add_part / assemble sequences ----------------------------------------------------
    data = rng.integers(0, 256, 900, dtype=np.uint8).tobytes()
    parts = [data[:300], data[300:600], data[600:]]
    crc = zlib.crc32(data) & 0xffffffff
    seqs = {
        "inorder": [(0, 0, None), (1, 1, None), (2, 2, None)],
        "reverse": [(2, 2, None), (1, 1, None), (0, 0, None)],
        "dup_better": [(0, 0, 0.1), (0, 0, 0.9), (1, 1, None), (2, 2, None)],
        "dup_worse": [(0, 0, 0.9), (0, 0, 0.1), (1, 1, None), (2, 2, None)],
        "bad_index": [(5, 0, None), (-1, 1, None), (0, 0, None)],
        "missing": [(0, 0, None), (2, 2, None)],
        "wrong_crc": [(0, 0, None), (1, 2, None), (2, 1, None)],
    }
    for name, seq in seqs.items():
        asm = decoder.AdvancedFileAssembly("f.bin", 3, 900, crc)
        rets = []
        with contextlib.redirect_stdout(io.StringIO()):
            for idx, src, q in seq:
                rets.append(asm.add_part(idx, parts[src], q))
        rec = {"id": f"assemble.{name}", "seq": seq, "add_part": rets, "quality": asm.parts_quality,
               "received": asm.received_parts, "progress": asm.get_progress(), "missing": asm.get_missing_parts(),
               "report": asm.get_quality_report()}
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                out = asm.assemble_file()
            arrays[f"assemble.{name}.out"] = b(out)
            rec["status"] = "ok"
        except Exception as e:
            rec.update(status="err", etype=type(e).__name__, emsg=str(e))
        cases.append(rec)
    for i, p in enumerate(parts):
        arrays[f"parts.{i}"] = b(p)
    cases.append({"id": "parts.meta", "crc": crc, "size": 900})

    # --- save_decoded_files on tuple entries ---------------------------------------------
    single = rng.integers(0, 256, 400, dtype=np.uint8).tobytes()
    entries = [("one.bin", b"ZLIB" + zlib.compress(single), False, 0, 1, 400, 0),
               ("two raw!.txt", b"RAW_payload", False, 0, 1, 0, 0),
               ("m.bin", parts[1], True, 1, 3, 900, crc),
               ("m.bin", parts[0], True, 0, 3, 900, crc),
               ("m.bin", parts[0], True, 0, 3, 900, crc),          # duplicate, equal quality: ignored
               ("m.bin", parts[2], True, 2, 3, 900, crc),
               ("bad.bin", b"LZMAnot-lzma", False, 0, 1, 0, 0)]
    arrays["save.single"] = b(single)
    before = dict(decoder.reception_stats)
    os.makedirs("recv", exist_ok=True)
    existing = set(glob.glob("recv/*"))
    with contextlib.redirect_stdout(io.StringIO()):
        saved = decoder.save_decoded_files(entries)
    stats = {k: decoder.reception_stats[k] - before[k] for k in ("total_files", "total_bytes")}
    rec = {"id": "save", "entries": [[e[0], e[2], e[3], e[4], e[5], e[6]] for e in entries],
           "saved_suffixes": [os.path.basename(p).split("_", 2)[2] for p in saved],
           "stats_delta": stats, "success_rate": decoder.reception_stats["success_rate"]}
    for k, e in enumerate(entries):
        arrays[f"save.entry.{k}"] = b(e[1])
    for k, p in enumerate(saved):
        with open(p, "rb") as f:
            arrays[f"save.out.{k}"] = b(f.read())
    assert not (set(glob.glob("recv/*")) - existing - set(saved))
    cases.append(rec)

    # --- decode_with_retry ------------------------------------------------------------------
    frame = synth.frame_data("r.bin", b"RAW" + rng.integers(0, 256, 150, dtype=np.uint8).tobytes())
    x = modem.qpsk_modulate(frame, baud=1500)
    x = (x + rng.normal(0, 0.02, x.size)).astype(np.float32)
    arrays["retry.x"] = x
    for mode, sr, tag in (("QPSK", 1500, "qpsk"), ("8PSK", 1500, "psk8"), ("FSK9600", 9600, "fsk"),
                          ("NOPE", 1500, "fallback")):
        for f in glob.glob("demodulated_attempt_*.bin"):
            os.remove(f)
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            out = decoder.decode_with_retry(x, mode, sr)
        dumps = sorted(glob.glob("demodulated_attempt_*.bin"))
        for f in dumps:
            with open(f, "rb") as fh:
                arrays[f"retry.{tag}.{os.path.basename(f)}"] = b(fh.read())
        cases.append({"id": f"retry.{tag}", "mode": mode, "symbol_rate": sr, "value": out,
                      "dumps": [os.path.basename(f) for f in dumps]})

    os.chdir(cwd)
    np.savez_compressed(os.path.join(HERE, "assembly.npz"), **arrays)
    with open(os.path.join(HERE, "assembly_manifest.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_assembly_golden.py", "cases": cases}, f, indent=0)
    print(f"{len(cases)} cases")


if __name__ == "__main__":
    main()
