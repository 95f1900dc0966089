#!/usr/bin/env python3
"""Frame-parse fixtures from the REFERENCE itself (this container only).

Runs the reference's decoder.parse_fbp_stream_enhanced (decoder.py:142-208)
on every crafted stream of tests/frame_streams.py and records, per stream,
the frames it returns (name, payload, final_crc) and everything it prints.
Nothing of the reference is copied: frames.json holds data only (the input
streams as hex and the reference's outputs).

Run:  python tests/golden/make_frames_golden.py        (needs /root/reference)
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))          # tests/ (frame_streams)
sys.path.insert(0, HERE)

import frame_streams  # noqa: E402
from make_golden import _import_reference  # noqa: E402


def main():
    out_path = os.path.join(HERE, "frames.json")
    scratch = tempfile.mkdtemp(prefix="amr_frames_")
    cwd = os.getcwd()
    _, _, decoder = _import_reference(scratch)
    cases = []
    for i, raw in enumerate(frame_streams.streams()):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            frames = decoder.parse_fbp_stream_enhanced(raw)
        cases.append({"id": i, "raw": raw.hex(),
                      "frames": [{"name": f["name"], "data": bytes(f["data"]).hex(), "final_crc": int(f["final_crc"])}
                                 for f in frames],
                      "log": buf.getvalue()})
    os.chdir(cwd)
    with open(out_path, "w") as f:
        json.dump({"generator": "tests/golden/make_frames_golden.py",
                   "reference": "decoder.parse_fbp_stream_enhanced (decoder.py:142-208)", "cases": cases}, f)
    print(f"{len(cases)} frame-parse cases -> {out_path}")


if __name__ == "__main__":
    main()
