"""The host restatement of decoder.parse_fbp_stream_enhanced (decoder.py:142-208)
against the reference's own output on the crafted streams (CPU; the GPU parse
is checked against the same fixtures in test_gpu_frames.py)."""
import contextlib
import io
import json
import os

from frame_streams import streams

HERE = os.path.dirname(os.path.abspath(__file__))


def test_fixture_streams_are_the_shared_ones():
    with open(os.path.join(HERE, "golden", "frames.json")) as f:
        cases = json.load(f)["cases"]
    assert [bytes.fromhex(c["raw"]) for c in cases] == streams()


def test_host_parse_matches_reference_fixtures():
    import decoder
    with open(os.path.join(HERE, "golden", "frames.json")) as f:
        cases = json.load(f)["cases"]
    for c in cases:
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            got = decoder.parse_fbp_stream_enhanced(bytes.fromhex(c["raw"]))
        assert [{"name": f["name"], "data": bytes(f["data"]).hex(), "final_crc": int(f["final_crc"])}
                for f in got] == c["frames"], c["id"]
        assert buf.getvalue() == c["log"], c["id"]
