"""GPU frame parse (k_frame_parse) against the REFERENCE's own
decoder.parse_fbp_stream_enhanced (decoder.py:142-208) output on the same
streams (tests/golden/frames.json, written by make_frames_golden.py): the
same frames (name, payload, final_crc) and the same log lines, stream by
stream, over every branch of the reference's candidate checks."""
import contextlib
import io

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


from frame_streams import streams  # noqa: E402  (shared with tests/golden/make_frames_golden.py)


def golden_frames():
    import json
    import os
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "frames.json")) as f:
        return json.load(f)["cases"]


def host_parse(raw):
    import decoder
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = decoder.parse_fbp_stream_enhanced(raw)
    return res, buf.getvalue()


@pytest.mark.parametrize("max_cands", [64, 256])
def test_batch_parse_matches_reference_fixtures(max_cands):
    """The GPU batch parse == the reference's frames and log lines, per stream
    (streams with more magics than max_cands take the host restatement)."""
    import decoder
    cases = golden_frames()
    raws = [bytes.fromhex(c["raw"]) for c in cases]
    assert raws == streams()
    for raw, c in zip(raws, cases):
        buf = io.StringIO()
        with contextlib.redirect_stdout(buf):
            got = decoder.parse_fbp_stream_enhanced_batch([raw], max_cands=max_cands)[0]
        assert [{"name": f["name"], "data": bytes(f["data"]).hex(), "final_crc": int(f["final_crc"])}
                for f in got] == c["frames"], c["id"]
        assert buf.getvalue() == c["log"], c["id"]
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        allg = decoder.parse_fbp_stream_enhanced_batch(raws, max_cands=max_cands)   # one launch, all streams
    assert [[{"name": f["name"], "data": bytes(f["data"]).hex(), "final_crc": int(f["final_crc"])} for f in g]
            for g in allg] == [c["frames"] for c in cases]
    assert buf.getvalue() == "".join(c["log"] for c in cases)


def test_records_follow_the_reference_checks():
    import _amr
    raws = streams()
    res = _amr.frame_parse(raws, max_cands=64)
    st = lambda i: [int(r["status"]) for r in res[i][1]]   # noqa: E731
    assert res[0][0] == 0 and res[0][1].size == 0
    assert st(2) == [_amr.FRAME_OK]
    assert st(3) == [_amr.FRAME_OK, _amr.FRAME_OK]
    assert st(4) == [_amr.FRAME_CRC_BAD]
    assert st(5) == [_amr.FRAME_INCOMPLETE]
    assert st(6) == [_amr.FRAME_NONAME]
    assert st(7)[0] == _amr.FRAME_BADLEN and st(8)[0] == _amr.FRAME_BADLEN
    assert st(9) == [_amr.FRAME_SHORT]
    assert st(10) == [_amr.FRAME_NOMETA]
    assert res[13][0] == 101                     # counted beyond max_cands
    r = res[2][1][0]
    assert (int(r["part"]), int(r["total"])) == (2, 5)
    assert int(r["calc_crc"]) == int(r["pcrc"])


def test_many_streams_and_the_demod_output():
    """A batch of demodulated streams: QPSK @ 1000 Bd (round-trips in the
    reference) carrying real frames, parsed on the GPU == parsed on the host."""
    import decoder
    import modem
    import synth
    rng = np.random.default_rng(3)
    fr = [synth.random_frame(rng, 200 + 10 * i, name=f"f{i}.bin") for i in range(6)]
    N = max(len(synth.qpsk_waveform(f, 1000)) for f in fr) + 960
    x = np.stack([synth.fit(synth.qpsk_waveform(f, 1000), N) + rng.normal(0, 0.02, N).astype(np.float32) for f in fr])
    raws = modem.qpsk_demodulate_batch(x, baud=1000)
    with contextlib.redirect_stdout(io.StringIO()):
        got = decoder.parse_fbp_stream_enhanced_batch(raws)
    for raw, g in zip(raws, got):
        w, _ = host_parse(raw)
        assert g == w
    assert sum(len(g) for g in got) >= 1
