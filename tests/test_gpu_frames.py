"""GPU frame parse (k_frame_parse) against the host restatement of
the reference's decoder.parse_fbp_stream_enhanced (decoder.py:142-208): the
same frames (name, payload, final_crc) and the same log lines, stream by
stream, over every branch of the reference's candidate checks."""
import binascii
import contextlib
import io
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def frame(name: bytes, payload: bytes, part=0, total=1, fsize=None, fcrc=0x1234, pcrc=None, dlen=None) -> bytes:
    meta = struct.pack('<IIIIII', part, total, len(payload) if fsize is None else fsize, fcrc,
                       len(payload) if dlen is None else dlen,
                       (binascii.crc32(payload) & 0xFFFFFFFF) if pcrc is None else pcrc)
    return b'FBPC' + bytes([len(name)]) + name + meta + payload


def streams():
    rng = np.random.default_rng(11)
    rnd = lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()   # noqa: E731
    ok1 = frame(b"a.txt", b"RAW" + rnd(300), part=2, total=5)
    ok2 = frame("ção.bin".encode(), rnd(1000))
    return [
        b"",                                                   # nothing
        rnd(2000),                                             # noise
        ok1,                                                   # one valid frame
        rnd(37) + ok1 + rnd(5) + ok2 + rnd(11),                # two frames, unaligned
        frame(b"x", rnd(64), pcrc=0xDEADBEEF),                 # CRC error
        frame(b"y", rnd(64))[:-10],                            # payload past the end
        b"FBPC" + bytes([0]) + rnd(40),                        # name_len == 0
        frame(b"z", rnd(8), dlen=0) + rnd(8),                  # dlen == 0
        frame(b"z", rnd(8), dlen=60_000_000) + rnd(8),         # absurd dlen
        rnd(10) + b"FBPC" + rnd(20),                           # start + 30 > len
        b"FBPC" + bytes([200]) + rnd(60),                      # meta past the end
        b"FBPCFBPC" + ok1,                                     # overlapping magics
        ok1 + b"FBPC",                                         # magic in the last 4 bytes
        b"FBPC" * 100 + ok2,                                   # more magics than max_cands
        rnd(5000) + ok2 + rnd(3000) + ok1,                     # long stream
        frame(b"\xff\xfe", rnd(17)),                           # undecodable name bytes
    ]


def host_parse(raw):
    import decoder
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        res = decoder.parse_fbp_stream_enhanced(raw)
    return res, buf.getvalue()


def test_batch_parse_matches_host_parse():
    import decoder
    raws = streams()
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        got = decoder.parse_fbp_stream_enhanced_batch(raws, max_cands=64)
    want_log = []
    for raw, g in zip(raws, got):
        w, log = host_parse(raw)
        assert g == w
        want_log.append(log)
    assert buf.getvalue() == "".join(want_log)


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
