"""The crafted decoded-byte streams the frame-parse tests and their golden
generator share (tests/golden/make_frames_golden.py runs the REFERENCE's
decoder.parse_fbp_stream_enhanced, decoder.py:142-208, on exactly these).
Every branch of the reference's candidate checks is hit at least once."""
import binascii
import struct

import numpy as np


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
        b"FBPC" * 300 + ok1,                                   # more magics than the kernel keeps (256)
        frame(b"q", b"", dlen=5) + b"abc",                     # dlen > remaining: incomplete
        frame(b"w" * 255, rnd(33)),                            # longest name
        ok2 + ok2 + frame(b"v", rnd(9), part=1, total=2),      # repeated + multi-part headers
    ]
