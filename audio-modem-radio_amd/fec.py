"""fec.py -- drop-in for the reference's fec module; decode runs on the GPU.

  ReedSolomonFEC.encode   fec.py:11-32  (host; transmit side)
  ReedSolomonFEC.decode   fec.py:34-69  -> k_fec_decode (util_kernels.hip)
  ReedSolomonFEC.decode_batch           batched form (one wave per stream)
Despite its name the reference "Reed-Solomon" is parity-XOR triples plus a
CRC32 trailer; that is what is reproduced, bit for bit.
ConvolutionalEncoder / ViterbiDecoder (fec.py:72-155) are kept as plain
host code for import compatibility; they are outside the hot path.
"""
from __future__ import annotations

import struct
import zlib

import _amr


class ReedSolomonFEC:
    def __init__(self, nsym=32):
        self.nsym = nsym

    def encode(self, data: bytes) -> bytes:
        """fec.py:11-32: (b1, b2, b1^b2) triples, odd tail padded with 0xFF, CRC32 LE."""
        encoded = bytearray()
        for i in range(0, len(data), 2):
            if i + 1 < len(data):
                b1, b2 = data[i], data[i + 1]
                encoded.extend([b1, b2, b1 ^ b2])
            else:
                encoded.append(data[i])
                encoded.append(0xFF)
        encoded.extend(struct.pack('<I', zlib.crc32(data) & 0xFFFFFFFF))
        return bytes(encoded)

    def decode(self, data: bytes) -> bytes:
        """fec.py:34-69 on the GPU; prints the reference's warning on a CRC mismatch."""
        if len(data) < 4:
            return data
        out, ok = _amr.fec_decode_host([data])
        if not ok[0]:
            print("Aviso: CRC não corresponde - dados podem estar corrompidos")
        return out[0]

    def decode_batch(self, datas, warn: bool = False):
        """Decode many byte strings in one launch. Returns (list[bytes], list[crc_ok])."""
        outs, oks = _amr.fec_decode_host(datas)
        if warn:
            for d, ok in zip(datas, oks):
                if len(d) >= 4 and not ok:
                    print("Aviso: CRC não corresponde - dados podem estar corrompidos")
        return outs, oks


class ConvolutionalEncoder:
    """fec.py:72-111 (rate 1/2, K=7, polynomials 171/133 octal)."""

    def __init__(self, constraint_length=7):
        self.constraint_length = constraint_length
        self.g1 = 0b1111001
        self.g2 = 0b1011011

    def encode(self, data: bytes) -> bytes:
        bits = []
        sr = 0
        for byte in data:
            for bp in range(8):
                sr = ((sr << 1) | ((byte >> (7 - bp)) & 1)) & 0x7F
                bits += [bin(sr & self.g1).count('1') % 2, bin(sr & self.g2).count('1') % 2]
        for _ in range(6):
            sr = (sr << 1) & 0x7F
            bits += [bin(sr & self.g1).count('1') % 2, bin(sr & self.g2).count('1') % 2]
        out = bytearray()
        for i in range(0, len(bits), 8):
            v = 0
            for j in range(8):
                if i + j < len(bits):
                    v = (v << 1) | bits[i + j]
            out.append(v)
        return bytes(out)


class ViterbiDecoder:
    """fec.py:114-155 -- the reference's stub (it does not invert the encoder)."""

    def __init__(self, constraint_length=7):
        self.constraint_length = constraint_length
        self.g1 = 0b1111001
        self.g2 = 0b1011011
        self.trellis = {}

    def decode(self, data: bytes) -> bytes:
        bits = [(byte >> (7 - i)) & 1 for byte in data for i in range(8)]
        if len(bits) >= 12:
            bits = bits[:-12]
        used = bits[0::2]
        out = bytearray()
        for i in range(0, len(used), 8):
            v = 0
            for j in range(8):
                if i + j < len(used):
                    v = (v << 1) | used[i + j]
            out.append(v)
        return bytes(out)
