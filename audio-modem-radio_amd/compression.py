"""Decompression tail of the receive path (host side).

Restates the decode half of the reference's utils/compression.py:
  intelligent_decompress  utils/compression.py:103-123
  delta_decompress        utils/compression.py:131-144 (vectorised: a running
                          byte sum mod 256 is a cumulative sum mod 256)
  delta_compress          utils/compression.py:114-128 (for round-trip tests)
The reference's off-by-one is kept on purpose: b'RAW' is a 3-byte tag but the
decoder strips 4 bytes (utils/compression.py:77 vs :114).
"""
from __future__ import annotations

import lzma
import zlib

import numpy as np


def delta_compress(data: bytes) -> bytes:
    if len(data) <= 1:
        return bytes(data)
    a = np.frombuffer(bytes(data), np.uint8)
    out = np.empty_like(a)
    out[0] = a[0]
    out[1:] = (a[1:].astype(np.int16) - a[:-1]) & 0xFF
    return out.tobytes()


def delta_decompress(compressed: bytes) -> bytes:
    if not compressed:
        return b''
    a = np.frombuffer(bytes(compressed), np.uint8).astype(np.uint64)
    return (np.cumsum(a) & 0xFF).astype(np.uint8).tobytes()


def intelligent_decompress(compressed_data: bytes) -> bytes:
    try:
        if compressed_data.startswith(b'LZMA'):
            return lzma.decompress(compressed_data[4:])
        elif compressed_data.startswith(b'DLZM'):
            return delta_decompress(lzma.decompress(compressed_data[4:]))
        elif compressed_data.startswith(b'ZLIB'):
            return zlib.decompress(compressed_data[4:])
        elif compressed_data.startswith(b'RAW'):
            return compressed_data[4:]
        else:
            try:
                return zlib.decompress(compressed_data)
            except Exception:
                return compressed_data
    except Exception as e:
        print(f"⚠️ Erro na descompressão inteligente: {e}")
        return compressed_data
