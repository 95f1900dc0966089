"""Compression around the modem path (host side).

Restates the reference's utils/compression.py (host zlib/lzma; no GPU work --
these run once per file, not per sample):
  decode half (receive tail, decoder.py:447):
    intelligent_decompress  utils/compression.py:103-123
    delta_decompress        utils/compression.py:260-273 (vectorised: a running
                            byte sum mod 256 is a cumulative sum mod 256)
    decompress_data         utils/compression.py:159-165
    super_decompress        utils/compression.py:229-240
  encode half (encoder.encode_file, encoder.py:276):
    IntelligentCompressor   utils/compression.py:11-69 (entropy, repeated
                            fixed-stride blocks, text sniff -- vectorised)
    intelligent_compress    utils/compression.py:72-100
    compress_data           utils/compression.py:152-156
    super_compress          utils/compression.py:201-226
    delta_compress          utils/compression.py:243-257
    adaptive_compress       utils/compression.py:276-285
The reference's off-by-one is kept on purpose: b'RAW' is a 3-byte tag but the
decoder strips 4 bytes (utils/compression.py:77 vs :114), so a RAW-tagged
payload loses its first byte on the way back.  The reference reads its
switches from config.CONFIG (config.py:34-39, all enabled by default); here
they are the module-level COMPRESSION dict with the same keys and defaults.
"""
from __future__ import annotations

import math
import lzma
import zlib

import numpy as np

LZMA_AVAILABLE = True
# config.py:34-39 ('compression.*'), defaults of the reference's ConfigManager
COMPRESSION = {"enabled": True, "aggressive_threshold": 1024,
               "lzma_enabled": True, "delta_compression": True}


class IntelligentCompressor:
    """utils/compression.py:11-69: picks 'none' / 'lzma' / 'zlib' / 'delta+lzma'."""

    def __init__(self):
        self.compression_stats = {}
        self.enabled = COMPRESSION.get("enabled", True)

    def analyze_data_pattern(self, data: bytes) -> dict:
        if len(data) < 100:
            return {"recommended": "none", "ratio": 1.0}
        a = np.frombuffer(bytes(data), np.uint8)
        # byte histogram in first-occurrence order: the reference sums the
        # entropy terms in dict insertion order (utils/compression.py:22-30)
        _, first, counts = np.unique(a, return_index=True, return_counts=True)
        total = len(a)
        entropy = 0
        for c in counts[np.argsort(first)]:
            p = int(c) / total
            entropy -= p * math.log2(p)
        repeated = self._detect_repeated_patterns(data)
        is_text = self._is_likely_text(data)
        if entropy < 2.0 or repeated:
            return {"recommended": "lzma", "ratio": 0.3, "entropy": entropy}
        elif is_text:
            return {"recommended": "zlib", "ratio": 0.5, "entropy": entropy}
        return {"recommended": "delta+lzma", "ratio": 0.4, "entropy": entropy}

    def _detect_repeated_patterns(self, data: bytes, min_pattern=4, max_pattern=32) -> bool:
        """utils/compression.py:44-56: some block of length L at offsets 0, L, 2L, ...
        (offsets < len-L) occurs more than 3 times, for any L in [min, min(max, len//10))."""
        n = len(data)
        if n < min_pattern * 10:
            return False
        a = np.frombuffer(bytes(data), np.uint8)
        for L in range(min_pattern, min(max_pattern, n // 10)):
            k = len(range(0, n - L, L))
            if k <= 3:
                continue
            blocks = np.ascontiguousarray(a[:k * L]).view(np.dtype((np.void, L)))
            _, cnt = np.unique(blocks, return_counts=True)
            if cnt.max() > 3:
                return True
        return False

    def _is_likely_text(self, data: bytes) -> bool:
        if len(data) == 0:
            return False
        head = np.frombuffer(bytes(data[:1000]), np.uint8)
        text = np.count_nonzero(((head >= 32) & (head <= 126)) | (head == 9) | (head == 10) | (head == 13))
        return text / min(1000, len(data)) > 0.8


def intelligent_compress(data: bytes, mode: str = "auto") -> bytes:
    """utils/compression.py:72-100 (tags LZMA / DLZM / ZLIB / RAW)."""
    data = bytes(data)
    compressor = IntelligentCompressor()
    if not COMPRESSION.get("enabled", True) or len(data) < 200:
        return b'RAW' + data
    if mode == "auto":
        mode = compressor.analyze_data_pattern(data)["recommended"]
    try:
        if mode == "lzma" and COMPRESSION.get("lzma_enabled", True):
            return b'LZMA' + lzma.compress(data, preset=9)
        elif mode == "delta+lzma" and COMPRESSION.get("delta_compression", True):
            return b'DLZM' + lzma.compress(delta_compress(data), preset=9)
        return b'ZLIB' + zlib.compress(data, level=9)
    except Exception as e:
        print(f"⚠️ Erro na compressão inteligente, usando fallback: {e}")
        return b'RAW' + data


def compress_data(data: bytes, level=9) -> bytes:
    """utils/compression.py:152-156: untagged zlib, identity under 100 bytes."""
    if len(data) < 100:
        return data
    return zlib.compress(data, level)


def decompress_data(b: bytes) -> bytes:
    """utils/compression.py:159-165."""
    try:
        return zlib.decompress(b)
    except zlib.error:
        return b


def super_compress(data: bytes) -> bytes:
    """utils/compression.py:201-226: LZMA when it beats zlib by 20 % (inputs over 1000 B)."""
    data = bytes(data)
    if len(data) < 500:
        return b'RAW' + data
    try:
        z = zlib.compress(data, level=9)
        if len(data) > 1000:
            x = lzma.compress(data, preset=9)
            if len(x) < len(z) * 0.8:
                return b'LZMA' + x
        return b'ZLIB' + z
    except Exception as e:
        print(f"Erro na super compressão, usando dados brutos: {e}")
        return b'RAW' + data


def super_decompress(b: bytes) -> bytes:
    """utils/compression.py:229-240 (same RAW off-by-one as intelligent_decompress)."""
    if b.startswith(b'LZMA'):
        return lzma.decompress(b[4:])
    elif b.startswith(b'ZLIB'):
        return zlib.decompress(b[4:])
    elif b.startswith(b'RAW'):
        return b[4:]
    return decompress_data(b)


def adaptive_compress(data: bytes, mode: str) -> bytes:
    """utils/compression.py:276-285 (the encoder has its own variant, encoder.adaptive_compress)."""
    if len(data) < 200:
        return data
    if mode in ["8PSK", "FSK19200", "OFDM4", "OFDM8"]:
        return super_compress(data)
    return compress_data(data)


def delta_compress(data: bytes) -> bytes:
    """utils/compression.py:243-257: first byte, then byte-to-byte differences mod 256."""
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


def prepare_sstv_like(path: str, jpeg_quality=30, max_size=(400, 300)) -> bytes:
    """utils/compression.py:168-196: image -> RGB thumbnail -> JPEG -> zlib(6);
    anything else (or no PIL) -> zlib(6) of the file."""
    try:
        from PIL import Image
    except ImportError:
        Image = None
    import os
    from io import BytesIO
    if Image is not None and os.path.splitext(path)[1].lower() in {'.jpg', '.jpeg', '.png', '.bmp', '.gif', '.tiff'}:
        try:
            img = Image.open(path)
            if img.mode != 'RGB':
                img = img.convert('RGB')
            img.thumbnail(max_size, Image.Resampling.LANCZOS)
            buf = BytesIO()
            img.save(buf, format="JPEG", quality=jpeg_quality, optimize=True)
            return zlib.compress(buf.getvalue(), level=6)
        except Exception as e:
            print(f"Erro no processamento de imagem, usando compressão padrão: {e}")
    with open(path, "rb") as f:
        return zlib.compress(f.read(), level=6)
