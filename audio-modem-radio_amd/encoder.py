"""Drop-in for the reference's encoder.py (transmit orchestration).

`filebeep_advanced_v2.py:23` imports `encode_file, cancel_encoding,
get_encoding_stats` from here; the rest of the reference module's names are
kept too.  File handling, compression and framing stay on the host (once per
file); the per-sample work -- the modulators -- runs on the GPU through
`modem.*_modulate` (tx_kernels.hip), and `encode_files_batch` modulates many
files in ONE batched launch (`modem.modulate_batch`).

Reference map (encoder.py):
  get_file_signature / clear_encoding_cache   :27-35
  cancel_encoding / reset_encoding_cancel     :41-47
  adaptive_compress                           :50-60
  calculate_transmission_stats                :63-91
  _frame_data                                 :94-114
  split_file_for_transmission                 :117-151
  encode_file_parts                           :154-252
  encode_hellschreiber_text                   :255-257
  encode_file                                 :260-306
  get_encoding_stats                          :309-315
  verify_audio_output                         :318-348
Differences: CACHE_DIR is created when the first WAV is written, not at import
(the reference runs os.makedirs at import, encoder.py:20-21); HELLSCHREIBER
(hellschreiber.py) is outside this build's scope and raises
NotImplementedError.  The reference's modulator calls are kept as written, so
the ones that pass keywords the aliases do not take (8PSK, APSK16, DSSS, MSK,
FT8, PSK31, FELD_HELL in encode_file_parts) raise the same TypeError here.
"""
from __future__ import annotations

import binascii
import hashlib
import logging
import math
import os
from functools import lru_cache
from typing import List

import numpy as np

import modem
from compression import compress_data, delta_compress, intelligent_compress, super_compress
from modem import (SAMPLE_RATE, apsk16_modulate, bpsk_modulate, dsss_modulate, feld_hell_modulate,  # noqa: F401
                   fsk_high_speed_modulate, fsk_modulate, ft8_modulate, msk_modulate, ofdm_modulate_simple,
                   psk8_modulate, psk31_modulate, qpsk_modulate, wav_from_array)
from synth import frame_data

logger = logging.getLogger('filebeep')
CACHE_DIR = "cache"

# bytes/s per mode (encoder.py:66-73 and :127-134, identical tables)
def _efficiency(mode: str, symbol_rate: int) -> int:
    table = {
        "FSK1200": 100, "FSK9600": 800, "BPSK": symbol_rate // 8,
        "QPSK": symbol_rate // 4, "8PSK": (symbol_rate * 3) // 8,
        "FSK19200": 1600, "OFDM4": symbol_rate // 2, "OFDM8": symbol_rate,
        "SSTV": 50, "APSK16": symbol_rate * 4 // 8,
        "DSSS": symbol_rate // 16, "MSK": symbol_rate // 4, "HELLSCHREIBER": 15,
    }
    return table.get(mode, symbol_rate // 4)


@lru_cache(maxsize=50)
def get_file_signature(file_path: str, mode: str, compress: bool, symbol_rate: int) -> str:
    s = os.stat(file_path)
    return hashlib.md5(f"{file_path}_{s.st_size}_{s.st_mtime}_{mode}_{compress}_{symbol_rate}".encode()).hexdigest()


def clear_encoding_cache():
    get_file_signature.cache_clear()


_encoding_cancelled = False


def cancel_encoding():
    global _encoding_cancelled
    _encoding_cancelled = True


def reset_encoding_cancel():
    global _encoding_cancelled
    _encoding_cancelled = False


def adaptive_compress(data: bytes, mode: str) -> bytes:
    """encoder.py:50-60 (not utils.compression.adaptive_compress: 1 KiB floor, APSK16, delta pass)."""
    if len(data) < 1024:
        return data
    if mode in ["8PSK", "FSK19200", "OFDM4", "OFDM8", "APSK16"]:
        return delta_compress(super_compress(data))
    return compress_data(data)


def calculate_transmission_stats(file_size: int, mode: str, symbol_rate: int, compress: bool = True) -> dict:
    bytes_per_sec = _efficiency(mode, symbol_rate)
    compression_ratio = 0.4 if compress and mode not in ["SSTV", "HELLSCHREIBER"] else 1.0
    effective_size = file_size * compression_ratio
    duration_sec = effective_size / bytes_per_sec if bytes_per_sec > 0 else float('inf')
    return {
        'original_size': file_size,
        'effective_size': int(effective_size),
        'compression_ratio': compression_ratio,
        'bytes_per_sec': bytes_per_sec,
        'duration_sec': duration_sec,
        'duration_min': duration_sec / 60,
        'bitrate_bps': bytes_per_sec * 8,
    }


def _frame_data(fname: str, data: bytes, part_number: int = 0, total_parts: int = 1,
                file_size: int = 0, file_crc: int = 0) -> bytes:
    """encoder.py:94-114: b'FBPC' | len(name) | name[:255] | <IIIIII part, total,
    fsize, fcrc, dlen, pcrc> | data."""
    return frame_data(fname, data, part_number, total_parts, file_size, file_crc)


def split_file_for_transmission(file_path: str, mode: str, symbol_rate: int,
                                target_duration_sec: int = 60) -> List[tuple]:
    file_size = os.path.getsize(file_path)
    fname = os.path.basename(file_path)
    with open(file_path, 'rb') as f:
        file_data = f.read()
    file_crc = binascii.crc32(file_data) & 0xffffffff
    part_size = int(_efficiency(mode, symbol_rate) * target_duration_sec * 0.9)
    if file_size <= part_size:
        return [(fname, file_data, 0, 1, file_size, file_crc)]
    total_parts = math.ceil(file_size / part_size)
    parts = []
    for i in range(total_parts):
        start = i * part_size
        parts.append((f"{fname}.part{i + 1}", file_data[start:min(start + part_size, file_size)],
                      i, total_parts, file_size, file_crc))
    return parts


# encode_file_parts' modulator dispatch (encoder.py:179-212): mode -> (modulator,
# keyword arguments; SR stands for the call's symbol_rate).  The calls are the
# reference's, keywords included -- the aliases that do not take them raise the
# reference's TypeError.
_SR = object()
_PART_CALLS = {
    "FSK1200": (fsk_modulate, {"baud": 1200, "mark_freq": 1200.0, "space_freq": 2200.0}),
    "FSK9600": (fsk_modulate, {"baud": 9600}),
    "BPSK": (bpsk_modulate, {"baud": _SR, "carrier": 3000.0}),
    "QPSK": (qpsk_modulate, {"baud": _SR, "carrier": 3000.0}),
    "8PSK": (psk8_modulate, {"baud": _SR, "carrier": 12000.0}),
    "FSK19200": (fsk_high_speed_modulate, {"baud": 19200}),
    "OFDM4": (ofdm_modulate_simple, {"baud": _SR, "carrier": 12000.0, "num_subcarriers": 4}),
    "OFDM8": (ofdm_modulate_simple, {"baud": _SR, "carrier": 12000.0, "num_subcarriers": 8}),
    "APSK16": (apsk16_modulate, {"baud": _SR, "carrier": 12000.0}),
    "DSSS": (dsss_modulate, {"baud": _SR, "carrier": 3000.0}),
    "MSK": (msk_modulate, {"baud": _SR, "carrier": 6000.0}),
    "FT8": (ft8_modulate, {"baud": _SR, "carrier": 3000.0}),
    "PSK31": (psk31_modulate, {"baud": _SR, "carrier": 3000.0}),
    "FELD_HELL": (feld_hell_modulate, {"baud": 122.5, "carrier": 1000.0}),
}


def _modulate_part(framed: bytes, mode: str, symbol_rate: int) -> np.ndarray:
    if mode == "HELLSCHREIBER":
        raise NotImplementedError("Hellschreiber (hellschreiber.py) is outside this build's scope (SURVEY §2)")
    if mode not in _PART_CALLS:
        raise ValueError(f"Modo desconhecido: {mode}")
    fn, kw = _PART_CALLS[mode]
    return fn(framed, **{k: (symbol_rate if v is _SR else v) for k, v in kw.items()})


def _test_tone(n_framed: int, symbol_rate: float) -> np.ndarray:
    """Last-resort 1 kHz tone of encode_file_parts (encoder.py:225-228)."""
    duration = max(n_framed / symbol_rate, 1.0)
    t = np.linspace(0, duration, int(SAMPLE_RATE * duration))
    return 0.8 * np.sin(2 * np.pi * 1000 * t).astype(np.float32)


def _write_wav(outname: str, wavb: bytes) -> None:
    os.makedirs(os.path.dirname(outname) or ".", exist_ok=True)
    with open(outname, 'wb') as wf:
        wf.write(wavb)


def encode_file_parts(file_parts: List[tuple], mode: str, compress: bool, symbol_rate: int,
                      progress_callback=None, is_cancelled=None) -> List[str]:
    """encoder.py:154-252: per part adaptive_compress -> frame -> modulate; invalid
    audio falls back to BPSK at min(symbol_rate, 4800), then to a test tone."""
    written = []
    for k, (fname, data, part_number, total_parts, file_size, file_crc) in enumerate(file_parts):
        if is_cancelled and is_cancelled():
            raise RuntimeError("Codificação cancelada pelo usuário")
        payload = adaptive_compress(data, mode) if compress else data
        framed = _frame_data(fname, payload, part_number, total_parts, file_size, file_crc)
        audio = _modulate_part(framed, mode, symbol_rate)
        if not verify_audio_output(audio):
            slow = min(symbol_rate, 4800)
            audio = bpsk_modulate(framed, baud=slow, carrier=3000.0)
            if not verify_audio_output(audio):
                audio = _test_tone(len(framed), slow)
                if not verify_audio_output(audio):
                    raise ValueError(
                        "Falha crítica na geração de áudio modulado - não foi possível produzir áudio válido")
        wav = wav_from_array(audio, SAMPLE_RATE)
        if len(wav) < 100:
            logger.warning("WAV under 100 bytes for %s", fname)
        path = os.path.join(CACHE_DIR, f"{fname}.{mode}.sr{symbol_rate}.wav")
        _write_wav(path, wav)
        if not (os.path.exists(path) and os.path.getsize(path) > 100):
            raise IOError(f"Falha ao salvar arquivo codificado: {path}")
        written.append(path)
        if progress_callback:
            progress_callback(k + 1, total_parts)
    return written


def encode_hellschreiber_text(text: str):
    return "hellschreiber.wav"  # encoder.py:255-257 (placeholder in the reference too)


def _encode_framed(path: str, compress: bool):
    fname = os.path.basename(path)
    with open(path, 'rb') as f:
        raw_data = f.read()
    file_crc = binascii.crc32(raw_data) & 0xffffffff
    data = intelligent_compress(raw_data) if compress else raw_data
    return fname, _frame_data(fname, data, 0, 1, len(raw_data), file_crc)


# encode_file's mode -> (batched tx kind, baud, f0, f1) (encoder.py:283-294);
# every other mode falls back to QPSK at symbol_rate, as the reference does.
def _encode_file_modulator(mode: str, symbol_rate: int):
    if mode == "FSK1200":
        return "fsk", 1200, 1200.0, 2200.0
    if mode == "FSK9600":
        return "fsk", 9600, 1200.0, 2200.0
    if mode == "FSK19200":
        return "fsk", 19200, 8000.0, 16000.0
    if mode == "BPSK":
        return "bpsk", symbol_rate, 3000.0, 0.0
    return "qpsk", symbol_rate, 3000.0, 0.0


def encode_file(path: str, mode: str = "QPSK", compress: bool = True,
                symbol_rate: int = 9600, split_large_files: bool = True,
                target_duration_min: int = 1, progress_callback=None,
                is_cancelled=None) -> str:
    """encoder.py:260-306: intelligent_compress -> FBPC frame -> modulate -> WAV in CACHE_DIR.
    Returns the WAV path, or "" when the modulator raises (logged, as the reference)."""
    global _encoding_cancelled
    _encoding_cancelled = False
    fname, framed = _encode_framed(path, compress)
    logger.info(f"Modulando {len(framed)} bytes em modo {mode}...")
    kind, baud, f0, f1 = _encode_file_modulator(mode, symbol_rate)
    try:
        if kind == "fsk":
            arr = fsk_modulate(framed, baud=baud, mark_freq=f0, space_freq=f1)
        elif kind == "bpsk":
            arr = bpsk_modulate(framed, baud=baud)
        else:
            arr = qpsk_modulate(framed, baud=baud)
    except Exception as e:
        logger.error(f"Erro modulando: {e}")
        return ""
    outname = os.path.join(CACHE_DIR, f"{fname}.{mode}.wav")
    _write_wav(outname, wav_from_array(arr, SAMPLE_RATE))
    return outname


def encode_files_batch(paths, mode: str = "QPSK", compress: bool = True, symbol_rate: int = 9600) -> List[str]:
    """Batched encode_file: host compression + framing per file, then every
    file's waveform in ONE GPU launch (modem.modulate_batch, pcm=True) and one
    WAV per file -- byte-identical to calling encode_file on each path."""
    if not paths:
        return []
    framed = [_encode_framed(p, compress) for p in paths]
    kind, baud, f0, f1 = _encode_file_modulator(mode, symbol_rate)
    _, pcm = modem.modulate_batch(kind, [fr for _, fr in framed], baud, f0, f1, pcm=True)
    import _amr
    outs = []
    for i, (fname, fr) in enumerate(framed):
        n = _amr.tx_samples(_amr.TX_MODES[kind], len(fr), baud, SAMPLE_RATE)
        outname = os.path.join(CACHE_DIR, f"{fname}.{mode}.wav")
        _write_wav(outname, _pcm_wav(pcm[i, :n], SAMPLE_RATE))
        outs.append(outname)
    return outs


def _pcm_wav(pcm: np.ndarray, sr: int) -> bytes:
    import io
    import wave
    bio = io.BytesIO()
    with wave.open(bio, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sr)
        wf.writeframes(np.ascontiguousarray(pcm, np.int16).tobytes())
    return bio.getvalue()


def get_encoding_stats(file_path, mode, compress, symbol_rate):
    """encoder.py:309-315 (a stub in the reference too)."""
    sz = os.path.getsize(file_path)
    return {
        'original_size': sz, 'effective_size': sz, 'compression_ratio': 1.0,
        'bytes_per_sec': symbol_rate / 4, 'duration_min': 1.0, 'bitrate_bps': symbol_rate,
    }


# encoder.py:321-330, in the reference's order (a failure is logged by name)
_AUDIO_CHECKS = (
    ("Array não é None", lambda a: a is not None),
    ("Array não vazio", lambda a: len(a) > 0),
    ("Não é tudo zero", lambda a: not np.all(a == 0)),
    ("Duração mínima", None),                       # needs expected_min_duration
    ("Tem variação", lambda a: np.std(a) >= 0.01),
    ("Sem NaN", lambda a: not np.any(np.isnan(a))),
    ("Sem infinitos", lambda a: not np.any(np.isinf(a))),
    ("Valores dentro do range", lambda a: np.all(np.abs(a) <= 1.0)),
)


def verify_audio_output(audio_array: np.ndarray, expected_min_duration: float = 0.1) -> bool:
    """encoder.py:318-348: True when every check passes."""
    failed = []
    for name, pred in _AUDIO_CHECKS:
        ok = (len(audio_array) / SAMPLE_RATE >= expected_min_duration) if pred is None else pred(audio_array)
        if not ok:
            failed.append(name)
    if failed:
        logger.error("audio rejected: %s", ", ".join(failed))
        return False
    return True
