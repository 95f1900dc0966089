"""decoder.py -- drop-in for the reference's decoder module (host side).

Keeps the call surface filebeep_advanced_v2.py:24 imports
(decode_wav_file, decode_from_buffer, get_assembly_status, get_reception_stats)
with the reference's dispatch, frame parsing, decompression, file writing and
error behaviour; the demodulation itself runs on the MI355X via modem.py.

  decode_wav_file            decoder.py:380-389
  decode_from_buffer         decoder.py:417-464   (+ decode_from_buffer_batch)
  parse_fbp_stream_enhanced  decoder.py:142-208   (+ parse_fbp_stream_enhanced_batch:
                             the scan and payload CRCs on the GPU, k_frame_parse)
  smart_decompress           decoder.py:210-243
  find_frame_start           decoder.py:470-478
  get_assembly_status / get_reception_stats / clear_reception_stats
                             decoder.py:467, 481-513

Differences, all outside the hot path: ./recv is created on first write
rather than at import time, and WAV files are read with soundfile when it is
installed, else with the stdlib wave module using libsndfile's default
PCM16 -> float64 normalisation (int16 / 32768).
"""
from __future__ import annotations

import binascii
import os
import struct
import time
import traceback
import wave
from typing import Dict

import numpy as np

import _amr
import modem
from compression import intelligent_decompress, delta_decompress

SAMPLE_RATE = modem.SAMPLE_RATE
RECV_DIR = "recv"
active_file_assemblies: Dict[str, object] = {}
file_assemblies: dict = {}


def _fresh_stats():
    return {'total_files': 0, 'total_bytes': 0, 'success_rate': 0.0, 'last_reception': None,
            'average_quality': 0.0, 'duplicates_rejected': 0, 'parts_reordered': 0,
            'total_quality': 0.0, 'quality_samples': 0}


reception_stats = _fresh_stats()


# ---------------------------------------------------------------------------
def parse_fbp_stream_enhanced(raw: bytes) -> list:
    """Find every b'FBPC' frame with a valid CRC32 payload (decoder.py:142-208)."""
    parsed_files = []
    magic = b'FBPC'
    start_indices = []
    offset = 0
    while True:
        idx = raw.find(magic, offset)
        if idx == -1:
            break
        start_indices.append(idx)
        offset = idx + 1
    print(f"Encontrados {len(start_indices)} candidatos a cabeçalho.")
    for start in start_indices:
        try:
            if start + 30 > len(raw):
                continue
            name_len = raw[start + 4]
            if name_len == 0:
                continue
            name_start = start + 5
            fname = raw[name_start: name_start + name_len].decode('utf-8', 'ignore')
            meta_start = name_start + name_len
            if meta_start + 24 > len(raw):
                continue
            (part_num, total_parts, fsize, fcrc, dlen, pcrc) = struct.unpack('<IIIIII', raw[meta_start:meta_start + 24])
            if dlen > 50_000_000 or dlen == 0:
                continue
            payload_start = meta_start + 24
            if payload_start + dlen > len(raw):
                print(f"Dados incompletos para {fname}")
                continue
            payload = raw[payload_start: payload_start + dlen]
            calc_crc = binascii.crc32(payload) & 0xffffffff
            if calc_crc == pcrc:
                print(f"✅ CRC VÁLIDO: {fname} (Parte {part_num + 1}/{total_parts})")
                parsed_files.append({'name': fname, 'data': payload, 'final_crc': fcrc})
            else:
                print(f"❌ Erro de CRC para {fname}")
        except Exception as e:
            print(f"Erro no parse candidato {start}: {e}")
    return parsed_files


def parse_fbp_stream_enhanced_batch(raws, max_cands: int = 64) -> list:
    """parse_fbp_stream_enhanced over a batch of decoded streams, the scan on
    the GPU (k_frame_parse: magic search, the reference's checks, payload
    CRC32); the same frames and log lines per stream as the host version.  A
    stream with more than max_cands magics is parsed on the host instead."""
    import _amr
    out = []
    for raw, (n, recs) in zip(raws, _amr.frame_parse(raws, max_cands)):
        if n > max_cands:
            out.append(parse_fbp_stream_enhanced(raw))
            continue
        print(f"Encontrados {n} candidatos a cabeçalho.")
        parsed = []
        for r in recs:
            st = int(r["status"])
            if st < _amr.FRAME_INCOMPLETE:       # short / no name / no meta / bad length: silent
                continue
            ns, nl = int(r["name_start"]), int(r["name_len"])
            fname = raw[ns: ns + nl].decode('utf-8', 'ignore')
            if st == _amr.FRAME_INCOMPLETE:
                print(f"Dados incompletos para {fname}")
            elif st == _amr.FRAME_OK:
                ps = int(r["payload_start"])
                print(f"✅ CRC VÁLIDO: {fname} (Parte {int(r['part']) + 1}/{int(r['total'])})")
                parsed.append({'name': fname, 'data': raw[ps: ps + int(r["dlen"])], 'final_crc': int(r["fcrc"])})
            else:
                print(f"❌ Erro de CRC para {fname}")
        out.append(parsed)
    return out


def smart_decompress(compressed_data: bytes) -> bytes:
    """decoder.py:210-243."""
    import lzma
    import zlib
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


# ---------------------------------------------------------------------------
def _read_wav(path: str):
    try:
        import soundfile as sf  # the reference's reader (decoder.py:381)
        return sf.read(path)
    except ImportError:
        pass
    with wave.open(path, 'rb') as w:
        sr = w.getframerate()
        nch = w.getnchannels()
        width = w.getsampwidth()
        raw = w.readframes(w.getnframes())
    if width != 2:
        raise ValueError(f"only 16-bit PCM WAV is supported without soundfile (got {8 * width}-bit)")
    data = np.frombuffer(raw, dtype='<i2').astype(np.float64) / 32768.0
    if nch > 1:
        data = data.reshape(-1, nch)
    return data, sr


def decode_wav_file(path: str, mode: str, symbol_rate: int) -> list:
    """decoder.py:380-389: read, channel 0, FFT-resample to 96 kHz (GPU), decode."""
    data, sr = _read_wav(path)
    if len(data.shape) > 1:
        data = data[:, 0]
    if sr != SAMPLE_RATE:
        number_of_samples = int(round(len(data) * float(SAMPLE_RATE) / sr))
        data = _amr.resample(np.asarray(data, np.float64), number_of_samples)   # scipy.signal.resample, on the GPU
    return decode_from_buffer(data, mode, symbol_rate)


def _demod_bytes(data, mode: str, symbol_rate):
    """The reference's mode dispatch (decoder.py:421-434)."""
    if mode == "BPSK":
        return modem.bpsk_demodulate(data, baud=symbol_rate)
    elif mode == "QPSK" or mode == "8PSK":
        return modem.qpsk_demodulate(data, baud=symbol_rate)
    elif mode.startswith("FSK"):
        baud = 1200
        if "9600" in mode:
            baud = 9600
        elif "19200" in mode:
            baud = 19200
        return modem.fsk_demodulate(data, baud=baud)
    else:
        return modem.qpsk_demodulate(data, baud=symbol_rate)


def _save_frames(raw_bytes: bytes, frames=None) -> list:
    if frames is None:
        frames = parse_fbp_stream_enhanced(raw_bytes)
    saved = []
    for frame in frames:
        try:
            final_data = intelligent_decompress(frame['data'])
            ts = int(time.time())
            clean_name = os.path.basename(frame['name'])
            os.makedirs(RECV_DIR, exist_ok=True)
            path = os.path.join(RECV_DIR, f"{ts}_{clean_name}")
            with open(path, 'wb') as f:
                f.write(final_data)
            saved.append(path)
        except Exception as e:
            print(f"Erro salvando arquivo: {e}")
    return saved


def decode_from_buffer(data: np.ndarray, mode: str, symbol_rate: int) -> list:
    """decoder.py:417-464: demodulate, parse frames, decompress, save; [] on any error."""
    print(f"Demodulando {len(data)} amostras em modo {mode}...")
    try:
        raw_bytes = _demod_bytes(data, mode, symbol_rate)
        print(f"Bytes brutos demodulados: {len(raw_bytes)}")
        return _save_frames(raw_bytes)
    except Exception as e:
        print(f"Erro crítico na demodulação: {e}")
        traceback.print_exc()
        return []


def decode_from_buffer_batch(data: np.ndarray, mode: str, symbol_rate: int) -> list:
    """Batched decode_from_buffer: [B, N] streams in one GPU call; list of saved-path lists."""
    data = np.asarray(data)
    try:
        if mode == "BPSK":
            raws = modem.bpsk_demodulate_batch(data, baud=symbol_rate)
        elif mode.startswith("FSK"):
            baud = 9600 if "9600" in mode else 19200 if "19200" in mode else 1200
            raws = modem.fsk_demodulate_batch(data, baud=baud)
        else:
            raws = modem.qpsk_demodulate_batch(data, baud=symbol_rate)
    except Exception as e:
        print(f"Erro crítico na demodulação: {e}")
        traceback.print_exc()
        return [[] for _ in range(len(data))]
    try:
        framesets = parse_fbp_stream_enhanced_batch(raws)
    except Exception as e:
        print(f"Erro crítico na demodulação: {e}")
        traceback.print_exc()
        return [[] for _ in range(len(data))]
    return [_save_frames(r, fr) for r, fr in zip(raws, framesets)]


def get_assembly_status():
    return []


def find_frame_start(data: bytes, start_pos: int = 0) -> int:
    """decoder.py:470-478."""
    preamble = b'\xAA\xAA\xAA\xAA'
    magic = b'FBPC'
    for i in range(start_pos, len(data) - 8):
        if data[i:i + 4] == preamble and data[i + 4:i + 8] == magic:
            return i
    return -1


def calculate_global_average_quality() -> float:
    total_quality, total_parts = 0.0, 0
    for assembly in active_file_assemblies.values():
        q = [v for v in getattr(assembly, 'parts_quality', []) if v > 0]
        total_quality += sum(q)
        total_parts += len(q)
    return (total_quality / total_parts) if total_parts > 0 else 0.0


def get_reception_stats():
    stats = reception_stats.copy()
    stats['average_quality'] = calculate_global_average_quality()
    return stats


def clear_reception_stats():
    global reception_stats
    reception_stats = _fresh_stats()


def debug_demodulation(samples: np.ndarray, mode: str, symbol_rate: int):
    print("🔍 DEBUG Demodulação:")
    print(f"   - Modo: {mode}")
    print(f"   - Taxa: {symbol_rate}")
    print(f"   - Amostras: {len(samples)}")
    print(f"   - Primeiras 20 amostras: {samples[:20]}")
    print(f"   - Média: {np.mean(samples):.6f}")
    print(f"   - Std: {np.std(samples):.6f}")
    print(f"   - Min/Max: {np.min(samples):.6f}/{np.max(samples):.6f}")
