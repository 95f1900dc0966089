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
  FileAssembly / AdvancedFileAssembly
                             decoder.py:20-122  (multi-part reassembly, part quality)
  save_decoded_files         decoder.py:247-310
  decode_with_retry          decoder.py:313-377 (three demod attempts at
                             symbol_rate, x0.95, x1.05 -- each on the GPU)
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
class FileAssembly:
    """Multi-part file reassembly (decoder.py:20-116): parts keep the copy of best
    signal quality; the file is the parts in order (size / CRC mismatches are
    only reported, as the reference does)."""

    def __init__(self, filename: str, total_parts: int, file_size: int, file_crc: int):
        self.filename = filename
        self.total_parts = total_parts
        self.file_size = file_size
        self.expected_crc = file_crc
        self.parts = [None] * total_parts
        self.parts_quality = [0.0] * total_parts
        self.received_parts = 0
        self.creation_time = self.last_update = time.time()

    def calculate_signal_quality(self, data: bytes) -> float:
        """(1 - zero fraction) * distinct bytes / 256, halved when the payload is
        its first 5 bytes repeated (decoder.py:32-55)."""
        try:
            n = len(data)
            if n == 0:
                return 0.0
            zero_ratio = data.count(b'\x00') / n
            unique_bytes = len(set(data)) / 256
            penalty = 0.5 if n > 10 and data[:5] * (n // 5) == data[:n - n % 5] else 0
            return max(0.0, min(1.0, (1 - zero_ratio) * unique_bytes * (1 - penalty)))
        except Exception:
            return 0.5

    def add_part(self, part_number: int, data: bytes, signal_quality: float = None) -> bool:
        """Store a part (a duplicate replaces the stored copy only if of higher
        quality); True once every part is present (decoder.py:57-84)."""
        if not 0 <= part_number < self.total_parts:
            return False
        q = self.calculate_signal_quality(data) if signal_quality is None else signal_quality
        if self.parts[part_number] is None:
            self.received_parts += 1
        elif q > self.parts_quality[part_number]:
            print(f"Substituindo parte {part_number} (qualidade {self.parts_quality[part_number]:.3f} -> {q:.3f})")
        else:
            print(f"Ignorando parte {part_number} duplicada com qualidade inferior "
                  f"({q:.3f} <= {self.parts_quality[part_number]:.3f})")
            return self.received_parts == self.total_parts
        self.parts[part_number] = data
        self.parts_quality[part_number] = q
        self.last_update = time.time()
        return self.received_parts == self.total_parts

    def get_progress(self) -> float:
        return (self.received_parts / self.total_parts) * 100 if self.total_parts > 0 else 0

    def get_missing_parts(self) -> list:
        return [i for i, part in enumerate(self.parts) if part is None]

    def assemble_file(self) -> bytes:
        if self.received_parts != self.total_parts:
            raise ValueError(f"Partes insuficientes: {self.received_parts}/{self.total_parts}. "
                             f"Faltando: {self.get_missing_parts()}")
        data = b''.join(self.parts)
        if len(data) != self.file_size:
            print(f"Aviso: Tamanho do arquivo diferente. Esperado: {self.file_size}, Obtido: {len(data)}")
        crc = binascii.crc32(data) & 0xffffffff
        if crc != self.expected_crc:
            print(f"Aviso: CRC diferente. Esperado: {self.expected_crc:08X}, Obtido: {crc:08X}")
        return data

    def is_expired(self, timeout_seconds: int = 3600) -> bool:
        return (time.time() - self.last_update) > timeout_seconds

    def get_quality_report(self) -> dict:
        q = self.parts_quality
        return {'average_quality': sum(q) / len(q) if q else 0, 'min_quality': min(q) if q else 0,
                'max_quality': max(q) if q else 0, 'completed_parts': self.received_parts,
                'total_parts': self.total_parts}


class AdvancedFileAssembly(FileAssembly):
    """decoder.py:119-122 (no additions in the reference)."""


def _safe_name(fname: str) -> str:
    return "".join(c for c in fname if c.isalnum() or c in (' ', '-', '_', '.'))


def _write_received(fname: str, data: bytes) -> str:
    os.makedirs(RECV_DIR, exist_ok=True)
    path = os.path.join(RECV_DIR, f"recv_{int(time.time())}_{_safe_name(fname)}")
    with open(path, 'wb') as f:
        f.write(data)
    reception_stats['total_files'] += 1
    reception_stats['total_bytes'] += len(data)
    reception_stats['last_reception'] = time.time()
    return path


def save_decoded_files(parsed: list) -> list:
    """decoder.py:247-310.  Entries are (fname, payload, is_multi, part, total,
    file_size, file_crc) tuples: single files are smart_decompress'ed and saved,
    multi-part ones go through a FileAssembly keyed by name + CRC and are saved
    (undecompressed) once complete; assemblies idle for an hour are dropped."""
    saved = []
    for fname, payload, is_multi, part_number, total_parts, file_size, file_crc in parsed:
        if is_multi:
            key = f"{fname}_{file_crc}"
            if key not in file_assemblies:
                file_assemblies[key] = AdvancedFileAssembly(fname, total_parts, file_size, file_crc)
            asm = file_assemblies[key]
            if asm.add_part(part_number, payload):
                try:
                    data = asm.assemble_file()
                    if len(data) != asm.file_size:
                        print(f"ALERTA: Tamanho do arquivo montado não corresponde! "
                              f"Esperado: {asm.file_size}, Obtido: {len(data)}")
                    crc = binascii.crc32(data) & 0xffffffff
                    if crc != asm.expected_crc:
                        print(f"ALERTA FINAL: CRC do arquivo montado não corresponde! "
                              f"Esperado: {asm.expected_crc:08X}, Obtido: {crc:08X}")
                    saved.append(_write_received(fname, data))
                    print(f"Arquivo multi-partes montado com sucesso: {fname}")
                    print(f"Relatório de qualidade: {asm.get_quality_report()}")
                    del file_assemblies[key]
                except Exception as e:
                    print(f"Erro ao montar arquivo {fname}: {e}")
            continue
        try:
            saved.append(_write_received(fname, smart_decompress(payload)))
        except Exception as e:
            print(f"Erro ao salvar arquivo {fname}: {e}")
    for key in [k for k, a in file_assemblies.items() if a.is_expired()]:
        a = file_assemblies.pop(key)
        print(f"Removendo arquivo incompleto expirado: {a.filename} ({a.received_parts}/{a.total_parts} partes)")
    if parsed:
        reception_stats['success_rate'] = (len(saved) / len(parsed)) * 100
    return saved


# decode_with_retry's demodulator map (decoder.py:329-341): mode -> (demod, kwargs;
# _SR = the attempt's symbol rate), calls as the reference writes them
_SR = object()
_RETRY_CALLS = {
    "FSK1200": (modem.fsk_demodulate, {"baud": 1200, "mark_freq": 1200.0, "space_freq": 2200.0}),
    "FSK9600": (modem.fsk_demodulate, {"baud": 9600}),
    "BPSK": (modem.bpsk_demodulate, {"baud": _SR, "carrier": 3000.0}),
    "QPSK": (modem.qpsk_demodulate, {"baud": _SR, "carrier": 3000.0}),
    "8PSK": (modem.psk8_demodulate, {"baud": _SR, "carrier": 12000.0}),
    "FSK19200": (modem.fsk_high_speed_demodulate, {"baud": 19200}),
    "OFDM4": (modem.ofdm_demodulate_simple, {"baud": _SR, "carrier": 12000.0, "num_subcarriers": 4}),
    "OFDM8": (modem.ofdm_demodulate_simple, {"baud": _SR, "carrier": 12000.0, "num_subcarriers": 8}),
    "FT8": (modem.ft8_demodulate, {"baud": _SR, "carrier": 3000.0}),
    "PSK31": (modem.psk31_demodulate, {"baud": _SR, "carrier": 3000.0}),
    "FELD_HELL": (modem.feld_hell_demodulate, {"baud": 122.5, "carrier": 1000.0}),
}


def decode_with_retry(data: np.ndarray, mode: str, symbol_rate: int, max_retries: int = 3):
    """decoder.py:313-377: up to max_retries demodulations (the 2nd at
    int(rate*0.95), the 3rd at int(that*1.05)); a result over 100 bytes is
    dumped to demodulated_attempt_<k>.bin, parsed and handed to
    save_decoded_files; the first attempt that saves files wins.  Errors in an
    attempt are printed and the next attempt runs.  (The reference hands the
    parser's dicts to save_decoded_files, which unpacks tuples -- kept, so
    frame-bearing attempts fail exactly as there.)"""
    for attempt in range(max_retries):
        try:
            if attempt == 1:
                symbol_rate = int(symbol_rate * 0.95)
            elif attempt == 2:
                symbol_rate = int(symbol_rate * 1.05)
            if mode in _RETRY_CALLS:
                fn, kw = _RETRY_CALLS[mode]
                raw = fn(data, **{k: (symbol_rate if v is _SR else v) for k, v in kw.items()})
            else:
                raw = modem.qpsk_demodulate(data, baud=symbol_rate, carrier=3000.0)
            if len(raw) <= 100:
                print(f"⚠️ Tentativa {attempt + 1}: demodulação retornou apenas {len(raw)} bytes")
                continue
            with open(f"demodulated_attempt_{attempt}.bin", "wb") as f:
                f.write(raw)
            parsed = parse_fbp_stream_enhanced(raw)
            if not parsed:
                print(f"⚠️ Tentativa {attempt + 1}: nenhum frame encontrado")
                continue
            saved_files = save_decoded_files(parsed)
            if saved_files:
                return saved_files
            print(f"⚠️ Tentativa {attempt + 1}: frames encontrados mas não salvos")
        except Exception as e:
            print(f"❌ Erro na tentativa {attempt + 1}: {e}")
            traceback.print_exc()
    print(f"❌ Falha na demodulação após {max_retries} tentativas")
    return []


# ---------------------------------------------------------------------------
class _Pcm16:
    """A 16-bit WAV channel as read from the file: samples = pcm / 32768, the
    float64 libsndfile hands the reference.  The demodulators take it as int16
    (a quarter of the float64 bytes over PCIe, converted exactly on the GPU)."""

    def __init__(self, pcm: np.ndarray):
        self.pcm = np.ascontiguousarray(pcm, np.int16)

    def __len__(self):
        return len(self.pcm)

    def as_float(self) -> np.ndarray:
        return self.pcm.astype(np.float64) / 32768.0


def _read_wav(path: str):
    """(data, sr): soundfile.read's float64 [n] or [n, channels] when soundfile
    is installed; else the raw int16 samples of a 16-bit PCM file, which
    decode_wav_file scales by 1/32768 or hands to the GPU as int16."""
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
    pcm = np.frombuffer(raw, dtype='<i2')
    if nch > 1:
        pcm = pcm.reshape(-1, nch)
    return pcm, sr


def decode_wav_file(path: str, mode: str, symbol_rate: int) -> list:
    """decoder.py:380-389: read, channel 0, FFT-resample to 96 kHz (GPU), decode."""
    data, sr = _read_wav(path)
    if len(data.shape) > 1:
        data = data[:, 0]
    pcm = data.dtype == np.int16                    # read without soundfile: int16 PCM
    if sr != SAMPLE_RATE:
        number_of_samples = int(round(len(data) * float(SAMPLE_RATE) / sr))
        x = data.astype(np.float64) / 32768.0 if pcm else np.asarray(data, np.float64)
        data = _amr.resample(x, number_of_samples)   # scipy.signal.resample, on the GPU
    elif pcm:
        data = _Pcm16(data)
    return decode_from_buffer(data, mode, symbol_rate)


def _demod_bytes(data, mode: str, symbol_rate):
    """The reference's mode dispatch (decoder.py:421-434)."""
    if isinstance(data, _Pcm16):
        return _demod_pcm16(data.pcm, mode, symbol_rate)
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


def _demod_pcm16(pcm: np.ndarray, mode: str, symbol_rate):
    """_demod_bytes for int16 WAV samples (same dispatch, same defaults)."""
    if mode == "BPSK":
        return modem._pcm16_psk("bpsk", pcm, symbol_rate)
    elif mode.startswith("FSK"):
        baud = 9600 if "9600" in mode else 19200 if "19200" in mode else 1200
        return modem._pcm16_fsk(pcm, baud)
    return modem._pcm16_psk("qpsk", pcm, symbol_rate)      # QPSK, 8PSK and every other mode


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


def decode_from_buffer_batch(data: np.ndarray, mode: str, symbol_rate: int, transport=None, root: int = 0) -> list:
    """Batched decode_from_buffer (decoder.py:417-464): [B, N] streams in one
    GPU call; a list of saved-path lists, one per stream.

    transport (multi.RcclTransport, one process per GPU): the global batch is
    sharded over the ranks -- each demodulates its contiguous shard on its own
    GPU, the decoded bytes are all-gathered over RCCL (multi.demod_sharded) --
    and rank `root` parses the frames and writes the files of the whole batch;
    the other ranks return an empty list per stream."""
    data = np.asarray(data)

    def demod(x):
        if mode == "BPSK":
            return modem.bpsk_demodulate_batch(x, baud=symbol_rate)
        if mode.startswith("FSK"):
            baud = 9600 if "9600" in mode else 19200 if "19200" in mode else 1200
            return modem.fsk_demodulate_batch(x, baud=baud)
        return modem.qpsk_demodulate_batch(x, baud=symbol_rate)
    try:
        if transport is None:
            raws = demod(data)
        else:
            import multi
            raws = multi.demod_sharded(data, demod, transport)
            if transport.rank != root:
                return [[] for _ in range(len(data))]
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
