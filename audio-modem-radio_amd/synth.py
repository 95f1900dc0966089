"""Synthetic transmit side: framing + vectorised modulators.

Host-side (numpy) restatements of the reference transmit path, used to make
benchmark and test input of the shapes BASELINE.json names.  This is NOT the
hot path (SURVEY.md §8f row 3 marks the transmit side "next"); it exists so
that bench.py and the tests can build batches of thousands of streams quickly.

Reference behaviour restated here:
  * ``frame_data``        -> encoder._frame_data        (encoder.py:94-114)
  * ``qpsk_waveform``     -> modem.qpsk_modulate         (modem.py:138-186)
  * ``bpsk_waveform``     -> modem.bpsk_modulate         (modem.py:28-65)
  * ``fsk_waveform``      -> modem.fsk_modulate          (modem.py:270-295)
  * ``dpsk8_waveform``    -> (new) 8-ary differential PSK; the reference's
    "8PSK" transmitter is a QPSK alias that crashes at sps=5
    (modem.py:345, modem.py:181-183), so config 5's input is our own.

The vectorised forms evaluate the same expressions per symbol as the
reference loops; sample values can differ from the reference modulator in the
last ulp where numpy picks a different SIMD sin kernel for a 2-D call.  Golden
fixtures therefore store the modulated input itself, never a seed.
"""
from __future__ import annotations

import binascii
import struct

import numpy as np

SAMPLE_RATE = 96000
FB_MAGIC = b"FBPC"


def frame_data(fname: str, data: bytes, part_number: int = 0, total_parts: int = 1,
               file_size: int = 0, file_crc: int = 0) -> bytes:
    """FBPC frame header + payload (encoder.py:94-114)."""
    fname_b = fname.encode("utf-8")[:255]
    part_crc = binascii.crc32(data) & 0xFFFFFFFF
    header = (FB_MAGIC + bytes([len(fname_b)]) + fname_b
              + struct.pack("<IIIIII", part_number, total_parts, file_size,
                            file_crc, len(data), part_crc))
    return header + data


def _bytes_to_bits(data: bytes) -> np.ndarray:
    return np.unpackbits(np.frombuffer(bytes(data), dtype=np.uint8))


def _ramp_envelope(sps: int) -> np.ndarray:
    # modem.py:56-61 / 180-183: 10 % linear ramps at both symbol edges
    env = np.ones(sps)
    ramp = int(sps * 0.1)
    if ramp > 0:
        env[:ramp] = np.linspace(0, 1, ramp)
        env[-ramp:] = np.linspace(1, 0, ramp)
    return env


def _psk_waveform(phases: np.ndarray, sps: int, carrier: float, samp_rate: float) -> np.ndarray:
    t_symbol = np.arange(sps) / samp_rate
    w = 2 * np.pi * carrier * t_symbol
    sym = np.sin(w[None, :] + phases[:, None]) * _ramp_envelope(sps)[None, :]
    return sym.ravel().astype(np.float32)


# QPSK dibit -> phase step, Gray (modem.py:160-165)
_QPSK_STEP = np.array([0.0, np.pi / 2, -np.pi / 2, np.pi])   # index = 2*b_hi + b_lo


def qpsk_waveform(data: bytes, baud=1200, carrier=3000.0, samp_rate=SAMPLE_RATE) -> np.ndarray:
    """DQPSK waveform as modem.qpsk_modulate (modem.py:138-186)."""
    bits = _bytes_to_bits(data)
    pre = np.array([0, 0] * 30 + [1, 1] * 10, dtype=np.uint8)      # modem.py:148
    bits = np.concatenate([pre, bits])
    if bits.size % 2:
        bits = np.concatenate([bits, [0]])                            # modem.py:171
    idx = 2 * bits[0::2].astype(np.int64) + bits[1::2]
    phases = np.cumsum(_QPSK_STEP[idx])                               # modem.py:170-174
    return _psk_waveform(phases, int(samp_rate / baud), carrier, samp_rate)


def bpsk_waveform(data: bytes, baud=1200, carrier=3000.0, samp_rate=SAMPLE_RATE) -> np.ndarray:
    """DBPSK waveform as modem.bpsk_modulate (modem.py:28-65)."""
    bits = np.concatenate([np.array([1, 0] * 40, dtype=np.uint8), _bytes_to_bits(data)])
    phases = np.cumsum(np.where(bits == 1, np.pi, 0.0))
    return _psk_waveform(phases, int(samp_rate / baud), carrier, samp_rate)


def dpsk8_waveform(symbols: np.ndarray, baud=19200, carrier=3000.0, samp_rate=SAMPLE_RATE) -> np.ndarray:
    """8-ary differential PSK: phase advances by k*pi/4 per symbol (new; config 5 input)."""
    phases = np.cumsum(np.asarray(symbols, dtype=np.int64) * (np.pi / 4))
    return _psk_waveform(phases, int(samp_rate / baud), carrier, samp_rate)


def fsk_waveform(data: bytes, baud=1200, mark_freq=1200.0, space_freq=2200.0,
                 samp_rate=SAMPLE_RATE) -> np.ndarray:
    """CPFSK waveform as modem.fsk_modulate (modem.py:270-295)."""
    spb = int(round(samp_rate * (1.0 / baud)))
    t = np.arange(spb) / samp_rate
    bits = _bytes_to_bits(b"\xAA\xAA\xAA\xAA" + bytes(data))
    freqs = np.where(bits == 1, mark_freq, space_freq)
    out = np.empty((bits.size, spb))
    phase = 0.0
    for i, f in enumerate(freqs):            # phase recursion is sequential in the reference
        out[i] = np.sin(2 * np.pi * f * t + phase)
        phase += 2 * np.pi * f * (spb / samp_rate)
        phase %= 2 * np.pi
    return (out.ravel().astype(np.float32) * 0.9).astype(np.float32)


def random_frame(rng: np.random.Generator, payload_len: int, name: str = "f.bin") -> bytes:
    payload = rng.integers(0, 256, payload_len, dtype=np.uint8).tobytes()
    return frame_data(name, b"RAW" + payload, 0, 1, payload_len, binascii.crc32(payload) & 0xFFFFFFFF)


def fit(wave: np.ndarray, n: int) -> np.ndarray:
    """Truncate or zero-pad a waveform to exactly n samples."""
    if wave.size >= n:
        return wave[:n]
    return np.concatenate([wave, np.zeros(n - wave.size, dtype=wave.dtype)])


def qpsk_batch(n_streams: int, n_samples: int, baud=9600, carrier=3000.0, samp_rate=SAMPLE_RATE,
               noise=0.05, seed=0, distinct=None) -> np.ndarray:
    """[B][N] float32 batch of framed-DQPSK streams + N(0, noise^2).

    ``distinct`` (default: all) streams are synthesised; the rest of the batch
    cycles through them with an independent noise draw per stream, so the
    batch is still all-distinct sample data but builds in seconds at B=4096.
    """
    rng = np.random.default_rng(seed)
    sps = int(samp_rate / baud)
    n_sym = n_samples // sps
    payload = max(1, (n_sym - 40) // 4 - 40)
    distinct = n_streams if distinct is None else min(distinct, n_streams)
    base = np.stack([fit(qpsk_waveform(random_frame(rng, payload), baud, carrier, samp_rate), n_samples)
                     for _ in range(distinct)])
    out = np.empty((n_streams, n_samples), dtype=np.float32)
    for s in range(n_streams):
        out[s] = base[s % distinct]
        if noise:
            out[s] += rng.normal(0.0, noise, n_samples).astype(np.float32)
    return out


def dpsk8_batch(n_streams: int, n_samples: int, baud=19200, carrier=3000.0, samp_rate=SAMPLE_RATE,
                noise=0.05, seed=0, distinct=None) -> np.ndarray:
    rng = np.random.default_rng(seed)
    sps = int(samp_rate / baud)
    n_sym = -(-n_samples // sps)
    distinct = n_streams if distinct is None else min(distinct, n_streams)
    base = np.stack([fit(dpsk8_waveform(rng.integers(0, 8, n_sym), baud, carrier, samp_rate), n_samples)
                     for _ in range(distinct)])
    out = np.empty((n_streams, n_samples), dtype=np.float32)
    for s in range(n_streams):
        out[s] = base[s % distinct]
        if noise:
            out[s] += rng.normal(0.0, noise, n_samples).astype(np.float32)
    return out


def fsk_batch(n_streams: int, n_samples: int, baud=9600, mark=12000.0, space=24000.0,
              samp_rate=SAMPLE_RATE, noise=0.05, seed=0, distinct=None) -> np.ndarray:
    rng = np.random.default_rng(seed)
    spb = int(round(samp_rate / baud))
    n_bits = n_samples // spb
    payload = max(1, n_bits // 8 - 4 - 40)
    distinct = n_streams if distinct is None else min(distinct, n_streams)
    base = np.stack([fit(fsk_waveform(random_frame(rng, payload), baud, mark, space, samp_rate), n_samples)
                     for _ in range(distinct)])
    out = np.empty((n_streams, n_samples), dtype=np.float32)
    for s in range(n_streams):
        out[s] = base[s % distinct]
        if noise:
            out[s] += rng.normal(0.0, noise, n_samples).astype(np.float32)
    return out


def wav_bytes(arr: np.ndarray, sr: int = SAMPLE_RATE) -> bytes:
    """16-bit mono WAV as modem.wav_from_array (modem.py:360-368): int16 truncation of arr*32767."""
    import io
    import wave
    bio = io.BytesIO()
    with wave.open(bio, "wb") as wf:
        wf.setnchannels(1)
        wf.setsampwidth(2)
        wf.setframerate(sr)
        wf.writeframes((np.asarray(arr) * 32767).astype(np.int16).tobytes())
    return bio.getvalue()
