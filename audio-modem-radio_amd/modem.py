"""modem.py -- drop-in for the reference's modem module, demodulators on MI355X.

Same names and signatures as szumanski/Audio-Modem-Radio modem.py, so
decoder.py / encoder.py / filebeep_advanced_v2.py import it unchanged
(put this directory first on sys.path).  Every demodulator runs on the GPU
through libamr.so (see _amr.py); there is no CPU fallback.

Receive side (the hot path, bit-exact with the reference):
  qpsk_demodulate   modem.py:189-266     bpsk_demodulate  modem.py:68-135
  psk8_demodulate   modem.py:348         ofdm_demodulate_simple modem.py:375-376
  psk31_demodulate  modem.py:397         fsk_demodulate   modem.py:298-341
  fsk_high_speed_demodulate modem.py:355-356   ft8_demodulate modem.py:391
plus batched forms (*_demodulate_batch) that take a [B, N] array and return
one bytes object per stream -- the form the GPU is built for.

Transmit side (on the GPU: tx_kernels.hip):
  qpsk_modulate modem.py:138-186   bpsk_modulate modem.py:28-65
  fsk_modulate  modem.py:270-295   (+ aliases) and modulate_batch; the float32
  samples equal the reference's up to the last-ulp sin difference the tests bound.
  wav_from_array modem.py:360-368 (host WAV writer).
"""
from __future__ import annotations

import numpy as np

import _amr
import synth

SAMPLE_RATE = 96000


class AdvancedModem:
    """modem.py:14-22 (holds the sample rate; AGC helper)."""

    def __init__(self):
        self.sample_rate = SAMPLE_RATE

    def _adaptive_gain_control(self, data: np.ndarray) -> np.ndarray:
        max_val = np.max(np.abs(data))
        if max_val > 0:
            return data / max_val * 0.95
        return data


# ---------------------------------------------------------------------------
# input normalisation
def _as_batch(samples) -> np.ndarray:
    """The caller's samples as an array, in THEIR dtype: the reference hands
    them to filtfilt as they are (modem.py:77, 198, 308), which forms its odd
    extension 2*x[0] - x[k] in that dtype -- a full-scale int16 capture's
    extension wraps.  float32 / float64 go to the kernels as they are; other
    real dtypes (integers of every width, bool, float16) go with the extension
    numpy forms in their own dtype (_amr.raw_input);
    anything else as float64."""
    x = np.asarray(samples)
    if not _amr.is_kernel_dtype(x.dtype) and x.dtype.kind not in "biuf":
        x = x.astype(np.float64)
    return x


def _psk_batch(kind: str, x2d: np.ndarray, baud, carrier, samp_rate):
    if x2d.ndim != 2:
        raise ValueError("batch input must be a 2-D [streams, samples] array")
    x2d = _as_batch(x2d)
    B, n = x2d.shape
    if B == 0:
        return []
    plan = _amr.get_psk_plan(kind, n, baud, carrier, samp_rate, B)
    outs, _ = plan.demod_host(x2d) if _amr.is_kernel_dtype(x2d.dtype) else plan.demod_host_raw(x2d)
    return outs


# 16-bit WAV samples straight from the file (decoder.decode_wav_file): the
# plans take int16 as pcm / 32768 -- exactly the float64 libsndfile gives the
# reference -- so a quarter of the float64 bytes cross PCIe.  Internal: the
# public functions treat integer input as raw values, as the reference does
# (its odd extension wrapping in the integer dtype included).
def _pcm16_psk(kind: str, pcm: np.ndarray, baud, carrier=3000.0, samp_rate=96000) -> bytes:
    x = np.ascontiguousarray(pcm, np.int16)[None, :]
    plan = _amr.get_psk_plan(kind, x.shape[1], baud, carrier, samp_rate, 1)
    return plan.demod_host(x)[0][0]


def _pcm16_fsk(pcm: np.ndarray, baud, mark_freq=1200.0, space_freq=2200.0, samp_rate=96000) -> bytes:
    import _fsk
    return _fsk.fsk_demodulate_batch(np.ascontiguousarray(pcm, np.int16)[None, :], baud, mark_freq, space_freq,
                                     samp_rate)[0]


# ---------------------------------------------------------------------------
# PSK receive side
def qpsk_demodulate(samples: np.ndarray, baud=1200, carrier=3000.0, samp_rate=96000) -> bytes:
    """DQPSK demodulation of one stream (modem.py:189-266), on the GPU."""
    x = _as_batch(samples)
    if x.ndim != 1:
        raise ValueError("qpsk_demodulate expects a 1-D sample array (use qpsk_demodulate_batch)")
    return _psk_batch("qpsk", x[None, :], baud, carrier, samp_rate)[0]


def bpsk_demodulate(samples: np.ndarray, baud=1200, carrier=3000.0, samp_rate=96000) -> bytes:
    """DBPSK demodulation of one stream (modem.py:68-135), on the GPU."""
    x = _as_batch(samples)
    if x.ndim != 1:
        raise ValueError("bpsk_demodulate expects a 1-D sample array (use bpsk_demodulate_batch)")
    return _psk_batch("bpsk", x[None, :], baud, carrier, samp_rate)[0]


def qpsk_demodulate_batch(samples: np.ndarray, baud=1200, carrier=3000.0, samp_rate=96000) -> list:
    """[B, N] equal-length streams -> B bytes objects (each == qpsk_demodulate(row))."""
    return _psk_batch("qpsk", np.asarray(samples), baud, carrier, samp_rate)


def bpsk_demodulate_batch(samples: np.ndarray, baud=1200, carrier=3000.0, samp_rate=96000) -> list:
    return _psk_batch("bpsk", np.asarray(samples), baud, carrier, samp_rate)


def demodulate_ragged(kind: str, streams, baud, carrier=3000.0, samp_rate=96000) -> list:
    """Ragged batch: streams of different lengths, grouped by length on the host."""
    fn = {"qpsk": qpsk_demodulate_batch, "bpsk": bpsk_demodulate_batch}[kind]
    by_len: dict = {}
    for i, s in enumerate(streams):
        by_len.setdefault(len(s), []).append(i)
    out = [b""] * len(streams)
    for n, idx in by_len.items():
        res = fn(np.stack([_as_batch(streams[i]) for i in idx]), baud, carrier, samp_rate)
        for i, r in zip(idx, res):
            out[i] = r
    return out


# ---------------------------------------------------------------------------
# FSK receive side (modem.py:298-341): tone band-passes + |hilbert| envelopes
def fsk_demodulate(samples: np.ndarray, baud=1200, mark_freq=1200.0, space_freq=2200.0, samp_rate=96000) -> bytes:
    x = _as_batch(samples)
    if x.ndim != 1:
        raise ValueError("fsk_demodulate expects a 1-D sample array (use fsk_demodulate_batch)")
    return fsk_demodulate_batch(x[None, :], baud, mark_freq, space_freq, samp_rate)[0]


def fsk_demodulate_batch(samples: np.ndarray, baud=1200, mark_freq=1200.0, space_freq=2200.0,
                         samp_rate=96000) -> list:
    import _fsk
    return _fsk.fsk_demodulate_batch(_as_batch(np.asarray(samples)), baud, mark_freq, space_freq, samp_rate, raw=True)


# ---------------------------------------------------------------------------
# aliases kept from the reference (modem.py:344-403)
def psk8_modulate(d, b=1200, c=3000.0, s=96000):
    return qpsk_modulate(d, b, c, s)


def psk8_demodulate(s, b=1200, c=3000.0, s_r=96000):
    return qpsk_demodulate(s, b, c, s_r)


def fsk_high_speed_modulate(d, baud=19200, s=96000):
    return fsk_modulate(d, baud, 8000, 16000, s)


def fsk_high_speed_demodulate(s, baud=19200, s_r=96000):
    return fsk_demodulate(s, baud, 8000, 16000, s_r)


def ofdm_modulate_simple(d, baud, carrier, num_subcarriers, samp_rate=96000):
    return qpsk_modulate(d, baud, carrier, samp_rate)


def ofdm_demodulate_simple(s, baud, carrier, num_subcarriers, samp_rate=96000):
    return qpsk_demodulate(s, baud, carrier, samp_rate)


def apsk16_modulate(d, b, c, s=96000):
    return qpsk_modulate(d, b, c, s)


def dsss_modulate(d, b, c, s=96000):
    return bpsk_modulate(d, b, c, s)


def msk_modulate(d, b, c, s=96000):
    return fsk_modulate(d, b, c, c + b, s)


def ft8_modulate(d, b, c, s=96000):
    return fsk_modulate(d, 50, c, c + 50, s)


def ft8_demodulate(s, b, c, sr=96000):
    return fsk_demodulate(s, 50, c, c + 50, sr)


def psk31_modulate(d, b, c, s=96000):
    return bpsk_modulate(d, 31.25, c, s)


def psk31_demodulate(s, b, c, sr=96000):
    return bpsk_demodulate(s, 31.25, c, sr)


def feld_hell_modulate(d, b, c, s=96000):
    raise NotImplementedError("Hellschreiber (hellschreiber.py) is outside this build's scope (SURVEY §2)")


def feld_hell_demodulate(s, b, c, sr=96000):
    raise NotImplementedError("Hellschreiber (hellschreiber.py) is outside this build's scope (SURVEY §2)")


# ---------------------------------------------------------------------------
# transmit side on the GPU (tx_kernels.hip): the same float32
# samples as the reference's modulators; wav_from_array stays a host WAV writer.
def bpsk_modulate(data_bytes: bytes, baud=1200, carrier=3000.0, samp_rate=96000) -> np.ndarray:
    """modem.py:28-65 (DBPSK)."""
    return _amr.modulate(_amr.TX_BPSK, [bytes(data_bytes)], baud, carrier, 0.0, samp_rate)[0]


def qpsk_modulate(data_bytes: bytes, baud=1200, carrier=3000.0, samp_rate=96000) -> np.ndarray:
    """modem.py:138-186 (DQPSK)."""
    return _amr.modulate(_amr.TX_QPSK, [bytes(data_bytes)], baud, carrier, 0.0, samp_rate)[0]


def fsk_modulate(data_bytes: bytes, baud=1200, mark_freq=1200.0, space_freq=2200.0, samp_rate=96000) -> np.ndarray:
    """modem.py:270-295 (CPFSK)."""
    return _amr.modulate(_amr.TX_FSK, [bytes(data_bytes)], baud, mark_freq, space_freq, samp_rate)[0]


def modulate_batch(kind: str, datas, baud=1200, f0=None, f1=None, samp_rate=96000, n_out=None, pcm=False):
    """Batched modulators: [B, n_out] float32 (each row == <kind>_modulate(datas[b])
    cut / zero-padded to n_out; default the longest), plus wav_from_array's
    int16 samples when pcm=True.  kind: 'bpsk' | 'qpsk' (f0 = carrier) or
    'fsk' (f0 = mark_freq, f1 = space_freq)."""
    mode = _amr.TX_MODES[kind]
    if f0 is None:
        f0 = 1200.0 if kind == "fsk" else 3000.0
    if f1 is None:
        f1 = 2200.0 if kind == "fsk" else 0.0
    return _amr.modulate(mode, [bytes(d) for d in datas], baud, f0, f1, samp_rate, n_out, pcm)


def wav_from_array(arr, sr=96000):
    """modem.py:360-368: 16-bit mono WAV of int16(arr * 32767)."""
    return synth.wav_bytes(arr, sr)
