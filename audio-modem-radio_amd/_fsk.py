"""FSK host layer: filter design with the reference's scipy calls + GPU launch.

fsk_demodulate (modem.py:298-341): per tone butter(3, [(f-baud)/nyq, (f+baud)/nyq],
'band') WITHOUT clamping -- scipy raises for an edge <= 0 or >= 1, which is the
reference's behaviour at its own defaults -- then filtfilt,
|hilbert|, per-sample compare, windowed majority, sync + pack.
"""
from __future__ import annotations

import numpy as np

import _amr


def design_fsk(n: int, baud, mark_freq, space_freq, samp_rate):
    """Raise exactly where the reference raises, in the reference's order."""
    from scipy import signal
    nyq = samp_rate / 2
    out = []
    for f in (mark_freq, space_freq):      # mark envelope is computed first (modem.py:311-312)
        b, a = signal.butter(3, [(f - baud) / nyq, (f + baud) / nyq], btype='band')
        nt = max(len(a), len(b))
        if n <= 3 * nt:
            raise ValueError("The length of the input vector x must be greater than padlen, which is %d." % (3 * nt))
        out.append(tuple(np.ascontiguousarray(v, np.float64) for v in (b, a, signal.lfilter_zi(b, a))))
    return out


def fsk_demodulate_batch(x: np.ndarray, baud, mark_freq, space_freq, samp_rate) -> list:
    if x.ndim != 2:
        raise ValueError("batch input must be a 2-D [streams, samples] array")
    design_fsk(x.shape[1], baud, mark_freq, space_freq, samp_rate)
    _amr.require_gpu()
    raise _amr.AmrError(_amr.AMR_E_INVALID, "FSK GPU kernels are not built yet")
