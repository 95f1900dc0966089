"""Transmit side, CPU checks: the oracle's modulators and the
C-ABI's length/error contract against the reference's own outputs
(tests/golden/tx.npz, written by tests/golden/make_tx_golden.py)."""
import json
import os

import numpy as np
import pytest

from oracle import oracle

G = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def tx():
    with open(os.path.join(G, "tx_manifest.json")) as f:
        return json.load(f)["cases"], np.load(os.path.join(G, "tx.npz"))


def _mode_args(c):
    import _amr
    p = c["params"]
    mode = {"bpsk_modulate": _amr.TX_BPSK, "qpsk_modulate": _amr.TX_QPSK, "fsk_modulate": _amr.TX_FSK}[c["fn"]]
    return mode, p.get("baud", 1200), p.get("samp_rate", 96000)


def test_oracle_modulators_match_reference_bitwise(tx):
    cases, d = tx
    for c in cases:
        fn = getattr(oracle, c["fn"])
        data = d[c["id"] + ".in"].tobytes()
        if c["status"] == "err":
            with pytest.raises(ValueError) as e:
                fn(data, **c["params"])
            assert str(e.value) == c["emsg"]
            continue
        y = fn(data, **c["params"])
        r = d[c["id"] + ".out"]
        assert y.dtype == r.dtype and y.shape == r.shape
        assert np.array_equal(y.view(np.uint32), r.view(np.uint32)), c["id"]
        assert np.array_equal(oracle.wav_pcm(y), d[c["id"] + ".wav"][44:].view(np.int16)), c["id"]


def test_wav_from_array_bytes(tx, built_lib):
    import modem
    cases, d = tx
    for c in cases:
        if c["status"] == "ok":
            assert modem.wav_from_array(d[c["id"] + ".out"]) == d[c["id"] + ".wav"].tobytes(), c["id"]


def test_tx_lengths_and_errors_through_the_abi(tx, built_lib):
    """amr_tx_samples == len(reference output); the reference's ValueError cases
    come back with its message.  Host-only entry points: no GPU needed."""
    import _amr
    cases, _ = tx
    for c in cases:
        mode, baud, sr = _mode_args(c)
        if c["status"] == "err":
            with pytest.raises(ValueError) as e:
                _amr.tx_samples(mode, c["n_bytes"], baud, sr)
            assert str(e.value) == c["emsg"]
        else:
            assert _amr.tx_samples(mode, c["n_bytes"], baud, sr) == c["n"], c["id"]
    with pytest.raises(ZeroDivisionError):
        _amr.tx_samples(_amr.TX_QPSK, 4, 0, 96000)
    # work = 3 tables of sps doubles + one phase per symbol per stream (+ alignment slack)
    wb = _amr.lib().amr_tx_work_bytes(_amr.TX_QPSK, 9600.0, 96000.0, 4096, 96000)
    assert wb == (3 * 10 + 4096 * 9600) * 8 + 256


def test_modulate_argument_checks(built_lib):
    import ctypes
    import _amr
    L = _amr.lib()
    nb = np.zeros(1, np.int64)
    out = np.zeros((1, 8), np.float32)
    assert L.amr_modulate_host(7, 1200.0, 3000.0, 0.0, 96000.0, None, 0, _amr.ptr(nb), 1, _amr.ptr(out), 8, 8,
                               None, 0) == _amr.AMR_E_INVALID
    assert L.amr_modulate_host(1, 1200.0, 3000.0, 0.0, 96000.0, None, 0, _amr.ptr(nb), 1, _amr.ptr(out), 4, 8,
                               None, 0) == _amr.AMR_E_INVALID              # out_stride < n_out
    nb[0] = 5
    assert L.amr_modulate_host(1, 1200.0, 3000.0, 0.0, 96000.0, None, 4, _amr.ptr(nb), 1, _amr.ptr(out), 8, 8,
                               None, 0) == _amr.AMR_E_INVALID              # n_bytes > data_stride
    assert L.amr_modulate_device(None, 1, 1200.0, 3000.0, 0.0, 96000.0, ctypes.c_void_p(8), 4, ctypes.c_void_p(8),
                                 1, ctypes.c_void_p(8), 8, 8, None, 0, None, 0) == _amr.AMR_E_INVALID  # no work buffer
