"""The slicer stage (K4a) at its decision edges, against the reference's own
steps: the differential product symbols[1:] * np.conj(symbols[:-1]) and, per
diff, np.angle + the +2*pi normalisation + the four sector comparisons
(QPSK, /root/reference/modem.py:214-241) or np.real(s) < 0 (BPSK,
modem.py:100-105) -- evaluated here with numpy exactly as the reference
evaluates them (a numpy complex128 array, per-element np.angle).

Symbols are [1, d0, 1, d1, ...] so that the diffs are d_k and conj(d_k):
d_k sit ON the sector edges k*pi/4 and a few ulp either side (|dr| vs |di|
within ulps: the band where K4a replays numpy's arctan2), at magnitudes
1e-300 .. 1e289, plus the axes at magnitudes from the smallest denormal to
1e300, signed zeros, infinities and NaN.

Ulp ties of np.angle with components below 2^-1015 or above 2^985 are not
covered:
numpy's AVX-512 arctan2 takes internal paths there that K4a does not model
(it uses ocml's atan2), so a decision exactly at an edge may differ; such a
diff is 2^-30-rare among near-ties of real signals, themselves ~2^-30-rare
per symbol."""
import numpy as np
import pytest

from slicer_cases import (edge_diffs, near_tie_diffs, numpy_is_fixture_host, reference_bits, reference_dibits,
                          symbols_for)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


@pytest.mark.parametrize("kind", ["qpsk", "bpsk"])
def test_slicer_edges_match_reference_steps(kind):
    import _amr
    if kind == "qpsk" and not numpy_is_fixture_host():
        pytest.skip("this host's numpy arctan2 is not the fixtures' AVX-512 kernel: near-tie angles differ by design")
    ds = edge_diffs()
    rows = [symbols_for(ds[i:i + 61]) for i in range(0, len(ds), 61)]
    S = max(len(r) for r in rows)
    sym = np.zeros((len(rows), S), np.complex128)
    sym[:] = 1.0
    for i, r in enumerate(rows):
        sym[i, :len(r)] = r
    got = _amr.psk_slice(kind, sym)
    bad = []
    for i in range(len(rows)):
        want = reference_bits(kind, sym[i])
        if not np.array_equal(got[i], want):
            j = int(np.flatnonzero(got[i] != want)[0]) // (2 if kind == "qpsk" else 1)
            bad.append((i, j, sym[i, j], sym[i, j + 1]))
    assert not bad, f"{len(bad)} rows differ, first {bad[:3]}"


def test_slicer_random_symbols_match_reference_steps():
    import _amr
    rng = np.random.default_rng(7)
    sym = (rng.normal(size=(16, 997)) + 1j * rng.normal(size=(16, 997))) * 10 ** rng.uniform(-3, 3, (16, 1))
    for kind in ("qpsk", "bpsk"):
        got = _amr.psk_slice(kind, sym)
        for i in range(16):
            assert np.array_equal(got[i], reference_bits(kind, sym[i])), (kind, i)


def test_slicer_near_ties_match_numpy_and_oracle():
    """400 k products within ulps of the sector edges (slicer_cases.near_tie_diffs)
    through K4a: the decisions equal numpy's (the reference's np.angle steps)
    and the oracle's (oracle/amr_oracle.c qpsk_dibit, the batch tests' checker)."""
    import _amr
    from oracle import oracle
    if not numpy_is_fixture_host():
        pytest.skip("this host's numpy arctan2 is not the fixtures' AVX-512 kernel")
    rows, per = 32, 6250
    ds = near_tie_diffs(rows * per, seed=31).reshape(rows, per)
    sym = np.stack([symbols_for(r) for r in ds])
    bits = _amr.psk_slice("qpsk", sym)
    got = (bits[:, 0::2] * 2 + bits[:, 1::2]).astype(np.uint8)
    prods = sym[:, 1:] * np.conj(sym[:, :-1])
    want = reference_dibits(prods)
    assert np.array_equal(got, want), int(np.count_nonzero(got != want))
    assert np.array_equal(oracle.qpsk_slice(prods).reshape(got.shape), want)
