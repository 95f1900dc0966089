"""The oracle's QPSK slicer (oracle/amr_oracle.c qpsk_dibit) against the
reference's own steps evaluated with numpy (np.angle, +2*pi, the four sector
comparisons; /root/reference/modem.py:214-241) where an ulp of np.angle decides
the sector: every crafted sector-edge product of tests/slicer_cases.edge_diffs
and 1.5 M near-tie products.  numpy's arctan2 there is its AVX-512 (SVML)
kernel, which libm's atan2 does not reproduce; the oracle models it exactly as
the GPU slicer does (psk_common.h numpy_atan2_near_diag)."""
import numpy as np
import pytest

from slicer_cases import edge_diffs, near_tie_diffs, numpy_is_fixture_host, reference_bits, reference_dibits, symbols_for


@pytest.fixture(scope="module", autouse=True)
def fixture_host():
    if not numpy_is_fixture_host():
        pytest.skip("this host's numpy arctan2 dispatch differs from the golden fixtures' host "
                    "(tests/golden/manifest.json numpy_cpu_features)")


def test_edge_products_match_reference_steps():
    from oracle import oracle
    sym = symbols_for(edge_diffs())
    ds = sym[1:] * np.conj(sym[:-1])                  # the reference's products (modem.py:214)
    bits = reference_bits("qpsk", sym)
    want = (bits[0::2] * 2 + bits[1::2]).astype(np.uint8)
    got = oracle.qpsk_slice(ds)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, [(ds[i], got[i], want[i]) for i in bad[:5]]


def test_near_tie_products_match_numpy():
    from oracle import oracle
    ds = near_tie_diffs(1_500_000, seed=3)
    want = reference_dibits(ds)
    got = oracle.qpsk_slice(ds)
    bad = np.flatnonzero(got != want)
    assert bad.size == 0, f"{bad.size} of {ds.size} differ, first {[(ds[i], got[i], want[i]) for i in bad[:3]]}"
    # libm's atan2 (the oracle's slicer before this model) flips some of them
    import math
    libm = np.array([math.atan2(d.imag, d.real) for d in ds[:200_000]])
    assert np.count_nonzero(libm != np.angle(ds[:200_000])) > 0


@pytest.mark.parametrize("seed", [21, 22])
def test_near_tie_angles_bit_exact(seed):
    """Stronger than the decisions: the modelled angle itself equals numpy's,
    bit for bit, on 2 M near-ties per seed (signed zeros compared as bits)."""
    from oracle import oracle
    ds = near_tie_diffs(2_000_000, seed=seed)
    got = oracle.np_angle(ds)
    want = np.angle(ds)
    bad = np.flatnonzero(got.view(np.int64) != want.view(np.int64))
    assert bad.size == 0, [(ds[i], got[i].hex(), want[i].hex()) for i in bad[:3]]


def test_vectorised_angle_is_the_reference_per_element_angle():
    """reference_dibits runs np.angle over an array; the reference calls it on
    one numpy scalar at a time (modem.py:219).  Same kernel, same bits."""
    ds = near_tie_diffs(20_000, seed=9)
    vec = np.angle(ds)
    per = np.array([np.angle(d) for d in ds])
    assert np.array_equal(vec.view(np.int64), per.view(np.int64))
