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

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def reference_bits(kind, symbols):
    diff_symbols = symbols[1:] * np.conj(symbols[:-1])
    bits = []
    for s in diff_symbols:
        if kind == "bpsk":
            bits.append(1 if np.real(s) < 0 else 0)
            continue
        decision_angle = np.angle(s)
        if decision_angle < 0:
            decision_angle += 2 * np.pi
        if decision_angle < np.pi / 4 or decision_angle > 7 * np.pi / 4:
            bits.extend([0, 0])
        elif np.pi / 4 <= decision_angle < 3 * np.pi / 4:
            bits.extend([0, 1])
        elif 3 * np.pi / 4 <= decision_angle < 5 * np.pi / 4:
            bits.extend([1, 1])
        else:
            bits.extend([1, 0])
    return np.array(bits, np.uint8)


def edge_diffs():
    d = []
    specials = [0.0, -0.0, np.inf, -np.inf, np.nan]
    for a in specials + [1.0, -1.0]:
        for b in specials + [1.0, -1.0]:
            d.append(complex(a, b))
    for m in (5e-324, 2.2250738585072014e-308, 1e-300, 1e-20, 0.7, 1.0, 3.0, 1e20, 1e289, 1e300):
        for sr in (1.0, -1.0):
            for si in (1.0, -1.0):
                base_r, base_i = sr * m, si * m
                # |dr| vs |di| within 3 ulp of equal: the pi/4 + k*pi/2 edges, where
                # an ulp of np.angle decides -- inside the domain of K4a's model of
                # numpy's arctan2 (component magnitudes 2^-1015 .. 2^985)
                for k in (range(-3, 4) if 1e-300 <= m <= 1e289 else ()):
                    r = base_r
                    for _ in range(abs(k)):
                        r = np.nextafter(r, np.inf if k > 0 else -np.inf)
                    d.append(complex(r, base_i))
                    d.append(complex(base_i, r))
                d.append(complex(base_r, 0.0))     # the 0, pi/2, pi, 3pi/2 axes, both zero signs
                d.append(complex(base_r, -0.0))
                d.append(complex(0.0, base_i))
                d.append(complex(-0.0, base_i))
    rng = np.random.default_rng(5)
    for k in range(8):                             # just off the edges, by relative 1e-16 .. 1e-9
        for e in (1e-16, 3e-16, 1e-15, 1e-12, 1e-9):
            for sgn in (1, -1):
                th = k * np.pi / 4 + sgn * e
                r = 10 ** rng.uniform(-5, 5)
                d.append(complex(r * np.cos(th), r * np.sin(th)))
    return d


def symbols_for(ds):
    s = np.empty(2 * len(ds) + 1, np.complex128)
    s[0::2] = 1.0 + 0.0j
    s[1::2] = ds
    return s


@pytest.mark.parametrize("kind", ["qpsk", "bpsk"])
def test_slicer_edges_match_reference_steps(kind):
    import _amr
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
