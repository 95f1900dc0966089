"""Slicer decision-edge cases shared by tests/test_gpu_slicer.py (the GPU
slicer, K4a) and tests/test_oracle_slicer.py (the oracle's): the reference's
own steps for one differential product (/root/reference/modem.py:214-241 QPSK,
:100-105 BPSK) evaluated with numpy exactly as the reference does, and the
differential products that sit on / within ulps of the sector edges."""
import json
import os

import numpy as np

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


def numpy_is_fixture_host() -> bool:
    """True when this host's numpy dispatches arctan2 as the golden fixtures'
    host did (tests/golden/manifest.json numpy_cpu_features): only then is
    numpy's np.angle at an ulp-tie the reference's."""
    from numpy._core._multiarray_umath import __cpu_features__ as f
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "manifest.json")) as fh:
        want = json.load(fh).get("numpy_cpu_features", {})
    return bool(want) and all(bool(f.get(k, False)) == v for k, v in want.items())


def near_tie_diffs(n: int, seed: int = 0) -> np.ndarray:
    """n differential products within a few ulp (or up to 2^-29 relative) of
    the diagonals |re| = |im|, every sign combination, magnitudes 1e-290 ..
    1e290 (inside the domain where numpy's AVX-512 arctan2 is modelled)."""
    rng = np.random.default_rng(seed)
    mag = 10.0 ** rng.uniform(-290, 290, n)
    mag[: n // 2] = 10.0 ** rng.uniform(-6, 6, n // 2)          # half at signal-like scales
    k = rng.integers(-4, 5, n).astype(np.float64)
    other = mag + k * np.spacing(mag)                           # a few ulp off the diagonal
    far = rng.random(n) < 0.25
    other[far] = mag[far] * (1.0 + rng.uniform(-2.0 ** -29, 2.0 ** -29, int(far.sum())))
    swap = rng.random(n) < 0.5
    re = np.where(swap, other, mag) * rng.choice([-1.0, 1.0], n)
    im = np.where(swap, mag, other) * rng.choice([-1.0, 1.0], n)
    return re + 1j * im


def reference_dibits(diffs: np.ndarray) -> np.ndarray:
    """The reference's QPSK decision per product (modem.py:219-241), vectorised:
    np.angle over the array (the same arctan2 loop the per-element call runs;
    test_oracle_slicer checks that on a sample), then the +2*pi and the four
    comparisons.  Returns 2*hi + lo."""
    ang = np.angle(diffs)
    ang = np.where(ang < 0, ang + 2 * np.pi, ang)
    out = np.full(ang.shape, 2, np.uint8)                              # else: 10
    out[(np.pi / 4 <= ang) & (ang < 3 * np.pi / 4)] = 1
    out[(3 * np.pi / 4 <= ang) & (ang < 5 * np.pi / 4)] = 3
    out[(ang < np.pi / 4) | (ang > 7 * np.pi / 4)] = 0
    return out
