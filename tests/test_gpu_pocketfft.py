"""The device restatement of pocketfft (csrc/pocketfft_dev.h) -- the FSK exact
path's envelope stage and decode_wav_file's resample -- against the oracle
(oracle/amr_pocketfft.c, itself pinned bit for bit against scipy + numpy on
every length 1..2000 by tests/test_oracle_golden.py) and against scipy:
bit-exact, every length, every plan kind (FFTPACK-style radices 2, 3, 4, 5,
7, 8, 11, the generic passes, Bluestein)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def test_exact_hilbert_env_every_length():
    """|hilbert| on the GPU == the oracle, bit for bit, on every length
    1..2000 (noise, and signal between exact-zero stretches)."""
    import _amr
    from oracle import oracle
    rng = np.random.default_rng(12)
    bad = []
    for n in range(1, 2001):
        x = rng.standard_normal((2, n))
        x[1, : n // 3] = 0.0
        x[1, 2 * n // 3:] = 0.0
        got = _amr.hilbert_env_exact(x)
        for r in range(2):
            if not np.array_equal(got[r], oracle.hilbert_env(x[r])):
                bad.append((n, r))
    assert not bad, bad[:20]


@pytest.mark.parametrize("n", [9600, 24001, 30011, 77880, 96000, 96001, 400001, 441000])
def test_exact_hilbert_env_fsk_lengths(n):
    """The FSK lengths, 5-smooth, Bluestein (24001, 30011, 96001, 400001) and
    generic-radix (77880 = 59 * 1320, 441000 = 2^3 3^2 5^3 7^2), on the
    inputs whose envelopes are rounding noise: digital silence, a stretch
    1e-17 below the signal, a DC stretch -- == the oracle and scipy."""
    import _amr
    from oracle import oracle
    from scipy import signal
    rng = np.random.default_rng(n)
    x = rng.standard_normal((3, n))
    x[0, : n // 3] = 0.0
    x[1, n // 4: n // 2] *= 1e-17
    x[2, n // 2:] = -0.25
    got = _amr.hilbert_env_exact(x)
    for r in range(3):
        want = oracle.hilbert_env(x[r])
        assert np.array_equal(got[r], want), (n, r)
        assert np.array_equal(got[r], np.abs(signal.hilbert(x[r])))


@pytest.mark.parametrize("nx,num,batch", [(441000, 960000, 1), (480000, 960000, 1), (44100, 96000, 2),
                                          (48000, 96000, 2), (22050, 96000, 1), (8000, 96000, 1),
                                          (100000, 96000, 1), (1000, 2177, 2), (2177, 1000, 2), (999, 1500, 1),
                                          (1001, 1001, 1), (24001, 52247, 1)])
def test_resample_bit_exact(nx, num, batch):
    """_amr.resample == scipy.signal.resample, bit for bit (decoder.py:385-387):
    decode_wav_file's 44.1 / 48 / 22.05 / 8 kHz -> 96 kHz lengths, down-
    sampling, odd and Bluestein lengths."""
    import _amr
    from scipy import signal
    rng = np.random.default_rng(nx + num)
    x = rng.normal(size=(batch, nx))
    got = _amr.resample(x, num)
    want = signal.resample(x, num, axis=1)
    assert np.array_equal(got, want), np.abs(got - want).max()
    assert np.array_equal(_amr.resample(x[0], num), got[0])
