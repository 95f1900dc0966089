"""Device-memory bound of the drop-in path's plan caches (_amr.PlanCache):
a long-running receiver decoding captures of ever-different lengths
(filebeep_advanced_v2.py:324) must not accumulate one plan per length."""
import numpy as np
import pytest


class FakePlan:
    alive = 0

    def __init__(self, nbytes, streams):
        self.nbytes, self.max_streams = nbytes, streams
        FakePlan.alive += 1

    def scratch_bytes(self):
        return self.nbytes

    def __del__(self):
        FakePlan.alive -= 1


def test_lru_stays_within_budget():
    import _amr
    c = _amr.PlanCache(budget_bytes=1000, max_entries=8)
    for n in range(100):
        c.get(("k", n), 1, lambda m, n=n: FakePlan(100 + n % 7, m))
        assert c.total_bytes() <= 1000
        assert len(c) <= 8
    assert FakePlan.alive <= 8              # evicted plans are released


def test_lru_hit_and_resize():
    import _amr
    c = _amr.PlanCache(budget_bytes=10_000)
    a = c.get("k", 4, lambda m: FakePlan(10, m))
    assert c.get("k", 2, lambda m: FakePlan(10, m)) is a        # big enough: reused
    b = c.get("k", 8, lambda m: FakePlan(10, m))                # too small: replaced
    assert b is not a and b.max_streams == 8 and len(c) == 1


def test_lru_keeps_the_newest_even_over_budget():
    import _amr
    c = _amr.PlanCache(budget_bytes=50)
    c.get("a", 1, lambda m: FakePlan(40, m))
    big = c.get("b", 1, lambda m: FakePlan(500, m))
    assert len(c) == 1 and c.get("b", 1, lambda m: FakePlan(1, m)) is big


def test_stream_bucket():
    import _amr
    assert [_amr.stream_bucket(b, 4096) for b in (1, 2, 3, 64, 65, 5000)] == [1, 2, 4, 64, 128, 4096]


@pytest.mark.gpu
def test_many_lengths_bounded_on_device():
    """100 distinct stream lengths through the drop-in modem functions: the
    summed device bytes of the cached plans stay within the cache budget."""
    import _amr
    import _fsk
    import modem
    budget = 2_000_000_000
    old_p, old_f = _amr._psk_cache, _fsk._fsk_cache
    _amr._psk_cache = _amr.PlanCache(budget)
    _fsk._fsk_cache = _amr.PlanCache(budget)
    try:
        rng = np.random.default_rng(3)
        for k in range(100):
            n = 24000 + 997 * k
            x = rng.standard_normal(n).astype(np.float32)
            modem.qpsk_demodulate(x, baud=9600)
            if k % 10 == 0:
                modem.fsk_demodulate(x, baud=9600, mark_freq=12000.0, space_freq=24000.0)
            assert _amr._psk_cache.total_bytes() <= budget
            assert _fsk._fsk_cache.total_bytes() <= budget
        assert len(_amr._psk_cache) < 100
    finally:
        _amr._psk_cache, _fsk._fsk_cache = old_p, old_f
