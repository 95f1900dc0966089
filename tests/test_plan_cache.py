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


def test_lru_evicts_for_the_new_plan_first():
    """With an estimate, room is made BEFORE the new plan is created: the
    cache never holds more than the budget, not even while creating."""
    import _amr
    c = _amr.PlanCache(budget_bytes=100)
    c.get("a", 1, lambda m: FakePlan(40, m))
    c.get("b", 1, lambda m: FakePlan(40, m))
    seen = []

    def make(m):
        seen.append(c._total_unlocked())
        return FakePlan(50, m)
    c.get("c", 1, make, estimate=lambda m: 50)
    assert seen == [40] and len(c) == 2 and c.total_bytes() == 90


def test_one_cache_for_psk_and_fsk():
    import _amr
    import _fsk
    assert _fsk._amr.plan_cache is _amr.plan_cache


@pytest.mark.gpu
def test_many_lengths_bounded_on_device():
    """100 distinct stream lengths through the drop-in modem functions (PSK
    and FSK plans in the one cache): the summed device bytes of the cached
    plans stay within the budget, and each plan's estimate (made before it
    was created) equals the bytes it then reports."""
    import _amr
    import modem
    budget = 2_000_000_000
    old = _amr.plan_cache
    _amr.plan_cache = _amr.PlanCache(budget)
    try:
        rng = np.random.default_rng(3)
        for k in range(100):
            n = 24000 + 997 * k
            x = rng.standard_normal(n).astype(np.float32)
            modem.qpsk_demodulate(x, baud=9600)
            if k % 10 == 0:
                modem.fsk_demodulate(x, baud=9600, mark_freq=12000.0, space_freq=24000.0)
            assert _amr.plan_cache.total_bytes() <= budget
        assert len(_amr.plan_cache) < 100
        L = _amr.lib()
        for key, pl in list(_amr.plan_cache._d.items()):
            if key[0] == "psk":
                est = L.amr_psk_plan_bytes_estimate(_amr.PSK_QPSK, pl.n, pl.sps, pl.first, 9, 5, pl.max_streams)
            else:
                est = L.amr_fsk_plan_bytes_estimate(pl.n, pl.sps, 7, pl.max_streams)
            assert est == pl.scratch_bytes(), (key, est, pl.scratch_bytes())
    finally:
        _amr.plan_cache = old


@pytest.mark.gpu
def test_full_size_fsk_plan_fits_the_default_budget():
    """BASELINE configs[2]'s 16384 x 96000 FSK plan (live-column layout) is
    admitted by the default cache budget with room left, and its estimate
    is what it reports."""
    import _amr
    import _fsk
    est = _amr.lib().amr_fsk_plan_bytes_estimate(96000, 10, 7, 16384)
    assert est <= 56e9 and est <= _amr._cache_budget()
    pl = _fsk.FskPlan(96000, 9600, 12000.0, 24000.0, max_streams=16384)
    assert pl.live_columns and pl.scratch_bytes() == est
