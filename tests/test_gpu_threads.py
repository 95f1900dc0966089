"""Reentrancy: the reference decodes from its capture QThread and
its GUI thread at once (filebeep_advanced_v2.py:324,1112).  ctypes drops the
GIL inside every libamr call, so these threads really overlap on the device:
same-shape calls share one cached plan (its mutex serialises them), others get
their own plans and streams.  Every result must equal the single-threaded one."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def test_concurrent_demod_threads_match_serial():
    import modem
    import synth
    xq = synth.qpsk_batch(24, 24000, 9600, seed=11)
    xb = synth.qpsk_batch(6, 30000, 2400, seed=12)
    xf = synth.fsk_batch(6, 24000, 9600, seed=13)
    jobs = ([("q", i) for i in range(24)] + [("qb", 0), ("qb", 1)] + [("b", i) for i in range(6)]
            + [("f", i) for i in range(6)] + [("fb", 0)])

    def run(job):
        kind, i = job
        if kind == "q":
            return modem.qpsk_demodulate(xq[i], 9600)
        if kind == "qb":
            return tuple(modem.qpsk_demodulate_batch(xq[12 * i:12 * i + 12], 9600))
        if kind == "b":
            return modem.bpsk_demodulate(xb[i], 2400)
        if kind == "f":
            return modem.fsk_demodulate(xf[i], 9600, 12000.0, 24000.0)
        return tuple(modem.fsk_demodulate_batch(xf, 9600, 12000.0, 24000.0))

    serial = {j: run(j) for j in jobs}
    results, errors = {}, []

    def worker(my_jobs):
        try:
            for _ in range(3):
                for j in my_jobs:
                    got = run(j)
                    if results.setdefault(j, got) != got:
                        errors.append(("unstable", j))
        except Exception as e:            # surfaced below, with the job list
            errors.append(("raised", repr(e)))

    rng = np.random.default_rng(0)
    threads = []
    for t in range(6):
        order = [jobs[k] for k in rng.permutation(len(jobs))]
        threads.append(threading.Thread(target=worker, args=(order,)))
    for th in threads:
        th.start()
    for th in threads:
        th.join(timeout=100)
    assert not any(th.is_alive() for th in threads), "a demod thread did not finish"
    assert not errors, errors[:5]
    for j in jobs:
        assert results[j] == serial[j], j
    assert all(len(serial[("q", i)]) > 0 for i in range(24))
