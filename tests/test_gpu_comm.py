"""RCCL gather on one GPU (a 1-rank communicator): two plans (two batches in
flight on two streams, as bench.py runs them) share one communicator; every
gathered buffer equals its plan's own output (amr_allgather orders itself
after the plan's queued work and before its later work)."""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_plans_one_comm():
    import _amr
    import synth
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")
    L = _amr.lib()
    _amr.check(L.amr_set_device(0))
    B, N = 64, 20000
    xs = [synth.qpsk_batch(B, N, 9600, seed=s, distinct=4) for s in (1, 2)]
    plans = [_amr.PskPlan("qpsk", N, 9600, max_streams=B, device=0) for _ in range(2)]
    cap = plans[0].out_cap

    def dmalloc(n):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), int(n)))
        return p
    uid = (ctypes.c_uint8 * 128)()
    _amr.check(L.amr_comm_unique_id(uid))
    comm = ctypes.c_void_p()
    _amr.check(L.amr_comm_create(ctypes.byref(comm), uid, 1, 0, 0))
    bufs = []
    for x, pl in zip(xs, plans):
        d_x = dmalloc(x.nbytes)
        _amr.check(L.amr_memcpy_h2d(d_x, _amr.ptr(x), x.nbytes))
        bufs.append(dict(x=d_x, out=dmalloc(B * cap), len=dmalloc(B * 8), sync=dmalloc(B * 8),
                         g=dmalloc(B * cap), glen=dmalloc(B * 8)))
    for rep in range(3):                                  # several rounds, both plans in flight
        for b, pl in zip(bufs, plans):
            _amr.check(L.amr_psk_demod_device(pl.handle, b["x"], _amr.DTYPE_F32, B, N, b["out"], cap, b["len"],
                                              b["sync"]))
            _amr.check(L.amr_allgather(comm, b["out"], b["g"], B * cap, pl.handle))
            _amr.check(L.amr_allgather(comm, b["len"], b["glen"], B * 8, pl.handle))
    _amr.check(L.amr_device_synchronize())
    for x, b in zip(xs, bufs):
        out, g = np.empty((B, cap), np.uint8), np.empty((B, cap), np.uint8)
        ln, gl = np.empty(B, np.int64), np.empty(B, np.int64)
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(out), b["out"], B * cap))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(g), b["g"], B * cap))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(ln), b["len"], B * 8))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(gl), b["glen"], B * 8))
        assert np.array_equal(out, g) and np.array_equal(ln, gl)
        got = [out[i, :ln[i]].tobytes() for i in range(B)]
        assert got == __import__("modem").qpsk_demodulate_batch(x, baud=9600)
        for p in b.values():
            _amr.check(L.amr_free(p))
    _amr.check(L.amr_comm_destroy(comm))
