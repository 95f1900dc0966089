"""RCCL gather on one GPU (a 1-rank communicator): two plans (two batches in
flight on two streams, as bench.py runs them) share one communicator; every
gathered buffer equals its plan's own output of that round (amr_allgather
orders itself after the plan's queued work, and the plan's later work waits
for it before writing outputs)."""
import ctypes
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_two_plans_one_comm():
    """Each plan demodulates a different batch every round into the same
    output buffers, and each round's gather goes to a buffer of its own: a
    gather that read its plan's outputs after the next round had rewritten
    them (or before they were written) would show the wrong round's bytes.
    amr_psk_plan_synchronize alone must cover the plan's last gather."""
    import _amr
    import synth
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")
    L = _amr.lib()
    _amr.check(L.amr_set_device(0))
    B, N, R = 64, 20000, 3
    xs = [[synth.qpsk_batch(B, N, 9600, seed=10 * p + r, distinct=4) for r in range(R)] for p in range(2)]
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
    for p in range(2):
        d_x = []
        for x in xs[p]:
            d = dmalloc(x.nbytes)
            _amr.check(L.amr_memcpy_h2d(d, _amr.ptr(x), x.nbytes))
            d_x.append(d)
        bufs.append(dict(x=d_x, out=dmalloc(B * cap), len=dmalloc(B * 8), sync=dmalloc(B * 8),
                         g=[dmalloc(B * cap) for _ in range(R)], glen=[dmalloc(B * 8) for _ in range(R)]))
    for r in range(R):                                    # several rounds, both plans in flight
        for b, pl in zip(bufs, plans):
            _amr.check(L.amr_psk_demod_device(pl.handle, b["x"][r], _amr.DTYPE_F32, B, N, b["out"], cap, b["len"],
                                              b["sync"]))
            _amr.check(L.amr_allgather(comm, b["out"], b["g"][r], B * cap, pl.handle))
            _amr.check(L.amr_allgather(comm, b["len"], b["glen"][r], B * 8, pl.handle))
    for pl in plans:
        _amr.check(L.amr_psk_plan_synchronize(pl.handle))   # the plan and its gathers, nothing else
    import modem
    for p, b in enumerate(bufs):
        for r in range(R):
            g, gl = np.empty((B, cap), np.uint8), np.empty(B, np.int64)
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(g), b["g"][r], B * cap))
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(gl), b["glen"][r], B * 8))
            assert [g[i, :gl[i]].tobytes() for i in range(B)] == modem.qpsk_demodulate_batch(xs[p][r], baud=9600), \
                (p, r)
        for v in b.values():
            for q in (v if isinstance(v, list) else [v]):
                _amr.check(L.amr_free(q))
    _amr.check(L.amr_comm_destroy(comm))


def test_rccl_transport_one_rank(tmp_path):
    """multi.RcclTransport (the product's torch-free sharded path) as one
    rank: the unique id through a FileStore, host all-gather / max / barrier
    over RCCL, and decoder.decode_from_buffer_batch / multi.demodulate_sharded
    through it == the unsharded calls."""
    import contextlib
    import io
    import _amr
    import decoder
    import modem
    import multi
    import synth
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")
    tp = multi.RcclTransport(multi.FileStore(str(tmp_path / "store")), 0, 1, 0)
    try:
        a = np.arange(37, dtype=np.int64)
        assert np.array_equal(tp.all_gather(a), a[None])
        assert tp.max(2.5) == 2.5
        tp.barrier()
        x = synth.qpsk_batch(40, 24000, 1000, seed=8, distinct=5)
        assert multi.demodulate_sharded("qpsk", x, 1000, tp) == modem.qpsk_demodulate_batch(x, baud=1000)
        with contextlib.redirect_stdout(io.StringIO()):
            os.chdir(tmp_path)
            want = decoder.decode_from_buffer_batch(x, "QPSK", 1000)
            got = decoder.decode_from_buffer_batch(x, "QPSK", 1000, transport=tp)
        names = lambda r: [[os.path.basename(p).split("_", 1)[1] for p in ps] for ps in r]
        assert names(got) == names(want) and sum(map(len, got)) == 40
    finally:
        tp.close()
