"""The N > 1 path on CPU (multi.py): ranks shard a batch, demodulate their
shards (the oracle stands in for the per-rank GPU call here) and all-gather
the packed decoded bytes; the result must equal the single-process batch.
The packing, the several-batches-per-launch layout and the gather check run
over two transports: the product's torch-free StoreTransport (FileStore and
TcpStore bootstrap, world 2 and 3) and a torch.distributed gloo transport
defined here -- the same multi.py code either way.  The RCCL transport is
the GPU tests' (tests/test_gpu_comm.py, tests/test_gpu_bench_comm.py)."""
import multiprocessing as mproc
import os
import socket

import numpy as np
import pytest


def test_shard_ranges_cover_exactly():
    from multi import shard_range
    for B in (0, 1, 7, 64, 4096, 4097):
        for world in (1, 2, 3, 8):
            spans = [shard_range(B, r, world) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == B
            for (a, b), (c, d) in zip(spans, spans[1:]):
                assert b == c and b >= a
            assert max(h - l for l, h in spans) - min(h - l for l, h in spans) <= 1


def test_pack_unpack_roundtrip():
    from multi import pack, unpack
    outs = [b"", b"a", b"xyz" * 10]
    p, ln = pack(outs, 5, 40)
    assert unpack(p[None], ln[None]) == outs


def test_shard_layout_several_steps_per_launch():
    """ShardLayout: C steps of a global batch per launch; gathering the ranks'
    slots in any world size returns every step's streams in global order."""
    from multi import ShardLayout
    rng = np.random.default_rng(0)
    for world in (1, 2, 3, 8):
        for B, C in ((7, 1), (8, 3), (17, 2), (3, 4)):
            lay = ShardLayout(B, world, C)
            steps = [[bytes(rng.integers(0, 256, rng.integers(0, 9), dtype=np.uint8)) for _ in range(B)]
                     for _ in range(C)]
            slots = []
            for r in range(world):
                lo, hi = lay.shard(r)
                outs = [o for st in steps for o in st[lo:hi]]          # the rank's launch, step-major
                assert len(outs) == lay.launch_rows(r)
                slots.append(lay.pack(outs, 8))
            got = lay.unpack(np.stack([p for p, _ in slots]), np.stack([ln for _, ln in slots]))
            assert got == [o for st in steps for o in st]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class GlooTransport:
    """A test transport over torch.distributed (gloo): the multi.py transport interface."""

    def __init__(self, dist):
        self.dist, self.rank, self.world = dist, dist.get_rank(), dist.get_world_size()

    def all_gather(self, a):
        import torch
        t = torch.from_numpy(np.ascontiguousarray(a))
        parts = [torch.empty_like(t) for _ in range(self.world)]
        self.dist.all_gather(parts, t)
        return np.stack([p.numpy() for p in parts])

    def max(self, v):
        return float(self.all_gather(np.array([v], np.float64)).max())

    def barrier(self):
        self.dist.barrier()


def _paths():
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (os.path.join(root, "audio-modem-radio_amd"), root):
        if p not in sys.path:
            sys.path.insert(0, p)


def _make_transport(kind, rank, world, port, tmp):
    _paths()
    import multi
    if kind == "gloo":
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        dist.init_process_group("gloo", rank=rank, world_size=world)
        return GlooTransport(dist)
    store = multi.TcpStore("127.0.0.1", port, is_server=rank == 0) if kind == "tcp" else multi.FileStore(tmp)
    return multi.StoreTransport(store, rank, world)


def _close(kind, tp):
    if kind == "gloo":
        tp.dist.barrier()
        tp.dist.destroy_process_group()
    else:
        tp.close()


def _demod_worker(rank, world, kind, port, tmp, x, baud, result_file):
    tp = _make_transport(kind, rank, world, port, tmp)
    import multi
    from oracle import oracle
    got = multi.demod_sharded(x, lambda xs: oracle.psk_demod_batch("qpsk", xs, baud)[0], tp)
    if rank == 0:
        np.save(result_file, np.array([g.hex() for g in got]))
    _close(kind, tp)


def _spawn(target, world, args):
    ctx = mproc.get_context("spawn")
    procs = [ctx.Process(target=target, args=(r, world) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.mark.parametrize("kind,world", [("gloo", 2), ("file", 2), ("tcp", 3)])
def test_sharded_demod_equals_single_process(tmp_path, kind, world):
    import synth
    from oracle import oracle
    x = synth.qpsk_batch(7, 6000, 9600, seed=3, distinct=3)
    out = str(tmp_path / "res.npy")
    _spawn(_demod_worker, world, (kind, _free_port(), str(tmp_path / "store"), x, 9600, out))
    got = list(np.load(out))
    want = [w.hex() for w in oracle.psk_demod_batch("qpsk", x, 9600)[0]]
    assert got == want


def _bench_gather_worker(rank, world, kind, port, tmp, B_global, cap, corrupt_rank, result_file, C=1):
    """bench.py's N>1 bookkeeping end to end: each rank takes its shard of C
    consecutive strong-scaling global batches (bench.workload_sizes; C steps
    per launch, bench --coalesce), decodes them as one launch (the oracle
    stands in for the GPU), packs its [C * B_slot][cap] slot, the slots are
    all-gathered over the transport, and the gathered buffer is checked
    against every rank's own output exactly as bench.py does it
    (multi.gather_check); every step's global batch is then read back out of
    the gathered buffer (ShardLayout.unpack)."""
    tp = _make_transport(kind, rank, world, port, tmp)
    import bench
    import multi
    import synth
    from oracle import oracle
    B, Bg, lo, B_slot = bench.workload_sizes("ofdm8", B_global, world, rank)
    lay = multi.ShardLayout(B_global, world, C)
    assert lay.b_slot == B_slot and lay.launch_rows(rank) == C * B
    steps = [synth.qpsk_batch(B_global, 4000, 9600, seed=5 + c, distinct=B_global) for c in range(C)]
    outs, _ = oracle.psk_demod_batch("qpsk", lay.local_rows(steps, rank), 9600)
    own, lens = lay.pack(outs, cap)
    gp = tp.all_gather(own)
    gl = tp.all_gather(lens)
    if corrupt_rank is not None:
        gp[corrupt_rank, 0, 0] ^= 0xFF                    # a wrong byte in that rank's slice, as every rank sees it
    bad = multi.gather_check(gp, gl, own, lens, lay, tp)
    if rank == 0:
        want = [w for x in steps for w in oracle.psk_demod_batch("qpsk", x, 9600)[0]]
        got = want if corrupt_rank is not None else lay.unpack(gp, gl)
        np.save(result_file, np.array([str(bad), str(got == want)]))
    _close(kind, tp)


@pytest.mark.parametrize("kind,world,B_global,corrupt,C", [("gloo", 2, 7, None, 1), ("file", 3, 8, None, 1),
                                                          ("tcp", 3, 8, 2, 1), ("file", 2, 7, None, 3),
                                                          ("gloo", 3, 8, 1, 2)])
def test_bench_gather_bookkeeping(tmp_path, kind, world, B_global, corrupt, C):
    out = str(tmp_path / "res.npy")
    cap = 2 * 4000 // 10 // 8 + 8
    _spawn(_bench_gather_worker, world, (kind, _free_port(), str(tmp_path / "store"), B_global, cap, corrupt, out, C))
    bad, same = list(np.load(out))
    assert same == "True"
    assert bad == ("[]" if corrupt is None else f"[{corrupt}]")


@pytest.mark.parametrize("world", [1, 2, 4, 8])
def test_bench_launch_plan(world):
    """bench.py's steps per launch: every step's streams are launched exactly
    once (K x the rank's shard), launches hold >= 4096 streams on small
    strong-scaling shards, weak scaling stays one step per launch."""
    _paths()
    import bench
    for K in (1, 5, 20, 64):
        B = bench.workload_sizes("ofdm8", 0, world, 0)[0]
        C, BL, n, sizes = bench.launch_plan(K, B, True)
        assert C == min(K, max(1, -(-4096 // B))) and BL == C * B and len(sizes) == n
        assert sum(sizes) == K * B and all(0 < x <= BL and x % B == 0 for x in sizes)
        assert all(x == BL for x in sizes[:-1])
        Bw = bench.workload_sizes("qpsk9600", 0, world, 0)[0]
        assert bench.launch_plan(K, Bw, False) == (1, Bw, K, [Bw] * K)


def test_product_package_is_torch_free():
    """north_star: no PyTorch in the host code (grep of the package sources)."""
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-modem-radio_amd")
    hits = []
    for dp, _, fs in os.walk(root):
        for f in fs:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                with open(os.path.join(dp, f), encoding="utf-8") as fh:
                    for i, line in enumerate(fh, 1):
                        code = line.split("#")[0]
                        if "import torch" in code or "from torch" in code:
                            hits.append(f"{f}:{i}")
    assert not hits, hits


def _many_exchanges_worker(rank, world, kind, port, tmp, result_file):
    tp = _make_transport(kind, rank, world, port, tmp)
    for i in range(60):
        got = tp.all_gather(np.array([rank, i], np.int64))
        assert got.tolist() == [[r, i] for r in range(world)]
    tp.barrier()
    if rank == 0 and kind == "file":
        np.save(result_file, np.array([len(os.listdir(tmp))]))
    tp.barrier()
    _close(kind, tp)


@pytest.mark.parametrize("kind", ["file", "tcp"])
def test_store_transport_keeps_few_keys(tmp_path, kind):
    """A long-lived StoreTransport deletes each exchange's keys once every rank
    has moved past it: after 60 all-gathers (+ barriers) the file store holds
    at most the last two exchanges' keys, and every gather is right."""
    out = str(tmp_path / "n.npy")
    _spawn(_many_exchanges_worker, 3, (kind, _free_port(), str(tmp_path / "store"), out))
    if kind == "file":
        assert int(np.load(out)[0]) <= 2 * 3


def _failing_rank_worker(rank, world, kind, port, tmp, result_file):
    tp = _make_transport(kind, rank, world, port, tmp)
    import multi

    def demod(xs):
        if rank == 1:
            raise ValueError("rank 1's demodulation fails")
        return [bytes(8)] * len(xs)
    try:
        multi.demod_sharded(np.zeros((6, 100), np.float32), demod, tp)
        what = "no error"
    except ValueError as e:
        what = f"ValueError: {e}"
    except RuntimeError as e:
        what = f"RuntimeError: {e}"
    np.save(result_file.format(rank=rank), np.array([what]))
    _close(kind, tp)


def test_failing_rank_is_reported_on_every_rank(tmp_path):
    """A rank whose demodulation raises still joins the status collective:
    it re-raises its own error, the other ranks raise naming it -- nobody is
    left waiting in the gather."""
    out = str(tmp_path / "r{rank}.npy")
    _spawn(_failing_rank_worker, 3, ("file", _free_port(), str(tmp_path / "store"), out))
    got = [str(np.load(out.format(rank=r))[0]) for r in range(3)]
    assert got[1] == "ValueError: rank 1's demodulation fails"
    assert got[0] == got[2] == "RuntimeError: demodulation failed on rank(s) [1]"
