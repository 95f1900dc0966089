#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X, plus BASELINE's other
GPU configurations as sub-objects of the same JSON line.

metric : demod Msymbols/s (batch) + achieved HBM GB/s, QPSK@9600/96kHz
workload (N=1): BASELINE configs[1] -- QPSK @ 9600 sym/s, 96 kHz, batch 4096
          synthetic 1-s streams (N = 96000 float32 samples each), inputs
          resident in HBM before the timed region.
step   : one pass of the whole demod path over ONE batch: band-pass filtfilt
          + mixer -> low-pass filtfilt -> [exact-path fixups] -> slicer + sync
          + pack (and, for N>1 GPUs, the RCCL all-gather of the decoded bytes).
          K steps = K distinct batches (each in-flight slot has its own input
          buffer and noise draw), at most P of them in flight at once on P
          plans / HIP streams (P = --inflight, default `default_inflight`:
          K itself up to 20 (16 for 8192-stream batches), else a divisor of
          K near 16, so the timed region is whole pipeline rounds).
scaling: weak for qpsk9600 / fsk9600 (every rank its own batch), strong for
          ofdm8 / psk8fec (a global batch of 8192 sharded over the ranks).

Also reported: the one-batch-at-a-time latency, per-kernel HIP-event times
(in flight and solo), the roofline (contract form + solo + pipeline + FP64),
the CPU baseline (the C oracle on the host cores), bit-exact parity of
sampled streams of in-flight slots against the oracle, and for N>1 a check
that the gathered buffer equals every rank's own output.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload W] [--inflight P]
        multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
        (the launcher only starts the ranks: bootstrap, barriers and gathers
        are multi.py's -- a file store and RCCL, no torch in the process)
"""
from __future__ import annotations

import os
import sys

# HIP reads GPU_MAX_HW_QUEUES when it initialises (the first HIP call, below).
# One hardware queue per in-flight batch lets their kernels run side by side
# (the lane-per-stream kernels need ~16 batches resident to fill the chip).
_q = sys.argv[sys.argv.index("--hw-queues") + 1] if "--hw-queues" in sys.argv else "32"
os.environ["GPU_MAX_HW_QUEUES"] = str(min(32, int(_q)))

import argparse  # noqa: E402
import ctypes  # noqa: E402
import gc  # noqa: E402
import hashlib  # noqa: E402
import json  # noqa: E402
import time  # noqa: E402

import numpy as np  # noqa: E402

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-modem-radio_amd"))
sys.path.insert(0, ROOT)

import _amr  # noqa: E402
import synth  # noqa: E402

FS = 96000
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
HBM_MIXED_GBS = 5200.0         # measured streaming rate at 1:1..2:1 read:write (tools/hbm_mix_probe.hip, profiles/)
def _newest_pmc_round():
    """The newest profiles/r<NN>_pmc.json (the PMC traffic per timing slot of
    the latest profiled round; profiles/<round>_summary.md folds it)."""
    import glob
    import re
    rounds = [m.group(1) for f in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json"))
              if (m := re.fullmatch(r"(r\d+)_pmc\.json", os.path.basename(f)))]
    return max(rounds, key=lambda r: int(r[1:])) if rounds else None


PROFILE_ROUND = _newest_pmc_round()
FP64_PEAK_TOPS = 39.3          # non-fused FP64 vector ops/s (78.6 TFLOP/s counts an FMA as 2)

# BASELINE.json configs[1..4], 0-based (configs[0] is the reference's CPU plumbing case)
WORKLOADS = {
    "qpsk9600": dict(baud=9600.0, batch=4096, strong=False, fsk=False, fec=False,
                     metric="demod Msymbols/s (batch) + achieved HBM GB/s, QPSK@9600/96kHz, 1/2/4/8 GPU"),
    "fsk9600": dict(baud=9600.0, batch=16384, strong=False, fsk=True, fec=False,
                    metric="FSK demod Msymbols/s (batch), FSK9600 96kHz mark/space 12k/24k"),
    "ofdm8": dict(baud=9600.0, batch=8192, strong=True, fsk=False, fec=False,
                  metric="OFDM8 (qpsk_demodulate alias) demod Msymbols/s, global batch sharded + RCCL gather"),
    "psk8fec": dict(baud=19200.0, batch=8192, strong=True, fsk=False, fec=True,
                    metric="8PSK@19200 demod + fused FEC decode Msymbols/s, global batch sharded + RCCL gather"),
}
# the reference's own numpy/scipy code (measured in the build
# container, 8 cores): not on the GPU box; the north-star basis
REF_PY = {"qpsk9600": (0.292, 1.66), "ofdm8": (0.292, 1.66), "psk8fec": (0.310, 2.43), "fsk9600": (0.180, 1.15)}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(force=False):
    """The N > 1 control plane, torch-free (multi.py): the RCCL unique id
    through a bootstrap store (multi.store_from_env: a FileStore named after
    torch.distributed.run's MASTER_PORT and agent process), then one RCCL
    communicator per rank (multi.RcclTransport) that carries the barriers,
    the max over ranks, the gather check and the per-launch all-gathers of
    decoded bytes.  With `force`, the same for one rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or force:
        import multi
        return multi.RcclTransport(multi.store_from_env(rank, world), rank, world, local), world, rank, local
    return None, 1, 0, local


def host_cores():
    """(threads for the CPU baseline, how they were counted): every CPU in
    this process's affinity mask, capped by its cgroup CPU quota when one is
    set (the GPU box's share of a many-core host: threads beyond the quota
    only time-slice, e.g. 256 threads on a 16-CPU quota ran the oracle at
    28 Msym/s against 72 for 16)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), open(
                            "/sys/fs/cgroup/cpu/cpu.cfs_period_us").read().strip()])):
        try:
            with open(path) as f:
                q, per = parse(f.read())[:2]
            if q not in ("max", "-1") and int(per) > 0:
                quota = -(-int(q) // int(per))
            break
        except (OSError, ValueError, IndexError):
            continue
    n = min(aff, quota) if quota else aff
    how = (f"{n} threads: the {aff} CPUs of os.sched_getaffinity(0)"
           + (f", capped by the cgroup CPU quota of {quota} CPUs" if quota and quota < aff else "")
           + f" (os.cpu_count() {os.cpu_count()}, OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS', 'unset')})")
    return max(1, n), how


def barrier(tp):
    if tp is not None:
        tp.barrier()


def max_over_ranks(tp, v: float) -> float:
    return v if tp is None else tp.max(v)


class Dev:
    """Device buffers through the C ABI (freed at close)."""

    def __init__(self, L):
        self.L, self.ptrs = L, []

    def alloc(self, nbytes):
        p = ctypes.c_void_p()
        _amr.check(self.L.amr_malloc(ctypes.byref(p), int(max(1, nbytes))))
        self.ptrs.append(p)
        return p

    def close(self):
        for p in self.ptrs:
            self.L.amr_free(p)
        self.ptrs = []


def workload_sizes(name, batch_arg, world, rank):
    """(B local, B global, first global stream, gather slot) for a rank: a
    strong-scaling global batch sharded by multi.ShardLayout, or (weak) every
    rank its own batch -- the same layout over world x B streams."""
    import multi
    W = WORKLOADS[name]
    B_global = (batch_arg or W["batch"]) * (1 if W["strong"] else world)
    lay = multi.ShardLayout(B_global, world)
    lo_s, hi_s = lay.shard(rank)
    return hi_s - lo_s, B_global, lo_s, lay.b_slot


def run_workload(name, args, tp, world, rank, dev, comm, headline):
    W = WORKLOADS[name]
    L = _amr.lib()
    fsk, fec_fused, strong = W["fsk"], W["fec"], W["strong"]
    import multi
    B, B_global, lo_s, B_slot = workload_sizes(name, args.batch, world, rank)
    N = args.samples
    baud = W["baud"]
    mark, space = args.mark, args.space
    # the sub-workloads of the default run keep their own timed region
    # (--sub-steps), whatever --steps the headline is given: at N = 8 a
    # strong-scaling shard of 20 steps is too little work to fill a GPU
    K = args.steps if headline else args.sub_steps
    # steps per launch: a strong-scaling shard too small to fill the GPU on its
    # own (8192 / N streams) takes C consecutive global batches per launch, so a
    # launch holds >= 4096 streams (what one batch of the headline holds); the
    # timed region is still exactly K steps (the last launch may be partial)
    C, BL, n_launch, launch_sizes = launch_plan(K, B, strong, args.coalesce)
    # fsk9600: 4 in flight (a device-entry 16384-stream plan holds ~37 GB, `plan_bytes` in the line,
    # DESIGN.md §3b; round 5, one MI355X: P = 3 35.85 ms/step, 4 35.30, 5 35.22)
    P = args.inflight or (min(4, max(1, n_launch // 2)) if fsk else default_inflight(n_launch, 20 if BL <= 4096 else 16))

    # ---- inputs: clean frames on the host, one noisy batch per slot in HBM ----
    t0 = time.perf_counter()
    D = min(args.distinct, B)
    if fsk:
        base = synth.fsk_batch(D, N, baud, mark, space, seed=1000 + rank, noise=0.0)
    elif fec_fused:
        base = synth.dpsk8_batch(D, N, baud, seed=1000 + rank, noise=0.0)
    else:
        base = synth.qpsk_batch(D, N, baud, seed=1000 + rank, noise=0.0)
    mem = Dev(L)
    d_base = mem.alloc(base.nbytes)
    _amr.check(L.amr_memcpy_h2d(d_base, _amr.ptr(base), base.nbytes))
    d_x = []
    for k in range(P):
        d = mem.alloc(BL * N * 4)
        seed = int.from_bytes(hashlib.blake2b(f"{name}/{rank}/{k}".encode(), digest_size=8).digest(), "little")
        _amr.check(L.amr_synth_tile_noise(d_base, D, N, d, BL, lo_s + 17 * k, ctypes.c_float(0.05), seed))
        d_x.append(d)
    log(f"[rank {rank}] {name}: {P} distinct {BL}x{N} float32 launch inputs ({C} step(s) of {B} streams each) in HBM "
        f"in {time.perf_counter() - t0:.1f}s")

    # ---- plans: one per in-flight batch (own HIP stream + scratch) ----
    if fsk:
        import _fsk
        plans = [_fsk.FskPlan(N, baud, mark, space, FS, max_streams=BL, device=dev) for _ in range(P)]
        sym_per_stream = (N - plans[0].sps // 2 + plans[0].sps - 1) // plans[0].sps   # decided bits (modem.py:320)
        demod, sync_fn, names = L.amr_fsk_demod_device, L.amr_fsk_plan_synchronize, _amr.TF_NAMES
        gather_fn = L.amr_fsk_allgather
    else:
        plans = [_amr.PskPlan("qpsk", N, baud, 3000.0, FS, max_streams=BL, device=dev) for _ in range(P)]
        S = (N - plans[0].first + plans[0].sps - 1) // plans[0].sps
        sym_per_stream = S - 1                          # differential symbols decided per stream
        demod, sync_fn, names = L.amr_psk_demod_device, L.amr_psk_plan_synchronize, _amr.T_NAMES
        gather_fn = L.amr_allgather
    for pl in plans:
        pl.enable_timing(True)
        if not fsk:
            pl.set_inflight(P)
    cap = plans[0].out_cap
    # a launch's rows: C steps of B real streams; every rank sends C * B_slot
    # rows to the gather (the strong-scaling slot padding stays at the end)
    R = C * B_slot
    ctx = []
    for k, pl in enumerate(plans):
        c = {"plan": pl, "x": d_x[k], "out": mem.alloc(R * cap), "len": mem.alloc(R * 8), "sync": mem.alloc(R * 8)}
        if fec_fused:
            c.update(fec=mem.alloc(R * cap), flen=mem.alloc(R * 8), ok=mem.alloc(R * 4))
        if comm is not None:
            c["gather"], c["gather_len"] = mem.alloc(world * R * cap), mem.alloc(world * R * 8)
            c["gather_sync"] = mem.alloc(world * R * 8)
        ctx.append(c)

    def step(c, nb=BL):
        pl = c["plan"]
        if fec_fused:
            _amr.check(L.amr_psk_demod_fec_device(pl.handle, c["x"], _amr.DTYPE_F32, nb, N, c["out"], cap, c["len"],
                                                  c["sync"], c["fec"], cap, c["flen"], c["ok"]))
        else:
            _amr.check(demod(pl.handle, c["x"], _amr.DTYPE_F32, nb, N, c["out"], cap, c["len"], c["sync"]))
        if comm is not None:
            # the bytes every rank hands to the gather (the FEC output for
            # psk8fec), to every rank (RCCL over xGMI), ordered after this
            # plan's queued demod and before its next batch
            g_out, g_len = (c["fec"], c["flen"]) if fec_fused else (c["out"], c["len"])
            _amr.check(gather_fn(comm, g_out, c["gather"], R * cap, pl.handle))
            _amr.check(gather_fn(comm, g_len, c["gather_len"], R * 8, pl.handle))
            # the sync indices: SURVEY §8(e)'s wire format is bytes, lengths and sync_idx
            _amr.check(gather_fn(comm, c["sync"], c["gather_sync"], R * 8, pl.handle))

    def launch_streams(j):
        """streams of launch j of the timed region (the last one may hold fewer steps)"""
        return launch_sizes[j]

    names = [k for k in names if k != "launch"]
    kt = {k: 0.0 for k in names}
    nt = [0]
    launch_ms = []                   # whole launches: first kernel -> outputs written (N = 1) / gathered (N > 1)

    def collect(c):
        _amr.check(sync_fn(c["plan"].handle))
        t = c["plan"].timings()
        if "launch" in t:
            launch_ms.append(t.pop("launch"))
        for k, v in t.items():
            kt[k] += v
        nt[0] += 1

    # ---- warmup: one batch at a time (solo kernel times + latency) ----------
    lat = []
    for i in range(max(1, args.warmup)):
        c = ctx[i % P]
        t1 = time.perf_counter()
        step(c)
        _amr.check(sync_fn(c["plan"].handle))
        if comm is not None:
            _amr.check(L.amr_comm_synchronize(comm))
        if i == 0 and args.warmup > 1:                  # the first launch is cold: not counted
            continue
        lat.append(time.perf_counter() - t1)
        collect(c)
    solo = {k: v / max(1, nt[0]) for k, v in kt.items() if v > 0}
    latency_layout = ctx[0]["plan"].last_layout() if not fsk else "fsk"
    for c in ctx:                                       # every plan / stream once before timing
        step(c)
    _amr.check(L.amr_device_synchronize())
    kt = {k: 0.0 for k in names}
    nt = [0]
    launch_ms.clear()

    # ---- timed region: exactly K batches, at most P in flight ----------------
    barrier(tp)
    _amr.check(L.amr_device_synchronize())
    t0 = time.perf_counter()
    if args.host_wait:
        # the host waits for a plan's previous batch before reusing it (and
        # reads its kernel timings every batch)
        for j in range(n_launch):
            c = ctx[j % P]
            if j >= P:
                collect(c)                              # that context's previous batch (the others keep running)
            step(c, launch_streams(j))
        for j in range(max(0, n_launch - P), n_launch):
            collect(ctx[j % P])
    else:
        # launch j is queued on plan j % P's stream behind that plan's previous
        # launch: stream order keeps each plan's batches (and scratch) in
        # sequence, so at most P run at once, and the host never stalls the
        # pipeline between rounds; kernel timings from each plan's last launch
        for j in range(n_launch):
            step(ctx[j % P], launch_streams(j))
        for j in range(max(0, n_launch - P), n_launch):
            collect(ctx[j % P])
    _amr.check(L.amr_device_synchronize())
    barrier(tp)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(tp, dt)
    layout = ctx[0]["plan"].last_layout() if not fsk else "fsk"
    ms_per_step = dt / K * 1e3
    value = B_global * sym_per_stream / (dt / K) / 1e6
    kavg = {k: v / max(1, nt[0]) for k, v in kt.items() if v > 0}

    # ---- sustained: the same pipeline for about --sustain-seconds (headline
    # only, after the timed region; a longer run settles at a lower clock) ----
    sustained = None
    if headline and args.sustain_seconds > 0:
        n_s = max(P, int(round(args.sustain_seconds / max(1e-4, dt / n_launch) / P)) * P)
        barrier(tp)
        _amr.check(L.amr_device_synchronize())
        t1 = time.perf_counter()
        for j in range(n_s):
            step(ctx[j % P])
        _amr.check(L.amr_device_synchronize())
        barrier(tp)
        ds = max_over_ranks(tp, time.perf_counter() - t1)
        sustained = {"steps": n_s * C, "seconds": round(ds, 3), "ms_per_step": round(ds / (n_s * C) * 1e3, 4),
                     "value": round(B_global * sym_per_stream * n_s * C / ds / 1e6, 3),
                     "what": f"{n_s} more launches of the same pipeline ({P} in flight), timed as the headline"}

    # ---- one batch alone, as a single-batch caller runs it (after timing) ------
    # a plan without the in-flight hint picks the latency layout (row kernels,
    # DESIGN.md §3.2); its bytes must equal the lane layout's on the same input
    lat1 = None
    if headline and not fsk and not args.no_latency:
        lp = _amr.PskPlan("qpsk", N, baud, 3000.0, FS, max_streams=B, device=dev)
        lo_, ll_, ls_ = mem.alloc(B * cap), mem.alloc(B * 8), mem.alloc(B * 8)
        ts = []
        for i in range(3):
            t1 = time.perf_counter()
            _amr.check(demod(lp.handle, ctx[0]["x"], _amr.DTYPE_F32, B, N, lo_, cap, ll_, ls_))
            _amr.check(sync_fn(lp.handle))
            ts.append(time.perf_counter() - t1)
        o1, l1 = np.empty((B, cap), np.uint8), np.empty(B, np.int64)
        o0, l0 = np.empty((B, cap), np.uint8), np.empty(B, np.int64)
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(o1), lo_, B * cap))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(l1), ll_, B * 8))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(o0), ctx[0]["out"], B * cap))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(l0), ctx[0]["len"], B * 8))
        same = bool(np.array_equal(l0, l1) and all(o0[i, :l0[i]].tobytes() == o1[i, :l1[i]].tobytes() for i in range(B)))
        lat1 = {"ms": round(float(np.median(ts[1:])) * 1e3, 3), "layout": lp.last_layout(),
                "bytes_equal_lane_layout": same}
        del lp

    # ---- outputs of every slot (after timing) --------------------------------
    # (a slot whose last launch was partial keeps, past it, its previous
    # launch's rows of the same input)
    outs = []
    for c in ctx:
        o = np.empty((BL, cap), np.uint8)
        ln = np.empty(BL, np.int64)
        sy = np.empty(BL, np.int64)
        g_out, g_len = (c["fec"], c["flen"]) if fec_fused else (c["out"], c["len"])
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(o), g_out, BL * cap))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(ln), g_len, BL * 8))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(sy), c["sync"], BL * 8))
        outs.append((o, ln, sy))

    # ---- N>1: the gathered buffer must equal every rank's own output ----------
    gather_check = None
    if comm is not None:
        last = (n_launch - 1) % P
        o, ln, sy = outs[last]
        gp = np.empty((world, R, cap), np.uint8)
        gl = np.empty((world, R), np.int64)
        gs = np.empty((world, R), np.int64)
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(gp), ctx[last]["gather"], gp.nbytes))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(gl), ctx[last]["gather_len"], gl.nbytes))
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(gs), ctx[last]["gather_sync"], gs.nbytes))
        shards = multi.ShardLayout(B_global, world, C)
        assert shards.rows == R and shards.launch_rows(rank) == C * B
        bad_any = multi.gather_check(gp, gl, o, ln, shards, tp, gs, sy)
        # the RCCL communicator's own view of the job: every rank joined
        cw, cr = ctypes.c_int(0), ctypes.c_int(-1)
        _amr.check(L.amr_comm_world(comm, ctypes.byref(cw), ctypes.byref(cr)))
        gather_check = (f"ok: every rank's gathered [{world}][{R}][{cap}] buffer == each rank's own bytes, "
                        f"lengths and sync indices; RCCL world {cw.value}, this rank {cr.value}"
                        if not bad_any else f"MISMATCH: slices of ranks {bad_any}")

    # ---- parity: sampled streams of in-flight slots vs the oracle; CPU baseline
    result = None
    host_res = None
    if rank == 0:
        from oracle import oracle
        # the CPU baseline runs on every core this process may use (its
        # affinity mask, within its cgroup CPU quota: the GPU box's host cores
        # as the scheduler grants them)
        threads, cores_how = host_cores()
        xh = np.empty((BL, N), np.float32)
        if headline and not fsk and not args.no_cpu and world == 1:
            # how many threads these host cores run fastest at: the affinity /
            # quota count, or the box's OMP_NUM_THREADS share -- when the
            # scheduler grants fewer CPUs than the mask shows, threads beyond
            # them only time-slice.  The baseline then uses the fastest.
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(xh), ctx[0]["x"], xh.nbytes))
            cands = sorted({threads, *([int(os.environ["OMP_NUM_THREADS"])] if os.environ.get(
                "OMP_NUM_THREADS", "").isdigit() else [])} - {0})
            probe = {}
            for nt_ in cands:
                xs_ = xh[:min(B, 1024)]
                t1 = time.perf_counter()
                oracle.psk_demod_batch("qpsk", xs_, baud, n_threads=nt_)
                probe[nt_] = round(len(xs_) * sym_per_stream / (time.perf_counter() - t1) / 1e6, 2)
            if len(probe) > 1:
                best = max(probe, key=probe.get)
                cores_how += (f"; probed {', '.join(f'{k} threads {v} Msym/s' for k, v in probe.items())} on "
                              f"{min(B, 1024)} streams: {best} used")
                threads = best
        checked, n_slots, bad_total = 0, 0, []
        cpu = None
        slots = [] if args.no_cpu else range(P) if args.parity_all_slots else sorted({0, 1 % P, P - 1})
        for k in slots:
            if headline and k == 0 and not fsk:
                idx = np.arange(B)                                  # the whole batch of slot 0
            else:
                idx = np.linspace(0, BL - 1, num=min(BL, (1024 if fsk else 256) if k == 0 else 16)).astype(int)
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(xh), ctx[k]["x"], xh.nbytes))
            xs = xh[idx]
            t1 = time.perf_counter()
            if fsk:
                from concurrent.futures import ThreadPoolExecutor
                with ThreadPoolExecutor(threads) as ex:
                    want = list(ex.map(lambda r: oracle.fsk_demodulate(r, baud, mark, space), xs))
            else:
                want, _ = oracle.psk_demod_batch("qpsk", xs, baud, n_threads=threads)
                if fec_fused:
                    want = [oracle.fec_decode(w)[0] for w in want]
            cdt = time.perf_counter() - t1
            reps = 1
            if k == 0 and headline and not fsk and world == 1:
                # the CPU baseline: the same streams again until about
                # --cpu-seconds of wall time have been spent on them
                while cdt < args.cpu_seconds:
                    t1 = time.perf_counter()
                    oracle.psk_demod_batch("qpsk", xs, baud, n_threads=threads)
                    cdt += time.perf_counter() - t1
                    reps += 1
            if k == 0 and world == 1:                     # the CPU baseline: rank 0 at N = 1 only
                how = ("oracle.fsk_demodulate (C filtfilt + the C restatement of pocketfft's Hilbert "
                       "(oracle/amr_pocketfft.c) + C decide), thread pool over streams"
                       if fsk else "the C restatement oracle/amr_oracle.c, OpenMP over streams" +
                       (" + oracle.fec_decode" if fec_fused else ""))
                cpu = {"value": round(reps * len(idx) * sym_per_stream / cdt / 1e6, 3), "unit": "Msym/s",
                       "cores": threads, "kind": "port",
                       "cores_note": cores_how,
                       "sample": f"{len(idx)} of the {BL} streams of benchmark batch 0 ({N} samples each)"
                                 + (f", {reps} passes" if reps > 1 else "") + f" through {how}, {cdt:.2f} s wall"}
            o, ln = outs[k][:2]
            bad_total += [(k, int(i)) for j, i in enumerate(idx) if o[i, :ln[i]].tobytes() != want[j]]
            checked += len(idx)
            n_slots += 1
        if bad_total:
            log(f"[rank {rank}] {name}: streams differing from the oracle (slot, stream): {bad_total[:16]}")
        parity = (f"{checked - len(bad_total)}/{checked} streams bit-exact vs oracle (sampled from {n_slots} of the "
                  f"{P} in-flight batches)" + (" (FEC output)" if fec_fused else "")) if checked else "skipped (--no-cpu)"
        if headline and not fsk and cpu is not None:
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(xh), ctx[0]["x"], xh.nbytes))
            n1 = min(B, 256)
            t1 = time.perf_counter()
            oracle.psk_demod_batch("qpsk", xh[:n1], baud, n_threads=1)
            d1 = time.perf_counter() - t1
            cpu["value_1core"] = round(n1 * sym_per_stream / d1 / 1e6, 3)
            cpu["sample_1core"] = f"{n1} streams of batch 0, 1 thread, {d1:.2f} s wall"

        # ---- roofline ----
        # algorithmic bytes per launch: the path's compulsory input + output,
        # float32 samples in + the decided bits out (40.25 B/symbol at sps 10)
        out_bytes = sym_per_stream * (1 if fsk else 2) / 8
        alg_bytes = BL * (N * 4 + out_bytes)
        step_bytes = B * (N * 4 + out_bytes)
        # the dominant kernel and its duration: one launch alone on the GPU
        # (the warmup launches, HIP events on the plan's stream), so the
        # duration is the kernel's own and not its share of an in-flight round
        dom = max(solo, key=solo.get) if solo else max(kavg, key=kavg.get)
        dom_ms = solo.get(dom) or kavg[dom]
        # FP64 ops the reference arithmetic needs per sample (scipy's DF-II-T,
        # no FMA): band-pass 33/pass (9 taps), low-pass 17/pass/component,
        # mixer 1/component (PSK); FSK filtfilt 25/pass/tone + FFT ~5 n log2 n
        if fsk:
            fp64 = B * (2 * 2 * (N + 42) * 25 + 2 * 2 * 5 * N * np.log2(N))
        else:
            fp64 = B * (2 * (N + 54) * 33 + 2 * (N + 30) * 2 * 17 + 2 * N)    # per step
        # HBM bytes per launch from the rocprofv3 PMC passes (profiles/), when
        # this run's launches are the profiled ones: same workload, samples,
        # streams per launch and kernel layout (bytes per launch do not depend
        # on how many launches are in flight or on the rank count)
        traffic, step_traffic, traffic_src = None, None, None
        pmc_file = os.path.join(ROOT, "profiles", f"{PROFILE_ROUND}_pmc.json")
        if PROFILE_ROUND and os.path.exists(pmc_file) and N == 96000 and BL == W["batch"]:
            with open(pmc_file) as f:
                pm = json.load(f).get(name, {})
            if pm.get("layout", layout) == layout:
                traffic_src = (f"profiles/{PROFILE_ROUND}_pmc.json: rocprofv3 FETCH_SIZE x2 + WRITE_SIZE per launch "
                               f"({pm.get('steps')} timed launches at {pm.get('inflight')} in flight, layout "
                               f"{pm.get('layout')})")
                traffic = pm.get("slots", {}).get(dom, {}).get("hbm_bytes_per_launch")
                # the step's kernels only (not the input synthesis before the timed region)
                step_traffic = sum(v.get("hbm_bytes_per_dispatch", 0) for k, v in pm.get("kernels", {}).items()
                                   if "synth" not in k) or None
        ach = alg_bytes / (dom_ms / 1e3) / 1e9
        ach_if = alg_bytes / (kavg[dom] / 1e3) / 1e9 if dom in kavg else None
        roofline = {
            "bound": "hbm", "kernel": dom, "achieved": round(ach, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(ach / HBM_PEAK_GBS, 5),
            "frac_throughput": round(step_bytes / ms_per_step / 1e6 / HBM_PEAK_GBS, 5),
            "frac_note": (f"frac = one launch's algorithmic bytes / the dominant kernel's duration as ONE launch alone "
                          f"on the GPU ({dom_ms:.3f} ms, longer than the {ms_per_step:.3f} ms step because {P} launches "
                          "overlap in the timed region); frac_throughput = the algorithmic bytes of a step / the step "
                          "time, the figure consistent with `value` (= pipeline.frac)"),
            "traffic": int(traffic) if traffic else None,
            "traffic_ratio": round(traffic / alg_bytes, 2) if traffic else None, "traffic_source": traffic_src,
            "alg_bytes_per_launch": int(alg_bytes),
            "alg_bytes_def": "SURVEY 8(d): per stream N x 4 B float32 samples in + decided bits / 8 out "
                             f"({(N * 4 + out_bytes) / sym_per_stream:.2f} B/symbol here) x {BL} streams per launch",
            "kernel_ms_used": round(dom_ms, 4),
            "kernel_ms_note": "the dominant kernel's average HIP-event duration (on its plan's stream) over the "
                              f"warmup launches, each alone on the GPU ({latency_layout} layout, as in the timed "
                              "region); rocprofv3 reproduces it from the same dispatches (profiles/<round>_summary.md)",
            "inflight": {"kernel_ms": round(kavg[dom], 4) if dom in kavg else None,
                         "achieved": round(ach_if, 2) if ach_if else None,
                         "frac": round(ach_if / HBM_PEAK_GBS, 5) if ach_if else None,
                         "note": f"the same kernel's average duration over the timed region, where {P} launches share "
                                 "the GPU (so it is up to P x its share of a step)"},
            "pipeline": {"ms_per_step": round(ms_per_step, 4), "achieved": round(step_bytes / ms_per_step / 1e6, 2),
                         "frac": round(step_bytes / ms_per_step / 1e6 / HBM_PEAK_GBS, 5),
                         "hbm_traffic_per_step": int(step_traffic / C) if step_traffic else None,
                         "hbm_traffic_gbs": round(step_traffic / C / ms_per_step / 1e6, 1) if step_traffic else None,
                         "hbm_traffic_frac_of_measured_stream": round(step_traffic / C / ms_per_step / 1e6 / HBM_MIXED_GBS, 3)
                         if step_traffic else None,
                         "measured_stream_gbs": HBM_MIXED_GBS,
                         "measured_stream_source": "tools/hbm_mix_probe.hip on one MI355X: a streaming kernel's rate "
                                                   "at 1:1 and 2:1 read:write, 8 accesses per lane in flight "
                                                   "(profiles/r02_hbm_mix_probe.txt)"},
            "fp64_valu": {"ops_per_step": float(fp64), "achieved_tops": round(fp64 / ms_per_step / 1e9, 3),
                          "peak_tops": FP64_PEAK_TOPS, "frac": round(fp64 / ms_per_step / 1e9 / FP64_PEAK_TOPS, 4),
                          "note": "the binding roof of the bit-exact path (SURVEY §0.7): FP64 ops the reference's "
                                  "arithmetic needs per step over the step time"},
        }
        if fsk:
            workload = (f"FSK@{int(baud)} 96kHz tones {mark:g}/{space:g} Hz, batch {B} x {N} float32 streams per GPU "
                        "(BASELINE.json configs[2] at SURVEY §6's valid tones: the reference's defaults raise)")
        elif name == "ofdm8":
            workload = (f"OFDM8 = QPSK@{int(baud)} 96kHz (modem.py:375-376), global batch {B_global} x {N} float32 "
                        f"streams sharded over {world} GPU(s) (BASELINE.json configs[3])")
        elif fec_fused:
            workload = (f"8PSK@{int(baud)} = QPSK path (modem.py:348) + ReedSolomonFEC.decode fused, global batch "
                        f"{B_global} x {N} float32 streams sharded over {world} GPU(s) (BASELINE.json configs[4])")
        else:
            workload = f"QPSK@{int(baud)} 96kHz, batch {B} x {N} float32 streams per GPU (BASELINE.json configs[1])"
        result = {
            "metric": W["metric"], "value": round(value, 3), "unit": "Msym/s", "n_gpus": world, "steps": K,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload, "global_batch": B_global, "samples_per_stream": N,
                       "symbols_per_stream": sym_per_stream, "parallelism": f"streams sharded over {world} GPU(s)",
                       "batches_in_flight": P, "steps_per_launch": C, "streams_per_launch": BL,
                       "kernel_layout": layout,
                       "hw_queues": int(os.environ.get("GPU_MAX_HW_QUEUES", "4")),
                       "inputs": f"{P} distinct device batches per rank: {D} clean frames + per-slot N(0, 0.05^2) "
                                 "noise (amr_synth_tile_noise)"},
            "latency_ms_one_batch": lat1["ms"] if lat1 else (round(float(np.median(lat)) * 1e3, 3) if lat else None),
            "latency_ms_per_global_batch": round(float(np.mean(launch_ms)), 3) if launch_ms else None,
            "latency_per_global_batch_note": (
                f"in the timed pipeline ({P} launches in flight, {C} global batch(es) per launch): HIP events from "
                "a launch's first kernel to its outputs " + ("all-gathered (RCCL, the comm stream)" if comm is not None
                                                             else "written") +
                f", averaged over the last {len(launch_ms)} timed launches; every global batch of a launch "
                "finishes with it") if launch_ms else None,
            "latency_layout": lat1["layout"] if lat1 else latency_layout,
            "latency_note": ("one batch on a plan without the in-flight hint (a single-batch caller's layout), bytes "
                             f"equal to the lane layout's: {lat1['bytes_equal_lane_layout']}; the lane layout alone: "
                             f"{round(float(np.median(lat)) * 1e3, 3) if lat else None} ms") if lat1 else None,
            "roofline": roofline,
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "kernel_ms_solo": {k: round(v, 4) for k, v in solo.items()},
            "cpu_baseline": cpu,
            "parity": parity,
            "vs_reference_python": {
                "reference_1core_msym_s": REF_PY[name][0], "reference_8proc_msym_s": REF_PY[name][1],
                "ratio_1core": round(value / REF_PY[name][0], 1), "ratio_8proc": round(value / REF_PY[name][1], 1),
                "source": "BASELINE.md §2: the reference's modem.py on numpy 2.2.6 / scipy 1.15.3, measured in the "
                          "build container (8 cores), not on the GPU box"},
        }
        if sustained is not None:
            result["sustained"] = sustained
        if headline and name == "qpsk9600":
            # BASELINE.json north_star's three measurable targets, as this run meets them
            pl_ = roofline["pipeline"]
            result["north_star"] = {
                "x_reference_1core": round(value / REF_PY[name][0], 1), "target_x": 1e4,
                "hbm_frac_algorithmic": pl_["frac"],
                "hbm_frac_pmc_traffic": round(pl_["hbm_traffic_gbs"] / HBM_PEAK_GBS, 3) if pl_.get("hbm_traffic_gbs")
                else None,
                "target_hbm_frac": 0.40,
                "hbm_note": "algorithmic = the float32 input + decided bits per step (SURVEY 8(d)); a bit-exact "
                            "filtfilt must also move its f64 intermediates (SURVEY 0.7 caps the algorithmic "
                            "fraction near 0.16), so the PMC-counted traffic per step is the bandwidth actually "
                            "drawn from HBM",
                "parity": parity, "scaling_1_to_8": "measured by the driver from this line at N = 1, 2, 4, 8"}
        if gather_check is not None:
            result["gather_check"] = gather_check
        result["exact_path_streams"] = sum(pl.exact_streams() for pl in plans)
        if fsk:
            # device memory per plan: what the device entry holds (no dd, no
            # staging) beside what a host-entry plan of this shape takes
            result["plan_bytes"] = {"resident_per_plan": plans[0].resident_bytes(),
                                    "host_entry_plan": plans[0].scratch_bytes(), "plans": P,
                                    "resident_all_plans": sum(pl.resident_bytes() for pl in plans)}

        # PCIe-inclusive rate (never `value`): the host API on the
        # same batch from host memory, H2D + demod + D2H, one batch at a time
        if headline and world == 1 and not fec_fused and not args.no_host_path:
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(xh), ctx[0]["x"], xh.nbytes))
            o0, ln0 = outs[0][:2]
            host_res = (xh, o0, ln0)
    elif gather_check is not None and "MISMATCH" in gather_check:
        log(f"[rank {rank}] {name}: {gather_check}")
    fsk_one = None
    if result is not None and fsk and world == 1 and not args.no_dropin:
        n1 = min(BL, 8)
        x8 = np.empty((n1, N), np.float32)
        _amr.check(L.amr_memcpy_d2h(_amr.ptr(x8), ctx[0]["x"], x8.nbytes))
        fsk_one = (x8, outs[0][0][:n1].copy(), outs[0][1][:n1].copy())
    for c in ctx:
        c.clear()
    del plans, ctx
    gc.collect()
    mem.close()
    if result is not None and host_res is not None:
        # after the benchmark's plans and buffers are released
        result["host_path_pcie_inclusive"] = host_path(L, fsk, host_res[0], B, N, baud, mark, space, dev, cap,
                                                       sym_per_stream, host_res[1], host_res[2], args.host_plans)
        if not args.no_dropin and not fsk:
            result["dropin"] = dropin_path(host_res[0], baud, sym_per_stream, host_res[1], host_res[2])
    if result is not None and fsk and world == 1 and not args.no_cpu:
        result["exact_probe"] = fsk_exact_probe(N, baud, mark, space, dev)
    if result is not None and fsk_one is not None:
        result["dropin"] = fsk_dropin_path(*fsk_one, baud, mark, space)
    return result


def fsk_dropin_path(xh, out_dev, len_dev, baud, mark, space):
    """modem.fsk_demodulate(x) on one 1-s capture at a time -- the reference's
    own call pattern (filebeep_advanced_v2.py:324) -- which runs the FSK
    time-split F1, beside the serial F1 on the same captures
    and the C port on one host core; bytes checked against the device path's.
    Never `value`."""
    import _fsk
    import modem
    args = dict(baud=baud, mark_freq=mark, space_freq=space)
    n1, N = xh.shape
    modem.fsk_demodulate(xh[0], **args)                    # plan and scratch
    plan1 = _fsk.get_fsk_plan(N, baud, mark, space, FS, 1)
    ts, flagged, same = [], 0, True
    for i in range(n1):
        t1 = time.perf_counter()
        r = modem.fsk_demodulate(xh[i], **args)
        ts.append(time.perf_counter() - t1)
        same &= r == out_dev[i, :len_dev[i]].tobytes()
        flagged += plan1.exact_streams()
    ser = _fsk.FskPlan(N, baud, mark, space, FS, max_streams=1)
    ser.set_layout("serial")
    ser.demod_host(xh[:1])
    tr = []
    for i in range(n1):
        t1 = time.perf_counter()
        ser.demod_host(xh[i:i + 1])
        tr.append(time.perf_counter() - t1)
    del ser
    from oracle import oracle
    tc = []
    for i in range(3):
        t1 = time.perf_counter()
        oracle.fsk_demodulate(xh[i], **args)
        tc.append(time.perf_counter() - t1)
    info = plan1.split_info()
    info["strict"] = plan1.last_strict()
    info["margin"] = plan1.margin()
    # round 5's kappa margin on the same captures (AMR_FSK_SPLIT_STRICT=0): latency and exact-path count
    plan1.set_split_strict(False)
    tk, fk = [], 0
    for i in range(n1):
        t1 = time.perf_counter()
        r = modem.fsk_demodulate(xh[i], **args)
        tk.append(time.perf_counter() - t1)
        same &= r == out_dev[i, :len_dev[i]].tobytes()
        fk += plan1.exact_streams()
    plan1.set_split_strict(None)
    info["kappa_margin"] = {"ms": round(float(np.median(tk)) * 1e3, 3), "flagged_of": f"{fk}/{n1}"}
    # a capture that opens with digital silence (as a padded WAV does): its
    # compares there sit inside the margin, so the call also runs the exact
    # path (the serial F1 again, then pocketfft's envelopes)
    xs = xh[0].copy()
    xs[:N // 5] = 0.0
    want = oracle.fsk_demodulate(xs, **args)
    tf, fl_s = [], 0
    for _ in range(3):
        t1 = time.perf_counter()
        r = modem.fsk_demodulate(xs, **args)
        tf.append(time.perf_counter() - t1)
        fl_s = plan1.exact_streams()
    flagged_capture = {"ms": round(float(np.median(tf)) * 1e3, 3), "flagged": int(fl_s), "bytes_equal": r == want,
                       "what": "the same call on capture 0 with its first fifth set to digital silence"}
    return {"one_capture": {"ms": round(float(np.median(ts)) * 1e3, 3), "ms_min": round(min(ts) * 1e3, 3),
                            "split": info, "flagged_of": f"{flagged}/{n1}", "flagged_capture": flagged_capture,
                            "serial_f1_ms": round(float(np.median(tr)) * 1e3, 3),
                            "c_port_1core_ms": round(float(np.median(tc)) * 1e3, 3), "bytes_equal": bool(same),
                            "what": f"modem.fsk_demodulate(x, baud={int(baud)}) on one {N}-sample float32 capture "
                                    f"(H2D + demod + D2H, cached plan), median over {n1} distinct captures of the "
                                    "benchmark batch; serial_f1_ms: the same calls with the serial F1; "
                                    "c_port_1core_ms: the oracle's C restatement (filtfilt + pocketfft) on one core"}}


def fsk_exact_probe(N, baud, mark, space, dev, B=2048):
    """The FSK exact path at scale (never `value`): B
    zero-padded captures -- digital silence before the frame, as a gated
    receiver records them -- whose compares F2 flags, every stream forced
    through the exact path (mode 2), and the same batch with a noise floor
    (nothing flagged); device time of one launch (HIP events, first kernel to
    last output), H2D / D2H excluded, median of 3."""
    import _fsk
    import synth
    rng = np.random.default_rng(5)
    rows = []
    for i in range(B):
        w = synth.fsk_waveform(synth.random_frame(rng, 40), baud, mark, space, float(FS))
        off = 2000 + 37 * (i % 512)
        row = np.zeros(N, np.float32)
        seg = w[:N - off]
        row[off:off + seg.size] = seg
        rows.append(row)
    x = np.stack(rows)
    pl = _fsk.FskPlan(N, baud, mark, space, FS, max_streams=B, device=dev)
    pl.enable_timing(True)
    res = {"streams": B, "samples": N, "unit": "ms"}
    if os.environ.get("AMR_FSK_EXACT", "1") == "0":   # (an A/B run with the exact path off)
        return {**res, "skipped": "AMR_FSK_EXACT=0"}
    for label, xx, mode in (("silent_padded", x, 1), ("all_exact", x, 2),
                            ("noise_floor", x + rng.normal(0, 0.01, x.shape).astype(np.float32), 1)):
        pl.set_exact_mode(mode)
        pl.demod_host(xx)
        ts, ex = [], []
        for _ in range(3):
            pl.demod_host(xx)
            t = pl.timings()
            ts.append(t["launch"])
            ex.append(t.get("exact", 0.0))
        res[label] = {"launch_ms": round(float(np.median(ts)), 2), "exact_stage_ms": round(float(np.median(ex)), 2),
                      "exact_path_streams": pl.exact_streams()}
    del pl
    gc.collect()
    return res


def row_bytes(x, baud):
    """One capture through a plan forced to the serial row layout."""
    pl = _amr.PskPlan("qpsk", x.size, baud, max_streams=1)
    pl.set_layout("row")
    return pl.demod_host(np.ascontiguousarray(x)[None])[0][0]


def dropin_path(xh, baud, sym_per_stream, out_dev, len_dev):
    """The reference's own call surface, as filebeep_advanced_v2.py uses it
    (never `value`): the drop-in modules from host memory.
      * one capture: modem.qpsk_demodulate(x) on one 1-s stream, the live
        receive path's call (plan cached after the first call);
      * a batch: modem.qpsk_demodulate_batch + decoder.parse_fbp_stream_enhanced_batch
        (GPU frame scan + payload CRC32) + intelligent_decompress of every
        frame -- decode_from_buffer without the file writes -- over the
        benchmark batch (outputs checked equal to the device path's bytes);
      * the same over 1024 captures at QPSK@1000, a rate at which the
        reference's own modulator and demodulator round-trip (at 9600 Bd they
        do not: SURVEY §0 finding 4, so the benchmark batch recovers no file,
        as the reference recovers none): files recovered = captures whose
        frame passed its payload CRC32."""
    import contextlib
    import io
    import modem
    import decoder
    from compression import intelligent_decompress
    B = xh.shape[0]
    res = {"unit": "ms"}
    x1 = np.ascontiguousarray(xh[0])
    one = modem.qpsk_demodulate(x1, baud=baud)
    # one capture at a time: the time-split layout, 8 distinct
    # captures of the benchmark batch, each call timed; bytes checked against
    # the device path's
    n1 = min(B, 8)
    plan1 = _amr.get_psk_plan("qpsk", x1.size, baud, 3000.0, FS, 1)
    ts, flagged, same = [], 0, True
    for i in range(n1):
        xi = np.ascontiguousarray(xh[i])
        t1 = time.perf_counter()
        r = modem.qpsk_demodulate(xi, baud=baud)
        ts.append(time.perf_counter() - t1)
        same &= r == out_dev[i, :len_dev[i]].tobytes()
        flagged += max(0, plan1.split_info()["flagged"])
    # the serial row layout on the same captures (round 4's one-capture path)
    row = _amr.PskPlan("qpsk", x1.size, baud, max_streams=1)
    row.set_layout("row")
    row.demod_host(x1[None])
    tr = []
    for i in range(n1):
        t1 = time.perf_counter()
        row.demod_host(np.ascontiguousarray(xh[i:i + 1]))
        tr.append(time.perf_counter() - t1)
    del row
    res["one_capture"] = {"ms": round(float(np.median(ts)) * 1e3, 3), "ms_min": round(min(ts) * 1e3, 3),
                          "layout": plan1.last_layout(), "split": plan1.split_info(),
                          "flagged_of": f"{flagged}/{n1}", "row_layout_ms": round(float(np.median(tr)) * 1e3, 3),
                          "what": f"modem.qpsk_demodulate(x, baud={int(baud)}) on one {x1.size}-sample float32 capture "
                                  f"(H2D + demod + D2H, cached plan), median over {n1} distinct captures of the "
                                  "benchmark batch; row_layout_ms: the same calls on the serial row layout",
                          "bytes_equal": bool(one == out_dev[0, :len_dev[0]].tobytes() and same)}
    # a capture that opens with digital silence: exact zero products are
    # flagged, so the call also runs the gated serial kernels
    xs = x1.copy()
    xs[:x1.size // 5] = 0.0
    want_s = modem.qpsk_demodulate(xs, baud=baud)
    tf = []
    for _ in range(3):
        t1 = time.perf_counter()
        r = modem.qpsk_demodulate(xs, baud=baud)
        tf.append(time.perf_counter() - t1)
    res["one_capture"]["flagged_capture"] = {
        "ms": round(float(np.median(tf)) * 1e3, 3), "flagged": int(plan1.split_info()["flagged"]),
        "bytes_equal_row_layout": r == want_s and r == row_bytes(xs, baud),
        "what": "the same call on capture 0 with its first fifth set to digital silence"}
    # how many single captures the margin sends to the serial path: the first
    # 1024 streams of the benchmark batch, 16 per call, time-split layout forced
    nsp = min(B, 1024)
    sp = _amr.PskPlan("qpsk", x1.size, baud, max_streams=16)
    sp.set_layout("split")
    fl, eq = 0, True
    for s0 in range(0, nsp, 16):
        g, _ = sp.demod_host(np.ascontiguousarray(xh[s0:s0 + 16]))
        fl += sp.split_info()["flagged"]
        eq &= all(g[j] == out_dev[s0 + j, :len_dev[s0 + j]].tobytes() for j in range(len(g)))
    res["split_flag_rate"] = {"flagged": fl, "streams": nsp, "fraction": round(fl / nsp, 5), "bytes_equal": bool(eq),
                              "kappa": sp.split_info()["kappa"],
                              "what": "time-split layout over the benchmark's noisy captures (16 per call): streams "
                                      "with a decision inside the error margin, re-run by the serial kernels"}
    # the same with the strict margin (a per-symbol rounding bound that holds
    # for every input) in place of kappa's measured premise
    sp.set_split_strict(True)
    fl, eq = 0, True
    for s0 in range(0, nsp, 16):
        g, _ = sp.demod_host(np.ascontiguousarray(xh[s0:s0 + 16]))
        fl += sp.split_info()["flagged"]
        eq &= all(g[j] == out_dev[s0 + j, :len_dev[s0 + j]].tobytes() for j in range(len(g)))
    res["split_flag_rate"]["strict"] = {"flagged": fl, "fraction": round(fl / nsp, 5), "bytes_equal": bool(eq),
                                        "last_strict": sp.last_strict()}
    del sp
    # one capture at a time with the strict margin: latency and how many of
    # the captures went to the serial kernels
    plan1.set_split_strict(True)
    modem.qpsk_demodulate(np.ascontiguousarray(xh[n1 % B]), baud=baud)   # the strict design and scratch, once
    ts, flagged, same = [], 0, True
    for i in range(n1):
        xi = np.ascontiguousarray(xh[i])
        t1 = time.perf_counter()
        r = modem.qpsk_demodulate(xi, baud=baud)
        ts.append(time.perf_counter() - t1)
        same &= r == out_dev[i, :len_dev[i]].tobytes()
        flagged += max(0, plan1.split_info()["flagged"])
    res["one_capture"]["strict"] = {"ms": round(float(np.median(ts)) * 1e3, 3), "ms_max": round(max(ts) * 1e3, 3),
                                    "flagged_of": f"{flagged}/{n1}", "bytes_equal": bool(same),
                                    "last_strict": plan1.last_strict(),
                                    "what": "the same calls with AMR_PSK_SPLIT_STRICT's margin on this plan "
                                            "(amr_psk_plan_set_split_strict): median and worst call"}
    plan1.set_split_strict(None)
    # the same capture through the C port on one host core (the CPU side of
    # the single-capture call pattern, filebeep_advanced_v2.py:324), and where
    # the GPU drop-in overtakes one core / all host cores as the batch grows
    from oracle import oracle
    threads, _ = host_cores()
    tc = []
    for _ in range(5):
        t1 = time.perf_counter()
        oracle.psk_demod_batch("qpsk", x1[None], baud, n_threads=1)
        tc.append(time.perf_counter() - t1)
    c1 = float(np.median(tc))
    res["one_capture"]["c_port_1core_ms"] = round(c1 * 1e3, 3)
    nb = min(B, 64)
    t1 = time.perf_counter()
    oracle.psk_demod_batch("qpsk", xh[:nb], baud, n_threads=threads)
    cn = (time.perf_counter() - t1) / nb
    gpu = {}
    for b in (1, 2, 4, 8, 16, 32, 64, 128, 256):
        if b > B:
            break
        xb = np.ascontiguousarray(xh[:b])
        modem.qpsk_demodulate_batch(xb, baud=baud)          # plan for this bucket
        tg = []
        for _ in range(3):
            t1 = time.perf_counter()
            modem.qpsk_demodulate_batch(xb, baud=baud)
            tg.append(time.perf_counter() - t1)
        gpu[b] = min(tg)
    over1 = next((b for b, t in gpu.items() if t < b * c1), None)
    overn = next((b for b, t in gpu.items() if t < b * cn), None)
    res["crossover"] = {
        "gpu_dropin_ms": {str(b): round(t * 1e3, 3) for b, t in gpu.items()},
        "cpu_1core_ms_per_capture": round(c1 * 1e3, 3),
        f"cpu_{threads}core_ms_per_capture": round(cn * 1e3, 3),
        "gpu_overtakes_1core_at_batch": over1, f"gpu_overtakes_{threads}core_at_batch": overn,
        "what": "modem.qpsk_demodulate_batch (host memory in and out, cached plans) vs the C port "
                "(oracle.psk_demod_batch) on the same 1-s captures; the first batch size measured at which "
                "the GPU call is faster (None: not within the sizes measured)"}

    def run():
        raws = modem.qpsk_demodulate_batch(xh, baud=baud)
        frames = decoder.parse_fbp_stream_enhanced_batch(raws)
        files = [[intelligent_decompress(f["data"]) for f in fs] for fs in frames]
        return raws, frames, files
    with contextlib.redirect_stdout(io.StringIO()):      # the reference's per-frame log lines
        run()
        ts = []
        for _ in range(2):
            t1 = time.perf_counter()
            raws, frames, files = run()
            ts.append(time.perf_counter() - t1)
    dt = min(ts)
    ok = sum(1 for fs in frames if len(fs) == 1)
    res["batch"] = {"ms": round(dt * 1e3, 2), "msym_per_s": round(B * sym_per_stream / dt / 1e6, 3),
                    "files_recovered": f"{ok}/{B} (the reference's QPSK@9600 does not round-trip)",
                    "bytes_equal": {"device_path": all(r == out_dev[i, :len_dev[i]].tobytes()
                                                       for i, r in enumerate(raws))},
                    "what": "qpsk_demodulate_batch + parse_fbp_stream_enhanced_batch + intelligent_decompress over "
                            f"the {B} x {xh.shape[1]} benchmark batch from pageable host memory (decode_from_buffer "
                            "per stream, without the file writes)"}

    # files end to end at a round-tripping rate
    b2, n2 = 1024, xh.shape[1]
    x2 = synth.qpsk_batch(b2, n2, 1000, seed=7, noise=0.05, distinct=64)
    with contextlib.redirect_stdout(io.StringIO()):
        raws = modem.qpsk_demodulate_batch(x2, baud=1000)
        ts = []
        for _ in range(2):
            t1 = time.perf_counter()
            raws = modem.qpsk_demodulate_batch(x2, baud=1000)
            frames = decoder.parse_fbp_stream_enhanced_batch(raws)
            files = [[intelligent_decompress(f["data"]) for f in fs] for fs in frames]
            ts.append(time.perf_counter() - t1)
    dt = min(ts)
    ok = sum(1 for fs in files if len(fs) == 1 and len(fs[0]) > 0)
    res["files"] = {"ms": round(dt * 1e3, 2), "files_per_s": round(ok / dt, 1), "files_recovered": f"{ok}/{b2}",
                    "what": f"decode_from_buffer's steps (without the file writes) over {b2} x {n2} float32 QPSK@1000 "
                            "captures of one FBPC frame each (synth.qpsk_batch, N(0, 0.05^2) noise), from host memory"}
    return res


def host_path(L, fsk, xh, B, N, baud, mark, space, dev, cap, sym_per_stream, out_dev, len_dev, host_plans=0):
    """PCIe-inclusive rates from host memory (never `value`):
      * one batch at a time: amr_*_demod_host from pageable memory, H2D +
        demod + D2H, on a plan without an in-flight hint (latency layout);
      * a stream of batches: amr_*_demod_host_async on 3 plans in turn from a
        page-locked buffer, so batch k+1's upload overlaps batch k's demod.
    Both outputs are checked equal to the device path's bytes."""
    mk = (lambda: __import__("_fsk").FskPlan(N, baud, mark, space, FS, max_streams=B, device=dev)) if fsk else \
        (lambda: _amr.PskPlan("qpsk", N, baud, 3000.0, FS, max_streams=B, device=dev))
    host_fn = L.amr_fsk_demod_host if fsk else L.amr_psk_demod_host
    async_fn = L.amr_fsk_demod_host_async if fsk else L.amr_psk_demod_host_async
    sync_fn = L.amr_fsk_plan_synchronize if fsk else L.amr_psk_plan_synchronize

    def same(o, ln):
        return bool(np.array_equal(ln, len_dev) and all(o[i, :ln[i]].tobytes() == out_dev[i, :ln[i]].tobytes()
                                                        for i in range(B)))
    res = {"input_gb_per_batch": round(xh.nbytes / 1e9, 3), "unit": "Msym/s"}
    plan = mk()
    h_out = np.empty((B, cap), np.uint8)
    h_len = np.empty(B, np.int64)
    h_sync = np.empty(B, np.int64)
    hts = []
    for _ in range(3):
        t1 = time.perf_counter()
        _amr.check(host_fn(plan.handle, _amr.ptr(xh), _amr.DTYPE_F32, B, N, _amr.ptr(h_out), cap, _amr.ptr(h_len),
                           _amr.ptr(h_sync)))
        hts.append(time.perf_counter() - t1)
    ht = min(hts[1:])
    res["one_batch"] = {"ms_per_batch": round(ht * 1e3, 2), "value": round(B * sym_per_stream / ht / 1e6, 3),
                        "what": "amr_%s_demod_host from pageable host float32 (H2D + demod + D2H)"
                                % ("fsk" if fsk else "psk"), "bytes_equal": {"device_path": same(h_out, h_len)}}
    del plan
    gc.collect()
    n_pl = host_plans or (2 if fsk else 3)
    n_batches = 2 * n_pl
    plans = [mk() for _ in range(n_pl)]
    if not fsk:
        for pl in plans:
            pl.set_inflight(n_pl)
    # the capture buffer and the per-plan outputs in page-locked memory
    # (amr_host_alloc), as a receiver would allocate them once
    pouts = [(_amr.PinnedArray((B, cap), np.uint8), _amr.PinnedArray((B,), np.int64), _amr.PinnedArray((B,), np.int64))
             for _ in range(n_pl)]
    outs = [tuple(a.array for a in t) for t in pouts]

    def stream(src, dtype):
        for k in range(n_pl):                                       # warm every plan once
            o, ln, sy = outs[k]
            _amr.check(async_fn(plans[k].handle, _amr.ptr(src), dtype, B, N, _amr.ptr(o), cap,
                                _amr.ptr(ln), _amr.ptr(sy)))
        for pl in plans:
            _amr.check(sync_fn(pl.handle))
        t1 = time.perf_counter()
        for k in range(n_batches):
            pl = plans[k % n_pl]
            if k >= n_pl:
                _amr.check(sync_fn(pl.handle))                      # its previous batch's bytes are read
            o, ln, sy = outs[k % n_pl]
            _amr.check(async_fn(pl.handle, _amr.ptr(src), dtype, B, N, _amr.ptr(o), cap,
                                _amr.ptr(ln), _amr.ptr(sy)))
        for pl in plans:
            _amr.check(sync_fn(pl.handle))
        return (time.perf_counter() - t1) / n_batches

    def entry(dt, nbytes, what, equal):
        return {"ms_per_batch": round(dt * 1e3, 2), "value": round(B * sym_per_stream / dt / 1e6, 3),
                "h2d_gbs": round(nbytes / dt / 1e9, 1), "what": what, "bytes_equal": equal}

    try:
        pin = _amr.PinnedArray(xh.shape, np.float32)
        pin.array[:] = xh
        dt = stream(pin.array, _amr.DTYPE_F32)
        res["stream_of_batches"] = entry(
            dt, xh.nbytes, f"amr_{'fsk' if fsk else 'psk'}_demod_host_async on {n_pl} plans in turn, {n_batches} "
            "float32 batches from a page-locked capture buffer (amr_host_alloc): uploads overlap demods",
            {"device_path": all(same(o, ln) for o, ln, _ in outs)})
        pin.close()
        # the same capture as 16-bit PCM (a WAV file's samples, modem.py's
        # read path): half the PCIe bytes; checked against the synchronous
        # host entry on the same int16 buffer
        pin16 = _amr.PinnedArray(xh.shape, np.int16)
        np.multiply(np.clip(xh, -3.9, 3.9), 8192.0, out=pin16.array, casting="unsafe")
        dt = stream(pin16.array, _amr.DTYPE_I16)
        ref = mk()
        _amr.check(host_fn(ref.handle, _amr.ptr(pin16.array), _amr.DTYPE_I16, B, N, _amr.ptr(h_out), cap,
                           _amr.ptr(h_len), _amr.ptr(h_sync)))
        del ref
        eq16 = all(np.array_equal(ln, h_len) and all(o[i, :ln[i]].tobytes() == h_out[i, :ln[i]].tobytes()
                                                     for i in range(B)) for o, ln, _ in outs)
        res["stream_of_batches_pcm16"] = entry(
            dt, pin16.array.nbytes, f"as stream_of_batches, the capture as int16 PCM ({pin16.array.nbytes / 1e9:.3f} GB "
            "per batch)", {"sync_host_entry": eq16})
        pin16.close()
    finally:
        for t in pouts:
            for a in t:
                a.close()
    res["value"] = res["stream_of_batches"]["value"]
    return res


def launch_plan(K, B, strong, coalesce=0):
    """(C, BL, n_launch, streams of each launch) for K timed steps of B
    streams per rank: a strong-scaling shard too small to fill the GPU alone
    takes C consecutive global batches per launch (>= 4096 streams, what one
    headline batch holds); the last launch holds the remaining steps."""
    C = max(1, min(K, coalesce or (-(-4096 // B) if strong else 1)))
    n_launch = -(-K // C)
    sizes = [C * B] * (n_launch - 1) + [(K - (n_launch - 1) * C) * B]
    return C, C * B, n_launch, sizes


def default_inflight(K, cap=20):
    """Batches in flight for K timed PSK steps.  Measured on one MI355X
    (DESIGN.md §4): whole rounds win -- a partial last round runs a few
    batches on an otherwise idle GPU (K=20: P=10 4.81 ms/step, P=16 5.05,
    P=20 3.97) -- and past ~20 HIP streams the hardware queues time-slice
    (K=64: P=16 4.1 ms, P=32 5.1).  So P = K up to `cap`, else the divisor of
    K in cap/2..cap closest to 16, else 16.  `cap` is 16 for the 8192-stream
    batches (HBM: ~13 GB of plan scratch + input per batch)."""
    if K <= cap:
        return max(1, K)
    divs = [d for d in range(max(1, cap // 2), cap + 1) if K % d == 0]
    return min(divs, key=lambda d: abs(d - 16)) if divs else min(16, cap)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--sub-steps", type=int, default=64,
                    help="timed steps of each sub-workload of the default run (fsk9600, ofdm8, psk8fec)")
    ap.add_argument("--workload", choices=list(WORKLOADS), default="qpsk9600",
                    help="the headline; qpsk9600 (BASELINE configs[1]) also reports the other configs as sub-objects")
    ap.add_argument("--no-sub", action="store_true", help="skip the sub-workloads of the default run")
    ap.add_argument("--batch", type=int, default=0,
                    help="streams per GPU (qpsk9600/fsk9600, default 4096/16384) or in total (ofdm8/psk8fec, 8192)")
    ap.add_argument("--samples", type=int, default=96000)
    ap.add_argument("--mark", type=float, default=12000.0, help="fsk9600: mark tone (SURVEY §6 config 3)")
    ap.add_argument("--space", type=float, default=24000.0, help="fsk9600: space tone")
    ap.add_argument("--distinct", type=int, default=64, help="clean frames per rank (noise is per stream and slot)")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-API timing")
    ap.add_argument("--sustain-seconds", type=float, default=2.0,
                    help="after the timed region, run the headline pipeline this long again and report it as "
                         "`sustained` (0 = skip)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the N > 1 path (RCCL communicator, per-launch all-gather, gather check) even for one "
                         "rank; needs torch.distributed.run's rendezvous variables")
    ap.add_argument("--host-plans", type=int, default=0,
                    help="plans the PCIe-inclusive stream of batches uses in turn (0 = 3 PSK / 2 FSK)")
    ap.add_argument("--no-dropin", action="store_true", help="skip the drop-in module timing (modem / decoder calls)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the oracle parity check and CPU baseline (profiling)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0,
                    help="wall time of the headline's CPU baseline (the oracle over batch 0, repeated)")
    ap.add_argument("--parity-all-slots", action="store_true", help="check sampled streams of every in-flight slot")
    ap.add_argument("--hw-queues", type=int, default=32, help="GPU_MAX_HW_QUEUES for this process (<= 32)")
    ap.add_argument("--no-latency", action="store_true",
                    help="skip the one-batch latency-layout run after timing (profiling)")
    ap.add_argument("--host-wait", action="store_true",
                    help="wait on the host for a plan's previous batch before queueing the next on it")
    ap.add_argument("--coalesce", type=int, default=0,
                    help="steps per launch (0 = enough for >= 4096 streams per launch on strong-scaling shards, "
                         "else 1)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight on separate plans / HIP streams (0 = default_inflight(steps); fsk9600 4)")
    args = ap.parse_args()

    L = _amr.lib()
    tp, world, rank, local = dist_setup(args.force_comm)
    dev = local
    _amr.check(L.amr_set_device(dev))
    comm = tp.comm if tp is not None else None

    result = run_workload(args.workload, args, tp, world, rank, dev, comm, headline=True)
    if args.workload == "qpsk9600" and not args.no_sub and not args.batch:
        subs = {}
        for name in ("fsk9600", "ofdm8", "psk8fec"):
            r = run_workload(name, args, tp, world, rank, dev, comm, headline=False)
            if rank == 0 and r is not None:
                subs[name] = {k: r[k] for k in ("metric", "value", "unit", "steps", "ms_per_step", "scaling", "parity",
                                                "latency_ms_one_batch", "latency_ms_per_global_batch", "kernel_ms",
                                                "kernel_ms_solo", "cpu_baseline", "config")}
                subs[name]["roofline"] = {k: r["roofline"][k] for k in ("kernel", "achieved", "frac", "frac_throughput", "kernel_ms_used", "inflight", "pipeline",
                                                                          "fp64_valu")}
                for k in ("gather_check", "exact_path_streams", "exact_probe", "plan_bytes", "dropin"):
                    if k in r:
                        subs[name][k] = r[k]
        if rank == 0 and result is not None:
            result["workloads"] = subs
    if rank == 0 and result is not None:
        result["build_id"] = L.amr_build_id().decode()
        print(json.dumps(result), flush=True)
    if tp is not None:
        tp.close()


if __name__ == "__main__":
    main()
