#!/usr/bin/env python3
"""bench.py -- BASELINE.json's headline metric on MI355X.

metric : demod Msymbols/s (batch) + achieved HBM GB/s, QPSK@9600/96kHz
workload (N=1): BASELINE configs[1] -- QPSK @ 9600 sym/s, 96 kHz, batch 4096
          synthetic 1-s streams (N = 96000 float32 samples each), inputs
          resident in HBM before the timed region.
step   : one pass of the whole demod path over the batch:
          band-pass filtfilt + mixer -> low-pass filtfilt + slicer ->
          [exact-path fixups] -> sync + pack  (and, for N>1 GPUs, the RCCL
          all-gather of the decoded bytes).
scaling: weak -- every rank demodulates its own 4096 streams; value is the
          whole-job symbols/s = (ranks * 4096 * 9599) / max-over-ranks time.

Usage:  python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
        multi-GPU: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "audio-modem-radio_amd"))
sys.path.insert(0, ROOT)

import _amr  # noqa: E402
import synth  # noqa: E402

FS = 96000
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PROFILE_ROUND = "r01"           # profiles/<round>_pmc.json holds the PMC traffic per timing slot
FP64_PEAK_TOPS = 39.3          # non-fused FP64 vector ops/s (78.6 TFLOP/s counts an FMA as 2)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def dist_setup(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
        return dist, world, rank, local
    return None, 1, 0, local


def barrier(dist):
    if dist is not None:
        dist.barrier()


def max_over_ranks(dist, v: float) -> float:
    if dist is None:
        return v
    import torch
    t = torch.tensor([v], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cpu_baseline(x_sample: np.ndarray, baud: float, threads: int):
    """The oracle (C restatement of the reference path) on the host cores."""
    from oracle import oracle
    oracle.lib()
    t0 = time.perf_counter()
    outs, _ = oracle.psk_demod_batch("qpsk", x_sample, baud, n_threads=threads)
    dt = time.perf_counter() - t0
    sps = int(FS / baud)
    S = (x_sample.shape[1] - sps // 2 + sps - 1) // sps
    return x_sample.shape[0] * (S - 1) / dt / 1e6, dt, outs


def cpu_baseline_fsk(x_sample: np.ndarray, baud, mark, space, threads: int):
    """oracle.fsk_demodulate (C filtfilt + scipy's hilbert + C decide) on the host cores."""
    from concurrent.futures import ThreadPoolExecutor

    from oracle import oracle
    oracle.lib()
    t0 = time.perf_counter()
    with ThreadPoolExecutor(threads) as ex:
        outs = list(ex.map(lambda r: oracle.fsk_demodulate(r, baud, mark, space), x_sample))
    dt = time.perf_counter() - t0
    sps = int(FS / baud)
    nb = (x_sample.shape[1] - sps // 2 + sps - 1) // sps
    return x_sample.shape[0] * nb / dt / 1e6, dt, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 20 batches: with 3 in flight the timed region starts and ends with a
    # part-full pipeline; 5 steps measured 8.4-9.3 ms/step, 24 steps 8.1-8.7
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=["qpsk9600", "fsk9600", "ofdm8", "psk8fec"], default="qpsk9600",
                    help="qpsk9600 = BASELINE configs[1] (the headline metric); fsk9600 = configs[3]; "
                         "ofdm8 = configs[4] (QPSK alias, global batch 8192 sharded); psk8fec = configs[5] "
                         "(8PSK@19200 + fused FEC decode, global batch 8192 sharded)")
    ap.add_argument("--batch", type=int, default=0,
                    help="streams per GPU (qpsk9600/fsk9600, default 4096/16384) or in total (ofdm8/psk8fec, "
                         "default 8192)")
    ap.add_argument("--samples", type=int, default=96000)
    ap.add_argument("--baud", type=float, default=None, help="default 9600 (19200 for psk8fec)")
    ap.add_argument("--mark", type=float, default=12000.0, help="fsk9600: mark tone (SURVEY §6 config 3)")
    ap.add_argument("--space", type=float, default=24000.0, help="fsk9600: space tone")
    ap.add_argument("--distinct", type=int, default=64, help="distinct waveforms (noise is per stream)")
    ap.add_argument("--cpu-streams", type=int, default=0, help="cpu_baseline sample size (0 = auto ~10 s CPU)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-host-path", action="store_true", help="skip the PCIe-inclusive host-API timing")
    ap.add_argument("--inflight", type=int, default=0,
                    help="batches in flight on separate HIP streams / plans (0 = 3 for the PSK workloads, 2 for "
                         "fsk9600): batch k+1's band-pass overlaps batch k's low-pass passes")
    args = ap.parse_args()

    dist, world, rank, local = dist_setup(args.gpus)
    dev = local
    fsk = args.workload == "fsk9600"
    fec_fused = args.workload == "psk8fec"
    strong = args.workload in ("ofdm8", "psk8fec")       # a fixed global batch sharded over the ranks
    if strong:
        from multi import shard_range
        B_global = args.batch or 8192
        lo_s, hi_s = shard_range(B_global, rank, world)
        B = hi_s - lo_s
        B_slot = -(-B_global // world)                    # all-gather slot (ranks' shards differ by <= 1)
    else:
        B = args.batch or (16384 if fsk else 4096)
        B_global = world * B
        lo_s = rank * B
        B_slot = B
    N = args.samples
    baud = args.baud or (19200.0 if fec_fused else 9600.0)
    L = _amr.lib()
    _amr.check(L.amr_set_device(dev))

    t0 = time.perf_counter()
    if fsk:
        x = synth.fsk_batch(B, N, baud, args.mark, args.space, seed=1000 + rank, distinct=args.distinct)
    elif fec_fused:
        x = synth.dpsk8_batch(B, N, baud, seed=1000 + rank, distinct=args.distinct)
    else:
        x = synth.qpsk_batch(B, N, baud, seed=1000 + rank, distinct=args.distinct)
    log(f"[rank {rank}] synthesised {B}x{N} float32 in {time.perf_counter() - t0:.1f}s")

    inflight = args.inflight or (2 if fsk else 3)         # same-box fsk9600: 1 -> 40.3, 2 -> 39.15 ms
    if fsk:
        import _fsk
        plans = [_fsk.FskPlan(N, baud, args.mark, args.space, FS, max_streams=B, device=dev) for _ in range(inflight)]
        plan = plans[0]
        sym_per_stream = (N - plan.sps // 2 + plan.sps - 1) // plan.sps     # decided bits (modem.py:320)
        demod, sync_fn, names = L.amr_fsk_demod_device, L.amr_fsk_plan_synchronize, _amr.TF_NAMES
    else:
        plans = [_amr.PskPlan("qpsk", N, baud, 3000.0, FS, max_streams=B, device=dev) for _ in range(inflight)]
        plan = plans[0]
        S = (N - plan.first + plan.sps - 1) // plan.sps
        sym_per_stream = S - 1                       # differential symbols decided per stream
        demod, sync_fn, names = L.amr_psk_demod_device, L.amr_psk_plan_synchronize, _amr.T_NAMES
    for pl in plans:
        pl.enable_timing(True)
        if not fsk:
            pl.set_inflight(inflight)
    cap = plan.out_cap

    def dmalloc(nbytes):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), int(nbytes)))
        return p

    d_x = dmalloc(x.nbytes)
    _amr.check(L.amr_memcpy_h2d(d_x, _amr.ptr(x), x.nbytes))
    # per batch in flight: its plan (stream + scratch) and its output / gather buffers
    ctx = []
    for pl in plans:
        c = {"plan": pl, "out": dmalloc(B_slot * cap), "len": dmalloc(B_slot * 8), "sync": dmalloc(B_slot * 8)}
        if fec_fused:
            c.update(fec=dmalloc(B_slot * cap), flen=dmalloc(B_slot * 8), ok=dmalloc(B_slot * 4))
        ctx.append(c)
    comm = None
    if world > 1:
        uid = (ctypes.c_uint8 * 128)()
        if rank == 0:
            _amr.check(L.amr_comm_unique_id(uid))
        obj = [bytes(uid)]
        dist.broadcast_object_list(obj, src=0)
        uid = (ctypes.c_uint8 * 128).from_buffer_copy(obj[0])
        comm = ctypes.c_void_p()
        _amr.check(L.amr_comm_create(ctypes.byref(comm), uid, world, rank, dev))
        for c in ctx:
            c["gather"], c["gather_len"] = dmalloc(world * B_slot * cap), dmalloc(world * B_slot * 8)

    def step(c):
        pl = c["plan"]
        if fec_fused:
            _amr.check(L.amr_psk_demod_fec_device(pl.handle, d_x, _amr.DTYPE_F32, B, N, c["out"], cap, c["len"],
                                                  c["sync"], c["fec"], cap, c["flen"], c["ok"]))
        else:
            _amr.check(demod(pl.handle, d_x, _amr.DTYPE_F32, B, N, c["out"], cap, c["len"], c["sync"]))
        if comm is not None:
            # the bytes every rank hands to the gather (the FEC output for psk8fec),
            # to every rank (RCCL over xGMI), on the plan's stream (FSK: the comm's)
            g_out, g_len = (c["fec"], c["flen"]) if fec_fused else (c["out"], c["len"])
            gs = None if fsk else pl.handle
            if fsk:
                _amr.check(sync_fn(pl.handle))
            _amr.check(L.amr_allgather(comm, g_out, c["gather"], B_slot * cap, gs))
            _amr.check(L.amr_allgather(comm, g_len, c["gather_len"], B_slot * 8, gs))
            if fsk:
                _amr.check(L.amr_comm_synchronize(comm))

    kt = {k: 0.0 for k in names}
    nt = [0]

    def collect(c):
        _amr.check(sync_fn(c["plan"].handle))
        for k, v in c["plan"].timings().items():
            kt[k] += v
        nt[0] += 1

    # warmup: one batch at a time (also the kernels' solo durations), then with the batches in flight
    for i in range(args.warmup):
        step(ctx[i % inflight])
        if i == 0 and args.warmup > 1:             # the first launch is cold: not counted
            _amr.check(sync_fn(ctx[0]["plan"].handle))
            continue
        collect(ctx[i % inflight])
    solo = {k: v / max(1, nt[0]) for k, v in kt.items() if v > 0}
    for i in range(min(args.warmup, inflight)):
        step(ctx[i])
    _amr.check(L.amr_device_synchronize())
    kt = {k: 0.0 for k in names}
    nt = [0]
    barrier(dist)
    _amr.check(L.amr_device_synchronize())
    t0 = time.perf_counter()
    # step k runs on ctx[k % inflight]; before a context is reused its previous
    # batch is waited for (the other batches keep running) and its kernel
    # timings are read
    for k in range(args.steps):
        c = ctx[k % inflight]
        if k >= inflight:
            collect(c)
        step(c)
    for k in range(max(0, args.steps - inflight), args.steps):
        collect(ctx[k % inflight])
    _amr.check(L.amr_device_synchronize())
    barrier(dist)
    dt = time.perf_counter() - t0
    dt = max_over_ranks(dist, dt)
    ms_per_step = dt / args.steps * 1e3
    total_sym = B_global * sym_per_stream
    value = total_sym / (dt / args.steps) / 1e6

    # per-kernel averages (HIP events on the plan's stream)
    kavg = {k: v / max(1, nt[0]) for k, v in kt.items() if v > 0}
    dom = max(kavg, key=kavg.get)
    # Algorithmic bytes per launch: each stage's
    # compulsory input + output at its minimal width.
    if fsk:
        #   bandpass : x float32 (4 B/sample) in, z = f_mark + i f_space (16 B) out
        #   hilbert  : z (16 B) in, compare byte (1 B) out -- the FFT's own passes
        #              over its intermediates are not algorithmic bytes
        #   decide   : compare bytes in the windows (sps//2 of every sps) + output bytes
        q = plan.sps // 4
        alg_bytes = {"bandpass": B * N * (4 + 16), "hilbert": B * N * 17,
                     "decide": B * (sym_per_stream * 2 * q + cap)}
        # FP64 ops: filtfilt 7 taps = 25 ops/sample/pass/tone; FFT ~ 5 n log2 n per transform
        fp64_ops = {"bandpass": B * 2 * 2 * (N + 42) * 25, "hilbert": B * 2 * 5 * N * np.log2(N)}
    else:
        #   bandpass    : x float32 (4 B/sample) in, filtered f float64 (8 B) out
        #   lowpass_fwd : f (8 B) in, forward low-pass complex128 (16 B) out
        #   lowpass_bwd : forward low-pass (16 B) in, symbol samples (16 B/symbol) out
        #   sync_pack   : symbols (16 B/symbol) in, packed bytes out
        S_sym = sym_per_stream + 1
        alg_bytes = {"bandpass": B * N * (4 + 8), "lowpass_fwd": B * N * (8 + 16),
                     "lowpass_bwd": B * (N * 16 + S_sym * 16), "sync_pack": B * (S_sym * 16 + cap),
                     "lowpass_exact": 0, "fec": B * 2 * cap}
        # FP64 operations scipy's arithmetic needs (no FMA): band-pass 30/sample per
        # pass (9 taps incl. the zero odd taps), low-pass 17/sample per pass per
        # component, mixer 2/sample
        fp64_ops = {"bandpass": B * 2 * (N + 54) * 30,
                    "lowpass_fwd": B * ((N + 30) * 2 * 17 + N * 2),
                    "lowpass_bwd": B * (N + 30) * 2 * 17}
    achieved = alg_bytes[dom] / (kavg[dom] / 1e3) / 1e9
    pipeline_bytes = B * N * 4 + B * sym_per_stream * (1 if fsk else 2) / 8
    fp64_achieved = fp64_ops.get(dom, 0) / (kavg[dom] / 1e3) / 1e12
    # the whole step's FP64 work over the step time: with batches in flight the
    # kernels share the SIMDs, so this (not the per-launch figure) is the
    # VALU-roofline view of the pipeline
    fp64_pipeline = sum(fp64_ops.values()) / (ms_per_step / 1e3) / 1e12
    traffic = None
    pipeline_traffic = None
    pmc_file = os.path.join(ROOT, "profiles", f"{PROFILE_ROUND}_pmc.json")
    # the PMC file was recorded at each workload's default size on one GPU
    pmc_cfg = {"qpsk9600": (4096, 9600), "fsk9600": (16384, 9600), "ofdm8": (8192, 9600), "psk8fec": (8192, 19200)}
    if ((B, int(baud)) == pmc_cfg[args.workload] and N == 96000 and world == 1 and os.path.exists(pmc_file)):
        with open(pmc_file) as f:
            pk = json.load(f).get(args.workload, {}).get("slots", {}).get(dom, {})
        if "hbm_bytes_per_launch" in pk:
            traffic = int(pk["hbm_bytes_per_launch"])
        with open(pmc_file) as f:
            wk = json.load(f).get(args.workload, {}).get("kernels", {})
        step_bytes = sum(v.get("hbm_bytes_per_dispatch", 0) for v in wk.values())
        if step_bytes > 0:
            # every kernel of one step, intermediates included (PMC, not algorithmic)
            pipeline_traffic = {"bytes_per_step": int(step_bytes),
                                "gbs": round(step_bytes / (ms_per_step / 1e3) / 1e9, 1),
                                "frac_of_peak": round(step_bytes / (ms_per_step / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
                                "source": f"profiles/{PROFILE_ROUND}_pmc.json: FETCH_SIZE x2 + WRITE_SIZE summed "
                                          "over the step's kernels, over this run's step time"}

    # parity spot-check after timing (not timed): GPU bytes vs the oracle
    out = np.empty((B, cap), np.uint8)
    ln = np.empty(B, np.int64)
    g_out, g_len = (ctx[0]["fec"], ctx[0]["flen"]) if fec_fused else (ctx[0]["out"], ctx[0]["len"])
    _amr.check(L.amr_memcpy_d2h(_amr.ptr(out), g_out, B * cap))
    _amr.check(L.amr_memcpy_d2h(_amr.ptr(ln), g_len, B * 8))

    # PCIe-inclusive rate (never `value`): the host API on the
    # same batch from pageable host memory -- H2D of the float32 samples, the
    # demod, D2H of the bytes -- one batch at a time; the first call is warmup
    host_path = None
    if rank == 0 and world == 1 and not fec_fused and not args.no_host_path:
        host_fn = L.amr_fsk_demod_host if fsk else L.amr_psk_demod_host
        h_out = np.empty((B, cap), np.uint8)
        h_len = np.empty(B, np.int64)
        h_sync = np.empty(B, np.int64)
        hts = []
        for _ in range(3):
            t1 = time.perf_counter()
            _amr.check(host_fn(plan.handle, _amr.ptr(x), _amr.DTYPE_F32, B, N, _amr.ptr(h_out), cap,
                               _amr.ptr(h_len), _amr.ptr(h_sync)))
            hts.append(time.perf_counter() - t1)
        ht = min(hts[1:])
        same = bool(np.array_equal(h_len, ln) and all(h_out[i, :ln[i]].tobytes() == out[i, :ln[i]].tobytes()
                                                      for i in range(B)))
        host_path = {"ms_per_batch": round(ht * 1e3, 2), "value": round(B * sym_per_stream / ht / 1e6, 3),
                     "unit": "Msym/s", "input_gb": round(x.nbytes / 1e9, 3),
                     "what": "amr_%s_demod_host from pageable host float32, one batch at a time (H2D + demod + D2H)"
                             % ("fsk" if fsk else "psk"),
                     "bytes_equal_device_path": same}

    result = None
    if rank == 0:
        threads = max(1, min(16, os.cpu_count() or 1))
        cpu = None
        parity = "skipped"
        if not args.no_cpu:
            if fsk:
                # ~16 ms of single-core work per stream (scipy's hilbert dominates):
                # 1024 streams ~ 15 s of CPU work spread over the host threads
                n_cpu = args.cpu_streams or 1024
                idx = np.linspace(0, B - 1, num=min(n_cpu, B)).astype(int)
                val, cdt, couts = cpu_baseline_fsk(x[idx], baud, args.mark, args.space, threads)
                how = "oracle.fsk_demodulate (C filtfilt + scipy.signal.hilbert + C decide), thread pool over streams"
            else:
                n_cpu = args.cpu_streams or B          # the whole batch: ~10 s of single-core work on the box
                idx = np.linspace(0, B - 1, num=min(n_cpu, B)).astype(int)
                val, cdt, couts = cpu_baseline(x[idx], baud, threads)
                how = "the C restatement oracle/amr_oracle.c, OpenMP over streams"
                if fec_fused:
                    from oracle import oracle
                    t1 = time.perf_counter()
                    couts = [oracle.fec_decode(c)[0] for c in couts]
                    cdt += time.perf_counter() - t1
                    val = len(idx) * sym_per_stream / cdt / 1e6
                    how += " + oracle.fec_decode"
            cpu = {"value": round(val, 3), "unit": "Msym/s", "cores": threads, "kind": "port",
                   "sample": f"{len(idx)} of the {B} benchmark streams ({N} samples each) through {how}, "
                             f"{cdt:.2f} s wall"}
            if not fsk and not fec_fused:
                # the same restatement on one core (1 core and all host cores)
                idx1 = idx[:64]
                v1, d1, _ = cpu_baseline(x[idx1], baud, 1)
                cpu["value_1core"] = round(v1, 3)
                cpu["sample_1core"] = f"{len(idx1)} streams, 1 thread, {d1:.2f} s wall"
            bad_idx = [int(i) for j, i in enumerate(idx) if out[i, :ln[i]].tobytes() != couts[j]]
            bad = len(bad_idx)
            if bad:
                log(f"[rank {rank}] streams differing from the oracle: {bad_idx[:32]}{' ...' if bad > 32 else ''}")
            parity = f"{len(idx) - bad}/{len(idx)} streams bit-exact vs oracle"
        if fsk:
            metric = "FSK demod Msymbols/s (batch), FSK9600 96kHz mark/space 12k/24k"
            workload = (f"FSK@{int(baud)} 96kHz tones {args.mark:g}/{args.space:g} Hz, batch {B} x {N} float32 "
                        "streams per GPU (BASELINE configs[3] at SURVEY §6's valid tones)")
        elif args.workload == "ofdm8":
            metric = "OFDM8 (qpsk_demodulate alias) demod Msymbols/s, global batch sharded + RCCL gather"
            workload = (f"OFDM8 = QPSK@{int(baud)} 96kHz (modem.py:375-376), {B_global} x {N} float32 streams "
                        f"sharded over {world} GPU(s) (BASELINE configs[4])")
        elif fec_fused:
            metric = "8PSK@19200 demod + fused FEC decode Msymbols/s, global batch sharded + RCCL gather"
            workload = (f"8PSK@{int(baud)} = QPSK path (modem.py:348) + ReedSolomonFEC.decode fused, {B_global} x "
                        f"{N} float32 streams sharded over {world} GPU(s) (BASELINE configs[5])")
        else:
            metric = "demod Msymbols/s (batch) + achieved HBM GB/s, QPSK@9600/96kHz, 1/2/4/8 GPU"
            workload = f"QPSK@{int(baud)} 96kHz, batch {B} x {N} float32 streams per GPU (BASELINE configs[1])"
        result = {
            "metric": metric,
            "value": round(value, 3), "unit": "Msym/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "strong" if strong else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
            "config": {"workload": workload, "global_batch": B_global, "samples_per_stream": N,
                       "symbols_per_stream": sym_per_stream, "parallelism": f"streams sharded over {world} GPU(s)",
                       "batches_in_flight": inflight},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic,
                         "traffic_source": f"profiles/{PROFILE_ROUND}_pmc.json (rocprofv3 FETCH_SIZE x2 + WRITE_SIZE, "
                                           "bytes/launch)",
                         "alg_bytes_per_launch": int(alg_bytes[dom]),
                         "fp64_valu": {"achieved_tops": round(fp64_achieved, 3), "peak_tops": FP64_PEAK_TOPS,
                                       "frac": round(fp64_achieved / FP64_PEAK_TOPS, 4)}},
            "pipeline_hbm_gbs": round(pipeline_bytes / (ms_per_step / 1e3) / 1e9, 2),
            "pipeline_hbm_traffic": pipeline_traffic,
            "pipeline_fp64": {"achieved_tops": round(fp64_pipeline, 3), "peak_tops": FP64_PEAK_TOPS,
                              "frac": round(fp64_pipeline / FP64_PEAK_TOPS, 4)},
            "kernel_ms": {k: round(v, 4) for k, v in kavg.items()},
            "kernel_ms_solo": {k: round(v, 4) for k, v in solo.items()},
            "cpu_baseline": cpu,
            "parity": parity,
            "host_path_pcie_inclusive": host_path,
        }
        # the reference's own numpy/scipy code is not on the GPU box; its rate as
        # measured in the build container is the north-star basis
        ref_py = {"qpsk9600": (0.292, 1.66), "ofdm8": (0.292, 1.66), "psk8fec": (0.310, 2.43),
                  "fsk9600": (0.180, 1.15)}[args.workload]
        result["vs_reference_python"] = {
            "reference_1core_msym_s": ref_py[0], "reference_8proc_msym_s": ref_py[1],
            "ratio_1core": round(value / ref_py[0], 1), "ratio_8proc": round(value / ref_py[1], 1),
            "source": "BASELINE.md §2: the reference's modem.py on numpy 2.2.6 / scipy 1.15.3, measured in the "
                      "build container (8 cores), not on the GPU box"}
        if not fsk:
            result["exact_path_streams"] = sum(pl.exact_streams() for pl in plans)
        if fec_fused:
            result["parity"] += " (FEC output)"
        print(json.dumps(result), flush=True)
    L.amr_free(d_x)
    for c in ctx:
        for key in ("out", "len", "sync", "fec", "flen", "ok", "gather", "gather_len"):
            if key in c:
                L.amr_free(c[key])
    if comm is not None:
        L.amr_comm_destroy(comm)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
