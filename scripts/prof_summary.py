#!/usr/bin/env python3
"""Fold rocprofv3 CSVs (scripts/profile.sh) into profiles/<tag>_*.

    python scripts/prof_summary.py gpurun_out/prof_<tag>_<workload> <tag> <workload>

Outputs:
  profiles/<tag>_<workload>_kernel_stats.csv  rocprofv3 --stats summary, verbatim
  profiles/<tag>_pmc.json    [workload]["kernels"][kernel]: avg duration (trace
                             pass), HBM bytes per dispatch from FETCH_SIZE (x2,
                             the gfx950 wide-read correction of
                             MI355X_MICROARCH.md §HBM) + WRITE_SIZE (KB);
                             [workload]["slots"][slot]: the same summed over the
                             kernels of one bench.py timing slot, per step
  profiles/<tag>_summary.md  the same as tables, one section per workload
"""
import csv
import glob
import json
import os
import shutil
import sys


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def find(d, pat):
    m = glob.glob(os.path.join(d, "**", pat), recursive=True)
    return m[0] if m else None


KERNELS = ["k_bp_lane2", "k_lp_lane2", "k_bp_lane", "k_lp_lane", "k_fsk_bandpass", "k_fsk_decide", "k_bandpass_row", "k_bandpass_g8", "k_bandpass_quad", "k_bandpass", "k_lowpass_fwd_q",
           "k_lowpass_bwd_q", "k_lowpass_fwd", "k_lowpass_bwd", "k_lowpass_exact", "k_slice",
           "k_sync_pack", "k_fec_decode",
           "k_fft_cols_live", "k_fft_mid_live", "k_fft_rows_live",
           "k_fft_cols", "k_fft_mid", "k_fft_rows", "k_bs_pre", "k_bs_post"]
# bench.py timing slot -> the kernels it brackets (one launch each per step)
SLOTS = {
    "qpsk9600": {"bandpass": ["k_bp_lane2", "k_bp_lane2_fixup", "k_bp_lane", "k_bandpass_row", "k_bandpass_g8", "k_bandpass_quad", "k_bandpass"],
                 "lowpass_fwd": ["k_lp_lane2", "k_lp_lane", "k_lowpass_fwd_q", "k_lowpass_fwd"], "lowpass_bwd": ["k_lowpass_bwd_q", "k_lowpass_bwd"],
                 "lowpass_exact": ["k_lowpass_exact"], "sync_pack": ["k_slice", "k_sync_pack"], "fec": ["k_fec_decode"]},
    "ofdm8": None, "psk8fec": None,
    "fsk9600": {"bandpass": ["k_fsk_bandpass"],
                "hilbert": ["k_fft_cols_live", "k_fft_mid_live", "k_fft_rows_live", "k_fft_cols", "k_fft_mid", "k_fft_rows"],
                "decide": ["k_fsk_decide", "k_sync_pack"]},
}


SLOTS["ofdm8"] = SLOTS["psk8fec"] = SLOTS["qpsk9600"]


def short(name):
    n = name.replace("amr::", "").replace("(amr::FftEpiMode)", "")
    if "k_bp_lane2<" in n:
        args = [t.strip() for t in n.split("k_bp_lane2<", 1)[1].split(">", 1)[0].split(",")]
        if len(args) >= 4 and args[3] == "true":
            return "k_bp_lane2_fixup"               # the zero-tap fallback launch (early exit)
    for k in KERNELS:
        if k in n:
            return k
    return name[:60]


def main():
    out, tag = sys.argv[1], sys.argv[2]
    workload = sys.argv[3] if len(sys.argv) > 3 else "qpsk9600"
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_{workload}_kernel_stats.csv"))
    res = {}
    for r in rows(stats):     # template instances of one kernel fold into one row
        d = res.setdefault(short(r["Name"]), {"calls": 0, "total_ns": 0.0})
        d["calls"] += int(r["Calls"])
        d["total_ns"] += float(r["TotalDurationNs"])
        d["avg_ns"] = d["total_ns"] / d["calls"]
    # the bench's timed steps are the last `steps` dispatches of each kernel
    # (warmup dispatches run one batch at a time, the timed ones in flight)
    trace = find(os.path.join(out, "trace"), "*kernel_trace.csv")
    bj = os.path.join(out, "trace_bench.json")
    steps = None
    warmup = 1
    cfg = {}
    if os.path.exists(bj):
        with open(bj) as f:
            for line in f:
                if line.startswith("{"):
                    steps = json.loads(line).get("steps")
                    warmup = json.loads(line).get("warmup", 1)
                    cfg = json.loads(line).get("config", {})
    launches = -(-steps // cfg.get("steps_per_launch", 1)) if steps else None
    if trace and steps:
        per = {}
        for r in rows(trace):
            per.setdefault(short(r["Kernel_Name"]), []).append(
                (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
        for k, v in per.items():
            v.sort()
            tail = [d for _, d in v[-launches:]]
            res.setdefault(k, {})["avg_ns_timed_steps"] = sum(tail) / len(tail)
            # the warmup launches run one at a time (bench.py); the first is cold
            head = [d for _, d in v[1:warmup]] if warmup > 1 else [d for _, d in v[:1]]
            if head:
                res[k]["avg_ns_solo"] = sum(head) / len(head)
    bench = {}
    if os.path.exists(bj):
        with open(bj) as f:
            for line in f:
                if line.startswith("{"):
                    bench = json.loads(line)
    for which, counter, scale in (("fetch", "FETCH_SIZE", 2.0), ("write", "WRITE_SIZE", 1.0)):
        f = find(os.path.join(out, which), "*counter_collection.csv")
        if not f:
            continue
        acc = {}
        for r in rows(f):
            if r.get("Counter_Name") != counter:
                continue
            k = short(r["Kernel_Name"])
            acc.setdefault(k, []).append(float(r["Counter_Value"]) * 1024.0 * scale)
        for k, v in acc.items():
            res.setdefault(k, {})[f"{which}_bytes_per_dispatch"] = sum(v) / len(v)
    for k, v in res.items():
        if "fetch_bytes_per_dispatch" in v or "write_bytes_per_dispatch" in v:
            v["hbm_bytes_per_dispatch"] = v.get("fetch_bytes_per_dispatch", 0) + v.get("write_bytes_per_dispatch", 0)
    slots = {}
    for slot, ks in SLOTS.get(workload, {}).items():
        got = [res[k] for k in ks if k in res]
        if not got:
            continue
        d = {"kernels": [k for k in ks if k in res], "avg_ns": sum(g.get("avg_ns", 0) for g in got)}
        for key in ("avg_ns_timed_steps", "avg_ns_solo"):
            if all(key in g for g in got):
                d[key] = sum(g[key] for g in got)
        for key in ("fetch_bytes_per_dispatch", "write_bytes_per_dispatch", "hbm_bytes_per_dispatch"):
            if all(key in g for g in got):
                d[key.replace("_per_dispatch", "_per_launch")] = sum(g[key] for g in got)
        slots[slot] = d
    pmc_path = os.path.join(prof, f"{tag}_pmc.json")
    allres = {}
    if os.path.exists(pmc_path):
        with open(pmc_path) as f:
            allres = json.load(f)
        if "kernels" in allres:       # older single-workload layout
            allres = {}
    allres["source"] = "rocprofv3 kernel-trace --stats + separate --pmc FETCH_SIZE / WRITE_SIZE passes"
    allres["fetch_correction"] = "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads)"
    rl = bench.get("roofline", {})
    allres[workload] = {"kernels": res, "slots": slots, "inflight": cfg.get("batches_in_flight"),
                        "layout": cfg.get("kernel_layout"), "steps": steps,
                        "bench": {"dominant_slot": rl.get("kernel"), "alg_bytes_per_launch": rl.get("alg_bytes_per_launch"),
                                  "kernel_ms_hip_events": rl.get("kernel_ms_used"),
                                  "kernel_ms_hip_events_inflight": (rl.get("inflight") or {}).get("kernel_ms"),
                                  "ms_per_step": bench.get("ms_per_step"),
                                  "streams_per_step": cfg.get("global_batch"),
                                  "streams_per_launch": cfg.get("streams_per_launch"),
                                  "frac": rl.get("frac"), "frac_throughput": rl.get("frac_throughput"),
                                  "value": bench.get("value"), "unit": bench.get("unit")}}
    with open(pmc_path, "w") as f:
        json.dump(allres, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary ({tag})\n")
        for wl, r in allres.items():
            if not isinstance(r, dict) or "kernels" not in r:
                continue
            f.write(f"\n## {wl}\n\n| kernel | calls | avg ms (all) | avg ms (solo warmup launches) | "
                    "avg ms (timed launches, in flight) | "
                    "HBM read MB/disp (x2 corr.) | HBM write MB/disp |\n|---|---|---|---|---|---|---|\n")
            for k, v in sorted(r["kernels"].items(), key=lambda kv: -kv[1].get("avg_ns", 0)):
                ts = v.get("avg_ns_timed_steps")
                so = v.get("avg_ns_solo")
                f.write(f"| {k} | {v.get('calls', '')} | {v.get('avg_ns', 0) / 1e6:.3f} | "
                        f"{(so / 1e6) if so else float('nan'):.3f} | "
                        f"{(ts / 1e6) if ts else float('nan'):.3f} | "
                        f"{v.get('fetch_bytes_per_dispatch', 0) / 1e6:.1f} | "
                        f"{v.get('write_bytes_per_dispatch', 0) / 1e6:.1f} |\n")
            b = r.get("bench", {})
            sl = r.get("slots", {}).get(b.get("dominant_slot") or "", {})
            if b.get("alg_bytes_per_launch") and sl.get("avg_ns_solo"):
                ns = sl["avg_ns_solo"]
                ach = b["alg_bytes_per_launch"] / ns
                f.write(f"\nRoofline, reproduced from this profile ({r.get('steps')} timed steps, "
                        f"{r.get('inflight')} launches in flight, layout {r.get('layout')}): dominant slot "
                        f"`{b['dominant_slot']}` = {' + '.join(sl['kernels'])}; algorithmic bytes per launch "
                        f"{b['alg_bytes_per_launch']:,} (SURVEY 8(d)) / rocprofv3 average of the solo warmup "
                        f"launches {ns / 1e6:.3f} ms = {ach:.2f} GB/s = {ach / 8000:.5f} of 8000 GB/s.  The bench's "
                        f"HIP events over the same launches: {b.get('kernel_ms_hip_events')} ms.  In flight "
                        f"(timed launches): rocprofv3 {sl.get('avg_ns_timed_steps', 0) / 1e6:.3f} ms, HIP events "
                        f"{b.get('kernel_ms_hip_events_inflight')} ms; step {b.get('ms_per_step')} ms, "
                        f"{b.get('value')} {b.get('unit')}.\n")
                spl, sps_ = b.get("streams_per_launch"), b.get("streams_per_step")
                if b.get("ms_per_step") and spl and sps_:
                    step_bytes = b["alg_bytes_per_launch"] / spl * sps_
                    f.write(f"Throughput-consistent fraction (`frac_throughput`): the algorithmic bytes of a step "
                            f"({step_bytes:,.0f} B) / the step time {b['ms_per_step']} ms = "
                            f"{step_bytes / b['ms_per_step'] / 1e6:.2f} GB/s = "
                            f"{step_bytes / b['ms_per_step'] / 1e6 / 8000:.5f} of 8000 GB/s (the bench line: "
                            f"frac {b.get('frac')}, frac_throughput {b.get('frac_throughput')}); the solo duration "
                            f"exceeds the step because {r.get('inflight')} launches overlap in the timed region.\n")
                if sl.get("hbm_bytes_per_launch"):
                    f.write(f"HBM traffic of that slot per launch (FETCH_SIZE x2 + WRITE_SIZE): "
                            f"{sl['hbm_bytes_per_launch'] / 1e6:.1f} MB = "
                            f"{sl['hbm_bytes_per_launch'] / b['alg_bytes_per_launch']:.2f} x the algorithmic bytes.\n")
            tot = sum(v.get("hbm_bytes_per_dispatch", 0) for k, v in r["kernels"].items() if "synth" not in k)
            if tot:
                f.write(f"The step's kernels (one dispatch each; input synthesis excluded), HBM bytes per step: "
                        f"{tot / 1e9:.2f} GB.\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
