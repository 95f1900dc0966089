#!/usr/bin/env python3
"""Fold rocprofv3 CSVs (scripts/profile.sh) into profiles/<tag>_*.

Outputs:
  profiles/<tag>_kernel_stats.csv   rocprofv3 --stats summary, verbatim
  profiles/<tag>_pmc.json           per kernel: avg duration (trace pass), HBM
                                    bytes per dispatch from FETCH_SIZE (x2, the
                                    gfx950 wide-read correction of
                                    MI355X_MICROARCH.md §HBM) + WRITE_SIZE, both KB
  profiles/<tag>_summary.md         the same as a table
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


def short(name):
    for k in ("k_bandpass", "k_lowpass_fwd", "k_lowpass_bwd", "k_lowpass_exact", "k_slice", "k_sync_pack",
              "k_fec_decode", "k_fsk"):
        if k in name:
            return k
    return name[:60]


def main():
    out, tag = sys.argv[1], sys.argv[2]
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    prof = os.path.join(repo, "profiles")
    os.makedirs(prof, exist_ok=True)
    stats = find(os.path.join(out, "trace"), "*kernel_stats.csv")
    shutil.copy(stats, os.path.join(prof, f"{tag}_kernel_stats.csv"))
    res = {}
    for r in rows(stats):
        res.setdefault(short(r["Name"]), {})["avg_ns"] = float(r["AverageNs"])
        res[short(r["Name"])]["calls"] = int(r["Calls"])
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
    with open(os.path.join(prof, f"{tag}_pmc.json"), "w") as f:
        json.dump({"source": "rocprofv3 kernel-trace --stats + separate --pmc FETCH_SIZE / WRITE_SIZE passes",
                   "fetch_correction": "FETCH_SIZE x2 (gfx950 reports half of wide coalesced reads)",
                   "kernels": res}, f, indent=1)
    with open(os.path.join(prof, f"{tag}_summary.md"), "w") as f:
        f.write(f"# rocprofv3 summary ({tag})\n\n| kernel | calls | avg ms | HBM read MB/disp (x2 corr.) | HBM write MB/disp |\n|---|---|---|---|---|\n")
        for k, v in sorted(res.items(), key=lambda kv: -kv[1].get("avg_ns", 0)):
            f.write(f"| {k} | {v.get('calls', '')} | {v.get('avg_ns', 0) / 1e6:.3f} | "
                    f"{v.get('fetch_bytes_per_dispatch', 0) / 1e6:.1f} | {v.get('write_bytes_per_dispatch', 0) / 1e6:.1f} |\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
