"""Build libamr.so (gfx950) in-tree with hipcc; no JIT cache, no torch.

    python audio-modem-radio_amd/build.py [--force]

Compile flags that matter for parity:
  -ffp-contract=off   the reference's arithmetic (scipy lfilter, numpy) has no
                      contracted multiply-adds; every fma in the kernels is an
                      explicit one that numpy itself performs.
  -fno-fast-math      IEEE zeros/NaN/inf semantics are part of the contract.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libamr.so")
SOURCES = ["psk_kernels.hip", "psk_lane_kernels.hip", "psk_split_kernels.hip", "util_kernels.hip", "fft_kernels.hip", "fsk_kernels.hip", "fsk_exact_kernels.hip", "pocketfft_kernels.hip", "frame_kernels.hip", "tx_kernels.hip",
           "api.cpp", "tx_api.cpp",
           "fsk_api.cpp", "pocketfft_plan.cpp"]
HEADERS = ["amr_internal.h", "psk_common.h", "fft.h", "api_common.h", "fsk_exact.h", "pocketfft.h", "pocketfft_dev.h",
           "iir_design.h", "split_chain.h", "odd_ext.h", "split_strict.h", os.path.join(INCLUDE, "amr.h")]
ARCH = os.environ.get("AMR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"--offload-arch={ARCH}",
          "-I", CSRC, "-I", INCLUDE, "-Wall", "-Wno-unused-function"]


def _digest(paths, extra: str = "") -> str:
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode() + b"\0" + f.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def _headers():
    return [x if os.path.isabs(x) else os.path.join(CSRC, x) for x in HEADERS]


def source_hash() -> str:
    """sha256 prefix over every source, header, this script and the flags:
    the build id libamr.so reports (amr_build_id), which ties a loaded
    library to the sources of the tree it runs in."""
    # the flags without the tree's absolute include paths: the id depends on
    # what is compiled, not on where the tree sits (the GPU box runs a copy)
    flags = [f for f in CFLAGS if f not in (CSRC, INCLUDE)]
    return _digest([os.path.join(CSRC, s) for s in SOURCES] + _headers() + [os.path.abspath(__file__)],
                   " ".join(flags))


def build(force: bool = False, verbose: bool = False) -> str:
    """Rebuild what changed BY CONTENT (each object records the digest of its
    source + headers + flags next to it), never by modification time alone."""
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    hdrs = _headers()
    bid = source_hash()
    objs = []
    jobs = []
    relink = force or not os.path.exists(LIB)
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        defs = [f'-DAMR_BUILD_ID="{bid}"'] if src == "api.cpp" else []
        dig = _digest([sp, *hdrs, os.path.abspath(__file__)], " ".join(CFLAGS + defs))
        stamp = obj + ".sha"
        have = open(stamp).read().strip() if os.path.exists(stamp) and os.path.exists(obj) else ""
        if force or have != dig:
            jobs.append(([HIPCC, *CFLAGS, *defs, "-c", sp, "-o", obj], stamp, dig))

    def compile_one(job):
        cmd, stamp, dig = job
        if verbose:
            print(" ".join(cmd), flush=True)
        subprocess.run(cmd, check=True)
        with open(stamp, "w") as f:
            f.write(dig + "\n")

    if jobs:
        from concurrent.futures import ThreadPoolExecutor
        workers = max(1, min(len(jobs), int(os.environ.get("MAX_JOBS", "0")) or min(8, os.cpu_count() or 1)))
        with ThreadPoolExecutor(workers) as ex:
            list(ex.map(compile_one, jobs))
        relink = True
    if relink:
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
