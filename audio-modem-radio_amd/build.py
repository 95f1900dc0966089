"""Build libamr.so (gfx950) in-tree with hipcc; no JIT cache, no torch.

    python audio-modem-radio_amd/build.py [--force]

Compile flags that matter for parity:
  -ffp-contract=off   the reference's arithmetic (scipy lfilter, numpy) has no
                      contracted multiply-adds; every fma in the kernels is an
                      explicit one that numpy itself performs.
  -fno-fast-math      IEEE zeros/NaN/inf semantics are part of the contract.
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(os.path.dirname(HERE), "include")
LIB = os.path.join(HERE, "libamr.so")
SOURCES = ["psk_kernels.hip", "util_kernels.hip", "fft_kernels.hip", "fsk_kernels.hip", "frame_kernels.hip", "tx_kernels.hip",
           "api.cpp", "tx_api.cpp",
           "fsk_api.cpp"]
HEADERS = ["amr_internal.h", "fft.h", "api_common.h", os.path.join(INCLUDE, "amr.h")]
ARCH = os.environ.get("AMR_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"--offload-arch={ARCH}",
          "-I", CSRC, "-I", INCLUDE, "-Wall", "-Wno-unused-function"]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(force: bool = False, verbose: bool = False) -> str:
    objdir = os.path.join(HERE, "build")
    os.makedirs(objdir, exist_ok=True)
    hdrs = [h if os.path.isabs(h) else os.path.join(CSRC, h) for h in HEADERS]
    objs = []
    for src in SOURCES:
        sp = os.path.join(CSRC, src)
        obj = os.path.join(objdir, src + ".o")
        objs.append(obj)
        if force or _stale(obj, [sp, *hdrs, __file__]):
            cmd = [HIPCC, *CFLAGS, "-c", sp, "-o", obj]
            if verbose:
                print(" ".join(cmd))
            subprocess.run(cmd, check=True)
    if force or _stale(LIB, objs):
        cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs,
               "-L/opt/rocm/lib", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"]
        if verbose:
            print(" ".join(cmd))
        subprocess.run(cmd, check=True)
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
