#!/usr/bin/env python3
"""Kernel time of the device pocketfft envelope (the FSK exact path's E2) by
half, for the rocprofv3 kernel trace: AMR_PF_STAGE=0 the whole |hilbert|,
1 the real forward transform alone, 2 the complex half alone; AMR_PF_FUSE=0
the pass-by-pass executor.  GPU box:
  rocprofv3 --kernel-trace --stats -- python3 tools/pf_stage_timing.py [rows] [n]"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "audio-modem-radio_amd"))
import _amr  # noqa: E402

rows = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
n = int(sys.argv[2]) if len(sys.argv) > 2 else 96000
x = np.random.default_rng(1).standard_normal((rows, n))
for rep in range(3):
    t = time.perf_counter()
    _amr.hilbert_env_exact(x)
    print(f"rep {rep}: {1e3 * (time.perf_counter() - t):.1f} ms host entry "
          f"(stage {os.environ.get('AMR_PF_STAGE', '0')}, fuse {os.environ.get('AMR_PF_FUSE', '1')})", flush=True)
