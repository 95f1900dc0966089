"""bench.py's N > 1 path on one GPU (`--force-comm`: torch.distributed.run
with one rank -- the launcher only; bootstrap, barriers, max over ranks and
gathers are multi.py's RcclTransport -- a one-rank RCCL communicator, the
all-gather after every launch, the gather check), small sizes: the headline layout, a
strong-scaling workload with two global batches per launch (`--coalesce`),
and the FSK plans' gather (amr_fsk_allgather).
The 8-GPU run is the driver's; this keeps the code it runs exercised."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("extra", [["--batch", "256"], ["--workload", "ofdm8", "--batch", "512", "--coalesce", "2"],
                                   ["--workload", "fsk9600", "--batch", "256"]])
def test_force_comm_gather_check(extra):
    # a fresh box's first `import torch` pages the image in (1-2 minutes); do
    # it in a throwaway process so the bench run below starts warm and the
    # pytest process itself never loads torch
    subprocess.run([sys.executable, "-c", "import torch"], timeout=400, check=True)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(ROOT, "bench.py"),
           "--force-comm", "--steps", "4", "--warmup", "1", "--no-sub", "--no-host-path", "--no-latency",
           "--no-dropin", "--sustain-seconds", "0", "--cpu-seconds", "0", "--samples", "24000", *extra]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert line, r.stdout[-2000:] + r.stderr[-2000:]
    d = json.loads(line[-1])
    assert d["gather_check"].startswith("ok"), d["gather_check"]
    assert d["latency_ms_per_global_batch"] and d["latency_ms_per_global_batch"] > 0
    assert "bit-exact" in d["parity"] and d["parity"].split("/")[0] == d["parity"].split("/")[1].split()[0], d["parity"]
