#!/bin/bash
# PMC passes (counters only, no trace domains) over a small fsk9600 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-pmc}
B=${B:-2048}
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = suffix, rest = counters
  local sfx=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d "$ROOT/gpurun_out/${TAG}_$sfx" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload fsk9600 --steps 1 --warmup 0 --no-cpu --batch $B ${BENCH_ARGS:-} > "$ROOT/gpurun_out/${TAG}_$sfx.log" 2>&1
}
run sq SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD && \
run fetch FETCH_SIZE && run write WRITE_SIZE
echo "pmc rc=$?"
