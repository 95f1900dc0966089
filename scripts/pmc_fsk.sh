#!/bin/bash
# PMC passes (counters only, no trace domains) over a small fsk9600 bench:
# two SQ passes (8 SQ counters each), FETCH_SIZE, WRITE_SIZE -- each its own
# run under its own time limit.  scripts/pmc_show.py folds them per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-pmc}
B=${B:-2048}
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = suffix, rest = counters
  local sfx=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d "$ROOT/gpurun_out/${TAG}_$sfx" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload fsk9600 --steps 1 --warmup 0 --no-cpu --batch $B ${BENCH_ARGS:-} > "$ROOT/gpurun_out/${TAG}_$sfx.log" 2>&1
}
run sq SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD && \
run sq2 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES && \
run fetch FETCH_SIZE && run write WRITE_SIZE
echo "pmc rc=$?"
