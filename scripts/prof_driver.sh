#!/bin/bash
# rocprofv3 --kernel-trace --stats of the driver's exact bench command (the
# contract's "same command"), folded like the per-workload profiles.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG:-r03}_driver
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"; exit $rc
