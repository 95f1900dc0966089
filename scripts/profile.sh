#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box):
#   1. --kernel-trace --stats          per-kernel durations  -> gpurun_out/prof_<tag>/trace
#   2. --pmc FETCH_SIZE (own pass)     HBM read KB per dispatch
#   3. --pmc WRITE_SIZE (own pass)     HBM write KB per dispatch
# Counters never share a run with trace domains (pool rule).  Then
# scripts/prof_summary.py folds them into profiles/<tag>_*.{csv,json,md}.
set -u
TAG=${TAG:-r02}
WORKLOAD=${WORKLOAD:-qpsk9600}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/prof_${TAG}_$WORKLOAD
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
ARGS="--workload $WORKLOAD --steps ${STEPS:-64} --warmup 3 --no-cpu --no-host-path --no-sub --no-latency --no-dropin --sustain-seconds 0 ${BENCH_ARGS:-}"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace.err"
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/fetch_bench.json" 2> "$OUT/fetch.err"
rc=$?; echo "fetch rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 "$ROOT/bench.py" $ARGS > "$OUT/write_bench.json" 2> "$OUT/write.err"
rc=$?; echo "write rc=$rc"; [ $rc -ne 0 ] && exit $rc
cd "$ROOT" && python3 scripts/prof_summary.py "$OUT" "$TAG" "$WORKLOAD"
