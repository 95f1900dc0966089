#!/bin/bash
# One rocprofv3 --pmc pass of SQ counters over a short bench run (no trace
# domains in the same run -- pool rule).  Usage (GPU box):
#   COUNTERS="SQ_WAVE_CYCLES SQ_WAIT_ANY ..." OUT=gpurun_out/pmc_x bash scripts/pmc_sq.sh [bench args]
# PROG / BASEARGS select another driver (e.g. PROG=tools/bench_tx.py BASEARGS="--steps 1 --warmup 0").
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
OUT=${OUT:-gpurun_out/pmc_sq}; case "$OUT" in /*) ;; *) OUT=$ROOT/$OUT;; esac
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc ${COUNTERS} -d "$OUT" -o run --output-format csv -- python3 "$ROOT/${PROG:-bench.py}" ${BASEARGS:---steps 1 --warmup 0 --no-cpu} "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "pmc rc=$rc"; exit $rc
