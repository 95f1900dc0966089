#!/bin/bash
# FSK GPU check: FSK/FFT parity tests, then a rocprofv3 kernel trace of the fsk9600 bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
TAG=${TAG:-fsk}
timeout -k 10 600 python -m pytest tests/test_gpu_fsk.py -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/gpu_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/gpu_$TAG.log
case $rc in 124|134|137|139) exit $rc;; esac
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/prof_$TAG" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload fsk9600 --steps 3 --warmup 1 --no-cpu ${BENCH_ARGS:-} > "$ROOT/gpurun_out/prof_$TAG.json" 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 "$ROOT/gpurun_out/prof_$TAG.json" | cut -c1-600
