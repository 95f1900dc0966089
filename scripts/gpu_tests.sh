#!/bin/bash
# A subset of the -m gpu suite on the box, one process, its own time limit:
#   TESTS='tests/test_gpu_multi.py tests/test_gpu_comm.py' K='' T=multi bash scripts/gpu_tests.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
T=${T:-sub}
timeout -k 10 ${LIMIT:-900} python -u -m pytest ${TESTS:-tests} -m gpu -v -rP --timeout 400 --timeout-method thread ${K:+-k "$K"} > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; tail -3 gpurun_out/gputest_$T.log; exit $rc
