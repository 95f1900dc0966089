# round 3: known-answer loopbacks
set -o pipefail
T=${T:-r3o}
timeout -k 10 600 python -u -m pytest tests/test_gpu_loopback.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; exit $rc
