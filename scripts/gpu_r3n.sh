# round 3: 10-s captures past 2^31 samples in both PSK layouts
set -o pipefail
T=${T:-r3n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 400 --timeout-method thread -k "ten_second" > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; exit $rc
