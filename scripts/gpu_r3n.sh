# round 3: batches past 2^31 samples: 10-s captures in both PSK layouts, 22400 FSK streams
set -o pipefail
T=${T:-r3n}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread -k "ten_second or past_2g" > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; exit $rc
