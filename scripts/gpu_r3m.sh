# round 3: the product's sharded path at world 2 / 3 on one GPU (StoreTransport)
set -o pipefail
T=${T:-r3m}
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_comm.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; exit $rc
