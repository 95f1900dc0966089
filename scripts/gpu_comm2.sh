set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_abi.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/comm_test.log 2>&1 || exit 1
bash scripts/gpu_comm.sh
