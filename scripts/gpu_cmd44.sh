set -o pipefail
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest44.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gputest44.log
