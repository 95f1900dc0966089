set -o pipefail
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest10.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gputest10.log
AMR_LP_SPLIT=1 timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 280 --timeout-method thread >> gpurun_out/gputest10.log 2>&1
echo "lp-split pytest rc=$?" >> gpurun_out/gputest10.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_d20.json 2> gpurun_out/bench_d20.err
