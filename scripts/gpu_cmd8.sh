set -o pipefail
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 280 --timeout-method thread > gpurun_out/gputest8.log 2>&1 || { echo "pytest failed" >> gpurun_out/gputest8.log; exit 1; }
AMR_LANE_WPB=4 AMR_LANE_WPB=4 timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 280 --timeout-method thread >> gpurun_out/gputest8.log 2>&1 || { echo "pytest wpb4 failed" >> gpurun_out/gputest8.log; exit 1; }
for cfg in "1 20" "4 20" "1 32" "4 32"; do
  set -- $cfg
  AMR_LANE_WPB=$1 timeout -k 10 150 python -u bench.py --steps $2 --no-sub --no-host-path --no-cpu > gpurun_out/bench_s_w$1_k$2.json 2> gpurun_out/bench_s_w$1_k$2.err || exit 1
done
