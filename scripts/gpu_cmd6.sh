set -o pipefail
timeout -k 10 300 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 280 --timeout-method thread > gpurun_out/gputest6.log 2>&1 || { echo "pytest failed" >> gpurun_out/gputest6.log; exit 1; }
for wpb in 1 2 4; do
  AMR_LANE_WPB=$wpb timeout -k 10 150 python -u bench.py --steps 32 --no-sub --no-host-path --no-cpu > gpurun_out/bench_wpb$wpb.json 2> gpurun_out/bench_wpb$wpb.err || exit 1
done
