set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_gpu_slicer.py tests/test_plan_cache.py "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest3.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/gputest3.log
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --inflight 8 --no-host-path > gpurun_out/bench_lane8.json 2> gpurun_out/bench_lane8.err && \
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --inflight 4 --no-host-path --no-cpu > gpurun_out/bench_lane4.json 2> gpurun_out/bench_lane4.err && \
timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --inflight 12 --no-host-path --no-cpu > gpurun_out/bench_lane12.json 2> gpurun_out/bench_lane12.err
