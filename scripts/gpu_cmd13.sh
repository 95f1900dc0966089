set -o pipefail
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" "tests/test_gpu_parity.py::test_async_host_entry_stream_of_batches" "tests/test_gpu_parity.py::test_every_golden_psk_case_bit_exact" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest13.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest13.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sub > gpurun_out/bench_zo1.json 2> gpurun_out/bench_zo1.err || exit 1
AMR_BP_ZO=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sub --no-cpu --no-host-path > gpurun_out/bench_zo0.json 2> gpurun_out/bench_zo0.err || exit 1
