# round 3: fixes of r3a's failures, the torch-free RCCL transport, the bench
# N > 1 path through multi.py, then the default bench line (FSK live columns)
set -o pipefail
T=${T:-r3b}
timeout -k 10 900 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_bench_comm.py \
  "tests/test_gpu_parity.py::test_batch_of_flagged_streams" \
  "tests/test_gpu_fsk.py::test_fsk_live_column_layout_chosen" \
  "tests/test_gpu_fsk.py::test_fsk_timing_hooks" "tests/test_gpu_parity.py::test_timing_hooks" tests/test_plan_cache.py \
  -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
