set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_slicer.py tests/test_plan_cache.py "tests/test_gpu_parity.py::test_async_host_entry_stream_of_batches" tests/test_gpu_frames.py -m gpu -v --timeout 280 --timeout-method thread > gpurun_out/gputest11.log 2>&1
echo "pytest rc=$?" >> gpurun_out/gputest11.log
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_d20b.json 2> gpurun_out/bench_d20b.err
