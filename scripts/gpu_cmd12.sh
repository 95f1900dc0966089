set -o pipefail
HSA_ENABLE_SDMA=0 timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sub --no-cpu > gpurun_out/bench_nosdma.json 2> gpurun_out/bench_nosdma.err || exit 1
