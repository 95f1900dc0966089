set -o pipefail
timeout -k 10 900 python -u bench.py > gpurun_out/bench_default2.json 2> gpurun_out/bench_default2.err || exit 1
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 --no-host-path > gpurun_out/bench_k20.json 2> gpurun_out/bench_k20.err || exit 1
