set -o pipefail
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err
