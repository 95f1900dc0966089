# the headline with the drop-in timing
set -o pipefail
timeout -k 10 300 python -u bench.py --no-sub > gpurun_out/exp2.json 2> gpurun_out/exp2.err || exit 1
