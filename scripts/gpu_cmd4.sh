set -o pipefail
for cfg in "8 8" "16 16" "32 16" "16 24"; do
  set -- $cfg
  timeout -k 10 150 python -u bench.py --steps 32 --warmup 3 --hw-queues $1 --inflight $2 --no-host-path --no-cpu > gpurun_out/bench_q$1_f$2.json 2> gpurun_out/bench_q$1_f$2.err || exit 1
done
