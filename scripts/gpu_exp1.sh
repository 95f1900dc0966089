# A/B: FSK in-flight depth; the headline at the driver's K = 20
set -o pipefail
for p in 2 3 4; do
  timeout -k 10 300 python -u bench.py --workload fsk9600 --inflight $p --no-host-path --no-cpu --no-latency > gpurun_out/exp1_fsk_p$p.json 2> gpurun_out/exp1_fsk_p$p.err || exit 1
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-sub --no-host-path --no-cpu > gpurun_out/exp1_k20.json 2> gpurun_out/exp1_k20.err || exit 1
