# strong-scaling shards on one GPU: each run is exactly one rank's work at N = 8192 / batch
set -o pipefail
T=${T:-s}
timeout -k 10 300 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
for wl in ofdm8 psk8fec; do
  for b in 1024 2048; do
    timeout -k 10 300 python -u bench.py --workload $wl --batch $b --no-host-path > gpurun_out/bench_${T}_${wl}_$b.json 2> gpurun_out/bench_${T}_${wl}_$b.err || exit 1
  done
done
