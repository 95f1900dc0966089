set -o pipefail
for P in 8 16 24 32; do
  timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu --steps 64 --warmup 3 --inflight $P > gpurun_out/bench_p$P.json 2> gpurun_out/bench_p$P.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/bench_p$P.json') if l.startswith('{')][0])
print('P=$P', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
