set -o pipefail
for cfg in "0 64" "30 64" "30 128" "0 128"; do
  set -- $cfg
  AMR_BENCH_STAGGER_MS=$1 timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu --steps $2 --warmup 3 --inflight 16 > gpurun_out/b21_$1_$2.json 2> gpurun_out/b21_$1_$2.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b21_$1_$2.json') if l.startswith('{')][0])
print('stagger $1 K=$2', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
