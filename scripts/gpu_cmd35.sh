set -o pipefail
for cfg in "20 10" "20 16" "20 20" "10 10" "10 5" "32 16" "40 20"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu --steps $1 --warmup 5 --inflight $2 > gpurun_out/b35.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b35.json') if l.startswith('{')][0])
print('K=$1 P=$2', d['value'], d['ms_per_step'])"
done
