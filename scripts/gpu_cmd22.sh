set -o pipefail
for cfg in "ofdm8 8192" "ofdm8 1024" "psk8fec 8192" "psk8fec 1024"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --workload $1 --batch $2 --no-cpu --no-host-path > gpurun_out/b22_$1_$2.json 2> gpurun_out/b22_$1_$2.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b22_$1_$2.json') if l.startswith('{')][0])
print('$1 B=$2', d['value'], d['ms_per_step'], d['config']['batches_in_flight'], d['config']['kernel_layout'], d.get('latency_ms_one_batch'), d['kernel_ms_solo'])"
done
