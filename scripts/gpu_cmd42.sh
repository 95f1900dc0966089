set -o pipefail
timeout -k 10 300 python -u bench.py --no-sub --no-host-path > gpurun_out/b42.json 2> gpurun_out/b42.err || exit 1
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b42.json') if l.startswith('{')][0])
print('lat', d['value'], d['ms_per_step'], d['latency_ms_one_batch'], d['latency_layout'], d['latency_note'], d['parity'])"
