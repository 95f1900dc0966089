set -o pipefail
for r in 1 2; do for cfg in "64 --host-wait" "64 " "32 --host-wait" "32 " "20 "; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu --steps $1 $2 > gpurun_out/b40.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b40.json') if l.startswith('{')][0])
print('K=$1 $2', d['value'], d['ms_per_step'], d['kernel_ms']['bandpass'], d['kernel_ms']['lowpass_fwd'])"
done; done
