# in-flight depth: timed region of whole rounds + 2 s sustained, per P
set -o pipefail
for cfg in ${CFGS:-"64 16" "80 20" "72 24" "60 12"}; do
  set -- $cfg
  timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps $1 --inflight $2 > gpurun_out/pscan_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.loads([l for l in open('gpurun_out/pscan_$2.json') if l.startswith('{')][0]);print('P=$2 K=$1', d['ms_per_step'], d['sustained']['ms_per_step'])"
done
