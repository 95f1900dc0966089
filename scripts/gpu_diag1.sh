# diagnostic only (wrong for flagged streams): what the band-pass fix-up launch costs in flight
set -o pipefail
for r in 1 2; do
  for v in 0 1; do
    for k in "qpsk9600 64 3" "qpsk9600 20 5" "ofdm8 64 3"; do
      set -- $k
      AMR_DIAG_NO_FIXUP=$v timeout -k 10 200 python bench.py --workload $1 --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps $2 --warmup $3 > gpurun_out/diag1.json 2>/dev/null || exit 1
      python -c "import json;d=json.loads([l for l in open('gpurun_out/diag1.json') if l.startswith('{')][0]);print('nofix=$v $1 K=$2', d['ms_per_step'], (d.get('sustained') or {}).get('ms_per_step'))"
    done
  done
done
