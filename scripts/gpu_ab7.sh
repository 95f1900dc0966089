# low-pass workgroups of one group (AMR_LP_WPB=2) vs two: same-box A/B (parity: the wpb2 lane variant covers the kernel)
set -o pipefail
for r in 1 2 3; do
  for v in 0 2; do
    for k in "64 3" "20 5"; do
      set -- $k
      AMR_LP_WPB=$v timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps $1 --warmup $2 > gpurun_out/ab7.json 2>/dev/null || exit 1
      python -c "import json;d=json.loads([l for l in open('gpurun_out/ab7.json') if l.startswith('{')][0]);print('lpwpb=$v K=$1', d['ms_per_step'], d['sustained']['ms_per_step'], d['kernel_ms_solo']['lowpass_fwd'])"
    done
  done
done
