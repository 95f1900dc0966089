# split band-pass forward (AMR_BP_PREFWD=1): lane parity, then same-box A/B at K = 64 and K = 20
set -o pipefail
timeout -k 10 500 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab3_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab3_parity.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2 3; do
  for v in 0 1; do
    for k in "64 3" "20 5"; do
      set -- $k
      AMR_BP_PREFWD=$v timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps $1 --warmup $2 > gpurun_out/ab3_$v.json 2>/dev/null || exit 1
      python -c "import json;d=json.loads([l for l in open('gpurun_out/ab3_$v.json') if l.startswith('{')][0]);print('prefwd=$v K=$1', d['ms_per_step'], d['sustained']['ms_per_step'], d['kernel_ms'])"
    done
  done
done
