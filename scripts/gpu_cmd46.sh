set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slicer.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest46.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest46.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for cfg in "AMR_FUSED_SLICE=1" "AMR_FUSED_SLICE=0"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-latency > gpurun_out/b46.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b46.json') if l.startswith('{')][0])
print('$cfg', d['value'], d['ms_per_step'], d['kernel_ms']['lowpass_fwd'], d['kernel_ms']['sync_pack'], d['parity'])"
done; done
