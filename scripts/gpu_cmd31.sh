set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_slicer.py "tests/test_gpu_parity.py::test_every_golden_psk_case_bit_exact" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest31.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest31.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do for cfg in "AMR_SLICE_V1=1" "AMR_SLICE_WAVES=4" "AMR_SLICE_WAVES=8" "AMR_SLICE_WAVES=16"; do
  env $cfg timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu > gpurun_out/b31.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b31.json') if l.startswith('{')][0])
print('$cfg', d['value'], d['ms_per_step'], d['kernel_ms']['sync_pack'], d['kernel_ms_solo']['sync_pack'])"
done; done
