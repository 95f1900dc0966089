set -o pipefail
timeout -k 10 900 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest50.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest50.log; [ $rc -ne 0 ] && exit $rc
bash scripts/gpu_cmd22.sh
timeout -k 10 300 python -u bench.py --no-sub --no-host-path > gpurun_out/b50.json 2>/dev/null || exit 1
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b50.json') if l.startswith('{')][0])
print('headline', d['value'], d['ms_per_step'], d['kernel_ms'], d['latency_ms_one_batch'])"
