set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slicer.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest29.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest29.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do timeout -k 10 300 python -u bench.py --no-sub --no-host-path > gpurun_out/b29_$i.json 2>/dev/null || exit 1
python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b29_$i.json') if l.startswith('{')][0])
print('symlayout', d['value'], d['ms_per_step'], d['kernel_ms'], d['parity'])"; done
