set -o pipefail
timeout -k 10 600 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" tests/test_gpu_slicer.py "tests/test_gpu_parity.py::test_every_golden_psk_case_bit_exact" -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest33.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest33.log; [ $rc -ne 0 ] && exit $rc
for w in qpsk9600 ofdm8 psk8fec; do
  timeout -k 10 300 python -u bench.py --workload $w --no-host-path > gpurun_out/b33_$w.json 2>/dev/null || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b33_$w.json') if l.startswith('{')][0])
print('$w', d['value'], d['ms_per_step'], d['kernel_ms'], d['parity'])"
done
