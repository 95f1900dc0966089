# quick A/B on the GPU box: lane parity + golden, then the headline bench
set -o pipefail
T=${T:-q}
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" "tests/test_gpu_parity.py::test_every_golden_psk_case_bit_exact" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --no-sub --no-host-path ${BENCH_ARGS:-} > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
python3 - <<PY
import json
d=json.loads([l for l in open('gpurun_out/bench_$T.json') if l.startswith('{')][0])
print("VALUE", d['value'], d['ms_per_step'], d['config']['batches_in_flight'], d['kernel_ms_solo'], d['kernel_ms'], d['parity'])
PY
