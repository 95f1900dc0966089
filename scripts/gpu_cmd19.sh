set -o pipefail
T=${T:-x}
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
for P in ${PS:-16 24}; do
  timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu --steps 48 --warmup 3 --inflight $P > gpurun_out/b19_${T}_$P.json 2> gpurun_out/b19_${T}_$P.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b19_${T}_$P.json') if l.startswith('{')][0])
print('$T P=$P', d['value'], d['ms_per_step'], d['kernel_ms'], d['kernel_ms_solo'])"
done
