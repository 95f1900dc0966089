#!/bin/bash
# PSK kernel iteration on the GPU box: parity tests, then bench lines for the
# PSK workloads (kernel times solo and with batches in flight).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py ${PYTEST_ARGS:-} > gpurun_out/psk_par.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -4 gpurun_out/psk_par.log; [ $rc -ne 0 ] && exit $rc
for wl in ${WLS:-"qpsk9600" "qpsk9600 --inflight 3" "ofdm8 --inflight 1" "ofdm8" "psk8fec"}; do
  timeout -k 10 180 python bench.py --workload ${wl//@/ } --steps 5 --warmup 2 --no-cpu > gpurun_out/psk_b.json 2>/dev/null
  rc=$?; [ $rc -ne 0 ] && { echo "bench $wl rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/psk_b.json'));print('$wl',d['ms_per_step'],d['value'],{k:round(v,2) for k,v in d['kernel_ms'].items()},{k:round(v,2) for k,v in d['kernel_ms_solo'].items()})"
done
