#!/bin/bash
# qpsk9600 step time vs batches in flight, band-pass layout (K1r / K1g) and
# band-pass waves per workgroup.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "${PARITY_ENV:-}" ]; then
  env $PARITY_ENV timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/scan_par.log 2>&1
  rc=$?; echo "parity ($PARITY_ENV) rc=$rc"; tail -2 gpurun_out/scan_par.log; [ $rc -ne 0 ] && exit $rc
fi
for wpb in ${WPBS:-4 1}; do
for g8 in ${G8S:-0 1}; do
  for n in ${NS:-2 3}; do
    AMR_BP_WPB=$wpb AMR_BP_G8=$g8 timeout -k 10 180 python bench.py --workload ${WL:-qpsk9600} --inflight $n --steps ${STEPS:-8} --warmup 2 --no-cpu > gpurun_out/scan.json 2>/dev/null || exit 1
    python -c "import json;d=json.load(open('gpurun_out/scan.json'));print('wpb=$wpb g8=$g8 inflight=$n',d['ms_per_step'],{k:round(v,2) for k,v in d['kernel_ms'].items()})"
  done
done
done
