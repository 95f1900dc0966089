# round 3: FSK middle pass (LDS position table, pruned last stage) and F1
# whole-sector stores -- parity, then A/B against AMR_FSK_WHOLE=0 / AMR_FFT_PRUNE=0
set -o pipefail
T=${T:-r3d}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
AMR_FSK_WHOLE=0 AMR_FFT_PRUNE=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -x -q -k "batch or live" --timeout 400 --timeout-method thread > gpurun_out/gputest_${T}_off.log 2>&1 || exit 1
run() {  # tag, env assignments..., then the bench command
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/fsk_${tag}_$T.json 2>gpurun_out/fsk_${tag}_$T.err || exit 1
}
B="python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight 2"
for i in 1 2; do
  run on_$i AMR_FSK_WHOLE=1 $B
  run whole0_$i AMR_FSK_WHOLE=0 $B
  run prune0_$i AMR_FFT_PRUNE=0 $B
done
