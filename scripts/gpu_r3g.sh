# round 3: F1 with wave 1 storing z (AMR_FSK_W1S, default on) and the live
# middle pass with global twiddles (default): parity, then A/B of W1S
set -o pipefail
T=${T:-r3g}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
AMR_FSK_W1S=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -x -q -k "batch or live or golden" --timeout 400 --timeout-method thread > gpurun_out/gputest_${T}_w1s0.log 2>&1 || exit 1
run() {  # tag, env assignments..., then the bench command
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/fsk_${tag}_$T.json 2>gpurun_out/fsk_${tag}_$T.err || exit 1
}
B="python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight 2"
for i in 1 2; do
  run w1s1_$i AMR_FSK_W1S=1 $B
  run w1s0_$i AMR_FSK_W1S=0 $B
done
run w1s1_p3 AMR_FSK_W1S=1 python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight 3
