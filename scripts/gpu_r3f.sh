# round 3: live middle pass variants -- pipelined LDS-DMA kernel (default),
# the one-tile kernel with the W_L table in global memory (AMR_FFT_MID_PIPE=0)
# and in LDS (+ AMR_FFT_MID_TWG=0): parity of each, then A/B
set -o pipefail
T=${T:-r3f}
AMR_FFT_MID_PIPE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_fsk.py -m gpu -x -v -k "batch_vs_oracle" --timeout 120 --timeout-method thread > gpurun_out/gputest_${T}_quick.log 2>&1 || exit 1
AMR_FFT_MID_PIPE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
AMR_FFT_MID_PIPE=0 AMR_FFT_MID_TWG=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -x -q -k "batch or live" --timeout 400 --timeout-method thread > gpurun_out/gputest_${T}_pipe0.log 2>&1 || exit 1
AMR_FFT_MID_PIPE=0 AMR_FFT_MID_TWG=0 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -x -q -k "batch or live" --timeout 400 --timeout-method thread > gpurun_out/gputest_${T}_twg0.log 2>&1 || exit 1
run() {  # tag, env assignments..., then the bench command
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/fsk_${tag}_$T.json 2>gpurun_out/fsk_${tag}_$T.err || exit 1
}
B="python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight 2"
for i in 1 2; do
  run pipe_$i AMR_FFT_MID_PIPE=1 $B
  run twg1_$i AMR_FFT_MID_PIPE=0 AMR_FFT_MID_TWG=1 $B
  run twg0_$i AMR_FFT_MID_PIPE=0 AMR_FFT_MID_TWG=0 $B
done
