# round 3: FSK column / final passes in 3-wave workgroups (AMR_FFT_CR_NT=192)
# against the default (middle pass 3 waves) -- variant parity, then A/B, K = 64
set -o pipefail
T=${T:-r3k}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 300 --timeout-method thread -k "variants or batch_vs_oracle or full_batch" > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for v in def cr192; do
    if [ $v = cr192 ]; then export AMR_FFT_CR_NT=192; else unset AMR_FFT_CR_NT; fi
    timeout -k 10 300 python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 > gpurun_out/fsk_${v}_${i}_$T.json 2> gpurun_out/fsk_${v}_${i}_$T.err || exit 1
  done
done
