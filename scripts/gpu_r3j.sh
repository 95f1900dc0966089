# round 3: FSK live middle pass in 3-wave workgroups (AMR_FFT_MID_NT=192, no
# VGPR spills) -- variant parity, then interleaved same-box A/B at K = 64
set -o pipefail
T=${T:-r3j}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 300 --timeout-method thread -k "variants or batch_vs_oracle" > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for nt in 256 192; do
    AMR_FFT_MID_NT=$nt timeout -k 10 300 python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 > gpurun_out/fsk_nt${nt}_${i}_$T.json 2> gpurun_out/fsk_nt${nt}_${i}_$T.err || exit 1
  done
done
