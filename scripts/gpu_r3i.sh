# round 3: FSK after wave-1 z stores -- parity (incl. the kernel-variant
# switches), then batches in flight P = 2 / 3 / 4 at K = 64
set -o pipefail
T=${T:-r3i}
timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
for i in 1 2; do
  for p in 2 3 4; do
    timeout -k 10 300 python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight $p > gpurun_out/fsk_p${p}_${i}_$T.json 2> gpurun_out/fsk_p${p}_${i}_$T.err || exit 1
  done
done
