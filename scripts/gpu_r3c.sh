# round 3: bench N > 1 path via multi.py, the 64-sample band-pass checkpoint
# variant's parity, the default bench line, then a same-box A/B of AMR_BP_CK
set -o pipefail
T=${T:-r3c}
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_comm.py \
  "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case[bp_ck2]" \
  "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case[bp_ck2_no_zero_taps]" \
  -m gpu -v -s --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --no-sub --no-host-path --no-dropin --cpu-seconds 0 > gpurun_out/ab_ck1_$i.json 2>/dev/null || exit 1
  AMR_BP_CK=2 timeout -k 10 200 python -u bench.py --no-sub --no-host-path --no-dropin --cpu-seconds 0 > gpurun_out/ab_ck2_$i.json 2>/dev/null || exit 1
done
