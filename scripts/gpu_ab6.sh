# fused slicer regions of 16 symbols (AMR_LP_REGION_SYMS=16) vs 8: lane parity on the variant, same-box A/B
set -o pipefail
AMR_LIB=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr_r16.so timeout -k 10 500 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab6_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab6_parity.log; [ $rc -ne 0 ] && exit $rc
OLD=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr.so
NEW=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr_r16.so
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$NEW; fi
    for k in "64 3" "20 5"; do
      set -- $k
      AMR_LIB=$L timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps $1 --warmup $2 > gpurun_out/ab6_$v.json 2>/dev/null || exit 1
      python -c "import json;d=json.loads([l for l in open('gpurun_out/ab6_$v.json') if l.startswith('{')][0]);print('$v K=$1', d['ms_per_step'], d['sustained']['ms_per_step'], d['kernel_ms_solo']['lowpass_fwd'], d['kernel_ms']['lowpass_fwd'])"
    done
  done
done
