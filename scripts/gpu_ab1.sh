# lane parity on the new library, then a same-box A/B of the headline (old vs new .so)
set -o pipefail
timeout -k 10 400 python -u -m pytest "tests/test_gpu_parity.py::test_lane_layout_forced_on_every_case" -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/ab1_parity.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/ab1_parity.log; [ $rc -ne 0 ] && exit $rc
OLD=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr_old.so
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr.so; fi
    AMR_LIB=$L timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin > gpurun_out/ab1_$v$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab1_$v$r.json') if l.startswith('{')][0]);print('$v', d['ms_per_step'], d['kernel_ms'])"
  done
  AMR_LIB=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr.so timeout -k 10 200 python bench.py --workload ofdm8 --no-host-path --no-cpu --no-latency --no-dropin > gpurun_out/ab1_ofdm$r.json 2>/dev/null || exit 1
  AMR_LIB=$OLD timeout -k 10 200 python bench.py --workload ofdm8 --no-host-path --no-cpu --no-latency --no-dropin > gpurun_out/ab1_ofdmold$r.json 2>/dev/null || exit 1
  python -c "import json;print('ofdm8 new', json.loads([l for l in open('gpurun_out/ab1_ofdm$r.json') if l.startswith('{')][0])['ms_per_step'], 'old', json.loads([l for l in open('gpurun_out/ab1_ofdmold$r.json') if l.startswith('{')][0])['ms_per_step'])"
done
