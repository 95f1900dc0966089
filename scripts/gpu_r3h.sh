# round 3: F1 whole-sector z stores (AMR_FSK_WHOLE=1, compact carry on the
# wave-1 store path): parity, A/B, and the PMC bytes of F1 both ways
set -o pipefail
T=${T:-r3h}
AMR_FSK_WHOLE=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_fsk.py -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
run() {  # tag, env assignments..., then the bench command
  local tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/fsk_${tag}_$T.json 2>gpurun_out/fsk_${tag}_$T.err || exit 1
}
B="python -u bench.py --workload fsk9600 --no-host-path --no-dropin --cpu-seconds 0 --inflight 2"
for i in 1 2; do
  run wh1_$i AMR_FSK_WHOLE=1 $B
  run wh0_$i AMR_FSK_WHOLE=0 $B
done
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for v in 0 1; do
  AMR_FSK_WHOLE=$v timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $R/gpurun_out/${T}_write$v -o run --output-format csv -- python3 $R/bench.py --workload fsk9600 --steps 1 --warmup 0 --no-cpu --batch 4096 --no-host-path --no-dropin > $R/gpurun_out/${T}_write$v.log 2>&1 || exit 1
done
