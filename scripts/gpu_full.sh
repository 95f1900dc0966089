# the driver's round-end checks: the whole -m gpu suite, smoke(), the default bench
set -o pipefail
T=${T:-full}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/gputest_$T.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/gputest_$T.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || exit 1
[ -n "$NO_BENCH" ] && exit 0
timeout -k 10 600 python -u bench.py > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || exit 1
