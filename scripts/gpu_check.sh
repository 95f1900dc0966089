#!/bin/bash
# One GPU session: smoke -> gpu tests -> short bench -> rocprofv3 kernel trace.
# Stops at the first crash/timeout (rc 124/134/137/139); plain test failures (rc 1) continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
crashed() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log
if crashed $rc || [ $rc -ne 0 ]; then exit $rc; fi
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 1200 python -m pytest tests -m gpu -q -x ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests rc=$rc"; tail -15 gpurun_out/gpu_tests.log
  if crashed $rc; then exit $rc; fi
fi
timeout -k 10 600 python bench.py --steps ${STEPS:-5} --warmup ${WARMUP:-2} ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err
if crashed $rc || [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-host-path ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof_bench.json" 2> "$GRAFT_REPO_ROOT/gpurun_out/prof.err"
  rc=$?; echo "rocprof rc=$rc"; cd "$GRAFT_REPO_ROOT"
  find gpurun_out/prof -name "*stats*" | head; 
fi
exit 0
