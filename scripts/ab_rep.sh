#!/bin/bash
# Same-box A/B (every A/B in DESIGN.md was run this way): each variant
# "ENV=.. ENV2=..|bench args" runs REPS times, interleaved, each under its own
# time limit; the JSON lines go to gpurun_out/ab_<TAG>_<rep>_<i>.json and a
# summary (ms/step, sustained, dominant kernel's solo ms) is printed.
#   VARIANTS='AMR_FFT_MID_NT=256|--workload fsk9600;|--workload fsk9600' REPS=2 TAG=mid bash scripts/ab_rep.sh
# Optional PYTEST='-k variants tests/test_gpu_fsk.py': a parity run first.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-ab}
if [ -n "${PYTEST:-}" ]; then
  timeout -k 10 900 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread $PYTEST > gpurun_out/ab_${TAG}_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/ab_${TAG}_pytest.log; [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra VARS <<< "$VARIANTS"
for r in $(seq ${REPS:-2}); do
  i=0
  for v in "${VARS[@]}"; do
    e="${v%%|*}"; a="${v#*|}"; i=$((i + 1))
    out=gpurun_out/ab_${TAG}_${r}_$i.json
    env $e timeout -k 10 300 python -u bench.py --no-host-path --no-dropin --cpu-seconds 0 $a > $out 2> ${out%.json}.err || { echo "fail: $v"; exit 1; }
    python - "$out" "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], (d.get("sustained") or {}).get("ms_per_step"), d["roofline"].get("kernel_ms_used"))
PY
  done
done
