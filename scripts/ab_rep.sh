#!/bin/bash
# Same-box A/B: each "ENV|bench args" variant run REPS times, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "$VARIANTS"
for r in $(seq ${REPS:-2}); do
  for v in "${VARS[@]}"; do
    e="${v%%|*}"; a="${v#*|}"
    env $e timeout -k 10 180 python bench.py $a --steps ${STEPS:-10} --warmup 2 --no-cpu > gpurun_out/ab.json 2>/dev/null || { echo "fail: $v"; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v',d['ms_per_step'])"
  done
done
