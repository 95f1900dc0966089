# Same-box A/B of the DEFAULT bench run (headline + sub-workloads) under
# environment variants: VARIANTS="ENV=..|args;..." (as scripts/ab_rep.sh)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
IFS=';' read -ra VARS <<< "${VARIANTS:-|--no-dropin}"
i=0
for v in "${VARS[@]}"; do
  e="${v%%|*}"; a="${v#*|}"; i=$((i + 1))
  out=gpurun_out/abd_${TAG:-d}_$i.json
  env $e timeout -k 10 600 python -u bench.py --cpu-seconds 1 $a > $out 2> ${out%.json}.err || exit 1
  python - $out "$v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["ms_per_step"], {k: v["ms_per_step"] for k, v in d.get("workloads", {}).items()})
PY
done
