#!/bin/bash
# rocprofv3 kernel traces of tools/pf_stage_timing.py per AMR_PF_STAGE (GPU box)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-pfst}
cd /tmp && export TMPDIR=/tmp
for st in ${STAGES:-0 1 2}; do
  AMR_PF_STAGE=$st timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/${TAG}_$st" -o run --output-format csv -- python3 "$ROOT/tools/pf_stage_timing.py" ${ROWS:-2048} ${N:-96000} > "$ROOT/gpurun_out/${TAG}_$st.log" 2>&1 || exit 1
done
