set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
TAG=r02 WORKLOAD=qpsk9600 bash scripts/profile.sh > gpurun_out/prof1.log 2>&1 || exit 1
COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" OUT=gpurun_out/pmc_sq_lane bash scripts/pmc_sq.sh --steps 32 --warmup 3 --no-sub --no-host-path > gpurun_out/prof1_sq.log 2>&1
