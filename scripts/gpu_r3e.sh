# round 3: SQ counters of the FSK passes (live-column layout), one --pmc pass
# per counter group, small batch (pmc_fsk.sh); B = 4096 streams
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
TAG=${TAG:-r3e}
cd /tmp && export TMPDIR=/tmp
run() {  # $1 = suffix, rest = counters
  local sfx=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d "$ROOT/gpurun_out/${TAG}_$sfx" -o run --output-format csv -- python3 "$ROOT/bench.py" --workload fsk9600 --steps 1 --warmup 0 --no-cpu --batch 4096 --no-host-path --no-dropin > "$ROOT/gpurun_out/${TAG}_$sfx.log" 2>&1
}
run sq1 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU && \
run sq2 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_INSTS_SALU SQ_ACTIVE_INST_LDS && \
run fetch FETCH_SIZE && run write WRITE_SIZE
echo "pmc rc=$?"
