#!/bin/bash
# every workload through scripts/profile.sh (trace + FETCH_SIZE + WRITE_SIZE
# passes), then two SQ counter passes over the headline's lane kernels
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
for wl in ${WORKLOADS:-qpsk9600 ofdm8 psk8fec fsk9600}; do
  WORKLOAD=$wl bash scripts/profile.sh || exit 1
done
[ -n "${NO_SQ:-}" ] && exit 0
SQARGS="--steps 32 --warmup 3 --no-cpu --no-sub --no-latency --no-host-path --no-dropin --sustain-seconds 0"
COUNTERS="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
  OUT=gpurun_out/pmc_sq1 BASEARGS="$SQARGS" bash scripts/pmc_sq.sh || exit 1
COUNTERS="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64" \
  OUT=gpurun_out/pmc_sq2 BASEARGS="$SQARGS" bash scripts/pmc_sq.sh || exit 1
