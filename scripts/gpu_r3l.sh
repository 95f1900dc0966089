# round 3 (late): the FSK 3-wave column/final pass A/B (scripts/gpu_r3k.sh),
# then the round's profiles of every workload and the bench lines
# (scripts/gpu_prof3.sh) with the default kernels
set -o pipefail
T=r3k bash scripts/gpu_r3k.sh || exit 1
unset AMR_FFT_CR_NT
bash scripts/gpu_prof3.sh || exit 1
