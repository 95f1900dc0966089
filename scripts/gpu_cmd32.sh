set -o pipefail
for w in qpsk9600 ofdm8 psk8fec fsk9600; do
  WORKLOAD=$w TAG=r02 bash scripts/profile.sh > gpurun_out/prof32_$w.log 2>&1 || exit 1
done
mkdir -p gpurun_out/profiles_r02 && cp profiles/r02_* gpurun_out/profiles_r02/
