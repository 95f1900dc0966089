# a round's profiles (TAG, default r03): rocprofv3 kernel trace + separate
# FETCH_SIZE / WRITE_SIZE passes for every bench workload (scripts/profile.sh),
# the driver's own command under the kernel trace (scripts/prof_driver.sh),
# then the driver-style bench line and the default one.  Fold locally
# afterwards: python scripts/prof_summary.py gpurun_out/prof_<TAG>_<w> <TAG> <w>
set -o pipefail
TAG=${TAG:-r03}
for w in qpsk9600 fsk9600 ofdm8 psk8fec; do
  TAG=$TAG WORKLOAD=$w bash scripts/profile.sh > gpurun_out/prof_${TAG}_$w.log 2>&1 || exit 1
done
TAG=$TAG bash scripts/prof_driver.sh > gpurun_out/prof_${TAG}_driver.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG}_driver.json 2> gpurun_out/bench_${TAG}_driver.err || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG}_default.json 2> gpurun_out/bench_${TAG}_default.err || exit 1
