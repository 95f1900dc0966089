# round profiles (TAG, default r04): rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE
# passes for every bench workload (scripts/profile.sh), then the driver-style
# bench line and the default one
set -o pipefail
for w in qpsk9600 fsk9600 ofdm8 psk8fec; do
  TAG=${TAG:-r04} WORKLOAD=$w bash scripts/profile.sh > gpurun_out/prof_${TAG:-r04}_$w.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_${TAG:-r04}_driver.json 2> gpurun_out/bench_${TAG:-r04}_driver.err || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_${TAG:-r04}_default.json 2> gpurun_out/bench_${TAG:-r04}_default.err || exit 1
