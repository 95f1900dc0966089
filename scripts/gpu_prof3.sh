# round 3 profiles: rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE
# passes for every bench workload (scripts/profile.sh), then the driver-style
# bench line and the default one
set -o pipefail
for w in qpsk9600 fsk9600 ofdm8 psk8fec; do
  TAG=r03 WORKLOAD=$w bash scripts/profile.sh > gpurun_out/prof_r03_$w.log 2>&1 || exit 1
done
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_r03_driver.json 2> gpurun_out/bench_r03_driver.err || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r03_default.json 2> gpurun_out/bench_r03_default.err || exit 1
