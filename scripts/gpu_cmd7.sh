set -o pipefail
for cfg in "20 0" "32 16" "48 24" "64 32" "64 16"; do
  set -- $cfg
  AMR_LANE_WPB=4 timeout -k 10 150 python -u bench.py --steps $1 --inflight $2 --no-sub --no-host-path --no-cpu > gpurun_out/bench_k$1_p$2.json 2> gpurun_out/bench_k$1_p$2.err || exit 1
done
