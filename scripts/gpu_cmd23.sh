set -o pipefail
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --workload ofdm8 --batch 1024 --no-cpu --no-host-path --steps 64 --warmup 3 $ARGS > gpurun_out/b23_$tag.json 2> gpurun_out/b23_$tag.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b23_$tag.json') if l.startswith('{')][0])
print('$tag', d['value'], d['ms_per_step'], d['config']['batches_in_flight'], d['config']['kernel_layout'], d['kernel_ms'])"
}
ARGS="--inflight 16" run lane16 A=1
ARGS="--inflight 32" run lane32 A=1
ARGS="--inflight 16" run row16 AMR_PSK_LANE=0
ARGS="--inflight 32" run row32 AMR_PSK_LANE=0
ARGS="--inflight 8" run row8 AMR_PSK_LANE=0
