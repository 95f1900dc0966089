set -o pipefail
run() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --no-sub --no-host-path --no-cpu > gpurun_out/b17_$tag.json 2> gpurun_out/b17_$tag.err || exit 1
  python3 -c "
import json
d=json.loads([l for l in open('gpurun_out/b17_$tag.json') if l.startswith('{')][0])
print('$tag', d['value'], d['ms_per_step'], d['kernel_ms'], d['kernel_ms_solo'])"
}
run base AMR_X=0
run lpsplit AMR_LP_SPLIT=1
run wpb2 AMR_LANE_WPB=2
run wpb2lp AMR_LANE_WPB=2 AMR_LP_SPLIT=1
run nobpsplit AMR_BP_SPLIT=0
