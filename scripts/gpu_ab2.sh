# same-box A/B at the driver's K = 20 (one round of 20 in flight): old vs new .so
set -o pipefail
OLD=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr_old.so
NEW=$GRAFT_REPO_ROOT/audio-modem-radio_amd/libamr.so
for r in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then L=$OLD; else L=$NEW; fi
    AMR_LIB=$L timeout -k 10 200 python bench.py --no-sub --no-host-path --no-cpu --no-latency --no-dropin --steps 20 --warmup 5 > gpurun_out/ab2_$v$r.json 2>/dev/null || exit 1
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab2_$v$r.json') if l.startswith('{')][0]);print('$v', d['ms_per_step'], d['sustained']['ms_per_step'])"
  done
done
