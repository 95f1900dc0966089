# PSK time-split A/B: KS0 convolution start states (default chunk rule) vs
# the w1-step warm-ups; extra variants as "VAR=value" words in $AB
set -e
for v in "CONV=1" "CONV=0" $AB; do
  echo "== $v"
  env AMR_PSK_SPLIT_${v} K=40 timeout -k 10 120 python tools/one_capture_probe.py
  env AMR_PSK_SPLIT_${v} timeout -k 10 120 python tools/split_batch_probe.py
done
