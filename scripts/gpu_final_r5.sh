# round-5 closing run: the driver's checks (scripts/gpu_full.sh), then the
# one-capture A/B of the convolution start states (both split layouts)
set -o pipefail
T=${T:-r5k} bash scripts/gpu_full.sh || exit 1
K=40 timeout -k 10 120 python tools/one_capture_probe.py > gpurun_out/oc_conv_final.txt 2>&1 || exit 1
echo "== AMR_PSK_SPLIT_CONV=0 AMR_FSK_SPLIT_CONV=0" >> gpurun_out/oc_conv_final.txt
AMR_PSK_SPLIT_CONV=0 AMR_FSK_SPLIT_CONV=0 K=40 timeout -k 10 120 python tools/one_capture_probe.py >> gpurun_out/oc_conv_final.txt 2>&1 || exit 1
timeout -k 10 120 python tools/split_batch_probe.py >> gpurun_out/oc_conv_final.txt 2>&1
