# the N > 1 path on one GPU: a one-rank RCCL communicator, every launch's all-gather, the gather check
set -o pipefail
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 \
  bench.py --force-comm --steps 32 --no-host-path --no-dropin > gpurun_out/comm1.json 2> gpurun_out/comm1.err || exit 1
