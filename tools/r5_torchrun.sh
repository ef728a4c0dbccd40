#!/bin/bash
# the driver's multi-GPU launcher form on one GPU: torch.distributed.run with
# one rank (RANK / WORLD_SIZE / MASTER_* from the launcher, a 1-rank RCCL
# communicator, the end-of-step gather), on the final round-5 tree
set -u
o=gpurun_out/r5torchrun; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --steps 32 --warmup 3 > $o/torchrun_n1.log 2>&1 || exit $?
