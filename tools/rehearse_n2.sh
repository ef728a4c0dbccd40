#!/bin/bash
# N = 2 rehearsal on a one-GPU box: two bench ranks on device 0 under the
# driver's launcher.  RCCL refuses two ranks on one device, so the expected
# outcome is a non-zero exit and no JSON value (bench.py: a run without its
# collective reports nothing); the log shows which HIP / RCCL libraries the
# measuring processes loaded (no torch in them).
set -u
out=${1:-gpurun_out/rehearse}; mkdir -p $out
HPA_DEVICE=0 timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 5 --warmup 2 --cpu-baseline off \
  > $out/n2.log 2>&1
rc=$?
echo "exit code: $rc" | tee -a $out/n2.log
grep -c '^{' $out/n2.log | sed 's/^/JSON lines: /' | tee -a $out/n2.log || true
exit 0
