#!/bin/bash
# layer-loop forms: bench ms/step per batch; MODES (default "2 0"): 0 five
# launches per layer, 2 full persistent layer, 3 attention launch + chain
# usage: [MODES="3 2 0"] tools/pl_ab.sh <tag> <batches...>
set -u
tag=$1; shift; out=gpurun_out/$tag; mkdir -p $out
for B in "$@"; do
  for pl in ${MODES:-2 0}; do
    HPA_LAYER_KERNEL=$pl timeout -k 10 200 python -u bench.py --batch $B --steps 30 --warmup 5 --cpu-baseline off > $out/bench_b${B}_pl$pl.log 2>&1 || exit $?
    grep "^{" $out/bench_b${B}_pl$pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B pl=$pl ms/step', d['ms_per_step'], 'tok/s', d['value'])"
  done
done
