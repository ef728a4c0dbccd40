#!/bin/bash
# chain form A/B on one box: the attention's ranges merged by attproj
# (default pick) vs merged in the attention kernel (HPA_CHAIN_SPLITS=1),
# bench.py at B = 8, 16, 32, 64.  usage: tools/chain_ab.sh <out.txt>
out=${1:-gpurun_out/chain_ab.txt}
: > "$out"
for B in ${BATCHES:-8 16 32 64}; do
  for cs in 0 1; do
    if [ "$cs" = 0 ]; then unset HPA_CHAIN_SPLITS; else export HPA_CHAIN_SPLITS=$cs; fi
    timeout -k 10 150 python bench.py --batch $B --steps 30 --warmup 5 --cpu-baseline off > gpurun_out/cab_${B}_${cs}.log 2>&1 || exit 1
    ms=$(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cab_${B}_${cs}.log | grep -o '[0-9.]*$')
    sp=$(grep -o '"attn_splits": [0-9]*' gpurun_out/cab_${B}_${cs}.log | grep -o '[0-9]*$')
    echo "B=$B chain_splits_env=$cs attn_splits=$sp ms_per_step=$ms" | tee -a "$out"
  done
done
unset HPA_CHAIN_SPLITS
