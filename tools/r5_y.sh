#!/bin/bash
# round 5: kernel-argument preload into SGPRs (-mllvm -amdgpu-kernarg-preload-count=16, libkp) vs product: parity + bench A/B
set -u
o=gpurun_out/r5y; mkdir -p $o; export TMPDIR=/tmp
HPA_LIB=$PWD/llm.c-paged_amd/libkp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > $o/pytest_kp.txt 2>&1 || exit $?
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16"
for rep in 1 2; do
for lib in libpaged_hip.so libkp.so; do
  for B in 64 8; do
    HPA_LIB=$PWD/llm.c-paged_amd/$lib timeout -k 10 200 python -u bench.py --batch $B --cpu-baseline off --steps 30 --warmup 3 > $o/b$B.txt 2>&1 || exit $?
    tail -1 $o/b$B.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib B=$B', d['value'], d['ms_per_step'])" >> $o/summary.txt
  done
done
done
for lib in libpaged_hip.so libkp.so; do
  HPA_LIB=$PWD/llm.c-paged_amd/$lib timeout -k 10 300 python -u bench.py $C5 --cpu-baseline off --steps 20 --warmup 3 > $o/c5.txt 2>&1 || exit $?
  tail -1 $o/c5.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib c5', d['value'], d['ms_per_step'])" >> $o/summary.txt
done
