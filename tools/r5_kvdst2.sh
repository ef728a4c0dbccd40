#!/bin/bash
# the same K/V-destination change in chain form 8 (XL) and the bf16 chain
# (config 5): the GPU suite, then a same-box A/B against the library before
# the change (ab_old/, HPA_LIB), alternating, XL and config 5
set -u
o=gpurun_out/r5kvdst2; mkdir -p $o; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
for r in 1 2; do
  for v in old new; do
    if [ $v = old ]; then L=$PWD/ab_old/libpaged_hip.so; else L=$PWD/llm.c-paged_amd/libpaged_hip.so; fi
    HPA_LIB=$L timeout -k 10 200 python -u bench.py --model XL --cpu-baseline off --steps 10 --warmup 2 > $o/xl_${v}_$r.txt 2>&1 || exit $?
    HPA_LIB=$L timeout -k 10 200 python -u bench.py $C5 --cpu-baseline off --steps 16 --warmup 3 > $o/c5_${v}_$r.txt 2>&1 || exit $?
  done
done
