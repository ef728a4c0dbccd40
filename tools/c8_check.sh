#!/bin/bash
# chain forms 6 / 7 / 8: parity, then bench per batch (124M) and XL, then phase traces
set -u
o=gpurun_out/c8; mkdir -p $o
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py -x -v -s --timeout 300 --timeout-method thread -k "chain6 or chain8 or 124m" > $o/pytest_layer.txt 2>&1 || exit $?
for B in 64 8; do
  for lk in 1 5 6 7; do
    timeout -k 10 120 python -u bench.py --batch $B --layer-kernel $lk --steps 30 --warmup 5 --cpu-baseline off --prof-steps 0 > $o/bench_b${B}_lk$lk.txt 2>&1 || exit $?
  done
done
for lk in 0 7; do
  timeout -k 10 200 python -u bench.py --model XL --page-size 32 --layer-kernel $lk --steps 8 --warmup 2 --cpu-baseline off --prof-steps 0 > $o/bench_xl_lk$lk.txt 2>&1 || exit $?
done
for f in $o/bench_*.txt; do
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'], d['status'])"
done | tee $o/summary.txt
for B in 64 8; do
  for m in 4 5 6; do
    HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 $m > $o/trace${m}_b$B.txt 2>&1 || exit $?
  done
done
