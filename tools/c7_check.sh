#!/bin/bash
# chain forms 6 / 7 (granule hand-offs): parity, then bench per batch against the default, then phase traces
set -u
o=gpurun_out/c7; mkdir -p $o
timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 200 --timeout-method thread -k "chain6 or 124m" > $o/pytest_layer.txt 2>&1 || exit $?
for B in 64 32 8; do
  for lk in 1 5 6; do
    timeout -k 10 120 python -u bench.py --batch $B --layer-kernel $lk --steps 30 --warmup 5 --cpu-baseline off --prof-steps 0 > $o/bench_b${B}_lk$lk.txt 2>&1 || exit $?
  done
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
