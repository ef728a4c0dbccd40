#!/bin/bash
# chain form 6: parity tests, then bench A/B against the current default (form 4 wide units) per batch
set -u
o=gpurun_out/c6; mkdir -p $o
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py -x -v --timeout 300 --timeout-method thread > $o/pytest_layer.txt 2>&1 || exit $?
for B in 64 32 8; do
  for lk in 1 5; do
    timeout -k 10 120 python -u bench.py --batch $B --layer-kernel $lk --steps 30 --warmup 5 --cpu-baseline off --prof-steps 0 > $o/bench_b${B}_lk$lk.txt 2>&1 || exit $?
  done
done
for f in $o/bench_*.txt; do
  python3 -c "
import json,sys
for l in open('$f'):
    if l.startswith('{'):
        d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"
done | tee $o/summary.txt
