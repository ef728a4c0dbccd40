#!/bin/bash
# chain form 6 vs the default per batch (bench), then the form-6 phase timeline (trace build)
set -u
o=gpurun_out/c6; mkdir -p $o
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
for B in 64 8; do
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 5 > $o/trace6_b$B.txt 2>&1 || exit $?
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 4 > $o/trace4_b$B.txt 2>&1 || exit $?
done
