#!/bin/bash
# round 5: form 6 with the fc prefetch held back on workgroups without an attproj unit (A/B: 0, 1, 2 us) at B = 8, 16, 64
set -u
o=gpurun_out/r5n; mkdir -p $o; export TMPDIR=/tmp
for B in 8 16 64; do
  timeout -k 10 200 python -u bench.py --batch $B --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b${B}_fd0.txt 2>&1 || exit $?
  for d in 100 200; do
    HPA_LIB=$PWD/llm.c-paged_amd/libfd$d.so timeout -k 10 200 python -u bench.py --batch $B --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b${B}_fd$d.txt 2>&1 || exit $?
  done
done
