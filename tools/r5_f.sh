#!/bin/bash
# round 5: phase timeline of the bf16 chain (trace build) at B = 256 and 64
set -u
o=gpurun_out/r5f2; mkdir -p $o; export TMPDIR=/tmp
for B in 256 64; do
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 200 python -u tools/pl_trace.py $B 2000 1 b16 > $o/trace_b16_b$B.txt 2>&1 || exit $?
done
