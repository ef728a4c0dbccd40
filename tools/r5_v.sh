#!/bin/bash
# round 5: chain form 6 timeline at B = 8 / 16, with the stats over the 48 workgroups holding attproj units
set -u
o=gpurun_out/r5v; mkdir -p $o; export TMPDIR=/tmp
for B in 8 16; do
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 200 python -u tools/pl_trace.py $B 990 5 - active 48 > $o/trace6_b$B.txt 2>&1 || exit $?
done
