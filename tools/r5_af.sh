#!/bin/bash
# round 5: per-wave timeline of XL chain form 8's fc phase (trace build)
set -u
o=gpurun_out/r5af; mkdir -p $o; export TMPDIR=/tmp
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 300 python -u tools/cx_wave_trace.py 64 200 > $o/cx_wave_b64.txt 2>&1 || exit $?
