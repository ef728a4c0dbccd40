#!/bin/bash
# round 5: gpt2_forward one-pass window + config-1 shape; chain form 6 with the
# attproj units placed on the fc-free workgroups (one row block): traces + A/B
set -u
o=gpurun_out/r5b; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_layer.py -x -v -s --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
for B in 8 16; do
  for v in trace trbp0; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip_trace.so; [ $v = trbp0 ] && lib=$PWD/llm.c-paged_amd/libpl_trbp0.so
    HPA_LIB=$lib timeout -k 10 120 python -u tools/pl_trace.py $B 990 5 > $o/trace_${v}_b$B.txt 2>&1 || exit $?
  done
done
for r in 1 2; do
  for v in base bp0; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = bp0 ] && lib=$PWD/llm.c-paged_amd/libpl_bp0.so
    for B in 8 16; do
      HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 60 --warmup 5 --cpu-baseline off --prof-steps 0 --spinup 1 > $o/ab_${v}_b${B}_$r.txt 2>&1 || exit $?
    done
  done
done
for f in $o/ab_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"; done | tee $o/ab_summary.txt
