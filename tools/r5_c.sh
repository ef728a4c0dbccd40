#!/bin/bash
# round 5: the attention launch carries chain form 6's attproj at one row block
# (decode_attn_ap_kernel): parity + A/B against DEC_ATTN_AP=0 + trace
set -u
o=gpurun_out/r5c; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_decode.py tests/test_gpu_multi_rank.py -x -v -s --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
for r in 1 2; do
  for v in base ap0; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = ap0 ] && lib=$PWD/llm.c-paged_amd/libpl_ap0.so
    for B in 8 16; do
      HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 60 --warmup 5 --cpu-baseline off --prof-steps 0 --spinup 1 > $o/ab_${v}_b${B}_$r.txt 2>&1 || exit $?
    done
  done
done
for f in $o/ab_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"; done | tee $o/ab_summary.txt
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py 8 990 5 > $o/trace_b8.txt 2>&1 || exit $?
