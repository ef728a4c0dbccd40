#!/bin/bash
# round 5: the attention launch carries chain form 6's attproj (decode_attn_ap_kernel):
# parity + A/B (default: every batch; ap1: one row block only; ap0: off) + traces
set -u
o=gpurun_out/r5c; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_layer.py tests/test_gpu_decode.py tests/test_gpu_multi_rank.py -x -v -s --timeout 300 --timeout-method thread > $o/pytest.txt 2>&1 || exit $?
ab() {  # variant batch round
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $1 != base ] && lib=$PWD/llm.c-paged_amd/libpl_$1.so
  HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $2 --steps 60 --warmup 5 --cpu-baseline off --prof-steps 0 --spinup 1 > $o/ab_$1_b$2_$3.txt 2>&1
}
for r in 1 2; do
  for B in 8 64; do for v in base ap1 ap0; do ab $v $B $r || exit $?; done; done
  for B in 16 32; do for v in base ap0; do ab $v $B $r || exit $?; done; done
done
for f in $o/ab_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"; done | tee $o/ab_summary.txt
for B in 8 64; do
HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 5 > $o/trace_b$B.txt 2>&1 || exit $?
done
