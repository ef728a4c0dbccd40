#!/bin/bash
# round 4: decode attention at B = 64 -- 8 waves per workgroup, and default-policy K/V loads
# (tools/ablib/libnt0.so, -DHPA_ATTN_NT=0) vs the product (4 waves, non-temporal)
set -u
o=gpurun_out/r4aab; mkdir -p $o; export TMPDIR=/tmp
X=$PWD/tools/ablib
for v in prod w8 nt0 prod w8 nt0; do
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; args=""
  [ $v = nt0 ] && lib=$X/libnt0.so
  [ $v = w8 ] && args="--attn-waves 8"
  HPA_LIB=$lib timeout -k 10 120 python -u bench.py $args --steps 40 --warmup 5 --cpu-baseline off \
    > $o/b_$v.txt 2>&1 || exit $?
  grep "^{" $o/b_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['ms_per_step'], d['value'], r['achieved'], r['avg_launch_ms'])" >> $o/summary.txt
done
for v in prod nt0; do
  lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = nt0 ] && lib=$X/libnt0.so
  HPA_LIB=$lib timeout -k 10 200 python -u bench.py --model XL --page-size 32 --steps 8 --warmup 2 --cpu-baseline off \
    > $o/xl_$v.txt 2>&1 || exit $?
  grep "^{" $o/xl_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('XL $v', d['ms_per_step'], d['value'], r['achieved'], r['avg_launch_ms'])" >> $o/summary.txt
done
cat $o/summary.txt
