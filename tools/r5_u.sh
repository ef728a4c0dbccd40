#!/bin/bash
# round 5: GPT-2 XL attention shape sweep (waves per workgroup, context ranges) at B = 64, page 32
set -u
o=gpurun_out/r5u; mkdir -p $o; export TMPDIR=/tmp
for cfg in "4 0" "2 0" "8 0" "4 2" "2 2"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --model XL --page-size 32 --attn-waves $1 --attn-splits $2 --cpu-baseline off --steps 8 --warmup 2 > $o/xl_w$1_s$2.txt 2>&1 || exit $?
  tail -1 $o/xl_w$1_s$2.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('XL waves $1 splits $2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['config']['attn_splits'])" >> $o/summary.txt
done
