#!/bin/bash
# round 4: GPT-2 XL attention launch shape A/B (waves per workgroup 4 / 8, split count 1 / 2) at B = 64, page 32
set -u
o=gpurun_out/r4xa; mkdir -p $o; export TMPDIR=/tmp
for v in "w0s0:" "w8s0:--attn-waves 8" "w0s2:--attn-splits 2" "w0s0:" "w8s0:--attn-waves 8" "w0s2:--attn-splits 2"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 200 python -u bench.py --model XL --page-size 32 $args --steps 8 --warmup 2 --cpu-baseline off \
    > $o/xl_$n.txt 2>&1 || exit $?
  grep "^{" $o/xl_$n.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('XL $n', d['ms_per_step'], d['value'], r['achieved'], r['avg_launch_ms'])" >> $o/summary.txt
done
cat $o/summary.txt
