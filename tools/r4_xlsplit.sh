#!/bin/bash
# round 4: GPT-2 XL attention at 1600 (sequence, head) workgroups (6.25 per CU) -- the split
# count's effect on the launch's tail: bench A/B at --attn-splits 1 / 2 / 3, and 124M B = 64 at 1 / 2
set -u
o=gpurun_out/r4xs; mkdir -p $o; export TMPDIR=/tmp
for s in 1 2 3 1 2 3; do
  timeout -k 10 200 python -u bench.py --model XL --page-size 32 --attn-splits $s --steps 8 --warmup 2 \
    --cpu-baseline off > $o/xl_s$s.txt 2>&1 || exit $?
  grep "^{" $o/xl_s$s.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('XL S=$s', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])" >> $o/summary.txt
done
for s in 1 2 1 2; do
  timeout -k 10 120 python -u bench.py --attn-splits $s --steps 40 --warmup 5 --cpu-baseline off \
    > $o/c2_s$s.txt 2>&1 || exit $?
  grep "^{" $o/c2_s$s.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('124M B=64 S=$s', d['ms_per_step'], d['value'], d['roofline']['achieved'], d['roofline']['avg_launch_ms'])" >> $o/summary.txt
done
cat $o/summary.txt
