#!/bin/bash
# round 5: config 5 attention waves per (sequence, head) workgroup (bf16 KV, page 8, B = 256)
set -u
o=gpurun_out/r5aa; mkdir -p $o; export TMPDIR=/tmp
C5="--batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off --steps 15 --warmup 2"
for w in 4 2 8 1; do
  timeout -k 10 300 python -u bench.py $C5 --attn-waves $w > $o/c5_w$w.txt 2>&1 || exit $?
  tail -1 $o/c5_w$w.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('c5 waves $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $o/summary.txt
done
