#!/bin/bash
# round 5: decode attention waves per (sequence, head) workgroup at B = 64 (1 / 2 / 4 product / 8) and B = 16
set -u
o=gpurun_out/r5r; mkdir -p $o; export TMPDIR=/tmp
for w in 4 2 1 8 4 2; do
  timeout -k 10 200 python -u bench.py --attn-waves $w --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b64_w$w.txt 2>&1 || exit $?
  tail -1 $o/bench_b64_w$w.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=64 waves $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $o/summary.txt
done
for w in 4 2; do
  timeout -k 10 200 python -u bench.py --batch 16 --attn-waves $w --cpu-baseline off --steps 30 --warmup 3 > $o/bench_b16_w$w.txt 2>&1 || exit $?
  tail -1 $o/bench_b16_w$w.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=16 waves $w', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])" >> $o/summary.txt
done
