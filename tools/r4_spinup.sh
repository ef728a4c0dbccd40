#!/bin/bash
# round 4: does a fresh box run its first bench slower?  --spinup 3 first, then --spinup 0 twice, then 3 again
set -u
o=gpurun_out/r4su2; mkdir -p $o; export TMPDIR=/tmp
for v in 0 0 3; do
  timeout -k 10 150 python -u bench.py --spinup $v --cpu-baseline off > $o/b_$v.txt 2>&1 || exit $?
  grep "^{" $o/b_$v.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('spinup $v', d['ms_per_step'], d['value'], r['achieved'])" >> $o/summary.txt
done
cat $o/summary.txt
