#!/bin/bash
# A/B bench lines: each argument is a quoted bench flag set; prints ms/step and attention us
set -u
out=gpurun_out/ab; mkdir -p $out
i=0
for flags in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --cpu-baseline off $flags > $out/b$i.log 2>&1 || { echo "fail: $flags"; tail -3 $out/b$i.log; exit 1; }
  grep "^{" $out/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('%-40s ms/step %.4f  tok/s %.0f' % ('$flags', d['ms_per_step'], d['value']))"
done
