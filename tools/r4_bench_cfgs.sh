#!/bin/bash
# final tree, default spin-up: configs 3 and 5 bench lines (smoke of the spin-up on those paths)
set -u
o=gpurun_out/r4bc; mkdir -p $o; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --model XL --page-size 32 --cpu-baseline off > $o/bench_xl.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --batch 256 --ctx 2048 --page-size 8 --kv-dtype bf16 --w-dtype bf16 --cpu-baseline off \
  > $o/bench_c5.log 2>&1 || exit $?
for f in bench_xl bench_c5; do
  grep "^{" $o/$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'], d['spinup_s'], d['roofline']['frac'], d['status'])"
done
