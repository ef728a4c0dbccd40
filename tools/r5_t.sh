#!/bin/bash
# round 5: attention beside chain form 6 -- is the slowdown the 256 pollers? poll interval / nap A/B
set -u
o=gpurun_out/r5t; mkdir -p $o; export TMPDIR=/tmp
run() {  # lib tag batch
  HPA_LIB=$PWD/llm.c-paged_amd/$1 timeout -k 10 200 python -u bench.py --batch $3 --cpu-baseline off --steps 30 --warmup 3 > $o/bench_$2_b$3.txt 2>&1 || exit $?
  tail -1 $o/bench_$2_b$3.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2 B=$3', d['value'], d['ms_per_step'])" >> $o/summary.txt
}
run libnb.so boundary 64
run libpaged_hip.so sleep8 64
run libsl127.so sleep127 64
run libnap.so nap50us 64
run libnb.so boundary 8
run libsl127.so sleep127 8
