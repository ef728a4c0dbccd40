#!/bin/bash
# two-lane step: graph vs eager at B = 64, and a kernel trace of the eager two-lane run (overlap check)
set -u
o=gpurun_out/r4ln2; mkdir -p $o; export TMPDIR=/tmp
for g in "" "--no-graph"; do
  for ln in 1 2; do
    timeout -k 10 120 python -u bench.py --batch 64 --lanes $ln $g --steps 30 --warmup 5 --cpu-baseline off \
      --prof-steps 0 > $o/bench_l$ln$g.txt 2>&1 || exit $?
    grep "^{" $o/bench_l$ln$g.txt | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lanes', d['config']['lanes'], 'graph', d['config']['hip_graph'], d['ms_per_step'])" >> $o/summary.txt
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/k -o run -- \
  python3 bench.py --lanes 2 --no-graph --steps 4 --warmup 2 --cpu-baseline off --prof-steps 0 > $o/k.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $o/kg -o run -- \
  python3 bench.py --lanes 2 --steps 4 --warmup 2 --cpu-baseline off --prof-steps 0 > $o/kg.log 2>&1 || exit $?
cat $o/summary.txt
