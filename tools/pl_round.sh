#!/bin/bash
# persistent layer vs five launches: bench at B = 64 / 8, kernel stats, phase
# timeline (trace build).  usage: tools/pl_round.sh <tag>
set -u
tag=$1; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for B in 64 8; do
  for pl in 1 0; do
    HPA_LAYER_KERNEL=$pl timeout -k 10 200 python -u bench.py --batch $B --steps 20 --warmup 5 --cpu-baseline off > $out/bench_b${B}_pl$pl.log 2>&1 || exit $?
    grep "^{" $out/bench_b${B}_pl$pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('B=$B pl=$pl ms/step', d['ms_per_step'], 'tok/s', d['value'])"
  done
done
for B in 64 8; do
  HPA_LIB=$PWD/llm.c-paged_amd/libpaged_hip_trace.so timeout -k 10 120 python -u tools/pl_trace.py $B 990 > $out/trace_b$B.txt 2>&1 || exit $?
  cat $out/trace_b$B.txt
done
for B in 64 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_b$B -o run -- python3 bench.py --batch $B --steps 10 --warmup 3 --cpu-baseline off > $out/prof_b$B.log 2>&1 || exit $?
  python3 tools/kstats.py $out/prof_b$B/run_kernel_trace.csv | grep -v rocclr | head -8 | sed "s/^/B=$B /"
done
