#!/bin/bash
# phase timelines of the chain forms (trace build) + kernel stats of the XL step on form 8
set -u
o=gpurun_out/r4t; mkdir -p $o; export TMPDIR=/tmp
lib=$PWD/llm.c-paged_amd/libpaged_hip_trace.so
for B in 64 8; do
  for m in 4 5 6; do
    HPA_LIB=$lib timeout -k 10 120 python -u tools/pl_trace.py $B 990 $m > $o/trace${m}_b$B.txt 2>&1 || exit $?
  done
done
HPA_LIB=$lib timeout -k 10 200 python -u tools/pl_trace.py 64 990 7 XL > $o/trace7_xl.txt 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_xl -o run -- python3 bench.py --model XL --page-size 32 --steps 6 --warmup 2 --cpu-baseline off --prof-steps 0 > $o/prof_xl.log 2>&1 || exit $?
python3 tools/kstats.py $o/prof_xl/run_kernel_trace.csv > $o/kstats_xl.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $o/prof_c2 -o run -- python3 bench.py --steps 10 --warmup 3 --cpu-baseline off --prof-steps 0 > $o/prof_c2.log 2>&1 || exit $?
python3 tools/kstats.py $o/prof_c2/run_kernel_trace.csv > $o/kstats_c2.txt 2>&1
# A/B: pipelined counter polls (HPA_PL_PIPEPOLL build)
for B in 64 8; do
  for v in base pp; do
    lib=$PWD/llm.c-paged_amd/libpaged_hip.so; [ $v = pp ] && lib=$PWD/llm.c-paged_amd/libpaged_hip_pp.so
    HPA_LIB=$lib timeout -k 10 120 python -u bench.py --batch $B --steps 40 --warmup 5 --cpu-baseline off --prof-steps 0 > $o/ab_${v}_b$B.txt 2>&1 || exit $?
  done
done
for f in $o/ab_*.txt; do python3 -c "
import json
for l in open('$f'):
    if l.startswith('{'): d=json.loads(l); print('$(basename $f)', d['ms_per_step'], d['value'])"; done | tee $o/ab_summary.txt
